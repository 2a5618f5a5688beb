# Round 5 (GPU box): the first run handing its arena back before it exits (IBWA_ALN_RELEASE=1) --
# its cost and the second run's wait, at 118 and 172 GiB arenas
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/backtoback.py --arena-gb 118 --cases fast,release,fast,release > gpurun_out/r05_b2b_rel.jsonl 2> gpurun_out/r05_b2b_rel.log || { tail -5 gpurun_out/r05_b2b_rel.log; exit 1; }
timeout -k 10 300 python tools/backtoback.py --arena-gb 172 --cases fast,release,release > gpurun_out/r05_b2b_rel172.jsonl 2> gpurun_out/r05_b2b_rel172.log
