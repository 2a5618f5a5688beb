# Round 5 (GPU box): why the second of two back-to-back `aln` runs waits in its arena when two
# alloc_bench processes of the same size do not -- the first run's exit (fast / clean / 2 s later),
# and mixed pairs (CLI then alloc_bench, alloc_bench then CLI)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/backtoback.py --arena-gb 118 --cases fast,clean,sleep2,fast > gpurun_out/r05_b2b.jsonl 2> gpurun_out/r05_b2b.log || { tail -5 gpurun_out/r05_b2b.log; exit 1; }
T=$(mktemp -d)
IBWA_ARENA_GB=118 IBWA_ALN_TIMES=1 timeout -k 10 120 ibwa_amd/bin/ibwa-amd aln -f $T/a.sai tests/golden/g1m tests/golden/reads_mixed.fq 2> gpurun_out/r05_b2b_cli1.log > /dev/null || exit 1
timeout -k 5 120 tools/_build/alloc_bench probe 118 118 >> gpurun_out/r05_b2b_mixed.jsonl || exit 1
sleep 12
timeout -k 5 120 tools/_build/alloc_bench hold 118 118 >> gpurun_out/r05_b2b_mixed.jsonl || exit 1
IBWA_ARENA_GB=118 IBWA_ALN_TIMES=1 timeout -k 10 120 ibwa_amd/bin/ibwa-amd aln -f $T/b.sai tests/golden/g1m tests/golden/reads_mixed.fq 2> gpurun_out/r05_b2b_cli2.log > /dev/null || exit 1
rm -rf $T
