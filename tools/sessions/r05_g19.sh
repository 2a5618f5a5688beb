# Round 5 (GPU box): the full-size configs[4] pipeline after the arena calibration and the two-groups-
# per-lane cut of small inputs (aln end 2 against end 1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --out gpurun_out/r05_pipe_full_v3.json > gpurun_out/r05_pipe_full_v3.log 2>&1
