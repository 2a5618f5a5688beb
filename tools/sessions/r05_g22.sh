# Round 5 (GPU box): the full-size configs[4] pipeline with each aln held to a 118 GiB arena in 0.85 GB
# pieces (two groups per lane): does end 2 still wait for end 1's memory?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
IBWA_ARENA_GB=118 IBWA_FQ_PIECE_BYTES=850000000 timeout -k 10 1000 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --out gpurun_out/r05_pipe_full_v4.json > gpurun_out/r05_pipe_full_v4.log 2>&1
