# Round 5 (GPU box): the full-size configs[4] pipeline with both ends' aln also run at once on the one
# GPU (each under ~128 GiB: two groups per lane for a 10 M-pair end), .sai compared
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --out gpurun_out/r05_pipe_full_v5.json > gpurun_out/r05_pipe_full_v5.log 2>&1
