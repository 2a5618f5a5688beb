# Round 6 (GPU box): sampe with 2 / 3 / 4 batch workers at full size (configs[4] shape)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 2000 --concurrent-ends 0 --sampe-workers 2,3,4,2 --out gpurun_out/r06_pipe_workers.json > gpurun_out/r06_pipe_workers.log 2>&1 || { tail -30 gpurun_out/r06_pipe_workers.log; exit 1; }
grep "sampe -R -G" gpurun_out/r06_pipe_workers.log
