# Round 5 (GPU box): sampe -G workers -- the sampe GPU tests (goldens with -G 2, small batches with
# -G 1/2/3), then the full-size pipeline with sampe -R at -G 1, 2 and 3 (SAM digests compared)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sampe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05_sampe_tests_g29.log 2>&1 || { tail -30 gpurun_out/r05_sampe_tests_g29.log; exit 1; }
tail -3 gpurun_out/r05_sampe_tests_g29.log
timeout -k 10 1000 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --concurrent-ends 0 --sampe-workers 1,2,3 --out gpurun_out/r05_pipe_full_v6.json > gpurun_out/r05_pipe_full_v6.log 2>&1 || { tail -30 gpurun_out/r05_pipe_full_v6.log; exit 1; }
grep "sampe" gpurun_out/r05_pipe_full_v6.log | tail -12
