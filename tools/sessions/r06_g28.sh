# Round 6 (GPU box): samse / sampe goldens after the parallel fix-up, then the full-size pipeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sampe_gpu.py tests/test_samse_gpu.py tests/test_paired_sw_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g28.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g28.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g28.log
timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --concurrent-lanes 1 --out gpurun_out/r06_pipe_full_v9.json > gpurun_out/r06_pipe_full_v9.log 2>&1 || { tail -30 gpurun_out/r06_pipe_full_v9.log; exit 1; }
grep "both ends\|sequential ends\|sampe -R -G\|sample " gpurun_out/r06_pipe_full_v9.log
