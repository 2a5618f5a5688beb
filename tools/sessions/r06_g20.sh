# Round 6 (GPU box): final same-build profiles (kernel trace, EA PMC, SQ, k_sw counters), the sampe
# goldens after the positions-pass change, then the full-size configs[4] pipeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/sessions/r06_g3.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_sampe_gpu.py tests/test_samse_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g20.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g20.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g20.log
timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --concurrent-lanes 1 --out gpurun_out/r06_pipe_full_v6.json > gpurun_out/r06_pipe_full_v6.log 2>&1 || { tail -30 gpurun_out/r06_pipe_full_v6.log; exit 1; }
grep "both ends\|sequential ends\|sampe -R -G\|sample " gpurun_out/r06_pipe_full_v6.log
