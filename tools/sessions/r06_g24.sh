# Round 6 (GPU box): the new parity tests -- reads at the reference's ends, the K = 14 scale set
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_properties.py -m gpu -x -v --timeout 300 --timeout-method thread -k "edge or gap_tab_k or tab_k" > gpurun_out/r06_gpu_tests_g24.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g24.log; exit 1; }
tail -3 gpurun_out/r06_gpu_tests_g24.log
