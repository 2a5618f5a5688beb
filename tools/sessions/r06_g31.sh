# Round 6 (GPU box): the whole -m gpu suite at the final tree (edge-read and K = 14 parity sets added)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g31.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g31.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g31.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_final.log 2>&1 || { tail -20 gpurun_out/r06_smoke_final.log; exit 1; }
tail -2 gpurun_out/r06_smoke_final.log
