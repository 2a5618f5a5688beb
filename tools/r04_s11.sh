#!/bin/bash
# Round 4 (GPU box): sampe / samse / CLI tests, then the configs[4] pipeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sampe_gpu.py tests/test_samse_gpu.py tests/test_paired_sw_gpu.py > gpurun_out/s11_tests.log 2>&1 || { tail -30 gpurun_out/s11_tests.log; exit 1; }
tail -2 gpurun_out/s11_tests.log
echo "=== pipe $(date +%T)"
bash tools/r04_pipe1.sh || exit 1
echo "=== done $(date +%T)"
