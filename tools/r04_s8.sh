#!/bin/bash
# Round 4 (GPU box), last: the GPU suite at HEAD, then the configs[4] pipeline (sampe's reader in bulk)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== gpu tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests_s8.log 2>&1 || { tail -30 gpurun_out/gpu_tests_s8.log; exit 1; }
tail -2 gpurun_out/gpu_tests_s8.log
echo "=== smoke $(date +%T)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s8.log 2>&1 || { tail -20 gpurun_out/smoke_s8.log; exit 1; }
tail -3 gpurun_out/smoke_s8.log
echo "=== pipe $(date +%T)"
bash tools/r04_pipe1.sh
echo "=== done $(date +%T)"
