#!/bin/bash
# Round 4 (GPU box), closing check: the whole GPU suite and smoke() at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== gpu tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests_s12.log 2>&1 || { tail -30 gpurun_out/gpu_tests_s12.log; exit 1; }
tail -2 gpurun_out/gpu_tests_s12.log
echo "=== smoke $(date +%T)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s12.log 2>&1 || { tail -20 gpurun_out/smoke_s12.log; exit 1; }
tail -2 gpurun_out/smoke_s12.log
echo "=== done $(date +%T)"
