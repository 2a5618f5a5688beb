#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sw_gpu.py tests/test_paired_sw_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sw.log 2>&1 || { tail -30 gpurun_out/t_sw.log; exit 1; }
tail -1 gpurun_out/t_sw.log
bash tools/r03_diag150.sh && bash tools/r03_pipe2.sh
