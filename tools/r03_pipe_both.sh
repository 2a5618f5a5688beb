#!/bin/bash
# sampe/samse GPU tests, then the full-genome pipeline (PAIRS pairs) with sampe stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sampe_gpu.py tests/test_samse_gpu.py tests/test_paired_sw_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_pipe.log 2>&1 || { tail -30 gpurun_out/t_pipe.log; exit 1; }
tail -1 gpurun_out/t_pipe.log
bash tools/r03_pipe_full.sh
grep "paired_sw\]" gpurun_out/pipe_full.log | head -4
