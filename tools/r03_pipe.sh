#!/bin/bash
# sampe / samse GPU tests, then the aln+sampe pipeline timing (tools/pipeline_bench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sampe_gpu.py tests/test_samse_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_pipe.log 2>&1 || { tail -30 gpurun_out/t_pipe.log; exit 1; }
tail -1 gpurun_out/t_pipe.log
IBWA_ALN_TIMES=1 IBWA_VERBOSE=1 timeout -k 10 900 python3 -u tools/pipeline_bench.py ${PIPE_ARGS:-} --out gpurun_out/pipe.json 2> gpurun_out/pipe.log || { tail -20 gpurun_out/pipe.log; exit 1; }
grep "\[pipeline\]" gpurun_out/pipe.log | tail -14
