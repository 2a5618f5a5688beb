#!/bin/bash
# GPU box: the whole -m gpu suite, then the PROF diagnostics at 10M reads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/diag1.sh
timeout -k 10 120 tools/_build/membench_w 4 100 > gpurun_out/membench_w.jsonl 2>&1; cat gpurun_out/membench_w.jsonl
