#!/bin/bash
# Round-3 check on the GPU box: coop parity tests + CLI tests, PROF diagnostics, a small bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scale_properties.py tests/test_gpu_parity.py tests/test_cli_gpu.py -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
bash tools/diag1.sh || exit 1
timeout -k 10 400 python bench.py --scale 0.1 --reads 2000000 --steps 2 --warmup 1 --cpu-budget 5 --heavy-budget 5 \
  --ref-budget 5 --exact-reads 1000000 --sw-leg 20000 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.log \
  || { tail -20 gpurun_out/bench_small.log; exit 1; }
tail -4 gpurun_out/bench_small.log
