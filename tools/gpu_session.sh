#!/bin/bash
# One GPU-box session: each GPU step has its own time limit; stop at the first failure.
# usage: tools/gpu_session.sh [tests] [smallbench] [bench] [prof]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  echo "=== $step $(date +%T)"
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_tests.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log ;;
    smallbench) timeout -k 10 400 python bench.py --scale 0.05 --reads 1000000 --steps 2 --warmup 1 --cpu-budget 5 --heavy-budget 5 --exact-reads 1000000 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.log; rc=$?; tail -8 gpurun_out/bench_small.log; cat gpurun_out/bench_small.json ;;
    bench) timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log; rc=$?; tail -8 gpurun_out/bench.log; cat gpurun_out/bench.json ;;
    bench20) timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.log; rc=$?; tail -8 gpurun_out/bench20.log; cat gpurun_out/bench20.json ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "=== $step rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
