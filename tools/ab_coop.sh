#!/bin/bash
# Same-box A/B of the cooperative pass at 10M reads: the round-2 library (ibwa_amd_ab/), this tree
# with k_coop_roots off, and on; twice each, kernel times per step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
ARGS="--reads ${READS:-10000000} --steps 2 --warmup 1 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0"
for r in 1 2; do
  for v in A B C; do
    case $v in
      A) env="IBWA_LIB=ibwa_amd_ab/lib/libibwa_amd.so"; opt="" ;;
      B) env=""; opt="--opt coop_roots=0" ;;
      C) env=""; opt="--opt coop_roots=1" ;;
    esac
    env $env timeout -k 10 300 python3 bench.py $ARGS $opt > gpurun_out/ab/$v$r.json 2> gpurun_out/ab/$v$r.log \
      || { tail -5 gpurun_out/ab/$v$r.log; exit 1; }
    echo "$v$r $(python3 -c "import json;d=json.load(open('gpurun_out/ab/$v$r.json'));print(round(d['ms_per_step']),{k:round(v,1) for k,v in d['extra']['kernel_ms_per_step'].items()})")"
  done
done
