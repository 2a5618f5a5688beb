#!/bin/bash
# Same-box A/B of two builds of libibwa_amd.so on the configs[2] bench (GPU box).
# usage: tools/ab_bench.sh <libA> <libB> <rounds> [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; B=$2; R=$3; shift 3
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    IBWA_LIB=$lib timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu --exact-leg 0 --sa2pos 0 "$@" \
      > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.log || { tail -5 gpurun_out/ab_$v$r.log; exit 1; }
    echo "$v$r $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$v$r.json'));print(round(d['ms_per_step']),d['extra']['kernel_ms_per_step'])")"
  done
done
