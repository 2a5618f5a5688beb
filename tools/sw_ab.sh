#!/bin/bash
# Same-box A/B of two builds of libibwa_amd.so on tools/sw_bench.py (GPU box).
# usage: tools/sw_ab.sh <libA> <libB> <rounds>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A=$1; B=$2; R=$3
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    for s in 2 0; do
      IBWA_LIB=$lib IBWA_SW_STOP=$s timeout -k 10 300 python tools/sw_bench.py --steps 3 --cpu-sample 100 \
        > gpurun_out/swab_$v$r$s.json 2> gpurun_out/swab.log || { tail -5 gpurun_out/swab.log; exit 1; }
      echo "$v$r stop=$s $(python3 -c "import json;d=json.load(open('gpurun_out/swab_$v$r$s.json'));print(round(d['kernel_ms'],1))")"
    done
  done
done
