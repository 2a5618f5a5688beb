#!/bin/bash
# 150 bp reads at 0.1 x GRCh37 (the pipeline's shape): kernel times of two builds, verbose pass stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/d150
ARGS="--reads 1000000 --read-len 150 --scale 0.1 --steps 2 --warmup 1 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0"
for v in A B; do
  lib=ibwa_amd_ab/lib/libibwa_amd.so; [ $v = B ] && lib=ibwa_amd/lib/libibwa_amd.so
  IBWA_LIB=$lib IBWA_VERBOSE=1 timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/d150/$v.json 2> gpurun_out/d150/$v.log || { tail -5 gpurun_out/d150/$v.log; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/d150/$v.json'));print(round(d['ms_per_step']),{k:round(v,1) for k,v in d['extra']['kernel_ms_per_step'].items()})")"
  grep "coop pass\|handed\|retry\|step 0" gpurun_out/d150/$v.log | head -6
done
