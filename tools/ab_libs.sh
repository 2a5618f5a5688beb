#!/bin/bash
# Same-box A/B of two builds of libibwa_amd.so on the gapped bench (10M reads by default), then one
# EA PMC pass (read / write requests) per build.  usage: tools/ab_libs.sh <libA> <libB> [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
A=$1; B=$2; R=${3:-2}
mkdir -p gpurun_out/ab
ARGS="--reads ${READS:-10000000} --steps 2 --warmup 1 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0 --e2e-leg 0 $EXTRA"
for r in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    IBWA_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab/$v$r.json 2> gpurun_out/ab/$v$r.log \
      || { tail -5 gpurun_out/ab/$v$r.log; exit 1; }
    echo "$v$r $(python3 -c "import json;d=json.load(open('gpurun_out/ab/$v$r.json'));print(round(d['ms_per_step']),{k:round(v,1) for k,v in d['extra']['kernel_ms_per_step'].items()})")"
  done
done
[ "$PMC" = 1 ] || exit 0
for v in A B; do
  lib=$A; [ $v = B ] && lib=$B
  IBWA_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv \
    -d gpurun_out/ab/pmc_$v -o run -- python3 bench.py --reads ${READS:-10000000} --steps 1 --warmup 0 --no-cpu --exact-leg 0 \
    --sa2pos 0 --sw-leg 0 > gpurun_out/ab/pmc_$v.log 2>&1 || { tail -5 gpurun_out/ab/pmc_$v.log; exit 1; }
  for k in k_gapped k_coop k_width; do
    echo "$v $(python3 tools/pmc_summary.py gpurun_out/ab/pmc_$v $k | tr '\n' ' ')"
  done
done
