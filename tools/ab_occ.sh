#!/bin/bash
# same-box k_coop A/B across builds and waves per CU: "label lib waves" triples on the command line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
ARGS="--reads ${READS:-10000000} --steps 2 --warmup 1 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0"
for r in 1 2; do
  set -- "${@}"
  i=0; arr=("$@")
  while [ $i -lt ${#arr[@]} ]; do
    lab=${arr[$i]}; lib=${arr[$((i+1))]}; w=${arr[$((i+2))]}; i=$((i+3))
    IBWA_LIB=$lib timeout -k 10 300 python3 bench.py $ARGS --opt coop_waves_per_cu=$w > gpurun_out/occ/$lab$r.json 2> gpurun_out/occ/$lab$r.log \
      || { tail -5 gpurun_out/occ/$lab$r.log; exit 1; }
    echo "$lab$r $(python3 -c "import json;d=json.load(open('gpurun_out/occ/$lab$r.json'));print(round(d['ms_per_step']),{k:round(v,1) for k,v in d['extra']['kernel_ms_per_step'].items()})")"
  done
done
