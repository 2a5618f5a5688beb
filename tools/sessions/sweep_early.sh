#!/bin/bash
# Sweep engine options on the gapped bench (one step after one warm-up, no CPU legs).
# usage: tools/sessions/sweep_early.sh <reads> "<key=val,key=val...>" ...   (an empty config is the default)
#   e.g. tools/sessions/sweep_early.sh 10000000 "" "gap_early_iters=2000,gap_early_entries=500" "gap_reads_per_chunk=16777216"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=$1; shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  opts=()
  IFS=, read -ra kv <<< "$cfg"
  for x in "${kv[@]}"; do [ -n "$x" ] && opts+=(--opt "$x"); done
  timeout -k 10 400 python bench.py --reads $N --steps 1 --warmup 1 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0 "${opts[@]}" \
    > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.log || { tail -5 gpurun_out/sweep_$i.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sweep_$i.json')); e=d['extra']; print('[$cfg]', round(d['ms_per_step']), 'heavy', e['n_heavy'], {k: round(v) for k, v in e['kernel_ms_per_step'].items()}, flush=True)"
done
