#!/bin/bash
# Sweep the first pass's early hand-off (gap_early_iters / gap_early_entries) on the gapped bench.
# usage: tools/sweep_early.sh <reads> "<iters:entries[:budget[:coop_waves_per_cu[:gap_pages_per_block]]]> ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=$1; shift
for cfg in $@; do
  IFS=: read -r it en bud cw pp <<< "$cfg"; bud=${bud:-8000}; cw=${cw:-12}; pp=${pp:-384}
  timeout -k 10 400 python bench.py --aln "" --reads $N --steps 1 --warmup 1 --no-cpu --check 0 --sa2pos 0 \
    --opt gap_early_iters=$it --opt gap_early_entries=$en --opt gap_iter_budget=$bud --opt coop_waves_per_cu=$cw --opt gap_pages_per_block=$pp > gpurun_out/sw_$cfg.json 2> gpurun_out/sw_$cfg.log || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sw_$cfg.json')); e=d['extra']; print('$cfg', round(d['ms_per_step']), e['n_retry'], round(e['k_width_or_pack_ms']), round(e['k_search_ms']), round(e['retry_ms']), flush=True)"
done
