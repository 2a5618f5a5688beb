# Round 6 (GPU box): the first pass's tail and budget knobs and the staging room re-swept with the level
# tables (one process, 50 M reads, hits compared)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r06_sweep_knobs.jsonl "" "gap_tail_lanes=8" "gap_tail_lanes=32" "gap_tail_iters=100" "gap_tail_iters=400" "gap_iter_budget=6000" "gap_iter_budget=12000" "coop_stg_room=2" "" > gpurun_out/r06_sweep_knobs.log 2>&1 || { tail -20 gpurun_out/r06_sweep_knobs.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/r06_sweep_knobs.jsonl'):
    d=json.loads(l); print(d['config'], round(d['ms_per_step']), round(d['width']), round(d['gapped']), round(d['coop']), d['n_resumed'], d['hits_equal_first_config'])"
