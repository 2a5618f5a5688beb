# Round 6 (GPU box): with the level tables in both passes -- same-process sweep at 50 M reads: the
# default (auto K = 13), K = 14, the hand-off rule (the first pass is cheaper now), hits compared
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r06_sweep_tab2.jsonl "" "coop_tab=0" "gap_tab_k=14" "gap_tab_k=0" "gap_resume_iters=3000,gap_resume_entries=500" "gap_resume_iters=4000,gap_resume_entries=1000" "gap_resume_iters=1500,gap_resume_entries=200" "" > gpurun_out/r06_sweep_tab2.log 2>&1 || { tail -20 gpurun_out/r06_sweep_tab2.log; exit 1; }
cat gpurun_out/r06_sweep_tab2.jsonl | python3 -c "import sys,json;[print(d['config'], round(d['ms_per_step']), round(d['gapped']), round(d['coop']), round(d['width']), d['n_resumed'], d['hits_equal_first_config']) for d in map(json.loads, sys.stdin)]"
