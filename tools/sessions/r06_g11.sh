# Round 6 (GPU box): device footprint of the engine -- first-pass chunks of 4 M / 6.25 M
# reads against the default (16 M: 4 chunks of 12.5 M) in one process, smallest first so that each
# config's buffer total is its own; then k_coop's phase / idle-lane counters at 50 M reads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r06_sweep_chunk.jsonl "gap_reads_per_chunk=4194304" "gap_reads_per_chunk=6250000" "" "gap_reads_per_chunk=4194304" > gpurun_out/r06_sweep_chunk.log 2>&1 || { tail -20 gpurun_out/r06_sweep_chunk.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/r06_sweep_chunk.jsonl'):
    d=json.loads(l); print(d['config'], round(d['ms_per_step']), round(d['width']), round(d['gapped']), round(d['coop']), [round(x/1e9,1) for x in d['lib_bytes']], round(d['resume_records_peak']*16/1e9,1), d['hits_equal_first_config'])"
READS=50000000 bash tools/sessions/diag1.sh > gpurun_out/r06_diag1.log 2>&1 || { tail -20 gpurun_out/r06_diag1.log; exit 1; }
cat gpurun_out/r06_diag1.log
