# Round 6 (GPU box): k_width's leading steps from the level tables -- the width parity sets, then an
# in-process A/B at 50 M reads (hits compared)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "width_jump or level or smoke or goldens" > gpurun_out/r06_gpu_tests_g10.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g10.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g10.log
timeout -k 10 900 python -u tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r06_sweep_wtab.jsonl "" "width_tab=0" "" "width_tab=0" > gpurun_out/r06_sweep_wtab.log 2>&1 || { tail -20 gpurun_out/r06_sweep_wtab.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/r06_sweep_wtab.jsonl'):
    d=json.loads(l); print(d['config'], round(d['ms_per_step']), round(d['width']), round(d['gapped']), round(d['coop']), d['hits_equal_first_config'])"
