# Round 6 (GPU box): k_coop's one-row exact-tail jump -- goldens through the heavy-read pass with the
# jump on / off, the 31 Mb oracle sets, then an in-process A/B at 50 M reads (hits compared)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_properties.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g13.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g13.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g13.log
timeout -k 10 900 python -u tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r06_sweep_cjump.jsonl "" "coop_jump=0" "" "coop_jump=0" > gpurun_out/r06_sweep_cjump.log 2>&1 || { tail -20 gpurun_out/r06_sweep_cjump.log; exit 1; }
python -c "
import json
for l in open('gpurun_out/r06_sweep_cjump.jsonl'):
    d=json.loads(l); print(d['config'], round(d['ms_per_step']), round(d['width']), round(d['gapped']), round(d['coop']), d['hits_equal_first_config'])"
