# Round 6 (GPU box): the level tables of the first pass (gap_tab_k) -- parity (goldens with tables,
# the 31 Mb scale sets incl. resume states carrying string-stored entries), then same-process timing at
# 50 M reads (tables off / K 10 / 12 / 13, hits compared), then the build before the tables against
# this one with tables off (same box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_properties.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g6.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g6.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g6.log
timeout -k 10 600 python -u tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r06_sweep_tab.jsonl "" "gap_tab_k=12" "gap_tab_k=10" "gap_tab_k=13" "" > gpurun_out/r06_sweep_tab.log 2>&1 || { tail -20 gpurun_out/r06_sweep_tab.log; exit 1; }
cat gpurun_out/r06_sweep_tab.jsonl | python3 -c "import sys,json;[print(d['config'], round(d['ms_per_step']), round(d['gapped']), round(d['coop']), round(d['width']), d['hits_equal_first_config']) for d in map(json.loads, sys.stdin)]"
READS=50000000 timeout -k 10 600 bash tools/ab_libs.sh ibwa_amd_ab/lib/libibwa_amd.so ibwa_amd/lib/libibwa_amd.so 1 > gpurun_out/r06_ab_tab.log 2>&1 || { tail -20 gpurun_out/r06_ab_tab.log; exit 1; }
cat gpurun_out/r06_ab_tab.log
