# Round 6 (GPU box): the whole -m gpu suite at HEAD (samse/sampe goldens incl. -G and stale cases
# after the round-5 rec_to_read / .pac extraction rewrites; the new compressed-input tests), the
# smoke, then the driver-default bench (with the new extra.e2e_gz)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_head.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_head.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_head.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_v1.json 2> gpurun_out/r06_bench_v1.log || { tail -30 gpurun_out/r06_bench_v1.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06_bench_v1.json'));e=d['extra'];print(d['value'], d['ms_per_step']);print(json.dumps(e.get('e2e_gz'))[:1500]);print(json.dumps({k:v for k,v in e.get('e2e',{}).items() if k in ('value','wall_s','parity')}))"
timeout -k 10 600 python -u tools/depth_stats.py --out gpurun_out/r06_depth_stats.json > gpurun_out/r06_depth_stats.log 2>&1 || { tail -30 gpurun_out/r06_depth_stats.log; exit 1; }
tail -60 gpurun_out/r06_depth_stats.log
