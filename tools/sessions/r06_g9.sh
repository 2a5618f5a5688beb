# Round 6 (GPU box): auto level-table K 14, cooperative pass on Occ blocks -- the whole -m gpu suite,
# then the driver-default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g9.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g9.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g9.log
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_v3.json 2> gpurun_out/r06_bench_v3.log || { tail -30 gpurun_out/r06_bench_v3.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06_bench_v3.json'));e=d['extra'];print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], e['kernel_ms_per_step']);print({k:e[k].get('value') for k in ('e2e','e2e_gz','exact_leg') if isinstance(e.get(k),dict)}, e['parity']['ok'])"
