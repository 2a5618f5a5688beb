# Round 6 (GPU box): final HEAD -- the whole -m gpu suite and the driver-default bench,
# then the full-size configs[4] pipeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g21.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g21.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g21.log
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_v6.json 2> gpurun_out/r06_bench_v6.log || { tail -30 gpurun_out/r06_bench_v6.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06_bench_v6.json'));e=d['extra'];print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic_source'], e['kernel_ms_per_step']);print({k:e[k].get('value') for k in ('e2e','e2e_gz','exact_leg') if isinstance(e.get(k),dict)}, e['parity']['ok'], e['e2e'].get('arena_peak_use_gb'), e['sw_leg']['roofline'])"
timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --out gpurun_out/r06_pipe_full_v7.json > gpurun_out/r06_pipe_full_v7.log 2>&1 || { tail -30 gpurun_out/r06_pipe_full_v7.log; exit 1; }
grep "both ends\|sequential ends\|sampe -R -G\|pipeline (ends\|sample \|peak use" gpurun_out/r06_pipe_full_v7.log
