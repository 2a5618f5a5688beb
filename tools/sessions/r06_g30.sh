# Round 6 (GPU box): bench.py after adding the GPU-side touches (a short run: the line must still come out)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py --steps 2 --warmup 1 > gpurun_out/r06_bench_touch.json 2> gpurun_out/r06_bench_touch.log || { tail -30 gpurun_out/r06_bench_touch.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06_bench_touch.json'));r=d['roofline'];print(d['value'], {k:(round(v['touches_per_read'],1), v['gpu_touches_per_read'] and round(v['gpu_touches_per_read'],1)) for k,v in r['per_kernel'].items()}, r['touches_note'][:60])"
