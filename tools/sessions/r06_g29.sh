# Round 6 (GPU box): the driver's bench command at the final tree (20 steps, 5 warm-up)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_final.json 2> gpurun_out/r06_bench_final.log || { tail -30 gpurun_out/r06_bench_final.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06_bench_final.json'));e=d['extra'];print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic_source'], e['kernel_ms_per_step']);print({k:e[k].get('value') for k in ('e2e','e2e_gz','exact_leg') if isinstance(e.get(k),dict)}, e['parity']['ok'], e['sw_leg']['roofline'].get('frac'), e['sw_leg']['roofline'].get('source'))"
