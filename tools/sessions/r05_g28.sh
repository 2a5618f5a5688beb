# Round 5 (GPU box): k_sw by pass -- forward only (IBWA_SW_STOP=1), forward + reverse (2), all (0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r05_sw_passes.jsonl
for stop in 1 2 0 1 2 0; do
  IBWA_SW_STOP=$stop timeout -k 10 300 python tools/sw_bench.py --pairs 200000 --steps 5 --cpu-sample 100 > gpurun_out/sw_one.json 2> gpurun_out/sw_one.log || { tail -5 gpurun_out/sw_one.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sw_one.json'));d['stop']=$stop;print(json.dumps(d))" >> gpurun_out/r05_sw_passes.jsonl
done
