# Round 5 (GPU box): process-exit cost with pinned host buffers / a large device allocation
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r05_exit.jsonl
: > $O
for args in "0 0 0" "4.5 0 0" "4.5 0 1" "0 232 0" "0 232 1" "4.5 232 0" "4.5 232 1"; do
  s=$(date +%s.%N)
  timeout -k 5 120 tools/_build/exit_bench $args > gpurun_out/exit_one.json || exit 1
  e=$(date +%s.%N)
  python3 -c "import json,sys; d=json.load(open('gpurun_out/exit_one.json')); d['process_wall_ms']=($e-$s)*1e3; print(json.dumps(d))" >> $O
  sleep 8
done
cat $O
