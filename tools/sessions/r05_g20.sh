# Round 5 (GPU box): what a process waits for right after another one released HBM -- alloc_bench
# holds then probes (the released amount vs the clean remainder), and the CLI back to back with the
# GPU runtime's start-up split from the arena reservation
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r05_alloc2.jsonl
: > $O
for hp in "133 133" "133 64" "200 80" "100 100"; do
  set -- $hp
  timeout -k 5 120 tools/_build/alloc_bench hold $1 >> $O || exit 1
  timeout -k 5 120 tools/_build/alloc_bench probe $2 8 >> $O || exit 1
  sleep 10
done
timeout -k 10 900 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse "" --host-parse-run 0 --ref-sample 0 --check 2000 --variants '[{"again": {}}, {"again2": {}}]' --out gpurun_out/r05_e2e_k.json > gpurun_out/r05_e2e_k.log 2>&1
