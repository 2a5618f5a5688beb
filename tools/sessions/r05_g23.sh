# Round 5 (GPU box): is it the single large allocation that waits after a released hold?  hold / probe
# 118 GiB as one block or as 8 GiB blocks
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r05_alloc4.jsonl
: > $O
for hp in "118 118" "118 8" "8 118" "8 8"; do
  set -- $hp
  timeout -k 5 120 tools/_build/alloc_bench hold 118 $1 >> $O || exit 1
  timeout -k 5 120 tools/_build/alloc_bench probe 118 $2 >> $O || exit 1
  sleep 12
done
