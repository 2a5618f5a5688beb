# Round 5 (GPU box): the largest allocation a process gets without waiting right after a process of
# the same size exited (alloc_bench hold X, then probe X)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r05_alloc3.jsonl
: > $O
for x in 112 120 126 104; do
  timeout -k 5 120 tools/_build/alloc_bench hold $x >> $O || exit 1
  timeout -k 5 120 tools/_build/alloc_bench probe $x 8 >> $O || exit 1
  sleep 12
done
