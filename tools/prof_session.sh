#!/bin/bash
# rocprofv3 passes over bench.py (kernel trace + stats; then PMC passes, each on its own).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu}"
echo "=== kernel-trace $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
tail -3 $OUT/trace.log
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $pmc | tr ' ' '_')
  echo "=== pmc $pmc $(date +%T)"
  timeout -k 10 600 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc_$tag -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu ${PMC_EXTRA} > $OUT/pmc_$tag.log 2>&1 || { tail -20 $OUT/pmc_$tag.log; exit 1; }
done
find $OUT -name "*.csv" | head -50
