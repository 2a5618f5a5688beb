#!/bin/bash
# usage: tools/pmc_session.sh "<counters pass 1>" "<counters pass 2>" ...   (BENCH_ARGS env for bench.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 1 --warmup 0 --no-cpu}"
i=0
for pmc in "$@"; do
  i=$((i+1))
  echo "=== pmc[$i] $pmc $(date +%T)"
  timeout -k 10 600 rocprofv3 --pmc $pmc --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
done
