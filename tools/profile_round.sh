#!/bin/bash
# Per-round profile of a bench.py configuration (run on the GPU box):
#   1. rocprofv3 --kernel-trace --stats   (kernel durations; must agree with bench.py's HIP events)
#   2. two --pmc passes, each on its own (no tracing domains): L2<->fabric read/write requests
#      by size and the DRAM-bound share, per dispatch
# then tools/profile_summary.py writes profiles/<round>_<tag>_{kernel_stats.csv,pmc.json}.
# usage: tools/profile_round.sh <round> <tag> <bench args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROUND=$1; TAG=$2; shift 2
OUT=gpurun_out/prof_$TAG
rm -rf $OUT; mkdir -p $OUT
echo "=== kernel-trace $TAG $(date +%T)"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py "$@" \
  > $OUT/trace.json 2> $OUT/trace.log || { tail -20 $OUT/trace.log; exit 1; }
i=0
for pmc in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum" \
           "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum"; do
  i=$((i+1))
  echo "=== pmc[$i] $pmc $(date +%T)"
  timeout -k 10 900 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py "$@" \
    > $OUT/pmc$i.json 2> $OUT/pmc$i.log || { tail -20 $OUT/pmc$i.log; exit 1; }
done
python3 tools/profile_summary.py $OUT $ROUND $TAG
