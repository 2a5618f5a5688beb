#!/bin/bash
# random-access calibration: plain timing, then FETCH_SIZE and EA request counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/membench
mkdir -p $OUT
timeout -k 10 300 tools/_build/membench 2 200 > $OUT/plain.jsonl 2> $OUT/plain.err || exit 1
cat $OUT/plain.jsonl
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
grep -oE "TCC_EA0_RDREQ[A-Z0-9_]*|TCC_EA_RDREQ[A-Z0-9_]*|TCC_BUBBLE[A-Z0-9_]*|TCC_REQ[A-Z0-9_]*" $OUT/counters_list.txt | sort -u | head -40
for pmc in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pmc | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc_$tag -o run -- tools/_build/membench 2 200 > $OUT/pmc_$tag.log 2>&1 || exit 1
done
