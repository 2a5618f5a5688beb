#!/bin/bash
# aln timing inside the pipeline with 1 and 2 lanes (slice times, large allocations)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in 1 2; do
  IBWA_ALN_LANES=$L IBWA_ALN_TIMES=1 IBWA_VERBOSE=1 timeout -k 10 600 python3 -u tools/pipeline_bench.py --sample 2000 --out gpurun_out/pipe_l$L.json 2> gpurun_out/pipe_l$L.log || { tail -20 gpurun_out/pipe_l$L.log; exit 1; }
  echo "== lanes $L"; grep "\[pipeline\]" gpurun_out/pipe_l$L.log | grep "aln\|sampe\|pairs/s" | head -12
done
