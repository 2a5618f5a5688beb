#!/bin/bash
# configs[4] shape on the full 3.1 Gbp genome (one GPU): 10 M pairs 2 x 150 bp at 2 %, aln x2 + sampe -R +
# samse, verbose (hipMalloc times, per-chunk passes) and with sampe's per-batch position counts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
IBWA_VERBOSE=1 IBWA_SAMPE_STATS=1 timeout -k 10 1000 python3 -u tools/pipeline_bench.py --scale 1.0 --pairs ${PAIRS:-10000000} \
  --sample 20000 --out gpurun_out/pipe_r04.json 2> gpurun_out/pipe_r04.log || { tail -20 gpurun_out/pipe_r04.log; exit 1; }
grep "\[pipeline\]" gpurun_out/pipe_r04.log | grep -v "batch of\|chunk at" | tail -30
