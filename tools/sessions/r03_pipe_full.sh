#!/bin/bash
# configs[4] shape on the full 3.1 Gbp genome: 10 M pairs 2 x 150 bp at 2 %, aln x2 + sampe -R (one GPU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
IBWA_SAMPE_STATS=1 timeout -k 10 1000 python3 -u tools/pipeline_bench.py --scale 1.0 --pairs ${PAIRS:-10000000} --sample 20000 \
  --out gpurun_out/pipe_full.json 2> gpurun_out/pipe_full.log || { tail -20 gpurun_out/pipe_full.log; exit 1; }
grep "\[pipeline\]" gpurun_out/pipe_full.log | tail -14
