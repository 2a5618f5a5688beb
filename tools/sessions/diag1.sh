#!/bin/bash
# k_coop / k_gapped diagnostics at 10M reads (GPU box): phase and idle-lane counters of the PROF
# kernel variants (IBWA_PROF_PHASES), then optionally an SQ counter pass (arg "sq").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/d1
ARGS="--reads ${READS:-10000000} --steps 1 --warmup 0 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0 $EXTRA"
IBWA_PROF_PHASES=1 IBWA_VERBOSE=1 timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/d1/prof.json 2> gpurun_out/d1/prof.log || exit 1
grep "k_coop\|coop pass\|k_gapped" gpurun_out/d1/prof.log
if [ "$1" = sq ]; then
  timeout -k 10 300 bash tools/sq_pass.sh d1 $ARGS > gpurun_out/d1/sq.txt 2>&1 || exit 1
  cat gpurun_out/d1/sq.txt
fi
