#!/bin/bash
# Round-3 profile of the bench workload (GPU box): kernel trace + two EA PMC passes
# (tools/profile_round.sh -> profiles/r03_<tag>_*), then one SQ pass (issue / wait / VALU per kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-gapped_v1}
ARGS="--steps 2 --warmup 1 --no-cpu --sa2pos 0"
timeout -k 10 1100 bash tools/profile_round.sh r03 $TAG $ARGS > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
grep -E "avg_ms|\"k_" gpurun_out/prof_$TAG.log | head -40
timeout -k 10 400 bash tools/sq_pass.sh $TAG $ARGS > gpurun_out/sq_$TAG.txt 2>&1 || { tail -5 gpurun_out/sq_$TAG.txt; exit 1; }
cat gpurun_out/sq_$TAG.txt
