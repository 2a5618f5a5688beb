#!/bin/bash
# Round 4 (GPU box): the resume hand-off rule at 150 bp / 2 % (configs[4]'s aln shape), one process,
# hits compared with the first config's
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
C='"" gap_resume_iters=1000 gap_resume_iters=1500 gap_resume_iters=3000 gap_resume_entries=150 gap_resume_entries=600 gap_resume_iters=1000,gap_resume_entries=150 gap_tail_lanes=32 ""'
echo "=== 150bp $(date +%T)"
eval timeout -k 10 600 python3 -u tools/sweep_inproc.py --reads 20000000 --read-len 150 --sub 0.02 --out gpurun_out/sweep150.jsonl $C > gpurun_out/sweep150.log 2>&1 || { tail -20 gpurun_out/sweep150.log; exit 1; }
cut -c1-260 gpurun_out/sweep150.log
echo "=== done $(date +%T)"
