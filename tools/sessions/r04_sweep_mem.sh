#!/bin/bash
# Round 4 (GPU box): what the footprint options cost in time (one process per read shape, hits
# compared with the first config's): static slots 2048, half the first-pass pool, a one-chain
# staging ring, half-size chunks, a 10 GiB cooperative pool
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
C='"" gap_resume_cap1=2048 gap_resume_ppb=48 coop_stg_room=1 gap_reads_per_chunk=8388608 coop_pool_gb=10 gap_resume_cap1=2048,gap_resume_ppb=48,coop_stg_room=1 ""'
echo "=== 100bp $(date +%T)"
eval timeout -k 10 500 python3 -u tools/sweep_inproc.py --reads 50000000 --out gpurun_out/sweep_mem100.jsonl $C > gpurun_out/sweep_mem100.log 2>&1 || { tail -20 gpurun_out/sweep_mem100.log; exit 1; }
cat gpurun_out/sweep_mem100.log | cut -c1-400
echo "=== 150bp $(date +%T)"
eval timeout -k 10 500 python3 -u tools/sweep_inproc.py --reads 20000000 --read-len 150 --sub 0.02 --out gpurun_out/sweep_mem150.jsonl $C > gpurun_out/sweep_mem150.log 2>&1 || { tail -20 gpurun_out/sweep_mem150.log; exit 1; }
cat gpurun_out/sweep_mem150.log | cut -c1-400
echo "=== done $(date +%T)"
