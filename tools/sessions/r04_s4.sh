#!/bin/bash
# Round 4 (GPU box): k_sw counters (r04_sw_pmc.json), the 150 bp bench shape's kernel trace + EA PMC
# (profiles r04_gapped150_*), the 150 bp resume-rule sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== sw pmc $(date +%T)"
bash tools/r04_sw_pmc.sh > gpurun_out/sw_pmc_r04.log 2>&1 || { tail -20 gpurun_out/sw_pmc_r04.log; exit 1; }
tail -c 700 gpurun_out/sw_pmc_r04.log; echo
echo "=== profile 150 $(date +%T)"
timeout -k 10 1000 bash tools/profile_round.sh r04 gapped150 --read-len 150 --sub 0.02 --reads 20000000 --steps 2 --warmup 2 \
  --no-cpu --sa2pos 0 --exact-leg 0 --sw-leg 0 > gpurun_out/prof_gapped150.log 2>&1 || { tail -20 gpurun_out/prof_gapped150.log; exit 1; }
grep -E "avg_ms|\"k_" gpurun_out/prof_gapped150.log | head -20
bash tools/r04_sweep150.sh
echo "=== done $(date +%T)"
