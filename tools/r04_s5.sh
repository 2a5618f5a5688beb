#!/bin/bash
# Round 4 (GPU box): CLI end to end at 50 M reads with the per-slice allocation time, then the
# k_sw counters, the 150 bp profile and the 150 bp resume-rule sweep (tools/r04_s4.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== e2e $(date +%T)"
timeout -k 10 800 python3 -u tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --ref-sample 0 --parse dev \
  --host-parse-run 0 --check 2000 --out gpurun_out/e2e_r04d.json 2> gpurun_out/e2e_r04d.log || { tail -20 gpurun_out/e2e_r04d.log; exit 1; }
grep -v "bwa_aln_core" gpurun_out/e2e_r04d.log | tail -22 | cut -c1-300
bash tools/r04_s4.sh
