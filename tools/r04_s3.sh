#!/bin/bash
# Round 4 (GPU box): the GPU suite, the CLI end to end at 50 M reads (GPU parse ahead), the configs[4]
# pipeline with sampe's finer phases
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== gpu tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests_s3.log 2>&1 || { tail -40 gpurun_out/gpu_tests_s3.log; exit 1; }
tail -2 gpurun_out/gpu_tests_s3.log
echo "=== e2e $(date +%T)"
timeout -k 10 800 python3 -u tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --ref-sample 0 --parse dev \
  --out gpurun_out/e2e_r04c.json 2> gpurun_out/e2e_r04c.log || { tail -20 gpurun_out/e2e_r04c.log; exit 1; }
grep -v "bwa_aln_core" gpurun_out/e2e_r04c.log | tail -32
echo "=== pipe $(date +%T)"
bash tools/r04_pipe1.sh
echo "=== done $(date +%T)"
