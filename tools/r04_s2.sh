#!/bin/bash
# Round 4 (GPU box): the CLI GPU tests (parse-ahead, views), the footprint-option sweep, then the CLI
# end to end at 50 M reads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== cli tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py > gpurun_out/cli_tests.log 2>&1 || { tail -30 gpurun_out/cli_tests.log; exit 1; }
tail -2 gpurun_out/cli_tests.log
bash tools/r04_sweep_mem.sh || exit 1
echo "=== e2e $(date +%T)"
timeout -k 10 800 python3 -u tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --ref-sample 0 --parse dev \
  --out gpurun_out/e2e_r04b.json 2> gpurun_out/e2e_r04b.log || { tail -20 gpurun_out/e2e_r04b.log; exit 1; }
grep -v "bwa_aln_core" gpurun_out/e2e_r04b.log | tail -30
echo "=== done $(date +%T)"
