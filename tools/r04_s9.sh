#!/bin/bash
# Round 4 (GPU box): sampe / samse tests, the configs[4] pipeline, the CLI end to end (GPU parse)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== sampe tests $(date +%T)"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_sampe_gpu.py tests/test_samse_gpu.py tests/test_cli_gpu.py > gpurun_out/s9_tests.log 2>&1 || { tail -30 gpurun_out/s9_tests.log; exit 1; }
tail -2 gpurun_out/s9_tests.log
echo "=== pipe $(date +%T)"
bash tools/r04_pipe1.sh || exit 1
echo "=== e2e $(date +%T)"
timeout -k 10 800 python3 -u tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --ref-sample 0 --parse dev \
  --host-parse-run 0 --check 2000 --out gpurun_out/e2e_r04f.json 2> gpurun_out/e2e_r04f.log || { tail -20 gpurun_out/e2e_r04f.log; exit 1; }
grep -E "configs\[2\]:|input parse|parsed on" gpurun_out/e2e_r04f.log | cut -c1-300
echo "=== done $(date +%T)"
