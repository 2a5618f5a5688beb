#!/bin/bash
# CLI tests (overlapped groups), then end-to-end configs[2] at 50M reads with 2 and 1 lanes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cli_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_cli.log 2>&1 || { tail -30 gpurun_out/t_cli.log; exit 1; }
tail -1 gpurun_out/t_cli.log
timeout -k 10 900 python3 -u tools/e2e_aln.py --reads ${READS:-50000000} --configs 2 --lanes 2,1 --ref-sample 0 \
  --out gpurun_out/e2e_50m.json 2> gpurun_out/e2e_50m.log || { tail -20 gpurun_out/e2e_50m.log; exit 1; }
grep "\[e2e\]" gpurun_out/e2e_50m.log | grep -v "cli: \[bwa_aln_core\]\|slice" | tail -20
