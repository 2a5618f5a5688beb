#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_scale_properties.py tests/test_gpu_parity.py tests/test_cli_gpu.py tests/test_sampe_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gg2.log 2>&1 || { tail -30 gpurun_out/t_gg2.log; exit 1; }
tail -2 gpurun_out/t_gg2.log
bash tools/ab_occ.sh "$@"
