#!/bin/bash
# gap groups: parity tests, then same-box A/B against ibwa_amd_ab (HEAD) with EA PMC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_properties.py tests/test_compat.py tests/test_cli_gpu.py tests/test_sampe_gpu.py tests/test_samse_gpu.py \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gg.log 2>&1 || { tail -30 gpurun_out/t_gg.log; exit 1; }
tail -2 gpurun_out/t_gg.log
PMC=1 bash tools/ab_libs.sh ibwa_amd_ab/lib/libibwa_amd.so ibwa_amd/lib/libibwa_amd.so 2
