set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_scale_properties.py tests/test_compat.py -m gpu > gpurun_out/r05_parity_g4.log 2>&1 || { tail -30 gpurun_out/r05_parity_g4.log; exit 1; }
READS=10000000 timeout -k 10 900 bash tools/ab_libs.sh ibwa_amd_va/lib/libibwa_amd.so ibwa_amd/lib/libibwa_amd.so 2 > gpurun_out/r05_ab_endread.log 2>&1
