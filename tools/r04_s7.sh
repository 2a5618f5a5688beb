#!/bin/bash
# Round 4 (GPU box): which HIP runtime settings keep small copies / memsets off the CUs (they wait for
# a grid that holds every CU: tools/copy_under_load.hip), then sampe's tests and the pipeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in "X=0" "GPU_BLIT_ENGINE_TYPE=1" "GPU_BLIT_ENGINE_TYPE=2" "GPU_CP_DMA_COPY_SIZE=0" "GPU_CP_DMA_COPY_SIZE=64" "ROC_ENABLE_LARGE_BAR=1" "GPU_FORCE_BLIT_COPY_SIZE=0"; do
  echo "=== $e $(date +%T)"
  env $e timeout -k 10 90 ./tools/copy_under_load > gpurun_out/cul_$e.txt 2>&1 || { cat gpurun_out/cul_$e.txt; exit 1; }
  grep "under load" gpurun_out/cul_$e.txt
done
echo "=== gpu tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/sampe_tests.log 2>&1 || { tail -30 gpurun_out/sampe_tests.log; exit 1; }
tail -2 gpurun_out/sampe_tests.log
echo "=== pipe $(date +%T)"
bash tools/r04_pipe1.sh
echo "=== done $(date +%T)"
