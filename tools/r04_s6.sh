#!/bin/bash
# Round 4 (GPU box): copies and memsets next to a grid that holds every CU, then tools/r04_s4.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== copy under load $(date +%T)"
timeout -k 10 90 ./tools/copy_under_load > gpurun_out/copy_under_load.txt 2>&1 || { cat gpurun_out/copy_under_load.txt; exit 1; }
cat gpurun_out/copy_under_load.txt
bash tools/r04_s4.sh
