#!/bin/bash
# Round 4 perf session (GPU box): A/B round-3 lib vs this tree at 10M reads, PC sampling of the -g
# build, then the round's profile of the bench workload (kernel trace, EA PMC, SQ) as r04_<tag>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== ab $(date +%T)"
bash tools/ab_libs.sh ibwa_amd_va/lib/libibwa_amd.so ibwa_amd/lib/libibwa_amd.so 1 || exit 1
echo "=== profile $(date +%T)"
bash tools/r04_profile.sh ${TAG:-gapped_v1} || exit 1
echo "=== done $(date +%T)"
