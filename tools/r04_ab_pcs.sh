#!/bin/bash
# Round 4: same-box A/B of the round-3 library (ibwa_amd_va) against this tree's at 10M reads, then
# PC sampling of this tree's -g build (ibwa_amd_vg) on one configs[2]-shaped step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_libs.sh ibwa_amd_va/lib/libibwa_amd.so ibwa_amd/lib/libibwa_amd.so ${ROUNDS:-2} || exit 1
[ "${PCS:-1}" = 1 ] || exit 0
bash tools/pcsamp.sh ibwa_amd_vg/lib/libibwa_amd.so pcs_r04 || exit 1
