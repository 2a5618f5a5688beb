#!/bin/bash
# Build a variant of libibwa_amd.so from the current sources (or a patched copy) for same-box A/Bs
# and profiling: tools/mk_variant.sh <dir> [extra hipcc flags]  ->  <dir>/lib/libibwa_amd.so
# (<dir> is git-ignored; the .so travels to the GPU box with the tree).
set -e
cd "$(dirname "$0")/.."
D=$1; shift
case $D in ibwa_amd_v*) ;; *) echo "variant dirs are ibwa_amd_v* (git- and gpurun-ignored sources)"; exit 1;; esac
mkdir -p $D/csrc
rm -rf $D/csrc && mkdir -p $D/csrc && cp -a ibwa_amd/csrc/. $D/csrc/
make -s -C $D/csrc -j8 HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../../include $*" \
  ../lib/libibwa_amd.so
echo "$D/lib/libibwa_amd.so"
