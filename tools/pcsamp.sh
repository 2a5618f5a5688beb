#!/bin/bash
# PC sampling of the gapped bench (GPU box): rocprofv3 stochastic PC samples of one configs[2]-shaped
# step (READS reads), summarised on the box per kernel and code offset (tools/pcsamp_summary.py).
# usage: tools/pcsamp.sh <lib> [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LIB=$1; TAG=${2:-pcs}
OUT=gpurun_out/$TAG
rm -rf $OUT; mkdir -p $OUT
IBWA_LIB=$LIB timeout -s KILL 600 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} \
  --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${INTERVAL:-1048576} --output-format csv -d $OUT/raw -o run \
  -- python3 bench.py --reads ${READS:-5000000} --steps 1 --warmup 0 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0 \
  > $OUT/run.json 2> $OUT/run.log || { tail -20 $OUT/run.log; ls -R $OUT/raw | head; exit 1; }
ls -la $(find $OUT/raw -type f) | head
python3 tools/pcsamp_summary.py $OUT/raw > $OUT/summary.txt || exit 1
head -60 $OUT/summary.txt
find $OUT/raw -name "*.csv" -size +20M -delete
