#!/bin/bash
# Round 4 (GPU box): CLI end to end at 50 M reads with the GPU FASTQ parse (parse-only rates of the
# device and host paths, then aln with each), then the 150 bp / 2 % bench line (configs[4]'s aln shape).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== e2e $(date +%T)"
timeout -k 10 800 python3 -u tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --ref-sample 0 \
  --out gpurun_out/e2e_r04.json 2> gpurun_out/e2e_r04.log || { tail -20 gpurun_out/e2e_r04.log; exit 1; }
tail -5 gpurun_out/e2e_r04.log
echo "=== bench150 $(date +%T)"
timeout -k 10 360 python3 bench.py --read-len 150 --sub 0.02 --reads ${R150:-20000000} --steps 2 --warmup 1 \
  --exact-leg 0 --sw-leg 0 > gpurun_out/bench150.json 2> gpurun_out/bench150.log || { tail -20 gpurun_out/bench150.log; exit 1; }
cat gpurun_out/bench150.json
echo "=== done $(date +%T)"
