#!/bin/bash
# Round 4 (GPU box), closing: the default bench line, the round's profile of it (kernel trace, EA PMC,
# SQ) as r04_gapped_v2, then the CLI end to end at 50 M reads with the GPU parse and the host parse
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "=== bench $(date +%T)"
timeout -k 10 600 python3 bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.log || { tail -20 gpurun_out/bench_final.log; exit 1; }
cut -c1-600 gpurun_out/bench_final.json
echo "=== profile $(date +%T)"
bash tools/r04_profile.sh gapped_v2 || exit 1
echo "=== e2e $(date +%T)"
timeout -k 10 800 python3 -u tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --ref-sample 0 --parse dev,host \
  --host-parse-run 1 --check 2000 --out gpurun_out/e2e_r04e.json 2> gpurun_out/e2e_r04e.log || { tail -20 gpurun_out/e2e_r04e.log; exit 1; }
grep -E "configs\[2\]:|device memory" gpurun_out/e2e_r04e.log | cut -c1-300
echo "=== done $(date +%T)"
