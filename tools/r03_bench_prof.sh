#!/bin/bash
# the driver's bench command at HEAD, then the round-3 profile passes (kernel trace, EA PMC, SQ)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-v2}
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['roofline']);print(d['extra'].get('kernel_ms_per_step'))"
bash tools/r03_profile.sh gapped_$TAG
