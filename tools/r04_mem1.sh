#!/bin/bash
# Round 4 (GPU box): buffer use of the search at the bench shapes (extra.buffer_use, library bytes),
# then the configs[4] pipeline (aln x2 + sampe + samse) verbose.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--steps 1 --warmup 1 --no-cpu --exact-leg 0 --sw-leg 0 --sa2pos 0"
echo "=== mem100 $(date +%T)"
IBWA_VERBOSE=1 timeout -k 10 300 python3 bench.py $Q > gpurun_out/mem100.json 2> gpurun_out/mem100.log || { tail -20 gpurun_out/mem100.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/mem100.json'));e=d['extra'];print(d['ms_per_step'],e['device_memory_gb'],e['buffer_use'])"
echo "=== mem150 $(date +%T)"
IBWA_VERBOSE=1 timeout -k 10 300 python3 bench.py $Q --read-len 150 --sub 0.02 --reads 20000000 > gpurun_out/mem150.json 2> gpurun_out/mem150.log || { tail -20 gpurun_out/mem150.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/mem150.json'));e=d['extra'];print(d['ms_per_step'],e['device_memory_gb'],e['buffer_use'])"
echo "=== pipe $(date +%T)"
bash tools/r04_pipe1.sh
echo "=== done $(date +%T)"
