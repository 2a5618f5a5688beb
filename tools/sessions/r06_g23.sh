# Round 6 (GPU box): k_coop's commit threshold (chains committed together: 32 vs 16 / 48 / 64) -- four
# builds of the library on the same 50 M-read bench step, one process each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
ARGS="--reads 50000000 --steps 2 --warmup 1 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0 --e2e-leg 0"
for v in main c48 c64 c16 main; do
  lib=ibwa_amd/lib/libibwa_amd.so; [ $v != main ] && lib=ibwa_amd_ab/$v/libibwa_amd.so
  IBWA_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.log || { tail -5 gpurun_out/ab/$v.log; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));print(round(d['ms_per_step']),{k:round(v,1) for k,v in d['extra']['kernel_ms_per_step'].items()}, d['extra']['parity']['ok'])")" | tee -a gpurun_out/ab/r06_commit_ab.txt
done
