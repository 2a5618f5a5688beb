# Round 6 (GPU box): same-build profiles -- configs[2] bench step + the configs[1] exact leg: kernel
# trace and EA PMC passes (tools/profile_round.sh), one SQ pass; k_sw counters (r06_sw_pmc.json)
set -o pipefail
mkdir -p gpurun_out/r06_prof
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu --sa2pos 0 --sw-leg 0 --e2e-leg 0 --exact-steps 1"
bash tools/profile_round.sh r06 gapped $ARGS > gpurun_out/r06_prof/profile_round.log 2>&1 || { tail -20 gpurun_out/r06_prof/profile_round.log; exit 1; }
cp profiles/r06_gapped_* gpurun_out/r06_prof/ && \
bash tools/sq_pass.sh r06_gapped $ARGS > gpurun_out/r06_prof/sq.txt 2>&1 || { tail -20 gpurun_out/r06_prof/sq.txt; exit 1; }
bash tools/sessions/r06_sw_pmc.sh > gpurun_out/r06_prof/sw_pmc.log 2>&1 || { tail -20 gpurun_out/r06_prof/sw_pmc.log; exit 1; }
tail -c 600 gpurun_out/r06_prof/sw_pmc.log; echo
