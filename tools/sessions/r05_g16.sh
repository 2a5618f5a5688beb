# Round 5 (GPU box) at HEAD: profiles of the configs[2] bench workload -- kernel trace + EA PMC passes
# (tools/profile_round.sh) and one SQ pass -- and the full-size configs[4] pipeline (aln end 1 / end 2
# with the smaller footprint, sampe -R, samse)
set -o pipefail
mkdir -p gpurun_out/r05_prof2
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu --exact-leg 0 --sa2pos 0 --sw-leg 0 --e2e-leg 0"
bash tools/profile_round.sh r05 gapped_v2 $ARGS > gpurun_out/r05_prof2/profile_round.log 2>&1 || { tail -20 gpurun_out/r05_prof2/profile_round.log; exit 1; }
cp profiles/r05_gapped_v2_* gpurun_out/r05_prof2/ && \
bash tools/sq_pass.sh r05_gapped_v2 $ARGS > gpurun_out/r05_prof2/sq.txt 2>&1
timeout -k 10 900 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --out gpurun_out/r05_pipe_full_v2.json > gpurun_out/r05_pipe_full_v2.log 2>&1
