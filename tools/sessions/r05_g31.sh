# Round 5 (GPU box): where sampe's host CPU goes -- full-size pipeline, sampe -R -G 1 with per-phase
# CPU seconds (IBWA_PHASE_CPU), the next batch read without overlap (IBWA_SAMPE_SYNC_READ) and the
# positions pass split (IBWA_SAMPE_STATS)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export IBWA_PHASE_CPU=1 IBWA_SAMPE_SYNC_READ=1 IBWA_SAMPE_STATS=1
timeout -k 10 1000 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 2000 --concurrent-ends 0 --sampe-workers 1 --out gpurun_out/r05_pipe_cpu.json > gpurun_out/r05_pipe_cpu.log 2>&1 || { tail -30 gpurun_out/r05_pipe_cpu.log; exit 1; }
grep "cpu s:\|wall s:" gpurun_out/r05_pipe_cpu.log | grep sampe | head -4
