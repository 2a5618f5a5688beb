# Round 6 (GPU box): sampe's host CPU by phase at full size (IBWA_PHASE_CPU: process CPU seconds per
# phase; IBWA_SAMPE_STATS: the positions pass's split) -- configs[4] shape, -G 1 and -G 2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
IBWA_PHASE_CPU=1 IBWA_SAMPE_STATS=1 timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 2000 --concurrent-ends 0 --out gpurun_out/r06_pipe_cpu.json > gpurun_out/r06_pipe_cpu.log 2>&1 || { tail -30 gpurun_out/r06_pipe_cpu.log; exit 1; }
grep "cpu s:\|wall s:" gpurun_out/r06_pipe_cpu.log | grep sampe | cut -c1-900
