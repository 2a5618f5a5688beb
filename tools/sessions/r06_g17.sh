# Round 6 (GPU box): the full-size configs[4] pipeline with the two ends at once at one lane per process
# (then two), sequential ends, sampe -G 1/2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 2000 --concurrent-lanes 1,2,1 --out gpurun_out/r06_pipe_full_v4.json > gpurun_out/r06_pipe_full_v4.log 2>&1 || { tail -30 gpurun_out/r06_pipe_full_v4.log; exit 1; }
grep "both ends\|sequential ends\|sampe -R -G\|pipeline (ends\|sample " gpurun_out/r06_pipe_full_v4.log
grep "wall s" gpurun_out/r06_pipe_full_v4.log | grep "aln" | cut -c1-330
