# Round 6 (GPU box): the full-size configs[4] pipeline -- both ends' aln at once, then one after the
# other (.sai compared), sampe -R -G 1/2 with the landed read-ahead queue and tabulated pairing penalty
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --out gpurun_out/r06_pipe_full_v1.json > gpurun_out/r06_pipe_full_v1.log 2>&1 || { tail -30 gpurun_out/r06_pipe_full_v1.log; exit 1; }
grep "both ends\|sequential ends\|sampe -R -G\|pipeline (ends\|sample " gpurun_out/r06_pipe_full_v1.log
