# Round 6 (GPU box): the whole -m gpu suite after pruning two options and reusing sampe/samse's SAM
# buffers, then the full-size configs[4] pipeline (sampe -G 1/2 rates)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g16.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g16.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g16.log
timeout -k 10 1100 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --out gpurun_out/r06_pipe_full_v3.json > gpurun_out/r06_pipe_full_v3.log 2>&1 || { tail -30 gpurun_out/r06_pipe_full_v3.log; exit 1; }
grep "both ends\|sequential ends\|sampe -R -G\|pipeline (ends\|sample " gpurun_out/r06_pipe_full_v3.log
grep "wall s" gpurun_out/r06_pipe_full_v3.log | grep "sampe\]" | head -2 | cut -c1-700
