# Round 5 (GPU box): sampe after the positions-pass changes (position-only radix key without
# remapping, sorted gather into the store, per-thread scratch): sampe GPU tests, then the full-size
# pipeline with sampe -R at -G 1 and 2 (SAM digests compared), per-phase CPU seconds
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sampe_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05_sampe_tests_g32.log 2>&1 || { tail -30 gpurun_out/r05_sampe_tests_g32.log; exit 1; }
tail -1 gpurun_out/r05_sampe_tests_g32.log
export IBWA_PHASE_CPU=1
timeout -k 10 1000 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --concurrent-ends 0 --sampe-workers 1,2 --out gpurun_out/r05_pipe_full_v7.json > gpurun_out/r05_pipe_full_v7.log 2>&1 || { tail -30 gpurun_out/r05_pipe_full_v7.log; exit 1; }
grep "sampe -R -G\|sampe SAM equal" gpurun_out/r05_pipe_full_v7.log
