# Round 5 (GPU box): samse / sampe goldens after the overlapped host loading; the full-size configs[4]
# pipeline after the arena calibration and the two-groups-per-lane cut of small inputs (aln end 2
# against end 1)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sampe_gpu.py tests/test_samse_gpu.py tests/test_sw_gpu.py tests/test_paired_sw_gpu.py -m gpu > gpurun_out/r05_tests_g19.log 2>&1 || { tail -30 gpurun_out/r05_tests_g19.log; exit 1; }
timeout -k 10 300 python tools/sw_bench.py --pairs 200000 --steps 5 --cpu-sample 300 > gpurun_out/r05_sw_v4zero.json 2> gpurun_out/r05_sw_v4zero.log || { tail -5 gpurun_out/r05_sw_v4zero.log; exit 1; }
timeout -k 10 1000 python -u tools/pipeline_bench.py --scale 1.0 --pairs 10000000 --sample 20000 --out gpurun_out/r05_pipe_full_v3.json > gpurun_out/r05_pipe_full_v3.log 2>&1
