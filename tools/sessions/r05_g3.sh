set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cli_gpu.py tests/test_sampe_gpu.py tests/test_scale_properties.py -m gpu > gpurun_out/r05_tests_g3.log 2>&1 || { tail -30 gpurun_out/r05_tests_g3.log; exit 1; }
timeout -k 10 900 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r05_bench_v1.json 2> gpurun_out/r05_bench_v1.log || { tail -30 gpurun_out/r05_bench_v1.log; exit 1; }
timeout -k 10 400 python -u tools/sweep_inproc.py --reads 50000000 --out gpurun_out/r05_sweep_overlap3.jsonl "" gap_overlap=1,gap_overlap_chunks=3 > gpurun_out/r05_sweep_overlap3.log 2>&1 || { tail -20 gpurun_out/r05_sweep_overlap3.log; exit 1; }
timeout -k 10 500 python -u tools/sweep_inproc.py --reads 20000000 --read-len 150 --sub 0.02 --out gpurun_out/r05_sweep_mem150.jsonl "" coop_pool_gb=10 > gpurun_out/r05_sweep_mem150.log 2>&1
