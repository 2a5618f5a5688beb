# Round 5 (GPU box) at HEAD: every GPU test, the driver's bench command at its defaults, smoke()
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05_gpu_tests_final.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_final.log; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/r05_bench_v3.json 2> gpurun_out/r05_bench_v3.log || { tail -30 gpurun_out/r05_bench_v3.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke_final.log 2>&1
