# Round 6 (GPU box): the pruned engine (no chunk overlap) -- scale properties (multi-chunk resume sets
# instead of the overlap ones) and parity; the depth / match-chain / unique-interval statistics of the
# search on the GRCh37-sized genome
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_scale_properties.py tests/test_gpu_parity.py tests/test_compat.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_gpu_tests_g2.log 2>&1 || { tail -40 gpurun_out/r06_gpu_tests_g2.log; exit 1; }
tail -2 gpurun_out/r06_gpu_tests_g2.log
timeout -k 10 600 python -u tools/depth_stats.py --out gpurun_out/r06_depth_stats_v2.json > gpurun_out/r06_depth_stats_v2.log 2>&1 || { tail -30 gpurun_out/r06_depth_stats_v2.log; exit 1; }
grep -v '"hist"' gpurun_out/r06_depth_stats_v2.log | head -90
timeout -k 10 900 python -u tools/gz_bench.py --reads 10000000 --out gpurun_out/r06_gz_bench.json > gpurun_out/r06_gz_bench.log 2>&1 || { tail -30 gpurun_out/r06_gz_bench.log; exit 1; }
grep gz_bench gpurun_out/r06_gz_bench.log
