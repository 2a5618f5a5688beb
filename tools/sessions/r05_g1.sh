set -o pipefail
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
(df -h /tmp "$TMPDIR" /dev/shm; mount | grep -E " on (/|/tmp|/dev/shm) ") > gpurun_out/r05_mounts.txt 2>&1 || true
timeout -k 10 150 tools/_build/fileread_bench --gb 8 > gpurun_out/r05_fileread.json 2> gpurun_out/r05_fileread.log && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_cli_gpu.py -m gpu > gpurun_out/r05_cli_tests.log 2>&1 && \
timeout -k 10 900 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse dev --host-parse-run 0 --ref-sample 0 --check 2000 --variants '[{"p2g_l2": {"IBWA_FQ_PIECE_BYTES": 2147483648}}, {"p3g_l2": {"IBWA_FQ_PIECE_BYTES": 3221225472}}, {"p3g_l1": {"IBWA_FQ_PIECE_BYTES": 3221225472, "IBWA_ALN_LANES": 1}}, {"p1g_l3": {"IBWA_ALN_LANES": 3}}]' --out gpurun_out/r05_e2e_a.json > gpurun_out/r05_e2e_a.log 2>&1
