# Round 5 (GPU box): all GPU tests at HEAD (K-mer K <= 14, cooperative pool by read length, staged
# pageable H2D, fetch_sai); the CLI end to end at 50 M reads (exit cost after the staged copies;
# 3 GiB pieces = 4 groups), one profiled run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05_gpu_tests_g13.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_g13.log; exit 1; }
timeout -k 10 1000 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse dev --host-parse-run 0 --ref-sample 0 --check 2000 --prof gpurun_out/r05_prof_cli4 --variants '[{"p3g": {"IBWA_FQ_PIECE_BYTES": 3221225472, "IBWA_ARENA_GB": 250}}, {"p2g5": {"IBWA_FQ_PIECE_BYTES": 2684354560, "IBWA_ARENA_GB": 240}}, {"again": {}}]' --out gpurun_out/r05_e2e_h.json > gpurun_out/r05_e2e_h.log 2>&1
rc=$?
T=$(find gpurun_out/r05_prof_cli4 -name '*kernel_trace.csv' 2>/dev/null | sort | tail -1)
[ -n "$T" ] && python tools/busy_timeline.py "$T" > gpurun_out/r05_prof_cli4_busy.json
exit $rc
