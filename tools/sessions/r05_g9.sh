# Round 5 (GPU box): CLI GPU tests after the mapped-file ingest + shared parse scratch; the CLI end to
# end at 50 M reads (mapped file vs pinned buffers), one profiled run, one arena-traced run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fq_scratch_gpu.py tests/test_cli_gpu.py -m gpu > gpurun_out/r05_cli_tests_g9.log 2>&1 || { tail -30 gpurun_out/r05_cli_tests_g9.log; exit 1; }
timeout -k 10 1000 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse dev --host-parse-run 0 --ref-sample 0 --check 2000 --prof gpurun_out/r05_prof_cli --arena-trace gpurun_out/r05_arena_trace.log --variants '[{"pinned": {"IBWA_FQ_MMAP": 0}}, {"mmap_again": {"IBWA_FQ_MMAP": 1}}]' --out gpurun_out/r05_e2e_e.json > gpurun_out/r05_e2e_e.log 2>&1
rc=$?
T=$(find gpurun_out/r05_prof_cli -name '*kernel_trace.csv' 2>/dev/null | sort | tail -1)
[ -n "$T" ] && python tools/busy_timeline.py "$T" > gpurun_out/r05_prof_cli_busy.json
exit $rc
