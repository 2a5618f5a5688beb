# Round 5 (GPU box): the CLI end to end at 50 M reads after the ingest buffers are freed early;
# one aln run under rocprofv3 --kernel-trace (the GPU's busy time in the align phase); 3 lanes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse dev --host-parse-run 0 --ref-sample 0 --check 2000 --prof gpurun_out/r05_prof_cli --variants '[{"l3_p1g": {"IBWA_ALN_LANES": 3, "IBWA_FQ_PIECE_BYTES": 1073741824}}, {"l2_default_again": {"IBWA_ALN_LANES": 2}}]' --out gpurun_out/r05_e2e_d.json > gpurun_out/r05_e2e_d.log 2>&1
rc=$?
T=$(find gpurun_out/r05_prof_cli -name '*kernel_trace.csv' | head -1)
[ -n "$T" ] && python tools/busy_timeline.py "$T" > gpurun_out/r05_prof_cli_busy.json
exit $rc
