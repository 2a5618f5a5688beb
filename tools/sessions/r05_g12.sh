# Round 5 (GPU box): resume parity after folding resume_fixup into k_coop; the bench workload with the
# memory knobs (K-mer K = 14, 10 GiB cooperative pool); the CLI end to end with variants that move
# the exit cost (pinned buffers, no arena, one lane) and one profiled run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_scale_properties.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05_parity_g12.log 2>&1 || { tail -30 gpurun_out/r05_parity_g12.log; exit 1; }
timeout -k 10 900 python tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r05_sweep_mem.jsonl "" "kmer_k=14" "coop_pool_gb=10" "kmer_k=14,coop_pool_gb=10" "" > gpurun_out/r05_sweep_mem.log 2>&1 || { tail -20 gpurun_out/r05_sweep_mem.log; exit 1; }
timeout -k 10 1000 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse "" --host-parse-run 0 --ref-sample 0 --check 2000 --prof gpurun_out/r05_prof_cli3 --variants '[{"pinned": {"IBWA_FQ_MMAP": 0}}, {"no_arena": {"IBWA_ARENA_GB": 0}}, {"one_lane": {"IBWA_ALN_LANES": 1}}, {"again": {}}]' --out gpurun_out/r05_e2e_g.json > gpurun_out/r05_e2e_g.log 2>&1
rc=$?
T=$(find gpurun_out/r05_prof_cli3 -name '*kernel_trace.csv' 2>/dev/null | sort | tail -1)
[ -n "$T" ] && python tools/busy_timeline.py "$T" > gpurun_out/r05_prof_cli3_busy.json
exit $rc
