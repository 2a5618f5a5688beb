# Round 5 (GPU box): CLI tests after unmapping consumed regions; the CLI end to end (exit cost);
# the bench workload in 2 first-pass chunks of 25 M reads (more resume-state room) against 3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cli_gpu.py tests/test_fq_scratch_gpu.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05_tests_g15.log 2>&1 || { tail -30 gpurun_out/r05_tests_g15.log; exit 1; }
timeout -k 10 900 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse "" --host-parse-run 0 --ref-sample 0 --check 2000 --variants '[{"probe": {"IBWA_ALN_EXIT_PROBE": 1}}, {"again": {}}]' --out gpurun_out/r05_e2e_j.json > gpurun_out/r05_e2e_j.log 2>&1 || { tail -20 gpurun_out/r05_e2e_j.log; exit 1; }
timeout -k 10 900 python tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r05_sweep_chunk.jsonl "" "gap_reads_per_chunk=25000000,gap_resume_gb=72" "" "gap_reads_per_chunk=25000000,gap_resume_gb=72" > gpurun_out/r05_sweep_chunk.log 2>&1
