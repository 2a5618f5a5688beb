# Round 6 (GPU box): device footprint of the CLI -- configs[2] 50 M reads end to end at
# the default piece size, with first-pass chunks of 4 M / 2.75 M reads inside each group (resume-state
# and width buffers sized per chunk), and with 1.5 GiB pieces: align time and arena peak use
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/e2e_aln.py --reads 50000000 --configs 2 --parse "" --host-parse-run 0 --ref-sample 0 --check 2000 \
  --variants '[{"chunk4m": {"IBWA_CTX_OPTS": "gap_reads_per_chunk=4194304"}}, {"chunk2750k": {"IBWA_CTX_OPTS": "gap_reads_per_chunk=2818048"}}, {"piece1536m": {"IBWA_FQ_PIECE_BYTES": 1610612736}}, {"default_again": {}}]' \
  --out gpurun_out/r06_e2e_mem.json > gpurun_out/r06_e2e_mem.log 2>&1 || { tail -30 gpurun_out/r06_e2e_mem.log; exit 1; }
grep "variant\|reads/s\|arena" gpurun_out/r06_e2e_mem.log | tail -20
