# Round 5 (GPU box): the CLI's memory knobs at 50 M reads -- K-mer table K, first-pass static slots,
# cooperative pool, piece size -- their align time and device-memory peak
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse "" --host-parse-run 0 --ref-sample 0 --check 2000 --variants '[{"k14": {"IBWA_CTX_OPTS": "kmer_k=14"}}, {"cap1_2048": {"IBWA_CTX_OPTS": "gap_resume_cap1=2048"}}, {"pool10": {"IBWA_CTX_OPTS": "coop_pool_gb=10"}}, {"all3": {"IBWA_CTX_OPTS": "kmer_k=14,gap_resume_cap1=2048,coop_pool_gb=10"}}, {"all3_p1536m": {"IBWA_CTX_OPTS": "kmer_k=14,gap_resume_cap1=2048,coop_pool_gb=10", "IBWA_FQ_PIECE_BYTES": 1610612736}}, {"base_again": {}}]' --out gpurun_out/r05_e2e_mem.json > gpurun_out/r05_e2e_mem.log 2>&1
