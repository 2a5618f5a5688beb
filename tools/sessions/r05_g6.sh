# Round 5 (GPU box): the CLI end to end at 50 M reads -- lanes / piece-size variants, phases split
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse dev --host-parse-run 0 --ref-sample 0 --check 2000 --variants '[{"l1_p3750m": {"IBWA_ALN_LANES": 1, "IBWA_FQ_PIECE_BYTES": 3932160000}}, {"l2_p1536m": {"IBWA_FQ_PIECE_BYTES": 1610612736}}, {"l2_default_again": {"IBWA_ALN_LANES": 2}}]' --out gpurun_out/r05_e2e_c.json > gpurun_out/r05_e2e_c.log 2>&1
