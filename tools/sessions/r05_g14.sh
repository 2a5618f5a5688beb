# Round 5 (GPU box): where the CLI's ~0.25 s of process exit goes (IBWA_ALN_EXIT_PROBE: the teardown
# timed part by part before _exit); 1 GiB pieces (the <= 140 GB footprint) against the default
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse "" --host-parse-run 0 --ref-sample 0 --check 2000 --variants '[{"probe": {"IBWA_ALN_EXIT_PROBE": 1}}, {"p1g": {"IBWA_FQ_PIECE_BYTES": 1073741824}}, {"probe2": {"IBWA_ALN_EXIT_PROBE": 1}}, {"p1g_again": {"IBWA_FQ_PIECE_BYTES": 1073741824}}, {"again": {}}]' --out gpurun_out/r05_e2e_i.json > gpurun_out/r05_e2e_i.log 2>&1
