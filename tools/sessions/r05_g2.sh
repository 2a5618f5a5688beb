set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_scale_properties.py tests/test_compat.py -m gpu > gpurun_out/r05_parity_g2.log 2>&1 || { tail -30 gpurun_out/r05_parity_g2.log; exit 1; }
B=tools/_build/alloc_bench
O=gpurun_out/r05_alloc.jsonl
timeout -k 5 90 $B probe 192 8 > $O && \
timeout -k 5 90 $B hold 200 && timeout -k 5 90 $B probe 192 8 >> $O && \
timeout -k 5 90 $B hold 200 && sleep 5 && timeout -k 5 90 $B probe 192 8 >> $O && \
timeout -k 5 90 $B hold 200 && timeout -k 5 90 $B probe 192 192 >> $O && \
timeout -k 5 90 $B probe 192 192 >> $O && \
timeout -k 5 90 $B hold 100 && timeout -k 5 90 $B probe 48 8 >> $O && \
timeout -k 10 900 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse dev --host-parse-run 0 --ref-sample 0 --check 2000 --variants '[{"noarena": {"IBWA_ARENA_GB": 0}}, {"p2g_l2": {"IBWA_FQ_PIECE_BYTES": 2147483648}}, {"p3g_l2": {"IBWA_FQ_PIECE_BYTES": 3221225472}}, {"p3g_l1": {"IBWA_FQ_PIECE_BYTES": 3221225472, "IBWA_ALN_LANES": 1}}, {"p1g_l2_again": {"IBWA_ALN_LANES": 2}}]' --out gpurun_out/r05_e2e_b.json > gpurun_out/r05_e2e_b.log 2>&1 && \
READS=10000000 timeout -k 10 900 bash tools/ab_libs.sh ibwa_amd_va/lib/libibwa_amd.so ibwa_amd/lib/libibwa_amd.so 2 > gpurun_out/r05_ab_shadow.log 2>&1 && \
timeout -k 10 400 python -u tools/sweep_inproc.py --reads 50000000 --out gpurun_out/r05_sweep_overlap.jsonl "" gap_overlap=0 > gpurun_out/r05_sweep_overlap.log 2>&1
