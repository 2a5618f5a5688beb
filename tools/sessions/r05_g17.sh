# Round 5 (GPU box): the chunk overlap with double-buffered width rows (gap_overlap 1: no own k_width
# or gap_shadow replay for the overlapped cooperative pass) -- parity, then the bench workload
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_scale_properties.py -m gpu > gpurun_out/r05_parity_g17.log 2>&1 || { tail -30 gpurun_out/r05_parity_g17.log; exit 1; }
timeout -k 10 900 python tools/sweep_inproc.py --reads 50000000 --steps 2 --out gpurun_out/r05_sweep_ovl2.jsonl "" "gap_overlap=1" "gap_overlap=1,gap_overlap_chunks=5" "gap_overlap=2" "" "gap_overlap=1" > gpurun_out/r05_sweep_ovl2.log 2>&1
