# Round 5 (GPU box) at HEAD: the double-buffered overlap's hits after the claim-counter fix; the
# driver's bench command at its defaults (N=1, e2e / sw / exact legs); smoke()
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/sweep_inproc.py --reads 50000000 --steps 1 --out gpurun_out/r05_sweep_ovl3.jsonl "" "gap_overlap=1" > gpurun_out/r05_sweep_ovl3.log 2>&1 || { tail -20 gpurun_out/r05_sweep_ovl3.log; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/r05_bench_v2.json 2> gpurun_out/r05_bench_v2.log || { tail -30 gpurun_out/r05_bench_v2.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke.log 2>&1
