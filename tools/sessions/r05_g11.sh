# Round 5 (GPU box): all GPU tests at HEAD (copy-engine zeroing, k_sw in three pass kernels); same-box
# A/B of k_sw (fused at HEAD~ / split, compiler's registers / split, 3 waves per SIMD); the CLI end to
# end at 50 M reads with one profiled run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05_gpu_tests_g11.log 2>&1 || { tail -30 gpurun_out/r05_gpu_tests_g11.log; exit 1; }
: > gpurun_out/r05_sw_ab.jsonl
for r in 1 2; do
  for v in va vb main; do
    lib=ibwa_amd_$v/lib/libibwa_amd.so; [ $v = main ] && lib=ibwa_amd/lib/libibwa_amd.so
    IBWA_LIB=$lib timeout -k 10 300 python tools/sw_bench.py --pairs 200000 --steps 5 --cpu-sample 300 > gpurun_out/sw_one.json 2> gpurun_out/sw_one.log || { tail -5 gpurun_out/sw_one.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/sw_one.json'));d['lib']='$v';d['round']=$r;print(json.dumps(d))" >> gpurun_out/r05_sw_ab.jsonl
  done
done
timeout -k 10 1000 python tools/e2e_aln.py --reads 50000000 --configs 2 --lanes 2 --parse "" --host-parse-run 0 --ref-sample 0 --check 2000 --prof gpurun_out/r05_prof_cli2 --variants '[{"again": {}}]' --out gpurun_out/r05_e2e_f.json > gpurun_out/r05_e2e_f.log 2>&1
rc=$?
T=$(find gpurun_out/r05_prof_cli2 -name '*kernel_trace.csv' 2>/dev/null | sort | tail -1)
[ -n "$T" ] && python tools/busy_timeline.py "$T" > gpurun_out/r05_prof_cli2_busy.json
exit $rc
