#!/bin/bash
# k_sw at HEAD: kernel trace, then one SQ and one EA counter pass over tools/sw_bench.py (200 k rescues)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/swp
rm -rf $OUT; mkdir -p $OUT
ARGS="--pairs 200000 --steps 3 --cpu-sample 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/sw_bench.py $ARGS > $OUT/kt.json 2> $OUT/kt.log || { tail -5 $OUT/kt.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
  --output-format csv -d $OUT/sq -o run -- python3 tools/sw_bench.py $ARGS > $OUT/sq.json 2> $OUT/sq.log || { tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/sq2 -o run -- python3 tools/sw_bench.py $ARGS > $OUT/sq2.json 2> $OUT/sq2.log || { tail -5 $OUT/sq2.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
  --output-format csv -d $OUT/ea -o run -- python3 tools/sw_bench.py $ARGS > $OUT/ea.json 2> $OUT/ea.log || { tail -5 $OUT/ea.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
res = {}
for f in glob.glob(f"{out}/kt/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_sw" in r["Name"] or "k_pack_cigar" in r["Name"]:
            res.setdefault("kernel_stats", {})[r["Name"][:40]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
for tag in ("sq", "sq2", "ea"):
    agg = collections.defaultdict(float)
    calls = collections.Counter()
    for f in glob.glob(f"{out}/{tag}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_sw" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                calls[r["Counter_Name"]] += 1
    res[tag] = {k: v / max(1, calls[k]) for k, v in agg.items()}  # per launch
print(json.dumps(res))
PY
