#!/bin/bash
# k_sw at HEAD (round 6): kernel trace, then SQ and EA counter passes over tools/sw_bench.py (200 k rescues);
# writes gpurun_out/r06_sw_pmc.json in the form bench.py's sw_leg reads (build_id, window, read_len)
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
sys.path.insert(0, ".")
from ibwa_amd import engine as E
n = 200000
sq = res["sq"]; sq2 = res["sq2"]; ea = res["ea"]
ks = ([v for k, v in res.get("kernel_stats", {}).items() if "k_sw" in k] or [{"avg_ns": float("nan"), "calls": 0}])[0]
d = {"workload": "tools/sw_bench.py --pairs 200000 --steps 3: 200 k mate-rescue pairs, 510 bp window x 150 bp read "
                 "(k_sw local core + global fill + CIGAR), HEAD of round 6",
     "build_id": E.lib().ibwa_build_id().decode(), "window": 510, "read_len": 150,
     # digest of the sources k_sw is built from (bench.py sw_leg: a counter file of the same kernel code)
     "sw_src_digest": __import__("bench").sw_src_digest(),
     "k_sw_avg_ms": ks["avg_ns"] / 1e6, "k_sw_calls": ks["calls"],
     "per_launch": dict(sq, **sq2, **ea),
     "valu_wave_insts_per_alignment": sq["SQ_INSTS_VALU"] / n,
     "valu_fraction": sq["SQ_INSTS_VALU"] * 64 / (39.3216e12 * ks["avg_ns"] * 1e-9),
     "valu_peak_note": "39.32 T lane-ops/s = 256 CU x 4 SIMD x 16 lanes x 2.4 GHz; one wave64 VALU instruction = 64 lane-ops",
     "wait_any_fraction": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
     "active_inst_fraction": sq["SQ_ACTIVE_INST_ANY"] / sq["SQ_WAVE_CYCLES"],
     "ea_requests_per_alignment": {"rd": ea["TCC_EA0_RDREQ_sum"] / n, "wr": ea["TCC_EA0_WRREQ_sum"] / n,
                                   "wr64": ea["TCC_EA0_WRREQ_64B_sum"] / n},
     "source": "gpurun_out/swp (rocprofv3 --kernel-trace --stats, then --pmc passes: SQ x8, SQ/GRBM x4, TCC EA x3), tools/r06_sw_pmc.sh"}
json.dump(d, open("gpurun_out/r06_sw_pmc.json", "w"), indent=1)
print(json.dumps(d)[:600])
PY
