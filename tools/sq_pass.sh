#!/bin/bash
# One SQ-counter rocprofv3 pass over a short gapped bench (issue vs wait breakdown per kernel).
# usage: tools/sq_pass.sh <tag> <bench args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/sq_$TAG
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
  --output-format csv -d $OUT/pmc -o run -- python3 bench.py "$@" > $OUT/run.json 2> $OUT/run.log || { tail -5 $OUT/run.log; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob(f"{out}/pmc/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        for h in ("k_gapped", "k_coop_roots", "k_coop", "k_width", "k_exact", "k_sw"):
            if h in name:
                agg[h][r["Counter_Name"]] += float(r["Counter_Value"])
                n[(h, r["Counter_Name"])] += 1
                break
for h, d in agg.items():
    print(h, {k: f"{v:.3g}" for k, v in sorted(d.items())})
PY
