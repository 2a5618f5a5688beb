#!/usr/bin/env python3
"""Summarise rocprofv3 PC-sampling CSVs: samples per kernel, then per kernel the hottest code
offsets with their instruction text (and stall reason columns when present)."""
import csv
import collections
import glob
import sys

root = sys.argv[1]
files = [f for f in glob.glob(f"{root}/**/*.csv", recursive=True) if "pc_sampling" in f.lower() or "pc" in f.lower()]
print("files:", files)
for f in files:
    with open(f) as fh:
        r = csv.DictReader(fh)
        print(f, "columns:", r.fieldnames)
        rows = list(r)
    if not rows:
        continue
    kcol = next((c for c in r.fieldnames if "kernel" in c.lower() and "name" in c.lower()), None)
    pcol = next((c for c in r.fieldnames if c.lower() in ("pc_offset", "offset", "code_object_offset", "pc")), None)
    icol = next((c for c in r.fieldnames if c.lower().startswith("instruction") and "comment" not in c.lower()), None)
    ccol = next((c for c in r.fieldnames if "comment" in c.lower()), None)
    extra = [c for c in r.fieldnames if "stall" in c.lower() or "reason" in c.lower() or "issued" in c.lower()]
    print("kernel col", kcol, "pc col", pcol, "inst col", icol, "extra", extra, "rows", len(rows))
    byk = collections.Counter(x.get(kcol, "?")[:90] for x in rows)
    for k, v in byk.most_common(8):
        print(f"{v:9d} {k}")
    for k, _ in byk.most_common(3):
        sub = [x for x in rows if x.get(kcol, "?")[:90] == k]
        byp = collections.Counter((x.get(pcol), x.get(icol), x.get(ccol)) for x in sub)
        print("==", k, len(sub))
        for (pc, ins, cm), v in byp.most_common(120):
            print(f"{v:8d} {100.0 * v / len(sub):5.2f}% {pc} {ins} {cm or ''}")
        for c in extra:
            cnt = collections.Counter(x.get(c) for x in sub)
            print("  ", c, cnt.most_common(12))
