#!/usr/bin/env python3
"""GPU busy time from a rocprofv3 kernel trace (CSV): the span from the first launch of a kernel
whose name matches --start to the end of the last kernel, the union of the kernels' intervals in it
(time at least one kernel ran), the idle gaps, and per kernel its summed duration.

  busy_timeline.py KERNEL_TRACE_CSV [--start k_width] [--gaps 12]
"""
import argparse
import csv
import json
import re
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--start", default="k_width", help="regex: the window starts at this kernel's first launch")
    ap.add_argument("--gaps", type=int, default=12)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    pat = re.compile(a.start)
    first = next((s for s, _, n in rows if pat.search(n)), None)
    if first is None:
        sys.exit(f"no kernel matches {a.start}")
    rows = [r for r in rows if r[1] > first]
    end = max(e for _, e, _ in rows)
    busy, gaps, cur_s, cur_e = 0, [], None, None
    for s, e, _ in rows:
        s = max(s, first)
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, (cur_e - first) / 1e6))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = {}
    for s, e, n in rows:
        k = re.sub(r"\(.*", "", n.replace("void ", "")).strip()
        k = re.sub(r"<.*", "", k)
        p = per.setdefault(k, [0, 0])
        p[0] += 1
        p[1] += e - max(s, first)
    gaps.sort(reverse=True)
    out = {"span_ms": (end - first) / 1e6, "busy_ms": busy / 1e6, "idle_ms": (end - first - busy) / 1e6,
           "n_gaps": len(gaps), "largest_gaps_ms_at_ms": [[g / 1e6, at] for g, at in gaps[:a.gaps]],
           "kernels_ms": {k: {"launches": v[0], "sum_ms": round(v[1] / 1e6, 1)}
                          for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
