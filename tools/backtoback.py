#!/usr/bin/env python3
"""Two `ibwa-amd aln` processes back to back (GPU box): how long the second one's device arena waits
after the first one exits, with the first one ending in different ways.  Small golden index and
reads; both processes reserve the same arena (IBWA_ARENA_GB) so the memory question is the same as
two full-size runs'.  One JSON line per case on stdout.
  backtoback.py [--arena-gb 118] [--cases fast,clean,sleep2,probe]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")
GOLD = os.path.join(ROOT, "tests", "golden")


def aln(env, out):
    t = time.perf_counter()
    r = subprocess.run([CLI, "aln", "-f", out, os.path.join(GOLD, "g1m"), os.path.join(GOLD, "reads_mixed.fq")],
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=300,
                       env=dict(os.environ, IBWA_ALN_TIMES="1", **env))
    wall = time.perf_counter() - t
    err = r.stderr.decode(errors="replace")
    if r.returncode:
        sys.exit(f"aln failed: {err[-1000:]}")
    ph = {}
    for ln in err.splitlines():
        m = re.search(r"arenas released in ([\d.]+) ms", ln)
        if m:
            ph["release_ms"] = float(m.group(1))
        if "wall s:" in ln:
            for name, v in re.findall(r"([a-z][a-z .()]*?) (\d+\.\d+)", ln.split("wall s:", 1)[1]):
                ph[name.strip()] = float(v)
    return wall, ph


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arena-gb", default="118")
    ap.add_argument("--cases", default="fast,clean,sleep2,release,fast")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    base = {"IBWA_ARENA_GB": a.arena_gb}
    for case in a.cases.split(","):
        first = dict(base)
        if case == "clean":
            first["IBWA_ALN_CLEAN_EXIT"] = "1"
        if case == "release":
            first["IBWA_ALN_RELEASE"] = "1"
        w1, p1 = aln(first, os.path.join(tmp, "a.sai"))
        if case == "sleep2":
            time.sleep(2.0)
        w2, p2 = aln(base, os.path.join(tmp, "b.sai"))
        print(json.dumps({"case": case, "arena_gb": a.arena_gb, "first": {"wall_s": w1, **p1},
                          "second": {"wall_s": w2, **p2}}), flush=True)
        time.sleep(12.0)  # the driver's wipe of both, before the next case
    subprocess.run(["rm", "-rf", tmp])


if __name__ == "__main__":
    main()
