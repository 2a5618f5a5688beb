#!/usr/bin/env python3
"""Stack pushes / pops / expansions by kind of entry on the bench's GRCh37-sized genome (GPU box:
the index is built on the device; the counting is the CPU restatement's instrumentation,
oracle.push_kinds).  Splits first-pass reads from the heavy reads the cooperative pass takes.
usage: tools/push_kinds.py [--reads 200000] [--normal 20000] [--heavy 2000]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=200_000)
    ap.add_argument("--normal", type=int, default=20_000)
    ap.add_argument("--heavy", type=int, default=2_000)
    a = ap.parse_args()
    import oracle
    from ibwa_amd import engine as E
    th = bench.host_threads()
    ascii_, codes, lens, _ = bench.make_genome(1_000_000, 1_000_000, 37, th)
    seq, off, lns = bench.make_reads(ascii_, lens, 3, a.reads, 100, 0.01, 0.05, th)
    eng = E.Engine(0)
    eng.build_index(codes)
    opt = E.parse_aln_args([])
    eng.aln(seq, off, lns, opt)
    ids, ps = eng.retry_info()
    heavy = np.sort(ids[ps == 1])
    normal = np.setdiff1d(np.arange(a.reads), ids)
    b0, b1 = bench.oracle_bwts(eng)
    oopt = bench.to_oracle_opt(opt)
    out = {"reads": a.reads, "heavy_fraction": heavy.size / a.reads}
    for tag, sel in (("normal", normal[:a.normal]), ("heavy", heavy[:a.heavy])):
        oracle.push_kinds(reset=True)
        oracle.cal_sa_reg_gap(b0, b1, seq, off[sel], lns[sel], oopt, n_threads=th)
        k = oracle.push_kinds(reset=True)
        n = max(sel.size, 1)
        out[tag] = {"n": int(sel.size), "per_read": {kk: [round(x / n, 1) for x in v] for kk, v in k.items()}}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
