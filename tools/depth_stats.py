#!/usr/bin/env python3
"""Where bwt_match_gap's rank queries fall by depth (VERDICT r05 "next round" #1): on the bench's
GRCh37-sized genome (GPU box: the index is built on the device), the CPU restatement's expansions,
pops and exact-tail steps by the depth of the node (BWT steps from the root = the length of the
node's reference string), for the reads the first pass resolves and for the heavy reads the
cooperative pass takes.  Also: what fraction of the GPU's round trips (one per pop, one per tail step)
is at a depth < K -- nodes whose SA interval is a pure function of their string, so a table of all
strings of length <= K answers them.
usage: tools/depth_stats.py [--reads 200000] [--normal 20000] [--heavy 2000] [--out FILE]"""
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
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import oracle
    from ibwa_amd import engine as E
    th = bench.host_threads()
    den = 1_000_000
    ascii_, codes, lens, _ = bench.make_genome(int(round(a.scale * den)), den, 37, th)
    seq, off, lns = bench.make_reads(ascii_, lens, 3, a.reads, 100, 0.01, 0.05, th)
    eng = E.Engine(0)
    eng.build_index(codes)
    del codes
    opt = E.parse_aln_args([])
    eng.aln(seq, off, lns, opt)
    ids, ps = eng.retry_info()
    heavy = np.sort(ids[ps >= 1])
    normal = np.setdiff1d(np.arange(a.reads), ids)
    b0, b1 = bench.oracle_bwts(eng)
    oopt = bench.to_oracle_opt(opt)
    out = {"reads": a.reads, "heavy_fraction": heavy.size / a.reads, "genome_bp": int(sum(lens))}
    for tag, sel in (("normal", normal[:a.normal]), ("heavy", heavy[:a.heavy])):
        oracle.push_kinds(reset=True)
        oracle.cal_sa_reg_gap(b0, b1, seq, off[sel], lns[sel], oopt, n_threads=th)
        h = oracle.depth_hist(reset=True)
        n = max(sel.size, 1)
        uq = {k: h.pop(k) for k in ("unique_pops", "unique_match_child_pops", "unique_tail_steps")}
        trips = h["pops"].astype(np.float64) + h["tail_steps"]
        tot = trips.sum()
        cum = np.cumsum(trips) / max(tot, 1)
        exp_cum = np.cumsum(h["expansions"].astype(np.float64)) / max(h["expansions"].sum(), 1)
        out[tag] = {"n": int(sel.size),
                    "per_read": {k: round(float(v.sum()) / n, 1) for k, v in h.items()},
                    "round_trips_per_read": round(tot / n, 1),
                    # pops of a match child at depth < K: popped right after the parent's expansion, so a
                    # table of shallow intervals could have fetched them with the parent's round trip
                    "frac_round_trips_match_child_below_depth": {
                        K: round(float(h["match_child_pops"][:K].sum()) / max(tot, 1), 4) for K in (8, 10, 12, 13, 14, 16)},
                    "frac_round_trips_unique": round((uq["unique_pops"] + uq["unique_tail_steps"]) / max(tot, 1), 4),
                    "frac_round_trips_unique_match_child": round(uq["unique_match_child_pops"] / max(tot, 1), 4),
                    "frac_round_trips_unique_tail": round(uq["unique_tail_steps"] / max(tot, 1), 4),
                    "frac_round_trips_below_depth": {K: round(float(cum[K - 1]), 4) for K in (8, 10, 12, 13, 14, 15, 16, 20)},
                    "frac_expansions_below_depth": {K: round(float(exp_cum[K - 1]), 4) for K in (8, 10, 12, 13, 14, 15, 16, 20)},
                    "hist": {k: [int(x) for x in v] for k, v in h.items()}}
    print(json.dumps({k: (v if k not in ("normal", "heavy") else {kk: vv for kk, vv in v.items() if kk != "hist"})
                      for k, v in out.items()}, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f)
    eng.close()


if __name__ == "__main__":
    main()
