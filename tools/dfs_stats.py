#!/usr/bin/env python3
"""Per-read statistics of bwt_match_gap's search on the bench workload (CPU restatement).

Prints distributions of pushes, pops, peak live entries, n_aln and touches, and
how many reads exceed given slot / hit capacities (sizing of gapped.hip).
Needs a GPU (index build).  usage: tools/dfs_stats.py [--scale 0.05] [--reads 100000] [--aln ""]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.05)
    ap.add_argument("--reads", type=int, default=100_000)
    ap.add_argument("--read-len", type=int, default=100)
    ap.add_argument("--aln", default="")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--save", default="", help="write the per-read stats (npy) here")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    den = 1_000_000
    ascii_, codes, lens, _ = bench.make_genome(int(round(a.scale * den)), den, 37, a.threads)
    seq, off, lns = bench.make_reads(ascii_, lens, 2, a.reads, a.read_len, 0.01, 0.05, a.threads)
    # index built on the GPU by the engine's builder (bit-identical to `bwa index`), exported
    from ibwa_amd import engine as E
    eng = E.Engine(0)
    eng.build_index(codes)
    bw = [eng.export_bwt(s_) for s_ in (0, 1)]
    eng.close()
    b0, b1 = [oracle.Bwt(primary=p, L2=l2, words=w) for p, l2, w in bw]
    opt, _ = oracle.parse_aln_args(a.aln.split())
    st = np.zeros(a.reads, dtype=oracle.STATS_DTYPE)
    n_aln, _, _ = oracle.cal_sa_reg_gap(b0, b1, seq, off, lns, opt, n_threads=a.threads, stats=st)
    if a.save:
        np.save(a.save, st)
    for f in ["pushes", "pops", "peak_entries", "peak_real", "peak_bucket", "n_aln", "touches", "tails", "tail_steps",
              "pruned_m", "pruned_w", "expansions", "hits", "distinct_exp", "chains", "rounds", "rounds_g4",
              "rounds_g16", "rounds_lvl"]:
        v = st[f].astype(np.float64)
        print(f"{f:13s} mean {v.mean():9.1f}  p50 {np.percentile(v, 50):8.0f}  p99 {np.percentile(v, 99):8.0f}  "
              f"p99.9 {np.percentile(v, 99.9):8.0f}  max {v.max():8.0f}")
    for cap in [4096, 16384, 65535]:
        print(f"pushes > {cap}: {(st['pushes'] > cap).sum()}   peak_entries > {cap}: {(st['peak_entries'] > cap).sum()}"
              f"   peak_real > {cap}: {(st['peak_real'] > cap).sum()}")
    for cap in [8, 16, 32, 64]:
        print(f"n_aln > {cap}: {(n_aln > cap).sum()}")
    # GPU loop iterations ~ pops + exact-tail steps beyond the first: where the heavy reads spend them
    it = st["pops"].astype(np.float64) + st["tail_steps"] - st["tails"]
    tot = {f: float(st[f].astype(np.float64).sum()) for f in st.dtype.names}
    print(f"all reads: iterations {it.sum():.4g} = pops {tot['pops']:.4g} (pruned m<0 {tot['pruned_m']:.4g}, "
          f"width {tot['pruned_w']:.4g}, expansions {tot['expansions']:.4g} [distinct {tot['distinct_exp']:.4g}], "
          f"tails {tot['tails']:.4g}) + tail steps {tot['tail_steps']:.4g}")
    order = np.argsort(-it)
    print(f"match chains: {tot['chains']:.4g}, mean length {it.sum() / max(tot['chains'], 1):.2f}; "
          f"wave rounds (64 chains of a level per window) {tot['rounds']:.4g}")
    print("heaviest reads: id iterations pops pruned_m pruned_w expansions distinct tails tail_steps hits n_aln peak chains rounds g4 g16 lvl")
    for r in order[:a.top]:
        x = st[r]
        print(f"  {r:8d} {it[r]:10.0f} {x['pops']:9d} {x['pruned_m']:9d} {x['pruned_w']:9d} {x['expansions']:9d} "
              f"{x['distinct_exp']:9d} {x['tails']:8d} {x['tail_steps']:9d} {x['hits']:5d} {x['n_aln']:5d} {x['peak_entries']:8d} {x['chains']:8d} {x['rounds']:7d} {x['rounds_g4']:7d} {x['rounds_g16']:7d} {x['rounds_lvl']:7d}")
    for thr in [1e4, 1e5, 1e6]:
        sel = it > thr
        print(f"reads with > {thr:.0e} iterations: {sel.sum()}, holding {it[sel].sum() / it.sum() * 100:.1f} % of all")


if __name__ == "__main__":
    main()
