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
    for f in ["pushes", "pops", "peak_entries", "peak_real", "peak_bucket", "n_aln", "touches"]:
        v = st[f].astype(np.float64)
        print(f"{f:13s} mean {v.mean():9.1f}  p50 {np.percentile(v, 50):8.0f}  p99 {np.percentile(v, 99):8.0f}  "
              f"p99.9 {np.percentile(v, 99.9):8.0f}  max {v.max():8.0f}")
    for cap in [4096, 16384, 65535]:
        print(f"pushes > {cap}: {(st['pushes'] > cap).sum()}   peak_entries > {cap}: {(st['peak_entries'] > cap).sum()}"
              f"   peak_real > {cap}: {(st['peak_real'] > cap).sum()}")
    for cap in [8, 16, 32, 64]:
        print(f"n_aln > {cap}: {(n_aln > cap).sum()}")


if __name__ == "__main__":
    main()
