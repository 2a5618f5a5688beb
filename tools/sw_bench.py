#!/usr/bin/env python3
"""Throughput of the batched Smith-Waterman (mate-rescue shape, BASELINE configs[4]).

Pairs: a 510 bp reference window (2 x 150 + 6 sigma, sigma = 35; bwasw.c:195-219)
around a 150 bp read drawn from inside it at 2 % substitutions (+ 30 % of reads
with 1-5 bp indels), from the GRCh37-sized synthetic genome at --scale.  Reports
alignments/s and forward-pass cell updates/s (len1 x len2 per alignment, the
VALU-bound part), the CPU restatement timed on a sample beside it, and checks a
sample bit-exact against it.  One JSON line on stdout.
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=200_000)
    ap.add_argument("--scale", type=float, default=0.05)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=2000)
    a = ap.parse_args()
    den = 1_000_000
    ascii_, codes, lens, _ = bench.make_genome(int(round(a.scale * den)), den, 37, 16)
    rng = np.random.default_rng(5)
    r = random.Random(5)
    n, W, L = a.pairs, 510, 150
    starts = rng.integers(0, codes.size - W, n)
    refs, reads = [], []
    for k in range(n):
        w = codes[starts[k]:starts[k] + W]
        o = r.randrange(0, W - L)
        rd = w[o:o + L].copy()
        m = rng.random(L) < 0.02
        rd[m] = (rd[m] + rng.integers(1, 4, int(m.sum()))) & 3
        if r.random() < 0.3:
            j, d = r.randrange(10, L - 10), r.randint(1, 5)
            rd = np.concatenate([rd[:j], rd[j + d:], rng.integers(0, 4, d).astype(np.uint8)])
        refs.append(w)
        reads.append(rd)
    from ibwa_amd import engine as E
    eng = E.Engine(0)
    eng.sw(refs[:1000], reads[:1000])  # warm-up
    t = time.perf_counter()
    ms = 0.0
    for _ in range(a.steps):
        out = eng.sw(refs, reads)
        ms += eng.stats().ms_sw
    wall = (time.perf_counter() - t) / a.steps
    k_ms = ms / a.steps
    cells = float(W) * L * n
    # CPU restatement on a sample (one core), and a bit-exact check
    s = min(a.cpu_sample, n)
    t = time.perf_counter()
    exp = [oracle.sw_local(refs[k], reads[k]) for k in range(s)]
    cpu_s = time.perf_counter() - t
    ok = all(out[k] == exp[k] for k in range(s))
    print(json.dumps({
        "metric": "SW mate-rescue alignments/s (aln_local_core, 510 x 150)", "value": n / (k_ms * 1e-3),
        "unit": "alignments/s", "kernel_ms": k_ms, "wall_ms_incl_transfers": wall * 1e3,
        "forward_GCUPS": cells / (k_ms * 1e-3) / 1e9, "pairs": n,
        "cpu_baseline": {"value": s / cpu_s, "unit": "alignments/s", "cores": 1, "kind": "port",
                         "sample": f"first {s} pairs, oracle/ibwa_oracle.c via ctypes"},
        "parity_sample_ok": ok}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
