#!/usr/bin/env python3
"""Which reads does the first gapped pass hand on to the cooperative pass, and can k_width's
features tell them apart up front?  (GPU box; diagnostics for DESIGN §6.)

Builds the GRCh37-sized synthetic index, aligns N reads (configs[2] shape) with option diag=1 and
prints, per feature threshold: heavy reads caught, light reads misrouted, and the share of
first-pass lane-iterations the caught heavy reads burned before their hand-off.
usage: tools/heavy_stats.py [--reads 4000000] [--scale 1.0] [--out gpurun_out/heavy_stats.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from ibwa_amd import engine as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=4_000_000)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--out", default="gpurun_out/heavy_stats.json")
    a = ap.parse_args()
    th = bench.host_threads()
    ascii_, codes, lens, _ = bench.make_genome(int(a.scale * 1e6), 1_000_000, 37, th)
    seq, off, lns = bench.make_reads(ascii_, lens, 3, a.reads, 100, 0.01, 0.05, th)
    del ascii_
    eng = E.Engine(0)
    eng.build_index(codes, sa_intv=0)
    del codes
    eng.set_option("diag", 1)
    eng.stage(seq, off, lns)
    opt = E.parse_aln_args([])
    t = time.perf_counter()
    eng.run(opt)
    st = eng.stats()
    print(f"run {time.perf_counter()-t:.2f} s: width {st.ms_width:.0f} gapped {st.ms_search:.0f} "
          f"retry {st.ms_retry:.0f} (coop {st.ms_coop:.0f}) ms, heavy {st.n_heavy}", flush=True)
    it, ft = eng.diag()
    ids, ps = eng.retry_info()
    heavy = np.zeros(a.reads, bool)
    heavy[ids] = True
    tot_it = float(it.sum())
    res = {"reads": a.reads, "heavy": int(heavy.sum()), "iters_total": tot_it,
           "iters_heavy": float(it[heavy].sum()), "ms": {"width": st.ms_width, "gapped": st.ms_search,
                                                         "coop": st.ms_coop, "retry": st.ms_retry},
           "iters_pct_light": [float(np.percentile(it[~heavy], q)) for q in (50, 90, 99, 99.9)],
           "features": {}}
    names = ["sum_log2w_full", "sum_log2w_seed", "min_bid_full", "min_bid_seed"]
    for j, nm in enumerate(names):
        f = ft[:, j].astype(np.int64)
        rows = []
        qs = np.unique(np.percentile(f, np.arange(50, 100, 1.0)).astype(np.int64))
        for thr in qs:
            sel = f >= thr if j < 2 else f <= thr
            caught = int((sel & heavy).sum())
            mis = int((sel & ~heavy).sum())
            saved = float(it[sel & heavy].sum()) / tot_it
            light_it = float(it[sel & ~heavy].sum()) / tot_it
            rows.append({"thr": int(thr), "sel": int(sel.sum()), "heavy_caught": caught, "light_misrouted": mis,
                         "iters_saved_frac": saved, "light_iters_moved_frac": light_it})
        res["features"][nm] = {"heavy_mean": float(f[heavy].mean()), "light_mean": float(f[~heavy].mean()),
                               "rows": rows}
        print(nm, json.dumps(res["features"][nm])[:3000], flush=True)
    print(json.dumps({k: v for k, v in res.items() if k != "features"}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    # raw per-read arrays for offline analysis (first-pass iterations, features, handed on)
    np.savez_compressed(a.out.rsplit(".", 1)[0] + ".npz", it=it, ft=ft, heavy=heavy, ids=ids, ps=ps)
    eng.close()


if __name__ == "__main__":
    main()
