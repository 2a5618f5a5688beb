#!/usr/bin/env python3
"""Sweep engine options on configs[2] in ONE process (GPU box): the synthetic GRCh37-sized genome,
its index and the reads are built once, then every config runs one warm-up and --steps timed runs
(same reads, same box), printing per-kernel times and the heavy-read count.  Each config's hits are
compared with the first config's (bit-exact: options that only move work between passes must not
change a single hit).
usage: tools/sweep_inproc.py [--reads 50000000] [--steps 1] "" "gap_resume_iters=3000,gap_resume_entries=500" ...
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


# engine defaults of the options a config may set (engine.hip)
DEFAULTS = {"gap_early_iters": 3000, "gap_early_entries": 1000, "gap_iter_budget": 8000,
            "gap_resume": 1, "gap_resume_gb": 48,
            "coop_roots": 1, "gap_reads_per_chunk": 16 << 20,
            "gap_resume_iters": 2000, "gap_resume_entries": 300, "gap_tail_lanes": 16, "gap_tail_iters": 200,
            "gap_pages_per_block": 384, "gap_cap1": 8192, "gap_resume_ppb": 48, "gap_resume_cap1": 4096,
            "coop_pool_gb": 0, "gap_lw_min_waves": 8, "coop_waves_per_cu": 12,
            "coop_stg_room": 1, "gap_resume_recs": 192, "kmer_k": -1, "gap_tab_k": -1, "width_tab": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50_000_000)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--read-len", type=int, default=100)
    ap.add_argument("--sub", type=float, default=0.01)
    ap.add_argument("--indel", type=float, default=0.05)
    ap.add_argument("--out", default="gpurun_out/sweep_inproc.jsonl")
    ap.add_argument("configs", nargs="*", default=[""])
    a = ap.parse_args()
    for cfg in a.configs:
        for x in cfg.split(","):
            if x and x.split("=")[0] not in DEFAULTS:
                sys.exit(f"unknown option {x} (known: {sorted(DEFAULTS)})")
    th = bench.host_threads()
    t0 = time.perf_counter()
    ascii_, codes, lens, _ = bench.make_genome(int(a.scale * 1e6), 1_000_000, 37, th)
    seq, off, lns = bench.make_reads(ascii_, lens, 3, a.reads, a.read_len, a.sub, a.indel, th)
    del ascii_
    eng = E.Engine(0)
    eng.build_index(codes, sa_intv=0)
    del codes
    eng.stage(seq, off, lns)
    opt = E.parse_aln_args([])
    print(f"setup {time.perf_counter() - t0:.1f} s", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    ref = None
    with open(a.out, "a") as fo:
        for cfg in a.configs:
            kv = [x.split("=") for x in cfg.split(",") if x]
            for k, v in kv:
                eng.set_option(k, int(v))
            eng.run(opt)  # warm-up
            ms = []
            for _ in range(a.steps):
                t = time.perf_counter()
                eng.run(opt)
                ms.append((time.perf_counter() - t) * 1e3)
            st = eng.stats()
            n_aln, alns = eng.fetch()
            same = None
            if ref is None:
                ref = (n_aln.copy(), alns.copy())
            else:
                same = bool(np.array_equal(ref[0], n_aln) and np.array_equal(ref[1], alns))
            rec = {"config": cfg, "ms_per_step": float(np.mean(ms)), "ms": ms, "n_heavy": int(st.n_heavy),
                   "width": st.ms_width, "gapped": st.ms_search, "coop": st.ms_coop, "retry": st.ms_retry,
                   "coop_roots": st.ms_coop_roots, "coop_width": st.ms_coop_width, "n_resumed": int(st.n_resumed),
                   "resume_records": int(st.resume_records), "resume_records_peak": int(st.resume_records_peak),
                   "coop_pages_peak": int(st.coop_pages_peak), "coop_pages_cap": int(st.coop_pages_cap),
                   "lib_bytes": E.Engine.device_bytes(),
                   "hits_equal_first_config": same}
            print(json.dumps(rec), flush=True)
            fo.write(json.dumps(rec) + "\n")
            for k, v in kv:  # back to the defaults for the next config
                eng.set_option(k, DEFAULTS[k])
    eng.close()


if __name__ == "__main__":
    main()
