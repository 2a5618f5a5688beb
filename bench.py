#!/usr/bin/env python3
"""bench.py -- `ibwa aln` reads/s on a GRCh37-sized index (BASELINE.json configs[1]).

Workload (N=1): a synthetic 3.10 Gbp genome with the 24 GRCh37 contig lengths,
45 % repeat-family copies and N runs (no GRCh37 FASTA exists
here), indexed ON THE GPU by the repo's builder (bit-identical to `bwa index`),
and 10M synthetic 100 bp single-end reads (1 % substitutions, 5 % with a
1-3 bp indel) aligned with `-n 0` (exact match only).  One step = one aln
pass over the 10M reads already resident in HBM (the batch C ABI,
ibwa_batch_run); results stay in HBM.

Multi-GPU (torchrun, one rank per GPU): reads shard embarrassingly -- every
rank holds a full index replica and its own 10M-read shard (weak scaling);
the only collectives are the timing barrier and the max-over-ranks.

Extra JSON fields: `roofline` (HIP-event kernel times x algorithmic bytes =
64 B x Occ-interval touches, counted by the CPU restatement on a sample) and
`cpu_baseline` (the CPU path timed on the host cores on a bounded sample).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def host_threads():
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cpu = os.cpu_count() or 8
    return max(1, min(n if n > 0 else cpu, cpu, 64))


def make_genome(scale_num, scale_den, seed, threads):
    from ibwa_amd import _native
    L = _native.lib()
    lens = (ctypes.c_uint64 * 24)()
    tot = L.ibwa_synth_grch37_lengths(scale_num, scale_den, lens)
    ascii_ = np.empty(tot, dtype=np.uint8)
    L.ibwa_synth_genome(seed, 24, lens, 0.45, 0.01, 300, ascii_.ctypes.data, threads)
    codes = np.empty(tot, dtype=np.uint8)
    n_amb = L.ibwa_pack_nt4_mt(ascii_.ctypes.data, tot, codes.ctypes.data, threads)
    return ascii_, codes, [int(x) for x in lens], int(n_amb)


def make_reads(ascii_, lens, seed, n, ln, sub, indel, threads):
    from ibwa_amd import _native
    L = _native.lib()
    c_lens = (ctypes.c_uint64 * len(lens))(*lens)
    raw = np.empty(n * ln, dtype=np.uint8)
    pos = np.empty(n, dtype=np.uint64)
    strand = np.empty(n, dtype=np.uint8)
    L.ibwa_synth_reads(seed, ascii_.ctypes.data, ascii_.size, len(lens), c_lens, n, ln, sub, indel,
                       raw.ctypes.data, pos.ctypes.data, strand.ctypes.data, threads)
    seq = np.empty(n * ln, dtype=np.uint8)
    off = np.empty(n, dtype=np.uint64)
    lns = np.empty(n, dtype=np.uint32)
    L.ibwa_encode_reads_fixed(raw.ctypes.data, n, ln, seq.ctypes.data, off.ctypes.data, lns.ctypes.data, threads)
    return seq, off, lns


def shard_seed(rank):
    """Reads seed of a rank: every rank aligns its own, disjoint synthetic reads (weak scaling)."""
    return 2 + 1000 * rank


def reduce_max(x, dist, device):
    """Max of a per-rank float over all ranks (the timed region ends on the slowest rank)."""
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of the
    same workload (profiles/<round>_<tag>_pmc.json, written by tools/profile_round.sh: separate
    --pmc passes, EA read/write requests by size).  None if no such profile exists."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        ks = [d.get("kernels", {}).get(n) for n in kernel.split("+")]
        if all(ks) and d.get("bench_line", {}).get("config", {}).get("workload") == workload:
            # a '+'-joined name prices kernels that run back to back on one batch (per-launch sums)
            return (sum(k["read_bytes_per_dispatch"] + k["write_bytes_per_dispatch"] for k in ks),
                    os.path.basename(f), sum(k.get("avg_ms") or 0.0 for k in ks))
    return None


def cpu_baseline(eng, opt_args, seq, off, lns, budget_s, threads):
    """Time the CPU path on a bounded sample of the same reads (rank 0, N=1 only).

    kind "reference": the reference's own bwa_cal_sa_reg_gap compiled from
    /root/reference into oracle/_ref (test infrastructure); else "port": the
    repo's C restatement (oracle/).  Both over `threads` host threads.
    """
    import oracle
    p0, L20, w0 = eng.export_bwt(0)
    p1, L21, w1 = eng.export_bwt(1)
    b0 = oracle.Bwt(primary=p0, L2=L20, words=w0)
    b1 = oracle.Bwt(primary=p1, L2=L21, words=w1)
    opt, _ = oracle.parse_aln_args(opt_args)
    # calibrate on a small slice, then size the sample for ~budget_s
    n_cal = min(len(lns), 20000)
    t = time.perf_counter()
    _, _, tch = oracle.cal_sa_reg_gap(b0, b1, seq[:int(off[n_cal - 1] + lns[n_cal - 1])], off[:n_cal], lns[:n_cal],
                                      opt, n_threads=threads, touches=True)
    dt = time.perf_counter() - t
    n_s = int(min(len(lns), max(n_cal, n_cal * budget_s / max(dt, 1e-3))))
    t = time.perf_counter()
    n_aln, alns, tch = oracle.cal_sa_reg_gap(b0, b1, seq[:int(off[n_s - 1] + lns[n_s - 1])], off[:n_s], lns[:n_s],
                                             opt, n_threads=threads, touches=True)
    dt = time.perf_counter() - t
    return {"value": n_s / dt, "unit": "reads/s", "cores": threads, "kind": "port",
            "sample": f"first {n_s} of the same reads, same index and options ({dt:.1f} s wall, "
                      f"{threads} pthreads, oracle/ibwa_oracle.c)"}, tch, n_s, (n_aln, alns)


def sa2pos_leg(eng, lns):
    """SA -> coordinate (bwtdb_sa2seq, dbset.c:240) of each read's first hit after the timed aln
    steps, as samse/sampe would ask for it: kernel time (HIP events) with the full SA resident
    (one gather per hit) and with the sampled SA (bwt_sa's LF walk, bwt.c:69), plus a check
    that both agree.  Not part of `value`."""
    n_aln, alns = eng.fetch()
    has = n_aln > 0
    first = np.concatenate([[0], np.cumsum(n_aln)[:-1]])[has]
    a = ((alns["info"][first] >> 24) & 1).astype(np.uint8)
    k = alns["k"][first]
    ln = lns[has]
    out = {"hits": int(k.size)}
    res = []
    for walk in (0, 1):
        eng.set_option("sa_walk", walk)
        eng.sa2pos(a, k, ln)  # warm
        pos = eng.sa2pos(a, k, ln)
        st = eng.stats()
        tag = "walk" if walk else "full"
        out[f"{tag}_ms"] = st.ms_sa2pos
        out[f"{tag}_Mpos_per_s"] = k.size / (st.ms_sa2pos * 1e-3) / 1e6 if st.ms_sa2pos > 0 else None
        out[f"{tag}_used_full_sa"] = int(st.sa2pos_full)
        res.append(pos)
    eng.set_option("sa_walk", 0)
    out["walk_equals_full"] = bool((res[0] == res[1]).all())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reads", type=int, default=10_000_000, help="reads per GPU")
    ap.add_argument("--read-len", type=int, default=100)
    ap.add_argument("--scale", type=float, default=1.0, help="genome size as a fraction of GRCh37")
    ap.add_argument("--aln", default="-n 0", help="aln options (reference syntax)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", type=int, default=20000, help="reads checked bit-exact vs the CPU restatement")
    ap.add_argument("--kmer-k", type=int, default=-1, help="K-mer table length for the exact path (-1 auto, 0 off)")
    ap.add_argument("--exact-path", type=int, default=1, help="use the exact-match kernel when max_diff == 0")
    ap.add_argument("--sweep-k", default="", help="comma list of K values to time after the main run")
    ap.add_argument("--sa2pos", type=int, default=1, help="also time SA->coordinate of every read's first hit")
    ap.add_argument("--opt", action="append", default=[], help="engine option key=value (repeatable)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_
        torch.cuda.set_device(local)
        dist_.init_process_group("nccl")
        dist = dist_

    def barrier_max(x):
        return reduce_max(x, dist, f"cuda:{local}")

    import oracle
    from ibwa_amd import engine as E
    threads = host_threads()
    tg = time.perf_counter()
    den = 1_000_000
    ascii_, codes, lens, n_amb = make_genome(int(round(args.scale * den)), den, 37, threads)
    log(f"genome {codes.size/1e9:.3f} Gbp ({n_amb} N->random), {time.perf_counter()-tg:.1f} s")
    tr = time.perf_counter()
    seq, off, lns = make_reads(ascii_, lens, shard_seed(rank), args.reads, args.read_len, 0.01, 0.05, threads)
    del ascii_
    log(f"{args.reads} reads x {args.read_len} bp, {time.perf_counter()-tr:.1f} s")

    eng = E.Engine(local)
    tb = time.perf_counter()
    eng.build_index(codes, sa_intv=32)  # the sampled SA too (bwa index's .sa/.rsa), for the sa2pos leg
    build_s = time.perf_counter() - tb
    del codes
    log(f"index built on device in {build_s:.1f} s")
    opt_args = args.aln.split()
    ropt, _ = oracle.parse_aln_args(opt_args)
    opt = E.GapOpt()
    for f, _ in E.GapOpt._fields_:
        setattr(opt, f, getattr(ropt, f))

    for kv in args.opt:
        k_, v_ = kv.split("=")
        eng.set_option(k_, int(v_))
    eng.set_option("kmer_k", args.kmer_k)
    eng.set_option("exact_path", args.exact_path)
    eng.stage(seq, off, lns)

    def progress(tag):
        st_ = eng.stats()
        log(f"{tag}: total {st_.ms_total:.1f} ms (width {st_.ms_width:.1f}, search {st_.ms_search:.1f}, "
            f"retry {st_.ms_retry:.1f} ms for {st_.n_retry} reads: {st_.n_stack_overflow} stack, "
            f"{st_.n_aln_overflow} hit overflows, {st_.n_heavy} heavy; coop pass {st_.ms_coop:.1f} ms "
            f"resolved {st_.n_coop})")

    for w in range(args.warmup):
        eng.run(opt)
        progress(f"warmup {w}")
    # timed region: inputs resident in HBM, results left in HBM
    ms_w = ms_s = ms_r = 0.0
    if dist is not None:
        dist.barrier()
    import torch  # noqa: F401  (torch.cuda.synchronize semantics via hipDeviceSynchronize below)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    for k_ in range(args.steps):
        eng.run(opt)
        progress(f"step {k_}")
        st = eng.stats()
        ms_w += st.ms_width
        ms_s += st.ms_search
        ms_r += st.ms_retry
    hip.hipDeviceSynchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = barrier_max(dt)
    n_retry = eng.stats().n_retry
    total_reads = args.reads * world * args.steps
    value = total_reads / dt
    ms_step = dt * 1e3 / args.steps

    cfg_name = "configs[1]" if ropt.max_diff == 0 and ropt.fnr <= 0 else "configs[2]"
    result = {
        "metric": "reads/s `ibwa aln` GRCh37-sized 100bp, achieved HBM GB/s vs peak",
        "value": value, "unit": "reads/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic",
        "config": {"workload": f"{cfg_name}: GRCh37-sized synthetic genome ({lens and sum(lens)/1e9:.2f} Gbp, "
                               f"index built on device), {args.reads} x {args.read_len} bp SE reads per GPU, "
                               f"aln {args.aln}",
                   "reads_per_gpu": args.reads, "read_len": args.read_len, "aln_options": args.aln,
                   "parallelism": f"replicated index, reads sharded x{world}"},
    }
    if rank == 0:
        # correctness check + per-read touch counts on a sample (CPU restatement)
        cpu = None
        check_ok = None
        if not args.no_cpu and world == 1:
            cpu, tch, n_s, (rn, ra) = cpu_baseline(eng, opt_args, seq, off, lns, args.cpu_budget, threads)
            n_aln, alns = eng.fetch()
            p = int(rn[:n_s].sum())
            check_ok = bool((n_aln[:n_s] == rn[:n_s]).all() and alns[:p].tobytes() == ra[:p].tobytes())
            touches = float(tch.mean())
            result["cpu_baseline"] = cpu
        else:
            touches = None
        launches = max(1, args.steps)
        path = eng.stats().path
        if touches:
            # touches of the path actually run: the exact-match kernel skips bwt_cal_width,
            # so its algorithmic bytes are priced from its own exact-search touches
            if path in (1, 3):
                n_t = min(len(lns), 200_000)
                p0, L20, w0 = eng.export_bwt(0)
                p1, L21, w1 = eng.export_bwt(1)
                b0 = oracle.Bwt(primary=p0, L2=L20, words=w0)
                b1 = oracle.Bwt(primary=p1, L2=L21, words=w1)
                kk = eng.stats().kmer_k
                path_touches = float(oracle.exact_touches(b0, b1, seq[:n_t * args.read_len], off[:n_t], lns[:n_t],
                                                          ropt.mode, kk, jump=path == 3).mean())
                result["extra_kmer_k"] = kk
                kname, k_ms = "k_exact", ms_s / launches
            else:
                # the general path runs the reference algorithm: its touches are the oracle's;
                # the two kernels (width, search) are priced together
                path_touches = touches
                kname = "k_width+k_gapped" if path == 2 else "k_width+k_search"
                k_ms = (ms_w + ms_s) / launches
            ach = path_touches * 64.0 * args.reads / (k_ms * 1e-3) / 1e9
            pmc = pmc_traffic(kname, result["config"]["workload"])
            result["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": ach / HBM_PEAK_GBS, "traffic": pmc[0] if pmc else None, "kernel": kname,
                                  "traffic_source": pmc[1] if pmc else None,
                                  "traffic_GBps": pmc[0] / (k_ms * 1e-3) / 1e9 if pmc else None,
                                  "profiled_kernel_ms": pmc[2] if pmc else None,
                                  "algorithmic_bytes_per_launch": path_touches * 64.0 * args.reads,
                                  "kernel_ms_per_launch": k_ms,
                                  "touches_per_read": path_touches, "bytes_per_touch": 64,
                                  "reference_touches_per_read": touches,
                                  "reference_equivalent_GBps": touches * 64.0 * args.reads / (k_ms * 1e-3) / 1e9}
        stl = eng.stats()
        result["extra"] = {"index_build_s": build_s, "n_retry": int(n_retry), "parity_sample_ok": check_ok,
                           "n_stack_overflow": int(stl.n_stack_overflow), "n_aln_overflow": int(stl.n_aln_overflow),
                           "path": {0: "width+search", 1: "exact", 2: "width+gapped", 3: "exact+jump"}.get(path, str(path)),
                           "k_width_or_pack_ms": ms_w / launches, "k_search_ms": ms_s / launches,
                           "retry_ms": ms_r / launches}
        if args.sa2pos:
            result["extra"]["sa2pos"] = sa2pos_leg(eng, lns)
        print(json.dumps(result), flush=True)
        for k in [int(x) for x in args.sweep_k.split(",") if x.strip()]:
            eng.set_option("kmer_k", k)
            eng.run(opt)
            t = time.perf_counter()
            for _ in range(args.steps):
                eng.run(opt)
            dt_k = (time.perf_counter() - t) / args.steps
            log(f"sweep K={k}: {args.reads / dt_k / 1e6:.1f} M reads/s, kernel {eng.stats().ms_search:.2f} ms")
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
