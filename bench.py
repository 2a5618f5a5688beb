#!/usr/bin/env python3
"""bench.py -- `ibwa aln` reads/s on a GRCh37-sized index (BASELINE.json configs[2], and configs[3]
per GPU under torchrun).

Workload (N=1): a synthetic 3.10 Gbp genome with the 24 GRCh37 contig lengths, 45 % repeat-family
copies and N runs (no GRCh37 FASTA exists here), indexed ON THE GPU by the repo's
builder (bit-identical to `bwa index`), and 50M synthetic 100 bp single-end reads (1 %
substitutions, 5 % with a 1-3 bp indel) aligned with the default options (`-n 0.04 -o 1`, the
gapped search, bwtaln.c:21-37).  One step = one bwa_cal_sa_reg_gap pass over the 50M reads
already resident in HBM (the batch C ABI, ibwa_batch_run: widths, the persistent gapped search,
the cooperative heavy-read pass and any retry); results stay in HBM.  Options are parsed by the
product's own parser (ibwa_aln_parse_args).

Multi-GPU (torchrun, one rank per GPU): reads shard embarrassingly -- every rank holds a full
index replica and its own 50M-read shard (weak scaling: 8 GPUs = configs[3]'s 400M reads); the
only collectives are the timing barrier and the max-over-ranks.

Extra JSON fields (rank 0, N=1):
  roofline      -- algorithmic bytes (64 B x Occ-interval touches per read, counted by the CPU
                   restatement on the measured reads) over the step's kernel time (HIP events);
                   `traffic` = HBM bytes per step from the committed rocprofv3 PMC profile of
                   this workload
  cpu_baseline  -- the CPU restatement timed on the host cores on a bounded sample
  extra.parity  -- GPU == CPU restatement on >= 200k reads plus reads the cooperative / wide /
                   general passes resolved
  extra.exact_leg -- configs[1] (10M reads, -n 0) on the same index, with its own roofline
  extra.e2e     -- the same reads end to end through the CLI (`ibwa-amd aln`: FASTQ file in, .sai out,
                   index load excluded), .sai == the timed step's hits for every read
  extra.e2e_gz  -- the same reads as BGZF-compressed FASTQ through the CLI (inflated on the host
                   threads, parsed on the GPU), .sai == the timed step's hits for every read
  extra.sw_leg  -- k_sw on 200k mate-rescue pairs (510 bp window x 150 bp read, configs[4]'s SW
                   shape) from the same genome: alignments/s, GCUPS over the forward cells, the
                   forward pass alone (engine option sw_stop=1) against its VALU roofline
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


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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


def make_reads(ascii_, lens, seed, n, ln, sub, indel, threads, keep_raw=0):
    """Synthetic reads, encoded as bwa_read_seq stores them (seq, offsets, lengths); with keep_raw,
    also the first keep_raw reads as sequenced (ASCII, one row per read)."""
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
    if keep_raw:
        return seq, off, lns, raw[:min(n, keep_raw) * ln].reshape(-1, ln).copy()
    return seq, off, lns


def shard_seed(rank, base=3):
    """Reads seed of a rank: every rank aligns its own, disjoint synthetic reads (weak scaling)."""
    return base + 1000 * rank


def reduce_max(x, dist, device):
    """Max of a per-rank float over all ranks (the timed region ends on the slowest rank)."""
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_traffic(kernels, workload):
    """HBM bytes per step of the named kernels from the newest committed rocprofv3 PMC summary of
    the same workload (profiles/<round>_<tag>_pmc.json, tools/profile_round.sh: separate --pmc
    passes, EA read/write requests by size, MI355X_MICROARCH.md HBM section).  A profile states
    per kernel how many aln runs of its command it took part in (`runs`); bytes per step = bytes
    over all its dispatches / runs.
    Returns (bytes, file, kernel ms per step) or None if no such profile exists."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if workload not in d.get("workloads", []):
            continue
        ks = [d.get("kernels", {}).get(n) for n in kernels]
        if not all(ks) or not all(k.get("runs") for k in ks):
            continue
        return (sum((k["total_read_bytes"] + k["total_write_bytes"]) / k["runs"] for k in ks), os.path.basename(f),
                sum(k["total_ms"] / k["runs"] for k in ks))
    return None


def oracle_bwts(eng):
    import oracle
    bw = []
    for s in (0, 1):
        p, L2, w = eng.export_bwt(s)
        bw.append(oracle.Bwt(primary=p, L2=L2, words=w))
    return bw


def to_oracle_opt(eopt):
    import oracle
    return oracle.GapOpt.from_buffer_copy(bytes(eopt))


def per_read(n_aln, alns, ids):
    """Hits of reads `ids` as bytes, from the concatenated per-read hit array."""
    first = np.concatenate([[0], np.cumsum(n_aln, dtype=np.int64)[:-1]])
    return [alns[first[i]:first[i] + n_aln[i]].tobytes() for i in ids]


def cpu_and_parity(eng, eopt, seq, off, lns, n_aln, alns, budget_s, check, heavy_budget_s, threads):
    """CPU baseline + touches + parity (rank 0, N=1).  The checker is the C restatement in oracle/
    (test infrastructure; pinned to the reference's .sai goldens by tests/test_oracle_golden.py).

    1. the first n_s reads (n_s >= `check`, sized so the CPU run takes ~budget_s): timed -> the
       CPU baseline; per-read Occ touches -> the roofline's algorithmic bytes; hits == GPU's;
    2. reads the first pass handed on (cooperative / wide / general passes), sampled evenly over
       the batch, in chunks until heavy_budget_s: hits == GPU's."""
    import oracle
    b0, b1 = oracle_bwts(eng)
    opt = to_oracle_opt(eopt)
    n = len(lns)
    n_cal = min(n, 20000)
    t = time.perf_counter()
    oracle.cal_sa_reg_gap(b0, b1, seq, off[:n_cal], lns[:n_cal], opt, n_threads=threads)
    dt = time.perf_counter() - t
    n_s = int(min(n, max(check, n_cal * budget_s / max(dt, 1e-3))))
    wtch = np.zeros(n_s, dtype=np.uint32)
    # where each resumed read left the first pass (pops made, from the GPU) -> its touches up to there
    hpop = np.ascontiguousarray(eng.handoff_pops()[:n_s])
    stch = np.zeros(n_s, dtype=np.uint32)
    t = time.perf_counter()
    rn, ra, tch = oracle.cal_sa_reg_gap(b0, b1, seq, off[:n_s], lns[:n_s], opt, n_threads=threads, touches=True,
                                        width_touches=wtch, split_pops=hpop, split_touches=stch)
    dt = time.perf_counter() - t
    p = int(rn.sum())
    ok_first = bool((n_aln[:n_s] == rn).all() and alns[:p].tobytes() == ra.tobytes())
    cpu = {"value": n_s / dt, "unit": "reads/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
           "sample": f"first {n_s} of the same reads, same index and options ({dt:.1f} s wall, {threads} pthreads, "
                     f"oracle/ibwa_oracle.c)"}
    # heavy reads: resolved outside the first pass
    ids, ps = eng.retry_info()
    by_pass = {int(k): int((ps == k).sum()) for k in (1, 2, 3, 4)}
    sel = []
    for k, cap in ((2, 2000), (3, 2000), (1, 1 << 30)):
        # the cooperative pass: from the start (1) or resuming the first pass's state (4)
        cand = ids[(np.isin(ps, (1, 4)) if k == 1 else ps == k) & (ids >= n_s)]
        if cand.size > cap:
            cand = cand[np.linspace(0, cand.size - 1, cap).astype(np.int64)]
        sel.append(cand)
    # wide/general first (few), then coop reads spread evenly over the batch
    coop = sel[2]
    order = np.concatenate([sel[0], sel[1], coop[np.argsort(np.arange(coop.size) % 64, kind="stable")]])
    checked = {1: 0, 2: 0, 3: 0, 4: 0}
    bad = []
    t0 = time.perf_counter()
    pass_of = dict(zip(ids.tolist(), ps.tolist()))
    chunk = 256
    for c0 in range(0, order.size, chunk):
        if c0 and time.perf_counter() - t0 > heavy_budget_s:
            break
        sub = np.sort(order[c0:c0 + chunk])
        hn, ha, _ = oracle.cal_sa_reg_gap(b0, b1, seq, off[sub], lns[sub], opt, n_threads=threads)
        got = per_read(n_aln, alns, sub)
        exp = per_read(hn, ha, range(sub.size))
        for j, i in enumerate(sub):
            checked[pass_of[int(i)]] += 1
            if got[j] != exp[j] or n_aln[i] != hn[j]:
                bad.append(int(i))
    parity = {"first_reads": n_s, "first_reads_ok": ok_first,
              "handed_on_reads": int(ids.size), "handed_on_by_pass": {"coop": by_pass[1], "coop_resumed": by_pass[4],
                                                                       "wide": by_pass[2], "general": by_pass[3]},
              "handed_on_checked": {"coop": checked[1], "coop_resumed": checked[4], "wide": checked[2],
                                    "general": checked[3]},
              "handed_on_mismatches": bad[:20], "handed_on_ok": not bad,
              "heavy_check_s": time.perf_counter() - t0}
    parity["ok"] = ok_first and not bad and n_s + sum(checked.values()) >= 200_000
    # which pass resolved each sampled first read (0: the first pass; retry_info's 1-4), for the
    # per-kernel roofline, and the touches of a resumed read (pass 4) before its hand-off
    pass_first = np.zeros(n_s, dtype=np.uint8)
    sel_ = ids < n_s
    pass_first[ids[sel_]] = ps[sel_]
    return cpu, (tch, wtch, pass_first, stch, hpop), parity


REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")


def write_fastq(path, raw):
    """Fixed-width FASTQ records '@r%010d', bases, '+', 'I' qualities (raw: one ASCII read per row)."""
    n, L = raw.shape
    rec = 12 + 1 + L + 3 + L + 1
    buf = np.empty((n, rec), dtype=np.uint8)
    buf[:, :12] = np.frombuffer("".join(f"@r{i:010d}" for i in range(n)).encode(), dtype=np.uint8).reshape(n, 12)
    buf[:, 12] = ord("\n")
    buf[:, 13:13 + L] = raw
    buf[:, 13 + L:16 + L] = np.frombuffer(b"\n+\n", dtype=np.uint8)
    buf[:, 16 + L:16 + 2 * L] = ord("I")
    buf[:, 16 + 2 * L] = ord("\n")
    buf.tofile(path)


def sai_records(path, n):
    """Per-read hit records (bytes) of the first n reads of a .sai (64 B header, n_aln + 16 B each)."""
    d = np.fromfile(path, dtype=np.uint8)
    p, out = 64, []
    for _ in range(n):
        k = int(d[p:p + 4].view(np.int32)[0])
        out.append(d[p + 4:p + 4 + 16 * k].tobytes())
        p += 4 + 16 * k
    return out


def ref_baseline(eng, raw, aln_argv, threads, n_aln, alns, budget_s):
    """The reference itself as the CPU baseline: oracle/_ref/ibwa_ref (compiled from the reference's own
    sources by oracle/Makefile; test infrastructure, never part of the product) runs `aln -t <threads>`
    (bwa_aln_core, bwtaln.c:173-241) on the first reads of the same workload, written as FASTQ, with
    the device-built index written as .bwt / .rbwt (bwt_dump_bwt, bwtio.c:7-15) -- files under
    oracle/_ref/bench/.  Its wall time less that of a 1 000-read run (index load, start-up) gives its
    alignment rate; its .sai records must equal the GPU's hits for those reads."""
    import subprocess
    if not os.path.exists(REF):
        return None
    d = os.path.join(ROOT, "oracle", "_ref", "bench")
    os.makedirs(d, exist_ok=True)
    pre = os.path.join(d, "g")
    try:
        for s_, ext in ((0, ".bwt"), (1, ".rbwt")):
            p, L2, w = eng.export_bwt(s_)
            with open(pre + ext, "wb") as f:
                np.array([p] + list(L2), dtype=np.uint32).tofile(f)
                w.astype(np.uint32, copy=False).tofile(f)

        def run(n):
            fq = os.path.join(d, f"s{n}.fq")
            write_fastq(fq, raw[:n])
            sai = os.path.join(d, f"s{n}.sai")
            t = time.perf_counter()
            r = subprocess.run([REF, "aln", "-t", str(threads), *aln_argv, "-f", sai, pre, fq], stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, timeout=600)
            dt = time.perf_counter() - t
            if r.returncode != 0:
                raise RuntimeError(r.stderr.decode(errors="replace")[-500:])
            return dt, sai

        t_small, _ = run(1000)
        # size the sample from a 20 000-read run to about budget_s of alignment
        t20, _ = run(20000)
        rate = 19000 / max(t20 - t_small, 1e-3)
        n = int(min(raw.shape[0], max(20000, rate * budget_s)))
        t_n, sai = run(n)
        got = per_read(n_aln, alns, range(n))
        same = sai_records(sai, n) == got
        return {"value": (n - 1000) / max(t_n - t_small, 1e-3), "unit": "reads/s", "cores": threads,
                "kind": "reference", "cpu_model": cpu_model(),
                "sample": f"first {n} of the same reads as FASTQ, same index (device-built, written as .bwt/.rbwt) "
                          f"and options: `oracle/_ref/ibwa_ref aln -t {threads}` (the reference compiled from its "
                          f"sources) {t_n:.1f} s wall, less {t_small:.1f} s for 1 000 reads (index load, start-up)",
                "sai_equals_gpu": bool(same)}
    finally:
        subprocess.run(["rm", "-rf", d])


def sa2pos_leg(eng, lns, n_aln, alns):
    """SA -> coordinate (bwtdb_sa2seq, dbset.c:240) of each read's first hit after the timed aln
    steps, as samse/sampe would ask for it: kernel time (HIP events) with the full SA resident
    (one gather per hit) and with the sampled SA (bwt_sa's LF walk, bwt.c:69), plus a check
    that both agree.  Not part of `value`."""
    has = n_aln > 0
    first = np.concatenate([[0], np.cumsum(n_aln, dtype=np.int64)[:-1]])[has]
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


def exact_leg(eng, ascii_, lens, args, threads, hip, do_cpu):
    """configs[1]: 10M x 100 bp, `-n 0`, on the same resident index (k_pack_reads + k_exact with
    the K-mer table and the unique-interval jump).  Kernel-time roofline priced with the exact
    path's own touches (oracle.exact_touches, jump-aware) and, for reference, the reference
    algorithm's touches."""
    import oracle
    from ibwa_amd import engine as E
    seq, off, lns = make_reads(ascii_, lens, 2, args.exact_reads, args.read_len, 0.01, 0.05, threads)
    opt = E.parse_aln_args(["-n", "0"])
    eng.stage(seq, off, lns)
    eng.run(opt)
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    ms_k = ms_p = 0.0
    for _ in range(args.exact_steps):
        eng.run(opt)
        st = eng.stats()
        ms_k += st.ms_search
        ms_p += st.ms_width
    hip.hipDeviceSynchronize()
    dt = time.perf_counter() - t0
    st = eng.stats()
    out = {"workload": f"configs[1]: {args.exact_reads} x {args.read_len} bp, aln -n 0, same index",
           "value": args.exact_reads * args.exact_steps / dt, "unit": "reads/s", "steps": args.exact_steps,
           "ms_per_step": dt * 1e3 / args.exact_steps, "k_exact_ms": ms_k / args.exact_steps,
           "k_pack_reads_ms": ms_p / args.exact_steps, "path": {1: "exact", 3: "exact+jump"}.get(st.path, st.path),
           "kmer_k": st.kmer_k}
    if do_cpu:
        n_aln, alns = eng.fetch()
        b0, b1 = oracle_bwts(eng)
        n_t = min(lns.size, 100_000)
        tch = oracle.exact_touches(b0, b1, seq, off[:n_t], lns[:n_t], opt.mode, st.kmer_k, jump=st.path == 3)
        n_c = min(lns.size, 100_000)
        t = time.perf_counter()
        rn, ra, rt = oracle.cal_sa_reg_gap(b0, b1, seq, off[:n_c], lns[:n_c], to_oracle_opt(opt), n_threads=threads,
                                           touches=True)
        cdt = time.perf_counter() - t
        p = int(rn.sum())
        out["parity_reads"] = n_c
        out["parity_ok"] = bool((n_aln[:n_c] == rn).all() and alns[:p].tobytes() == ra.tobytes())
        k_ms = ms_k / args.exact_steps
        ach = float(tch.mean()) * 64.0 * args.exact_reads / (k_ms * 1e-3) / 1e9
        pmc = pmc_traffic(["k_exact"], out["workload"])
        out["roofline"] = {"bound": "hbm", "kernel": "k_exact", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": ach / HBM_PEAK_GBS, "traffic": pmc[0] if pmc else None,
                           "traffic_source": pmc[1] if pmc else None,
                           "touches_per_read": float(tch.mean()), "reference_touches_per_read": float(rt.mean())}
        out["cpu_baseline"] = {"value": n_c / cdt, "unit": "reads/s", "cores": threads, "kind": "port",
                               "cpu_model": cpu_model(), "sample": f"first {n_c} reads ({cdt:.1f} s wall)"}
    return out


CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")


def e2e_leg(eng, ascii_, lens, args, threads, n_aln, alns):
    """configs[2] end to end through the product CLI: the timed step's own 50M reads
    (same generator and seed) written as a FASTQ file, the device-built index written as .bwt / .rbwt
    (bwt_dump_bwt, bwtio.c:7-15), then `ibwa-amd aln -f out.sai <prefix> <reads.fq>` as a child
    process -- file in, .sai out: FASTQ parsed on the GPU, groups of 0x40000-read batches aligned on
    two overlapped lanes, records written in input order (bwa_aln_core, bwtaln.c:173-241).  The
    bench's engine is closed first (the CLI needs the HBM).  Reported: the CLI's wall clock, its
    phases (index load, with the device arena reserved meanwhile; align), reads/s with and without
    them, and parity: the CLI's .sai must equal the timed step's hits for every read.

    With --e2e-gz (default on) the same reads also go in as a BGZF-compressed FASTQ (`reads.fq.gz`,
    deflate level 1 as `bgzip -l 1`, binned qualities in runs so that it compresses like real FASTQ;
    qualities do not enter the search without -q): members inflated on the host threads (gzsrc.h),
    records parsed on the GPU.  Returned under "gz" (bench.py puts it in extra.e2e_gz)."""
    import subprocess
    import tempfile
    from ibwa_amd import _native
    L = _native.lib()
    out = {"workload": f"configs[2] end to end: {args.reads} x {args.read_len} bp FASTQ -> .sai, `ibwa-amd aln` "
                       f"(defaults), one GPU"}
    d = tempfile.mkdtemp(prefix="ibwa_e2e_", dir=os.environ.get("IBWA_E2E_DIR", "/tmp"))
    try:
        pre = os.path.join(d, "g")
        for s_, ext in ((0, ".bwt"), (1, ".rbwt")):
            p_, L2, w = eng.export_bwt(s_)
            with open(pre + ext, "wb") as f:
                np.array([p_] + list(L2), dtype=np.uint32).tofile(f)
                w.astype(np.uint32, copy=False).tofile(f)
        eng.close()
        t = time.perf_counter()
        c_lens = (ctypes.c_uint64 * len(lens))(*lens)
        fq = os.path.join(d, "reads.fq")
        n = args.reads
        # the same call make_reads() made for the timed step (splitmix64 keyed by (seed, stream, index))
        raw = np.empty(n * args.read_len, dtype=np.uint8)
        pos = np.empty(n, dtype=np.uint64)
        strand = np.empty(n, dtype=np.uint8)
        L.ibwa_synth_reads(shard_seed(0, args.seed), ascii_.ctypes.data, ascii_.size, len(lens), c_lens, n,
                           args.read_len, args.sub, args.indel, raw.ctypes.data, pos.ctypes.data,
                           strand.ctypes.data, threads)
        del pos, strand
        if L.ibwa_synth_write_fastq(fq.encode(), raw.ctypes.data, 0, n, args.read_len, threads) != 0:
            raise RuntimeError(f"cannot write {fq}")
        out["fastq_bytes"] = os.path.getsize(fq)
        out["fastq_write_s"] = time.perf_counter() - t
        fqz = None
        gz = {}
        if args.e2e_gz:
            t = time.perf_counter()
            fqz = os.path.join(d, "reads.fq.gz")
            if L.ibwa_synth_write_fastq_gz(fqz.encode(), raw.ctypes.data, 0, n, args.read_len, threads, 1, 0, 1) != 0:
                raise RuntimeError(f"cannot write {fqz}")
            gz = {"workload": f"configs[2] end to end from compressed input: the same {n} x {args.read_len} bp reads "
                              f"as BGZF FASTQ (deflate level 1, binned qualities) -> .sai, `ibwa-amd aln` (defaults), "
                              f"one GPU",
                  "gz_bytes": os.path.getsize(fqz), "gz_write_s": time.perf_counter() - t}
        del raw
        import re

        def run(path, res):
            sai = os.path.join(d, "reads.sai")
            # parse-only first (IBWA_ALN_PARSE_ONLY: the file is read (and inflated) and parsed into groups,
            # nothing is aligned; no arena): the ingest rate of one process
            r = subprocess.run([CLI, "aln", *args.aln.split(), "-f", sai, pre, path], stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, timeout=600,
                               env=dict(os.environ, IBWA_ALN_TIMES="1", IBWA_ALN_PARSE_ONLY="1", IBWA_ARENA_GB="0"))
            err = r.stderr.decode(errors="replace")
            m_ = re.search(r"input parsed on the GPUs: (\d+) records, ([\d.]+) s parsing ahead", err)
            m2 = re.search(r"parse only: (\d+) reads, ([\d.]+) s parsing", err)
            m3 = re.search(r"inflated on (\d+) host threads: ([\d.]+) GB in ([\d.]+) s", err)
            if r.returncode == 0 and m_ and m2:
                res["parse_only"] = {"records": int(m_.group(1)), "producer_s": float(m_.group(2)),
                                     "records_per_s": int(m_.group(1)) / max(float(m2.group(2)), 1e-3),
                                     "consumer_wait_s": float(m2.group(2)),
                                     "note": "the whole file read, inflated if compressed, and parsed on the GPU with "
                                             "nothing aligned: producer_s = the parse calls' wall time; "
                                             "consumer_wait_s = the time the group loop waited for parsed groups "
                                             "(records_per_s = records / consumer_wait_s)"}
                if m3:
                    res["parse_only"]["inflate"] = {"threads": int(m3.group(1)), "gb": float(m3.group(2)),
                                                    "reader_thread_s": float(m3.group(3))}
            env = dict(os.environ, IBWA_ALN_TIMES="1")
            t = time.perf_counter()
            r = subprocess.run([CLI, "aln", *args.aln.split(), "-f", sai, pre, path], stdout=subprocess.DEVNULL,
                               stderr=subprocess.PIPE, env=env, timeout=900)
            wall = time.perf_counter() - t
            err = r.stderr.decode(errors="replace")
            if r.returncode != 0:
                raise RuntimeError(f"ibwa-amd aln failed ({r.returncode}): {err[-800:]}")
            phases = {}
            for ln in err.splitlines():
                if "wall s:" in ln:
                    for name, v in re.findall(r"([a-z][a-z .()]*?) (\d+\.\d+)", ln.split("wall s:", 1)[1]):
                        phases[name.strip()] = float(v)
                m_ = re.search(r"input parsed on the GPUs: (\d+) records, ([\d.]+) s parsing ahead.*\((\d+) ms of device", ln)
                if m_:
                    res["gpu_parse"] = {"records": int(m_.group(1)), "producer_s": float(m_.group(2)),
                                        "device_ms": int(m_.group(3)),
                                        "records_per_s": int(m_.group(1)) / max(float(m_.group(2)), 1e-3)}
                m_ = re.search(r"inflated on (\d+) host threads: ([\d.]+) GB in ([\d.]+) s", ln)
                if m_:
                    res["inflate"] = {"threads": int(m_.group(1)), "gb": float(m_.group(2)),
                                      "reader_thread_s": float(m_.group(3))}
                m_ = re.search(r"exiting at ([\d.]+) s", ln)
                if m_:  # the process's own clock at its end (the rest of the wall is start-up and exit)
                    res["process_clock_at_exit_s"] = float(m_.group(1))
                m_ = re.search(r"arena on GPU 0: ([\d.]+) GB, peak use ([\d.]+) GB", ln)
                if m_:
                    res["arena_gb"], res["arena_peak_use_gb"] = float(m_.group(1)), float(m_.group(2))
            load = phases.get("load index", 0.0)
            # the device arena's phase; until round 5 it also held the GPU runtime's start-up, now its own
            arena = phases.get("device arena", 0.0) + phases.get("gpu runtime start", 0.0)
            res.update({"wall_s": wall, "phases_s": phases, "value": n / max(wall - load - arena, 1e-9),
                        "unit": "reads/s", "value_excl_index_load_only": n / max(wall - load, 1e-9),
                        "value_incl_setup": n / wall,
                        "note": "wall clock of the child process (start-up, input read / inflated and parsed, "
                                "alignment, .sai writes, exit); `value` excludes its 'load index' phase (.bwt/.rbwt "
                                "read and relaid out on the GPU) and its 'gpu runtime start' and 'device arena' phases "
                                "(HIP start-up and the one device reservation, which waits for the driver to take "
                                "back the memory the previous process released); value_incl_setup counts everything"})
            t = time.perf_counter()
            first_bad = L.ibwa_sai_diff(sai.encode(), n, np.ascontiguousarray(n_aln, dtype=np.int32).ctypes.data,
                                        np.ascontiguousarray(alns).ctypes.data)
            res["parity"] = {"reads": n, "sai_equals_timed_step_hits": first_bad == -1,
                             "first_differing_read": int(first_bad), "check_s": time.perf_counter() - t}
            os.unlink(sai)

        run(fq, out)
        if fqz:
            os.unlink(fq)  # page cache for the next file
            try:
                run(fqz, gz)
            except Exception as e:  # the uncompressed leg's result stands
                gz["error"] = repr(e)[:500]
            out["gz"] = gz
        return out
    finally:
        subprocess.run(["rm", "-rf", d])


def sw_src_digest():
    """Digest of the sources k_sw is compiled from (sw.hip and the argument layout in engine.h): a
    counter profile of k_sw stays valid while they are unchanged, whatever else the build changes."""
    import hashlib
    h = hashlib.sha256()
    for f in ("sw.hip", "engine.h"):
        with open(os.path.join(ROOT, "ibwa_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


SW_OPS_PER_CELL = 18  # VALU instructions per cell of k_sw's branch-free forward strip (gfx950 asm)
VALU_PEAK_LANE_OPS = 256 * 64 * 2.4e9  # MI355X_MICROARCH.md: 256 CUs x 64 lanes/clk x 2.4 GHz


def make_sw_pairs(codes, n, seed=5):
    """bwa_paired_sw's rescue shape (tools/sw_bench.py): a 510 bp window around a 150 bp read
    drawn from inside it, 2 % substitutions, 30 % of reads with a 1-5 bp indel."""
    import random
    rng = np.random.default_rng(seed)
    r = random.Random(seed)
    W, L = 510, 150
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
    return refs, reads


def sw_leg(eng, refs, reads, do_cpu, steps=3):
    """k_sw (aln_local_core + aln_global_core + CIGAR) over the pairs; the forward pass alone with
    sw_stop=1.  Parity: a sample bit-exact against the CPU restatement."""
    n = len(refs)
    cells = 510.0 * 150.0 * n
    out = {"workload": f"{n} mate-rescue pairs, 510 bp window x 150 bp read", "pairs": n}
    for stop, tag in ((1, "forward"), (0, "full")):
        eng.set_option("sw_stop", stop)
        eng.sw(refs[:1000], reads[:1000])
        ms = 0.0
        for _ in range(steps):
            res = eng.sw(refs, reads)
            ms += eng.stats().ms_sw
        ms /= steps
        out[f"{tag}_kernel_ms"] = ms
        out[f"{tag}_GCUPS"] = cells / (ms * 1e-3) / 1e9
    eng.set_option("sw_stop", 0)
    out["value"] = n / (out["full_kernel_ms"] * 1e-3)
    out["unit"] = "alignments/s"
    # the VALU work per alignment measured by SQ_INSTS_VALU on this workload shape (the latest
    # profiles/*_sw_pmc.json, tools/sessions/r03_sw_pmc.sh) over the live kernel time: whole k_sw
    # Only a counter file of this build (its build_id) and of this workload shape counts; otherwise the
    # forward-pass estimate below stands in.
    import glob
    from ibwa_amd import engine as E
    bid = E.lib().ibwa_build_id().decode()
    sdig = sw_src_digest()
    pmc, sp = [], None
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_sw_pmc.json")), reverse=True):
        with open(fn) as f:
            d = json.load(f)
        same_code = d.get("build_id") == bid or d.get("sw_src_digest") == sdig
        if same_code and d.get("window") == 510 and d.get("read_len") == 150:
            pmc, sp = [fn], d
            break
    if sp is not None:
        ach = sp["valu_wave_insts_per_alignment"] * 64 * n / (out["full_kernel_ms"] * 1e-3)
        out["roofline"] = {"bound": "valu", "kernel": "k_sw (whole kernel)", "achieved": ach / 1e12,
                           "peak": VALU_PEAK_LANE_OPS / 1e12, "unit": "T lane-ops/s", "frac": ach / VALU_PEAK_LANE_OPS,
                           "valu_wave_insts_per_alignment": sp["valu_wave_insts_per_alignment"],
                           "source": os.path.basename(pmc[0]) + " (SQ_INSTS_VALU per alignment) x live alignments/s"}
    est = out["forward_GCUPS"] * 1e9 * SW_OPS_PER_CELL
    out["forward_pass_estimate"] = {"achieved": est / 1e12, "unit": "T lane-ops/s", "frac": est / VALU_PEAK_LANE_OPS,
                                    "ops_per_cell": SW_OPS_PER_CELL,
                                    "note": "forward pass alone, ops per cell from its gfx950 asm (not a counter)"}
    if "roofline" not in out:
        out["roofline"] = dict(out["forward_pass_estimate"], bound="valu", kernel="k_sw forward pass",
                               peak=VALU_PEAK_LANE_OPS / 1e12)
    if do_cpu:
        import oracle
        s = min(1000, n)
        t = time.perf_counter()
        exp = [oracle.sw_local(refs[k], reads[k]) for k in range(s)]
        cdt = time.perf_counter() - t
        out["parity_sample_ok"] = all(res[k] == exp[k] for k in range(s))
        out["cpu_baseline"] = {"value": s / cdt, "unit": "alignments/s", "cores": 1, "kind": "port",
                               "sample": f"first {s} pairs, oracle/ibwa_oracle.c"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reads", type=int, default=50_000_000, help="reads per GPU")
    ap.add_argument("--read-len", type=int, default=100)
    ap.add_argument("--sub", type=float, default=0.01, help="substitution rate of the synthetic reads "
                                                           "(configs[4]'s 2 x 150 bp: 0.02)")
    ap.add_argument("--indel", type=float, default=0.05, help="fraction of reads with one 1-3 bp indel")
    ap.add_argument("--scale", type=float, default=1.0, help="genome size as a fraction of GRCh37")
    ap.add_argument("--aln", default="", help="aln options (reference syntax); default: gap_init_opt's")
    ap.add_argument("--seed", type=int, default=3, help="reads seed (SURVEY §8d: configs[2] = 3)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work")
    ap.add_argument("--heavy-budget", type=float, default=20.0, help="seconds of CPU parity on handed-on reads")
    ap.add_argument("--ref-budget", type=float, default=15.0,
                    help="seconds of the reference binary's aln (oracle/_ref/ibwa_ref) for cpu_baseline (0: off)")
    ap.add_argument("--check", type=int, default=200_000, help="min. first reads checked bit-exact vs the CPU")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--exact-leg", type=int, default=1, help="also run configs[1] (-n 0) as extra.exact_leg")
    ap.add_argument("--exact-reads", type=int, default=10_000_000)
    ap.add_argument("--exact-steps", type=int, default=5)
    ap.add_argument("--sa2pos", type=int, default=1, help="also time SA->coordinate of every read's first hit")
    ap.add_argument("--e2e-leg", type=int, default=1, help="also run the CLI end to end on the same reads as a "
                                                          "FASTQ file (extra.e2e)")
    ap.add_argument("--e2e-gz", type=int, default=1, help="also run the CLI on the same reads as BGZF FASTQ "
                                                         "(extra.e2e_gz)")
    ap.add_argument("--sw-leg", type=int, default=200_000, help="SW mate-rescue pairs for extra.sw_leg (0: off)")
    ap.add_argument("--opt", action="append", default=[], help="engine option key=value (repeatable)")
    ap.add_argument("--shards", type=int, default=1,
                    help="single process: align the reads of ranks 0..K-1 as one batch (checks the sharded path)")
    ap.add_argument("--dump", default="", help="write this rank's hits to DUMP.rank<r>.npz after the timed steps")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    dev = local
    red_dev = f"cuda:{local}"
    if world > 1:
        import torch
        import torch.distributed as dist_
        n_dev = torch.cuda.device_count()  # does not initialise the GPU
        if world <= n_dev:
            torch.cuda.set_device(local)
            dist_.init_process_group("nccl")  # RCCL over xGMI: only the barrier and the max
        else:
            # more ranks than GPUs (a rehearsal of the sharded path on one box): ranks share
            # devices round-robin; RCCL refuses two ranks on one device, so the two
            # collectives go over gloo
            dev = local % max(n_dev, 1)
            red_dev = "cpu"
            dist_.init_process_group("gloo")
        dist = dist_

    from ibwa_amd import engine as E
    threads = host_threads()
    opt = E.parse_aln_args(args.aln.split())  # the product's own parser (bwtaln.c:249-284)
    tg = time.perf_counter()
    den = 1_000_000
    ascii_, codes, lens, n_amb = make_genome(int(round(args.scale * den)), den, 37, threads)
    log(f"genome {codes.size/1e9:.3f} Gbp ({n_amb} N->random), {time.perf_counter()-tg:.1f} s")
    tr = time.perf_counter()
    keep = 1_000_000 if world == 1 and rank == 0 and not args.no_cpu and args.ref_budget > 0 else 0
    parts = [make_reads(ascii_, lens, shard_seed(r, args.seed), args.reads, args.read_len, args.sub, args.indel, threads,
                        keep_raw=keep if j == 0 else 0)
             for j, r in enumerate([rank] if world > 1 else range(max(1, args.shards)))]
    raw_sample = None
    if keep:
        raw_sample = parts[0][3]
        parts[0] = parts[0][:3]
    if len(parts) == 1:
        seq, off, lns = parts[0]
    else:  # reads of shards 0..K-1 back to back, as one batch
        seq = np.concatenate([p[0] for p in parts])
        lns = np.concatenate([p[2] for p in parts])
        base = np.cumsum([0] + [p[0].size for p in parts[:-1]]).astype(np.uint64)
        off = np.concatenate([p[1] + b for p, b in zip(parts, base)])
    del parts
    args.reads = int(lns.size)
    log(f"{args.reads} reads x {args.read_len} bp, {time.perf_counter()-tr:.1f} s")

    eng = E.Engine(dev)
    tb = time.perf_counter()
    eng.build_index(codes, sa_intv=32)  # the sampled SA too (bwa index's .sa/.rsa), for the sa2pos leg
    build_s = time.perf_counter() - tb
    sw_pairs = make_sw_pairs(codes, args.sw_leg) if args.sw_leg and rank == 0 and world == 1 else None
    del codes
    log(f"index built on device in {build_s:.1f} s")
    for kv in args.opt:
        k_, v_ = kv.split("=")
        eng.set_option(k_, int(v_))
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
    ms_w = ms_s = ms_r = ms_c = ms_cw = ms_cr = 0.0
    if dist is not None:
        dist.barrier()
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
        ms_c += st.ms_coop
        ms_cw += st.ms_coop_width
        ms_cr += st.ms_coop_roots
    hip.hipDeviceSynchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = reduce_max(dt, dist, red_dev)
    if args.dump:
        n_d, a_d = eng.fetch()
        np.savez(f"{args.dump}.rank{rank}.npz", n_aln=n_d, alns=a_d.view(np.uint32))
    # device memory held once the timed steps ran (index, tables and this context's search buffers)
    free_b, total_b = ctypes.c_size_t(0), ctypes.c_size_t(0)
    hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b))
    dev_mem_gb = (total_b.value - free_b.value) / 1e9
    lib_now, lib_peak = E.Engine.device_bytes()
    total_reads = args.reads * world * args.steps
    value = total_reads / dt
    ms_step = dt * 1e3 / args.steps
    launches = max(1, args.steps)
    stl = eng.stats()
    path = stl.path
    exact_cfg = opt.max_diff == 0 and opt.fnr <= 0
    cfg_name = "configs[1]" if exact_cfg else "configs[2]" if world == 1 else "configs[3]"
    if args.read_len == 150 and not exact_cfg:
        cfg_name = "configs[4] aln shape"  # one end of 2 x 150 bp pairs
    reads_desc = "" if (args.sub, args.indel) == (0.01, 0.05) else \
        f" ({args.sub:.0%} substitutions, {args.indel:.0%} with a 1-3 bp indel)"
    result = {
        "metric": "reads/s `ibwa aln` GRCh37-sized 100bp, achieved HBM GB/s vs peak",
        "value": value, "unit": "reads/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic",
        "config": {"workload": f"{cfg_name}: GRCh37-sized synthetic genome ({sum(lens)/1e9:.2f} Gbp, index built on "
                               f"device), {args.reads} x {args.read_len} bp SE reads per GPU{reads_desc}, aln "
                               f"{args.aln or 'defaults (-n 0.04 -o 1)'}",
                   "reads_per_gpu": args.reads, "read_len": args.read_len, "substitution_rate": args.sub,
                   "indel_read_fraction": args.indel, "aln_options": args.aln or "defaults",
                   "parallelism": f"replicated index, reads sharded x{world}"},
    }
    if rank == 0:
        extra = {"index_build_s": build_s, "n_retry": int(stl.n_retry), "n_stack_overflow": int(stl.n_stack_overflow),
                 "n_aln_overflow": int(stl.n_aln_overflow), "n_heavy": int(stl.n_heavy), "n_coop": int(stl.n_coop),
                 "path": {0: "width+search", 1: "exact", 2: "width+gapped", 3: "exact+jump"}.get(path, str(path)),
                 "kernel_ms_per_step": {"k_width(first pass)": ms_w / launches, "k_gapped": ms_s / launches,
                                        "k_width(heavy reads)": ms_cw / launches,
                                        "k_coop_roots": ms_cr / launches,
                                        "k_coop": (ms_c - ms_cw - ms_cr) / launches,
                                        "wide+general retry": (ms_r - ms_c) / launches},
                 "device_memory_gb": {"in_use_after_steps": dev_mem_gb, "total": total_b.value / 1e9,
                                      "library_buffers": lib_now / 1e9, "library_peak": lib_peak / 1e9,
                                      "note": "hipMemGetInfo after the timed steps: index + tables + one context's "
                                              "search buffers (sized for this batch); library_*: the engine's own "
                                              "device buffers now and at their high-water mark (ibwa_device_bytes)"},
                 "buffer_use": {"resume_records_peak": int(stl.resume_records_peak),
                                "resume_records_cap": int(stl.resume_records_cap),
                                "resume_records_per_step": int(stl.resume_records), "n_resumed": int(stl.n_resumed),
                                "coop_pages_peak": int(stl.coop_pages_peak), "coop_pages_cap": int(stl.coop_pages_cap)},
                 "host_cores": threads, "cpu_model": cpu_model(),
                 # digest of the sources libibwa_amd.so was built from (checked against this tree on load)
                 "build_id": E.lib().ibwa_build_id().decode()}
        do_cpu = not args.no_cpu and world == 1
        n_aln = alns = None
        if do_cpu or args.sa2pos:
            n_aln, alns = eng.fetch()
        kernels = ["k_width", "k_gapped", "k_coop"] if path == 2 else ["k_pack_reads", "k_exact"]
        k_ms = (ms_w + ms_s + ms_r) / launches
        if do_cpu:
            tc = time.perf_counter()
            cpu, (tch, wtch, pass_first, stch, hpop), parity = cpu_and_parity(eng, opt, seq, off, lns, n_aln, alns, args.cpu_budget,
                                                                  args.check, args.heavy_budget, threads)
            log(f"CPU baseline + parity {time.perf_counter()-tc:.1f} s: {cpu['value']:.0f} reads/s, parity {parity}")
            result["cpu_baseline"] = cpu
            extra["parity"] = parity
            extra["parity_sample_ok"] = parity["ok"]
            if raw_sample is not None:
                tr_ = time.perf_counter()
                try:
                    ref = ref_baseline(eng, raw_sample, args.aln.split(), threads, n_aln, alns, args.ref_budget)
                    if ref is not None:
                        extra["cpu_port"] = cpu
                        result["cpu_baseline"] = ref
                        extra["parity"]["reference_sample_ok"] = ref["sai_equals_gpu"]
                        # the reference binary's .sai on the same reads is part of the parity verdict
                        extra["parity"]["ok"] = bool(extra["parity"]["ok"] and ref["sai_equals_gpu"])
                        extra["parity_sample_ok"] = extra["parity"]["ok"]
                except Exception as e:  # the headline line is printed regardless
                    extra["cpu_reference_error"] = repr(e)[:500]
                log(f"reference CPU baseline {time.perf_counter()-tr_:.1f} s: {result['cpu_baseline']}")
            del raw_sample
            touches = float(tch.mean())
            # algorithmic bytes: 64 B per Occ-interval touch of the reference algorithm, counted by
            # the CPU restatement on the sampled first reads and split per kernel -- bwt_cal_width's touches
            # (k_width); bwt_match_gap's of the reads the first pass resolves (k_gapped); of a read that left
            # its resume state after p pops (ibwa_batch_diag 2), the touches before pop p + 1 (k_gapped) and
            # the rest (k_coop); of a read the cooperative pass re-ran from the start, all of them (k_coop
            # with its level-0 prologue k_coop_roots: the first pass's partial work on it and its second
            # k_width are not algorithmic bytes)
            ns_ = tch.size
            scale = args.reads / ns_
            mg = tch.astype(np.float64) - wtch
            resumed = pass_first == 4
            scratch = pass_first == 1
            first = pass_first == 0
            g_t = float(mg[first].sum() + (stch[resumed].astype(np.float64) - wtch[resumed]).sum())
            c_t = float(mg[scratch].sum() + (tch[resumed].astype(np.float64) - stch[resumed]).sum())
            per_k = {"k_width": (float(wtch.sum()) * scale, ms_w / launches, ["k_width"]),
                     "k_gapped": (g_t * scale, ms_s / launches, ["k_gapped"]),
                     "k_coop": (c_t * scale, (ms_c - ms_cw) / launches, ["k_coop", "k_coop_roots"])}
            extra["touch_split"] = {"sample_reads": int(ns_), "resumed": int(resumed.sum()),
                                    "coop_from_start": int(scratch.sum()),
                                    "wide_or_general": int(((pass_first == 2) | (pass_first == 3)).sum()),
                                    "resumed_pops_mean": float(hpop[resumed].mean()) if resumed.any() else None,
                                    "resumed_touches_first_pass": float((stch[resumed].astype(np.float64) - wtch[resumed]).sum()),
                                    "resumed_touches_coop": float((tch[resumed].astype(np.float64) - stch[resumed]).sum()),
                                    "unsplit_resumed": int((resumed & (hpop == 0)).sum())}
            pk = {}
            for name, (tt, ms, kn) in per_k.items():
                ab = tt * 64.0
                ach = ab / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
                pmc = pmc_traffic(kn, result["config"]["workload"])
                pk[name] = {"algorithmic_bytes_per_step": ab, "kernel_ms_per_step": ms, "achieved": ach,
                            "frac": ach / HBM_PEAK_GBS, "touches_per_read": tt / args.reads,
                            # the GPU side of the same count: HBM bytes (the PMC file's) in 64 B units per read
                            "gpu_touches_per_read": pmc[0] / 64.0 / args.reads if pmc else None,
                            "traffic": pmc[0] if pmc else None, "traffic_source": pmc[1] if pmc else None,
                            "traffic_over_algorithmic": pmc[0] / ab if pmc and ab > 0 else None}
            ach = touches * 64.0 * args.reads / (k_ms * 1e-3) / 1e9
            pmc = pmc_traffic(kernels, result["config"]["workload"])
            if path != 2:  # the exact path: one kernel does the search
                pk = {"k_exact": {"algorithmic_bytes_per_step": touches * 64.0 * args.reads, "kernel_ms_per_step": k_ms,
                                  "achieved": ach, "frac": ach / HBM_PEAK_GBS, "touches_per_read": touches,
                                  "traffic": pmc[0] if pmc else None, "traffic_source": pmc[1] if pmc else None}}
            dom = max(pk, key=lambda x: pk[x]["kernel_ms_per_step"])
            d_ = pk[dom]
            result["roofline"] = {"bound": "hbm", "kernel": dom + (" (+ k_coop_roots)" if dom.endswith("k_coop") else ""),
                                  "achieved": d_["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": d_["frac"],
                                  "traffic": d_["traffic"], "traffic_source": d_["traffic_source"],
                                  "algorithmic_bytes_per_step": d_["algorithmic_bytes_per_step"],
                                  "kernel_ms_per_step": d_["kernel_ms_per_step"], "bytes_per_touch": 64,
                                  "per_kernel": pk,
                                  "step": {"kernels": "+".join(kernels) + " (one step's launches)", "achieved": ach,
                                           "frac": ach / HBM_PEAK_GBS, "algorithmic_bytes": touches * 64.0 * args.reads,
                                           "kernel_ms": k_ms, "touches_per_read": touches,
                                           "traffic": pmc[0] if pmc else None,
                                           "traffic_source": pmc[1] if pmc else None},
                                  "touches_note": "touches_per_read: the reference's 64 B rank-query touches per read "
                                                  "(oracle/ibwa_oracle.c counters on the sample); gpu_touches_per_read: "
                                                  "the kernel's measured HBM bytes per read / 64 (traffic_source)",
                                  "touches_sample": f"first {ns_} reads ({int(resumed.sum())} of them resumed and "
                                                    f"{int(scratch.sum())} re-run by the cooperative pass), "
                                                    f"oracle/ibwa_oracle.c touch counter split at each resumed "
                                                    f"read's hand-off pop"}
        # the extra legs cannot cost the headline line: a failure is recorded as extra.<leg>.error
        def leg(name, fn):
            t_ = time.perf_counter()
            try:
                extra[name] = fn()
            except Exception as e:
                extra[name] = {"error": repr(e)[:500]}
            log(f"{name} {time.perf_counter()-t_:.1f} s: {extra[name]}")

        if args.sa2pos and n_aln is not None:
            leg("sa2pos", lambda: sa2pos_leg(eng, lns, n_aln, alns))
        if sw_pairs is not None:
            leg("sw_leg", lambda: sw_leg(eng, sw_pairs[0], sw_pairs[1], do_cpu))
            del sw_pairs
        if args.exact_leg and world == 1 and not exact_cfg:
            del seq, off, lns
            leg("exact_leg", lambda: exact_leg(eng, ascii_, lens, args, threads, hip, do_cpu))
        if args.e2e_leg and world == 1 and not exact_cfg and n_aln is not None and os.path.exists(CLI):
            # last: it closes the engine (the CLI process needs the HBM)
            leg("e2e", lambda: e2e_leg(eng, ascii_, lens, args, threads, n_aln, alns))
            if isinstance(extra.get("e2e"), dict) and "gz" in extra["e2e"]:
                extra["e2e_gz"] = extra["e2e"].pop("gz")
        result["extra"] = extra
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
