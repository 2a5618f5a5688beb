#!/usr/bin/env python3
"""End-to-end `ibwa-amd aln` at GRCh37 scale (GPU box): FASTQ in -> .sai out through the CLI.

VERDICT r01 #9 / SURVEY §7: report kernel-only and end-to-end throughput separately.  Workload:
the bench's synthetic 3.10 Gbp genome (same seed), written as FASTA and indexed by `ibwa-amd index`
(byte-identical to `bwa index`), then for each config the bench's reads of that config (same
synthetic generator and seed) written as FASTQ and aligned by `ibwa-amd aln -f out.sai <prefix>
<fq>` -- 0x40000-read batches as bwtaln.c:193, the next batch parsed while the GPU aligns.

Reported per config: wall clock of the command, its own phase times (index load, FASTQ parsing,
align, .sai write), reads/s with and without the index load, and a parity check of the first
`--check` reads of the .sai against the CPU restatement (oracle/, test infrastructure).  The
reference binary built from its own sources (oracle/_ref/ibwa_ref, when present) runs `aln -t
<threads>` on a bounded sample of the same FASTQ with the same index files, and its .sai records
must equal ours for that sample.

usage: tools/e2e_aln.py [--reads 10000000] [--configs 2,1] [--out gpurun_out/e2e.json]
"""
import argparse
import ctypes
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
from pipeline_bench import write_fasta  # noqa: E402

CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
CONFIGS = {1: ("configs[1]", ["-n", "0"], 2), 2: ("configs[2]", [], 3)}  # name, aln options, reads seed


def log(*a):
    print("[e2e]", *a, file=sys.stderr, flush=True)


def synth_reads_ascii(ascii_, lens, seed, n, ln, threads):
    """The bench's reads (bench.make_reads, same generator and seed) as sequenced, ASCII."""
    from ibwa_amd import _native
    L = _native.lib()
    c_lens = (ctypes.c_uint64 * len(lens))(*lens)
    raw = np.empty(n * ln, dtype=np.uint8)
    pos = np.empty(n, dtype=np.uint64)
    strand = np.empty(n, dtype=np.uint8)
    L.ibwa_synth_reads(seed, ascii_.ctypes.data, ascii_.size, len(lens), c_lens, n, ln, 0.01, 0.05,
                       raw.ctypes.data, pos.ctypes.data, strand.ctypes.data, threads)
    return raw.reshape(n, ln)


def write_fastq(path, reads, first=0, count=None):
    """Fixed-width FASTQ records '@r%010d', bases, '+', 'I' qualities, built with numpy."""
    n, L = reads.shape
    count = n - first if count is None else count
    rec = 12 + 1 + L + 3 + L + 1
    with open(path, "wb") as f:
        step = 1_000_000
        for s in range(first, first + count, step):
            e = min(first + count, s + step)
            m = e - s
            buf = np.empty((m, rec), dtype=np.uint8)
            names = np.frombuffer("".join(f"@r{i:010d}" for i in range(s, e)).encode(), dtype=np.uint8)
            buf[:, :12] = names.reshape(m, 12)
            buf[:, 12] = ord("\n")
            buf[:, 13:13 + L] = reads[s:e]
            buf[:, 13 + L:16 + L] = np.frombuffer(b"\n+\n", dtype=np.uint8)
            buf[:, 16 + L:16 + 2 * L] = ord("I")
            buf[:, 16 + 2 * L] = ord("\n")
            f.write(buf.tobytes())


def run(argv, timeout=1800, env=None, save_stderr=None):
    t = time.perf_counter()
    r = subprocess.run(argv, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=timeout,
                       env=dict(os.environ, IBWA_ALN_TIMES="1", **(env or {})))
    dt = time.perf_counter() - t
    err = r.stderr.decode(errors="replace")
    if save_stderr:
        with open(save_stderr, "w") as f:
            f.write(err)
    if r.returncode != 0:
        raise RuntimeError(f"{argv[:2]} failed ({r.returncode}): {err[-1500:]}")
    phases = {}
    for ln in err.splitlines():
        if "slice" in ln or " sec" in ln:
            log("  cli:", ln.strip())
        if "wall s:" in ln:
            for name, v in re.findall(r"([a-z][a-z .()]*?) (\d+\.\d+)", ln.split("wall s:", 1)[1]):
                phases[name.strip()] = float(v)
        m = re.search(r"parse only: (\d+) reads, ([\d.]+) s parsing", ln)
        if m:
            log("  cli:", ln.strip())
            phases["parse only"] = {"reads": int(m.group(1)), "parse_s": float(m.group(2)),
                                    "reads_per_s": int(m.group(1)) / max(float(m.group(2)), 1e-9)}
        m = re.search(r"input parsed on the GPUs: (\d+) records, ([\d.]+) s parsing ahead of the alignment \((\d+) ms of device", ln)
        if m:
            log("  cli:", ln.strip())
            phases["gpu parse"] = {"records": int(m.group(1)), "producer_s": float(m.group(2)), "device_ms": int(m.group(3))}
        m = re.search(r"exit probe: (.*) ([\d.]+) ms", ln)
        if m:
            phases.setdefault("exit probe ms", {})[m.group(1)] = float(m.group(2))
        m = re.search(r"exiting at ([\d.]+) s", ln)
        if m:
            phases["exiting at"] = float(m.group(1))
        m = re.search(r"arena on GPU 0: ([\d.]+) GB, peak use ([\d.]+) GB", ln)
        if m:
            log("  cli:", ln.strip())
            phases["arena_gb"], phases["arena_peak_use_gb"] = float(m.group(1)), float(m.group(2))
        m = re.search(r"device memory: peak ([\d.]+) GB", ln)
        if m:
            log("  cli:", ln.strip())
            phases["device_memory_peak_gb"] = float(m.group(1))
        m = re.search(r"input parse: (\d+) reads in ([\d.]+) s on (\d+) host threads", ln)
        if m:
            log("  cli:", ln.strip())
            n_, s_, t_ = int(m.group(1)), float(m.group(2)), int(m.group(3))
            phases["input parse"] = {"reads": n_, "wall_s": s_, "threads": t_, "reads_per_s": n_ / max(s_, 1e-3),
                                     "reads_per_s_per_thread": n_ / max(s_, 1e-3) / t_}
    return dt, phases


def sai_records(path, n):
    """Per-read hit records of the first n reads of a .sai (64 B header, then n_aln + 16 B each)."""
    d = np.fromfile(path, dtype=np.uint8)
    p, out = 64, []
    for _ in range(n):
        k = int(d[p:p + 4].view(np.int32)[0])
        out.append(d[p + 4:p + 4 + 16 * k].tobytes())
        p += 4 + 16 * k
    return out


def oracle_check(prefix, fq, sai, opts, n):
    """First n reads of our .sai == the CPU restatement (pinned to the reference's goldens)."""
    import oracle
    recs = oracle.read_fastq_records(fq)[:n]  # fq holds the first n reads only
    opt, _ = oracle.parse_aln_args(opts)
    seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
    b0, b1 = oracle.Bwt(prefix + ".bwt"), oracle.Bwt(prefix + ".rbwt")
    rn, ra, _ = oracle.cal_sa_reg_gap(b0, b1, seqs, offs, lens, opt, n_threads=bench.host_threads())
    exp, o = [], 0
    for k in rn:
        exp.append(ra[o:o + k].tobytes())
        o += k
    return exp == sai_records(sai, len(exp))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--read-len", type=int, default=100)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--configs", default="2,1")
    ap.add_argument("--check", type=int, default=20000, help="first reads checked against the CPU restatement")
    ap.add_argument("--ref-sample", type=int, default=200_000, help="reads the reference binary aligns (0: skip)")
    ap.add_argument("--threads", type=int, default=bench.host_threads())
    ap.add_argument("--lanes", default="2", help="IBWA_ALN_LANES values to run (overlapped groups), e.g. 2,1")
    ap.add_argument("--parse", default="dev,host", help="input parse modes to time alone first (IBWA_ALN_PARSE_ONLY): "
                                                        "dev = on the GPU (default path), host = IBWA_ALN_GPU_PARSE=0")
    ap.add_argument("--host-parse-run", type=int, default=1, help="also align with the host parse and compare the .sai")
    ap.add_argument("--variants", default="", help="JSON list of {name: {ENV: value}}: extra aln runs of the same FASTQ "
                                                   "with these environment settings (.sai compared with the first run)")
    ap.add_argument("--prof", default="", help="directory: one more aln run of the FASTQ under rocprofv3 --kernel-trace "
                                               "--stats (the GPU's busy time inside the align phase)")
    ap.add_argument("--arena-trace", default="", help="file: one more aln run with IBWA_ARENA_TRACE=1, its stderr")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    P = os.path.join(tmp, "g")
    res = {"metric": "end-to-end `ibwa-amd aln` reads/s (FASTQ in, .sai out, one GPU)", "host_threads": a.threads,
           "cpu_model": bench.cpu_model(), "configs": {}}
    try:
        t = time.perf_counter()
        den = 1_000_000
        ascii_, codes, lens, _ = bench.make_genome(int(round(a.scale * den)), den, 37, a.threads)
        del codes
        write_fasta(P + ".fa", ascii_, lens)
        res["genome_bp"] = int(ascii_.size)
        log(f"genome {ascii_.size / 1e9:.2f} Gbp + FASTA in {time.perf_counter() - t:.1f} s")
        res["index_s"], _ = run([CLI, "index", "-p", P, P + ".fa"])
        os.unlink(P + ".fa")
        log(f"ibwa-amd index: {res['index_s']:.1f} s")
        for cid in [int(x) for x in a.configs.split(",") if x]:
            name, opts, seed = CONFIGS[cid]
            t = time.perf_counter()
            reads = synth_reads_ascii(ascii_, lens, seed, a.reads, a.read_len, a.threads)
            fq = os.path.join(tmp, f"c{cid}.fq")
            write_fastq(fq, reads)
            sfq = os.path.join(tmp, f"c{cid}_s.fq")
            if a.ref_sample:
                write_fastq(sfq, reads, 0, min(a.ref_sample, a.reads))
            cfq = os.path.join(tmp, f"c{cid}_c.fq")
            write_fastq(cfq, reads, 0, min(a.check, a.reads))
            del reads
            log(f"{name}: {a.reads} reads written in {time.perf_counter() - t:.1f} s")
            sai = os.path.join(tmp, f"c{cid}.sai")
            parse = {}
            for mode in [x for x in a.parse.split(",") if x]:
                env = {"IBWA_ALN_PARSE_ONLY": "1", "IBWA_ALN_GPU_PARSE": "1" if mode == "dev" else "0"}
                wall, ph = run([CLI, "aln"] + opts + ["-f", os.path.join(tmp, "p.sai"), P, fq], env=env)
                parse[mode] = {"wall_s": wall, "phases_s": ph, **ph.get("parse only", {})}
                log(f"{name}: parse only ({mode}): {parse[mode]}")
            c = None
            for li, lanes in enumerate(int(x) for x in a.lanes.split(",")):
                out_sai = sai if li == 0 else os.path.join(tmp, f"c{cid}_l{lanes}.sai")
                wall, ph = run([CLI, "aln"] + opts + ["-f", out_sai, P, fq], env={"IBWA_ALN_LANES": str(lanes)})
                load = ph.get("load index", 0.0)
                r_ = {"lanes": lanes, "wall_s": wall, "phases_s": ph, "reads_per_s": a.reads / wall,
                      "reads_per_s_excl_index_load": a.reads / max(wall - load, 1e-9)}
                log(f"{name}: aln (lanes {lanes}) {wall:.1f} s wall, phases {ph} -> "
                    f"{r_['reads_per_s_excl_index_load']:.0f} reads/s excl. index load")
                if c is None:
                    c = {"workload": f"{name}: {a.reads} x {a.read_len} bp SE FASTQ, aln {' '.join(opts) or 'defaults'}",
                         **r_, "runs": [],
                         "note": "wall clock of the CLI process incl. FASTQ parsing (overlapped with the GPU) and .sai "
                                 "writes; index load (phase 'load index') excluded in reads_per_s_excl_index_load; "
                                 "lanes = IBWA_ALN_LANES (consecutive groups overlapped on that many contexts)"}
                else:
                    r_["sai_equal_first_run"] = open(out_sai, "rb").read() == open(sai, "rb").read()
                    log(f"{name}: lanes {lanes} .sai equal to lanes {c['lanes']}: {r_['sai_equal_first_run']}")
                    os.unlink(out_sai)
                c["runs"].append(r_)
            for vv in (json.loads(a.variants) if a.variants else []):
                for vname, venv in vv.items():
                    vsai = os.path.join(tmp, f"c{cid}_v.sai")
                    wall, ph = run([CLI, "aln"] + opts + ["-f", vsai, P, fq], env={k: str(v) for k, v in venv.items()})
                    load = ph.get("load index", 0.0)
                    r_ = {"variant": vname, "env": venv, "wall_s": wall, "phases_s": ph,
                          "reads_per_s_excl_index_load": a.reads / max(wall - load, 1e-9),
                          "sai_equal_first_run": open(vsai, "rb").read() == open(sai, "rb").read()}
                    log(f"{name}: variant {vname} {venv}: {wall:.1f} s wall -> {r_['reads_per_s_excl_index_load']:.0f} "
                        f"reads/s excl. index load, .sai equal {r_['sai_equal_first_run']}")
                    os.unlink(vsai)
                    c["runs"].append(r_)
            c["parse_only"] = parse
            if a.arena_trace:
                tsai = os.path.join(tmp, f"c{cid}_t.sai")
                wall, ph = run([CLI, "aln"] + opts + ["-f", tsai, P, fq], env={"IBWA_ARENA_TRACE": "1"},
                               save_stderr=a.arena_trace)
                c["arena_trace_run"] = {"wall_s": wall, "phases_s": ph, "file": a.arena_trace}
                os.unlink(tsai)
            if a.prof:
                psai = os.path.join(tmp, f"c{cid}_p.sai")
                # a clean exit: the profiler writes its trace from exit handlers, which the CLI's fast
                # _exit skips
                wall, ph = run(["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", a.prof,
                                "-o", f"c{cid}_aln", "--", CLI, "aln"] + opts + ["-f", psai, P, fq],
                               env={"IBWA_ALN_CLEAN_EXIT": "1"})
                c["prof_run"] = {"wall_s": wall, "phases_s": ph, "dir": a.prof,
                                 "sai_equal_first_run": open(psai, "rb").read() == open(sai, "rb").read()}
                log(f"{name}: profiled aln run: {wall:.1f} s wall, phases {ph}")
                os.unlink(psai)
            if a.host_parse_run:
                hsai = os.path.join(tmp, f"c{cid}_h.sai")
                wall, ph = run([CLI, "aln"] + opts + ["-f", hsai, P, fq], env={"IBWA_ALN_GPU_PARSE": "0"})
                load = ph.get("load index", 0.0)
                c["host_parse"] = {"wall_s": wall, "phases_s": ph, "reads_per_s_excl_index_load": a.reads / max(wall - load, 1e-9),
                                   "sai_equal_gpu_parse": open(hsai, "rb").read() == open(sai, "rb").read()}
                log(f"{name}: host parse: {wall:.1f} s wall -> {c['host_parse']['reads_per_s_excl_index_load']:.0f} reads/s "
                    f"excl. index load; .sai equal to the GPU parse's: {c['host_parse']['sai_equal_gpu_parse']}")
                os.unlink(hsai)
            t = time.perf_counter()
            c["parity_first_reads"] = a.check
            c["parity_ok"] = bool(oracle_check(P, cfq, sai, opts, a.check))
            log(f"{name}: parity of the first {a.check} reads vs the CPU restatement: {c['parity_ok']} "
                f"({time.perf_counter() - t:.1f} s)")
            if a.ref_sample and os.path.exists(REF):
                n_s = min(a.ref_sample, a.reads)
                rsai = os.path.join(tmp, f"c{cid}_r.sai")
                rwall, _ = run([REF, "aln", "-t", str(a.threads)] + opts + ["-f", rsai, P, sfq])
                gsai = os.path.join(tmp, f"c{cid}_g.sai")
                gwall, gph = run([CLI, "aln"] + opts + ["-f", gsai, P, sfq])
                same = open(rsai, "rb").read()[64:] == open(gsai, "rb").read()[64:]
                c["reference"] = {"reads": n_s, "wall_s": rwall, "reads_per_s": n_s / rwall, "threads": a.threads,
                                  "kind": "reference", "sai_equal": bool(same),
                                  "note": "oracle/_ref/ibwa_ref (the reference compiled from its own sources), "
                                          "wall clock incl. its index load; ibwa-amd on the same sample: "
                                          f"{gwall:.1f} s wall"}
                log(f"{name}: reference aln -t {a.threads} on {n_s} reads: {rwall:.1f} s ({n_s / rwall:.0f} reads/s), "
                    f".sai equal {same}")
            for f_ in (fq, sfq, cfq, sai):
                if os.path.exists(f_):
                    os.unlink(f_)
            res["configs"][name] = c
    finally:
        subprocess.run(["rm", "-rf", tmp])
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
