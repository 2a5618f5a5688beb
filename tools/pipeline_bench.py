#!/usr/bin/env python3
"""End-to-end pipeline timing and parity on the GPU box: index -> aln x2 -> sampe -R, and samse.

Measures the SURVEY §8f rows built around the hot path (index builder, samse/sampe host
pipelines with their GPU steps) on a configs[4]-shaped workload -- synthetic GRCh37-scaled genome,
2 x 150 bp pairs at 2 % substitutions, insert N(350, 35) -- through the `ibwa-amd` CLI exactly as a
user runs it (files in, files out, wall clock per command).  The reference's own binary
(oracle/_ref/ibwa_ref, compiled from /root/reference by oracle/Makefile; test infrastructure) is
timed on a bounded sample of the same pairs with the same index files, and the SAM both write for
that sample is compared line by line (except @PG).

usage: tools/pipeline_bench.py [--scale 0.1] [--pairs 1000000] [--sample 20000] [--out json]
"""
import argparse
import gzip  # noqa: F401  (kept for ad-hoc inspection of outputs)
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
COMP = np.frombuffer(b"TGCAN", dtype=np.uint8)
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def log(*a):
    print("[pipeline]", *a, file=sys.stderr, flush=True)


LAST_ERR = [""]


def run(argv, stdout=None, timeout=1200):
    t = time.perf_counter()
    r = subprocess.run(argv, stdout=stdout, stderr=subprocess.PIPE, timeout=timeout)
    dt = time.perf_counter() - t
    LAST_ERR[0] = r.stderr.decode(errors="replace")
    if r.returncode != 0:
        raise RuntimeError(f"{argv[:2]} failed ({r.returncode}): {r.stderr.decode()[-1500:]}")
    for ln in r.stderr.decode(errors="replace").splitlines():
        if "wall s:" in ln or "cpu s:" in ln or "[ibwa-amd aln]" in ln or "hipMalloc" in ln or "coop pass" in ln or "retry" in ln or "batch of" in ln or "paired_sw]" in ln or "read-ahead" in ln:
            log(f"  {os.path.basename(argv[0])} {argv[1]}: {ln}")
    return dt


def run_both(argvs, timeout=1200, env=None):
    """Both commands at once (the two ends' aln on one GPU); wall of the pair and of each."""
    t = time.perf_counter()
    ps = [subprocess.Popen(a, stderr=subprocess.PIPE, env=env) for a in argvs]
    walls, errs = [], []
    for p_ in ps:
        _, err = p_.communicate(timeout=timeout)
        walls.append(time.perf_counter() - t)
        errs.append(err.decode(errors="replace"))
        if p_.returncode != 0:
            raise RuntimeError(f"failed ({p_.returncode}): {errs[-1][-1500:]}")
    for a, err in zip(argvs, errs):
        for ln in err.splitlines():
            if "wall s:" in ln or "[ibwa-amd aln]" in ln:
                log(f"  {os.path.basename(a[0])} {a[1]} (concurrent): {ln}")
    return time.perf_counter() - t, walls


def write_fasta(path, ascii_, lens):
    with open(path, "wb") as f:
        o = 0
        for i, ln in enumerate(lens):
            f.write(b">chr%d\n" % (i + 1))
            body = ascii_[o:o + ln]
            o += ln
            nl = (ln + 79) // 80
            pad = np.full(nl * 80, ord("\n"), dtype=np.uint8)
            pad[:ln] = body
            rows = np.concatenate([pad.reshape(nl, 80), np.full((nl, 1), ord("\n"), dtype=np.uint8)], axis=1)
            out = rows.reshape(-1)
            # the last row's padding newlines collapse into one line break
            last = ln - (nl - 1) * 80
            f.write(out[:(nl - 1) * 81 + last].tobytes() + b"\n")


def make_pairs(ascii_, n, L, sub, seed):
    """Fragments with insert N(350, 35) (>= L), read 1 forward at the fragment start, read 2 the
    reverse complement of its end (ends swapped for half), i.i.d. substitutions, no N."""
    rng = np.random.default_rng(seed)
    G = ascii_.size
    isn = (ascii_ != ord("A")) & (ascii_ != ord("C")) & (ascii_ != ord("G")) & (ascii_ != ord("T"))
    cn = np.concatenate([[0], np.cumsum(isn, dtype=np.int64)])
    r1 = np.empty((n, L), dtype=np.uint8)
    r2 = np.empty((n, L), dtype=np.uint8)
    got = 0
    while got < n:
        m = (n - got) * 2
        ins = np.maximum(L, rng.normal(350, 35, m).astype(np.int64))
        f = rng.integers(0, G - 1000, m)
        ok = cn[f + ins] - cn[f] == 0
        f, ins = f[ok][:n - got], ins[ok][:n - got]
        k = f.size
        idx = f[:, None] + np.arange(L)[None, :]
        a = ascii_[idx]
        e = ascii_[(f + ins - L)[:, None] + np.arange(L)[None, :]]
        b = COMP[np.searchsorted(np.frombuffer(b"ACGT", dtype=np.uint8), e)][:, ::-1]
        swap = rng.random(k) < 0.5
        a2 = np.where(swap[:, None], b, a)
        b2 = np.where(swap[:, None], a, b)
        for x in (a2, b2):
            mm = rng.random(x.shape) < sub
            code = np.searchsorted(np.frombuffer(b"ACGT", dtype=np.uint8), x)
            x[mm] = ACGT[(code[mm] + rng.integers(1, 4, int(mm.sum()))) & 3]
        r1[got:got + k] = a2
        r2[got:got + k] = b2
        got += k
    return r1, r2


def write_fastq(path, reads, tag, end, first=0, count=None):
    n, L = reads.shape
    count = n - first if count is None else count
    qual = b"I" * L
    with open(path, "wb") as f:
        chunk = 100000
        for s in range(first, first + count, chunk):
            e = min(first + count, s + chunk)
            f.write(b"".join(b"@%s%d/%d\n%s\n+\n%s\n" % (tag, i, end, reads[i].tobytes(), qual) for i in range(s, e)))


def load_s(err):
    """sampe's index load (with the first batch read meanwhile), from its phase line."""
    for ln in err.splitlines():
        if "wall s:" in ln and "load index" in ln:
            return float(ln.split("meanwhile)")[1].split()[0])
    return None


def file_digest(path):
    import hashlib
    h = hashlib.sha1()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def sam_body(path):
    with open(path, "rb") as f:
        return [ln for ln in f.read().split(b"\n") if ln and not ln.startswith(b"@PG")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.1)
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--sample", type=int, default=20000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--sub", type=float, default=0.02)
    ap.add_argument("--threads", type=int, default=bench.host_threads())
    ap.add_argument("--concurrent-ends", type=int, default=1, help="also align the two ends at once (one GPU)")
    ap.add_argument("--concurrent-lanes", default="1,2",
                    help="IBWA_ALN_LANES of each of the two processes aligning the ends at once (the first is "
                         "the pipeline's: one lane each, the other process overlapping it; then the others)")
    ap.add_argument("--sampe-workers", default="1,2", help="sampe -R -G values to time (the first is sampe_s)")
    ap.add_argument("--out", default="")
    ap.add_argument("--diag", action="store_true", help="only run `aln` on the sample's end 2 with IBWA_VERBOSE")
    a = ap.parse_args()
    res = {"workload": f"configs[4] shape on one GPU: {a.scale:g} x GRCh37 synthetic genome, {a.pairs} pairs "
                       f"2 x {a.read_len} bp at {a.sub:.0%} substitutions, insert N(350, 35)",
           "host_threads": a.threads}
    tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    P = os.path.join(tmp, "g")
    den = 1_000_000
    t = time.perf_counter()
    ascii_, _, lens, _ = bench.make_genome(int(round(a.scale * den)), den, 5, a.threads)
    write_fasta(P + ".fa", ascii_, lens)
    res["genome_bp"] = int(ascii_.size)
    log(f"genome {ascii_.size / 1e6:.0f} Mb + FASTA in {time.perf_counter() - t:.1f} s")
    res["index_s"] = run([CLI, "index", "-p", P, P + ".fa"])
    log(f"ibwa-amd index: {res['index_s']:.2f} s")
    t = time.perf_counter()
    r1, r2 = make_pairs(ascii_, a.pairs, a.read_len, a.sub, 5)
    del ascii_
    fq = [os.path.join(tmp, f"r{e}.fq") for e in (1, 2)]
    write_fastq(fq[0], r1, b"p", 1)
    write_fastq(fq[1], r2, b"p", 2)
    sfq = [os.path.join(tmp, f"s{e}.fq") for e in (1, 2)]
    write_fastq(sfq[0], r1, b"p", 1, 0, a.sample)
    write_fastq(sfq[1], r2, b"p", 2, 0, a.sample)
    log(f"{a.pairs} pairs written in {time.perf_counter() - t:.1f} s")
    if a.diag:
        env = dict(os.environ, IBWA_VERBOSE="1")
        for e in (0, 1):
            r = subprocess.run([CLI, "aln", "-f", os.path.join(tmp, "d.sai"), P, sfq[e]], env=env,
                               stderr=subprocess.PIPE, timeout=600)
            log(f"end {e + 1}:\n" + "\n".join(x for x in r.stderr.decode(errors="replace").splitlines()
                                               if " t " in x or "wall" in x or "hipMalloc" in x))
        subprocess.run(["rm", "-rf", tmp])
        return
    # ---- ibwa-amd over all pairs.  The pipeline's aln step runs the two ends at once on the one GPU
    # (two processes, each under ~128 GiB): neither waits for memory the other released, as a second
    # process started after the first one does.  The ends are then also aligned one
    # after the other, for the comparison and the .sai check.
    sai = [os.path.join(tmp, f"r{e}.sai") for e in (1, 2)]
    csai = [os.path.join(tmp, f"c{e}.sai") for e in (1, 2)]
    if a.concurrent_ends:
        # one lane per process by default: the other end's process overlaps it as a second lane would,
        # and the two arenas (~87 instead of ~139 GiB each for 10 M x 150 bp) leave the device room, so
        # neither waits for the other's allocation
        for li, lanes in enumerate(int(x) for x in a.concurrent_lanes.split(",")):
            time.sleep(8.0)  # the previous GPU process's memory wiped first (the next one waits for it)
            env = dict(os.environ, IBWA_ALN_LANES=str(lanes))
            pair_s, walls = run_both([[CLI, "aln", "-f", csai[e], P, fq[e]] for e in (0, 1)], env=env)
            if li == 0:
                res["aln_concurrent"] = {"pair_wall_s": pair_s, "walls_s": walls, "lanes_per_process": lanes}
                csai_first = [open(f_, "rb").read() for f_ in csai]
            else:
                res.setdefault("aln_concurrent_other_lanes", []).append(
                    {"lanes_per_process": lanes, "pair_wall_s": pair_s, "walls_s": walls,
                     "sai_equal_first": [open(f_, "rb").read() for f_ in csai] == csai_first})
            log(f"ibwa-amd: both ends' aln at once, {lanes} lane(s) per process: {pair_s:.2f} s for the pair")
    time.sleep(8.0)  # their memory wiped before the sequential runs
    res["aln_s"] = [run([CLI, "aln", "-f", sai[e], P, fq[e]]) for e in (0, 1)]
    if a.concurrent_ends:
        same = all(open(csai[e], "rb").read() == open(sai[e], "rb").read() for e in (0, 1))
        c = res["aln_concurrent"]
        c.update({"sai_equal_sequential": same, "one_end_wall_s": res["aln_s"][0],
                  "pair_over_one_end": c["pair_wall_s"] / res["aln_s"][0]})
        log(f"ibwa-amd: sequential ends {res['aln_s'][0]:.2f} + {res['aln_s'][1]:.2f} s; pair at once "
            f"{c['pair_wall_s']:.2f} s = {c['pair_over_one_end']:.2f} x one end; .sai equal {same}")
        for f_ in csai:
            os.unlink(f_)
    res["sampe_workers"] = {}
    for k, g in enumerate(a.sampe_workers.split(",")):
        pe = os.path.join(tmp, "pe.sam" if k == 0 else f"pe.G{g}.sam")
        dt = run([CLI, "sampe", "-R", "-G", g, "-f", pe, P, sai[0], sai[1], fq[0], fq[1]])
        ld = load_s(LAST_ERR[0])
        w = {"wall_s": dt, "load_s": ld, "pairs_per_s_excl_load": a.pairs / (dt - ld) if ld is not None else None}
        if k == 0:
            res["sampe_s"] = dt
            ref_digest = file_digest(pe)
        else:
            w["sam_equal_first"] = file_digest(pe) == ref_digest
            os.unlink(pe)
        res["sampe_workers"][g] = w
        log(f"ibwa-amd sampe -R -G {g}: {dt:.2f} s (index load {ld} s) -> "
            f"{w['pairs_per_s_excl_load'] or 0:.0f} pairs/s excluding the load" +
            (f", SAM equal -G {a.sampe_workers.split(',')[0]}: {w['sam_equal_first']}" if k else ""))
    res["samse_s"] = run([CLI, "samse", "-f", os.path.join(tmp, "se.sam"), P, sai[0], fq[0]])
    best_sampe = min(w["wall_s"] for w in res["sampe_workers"].values())
    tot = sum(res["aln_s"]) + res["sampe_s"]
    res["pairs_per_s_aln_sampe"] = a.pairs / tot
    if a.concurrent_ends:
        # the pipeline as run: both ends at once, then sampe with the fastest -G
        res["pairs_per_s_pipeline"] = a.pairs / (res["aln_concurrent"]["pair_wall_s"] + best_sampe)
    time.sleep(8.0)

    log(f"ibwa-amd: aln {res['aln_s'][0]:.2f} + {res['aln_s'][1]:.2f} s, sampe -R {res['sampe_s']:.2f} s, "
        f"samse {res['samse_s']:.2f} s -> {res['pairs_per_s_aln_sampe']:.0f} pairs/s (aln x2 + sampe, files in/out)"
        + (f"; pipeline (ends at once + fastest sampe) {res['pairs_per_s_pipeline']:.0f} pairs/s" if a.concurrent_ends else ""))
    # ---- the sample: ibwa-amd and the reference, SAM compared
    ssai = [os.path.join(tmp, f"s{e}.sai") for e in (1, 2)]
    rsai = [os.path.join(tmp, f"rs{e}.sai") for e in (1, 2)]
    g_aln = [run([CLI, "aln", "-f", ssai[e], P, sfq[e]]) for e in (0, 1)]
    g_pe = run([CLI, "sampe", "-R", "-f", os.path.join(tmp, "s_pe.sam"), P, ssai[0], ssai[1], sfq[0], sfq[1]])
    g_se = run([CLI, "samse", "-f", os.path.join(tmp, "s_se.sam"), P, ssai[0], sfq[0]])
    r_aln = [run([REF, "aln", "-t", str(a.threads), "-f", rsai[e], P, sfq[e]]) for e in (0, 1)]
    with open(os.path.join(tmp, "r_pe.sam"), "wb") as f:
        r_pe = run([REF, "sampe", "-R", "-t", str(a.threads), P, rsai[0], rsai[1], sfq[0], sfq[1]], stdout=f)
    with open(os.path.join(tmp, "r_se.sam"), "wb") as f:
        r_se = run([REF, "samse", P, rsai[0], sfq[0]], stdout=f)
    same_sai = all(open(ssai[e], "rb").read()[64:] == open(rsai[e], "rb").read()[64:] for e in (0, 1))
    pe_g, pe_r = sam_body(os.path.join(tmp, "s_pe.sam")), sam_body(os.path.join(tmp, "r_pe.sam"))
    se_g, se_r = sam_body(os.path.join(tmp, "s_se.sam")), sam_body(os.path.join(tmp, "r_se.sam"))
    res["sample"] = {
        "pairs": a.sample,
        "ibwa_amd_s": {"aln": g_aln, "sampe": g_pe, "samse": g_se},
        "reference_s": {"aln": r_aln, "sampe": r_pe, "samse": r_se, "threads": a.threads,
                        "note": "oracle/_ref/ibwa_ref (the reference compiled from its sources); aln and sampe -t"},
        "sai_equal": bool(same_sai),
        "sampe_sam_lines": len(pe_g), "sampe_sam_equal": pe_g == pe_r,
        "sampe_lines_differing": int(sum(x != y for x, y in zip(pe_g, pe_r)) + abs(len(pe_g) - len(pe_r))),
        "samse_sam_equal": se_g == se_r,
        "reference_pairs_per_s_aln_sampe": a.sample / (sum(r_aln) + r_pe),
    }
    log(f"sample {a.sample} pairs: reference aln {r_aln[0]:.2f} + {r_aln[1]:.2f} s, sampe {r_pe:.2f} s, samse {r_se:.2f} s; "
        f".sai equal {same_sai}, sampe SAM equal {pe_g == pe_r}, samse SAM equal {se_g == se_r}")
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    subprocess.run(["rm", "-rf", tmp])


if __name__ == "__main__":
    main()
