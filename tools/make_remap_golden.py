#!/usr/bin/env python3
"""Generate tests/golden/remap_*: an alternate-haplotype reference with a compound-sequence
remapping table, mate pairs over both references, their .sai and the reference's multi-database
`sampe [-R] <pri> <1.sai> <2.sai> <1.fq> <2.fq> <alt> <a1.sai> <a2.sai>` SAM (build container only).

TEST INFRASTRUCTURE.  The primary reference is the golden g1m genome.  The alternate reference
holds mutated copies of primary regions (SNPs, insertions, deletions), each described in alt.remap
in the format load_remappings reads (bwaremap.cpp:42-100): a header `>name-target|start|stop`
(1-based start, inclusive end) or `>name-target|exact|`, then the alt-vs-primary CIGAR over one or
more lines, one entry per alternate sequence in FASTA order.  Pairs come from the primary, from
the alternates (inside, across the edges and across the indels, so that refine_gapped's window
reaches past an alternate's ends and translate_cigar runs), and at random.  The reference's own
`index`, `aln` and `sampe` (oracle/_ref/ibwa_ref, built from /root/reference by oracle/Makefile)
produce the .sai files and the SAM; FASTA, .remap, FASTQ, .sai and gzip'd SAM are committed with
remap_manifest.json.
"""
import gzip
import json
import os
import random
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
sys.path.insert(0, ROOT)

from tests.synth_util import golden_genome_ascii  # noqa: E402

COMP = str.maketrans("ACGTN", "TGCAN")


def rc(s):
    return s.translate(COMP)[::-1]


def derive(rng, primary, beg, end, events, snp):
    """An alternate copy of primary[beg:end) with SNPs at rate `snp` and the given indels
    [(offset in the primary region, 'I' n | 'D' n)] -> (alt sequence, alt-vs-primary CIGAR)."""
    region = primary[beg:end]
    out, ops = [], []
    pos = 0

    def push(op, n):
        if n <= 0:
            return
        if ops and ops[-1][0] == op:
            ops[-1][1] += n
        else:
            ops.append([op, n])

    for off, op, n in sorted(events) + [(len(region), "E", 0)]:
        seg = list(region[pos:off])
        for i in range(len(seg)):
            if rng.random() < snp:
                seg[i] = rng.choice([b for b in "ACGT" if b != seg[i]])
        out.append("".join(seg))
        push("M", len(seg))
        pos = off
        if op == "I":
            out.append("".join(rng.choice("ACGT") for _ in range(n)))
            push("I", n)
        elif op == "D":
            pos += n
            push("D", n)
    return "".join(out), "".join(f"{n}{op}" for op, n in ops)


def mutate(rng, s, sub):
    out = list(s)
    for i in range(len(out)):
        if out[i] != "N" and rng.random() < sub:
            out[i] = rng.choice([b for b in "ACGT" if b != out[i]])
    return "".join(out)


def main():
    genome, names, lens = golden_genome_ascii()
    starts = [0]
    for L in lens:
        starts.append(starts[-1] + L)
    seqs = {n: genome[starts[i]:starts[i + 1]] for i, n in enumerate(names)}
    rng = random.Random(31)
    # alternates: (name, target, region, events, snp rate); exact ones copy a whole target
    alts = []
    for name, tgt, beg, end, ev, snp in [
        ("altA", "chr3", 10000, 40000, [(12000, "I", 6), (20000, "D", 9), (26000, "I", 1)], 0.004),
        ("altB", "chr7", 5000, 25000, [(3000, "D", 20), (9000, "I", 3), (15000, "D", 2)], 0.01),
        ("altD", "chr10", 2000, 17000, [(7000, "I", 12)], 0.006),
    ]:
        region = seqs[tgt][beg:end]
        assert "N" not in region, (name, tgt)
        s, cig = derive(rng, seqs[tgt], beg, end, ev, snp)
        alts.append((name, tgt, beg, end, s, cig, False))
    # an exact alternate: the whole of chrY with a few SNPs (positions map one to one)
    y = seqs["chrY"]
    ys = list(y)
    for _ in range(8):
        k = rng.randrange(len(ys))
        if ys[k] != "N":
            ys[k] = rng.choice([b for b in "ACGT" if b != ys[k]])
    alts.append(("altY", "chrY", 0, len(y), "".join(ys), None, True))

    with open(os.path.join(GOLD, "remap_alt.fa"), "w") as f:
        for name, *_rest in alts:
            s = _rest[3]
            f.write(f">{name}\n")
            for i in range(0, len(s), 60):
                f.write(s[i:i + 60] + "\n")
    with open(os.path.join(GOLD, "remap_alt.remap"), "w") as f:
        for name, tgt, beg, end, s, cig, exact in alts:
            if exact:
                f.write(f">{name}-{tgt}|exact|\n")
            else:
                f.write(f">{name}-{tgt}|{beg + 1}|{end}\n")
                for i in range(0, len(cig), 50):  # the CIGAR may span lines (load_remappings joins them)
                    f.write(cig[i:i + 50] + "\n")
    alt_prefix = os.path.join(GOLD, "remap_alt")
    subprocess.run([REF, "index", "-p", alt_prefix, alt_prefix + ".fa"], check=True, capture_output=True)
    # the same alternate reference without a .remap table (a database that is not remapped)
    for ext in ("amb", "ann", "bwt", "pac", "rbwt", "rpac", "rsa", "sa"):
        shutil.copy(f"{alt_prefix}.{ext}", os.path.join(GOLD, f"remap_altnr.{ext}"))

    # pairs
    L, avg, std = 100, 300.0, 30.0
    r1s, r2s = [], []
    G = len(genome)
    altseqs = [a[4] for a in alts]
    kinds = ["pri"] * 4 + ["alt", "alt", "altedge", "altindel", "rand", "altfar"]
    while len(r1s) < 1200:
        kind = kinds[len(r1s) % len(kinds)]
        ins = max(L + 10, int(rng.gauss(avg, std)))
        if kind == "pri":
            f0 = rng.randrange(0, G - ins)
            seg = genome[f0:f0 + ins]
        else:
            a = rng.randrange(len(alts))
            s = altseqs[a]
            if kind == "altedge":
                f0 = rng.choice([rng.randrange(0, 60), len(s) - ins - rng.randrange(0, 60)])
            elif kind == "altindel" and alts[a][5]:
                import re
                # a fragment over one of the alternate's indels (alt coordinates)
                ev = []
                apos = 0
                for n, op in re.findall(r"(\d+)([MID])", alts[a][5]):
                    n = int(n)
                    if op in "MI":
                        if op == "I":
                            ev.append(apos)
                        apos += n
                    else:
                        ev.append(apos)
                c = rng.choice(ev)
                f0 = max(0, min(len(s) - ins, c - rng.randrange(20, ins - 20)))
            else:
                f0 = rng.randrange(0, len(s) - ins)
            seg = s[f0:f0 + ins]
        if "N" in seg or len(seg) < ins:
            continue
        a_, b_ = mutate(rng, seg[:L], 0.005), mutate(rng, rc(seg[-L:]), 0.005)
        if kind == "rand":
            a_ = "".join(rng.choice("ACGT") for _ in range(L))
        elif kind == "altfar":  # end 2 from the primary far away
            g = rng.randrange(0, G - L)
            if "N" in genome[g:g + L]:
                continue
            b_ = mutate(rng, rc(genome[g:g + L]), 0.005)
        if rng.random() < 0.5:
            a_, b_ = b_, a_
        q = "".join(chr(33 + rng.randint(20, 40)) for _ in range(L))
        r1s.append((a_, q))
        r2s.append((b_, q))
    for end, recs in ((1, r1s), (2, r2s)):
        with open(os.path.join(GOLD, f"remap_{end}.fq"), "w") as f:
            for i, (s, q) in enumerate(recs):
                f.write(f"@rm{i}/{end}\n{s}\n+\n{q}\n")

    pri = os.path.join(GOLD, "g1m")
    man = {}
    sai = {}
    for ref in ("g1m", "remap_alt"):
        for end in (1, 2):
            fn = f"remap_{ref}_{end}.sai"
            subprocess.run([REF, "aln", "-f", os.path.join(GOLD, fn), os.path.join(GOLD, ref),
                            os.path.join(GOLD, f"remap_{end}.fq")], check=True, capture_output=True)
            sai[ref, end] = fn
    for key, argv, alt in [("remap.R", ["-R"], "remap_alt"), ("remap.R.n5N20", ["-R", "-n", "5", "-N", "20"], "remap_alt"),
                           ("remap.R.s", ["-R", "-s"], "remap_alt"), ("remap.noR", [], "remap_alt"),
                           ("remap.R.nofile", ["-R"], "remap_altnr")]:
        alt_sai = [sai["remap_alt", 1], sai["remap_alt", 2]]
        cmd = ([REF, "sampe"] + argv + [pri, os.path.join(GOLD, sai["g1m", 1]), os.path.join(GOLD, sai["g1m", 2]),
                                        os.path.join(GOLD, "remap_1.fq"), os.path.join(GOLD, "remap_2.fq"),
                                        os.path.join(GOLD, alt)] + [os.path.join(GOLD, x) for x in alt_sai])
        res = subprocess.run(cmd, capture_output=True)
        if res.returncode != 0:
            sys.exit(f"{key}: reference sampe failed ({res.returncode}): {res.stderr.decode()[-2000:]}")
        with open(os.path.join(GOLD, f"sampe_{key}.sam.gz"), "wb") as raw:
            with gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as f:
                f.write(res.stdout)
        man[key] = {"prefixes": ["g1m", alt], "sai": [[sai["g1m", 1], sai["g1m", 2]], alt_sai],
                    "reads": ["remap_1.fq", "remap_2.fq"], "argv": argv, "sam": f"sampe_{key}.sam.gz"}
        print(key, len(res.stdout.splitlines()), "lines", file=sys.stderr)
    json.dump(man, open(os.path.join(GOLD, "remap_manifest.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
