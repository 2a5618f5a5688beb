#!/usr/bin/env python3
"""Generate tests/golden/psw_*.tsv: bwa_paired_sw known answers (run in the build container).

TEST INFRASTRUCTURE.  Mate pairs are drawn from the golden g1m genome (regenerated
from synth.cpp, tests/synth_util.py) and given the bwa_seq_t state sampe has when it
calls bwa_paired_sw (bwape.c: after pairing, before bwa_refine_gapped): singletons,
discordant pairs, mates on either strand, pairs already flagged as proper (skipped),
low-mapQ pairs (skipped), N-rich mates (rejected by bwa_sw_core), chimeric mates whose
soft-clipped alignment loses the s_old/s_new comparison, fragments at the genome ends.
The reference's own bwa_paired_sw (bwasw.c:270-304, compiled into oracle/_ref/ibwa_ref
by oracle/Makefile) is run on them (`ibwa_ref psw`) and its output is committed:

  psw_<set>.in.tsv    end0 \\t end1, each "read strand type mapQ seQ extra_flag n_mm n_gapo n_gape pos"
  psw_<set>.out.tsv   end0 \\t end1, each "type strand pos remapped_pos dbidx remapped_dbidx mapQ seQ
                      n_mm n_gapo n_gape extra_flag n_cigar cigar"
  psw_manifest.json   per set: pe type, isize avg / std, ap_prior, and the reference's counters
"""
import json
import os
import random
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
sys.path.insert(0, ROOT)

from tests.synth_util import golden_genome_ascii  # noqa: E402

COMP = str.maketrans("ACGTN", "TGCAN")

# set name -> (pe type, read length, isize avg, isize std, ap_prior, substitution rate, pairs, seed)
SETS = {
    "std100": (1, 100, 300.0, 30.0, 1e-5, 0.01, 1200, 1),
    "std150": (1, 150, 350.0, 35.0, 1e-4, 0.02, 800, 2),
    "solid50": (2, 50, 250.0, 25.0, 1e-5, 0.01, 400, 3),
}


def rc(s):
    return s.translate(COMP)[::-1]


def mutate(rng, s, sub):
    out = list(s)
    for i in range(len(out)):
        if rng.random() < sub:
            out[i] = rng.choice([b for b in "ACGT" if b != out[i]])
    s = "".join(out)
    if rng.random() < 0.05:  # one short indel
        p = rng.randrange(10, len(s) - 10)
        if rng.random() < 0.5:
            s = (s[:p] + "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 3))) + s[p:])[:len(out)]
        else:
            d = rng.randint(1, 3)
            s = s[:p] + s[p + d:] + "".join(rng.choice("ACGT") for _ in range(d))
    return s


def end_fields(read, strand, typ, mapq, seq_q, xf, mm, go, ge, pos):
    return f"{read} {strand} {typ} {mapq} {seq_q} {xf} {mm} {go} {ge} {pos}"


def make_pairs(genome, rng, L, avg, std, sub, n):
    G = len(genome)
    lines = []
    kinds = ["single0", "single1", "disc", "both", "fpp", "lowq", "nrich", "chimera", "edge"]
    while len(lines) < n:
        kind = kinds[len(lines) % len(kinds)]
        I = max(L + 20, int(rng.gauss(avg, std)))
        if kind == "edge":
            f = rng.choice([rng.randrange(0, 60), G - I - rng.randrange(0, 60)])
        else:
            f = rng.randrange(0, G - I)
        seg = genome[f:f + I]
        if "N" in seg:
            continue
        r1 = mutate(rng, seg[:L], sub)          # forward read at f
        r2 = mutate(rng, rc(seg[I - L:]), sub)  # reverse read at f + I - L
        p1, p2 = f, f + I - L
        q1, q2 = rng.randint(17, 60), rng.randint(17, 60)
        mm1, mm2 = rng.randint(0, 3), rng.randint(0, 3)
        e1 = [r1, 0, rng.choice([1, 2]), q1, q1, 0, mm1, 0, 0, p1]
        e2 = [r2, 1, rng.choice([1, 2]), q2, q2, 0, mm2, 0, 0, p2]
        if kind == "single0":
            e2[2:5] = [0, 0, 0]
            e2[9] = rng.choice([0, rng.randrange(0, G)])  # an unmapped end's pos is not its locus
        elif kind == "single1":
            e1[2:5] = [0, 0, 0]
            e1[9] = rng.choice([0, rng.randrange(0, G)])
        elif kind == "disc":
            wrong = e2 if rng.random() < 0.5 else e1
            wrong[9] = rng.randrange(0, G - L)
            wrong[1] = rng.randint(0, 1)
            wrong[3] = wrong[4] = rng.randint(0, 60)
        elif kind == "fpp":
            e1[5] = e2[5] = 2
        elif kind == "lowq":
            e1[3] = e1[4] = rng.randint(0, 16)
            e2[3] = e2[4] = rng.randint(0, 16)
        elif kind == "nrich":
            m = e2 if rng.random() < 0.5 else e1
            s = list(m[0])
            for i in rng.sample(range(L), L // 3):
                s[i] = "N"
            m[0] = "".join(s)
            m[2:5] = [0, 0, 0] if rng.random() < 0.5 else m[2:5]
        elif kind == "chimera":
            m = e2 if rng.random() < 0.5 else e1
            t = L // 3
            m[0] = m[0][:L - t] + "".join(rng.choice("ACGT") for _ in range(t))
            m[9] = rng.randrange(0, G - L)  # mapped elsewhere, so the rescue is re-evaluated
        ends = [e1, e2] if rng.random() < 0.5 else [e2, e1]
        lines.append(end_fields(*ends[0]) + "\t" + end_fields(*ends[1]))
    return lines


def main():
    genome, _, _ = golden_genome_ascii()
    manifest = {}
    for name, (typ, L, avg, std, ap, sub, n, seed) in SETS.items():
        rng = random.Random(seed)
        lines = make_pairs(genome, rng, L, avg, std, sub, n)
        fin = os.path.join(GOLD, f"psw_{name}.in.tsv")
        with open(fin, "w") as f:
            f.write("\n".join(lines) + "\n")
        r = subprocess.run([REF, "psw", os.path.join(GOLD, "g1m"), fin, str(typ), repr(avg), repr(std), repr(ap)],
                           check=True, capture_output=True, text=True)
        with open(os.path.join(GOLD, f"psw_{name}.out.tsv"), "w") as f:
            f.write(r.stdout)
        cnt = [int(x) for x in re.findall(r"\] (\d+) out of (\d+)", r.stderr)[0] + re.findall(r"\] (\d+) out of (\d+)", r.stderr)[1]]
        manifest[name] = {"type": typ, "avg": avg, "std": std, "ap_prior": ap, "pairs": n,
                          "mated_singletons": cnt[0], "singletons": cnt[1], "fixed": cnt[2], "discordant": cnt[3]}
        print(name, manifest[name])
    with open(os.path.join(GOLD, "psw_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
