#!/usr/bin/env python3
"""Generate tests/golden/sw_vectors.tsv: aln_local_core known answers (build container only).

TEST INFRASTRUCTURE.  Pairs (reference window, read) shaped like the mate
rescues of bwa_paired_sw (bwasw.c:195-219: a window of 2 x read length + 6
sigma around the expected mate position, sigma = 35, read length 150) plus
edge cases -- partial overlaps, short windows, N runs, tandem repeats and
homopolymers (score ties), random reads, tiny and empty sequences -- are
aligned by the reference's own aln_local_core (stdaln.c:529-760, with
aln_param_bwa, `_thres` = 1) through oracle/_ref/ibwa_ref `swf`, and stored
with its outputs: score, path_len, start (i,j), end (i,j), CIGAR.
Scratch files stay under oracle/_ref/.
"""
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.synth_util import golden_genome_ascii  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
OUT = os.path.join(ROOT, "tests", "golden", "sw_vectors.tsv")
ACGT = "ACGT"


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle ref")
    genome, _, _ = golden_genome_ascii()
    rng = random.Random(5150)
    G = len(genome)

    def window(n):
        p = rng.randrange(0, G - n)
        return genome[p:p + n], p

    def mutate(s, sub, indel):
        out = []
        i = 0
        while i < len(s):
            r = rng.random()
            if r < sub:
                out.append(rng.choice([c for c in ACGT if c != s[i]] or ACGT))
            elif r < sub + indel / 2:
                i += rng.randint(1, 5)  # deletion from the read
                continue
            elif r < sub + indel:
                out.extend(rng.choice(ACGT) for _ in range(rng.randint(1, 5)))  # insertion
                out.append(s[i])
            else:
                out.append(s[i])
            i += 1
        return "".join(out)

    pairs = []
    # mate-rescue shaped: 510 bp window, 150 bp read inside at 2 % error (+ some indels)
    for _ in range(1200):
        w, _ = window(510)
        off = rng.randrange(0, 510 - 150)
        rd = mutate(w[off:off + 150], 0.02, 0.01 if rng.random() < 0.3 else 0.0)
        pairs.append((w, rd))
    # read overlapping a window edge (soft clips), varied lengths
    for _ in range(400):
        ln = rng.choice([36, 50, 76, 100, 150, 250])
        w, p = window(rng.randrange(60, 700))
        shift = rng.randrange(-ln + 20, len(w) - 20)
        s = genome[max(0, p + shift):max(0, p + shift) + ln]
        if len(s) < ln:
            s = s + "".join(rng.choice(ACGT) for _ in range(ln - len(s)))
        pairs.append((w, mutate(s, 0.02, 0.0)))
    # short windows (len1 < len2), long windows
    for _ in range(200):
        w, _ = window(rng.randrange(20, 150))
        rd = mutate(w + "".join(rng.choice(ACGT) for _ in range(rng.randrange(0, 100))), 0.03, 0.0)
        pairs.append((w, rd))
    for _ in range(100):
        w, _ = window(rng.randrange(700, 1200))
        off = rng.randrange(0, len(w) - 150)
        pairs.append((w, mutate(w[off:off + 150], 0.05, 0.02)))
    # N runs in window and read
    for _ in range(200):
        w, _ = window(510)
        w = list(w)
        for _ in range(rng.randrange(1, 4)):
            a = rng.randrange(0, 500)
            for k in range(a, min(510, a + rng.randrange(1, 30))):
                w[k] = "N"
        w = "".join(w)
        off = rng.randrange(0, 360)
        rd = list(mutate(w[off:off + 150].replace("N", "A"), 0.02, 0.0))
        for _ in range(rng.randrange(0, 6)):
            rd[rng.randrange(len(rd))] = "N"
        pairs.append((w, "".join(rd)))
    # ties: tandem repeats and homopolymers
    for unit in ["A", "AC", "ACG", "AAT", "ACGT", "CAGG", "TTAGGG"]:
        for _ in range(30):
            w = (unit * 600)[:rng.randrange(100, 600)]
            w = mutate(w, 0.01, 0.0)
            rd = mutate((unit * 100)[rng.randrange(0, len(unit)):][:rng.randrange(20, 150)], 0.02, 0.01)
            pairs.append((w, rd))
    # random reads: no real alignment
    for _ in range(200):
        w, _ = window(510)
        pairs.append((w, "".join(rng.choice(ACGT) for _ in range(rng.choice([20, 36, 100, 150])))))
    # tiny / degenerate
    pairs += [("A", "A"), ("A", "C"), ("ACGT", "ACGT"), ("ACGTACGT", "TGCA"), ("NNNN", "ACGT"), ("ACGT", "NNNN"),
              ("", "ACGT"), ("ACGT", ""), ("A" * 50, "A" * 50), ("A" * 50, "C" * 50)]

    scratch = os.path.join(ROOT, "oracle", "_ref", "sw_pairs.tsv")
    with open(scratch, "w") as f:
        for a, b in pairs:
            f.write(f"{a}\t{b}\n")
    out = subprocess.run([REF, "swf", scratch], check=True, stdout=subprocess.PIPE, text=True).stdout
    res = out.splitlines()
    assert len(res) == len(pairs), (len(res), len(pairs))
    with open(OUT, "w") as f:
        f.write("#ref\tread\tscore\tpath_len\tstart_ij\tend_ij\tcigar\n")
        for (a, b), r in zip(pairs, res):
            f.write(f"{a}\t{b}\t{r}\n")
    print(f"{len(pairs)} SW vectors -> {OUT}")


if __name__ == "__main__":
    main()
