#!/usr/bin/env python3
"""Generate tests/golden/sw_ties.tsv: aln_local_core known answers on score ties (build container only).

TEST INFRASTRUCTURE.  Pairs whose best local score is reached by many cells -- tandem copies of the
read inside the window (equal maxima in different rows and in different 32-column strips of the
forward pass), the read's halves swapped, short-period repeats with and without one mismatch
(equal maxima along diagonals and across strip edges: periods 1-5, 31, 32, 33), N runs -- aligned by
the reference's own aln_local_core (stdaln.c:529-760, aln_param_bwa, `_thres` = 1) through
oracle/_ref/ibwa_ref `swf`, stored with its outputs as in tools/make_sw_golden.py.  The reference keeps
the first maximum in row-major order (stdaln.c:615-626); these vectors pin that rule where a
strip-mined or prefetching pass could pick another of the equal cells.
"""
import os
import random
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
OUT = os.path.join(ROOT, "tests", "golden", "sw_ties.tsv")
ACGT = "ACGT"


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle ref")
    rng = random.Random(2024)
    rs = lambda n: "".join(rng.choice(ACGT) for _ in range(n))  # noqa: E731
    pairs = []
    for _ in range(400):
        l2 = rng.choice([7, 16, 31, 32, 33, 36, 64, 100, 150])
        rd = rs(l2)
        gap = rs(rng.choice([0, 1, 5, 31, 32, 33]))
        k = rng.choice([2, 3, 4])
        pairs.append((((rd + gap) * k)[:800], rd))
        h = l2 // 2
        pairs.append((rd[h:] + gap + rd[:h] + gap + rd[h:], rd))
    for period in (1, 2, 3, 4, 5, 31, 32, 33):
        unit = rs(period)
        for l1, l2 in ((64, 36), (510, 150), (300, 100), (33, 33), (96, 64)):
            ref = (unit * (l1 // period + 1))[:l1]
            rd = (unit * (l2 // period + 2))[rng.randrange(period):][:l2]
            pairs.append((ref, rd))
            m = list(rd)
            m[l2 // 2] = ACGT[(ACGT.index(m[l2 // 2]) + 1) % 4]  # one mismatch: many equal local hits
            pairs.append((ref, "".join(m)))
    for _ in range(200):
        l1, l2 = rng.choice([(510, 150), (200, 100), (64, 36)])
        ref = list(rs(l1))
        a0 = rng.randrange(0, l1 - l2)
        rd = ref[a0:a0 + l2]
        for _n in range(rng.randrange(1, 6)):
            q = rng.randrange(l2)
            for t in range(q, min(l2, q + rng.randrange(1, 8))):
                rd[t] = "N"
        q = rng.randrange(l1)
        for t in range(q, min(l1, q + rng.randrange(1, 40))):
            ref[t] = "N"
        pairs.append(("".join(ref), "".join(rd)))
    scratch = os.path.join(ROOT, "oracle", "_ref", "sw_ties_pairs.tsv")
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
    print(f"{len(pairs)} SW tie vectors -> {OUT}")


if __name__ == "__main__":
    main()
