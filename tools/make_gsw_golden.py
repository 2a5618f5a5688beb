#!/usr/bin/env python3
"""Generate tests/golden/gsw_vectors.tsv: aln_global_core known answers (build container only).

TEST INFRASTRUCTURE.  bwa_refine_gapped (bwase.c:333-417) runs aln_global_core with
aln_param_bwa (band 50, gap_end 5, stdaln.c:227) on a reference window of len + |gaps|
bases around each gapped read.  Pairs of that shape are drawn from the golden genome
(reads with 1-12 bp insertions / deletions, substitutions, N), plus windows shorter than
the read and tiny / lopsided shapes; the reference's own aln_global_core +
bwa_aln_path2cigar (compiled into oracle/_ref/ibwa_ref, `gswf`) gives score, path_len, CIGAR.
"""
import os
import random
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
sys.path.insert(0, ROOT)

from tests.synth_util import golden_genome_ascii  # noqa: E402


def main():
    genome, _, _ = golden_genome_ascii()
    G = len(genome)
    rng = random.Random(7)
    pairs = []
    while len(pairs) < 3000:
        L = rng.choice([20, 36, 50, 76, 100, 101, 150, 250])
        kind = rng.random()
        p = rng.randrange(0, G - 600)
        ref = genome[p:p + L + 40]
        if "N" in ref and rng.random() < 0.9:
            continue
        read = list(ref[20:20 + L])
        g = rng.randint(1, 12 if L >= 50 else 3)
        if kind < 0.45:      # deletion from the read: the window holds g more bases
            q = rng.randrange(5, max(6, L - 5))
            read = read[:q] + list(ref[20 + L:20 + L + g]) if False else read[:q] + read[q + g:] + list(ref[20 + L:20 + L + g])
        elif kind < 0.9:     # insertion into the read
            q = rng.randrange(5, max(6, L - 5))
            read = (read[:q] + [rng.choice("ACGT") for _ in range(g)] + read[q:])[:L]
        for i in range(L):
            if rng.random() < 0.02:
                read[i] = rng.choice("ACGTN" if rng.random() < 0.1 else "ACGT")
        ext = g if rng.random() < 0.8 else rng.randint(0, 3)
        if rng.random() < 0.5:
            win = ref[20:20 + L + ext]           # ext > 0: window starts at the read's position
        else:
            win = ref[20 - ext:20 + L]           # ext < 0: window ends at the read's end
        if rng.random() < 0.05:
            win = win[:rng.randint(1, len(win))]  # short window (near the reference end)
        pairs.append((win, "".join(read)))
    for a, b in [("A", "A"), ("A", "C"), ("ACGT", "A"), ("A", "ACGT"), ("ACGTACGTAC", "ACGT"), ("NNNN", "ACGT")]:
        pairs.append((a, b))
    with tempfile.NamedTemporaryFile("w", suffix=".tsv", delete=False) as f:
        for a, b in pairs:
            f.write(f"{a}\t{b}\n")
        tmp = f.name
    out = subprocess.run([REF, "gswf", tmp], check=True, capture_output=True, text=True).stdout.splitlines()
    os.unlink(tmp)
    assert len(out) == len(pairs)
    with open(os.path.join(GOLD, "gsw_vectors.tsv"), "w") as f:
        f.write("# ref\tread\tscore\tpath_len\tcigar  (aln_global_core, aln_param_bwa; tools/make_gsw_golden.py)\n")
        for (a, b), o in zip(pairs, out):
            f.write(f"{a}\t{b}\t{o}\n")
    print(len(pairs), "pairs")


if __name__ == "__main__":
    main()
