#!/usr/bin/env python3
"""Generate tests/golden/idx_quirks.fa and the reference's index of it (build container only).

TEST INFRASTRUCTURE.  A small FASTA that walks bns_fasta2bntseq's (bntseq.c:166-254) and
kseq_read's corners: lower case, N runs and runs of other IUPAC codes and '-' (holes, .amb),
a record without a comment after one with a comment (kseq keeps the old comment buffer), a
header whose comment is empty, tab-separated and CRLF headers, an empty record, lines of
uneven width, and l_pac % 4 == 0 (the extra .pac byte).  The reference's own `index`
(bwa_index, bwtindex.c:42-186, compiled into oracle/_ref/ibwa_ref by oracle/Makefile) is run on
it and its eight output files are committed as tests/golden/idx_quirks.{pac,ann,amb,rpac,bwt,
rbwt,sa,rsa}.
"""
import os
import random
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
EXTS = ("pac", "ann", "amb", "rpac", "bwt", "rbwt", "sa", "rsa")


def body(rng, n):
    s = []
    while len(s) < n:
        r = rng.random()
        if r < 0.004:
            s += ["N"] * rng.randint(1, 40)
        elif r < 0.006:
            s += [rng.choice("RYKMSWBDHV-n")] * rng.randint(1, 3)
        elif r < 0.2:
            s.append(rng.choice("acgt"))
        else:
            s.append(rng.choice("ACGT"))
    return "".join(s[:n])


def lines(s, rng, eol="\n"):
    out, i = [], 0
    while i < len(s):
        w = rng.choice((50, 60, 61, 80))
        out.append(s[i:i + w])
        i += w
    return eol.join(out) + eol


def main():
    rng = random.Random(7)
    recs = [
        ">seqA first comment with  spaces\n" + lines(body(rng, 20000), rng),
        ">seqB\n" + lines(body(rng, 9001), rng),
        ">seqC\ttab comment\r\n" + lines(body(rng, 7003), rng, "\r\n"),
        ">seqD \n" + lines(body(rng, 12000), rng),
        ">empty\n",
        ">seqE last one\n" + lines(body(rng, 3996), rng) + "\n\n",
    ]
    fa = os.path.join(GOLD, "idx_quirks.fa")
    with open(fa, "w", newline="") as f:
        f.write("".join(recs))
    tmp = tempfile.mkdtemp()
    try:
        subprocess.run([REF, "index", "-p", os.path.join(tmp, "q"), fa], check=True, capture_output=True)
        for e in EXTS:
            shutil.copy(os.path.join(tmp, "q." + e), os.path.join(GOLD, "idx_quirks." + e))
            print(e, os.path.getsize(os.path.join(GOLD, "idx_quirks." + e)))
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
