#!/usr/bin/env python3
"""Generate tests/golden/sa2pos_vectors.tsv (run in the build container).

TEST INFRASTRUCTURE.  Rows of the golden g1m index are sent through the
reference's own bwt_sa (bwt.c:69-79) over bwt_restore_sa (bwtio.c:29-49),
compiled from /root/reference into oracle/_ref/ibwa_ref (`ibwa_ref sa`), and
the position bwtdb_sa2seq (dbset.c:240-246) derives from it is recorded:

  strand  k  len  bwt_sa  pos

Rows: the SA-interval ends of every hit in the default / -n 0 / mixed golden
.sai files (what samse/sampe convert, bwase.c:133, saiset.c:136,147) with that
read's length, the edges (0, 1, primary +- 1, seq_len, sampling multiples)
and seeded random rows on both strands.
"""
import os
import random
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
sys.path.insert(0, ROOT)

import oracle  # noqa: E402


def sai_hits(path, lens):
    with open(path, "rb") as f:
        buf = f.read()
    p, i, out = 64, 0, []
    while p < len(buf):
        n = struct.unpack_from("<i", buf, p)[0]
        p += 4
        for _ in range(n):
            info, k, l, _sc = struct.unpack_from("<IIIi", buf, p)
            p += 16
            out.append(((info >> 24) & 1, k, l, int(lens[i])))
        i += 1
    return out


def main():
    rows = []
    for reads, sai in (("r100", "r100.default"), ("r100", "r100.n0"), ("mixed", "mixed.default"),
                       ("r150", "r150.default"), ("r36", "r36.default")):
        recs = oracle.read_fastq_records(os.path.join(GOLD, f"reads_{reads}.fq"))
        _, _, lens = oracle.encode_reads(recs, oracle.MODE_COMPREAD, 0)
        for a, k, l, ln in sai_hits(os.path.join(GOLD, sai + ".sai"), lens):
            rows.append((a, k, ln))
            if l != k:
                rows.append((a, l, ln))
    seq_len = oracle.Bwt(os.path.join(GOLD, "g1m.bwt")).seq_len()
    prim = [oracle.Bwt(os.path.join(GOLD, f"g1m.{w}")).primary() for w in ("bwt", "rbwt")]
    rng = random.Random(20261016)
    for strand in (0, 1):
        p = prim[0 if strand else 1]
        edges = [0, 1, 2, 31, 32, 33, 63, 64, 65, p - 1, p, p + 1, seq_len - 1, seq_len]
        edges += [32 * rng.randrange(1, seq_len // 32) for _ in range(16)]
        for k in edges:
            for ln in (1, 36, 100):
                rows.append((strand, k, ln))
        for _ in range(3000):
            rows.append((strand, rng.randrange(0, seq_len + 1), rng.choice((17, 36, 100, 150, 250))))
    # rows whose reverse-index suffix is shorter than the read: seq_len - (sa + len) wraps in u64
    with tempfile.NamedTemporaryFile("w", suffix=".tsv", delete=False) as f:
        for k in range(seq_len + 1):
            f.write("0\t%d\t1\n" % k)
        tmp = f.name
    out = subprocess.run([REF, "sa", os.path.join(GOLD, "g1m"), tmp], check=True, capture_output=True, text=True).stdout
    os.unlink(tmp)
    for ln in out.splitlines():
        _, k, _, sa, _ = (int(x) for x in ln.split("\t"))
        if seq_len - 250 < sa < seq_len:
            for L in (17, 36, 100, 150, 250):
                rows.append((0, k, L))
    with tempfile.NamedTemporaryFile("w", suffix=".tsv", delete=False) as f:
        for r in rows:
            f.write("%d\t%d\t%d\n" % r)
        tmp = f.name
    out = subprocess.run([REF, "sa", os.path.join(GOLD, "g1m"), tmp], check=True, capture_output=True, text=True).stdout
    os.unlink(tmp)
    with open(os.path.join(GOLD, "sa2pos_vectors.tsv"), "w") as f:
        f.write("# strand\tk\tlen\tbwt_sa\tpos  (ibwa_ref sa = bwt_sa bwt.c:69 + bwtdb_sa2seq dbset.c:240, tools/make_sa_golden.py)\n")
        f.write(out)
    print(f"{len(rows)} rows -> sa2pos_vectors.tsv")


if __name__ == "__main__":
    main()
