"""The CLI's FASTA/FASTQ reader (readers.h SeqReader, kseq_read semantics, kseq.h:156-195) and
fa2pac (bns_fasta2bntseq, bntseq.c:166-254) on random inputs, against a Python restatement of the
same two functions.  Pinned to the reference by tests/test_index_cli.py (idx_quirks.fa and the
golden genome); this adds breadth: headers with and without comments, '@'/'+' records, CR, blank
lines, IUPAC runs, lower case, characters that end a sequence early.  CPU only."""
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")
NT4 = {c: i for i, c in enumerate("ACGT")}
NT4.update({c: i for i, c in enumerate("acgt")})


def kseq_records(data):
    """kseq_read over bytes: (name, comment or None (never read), seq) per record; returns the
    comment buffer the way kseq keeps it (a record without one keeps the previous buffer)."""
    out, i, n, last = [], 0, len(data), 0
    comment_buf = None
    while True:
        if last == 0:
            while i < n and data[i] not in b">@":
                i += 1
            if i >= n:
                return out
            i += 1
        last = 0
        j = i
        while j < n and not chr(data[j]).isspace():
            j += 1
        name = data[i:j]
        if j >= n and j == i:
            return out
        c = data[j] if j < n else -1
        i = j + 1 if j < n else n
        if c != ord("\n") and c != -1:
            k = data.find(b"\n", i)
            k = n if k < 0 else k
            comment_buf = data[i:k]
            i = k + 1 if k < n else n
        seq = bytearray()
        c = -1
        while i < n:
            ch = data[i]
            i += 1
            if ch in b">+@":
                c = ch
                break
            if 33 <= ch <= 126:
                seq.append(ch)
        if c in (ord(">"), ord("@")):
            last = c
        if c == ord("+"):
            k = data.find(b"\n", i)
            if k < 0:
                return out
            i = k + 1
            q = 0
            while i < n:
                ch = data[i]
                i += 1
                if q >= len(seq):
                    break
                if 33 <= ch <= 127:
                    q += 1
            if q != len(seq):
                return out
        out.append((name, comment_buf, bytes(seq)))


class Lrand48:
    def __init__(self, s):
        self.x = ((s & 0xFFFFFFFF) << 16) | 0x330E

    def next(self):
        self.x = (0x5DEECE66D * self.x + 0xB) & ((1 << 48) - 1)
        return self.x >> 17


def fa2pac_py(data):
    """bns_fasta2bntseq: (.ann text, .amb text, .pac bytes)."""
    rnd = Lrand48(11)
    anns, holes, codes = [], [], []
    for name, comment, seq in kseq_records(data):
        off = anns[-1][3] + anns[-1][4] if anns else 0
        n_ambs, lasts = 0, 0
        for i, ch in enumerate(seq):
            c = NT4.get(chr(ch), 4)
            if c >= 4:
                if lasts == ch:
                    holes[-1][1] += 1
                else:
                    holes.append([off + i, 1, ch])
                    n_ambs += 1
                c = rnd.next() & 3
            lasts = ch
            codes.append(c)
        anno = b"(null)" if comment is None else comment
        anns.append([name, anno, n_ambs, off, len(seq)])
    l_pac = len(codes)
    ann = b"%d %d 11\n" % (l_pac, len(anns))
    for name, anno, n_ambs, off, ln in anns:
        ann += b"0 " + name + ((b" " + anno) if anno else b"") + b"\n" + b"%d %d %d\n" % (off, ln, n_ambs)
    amb = b"%d %d %d\n" % (l_pac, len(anns), len(holes)) + b"".join(b"%d %d %c\n" % (o, ln, c) for o, ln, c in holes)
    pac = bytearray((l_pac + 3) // 4)
    for i, c in enumerate(codes):
        pac[i >> 2] |= c << ((3 - (i & 3)) << 1)
    if l_pac % 4 == 0:
        pac.append(0)
    pac.append(l_pac % 4)
    return ann, amb, bytes(pac), l_pac


def random_input(rng):
    parts = []
    if rng.random() < 0.2:
        parts.append(b"junk before the first header\n")
    for _ in range(rng.randint(1, 6)):
        head = rng.choice(b">>>@")
        name = bytes(rng.choice(b"abcXYZ019_.|") for _ in range(rng.randint(1, 8)))
        sep = rng.choice([b"\n", b" ", b"\t", b"  ", b" \r"])
        comment = b"" if sep == b"\n" else bytes(rng.choice(b"abc def=1;") for _ in range(rng.randint(0, 12))) + b"\n"
        body = bytearray()
        for _ in range(rng.randint(0, 300)):
            r = rng.random()
            body.append(rng.choice(b"ACGT") if r < 0.8 else rng.choice(b"acgtNNNRY-n \r\n"))
        if rng.random() < 0.1:
            body[len(body) // 2:len(body) // 2] = b"+"  # a '+' inside a sequence ends it early (kseq)
        lines = b"\n".join(bytes(body[i:i + 60]) for i in range(0, len(body), 60))
        rec = bytes([head]) + name + sep + comment + lines + b"\n"
        if head == ord("@") and rng.random() < 0.7:
            seqlen = sum(1 for ch in body if 33 <= ch <= 126)
            rec += b"+\n" + bytes(rng.choice(b"!#II5") for _ in range(seqlen)) + b"\n"
        parts.append(rec)
        if rng.random() < 0.2:
            parts.append(b"\n\n")
    return b"".join(parts)


@pytest.mark.parametrize("seed", range(40))
def test_fa2pac_random_inputs(seed, tmp_path):
    rng = random.Random(seed)
    data = random_input(rng)
    ann, amb, pac, l_pac = fa2pac_py(data)
    fa = tmp_path / "x.fa"
    fa.write_bytes(data)
    pre = str(tmp_path / "x")
    r = subprocess.run([CLI, "fa2pac", str(fa), pre], capture_output=True, timeout=60)
    if l_pac == 0:
        assert r.returncode != 0  # "zero length sequence" (bntseq.c:235)
        return
    assert r.returncode == 0, r.stderr
    assert open(pre + ".ann", "rb").read() == ann
    assert open(pre + ".amb", "rb").read() == amb
    assert open(pre + ".pac", "rb").read() == pac
