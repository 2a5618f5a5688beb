#!/usr/bin/env python3
"""Generate the BAM-input goldens (run in the build container).

TEST INFRASTRUCTURE.  tests/golden/reads_mixed.fq is written as an (unaligned) BAM,
tests/golden/reads.bam, with the flag mix bwa_read_bam (bwaseqio.c:89-143) selects on:
single-end, read 1, read 2 (0x40 / 0x80), reverse-strand records (0x10: the stored
sequence is the reverse complement and the qualities reversed) and records without
qualities (0xff).  The file is gzip, which bamlite reads through gzread (bamlite.h:8-11)
like BGZF.  The reference's `aln -b` (bwtaln.c:159-171, compiled into oracle/_ref) is run
on it for each selection option and the .sai outputs are committed with a manifest
(bam_manifest.json: argv -> file).
"""
import gzip
import json
import os
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")
sys.path.insert(0, ROOT)

import oracle  # noqa: E402

NT16 = {"=": 0, "A": 1, "C": 2, "G": 4, "T": 8, "N": 15}
COMP = str.maketrans("ACGTN", "TGCAN")
FLAGS = [0x4, 0x14, 0x45, 0x85, 0x55, 0x95, 0x4, 0x45]
OPTS = {"all": ["-b"], "se": ["-b", "-0"], "r1": ["-b", "-1"], "r2": ["-b", "-2"], "r12": ["-b", "-1", "-2"],
        "q15": ["-b", "-q", "15"], "n0": ["-b", "-n", "0"]}


def record(name, seq, qual, flag):
    if flag & 0x10:
        seq = seq.translate(COMP)[::-1]
        qual = qual[::-1] if qual is not None else None
    l = len(seq)
    qn = name.encode() + b"\0"
    packed = bytearray((l + 1) // 2)
    for i, ch in enumerate(seq):
        packed[i >> 1] |= NT16.get(ch, 15) << (4 if i % 2 == 0 else 0)
    q = bytes(0xff for _ in range(l)) if qual is None else bytes(ord(c) - 33 for c in qual)
    core = struct.pack("<iiIIiiii", -1, -1, (4680 << 16) | (0 << 8) | len(qn), (flag << 16) | 0, l, -1, -1, 0)
    body = core + qn + bytes(packed) + q
    return struct.pack("<i", len(body)) + body


def main():
    recs = oracle.read_fastq_records(os.path.join(GOLD, "reads_mixed.fq"))
    out = bytearray(b"BAM\1" + struct.pack("<i", 0) + struct.pack("<i", 0))
    for j, rec in enumerate(recs):
        name, seq, qual = rec[0], rec[1].decode(), rec[2].decode() or None
        if j % 11 == 5:
            qual = None
        out += record(name, seq, qual, FLAGS[j % len(FLAGS)])
    path = os.path.join(GOLD, "reads.bam")
    with gzip.open(path, "wb") as f:
        f.write(bytes(out))
    manifest = {}
    for key, argv in OPTS.items():
        fo = os.path.join(GOLD, f"bam.{key}.sai")
        with open(fo, "wb") as f:
            subprocess.run([REF, "aln"] + argv + [os.path.join(GOLD, "g1m"), path], check=True, stdout=f,
                           stderr=subprocess.DEVNULL)
        manifest[key] = {"argv": argv, "sai": os.path.basename(fo)}
    with open(os.path.join(GOLD, "bam_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(len(recs), "records;", {k: os.path.getsize(os.path.join(GOLD, v["sai"])) for k, v in manifest.items()})


if __name__ == "__main__":
    main()
