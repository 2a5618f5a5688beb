#!/usr/bin/env python3
"""Golden fixtures for a FASTQ whose last record is truncated (run in the build container).

TEST INFRASTRUCTURE.  kseq_read (kseq.h:186, :191) returns -2 when the file ends inside a record's
quality; bwa_read_seq's loop (bwaseqio.c:159) stops there, keeping the reads before it, and aln
exits normally.  Two inputs, both the first 700 records of reads_r100.fq plus a truncated record:
  reads_trunc_q.fq   the last quality string shorter than its sequence (kseq.h:191)
  reads_trunc_p.fq   the file ends right after the '+' (kseq.h:186)
and the reference's `aln` .sai of each (oracle/_ref/ibwa_ref, built from /root/reference by
oracle/Makefile) go to tests/golden/ with trunc_manifest.json.
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference first: make -C oracle ref")
    lines = open(os.path.join(GOLD, "reads_r100.fq")).read().split("\n")
    head = "\n".join(lines[:4 * 700]) + "\n"
    tails = {"q": "@trunc_q\n" + "ACGT" * 20 + "\n+\n" + "I" * 37, "p": "@trunc_p\n" + "ACGT" * 20 + "\n+"}
    manifest = {}
    for tag, tail in tails.items():
        fq = os.path.join(GOLD, f"reads_trunc_{tag}.fq")
        with open(fq, "w") as f:
            f.write(head + tail)
        for oname, argv in (("default", []), ("n3o2e3", ["-n", "3", "-o", "2", "-e", "3"])):
            out = os.path.join(GOLD, f"trunc_{tag}.{oname}.sai")
            r = subprocess.run([REF, "aln", *argv, "-f", out, os.path.join(GOLD, "g1m"), fq], capture_output=True,
                               text=True)
            assert r.returncode == 0, r.stderr
            manifest[f"trunc_{tag}.{oname}"] = {"argv": argv, "reads": os.path.basename(fq),
                                                "sha1": hashlib.sha1(open(out, "rb").read()).hexdigest()}
    with open(os.path.join(GOLD, "trunc_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("truncated-input fixtures written to", GOLD)


if __name__ == "__main__":
    main()
