#!/usr/bin/env python3
"""Generate tests/golden/samse_*.sam.gz: the reference's samse output (build container only).

TEST INFRASTRUCTURE.  The reference's own `samse` (bwa_sai2sam_se, bwase.c:643-740, compiled
into oracle/_ref/ibwa_ref with the harness in place of main.cpp) is run on golden .sai files
and their reads; the SAM text is committed gzip'd with samse_manifest.json (key -> .sai,
reads, options).  The @PG line names the program that wrote the file and is not compared.
"""
import gzip
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref", "ibwa_ref")

CASES = {
    "r100.default": ("r100.default.sai", "reads_r100.fq", []),
    "r100.n0": ("r100.n0.sai", "reads_r100.fq", []),
    "r100.n3o2e3": ("r100.n3o2e3.sai", "reads_r100.fq", []),
    "r100.N": ("r100.N.sai", "reads_r100.fq", []),
    "r100.R1": ("r100.R1.sai", "reads_r100.fq", []),
    "r100.default.n10": ("r100.default.sai", "reads_r100.fq", ["-n", "10"]),
    "r36.default": ("r36.default.sai", "reads_r36.fq", []),
    "r150.default": ("r150.default.sai", "reads_r150.fq", []),
    "mixed.default": ("mixed.default.sai", "reads_mixed.fq", []),
    "mixed.default.rg": ("mixed.default.sai", "reads_mixed.fq", ["-r", "@RG\\tID:grp1\\tSM:s1"]),
    "mixed.q15": ("mixed.q15.sai", "reads_mixed.fq", []),
    "mixed.B4": ("mixed.B4.sai", "reads_mixed.fq", []),
    "mixed.N": ("mixed.N.sai", "reads_mixed.fq", ["-n", "5"]),
    "mixed.n3o2e3": ("mixed.n3o2e3.sai", "reads_mixed.fq", []),
    "mixed.m50": ("mixed.m50.sai", "reads_mixed.fq", []),
    "illumina.I": ("illumina.I.sai", "reads_illumina.fq", []),
    "bam.all": ("bam.all.sai", "reads.bam", []),
    "bam.q15": ("bam.q15.sai", "reads.bam", []),
    # tandem-array genome (tools/make_sampe_golden.py): > 1000 equal hits, XA with -n 2000
    "tandem.default": ("tandem_1.sai", "tandem_1.fq", [], "tandem"),
    "tandem.n2000": ("tandem_1.sai", "tandem_1.fq", ["-n", "2000"], "tandem"),
}


def main():
    manifest = {}
    for key, (sai, reads, argv, *pre) in CASES.items():
        prefix = pre[0] if pre else "g1m"
        out = subprocess.run([REF, "samse"] + argv + [os.path.join(GOLD, prefix), os.path.join(GOLD, sai),
                                                      os.path.join(GOLD, reads)],
                             check=True, capture_output=True).stdout
        with open(os.path.join(GOLD, f"samse_{key}.sam.gz"), "wb") as raw:
            with gzip.GzipFile(fileobj=raw, mode="wb", mtime=0) as f:
                f.write(out)
        manifest[key] = {"prefix": prefix, "sai": sai, "reads": reads, "argv": argv, "sam": f"samse_{key}.sam.gz"}
        print(key, len(out.splitlines()), "lines")
    with open(os.path.join(GOLD, "samse_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
