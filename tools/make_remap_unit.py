#!/usr/bin/env python3
"""Known answers for remap.h (sampe -R), from the reference's own functions (run in the build
container).

TEST INFRASTRUCTURE.  oracle/_ref/libibwa_ref.so (the reference compiled from its sources by
oracle/Makefile) is called through ctypes on seeded random and hand-picked cases of
read_mapping_extract, remap_cigar, is_remapped_sequence_identical (bwaremap.cpp) and
translate_cigar (translate_cigar.cpp); tests/golden/remap_unit.tsv holds each case and the
reference's answer in tests/host/host_check.cpp's `remap` format, which tests/test_remap_host.py
replays against remap.h (plain, ASan/UBSan and TSan builds)."""
import ctypes as C
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "libibwa_ref.so")
OUT = os.path.join(ROOT, "tests", "golden", "remap_unit.tsv")


class ReadMapping(C.Structure):  # read_mapping_t (bwaremap.h:9-17)
    _fields_ = [("seqname", C.c_char_p), ("exact", C.c_int), ("start", C.c_uint32), ("stop", C.c_uint32),
                ("cigar", C.c_char_p), ("n_gapo", C.c_int)]


def main():
    L = C.CDLL(REF, mode=os.RTLD_LAZY)  # its @PG printer lives in the harness executable, not needed here
    libc = C.CDLL("libc.so.6")
    L.read_mapping_extract.argtypes = [C.c_char_p, C.POINTER(ReadMapping)]
    L.remap_cigar.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32]
    L.is_remapped_sequence_identical.argtypes = [C.POINTER(ReadMapping), C.c_uint32, C.c_uint32]
    L.translate_cigar.restype = C.POINTER(C.c_uint32)
    L.translate_cigar.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32), C.c_int, C.c_int, C.POINTER(C.c_int)]
    rng = random.Random(20261017)

    def cigar(junk):
        s = ""
        for _ in range(rng.randrange(0, 6)):
            if junk and rng.random() < 0.05:
                s += "Q"
            if not (junk and rng.random() < 0.04):
                s += str(rng.randrange(1, 40) if rng.random() < 0.9 else 0)
            s += rng.choice("MMMMIDNX=")
        if junk and rng.random() < 0.1:
            s += str(rng.randrange(0, 9))
        return s or "-"

    rows = []
    for h in ["x-chr1|100|200", "a-b|exact", "a-b|exactly", "a--b|1|2", "a-b||2", "a-|1|2", "a-b|0|5", "a-b| 3|+4",
              "a-b|3|4x", "ab|1|2", "|a-b|1", "a-b|1|", "alt_7-chr17|41196312|41277500", "p|q-r|1|2", "a-b|1|2|3"]:
        m = ReadMapping()
        ok = L.read_mapping_extract(h.encode(), C.byref(m))
        rows.append((f"H {h}", f"{m.seqname.decode()} {m.exact} {m.start} {m.stop}" if ok else "fail"))
    for _ in range(3000):
        c = cigar(rng.random() < 0.25)
        # as the reference holds it (calloc'ed, bwaremap.cpp:79): bytes past the NUL are zero, which
        # its CIGAR cursor reads once the text is used up (translate_cigar.cpp:312-318)
        cc = C.create_string_buffer(b"" if c == "-" else c.encode(), len(c) + 16)
        pos, sl = rng.randrange(0, 120), rng.randrange(1, 150)
        r = C.c_uint32(0)
        ok = L.remap_cigar(cc, C.byref(r), pos, sl)
        rows.append((f"R {c} {pos} {sl}", str(r.value) if ok else "fail"))
        m = ReadMapping()
        m.cigar = C.cast(cc, C.c_char_p)
        m.exact = 1 if rng.random() < 0.1 else 0
        st = rng.randrange(0, 120) if rng.random() < 0.8 else 0xFFFFFFF0 + rng.randrange(0, 16)
        ln = rng.randrange(0, 120)
        rows.append((f"I {c} {m.exact} {st} {ln}", str(L.is_remapped_sequence_identical(C.byref(m), st, ln))))
        # translate: a read CIGAR of M/I/D/S/N runs, or none (an ungapped read)
        runs = [(rng.choice("MMMIDSN" if rng.random() < 0.9 else "MS"), rng.randrange(1, 30)) for _ in range(rng.randrange(0, 5))]
        rl = sum(n for op, n in runs if op in "MIS") or rng.randrange(1, 100)
        start = rng.randrange(0, 60)
        rc = "".join(f"{n}{op}" for op, n in runs) or "-"
        arr = (C.c_uint32 * (len(runs) + 1))(*[("MIDSN".index(op) << 29) | n for op, n in runs], 0)
        nout = C.c_int(0)
        p = L.translate_cigar(cc, start, arr if runs else None, len(runs), rl, C.byref(nout))
        if p:
            res = "".join(f"{p[j] & 0x1FFFFFFF}{'MIDSN'[p[j] >> 29]}" for j in range(nout.value))
            libc.free(p)
        else:
            res = "fail"
        rows.append((f"T {c} {start} {rc} {rl}", res))
    with open(OUT, "w") as f:
        for case, ans in rows:
            f.write(f"{case}\t{ans}\n")
    print(len(rows), "cases ->", OUT)


if __name__ == "__main__":
    main()
