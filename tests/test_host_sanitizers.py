"""Sanitizer builds of the CLI's host-only code: readers.h (FASTQ/FASTA and BAM
parsing), sam_common.h (bwa_read_seq / bwa_read_bam record preparation, the Background parser
thread, parallel_chunks, print_parallel, .ann/.amb/.pac loading), compiled with g++ under
AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer, driven by
tests/host/host_check.cpp over the golden inputs and over truncated / corrupt BAM records.
CPU only (no HIP code is built here)."""
import gzip
import os
import struct
import subprocess

import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
SRC = os.path.join(ROOT, "tests", "host", "host_check.cpp")
OUT = os.path.join(ROOT, "tests", "_build")

FLAVOURS = {
    "plain": ["-O2"],
    "asan": ["-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
    "tsan": ["-O1", "-fsanitize=thread"],
}
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
           TSAN_OPTIONS="halt_on_error=1", OMP_NUM_THREADS="4")


@pytest.fixture(scope="module")
def bins():
    os.makedirs(OUT, exist_ok=True)
    out = {}
    for name, flags in FLAVOURS.items():
        exe = os.path.join(OUT, f"host_check_{name}")
        deps = [SRC] + [os.path.join(ROOT, "ibwa_amd", "csrc", f) for f in ("readers.h", "sam_common.h", "remap.h")]
        if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(d) for d in deps):
            subprocess.run(["g++", "-std=c++17", "-g", "-pthread", *flags, "-I", os.path.join(ROOT, "include"),
                            "-I", os.path.join(ROOT, "ibwa_amd", "csrc"), SRC, "-o", exe, "-lz"], check=True)
        out[name] = exe
    return out


def run(exe, *args):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, env=ENV, timeout=300)
    assert b"Sanitizer" not in r.stderr and b"runtime error" not in r.stderr, r.stderr.decode()[-3000:]
    return r


@pytest.mark.parametrize("fq,mode,trim", [("reads_r100.fq", 3, 0), ("reads_mixed.fq", 3, 15),
                                         ("reads_illumina.fq", 3 | 0x100, 20), ("reads_mixed.fq", 3 | (4 << 24), 0),
                                         ("idx_quirks.fa", 1, 0)])
def test_reads_fastq(bins, fq, mode, trim):
    outs = {}
    for name, exe in bins.items():
        r = run(exe, "reads", os.path.join(GOLD, fq), mode, trim)
        assert r.returncode == 0, (name, r.stderr.decode()[-2000:])
        outs[name] = r.stdout
    assert outs["asan"] == outs["plain"] == outs["tsan"]
    lines = outs["plain"].decode().splitlines()
    if fq.endswith(".fq") and not (mode >> 24):
        recs = oracle.read_fastq_records(os.path.join(GOLD, fq))
        assert len(lines) == len(recs)
        assert all(ln.split("\t")[0] == r[0].split()[0].removesuffix("/1").removesuffix("/2")
                   for ln, r in zip(lines, recs))


def _bam_records(raw):
    """Offsets of the alignment records of an uncompressed BAM stream."""
    l_text = struct.unpack_from("<i", raw, 4)[0]
    p = 8 + l_text
    n_ref = struct.unpack_from("<i", raw, p)[0]
    p += 4
    for _ in range(n_ref):
        l_name = struct.unpack_from("<i", raw, p)[0]
        p += 4 + l_name + 4
    offs = []
    while p < len(raw):
        offs.append(p)
        p += 4 + struct.unpack_from("<i", raw, p)[0]
    return offs


def test_reads_bam_and_corrupt_records(bins, tmp_path):
    bam = os.path.join(GOLD, "reads.bam")
    raw = gzip.decompress(open(bam, "rb").read())
    offs = _bam_records(raw)
    assert len(offs) > 10
    full = {}
    for name, exe in bins.items():
        r = run(exe, "reads", bam, 3, 0, 7)
        assert r.returncode == 0, (name, r.stderr.decode()[-2000:])
        full[name] = r.stdout
    assert full["asan"] == full["plain"] == full["tsan"]
    n_full = len(full["plain"].splitlines())
    assert n_full == len(offs)
    cases = []
    # truncated inside the fixed part, inside the variable part, and one byte short of the end
    for j, cut in [(5, offs[5] + 20), (7, offs[7] + 40), (len(offs) - 1, len(raw) - 1)]:
        cases.append((j, raw[:cut]))
    # a record whose l_seq claims more bases than the record holds / a negative l_seq
    for j, val in [(3, 100000), (4, -5)]:
        b = bytearray(raw)
        struct.pack_into("<i", b, offs[j] + 4 + 16, val)
        cases.append((j, bytes(b)))
    for i, (j, data) in enumerate(cases):
        f = tmp_path / f"bad{i}.bam"
        f.write_bytes(gzip.compress(data))
        for name, exe in bins.items():
            r = run(exe, "reads", f, 3, 0, 7)
            assert r.returncode == 3, (i, name, r.returncode, r.stderr.decode()[-2000:])
            # every record before the damaged one comes out unchanged
            assert r.stdout.splitlines() == full["plain"].splitlines()[:j], (i, name)


def test_bns_and_chunks(bins):
    outs = {name: run(exe, "bns", os.path.join(GOLD, "g1m")).stdout for name, exe in bins.items()}
    assert len(set(outs.values())) == 1
    l_pac, n_seqs = map(int, open(os.path.join(GOLD, "g1m.ann")).readline().split()[:2])
    assert outs["plain"].split()[:2] == [str(l_pac).encode(), str(n_seqs).encode()]
    for name, exe in bins.items():
        for n, t in [(0, 4), (1, 8), (255, 3), (100000, 8), (12345, 0)]:
            r = run(exe, "chunks", n, t)
            assert r.returncode == 0 and r.stdout.startswith(b"ok"), (name, n, t)


def test_remap_known_answers(bins, tmp_path):
    """remap.h (sampe -R: read_mapping_extract, remap_cigar, is_remapped_sequence_identical,
    translate_cigar) on 9 015 cases answered by the reference's own functions
    (tools/make_remap_unit.py over oracle/_ref/libibwa_ref.so, bwaremap.cpp / translate_cigar.cpp),
    in the plain, ASan/UBSan and TSan builds."""
    rows = [ln.rstrip("\n").split("\t") for ln in open(os.path.join(GOLD, "remap_unit.tsv"))]
    cases = "".join(c + "\n" for c, _ in rows).encode()
    for name, exe in bins.items():
        r = subprocess.run([exe, "remap"], input=cases, capture_output=True, env=ENV, timeout=300)
        assert r.returncode == 0 and b"Sanitizer" not in r.stderr and b"runtime error" not in r.stderr, \
            (name, r.stderr.decode()[-2000:])
        got = r.stdout.decode().splitlines()
        assert len(got) == len(rows)
        bad = [(c, a, g) for (c, a), g in zip(rows, got) if a != g]
        assert not bad, (name, bad[:5])


@pytest.mark.parametrize("text,n_seqs,expect", [
    (">a-chr1|1|10\n5M2I3M\n>b-chr1|exact|\n", 2, "1 [chr1 0 0 11 5M2I3M 1] [chr1 1 0 0  0]"),
    (">a-chr1|1|10\n5M\n2D3M\n>b-chr2|3|4", 2, "1 [chr1 0 0 11 5M2D3M 1] []"),  # an unterminated last header
    (">a-chr1|1|10\n5M\n3M", 1, "1 [chr1 0 0 11 5M3M 0]"),                       # an unterminated last CIGAR line
    ("", 1, "-1"), ("x\n", 1, "-1"), (">a-chr1|1|10\n>b-c|1|2\n", 1, "-1"), (">bad\n", 1, "-1"),
    (">a-chr1|1|10", 1, "1 []")])
def test_remap_file(bins, tmp_path, text, n_seqs, expect):
    """load_remappings (bwaremap.cpp:42-100) on .remap texts: headers, multi-line CIGARs, the
    std::getline end-of-file behaviour, the errors."""
    f = tmp_path / "x.remap"
    f.write_text(text)
    r = subprocess.run([bins["plain"], "remap"], input=f"L {f} {n_seqs}\n".encode(), capture_output=True, timeout=60)
    assert r.stdout.decode().strip() == expect
