"""Compressed input inflated on all host threads (ibwa_amd/csrc/gzsrc.h: GzSource, ByteStream) against
zlib's gzread, the reader the reference's kseq / bamlite sit on (bwaseqio.c:34-41, kseq.h:156-195,
bamlite.h:8): for BGZF, plain multi-member, single-member and mixed files -- and for the shapes gzread
treats specially (trailing bytes after a member, a bad CRC, a truncated member, header fields of every
kind, false member starts inside a stored member) -- the bytes handed on must be gzread's; on a file
gzread reports an error on, every byte before the bad member is handed on and the error is reported
(BAD below).  CPU only: builds tools/gz_check.cpp with g++."""
import os
import subprocess

import pytest

from tests import gz_util as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gzc(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("gz") / "gz_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe, os.path.join(ROOT, "tools", "gz_check.cpp"),
                    "-lz"], check=True)
    return exe


FQ = G.fastq_text(6000, 1)
FQ2 = G.fastq_text(3000, 2)


def _inner_gzip_stored():
    # a stored member whose payload is a whole gzip file and a BGZF block: valid members that start
    # inside another member's compressed bytes
    inner = G.member(FQ2[:50_000]) + G.bgzf(FQ2[50_000:120_000])
    return G.member(FQ[:30_000], level=0) + G.member(inner + FQ[30_000:60_000], level=0) + G.multi(FQ[60_000:], 3)


CASES = {
    "bgzf": lambda: G.bgzf(FQ),
    "bgzf_no_eof_block": lambda: G.bgzf(FQ, eof=False),
    "bgzf_small_blocks": lambda: G.bgzf(FQ, block=999),
    "single": lambda: G.member(FQ),
    "single_level1": lambda: G.member(FQ, level=1),
    "multi": lambda: G.multi(FQ, 1),
    "multi_tiny_members": lambda: G.multi(FQ[:200_000], 2, lo=1, hi=3000),
    "mixed": lambda: G.bgzf(FQ[:300_000], eof=False) + G.multi(FQ[300_000:600_000], 4) + G.bgzf(FQ[600_000:]),
    "empty_member": lambda: G.member(b""),
    "bgzf_eof_only": lambda: G.BGZF_EOF,
    "trailing_garbage_bgzf": lambda: G.bgzf(FQ) + b"this is not gzip\n" * 10,
    "trailing_garbage_multi": lambda: G.multi(FQ, 5) + b"\0" * 4096,
    "trailing_magic_byte": lambda: G.bgzf(FQ) + b"\x1f",
    "trailing_bad_header": lambda: G.bgzf(FQ) + b"\x1f\x8b\x09\x00" + b"x" * 40,
    "bad_crc_bgzf": lambda: G.bgzf(FQ[:400_000]) [:-28] + G.member(FQ[400_000:460_000], bgzf=True, bad_crc=True) +
    G.bgzf(FQ[460_000:]),
    "bad_crc_multi": lambda: G.multi(FQ[:400_000], 6) + G.member(FQ[400_000:700_000], bad_crc=True) + G.multi(FQ[700_000:], 7),
    "truncated_single": lambda: G.member(FQ)[:-50_000],
    "truncated_bgzf": lambda: G.bgzf(FQ)[:-30_000],
    "truncated_multi": lambda: G.multi(FQ, 8)[:-1000],
    "truncated_trailer": lambda: G.bgzf(FQ, eof=False)[:-3],
    "header_fields": lambda: (G.member(FQ[:100_000], fname=b"reads.fq") + G.member(FQ[100_000:300_000], fcomment=b"c" * 300) +
                              G.member(FQ[300_000:500_000], fextra=b"XY\x03\x00abc") +
                              G.member(FQ[500_000:700_000], fhcrc=True) + G.member(FQ[700_000:], fname=b"x", fhcrc=True)),
    "bad_header_crc": lambda: G.member(FQ[:300_000]) + G.member(FQ[300_000:], fhcrc=True, bad_hcrc=True),
    "false_starts_in_stored": _inner_gzip_stored,
}


def run(exe, mode, path, size, env=None):
    r = subprocess.run([exe, mode, str(path), str(size)], capture_output=True, timeout=120,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    return r.stdout, r.stderr.decode()


# Cases gzread reports an error on, with the uncompressed bytes that come before the bad member and the
# bytes the whole file would hold.  Exactly where gzread's output stops on such a file depends on its
# internal 16 KiB output buffers (a chunk ending in an error is dropped whole), so here the bar is: every
# byte before the bad member is handed on, nothing that is not in the file, and an error is reported.
BAD = {
    "trailing_bad_header": (len(FQ), FQ),
    "bad_crc_bgzf": (400_000, FQ),
    "bad_crc_multi": (400_000, FQ),
    "bad_header_crc": (300_000, FQ),
    "truncated_single": (0, FQ),
    "truncated_bgzf": (0, FQ),
    "truncated_multi": (0, FQ),
    "truncated_trailer": (0, FQ),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_stream_equals_gzread(gzc, tmp_path, name):
    p = tmp_path / (name + ".gz")
    p.write_bytes(CASES[name]())
    ref, ref_err = run(gzc, "gzread", p, 1 << 20)
    for size in (1, 4097, 1 << 20, 1 << 26):
        for env in ({"IBWA_GZ_THREADS": "8"}, {"IBWA_GZ_THREADS": "1", "IBWA_GZ_LIBDEFLATE": "0"},
                    {"IBWA_GZ_THREADS": "3", "IBWA_GZ_LIBDEFLATE": "0"}):
            if size == 1 and env["IBWA_GZ_THREADS"] != "8":
                continue
            got, err = run(gzc, "stream", p, size, env)
            if name in BAD:
                good, full = BAD[name]
                assert full.startswith(got) and len(got) >= good, (name, size, env, len(got))
                if not name.startswith("truncated"):
                    assert "error" in err and "error" in ref_err, (name, size, env, err)
            else:
                assert got == ref and "error" not in ref_err, (name, size, env, len(got), len(ref))
                assert "error" not in err, (name, size, env, err)


@pytest.mark.parametrize("name", ["bgzf", "single", "multi", "mixed", "false_starts_in_stored", "bad_crc_multi",
                                  "bad_crc_bgzf", "truncated_bgzf"])
@pytest.mark.parametrize("cap", [1000, 65536, 1 << 21, 1 << 27])
def test_source_reads_verified_bytes(gzc, tmp_path, name, cap):
    """GzSource in calls of `cap` bytes (FastqGpu's regions): a prefix of gzread's bytes, all of them
    when the stream is good; at a problem it stops with failed() (ByteStream then continues with gzread)."""
    p = tmp_path / (name + ".gz")
    p.write_bytes(CASES[name]())
    ref, ref_err = run(gzc, "gzread", p, 1 << 20)
    for env in ({"IBWA_GZ_THREADS": "8"}, {"IBWA_GZ_THREADS": "2", "IBWA_GZ_LIBDEFLATE": "0"}):
        got, err = run(gzc, "source", p, cap, env)
        if name in BAD:
            good, full = BAD[name]
            assert full.startswith(got) and len(got) >= good and "failed at" in err, (name, cap, env, err)
        else:
            assert got == ref and "eof at" in err, (name, cap, env, err)


SAN = {"asan": ["-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
       "tsan": ["-O1", "-fsanitize=thread"]}


@pytest.mark.parametrize("flavour", sorted(SAN))
def test_gzsrc_under_sanitizers(gzc, tmp_path, flavour):
    """The parallel spans, the speculative member starts and the read-ahead thread under
    AddressSanitizer + UBSan and ThreadSanitizer."""
    exe = str(tmp_path / f"gz_check_{flavour}")
    subprocess.run(["g++", "-std=c++17", "-g", "-pthread", *SAN[flavour], "-o", exe,
                    os.path.join(ROOT, "tools", "gz_check.cpp"), "-lz"], check=True)
    env = {"TSAN_OPTIONS": "halt_on_error=1", "ASAN_OPTIONS": "detect_leaks=1", "IBWA_GZ_THREADS": "4"}
    for name in ("bgzf", "multi", "mixed", "false_starts_in_stored", "bad_crc_multi", "truncated_single"):
        p = tmp_path / (name + ".gz")
        p.write_bytes(CASES[name]())
        full = BAD[name][1] if name in BAD else run(gzc, "gzread", p, 1 << 20)[0]
        for mode, size in (("stream", 4097), ("source", 65536)):
            r = subprocess.run([exe, mode, str(p), str(size)], capture_output=True, timeout=300,
                               env=dict(os.environ, **env))
            assert r.returncode == 0 and b"Sanitizer" not in r.stderr and b"runtime error" not in r.stderr, \
                r.stderr.decode()[-3000:]
            assert full.startswith(r.stdout), (name, mode)
