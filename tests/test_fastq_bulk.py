"""The CLI's bulk FASTQ parser (readers.h FastqBulk: strict 4-line records split over threads)
against the serial kseq-semantics reader (SeqReader, bwaseqio.c / kseq.h record rules): for
regular and irregular inputs the records must be the same, in the same order, with the serial
reader taking over at the first record the bulk parser does not take.  CPU only: builds
tools/parse_check.cpp with g++."""
import gzip
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pc") / "parse_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-o", exe, os.path.join(ROOT, "tools", "parse_check.cpp"),
                    "-lz"], check=True)
    return exe


def fq(recs, nl="\n"):
    return "".join(f"@{n}{nl}{s}{nl}+{nl}{q}{nl}" for n, s, q in recs)


def reads(n, seed, lmin=30, lmax=150):
    r = random.Random(seed)
    out = []
    for k in range(n):
        ln = r.randint(lmin, lmax)
        s = "".join(r.choice("ACGTN") for _ in range(ln))
        q = "".join(chr(r.randint(33, 126)) for _ in range(ln))
        out.append((f"r{k} comment {k}", s, q))
    return out


CASES = {
    "regular": lambda: fq(reads(3000, 1)),
    "qual_starts_with_at": lambda: fq([(n, s, "@" + q[1:]) for n, s, q in reads(2000, 2)]),
    "crlf_midway": lambda: fq(reads(1000, 3)) + fq(reads(50, 4), "\r\n") + fq(reads(500, 5)),
    "fasta": lambda: "".join(f">c{k}\nACGTACGT\nGGCC\n" for k in range(300)),
    "multiline_seq_midway": lambda: fq(reads(800, 6)) + "@m1\nACGT\nACGT\n+\nIIIIIIII\n" + fq(reads(300, 7)),
    "long_qual_line": lambda: fq(reads(700, 8)) + "@x\nACGT\n+\nIIIII@y\n" + fq(reads(200, 9)),
    "short_qual": lambda: fq(reads(700, 10)) + "@x\nACGTACGT\n+\nIIII\n@y\nAC\n+\nII\n",
    "no_final_newline": lambda: fq(reads(900, 11))[:-1],
    "truncated_tail": lambda: fq(reads(900, 12)) + "@t\nACGT\n+",
    "blank_lines_between": lambda: fq(reads(400, 13)) + "\n\n" + fq(reads(400, 14)),
    "leading_garbage": lambda: "junk line\n" + fq(reads(400, 15)),
    "qual_with_space": lambda: fq(reads(600, 16)) + "@x\nACGT\n+\nII I\n" + fq(reads(100, 17)),
    "plus_line_with_name": lambda: "".join(f"@{n}\n{s}\n+{n}\n{q}\n" for n, s, q in reads(1500, 18)),
    "empty": lambda: "",
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("chunk,threads", [(1 << 28, 4), (4096, 3), (65536, 8)])
def test_bulk_equals_serial(checker, tmp_path, name, chunk, threads):
    text = CASES[name]()
    for gz in (False, True):
        p = tmp_path / (f"{name}.fq" + (".gz" if gz else ""))
        if gz:
            with gzip.open(p, "wt", newline="") as f:
                f.write(text)
        else:
            p.write_bytes(text.encode())
        ser = subprocess.run([checker, "serial", str(p)], capture_output=True, check=True).stdout
        blk = subprocess.run([checker, "bulk", str(p), str(chunk), str(threads)], capture_output=True, check=True).stdout
        assert blk == ser, (name, gz, chunk, threads)


SAN = {"asan": ["-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"],
       "tsan": ["-O1", "-fsanitize=thread"]}


@pytest.mark.parametrize("flavour", sorted(SAN))
def test_bulk_under_sanitizers(checker, tmp_path, flavour):
    """The threaded split (segment starts, per-thread record lists, the hand-off) under
    AddressSanitizer + UBSan and ThreadSanitizer."""
    exe = str(tmp_path / f"parse_check_{flavour}")
    subprocess.run(["g++", "-std=c++17", "-g", "-pthread", *SAN[flavour], "-o", exe,
                    os.path.join(ROOT, "tools", "parse_check.cpp"), "-lz"], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    for name in ("regular", "crlf_midway", "truncated_tail", "qual_starts_with_at"):
        p = tmp_path / f"{name}.fq"
        p.write_bytes(CASES[name]().encode())
        ser = subprocess.run([checker, "serial", str(p)], capture_output=True, check=True).stdout
        r = subprocess.run([exe, "bulk", str(p), "4096", "4"], capture_output=True, env=env, timeout=300)
        assert r.returncode == 0 and b"Sanitizer" not in r.stderr and b"runtime error" not in r.stderr, \
            r.stderr.decode()[-3000:]
        assert r.stdout == ser, name
