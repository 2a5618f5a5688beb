"""The `ibwa-amd aln` CLI (aln_main.cpp) against the reference's `aln` output: FASTQ input over
a cross-section of the option matrix, and BAM input (-b, -0/-1/-2, bwa_read_bam
bwaseqio.c:89-143) on tests/golden/reads.bam (tools/make_bam_golden.py).  Byte-identical .sai,
n_threads header field masked (bwtaln.c:192)."""
import json
import os
import subprocess

import pytest

import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")
FASTQ_KEYS = ["r100.default", "mixed.default", "r36.n0", "mixed.n3o2e3", "mixed.q15", "mixed.B4", "illumina.I",
              "mixed.c", "r100.t4", "mixed.N"]


def run_cli(argv, golden_dir, reads, tmp_path):
    out = tmp_path / "out.sai"
    r = subprocess.run([CLI, "aln"] + argv + ["-f", str(out), os.path.join(golden_dir, "g1m"),
                                              os.path.join(golden_dir, reads)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_bytes()


@pytest.mark.parametrize("key", FASTQ_KEYS)
def test_cli_fastq(golden_dir, sai_manifest, key, tmp_path):
    m = sai_manifest[key]
    got = run_cli(m["argv"], golden_dir, m["reads"], tmp_path)
    assert oracle.sai_body_equal(got, open(os.path.join(golden_dir, key + ".sai"), "rb").read())


@pytest.mark.parametrize("key", ["all", "se", "r1", "r2", "r12", "q15", "n0"])
def test_cli_bam(golden_dir, key, tmp_path):
    m = json.load(open(os.path.join(golden_dir, "bam_manifest.json")))[key]
    got = run_cli(m["argv"], golden_dir, "reads.bam", tmp_path)
    assert oracle.sai_body_equal(got, open(os.path.join(golden_dir, m["sai"]), "rb").read())


def test_cli_rejects_non_bam(golden_dir, tmp_path):
    r = subprocess.run([CLI, "aln", "-b", os.path.join(golden_dir, "g1m"), os.path.join(golden_dir, "reads_r36.fq")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "BAM" in r.stderr


def run_cli_env(argv, golden_dir, reads, tmp_path, env, name):
    out = tmp_path / name
    r = subprocess.run([CLI, "aln"] + argv + ["-f", str(out), os.path.join(golden_dir, "g1m"),
                                              os.path.join(golden_dir, reads)],
                       capture_output=True, text=True, timeout=120, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_bytes()


@pytest.mark.parametrize("key", ["r100.default", "r36.n0", "r150.default"])
def test_cli_grouped_batches_fixed_length(golden_dir, sai_manifest, key, tmp_path):
    """Batches of one read length share their batch-level options (bwtaln.c:86-93), so a GPU run
    over several of them (aln_main.cpp read_group) gives the reference's single-batch output."""
    m = sai_manifest[key]
    got = run_cli_env(m["argv"], golden_dir, m["reads"], tmp_path,
                      {"IBWA_ALN_SUBBATCH": "128", "IBWA_ALN_GROUP": "5"}, "g.sai")
    assert oracle.sai_body_equal(got, open(os.path.join(golden_dir, key + ".sai"), "rb").read())


@pytest.mark.parametrize("argv", [[], ["-q", "15"], ["-n", "0.01"]])
def test_cli_grouped_batches_equal_one_at_a_time(golden_dir, argv, tmp_path):
    """Mixed read lengths: small batches whose longest reads give different batch-level max_diff
    are split between groups; grouped runs == the same batches aligned one at a time."""
    reads = "reads_mixed.fq"
    one = run_cli_env(argv, golden_dir, reads, tmp_path, {"IBWA_ALN_SUBBATCH": "16", "IBWA_ALN_GROUP": "1"}, "a.sai")
    grp = run_cli_env(argv, golden_dir, reads, tmp_path, {"IBWA_ALN_SUBBATCH": "16", "IBWA_ALN_GROUP": "4"}, "b.sai")
    assert one[64:] == grp[64:]


@pytest.mark.parametrize("key", ["r100.default", "r36.n0"])
def test_cli_overlapped_groups(golden_dir, sai_manifest, key, tmp_path):
    """Consecutive groups overlapped on 1, 2 or 3 contexts sharing one index (IBWA_ALN_LANES,
    ibwa_ctx_share_index): the .sai keeps input order and equals the reference's."""
    m = sai_manifest[key]
    exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
    for lanes in ("1", "2", "3"):
        got = run_cli_env(m["argv"], golden_dir, m["reads"], tmp_path,
                          {"IBWA_ALN_SUBBATCH": "64", "IBWA_ALN_GROUP": "2", "IBWA_ALN_LANES": lanes}, f"l{lanes}.sai")
        assert oracle.sai_body_equal(got, exp), lanes


@pytest.mark.parametrize("argv", [[], ["-q", "15"], ["-B", "4"], ["-I"]])
def test_cli_bulk_parse_equals_serial(golden_dir, argv, tmp_path):
    """The threaded FASTQ path (readers.h FastqBulk) and its hand-off to the serial reader: a file
    whose strict 4-line records are followed by CRLF and multi-line records gives the .sai of
    the serial reader alone (IBWA_ALN_SERIAL_READ=1), with the switch falling inside a batch."""
    src = open(os.path.join(golden_dir, "reads_mixed.fq"), "rb").read().split(b"\n")
    recs = [src[i:i + 4] for i in range(0, len(src) - 3, 4)]
    head, mid, tail = recs[:len(recs) // 2], recs[len(recs) // 2:len(recs) // 2 + 40], recs[len(recs) // 2 + 40:]
    text = b"".join(b"\n".join(r) + b"\n" for r in head)
    text += b"".join(b"\r\n".join(r) + b"\r\n" for r in mid)  # CRLF: serial from here
    for r in tail:  # sequence wrapped over two lines
        s = r[1]
        text += r[0] + b"\n" + s[:len(s) // 2] + b"\n" + s[len(s) // 2:] + b"\n" + r[2] + b"\n" + r[3] + b"\n"
    fq = tmp_path / "mixed_irregular.fq"
    fq.write_bytes(text)
    env = {"IBWA_ALN_SUBBATCH": "96", "IBWA_ALN_GROUP": "3"}
    bulk = run_cli_env(argv, golden_dir, str(fq), tmp_path, env, "bulk.sai")
    ser = run_cli_env(argv, golden_dir, str(fq), tmp_path, dict(env, IBWA_ALN_SERIAL_READ="1"), "ser.sai")
    assert len(bulk) > 64 and bulk[64:] == ser[64:]


@pytest.mark.parametrize("key", ["trunc_q.default", "trunc_q.n3o2e3", "trunc_p.default", "trunc_p.n3o2e3"])
def test_cli_truncated_last_record(golden_dir, key, tmp_path):
    """A FASTQ that ends inside its last record (kseq_read's -2, kseq.h:186/:191): the reference's
    read loop stops there keeping every earlier read (bwaseqio.c:159) and aln exits 0; so does the
    CLI, with the bulk parser and with the serial reader (tools/make_trunc_golden.py)."""
    m = json.load(open(os.path.join(golden_dir, "trunc_manifest.json")))[key]
    gold = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
    got = run_cli(m["argv"], golden_dir, m["reads"], tmp_path)
    assert oracle.sai_body_equal(got, gold)
    got = run_cli_env(m["argv"], golden_dir, m["reads"], tmp_path, {"IBWA_ALN_SERIAL_READ": "1"}, "s.sai")
    assert oracle.sai_body_equal(got, gold)


@pytest.mark.parametrize("key", ["r100.default", "mixed.default", "r36.n0"])
def test_cli_multi_gpu_rehearsal(golden_dir, sai_manifest, key, tmp_path):
    """`aln -G 2` / `-G 3` on one GPU (slice g runs on device g mod the visible devices,
    aln_main.cpp): the index replicated device to device (ibwa_ctx_clone_index), each group split
    into per-GPU slices that keep the batch-level options (bwtaln.c:89-93), the slices' records
    written in input order, with two overlapped lanes per slice.  Small groups so that every slice
    holds reads.  The .sai equals -G 1's and the reference's."""
    m = sai_manifest[key]
    gold = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
    env = {"IBWA_ALN_SUBBATCH": "96", "IBWA_ALN_GROUP": "2", "IBWA_ALN_LANES": "2"}
    one = run_cli_env(m["argv"] + ["-G", "1"], golden_dir, m["reads"], tmp_path, env, "g1.sai")
    assert oracle.sai_body_equal(one, gold)
    for g in ("2", "3"):
        got = run_cli_env(m["argv"] + ["-G", g], golden_dir, m["reads"], tmp_path, env, f"g{g}.sai")
        assert got[64:] == one[64:], g


def _variety_fastq(path, n, seed, crlf_at=None, truncate=False):
    """Strict 4-line FASTQ of reads drawn from the golden genome with what bwa_read_seq branches on:
    lengths 20-160 (some not longer than a barcode), lower case, N, '-', low-quality tails, long and
    empty headers; optionally CRLF records from crlf_at on (the host readers take over there) and a
    truncated last record."""
    import random
    from tests.synth_util import golden_genome_ascii
    g, _, _ = golden_genome_ascii()
    rng = random.Random(seed)
    out = []
    for i in range(n):
        L = rng.choice([20, 36, 70, 100, 100, 100, 150, 160, 4, 8])
        p = rng.randrange(0, len(g) - L)
        s = list(g[p:p + L].replace("N", "A"))
        for _ in range(rng.randrange(0, 4)):
            s[rng.randrange(L)] = rng.choice("ACGTacgtN-")
        if rng.random() < 0.2:
            s = [c.lower() for c in s]
        q = [chr(33 + rng.randint(25, 40)) for _ in range(L)]
        if rng.random() < 0.3:
            for j in range(max(0, L - rng.randint(5, 40)), L):
                q[j] = chr(33 + rng.randint(2, 12))
        name = "" if rng.random() < 0.02 else f"v{i} some comment {rng.random()}"
        eol = "\r\n" if crlf_at is not None and i >= crlf_at else "\n"
        out.append(f"@{name}{eol}{''.join(s)}{eol}+{eol}{''.join(q)}{eol}")
    text = "".join(out)
    if truncate:
        text = text[:-7]
    path.write_text(text)


@pytest.mark.parametrize("argv", [[], ["-B", "5"], ["-q", "20"], ["-I", "-q", "15"], ["-n", "0"], ["-B", "3", "-q", "10"]])
@pytest.mark.parametrize("shape", ["plain", "crlf", "truncated"])
def test_cli_gpu_parse_equals_host(golden_dir, argv, shape, tmp_path):
    """FASTQ parsed on the GPU (ingest.h, fastq.hip) == the host readers (IBWA_ALN_GPU_PARSE=0) ==
    the serial kseq reader: small regions (IBWA_FQ_PIECE_BYTES) so that batches straddle regions and
    are parsed again, a second GPU slice (-G 2 on one device: pieces split at record starts), CRLF
    records in the middle (the host readers take over at the first batch they fall in) and a
    truncated last record."""
    fq = tmp_path / "v.fq"
    _variety_fastq(fq, 3000, 7, crlf_at=1700 if shape == "crlf" else None, truncate=shape == "truncated")
    env = {"IBWA_ALN_SUBBATCH": "200", "IBWA_ALN_GROUP": "3"}
    host = run_cli_env(argv, golden_dir, str(fq), tmp_path, dict(env, IBWA_ALN_GPU_PARSE="0"), "host.sai")
    ser = run_cli_env(argv, golden_dir, str(fq), tmp_path, dict(env, IBWA_ALN_SERIAL_READ="1"), "ser.sai")
    assert len(host) > 64 and host[64:] == ser[64:]
    # IBWA_FQ_MMAP: regions parsed where the mapped file holds them (default) or read into pinned buffers
    for extra, piece, mm in (([], "1000000000", "1"), ([], "40000", "1"), ([], "40000", "0"), (["-G", "2"], "30000", "1"),
                             (["-G", "2"], "30000", "0")):
        dev = run_cli_env(argv + extra, golden_dir, str(fq), tmp_path,
                          dict(env, IBWA_FQ_PIECE_BYTES=piece, IBWA_FQ_MMAP=mm), "dev.sai")
        assert dev[64:] == host[64:], (extra, piece, mm)


def test_cli_gpu_parse_carry_overflow(golden_dir, sai_manifest, tmp_path):
    """A batch whose bytes do not fit the carry room hands the rest to the host readers; the .sai is
    still the reference's."""
    m = sai_manifest["r100.default"]
    gold = open(os.path.join(golden_dir, "r100.default.sai"), "rb").read()
    for mm in ("1", "0"):
        got = run_cli_env(m["argv"], golden_dir, m["reads"], tmp_path,
                          {"IBWA_ALN_SUBBATCH": "500", "IBWA_FQ_PIECE_BYTES": "20000", "IBWA_FQ_CARRY_BYTES": "4096",
                           "IBWA_FQ_MMAP": mm}, "c.sai")
        assert oracle.sai_body_equal(got, gold), mm


def test_cli_gpu_parse_more_than_2_24_records(golden_dir, tmp_path):
    """One parsed block holding more than 2^24 records: the device scan packs each
    record's kept-read rank and code offset into one 64-bit key (fastq.hip KeptKey), 32 bits each
    -- a block is < 4 GiB, so neither half can wrap.  17 M tiny records (20 bp, empty headers, 46 B
    each: one 780 MB piece) aligned with -n 0 from the GPU parse == the host readers' .sai."""
    import numpy as np
    n, L = (1 << 24) + 300_000, 20
    rng = np.random.default_rng(5)
    rec = np.empty((n, 2 + L + 1 + 2 + L + 1), dtype=np.uint8)
    rec[:, 0] = ord("@")
    rec[:, 1] = ord("\n")
    rec[:, 2:2 + L] = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, (n, L), dtype=np.uint8)]
    rec[:, 2 + L] = ord("\n")
    rec[:, 3 + L] = ord("+")
    rec[:, 4 + L] = ord("\n")
    rec[:, 5 + L:5 + 2 * L] = ord("I")
    rec[:, 5 + 2 * L] = ord("\n")
    fq = tmp_path / "tiny.fq"
    rec.tofile(str(fq))
    del rec
    host = run_cli_env(["-n", "0"], golden_dir, str(fq), tmp_path, {"IBWA_ALN_GPU_PARSE": "0"}, "host.sai")
    dev = run_cli_env(["-n", "0"], golden_dir, str(fq), tmp_path, {"IBWA_FQ_PIECE_BYTES": str(1 << 30)}, "dev.sai")
    assert len(host) > 64 + 4 * n
    assert dev[64:] == host[64:]


def _gz(path, shape, seed=0):
    """The file at `path` recompressed as BGZF, plain multi-member gzip or one member (tests/gz_util.py)."""
    from tests import gz_util as G
    data = open(path, "rb").read()
    return {"bgzf": lambda: G.bgzf(data), "multi": lambda: G.multi(data, seed, 1, 40_000),
            "single": lambda: G.member(data)}[shape]()


@pytest.mark.parametrize("shape", ["bgzf", "multi", "single"])
@pytest.mark.parametrize("key", ["r100.default", "mixed.default", "mixed.q15", "r36.n0", "mixed.B4"])
def test_cli_gzip_fastq(golden_dir, sai_manifest, key, shape, tmp_path):
    """Compressed FASTQ (the reference reads it through gzread, bwaseqio.c:34-41): members inflated on
    the host threads (gzsrc.h GzSource: BGZF spans in place, plain members from speculative starts, one
    member on one thread) and the records parsed on the GPU (ingest.h), in regions small enough that
    batches straddle them; also through the host readers (ByteStream read-ahead) and through plain
    gzread (IBWA_GZ_PARALLEL=0).  Every .sai equals the reference's."""
    m = sai_manifest[key]
    gold = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
    gz = tmp_path / (m["reads"] + ".gz")
    gz.write_bytes(_gz(os.path.join(golden_dir, m["reads"]), shape))
    env = {"IBWA_ALN_SUBBATCH": "200", "IBWA_ALN_GROUP": "3"}
    for name, extra in (("dev", {}), ("dev_small", {"IBWA_FQ_PIECE_BYTES": "30000"}),
                        ("dev_g2", {"IBWA_FQ_PIECE_BYTES": "30000", "IBWA_GZ_THREADS": "3"}),
                        ("host", {"IBWA_ALN_GPU_PARSE": "0"}), ("gzread", {"IBWA_GZ_PARALLEL": "0"})):
        argv = m["argv"] + (["-G", "2"] if name == "dev_g2" else [])
        got = run_cli_env(argv, golden_dir, str(gz), tmp_path, dict(env, **extra), name + ".sai")
        assert oracle.sai_body_equal(got, gold), (shape, name)


def test_cli_gzip_corrupt_member(golden_dir, sai_manifest, tmp_path):
    """A BGZF file whose member in the middle has a bad CRC: the reference's read loop ends at gzread's
    error (kseq sees the end of the stream); the CLI keeps the reads before the bad member and exits 0,
    on the GPU-parse and host-reader paths alike.  Which records of the chunk before the error gzread
    drops depends on its internal buffers, so the bar is a prefix of the golden records holding every
    read of the members before the bad one."""
    from tests import gz_util as G
    m = sai_manifest["r100.default"]
    gold = open(os.path.join(golden_dir, "r100.default.sai"), "rb").read()
    data = open(os.path.join(golden_dir, m["reads"]), "rb").read()
    cut = len(data) * 2 // 3
    gz = tmp_path / "bad.fq.gz"
    gz.write_bytes(G.bgzf(data[:cut], eof=False) + G.member(data[cut:cut + 30000], bgzf=True, bad_crc=True) +
                   G.bgzf(data[cut + 30000:]))
    n_before = data[:cut].count(b"\n") // 4 - 1
    for extra in ({}, {"IBWA_ALN_GPU_PARSE": "0"}, {"IBWA_FQ_PIECE_BYTES": "30000"}):
        got = run_cli_env(m["argv"], golden_dir, str(gz), tmp_path, dict({"IBWA_ALN_SUBBATCH": "200"}, **extra), "x.sai")
        assert gold[64:].startswith(got[64:]), extra
        # every read before the bad member: n_aln records counted through the body
        body, k, pos = got[64:], 0, 0
        while pos < len(body):
            n = int.from_bytes(body[pos:pos + 4], "little", signed=True)
            pos += 4 + 16 * n
            k += 1
        assert k >= n_before - 200, (extra, k, n_before)


@pytest.mark.parametrize("shape", ["bgzf", "multi"])
def test_cli_gzip_bam_equals_golden(golden_dir, shape, tmp_path):
    """BAM through the parallel BGZF inflate (ByteStream): every golden BAM selection, and the same BAM
    re-blocked as plain gzip members."""
    from tests import gz_util as G
    import gzip as _gzip
    raw = _gzip.decompress(open(os.path.join(golden_dir, "reads.bam"), "rb").read())
    bam = tmp_path / "reads.bam"
    bam.write_bytes(G.bgzf(raw, block=20_000) if shape == "bgzf" else G.multi(raw, 3, 1, 9000))
    man = json.load(open(os.path.join(golden_dir, "bam_manifest.json")))
    for key in ("all", "r1", "q15"):
        m = man[key]
        got = run_cli_env(m["argv"], golden_dir, str(bam), tmp_path, {"IBWA_GZ_THREADS": "5"}, key + ".sai")
        assert oracle.sai_body_equal(got, open(os.path.join(golden_dir, m["sai"]), "rb").read()), key
