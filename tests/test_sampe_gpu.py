"""The `ibwa-amd sampe` CLI (sampe_main.cpp: bwa_sai2sam_pe_core, bwape.c:436-540, with SA->coordinate, mate-rescue SW and
bwa_refine_gapped's global alignments on the GPU) against the reference's own sampe output on the
golden paired .sai files (tools/make_sampe_golden.py).  Every SAM line is compared byte for byte except
@PG, which names the program that wrote the file (bwa_print_sam_PG)."""
import gzip
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")
MANIFEST = json.load(open(os.path.join(ROOT, "tests", "golden", "sampe_manifest.json")))


def _body(text):
    return [ln for ln in text.splitlines() if not ln.startswith("@PG")]


@pytest.mark.parametrize("key", sorted(MANIFEST))
def test_sampe_matches_reference(golden_dir, key, tmp_path):
    m = MANIFEST[key]
    out = tmp_path / "out.sam"
    r = subprocess.run([CLI, "sampe"] + m["argv"] + ["-f", str(out), os.path.join(golden_dir, m.get("prefix", "g1m")),
                                                     *[os.path.join(golden_dir, x) for x in m["sai"]],
                                                     *[os.path.join(golden_dir, x) for x in m["reads"]]],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    want = _body(gzip.open(os.path.join(golden_dir, m["sam"]), "rt").read())
    got = _body(out.read_text())
    assert len(got) == len(want)
    bad = [(i, g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, f"{len(bad)} lines differ; first:\n got {bad[0][1]}\nwant {bad[0][2]}"


REMAP = json.load(open(os.path.join(ROOT, "tests", "golden", "remap_manifest.json")))


@pytest.mark.parametrize("key", sorted(REMAP))
def test_sampe_several_references_and_remap(golden_dir, key, tmp_path):
    """`sampe [-R] <pri> <1.sai> <2.sai> <1.fq> <2.fq> <alt> <a1.sai> <a2.sai>` (pe_inputs_parse,
    bwape.c:548-581) over the primary genome and an alternate-haplotype reference with a .remap
    table (tools/make_remap_golden.py): alngrp_create's merge of both references' records,
    remapped primary coordinates with ZR:Z, translated CIGARs, @SQ without the mapped alternates;
    without -R, and with -R but no .remap file.  Byte for byte except @PG."""
    m = REMAP[key]
    g = lambda x: os.path.join(golden_dir, x)  # noqa: E731
    args = [g(m["prefixes"][0]), *map(g, m["sai"][0]), *map(g, m["reads"])]
    for pre, sai in zip(m["prefixes"][1:], m["sai"][1:]):
        args += [g(pre), *map(g, sai)]
    out = tmp_path / "out.sam"
    r = subprocess.run([CLI, "sampe"] + m["argv"] + ["-f", str(out)] + args, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    want = _body(gzip.open(g(m["sam"]), "rt").read())
    got = _body(out.read_text())
    assert len(got) == len(want)
    bad = [(i, gl, w) for i, (gl, w) in enumerate(zip(got, want)) if gl != w]
    assert not bad, f"{len(bad)} lines differ; first:\n got {bad[0][1]}\nwant {bad[0][2]}"
    if "-R" in m["argv"] and m["prefixes"][1] == "remap_alt":
        assert any("\tZR:Z:" in ln for ln in got)


STALE = json.load(open(os.path.join(ROOT, "tests", "golden", "stale_manifest.json")))


def test_stale_fixture_separates_thread_counts(golden_dir):
    """The fixture pins something: the reference wrote different SAM with -t 1 and -t 3."""
    sams = {k: _body(gzip.open(os.path.join(golden_dir, m["sam"]), "rt").read()) for k, m in STALE.items()}
    assert len(sams["stale.R.t1"]) == len(sams["stale.R.t3"])
    assert sams["stale.R.t1"] != sams["stale.R.t3"]


@pytest.mark.parametrize("key", sorted(STALE))
def test_sampe_stale_slots_per_thread_count(golden_dir, key, tmp_path):
    """`sampe -R -t T`: find_optimal_pair's overlap run reads past the pair's own positions into what
    the last pair of the same reference thread left there (bwapair.c:197, bwape.c:249-253), and
    select_mapping looks that stale slot's alignment index up in the current pair's alignments
    (tools/make_sampe_stale_golden.py: with -t 1 the mate of pair B takes the record of its exact
    hit elsewhere, with -t 2 / -t 3 its own one-mismatch record).  sampe_main.cpp's PosView follows
    the nearest-greater chain of the pair's residue class mod T; byte for byte except @PG."""
    m = STALE[key]
    g = lambda x: os.path.join(golden_dir, x)  # noqa: E731
    args = [g(m["prefixes"][0]), *map(g, m["sai"][0]), *map(g, m["reads"])]
    for pre, sai in zip(m["prefixes"][1:], m["sai"][1:]):
        args += [g(pre), *map(g, sai)]
    out = tmp_path / "out.sam"
    r = subprocess.run([CLI, "sampe"] + m["argv"] + ["-f", str(out)] + args, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    want = _body(gzip.open(g(m["sam"]), "rt").read())
    got = _body(out.read_text())
    assert len(got) == len(want)
    bad = [(i, gl, w) for i, (gl, w) in enumerate(zip(got, want)) if gl != w]
    assert not bad, f"{len(bad)} lines differ; first:\n got {bad[0][1]}\nwant {bad[0][2]}"


def test_sampe_incomplete_reference_group(golden_dir):
    """A trailing reference without both .sai files is refused (pe_inputs_parse)."""
    g = lambda x: os.path.join(golden_dir, x)  # noqa: E731
    r = subprocess.run([CLI, "sampe", g("g1m"), g("pe70few.default_1.sai"), g("pe70few.default_2.sai"),
                        g("pe70few_1.fq"), g("pe70few_2.fq"), g("g1m"), g("pe70few.default_1.sai")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "insufficient arguments" in r.stderr


@pytest.mark.parametrize("key", ["pe100.default", "pe100.q20", "pe100.k0n3", "pe150.default", "tandem.R"])
def test_aln_pe_reads_match_reference_sai(golden_dir, key, tmp_path):
    """`ibwa-amd aln` on each end of the paired fixtures writes the reference's .sai bytes."""
    import oracle
    m = MANIFEST[key]
    for sai, reads in zip(m["sai"], m["reads"]):
        out = tmp_path / "out.sai"
        r = subprocess.run([CLI, "aln"] + m["aln_argv"] + ["-f", str(out), os.path.join(golden_dir, m.get("prefix", "g1m")),
                                                           os.path.join(golden_dir, reads)],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert oracle.sai_body_equal(out.read_bytes(), open(os.path.join(golden_dir, sai), "rb").read())


@pytest.mark.parametrize("aln_opts", [["-B", "5"], ["-I", "-q", "15"], []])
def test_sampe_bulk_reader_equals_serial(golden_dir, aln_opts, tmp_path):
    """sampe's reads come from the bulk FASTQ parser on host threads (sampe_main.cpp Source::take,
    rec_to_read) until the first record it does not take, then from the serial kseq reader
    (bwaseqio.c:145-208).  With barcodes (-B), Illumina 1.3 qualities (-I) and trimming (-q) in the
    .sai header's mode, and end 2 holding a multi-line record midway (the hand-over), the SAM equals
    the one of the serial reader alone (IBWA_SAMPE_SERIAL_READ=1) byte for byte."""
    g = lambda x: os.path.join(golden_dir, x)  # noqa: E731
    recs = open(g("pe100_2.fq")).read().split("\n")
    k = 4 * (len(recs) // 8)  # a record in the middle: its sequence over two lines
    s = recs[k + 1]
    recs[k + 1] = s[:40] + "\n" + s[40:]
    fq2 = tmp_path / "r2.fq"
    fq2.write_text("\n".join(recs))
    fq = [g("pe100_1.fq"), str(fq2)]
    sai = []
    for j, f in enumerate(fq):
        out = tmp_path / f"{j}.sai"
        r = subprocess.run([CLI, "aln"] + aln_opts + ["-f", str(out), g("g1m"), f], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        sai.append(str(out))
    outs = []
    for serial in (False, True):
        out = tmp_path / f"out{int(serial)}.sam"
        env = dict(os.environ)
        if serial:
            env["IBWA_SAMPE_SERIAL_READ"] = "1"
        r = subprocess.run([CLI, "sampe", "-R", "-f", str(out), g("g1m"), *sai, *fq], capture_output=True, text=True,
                           timeout=120, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(_body(out.read_text()))
    assert len(outs[0]) > 1000
    assert outs[0] == outs[1]


def _sampe(argv, args, out, env=None):
    r = subprocess.run([CLI, "sampe"] + argv + ["-f", str(out)] + args, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-2000:]
    return out.read_text(), r.stderr


@pytest.mark.parametrize("key", sorted(MANIFEST))
def test_sampe_two_workers_match_reference(golden_dir, key, tmp_path):
    """`sampe -G 2` on one GPU (sampe_main.cpp Worker: the second worker's contexts share the first's
    index): the reference's SAM, byte for byte except @PG."""
    m = MANIFEST[key]
    g = lambda x: os.path.join(golden_dir, x)  # noqa: E731
    got, _ = _sampe(m["argv"] + ["-G", "2"], [g(m.get("prefix", "g1m")), *map(g, m["sai"]), *map(g, m["reads"])],
                    tmp_path / "out.sam")
    assert _body(got) == _body(gzip.open(g(m["sam"]), "rt").read())


def test_sampe_workers_equal_one_worker_on_small_batches(golden_dir, tmp_path):
    """The batch loop sharded over -G 2 / -G 3 workers (bwape.c:476-536 batch by batch) writes what
    one worker writes, on batches of 29 pairs (IBWA_SAMPE_BATCH) so that every worker takes many:
    the drand48 draws taken in batch order, the wide intervals' cached positions computed with their
    first use in the run (tandem: intervals of >= 1000 rows), the previous batch's insert size where a
    batch has too few good pairs (bwape.c:410-411), SAM in file order; one reference and two."""
    g = lambda x: os.path.join(golden_dir, x)  # noqa: E731
    env = {"IBWA_SAMPE_BATCH": "29"}
    cases = [(MANIFEST[k]["argv"], [g(MANIFEST[k].get("prefix", "g1m")), *map(g, MANIFEST[k]["sai"]),
                                    *map(g, MANIFEST[k]["reads"])])
             for k in ("pe100.default", "pe100.noR", "pe100.n5N20", "tandem.R", "tandemt.R.t3", "pe150.default")]
    for k in ("remap.R", "remap.noR"):
        m = REMAP[k]
        args = [g(m["prefixes"][0]), *map(g, m["sai"][0]), *map(g, m["reads"])]
        for pre, sai in zip(m["prefixes"][1:], m["sai"][1:]):
            args += [g(pre), *map(g, sai)]
        cases.append((m["argv"], args))
    fell_back = False
    for argv, args in cases:
        one, err = _sampe(argv + ["-G", "1"], args, tmp_path / "g1.sam", env)
        fell_back = fell_back or "too few good pairs" in err
        assert len(one.splitlines()) > 100
        for n, ahead in (("2", "2"), ("3", "5"), ("2", "1")):  # IBWA_SAMPE_READ_AHEAD: batches read ahead
            got, _ = _sampe(argv + ["-G", n], args, tmp_path / f"g{n}.sam", dict(env, IBWA_SAMPE_READ_AHEAD=ahead))
            assert got == one, (argv, n, ahead)
    assert fell_back  # some batch took the previous batch's insert size


def test_sampe_gzip_reads(golden_dir, tmp_path):
    """sampe reading both ends as compressed FASTQ -- end 1 BGZF, end 2 plain multi-member gzip, both
    inflated on the host threads (gzsrc.h) -- gives the reference's SAM on the uncompressed files."""
    from tests import gz_util as G
    key = sorted(MANIFEST)[0]
    m = MANIFEST[key]
    reads = []
    for j, x in enumerate(m["reads"]):
        data = open(os.path.join(golden_dir, x), "rb").read()
        p = tmp_path / f"r{j}.fq.gz"
        p.write_bytes(G.bgzf(data, block=9000) if j == 0 else G.multi(data, 5, 1, 30_000))
        reads.append(str(p))
    out = tmp_path / "out.sam"
    r = subprocess.run([CLI, "sampe"] + m["argv"] + ["-f", str(out), os.path.join(golden_dir, m.get("prefix", "g1m")),
                                                     *[os.path.join(golden_dir, x) for x in m["sai"]], *reads],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    want = _body(gzip.open(os.path.join(golden_dir, m["sam"]), "rt").read())
    assert _body(out.read_text()) == want
