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
