"""The `ibwa-amd samse` CLI (samse_main.cpp: bwa_sai2sam_se, bwase.c:643-740, with SA->coordinate and
bwa_refine_gapped's global alignments on the GPU) against the reference's own samse output on the
golden .sai files (tools/make_samse_golden.py).  Every SAM line is compared byte for byte except
@PG, which names the program that wrote the file (bwa_print_sam_PG)."""
import gzip
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")
MANIFEST = json.load(open(os.path.join(ROOT, "tests", "golden", "samse_manifest.json")))


def _body(text):
    return [ln for ln in text.splitlines() if not ln.startswith("@PG")]


@pytest.mark.parametrize("key", sorted(MANIFEST))
def test_samse_matches_reference(golden_dir, key, tmp_path):
    m = MANIFEST[key]
    out = tmp_path / "out.sam"
    r = subprocess.run([CLI, "samse"] + m["argv"] + ["-f", str(out), os.path.join(golden_dir, m.get("prefix", "g1m")),
                                                     os.path.join(golden_dir, m["sai"]),
                                                     os.path.join(golden_dir, m["reads"])],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    want = _body(gzip.open(os.path.join(golden_dir, m["sam"]), "rt").read())
    got = _body(out.read_text())
    assert len(got) == len(want)
    bad = [(i, g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, f"{len(bad)} lines differ; first:\n got {bad[0][1]}\nwant {bad[0][2]}"


def test_samse_rejects_bad_rg(golden_dir, tmp_path):
    r = subprocess.run([CLI, "samse", "-r", "RG\\tID:x", os.path.join(golden_dir, "g1m"),
                        os.path.join(golden_dir, "r36.default.sai"), os.path.join(golden_dir, "reads_r36.fq")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "@RG" in r.stderr


@pytest.mark.parametrize("aln_opts", [["-B", "5"], ["-I", "-q", "15"]])
def test_samse_bulk_reader_equals_serial(golden_dir, aln_opts, tmp_path):
    """samse's reads come from the bulk FASTQ parser on host threads (sam_common.h take_reads) up to
    the first record it does not take, then from the serial kseq reader: with a multi-line record
    midway, barcodes / Illumina 1.3 qualities / trimming in the .sai header's mode, the SAM equals the
    serial reader's alone (IBWA_SAMSE_SERIAL_READ=1) byte for byte."""
    g = lambda x: os.path.join(golden_dir, x)  # noqa: E731
    recs = open(g("pe100_1.fq")).read().split("\n")
    k = 4 * (len(recs) // 8)
    recs[k + 1] = recs[k + 1][:40] + "\n" + recs[k + 1][40:]
    fq = tmp_path / "r.fq"
    fq.write_text("\n".join(recs))
    sai = tmp_path / "r.sai"
    r = subprocess.run([CLI, "aln"] + aln_opts + ["-f", str(sai), g("g1m"), str(fq)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    outs = []
    for serial in (False, True):
        out = tmp_path / f"out{int(serial)}.sam"
        env = dict(os.environ)
        if serial:
            env["IBWA_SAMSE_SERIAL_READ"] = "1"
        r = subprocess.run([CLI, "samse", "-f", str(out), g("g1m"), str(sai), str(fq)], capture_output=True, text=True,
                           timeout=120, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(_body(out.read_text()))
    assert len(outs[0]) > 1000
    assert outs[0] == outs[1]


@pytest.mark.parametrize("shape", ["bgzf", "multi"])
def test_samse_gzip_reads(golden_dir, shape, tmp_path):
    """samse reading its FASTQ as BGZF / multi-member gzip (inflated on the host threads, gzsrc.h): the
    SAM equals the reference's on the uncompressed file."""
    from tests import gz_util as G
    key = next(k for k in sorted(MANIFEST) if MANIFEST[k]["reads"].endswith(".fq") and "-B" not in MANIFEST[k]["argv"])
    m = MANIFEST[key]
    data = open(os.path.join(golden_dir, m["reads"]), "rb").read()
    gz = tmp_path / "r.fq.gz"
    gz.write_bytes(G.bgzf(data, block=7000) if shape == "bgzf" else G.multi(data, 4, 1, 20_000))
    out = tmp_path / "out.sam"
    r = subprocess.run([CLI, "samse"] + m["argv"] + ["-f", str(out), os.path.join(golden_dir, m.get("prefix", "g1m")),
                                                     os.path.join(golden_dir, m["sai"]), str(gz)],
                       capture_output=True, text=True, timeout=120, env=dict(os.environ, IBWA_GZ_THREADS="4"))
    assert r.returncode == 0, r.stderr[-2000:]
    want = _body(gzip.open(os.path.join(golden_dir, m["sam"]), "rt").read())
    assert _body(out.read_text()) == want
