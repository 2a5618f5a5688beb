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
