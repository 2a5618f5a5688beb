"""`ibwa-amd index` / `fa2pac` / `pac_rev` (index_main.cpp) against the reference's `bwa index`
output, byte for byte: tests/golden/idx_quirks.* (tools/make_index_golden.py: IUPAC holes,
stale kseq comments, CRLF, empty record) and tests/golden/g1m.* (the golden genome, regenerated
from synth.cpp and written as FASTA).  fa2pac / pac_rev run on the CPU; `index` sorts on the GPU."""
import os
import subprocess

import pytest

from tests.synth_util import golden_genome_ascii

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "ibwa_amd", "bin", "ibwa-amd")
PACK_EXTS = ("pac", "ann", "amb", "rpac")
ALL_EXTS = PACK_EXTS + ("bwt", "rbwt", "sa", "rsa")


def _g1m_fasta(path):
    g, names, lens = golden_genome_ascii()
    with open(path, "w") as f:
        o = 0
        for nm, ln in zip(names, lens):
            f.write(f">{nm}\n")
            for i in range(o, o + ln, 70):
                f.write(g[i:min(i + 70, o + ln)] + "\n")
            o += ln


def _same(a, b):
    return open(a, "rb").read() == open(b, "rb").read()


@pytest.fixture(scope="module")
def fastas(tmp_path_factory, golden_dir):
    d = tmp_path_factory.mktemp("fa")
    _g1m_fasta(str(d / "g1m.fa"))
    return {"idx_quirks": os.path.join(golden_dir, "idx_quirks.fa"), "g1m": str(d / "g1m.fa")}


@pytest.mark.parametrize("name", ["idx_quirks", "g1m"])
def test_fa2pac_and_pac_rev(fastas, golden_dir, name, tmp_path):
    pre = str(tmp_path / "x")
    r = subprocess.run([CLI, "fa2pac", fastas[name], pre], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([CLI, "pac_rev", pre + ".pac", pre + ".rpac"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    for e in PACK_EXTS:
        assert _same(f"{pre}.{e}", os.path.join(golden_dir, f"{name}.{e}")), e


def test_index_rejects_color_space_and_unknown_algorithm(fastas, tmp_path):
    for argv in (["-c"], ["-a", "qsort"]):
        r = subprocess.run([CLI, "index"] + argv + ["-p", str(tmp_path / "x"), fastas["idx_quirks"]],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode != 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["idx_quirks", "g1m"])
def test_index_matches_reference(fastas, golden_dir, name, tmp_path):
    pre = str(tmp_path / "x")
    r = subprocess.run([CLI, "index", "-a", "bwtsw", "-p", pre, fastas[name]], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    for e in ALL_EXTS:
        assert _same(f"{pre}.{e}", os.path.join(golden_dir, f"{name}.{e}")), e
