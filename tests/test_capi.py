"""The C ABI library loads (no GPU needed) and exports every declared symbol."""
import ctypes
import os
import re

from ibwa_amd import _native
from ibwa_amd.engine import CAPI

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h"):
            src = open(os.path.join(ROOT, "include", fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            for m in re.finditer(r"\b([a-z_][a-z0-9_]*)\s*\(", src):
                nm = m.group(1)
                if nm.startswith(("ibwa_", "bwa_")) and not nm.endswith("_t"):
                    names.add(nm)
    return names


def test_library_exports_all_declared():
    L = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in sorted(declared_symbols()) if not hasattr(L, n)]
    assert not missing, missing


def test_binding_covers_header():
    hdr = {n for n in declared_symbols() if n.startswith("ibwa_")}
    compat = {"ibwa_gpu_init", "ibwa_gpu_init_ex", "ibwa_gpu_destroy"}
    assert hdr - compat <= set(CAPI), sorted(hdr - compat - set(CAPI))


def test_build_id_matches_sources():
    """The library reports the digest of the sources it was built from, and it is this tree's."""
    L = _native.lib()
    assert L.ibwa_build_id().decode() == _native.source_digest()


def test_cpu_only_calls():
    from ibwa_amd import engine
    o = engine.default_opt()
    assert (o.s_mm, o.s_gapo, o.s_gape, o.seed_len, o.max_top2) == (3, 11, 4, 32, 30)
    assert engine.lib().ibwa_cal_maxdiff(100, 0.02, 0.04) == 5


def test_product_option_parser_matches_reference_semantics():
    """ibwa_aln_parse_args (the product's getopt, used by the CLI and bench.py) against the
    oracle's restatement of bwa_aln's option handling, over every golden option set."""
    import json

    import oracle
    from ibwa_amd import engine
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "sai_manifest.json")))
    sets = [m["argv"] for m in man.values()] + [["-n", "0.01", "-e", "0"], ["-e", "5", "-N", "-R", "7"],
                                                ["-B", "4", "-q", "20", "-I", "-c", "-L", "-m", "1000"]]
    for argv in sets:
        got = engine.parse_aln_args(argv)
        exp, _ = oracle.parse_aln_args(argv)
        for f, _ in engine.GapOpt._fields_:
            assert getattr(got, f) == getattr(exp, f), (argv, f)
    # repeated calls start from the defaults again (getopt state is re-initialised)
    assert engine.parse_aln_args([]).max_diff == -1
    import pytest
    with pytest.raises(engine.IbwaError):
        engine.parse_aln_args(["-Z"])
