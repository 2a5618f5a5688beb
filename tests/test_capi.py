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
    compat = {"ibwa_gpu_init", "ibwa_gpu_destroy"}
    assert hdr - compat <= set(CAPI), sorted(hdr - compat - set(CAPI))


def test_cpu_only_calls():
    from ibwa_amd import engine
    o = engine.default_opt()
    assert (o.s_mm, o.s_gapo, o.s_gape, o.seed_len, o.max_top2) == (3, 11, 4, 32, 30)
    assert engine.lib().ibwa_cal_maxdiff(100, 0.02, 0.04) == 5
