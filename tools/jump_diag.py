#!/usr/bin/env python3
"""Diagnostics: exact path with / without the unique-interval jump on a device-built index."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from ibwa_amd import _native  # noqa: E402
from ibwa_amd import engine as E  # noqa: E402
from tests.test_scale_properties import reads  # noqa: E402

L = _native.lib()
lens = (ctypes.c_uint64 * 24)()
tot = L.ibwa_synth_grch37_lengths(1, 100, lens)
ascii_ = np.empty(tot, dtype=np.uint8)
L.ibwa_synth_genome(77, 24, lens, 0.45, 0.01, 120, ascii_.ctypes.data, 8)
codes = np.empty(tot, dtype=np.uint8)
L.ibwa_pack_nt4_mt(ascii_.ctypes.data, tot, codes.ctypes.data, 8)
eng = E.Engine(0)
eng.build_index(codes)
lens_ = [int(x) for x in lens]
for sub, tag in [(0.0, "exact reads"), (0.01, "1% sub")]:
    seq, off, lns, strand, raw = reads(ascii_, lens_, 5, 20000, 100, sub, 0.0)
    o, e = oracle.parse_aln_args(["-n", "0"])
    ge = E.GapOpt()
    for f, _ in E.GapOpt._fields_:
        setattr(ge, f, getattr(o, f))
    eng.set_option("exact_jump", 1)
    n1, a1 = eng.aln(seq, off, lns, ge)
    p1 = eng.stats().path
    eng.set_option("exact_jump", 0)
    n0, a0 = eng.aln(seq, off, lns, ge)
    p0 = eng.stats().path
    print(tag, "paths", p1, p0, "n_aln equal", (n1 == n0).all(), "alns equal", a1.tobytes() == a0.tobytes())
    first = np.concatenate([[0], np.cumsum(n0)[:-1]])
    shown = 0
    for r in range(len(n0)):
        if n0[r] != n1[r] or a0[first[r]:first[r] + n0[r]].tobytes() != a1[first[r]:first[r] + n1[r]].tobytes():
            print(" read", r, "nojump", a0[first[r]:first[r] + n0[r]].tolist(), "jump", a1[first[r]:first[r] + n1[r]].tolist())
            shown += 1
            if shown >= 8:
                break
