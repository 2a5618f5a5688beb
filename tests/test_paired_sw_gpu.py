"""bwa_paired_sw (bwasw.c:270-304) on the device: ibwa_paired_sw over mate pairs in
the reference's bwa_seq_t layout, against the reference's own outputs (tools/make_psw_golden.py):
every field it may change, the new CIGARs, and the stderr counters."""
import ctypes as c
import json
import os

import numpy as np
import pytest

import oracle
from ibwa_amd import engine as E

pytestmark = pytest.mark.gpu


def build_seqs(ends):
    """bwa_seq_t array as bwa_read_seq leaves it (bwaseqio.c:180-192) plus the pairing state"""
    arr = (E.RefSeq * len(ends))()
    keep = []
    for j, e in enumerate(ends):
        codes = oracle.nt4(e["read"])
        s = np.ascontiguousarray(codes[::-1])
        r = codes[::-1].copy()
        r[r < 4] = 3 - r[r < 4]
        # malloc'd like the reference's (the callee may free / replace cigar only)
        for name, v in (("seq", s), ("rseq", r)):
            buf = c.create_string_buffer(v.tobytes(), len(v))
            keep.append(buf)
            setattr(arr[j], name, c.cast(buf, c.c_void_p))
        x = arr[j]
        x.len = x.full_len = len(codes)
        for f in ("strand", "type", "mapQ", "seQ", "extra_flag", "n_mm", "n_gapo", "n_gape"):
            setattr(x, f, e[f])
        x.pos = x.remapped_pos = e["pos"]
    return arr, keep


def row(x):
    n = x.n_cigar
    cg = c.cast(x.cigar, c.POINTER(c.c_uint32)) if n else None
    cs = "".join(f"{cg[j] & 0x1FFFFFFF}{'MIDS'[cg[j] >> 29]}" for j in range(n)) or "*"
    return (x.type, x.strand, x.pos, x.remapped_pos, x.dbidx, x.remapped_dbidx, x.mapQ, x.seQ, x.n_mm, x.n_gapo,
            x.n_gape, x.extra_flag, n, cs)


@pytest.mark.parametrize("name", ["std100", "std150", "solid50"])
def test_paired_sw_matches_reference(golden_dir, gpu_engine, name):
    m = json.load(open(os.path.join(golden_dir, "psw_manifest.json")))[name]
    pin, pout = oracle.read_psw(golden_dir, name)
    s0, k0 = build_seqs([p[0] for p in pin])
    s1, k1 = build_seqs([p[1] for p in pin])
    popt = E.PeOpt(type=m["type"], is_sw=1, n_threads=1)
    ii = E.IsizeInfo(avg=m["avg"], std=m["std"], ap_prior=m["ap_prior"])
    pac = np.fromfile(os.path.join(golden_dir, "g1m.pac"), dtype=np.uint8)
    l_pac = int(open(os.path.join(golden_dir, "g1m.ann")).readline().split()[0])
    cnt = gpu_engine.paired_sw(s0, s1, popt, ii, pac, l_pac)
    assert cnt == [m["mated_singletons"], m["singletons"], m["fixed"], m["discordant"]]
    bad = []
    for i, q in enumerate(pout):
        for k, arr in ((0, s0), (1, s1)):
            exp = tuple(q[k][f] for f in oracle.PSW_OUT)
            if row(arr[i]) != exp:
                bad.append((i, k, row(arr[i]), exp))
    assert not bad, bad[:3]


def test_paired_sw_off(golden_dir, gpu_engine):
    """is_sw = 0 or an unknown insert size (avg < 0) leaves every read untouched (bwasw.c:279)."""
    pin, _ = oracle.read_psw(golden_dir, "std100")
    s0, k0 = build_seqs([p[0] for p in pin[:50]])
    s1, k1 = build_seqs([p[1] for p in pin[:50]])
    before = [row(x) for x in s0] + [row(x) for x in s1]
    pac = np.fromfile(os.path.join(golden_dir, "g1m.pac"), dtype=np.uint8)
    for popt, ii in ((E.PeOpt(type=1, is_sw=0), E.IsizeInfo(avg=300, std=30, ap_prior=1e-5)),
                     (E.PeOpt(type=1, is_sw=1), E.IsizeInfo(avg=-1, std=30, ap_prior=1e-5))):
        assert gpu_engine.paired_sw(s0, s1, popt, ii, pac, 1000000) == [0, 0, 0, 0]
    assert [row(x) for x in s0] + [row(x) for x in s1] == before
