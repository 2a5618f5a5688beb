"""On-device index builder vs the reference's `bwa index -a is` output.

The golden genome is regenerated from synth.cpp (seed 1), packed with the
lrand48 N-replacement of bntseq.c:181,224, indexed on the GPU, exported in
the reference .bwt layout and compared word for word with tests/golden/g1m.*.
"""
import os
import struct

import numpy as np
import pytest

from ibwa_amd import _native
from ibwa_amd import engine as E
from tests.synth_util import golden_genome_ascii


def _codes():
    g, _, _ = golden_genome_ascii()
    a = np.frombuffer(g.encode(), dtype=np.uint8)
    codes = np.empty(a.size, dtype=np.uint8)
    _native.lib().ibwa_pack_nt4_mt(a.ctypes.data, a.size, codes.ctypes.data, 4)
    return codes


def test_pack_matches_reference_pac(golden_dir):
    """.pac = 4 bases per byte, MSB first, + trailing count byte(s) (bntseq.c:238-246)."""
    codes = _codes()
    raw = open(os.path.join(golden_dir, "g1m.pac"), "rb").read()
    n = codes.size
    pac = np.frombuffer(raw[:(n + 3) // 4], dtype=np.uint8)
    unpacked = np.stack([(pac >> s) & 3 for s in (6, 4, 2, 0)], axis=1).reshape(-1)[:n]
    assert (unpacked == codes).all()


@pytest.mark.gpu
def test_device_index_is_bit_identical(golden_dir):
    codes = _codes()
    eng = E.Engine(0)
    eng.build_index(codes, sa_intv=32)
    for s, ext in enumerate(["bwt", "rbwt"]):
        primary, L2, words = E.read_bwt_file(os.path.join(golden_dir, "g1m." + ext))
        p, l2, w = eng.export_bwt(s)
        assert p == primary and tuple(l2) == tuple(L2), ext
        assert w.size == words.size and (w == words).all(), ext
        # sampled SA (bwt_dump_sa, bwtio.c:17-27)
        raw = open(os.path.join(golden_dir, "g1m." + ("sa" if s == 0 else "rsa")), "rb").read()
        hdr = struct.unpack("<7I", raw[:28])
        ref_sa = np.frombuffer(raw[28:], dtype=np.uint32)
        got = eng.export_sa(s, hdr[5])
        assert (got[1:] == ref_sa).all(), ext
    eng.close()


@pytest.mark.gpu
def test_device_index_aligns_like_file_index(golden_dir, sai_manifest):
    import oracle
    eng = E.Engine(0)
    eng.build_index(_codes())
    m = sai_manifest["r100.default"]
    opt, _ = oracle.parse_aln_args(m["argv"])
    recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
    seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
    e = E.GapOpt()
    for f, _ in E.GapOpt._fields_:
        setattr(e, f, getattr(opt, f))
    n_aln, alns = eng.aln(seqs, offs, lens, e)
    exp = open(os.path.join(golden_dir, "r100.default.sai"), "rb").read()
    assert oracle.sai_body_equal(oracle.sai_bytes(opt, n_aln, alns), exp)
    eng.close()
