"""SA row -> coordinate on the device: bwt_sa (bwt.c:69-79) inside
bwtdb_sa2seq (dbset.c:240-246), sampled-SA walk and full-SA gather.

* golden vectors from the compiled reference (tests/golden/sa2pos_vectors.tsv) on the
  reference-built g1m index loaded from its .bwt/.sa files: walk, expanded full SA;
* a 31 Mb index built on the device (full SA kept by the builder) against the CPU
  restatement over the exported BWT + sampled SA, at every row kind;
* error behaviour: rows past seq_len, a missing SA, an inconsistent .sa file.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from ibwa_amd import _native
from ibwa_amd import engine as E

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g1m_engine(golden_dir):
    eng = E.Engine(0)
    g = os.path.join(golden_dir, "g1m")
    eng.load_index_files(g)
    eng.load_sa_files(g)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def mid_genome_sa():
    """31 Mb synthetic genome indexed on the device with the sampled SA (interval 32) kept."""
    L = _native.lib()
    lens = (ctypes.c_uint64 * 24)()
    tot = L.ibwa_synth_grch37_lengths(1, 100, lens)
    ascii_ = np.empty(tot, dtype=np.uint8)
    L.ibwa_synth_genome(77, 24, lens, 0.45, 0.01, 120, ascii_.ctypes.data, 8)
    codes = np.empty(tot, dtype=np.uint8)
    L.ibwa_pack_nt4_mt(ascii_.ctypes.data, tot, codes.ctypes.data, 8)
    eng = E.Engine(0)
    eng.build_index(codes, sa_intv=32)
    bw = []
    for s in (0, 1):
        p, l2, w = eng.export_bwt(s)
        bw.append(oracle.Bwt(primary=p, L2=l2, words=w).set_sa(eng.export_sa(s, 32), 32))
    yield eng, bw[0], bw[1], ascii_, [int(x) for x in lens]
    eng.close()


def test_golden_vectors_walk_then_full(golden_dir, g1m_engine):
    s, k, ln, _, pos = oracle.read_sa2pos_vectors(os.path.join(golden_dir, "sa2pos_vectors.tsv"))
    eng = g1m_engine
    got = eng.sa2pos(s, k, ln)
    assert eng.stats().sa2pos_full == 0
    assert (got == pos).all(), np.nonzero(got != pos)[0][:10]
    eng.expand_sa()
    got = eng.sa2pos(s, k, ln)
    assert eng.stats().sa2pos_full == 1
    assert (got == pos).all(), np.nonzero(got != pos)[0][:10]
    eng.set_option("sa_walk", 1)
    assert (eng.sa2pos(s, k, ln) == pos).all() and eng.stats().sa2pos_full == 0
    eng.set_option("sa_walk", 0)
    # db offset (bwtdb_t.offset) is added after the u32 arithmetic
    assert (eng.sa2pos(s[:100], k[:100], ln[:100], offset=1 << 33) == pos[:100] + (1 << 33)).all()


def test_every_row_of_the_golden_index(golden_dir, g1m_engine):
    """All seq_len + 1 rows of both strands, full SA vs walk vs the restatement."""
    g = os.path.join(golden_dir, "g1m")
    b0 = oracle.Bwt(g + ".bwt").load_sa(g + ".sa")
    b1 = oracle.Bwt(g + ".rbwt").load_sa(g + ".rsa")
    n = b0.seq_len()
    k = np.concatenate([np.arange(n + 1, dtype=np.uint32)] * 2)
    s = np.concatenate([np.ones(n + 1, np.uint8), np.zeros(n + 1, np.uint8)])
    ln = np.full(k.size, 100, np.uint32)
    exp = oracle.sa2seq(b0, b1, s, k, ln)
    eng = g1m_engine
    eng.expand_sa()
    assert (eng.sa2pos(s, k, ln) == exp).all()
    eng.set_option("sa_walk", 1)
    assert (eng.sa2pos(s, k, ln) == exp).all()
    eng.set_option("sa_walk", 0)


def test_device_built_index_full_sa(mid_genome_sa):
    eng, b0, b1 = mid_genome_sa[:3]
    rng = np.random.default_rng(5)
    n = b0.seq_len()
    k = np.concatenate([rng.integers(0, n + 1, 200000, dtype=np.uint32),
                        np.array([0, 1, 31, 32, 33, b0.primary(), b1.primary(), n - 1, n], np.uint32)])
    s = (rng.integers(0, 2, k.size)).astype(np.uint8)
    ln = rng.choice(np.array([36, 100, 150], np.uint32), k.size)
    exp = oracle.sa2seq(b0, b1, s, k, ln)
    got = eng.sa2pos(s, k, ln)
    assert eng.stats().sa2pos_full == 1
    assert (got == exp).all()
    eng.set_option("sa_walk", 1)
    assert (eng.sa2pos(s, k, ln) == exp).all()
    eng.set_option("sa_walk", 0)


def drawn_reads(ascii_, lens, seed, n, ln):
    """error-free synthetic reads with the 0-based position and strand (0 fwd) they come from"""
    L = _native.lib()
    c_lens = (ctypes.c_uint64 * 24)(*lens)
    raw = np.empty(n * ln, dtype=np.uint8)
    pos = np.empty(n, dtype=np.uint64)
    st = np.empty(n, dtype=np.uint8)
    L.ibwa_synth_reads(seed, ascii_.ctypes.data, ascii_.size, 24, c_lens, n, ln, 0.0, 0.0, raw.ctypes.data,
                       pos.ctypes.data, st.ctypes.data, 8)
    seq = np.empty(n * ln, dtype=np.uint8)
    off = np.empty(n, dtype=np.uint64)
    lns = np.empty(n, dtype=np.uint32)
    L.ibwa_encode_reads_fixed(raw.ctypes.data, n, ln, seq.ctypes.data, off.ctypes.data, lns.ctypes.data, 8)
    return seq, off, lns, pos, st


def test_hits_map_back_to_their_reads(mid_genome_sa):
    """Round trip: each error-free read's -n 0 hit, through sa2pos, lands on the position and
    strand it was drawn from (a = 1: reverse strand, bwase.c bwa_aln2seq / dbset.c:240-246)."""
    eng, _, _, ascii_, lens = mid_genome_sa
    seq, off, lns, pos0, st0 = drawn_reads(ascii_, lens, 11, 20000, 100)
    o, _ = oracle.parse_aln_args(["-n", "0"])
    e = E.GapOpt()
    for f, _ in E.GapOpt._fields_:
        setattr(e, f, getattr(o, f))
    n_aln, alns = eng.aln(seq, off, lns, e)
    assert (n_aln >= 1).all()
    # every row of every hit interval of the read's drawn strand; the drawn position is among them
    a = ((alns["info"] >> 24) & 1).astype(np.uint8)
    rid = np.repeat(np.arange(lns.size), n_aln)
    sizes = (alns["l"] - alns["k"] + 1).astype(np.int64)
    assert sizes.max() < 5000
    hit = np.repeat(np.arange(alns.size), sizes)
    rows = (alns["k"][hit] + (np.arange(hit.size) - np.repeat(np.cumsum(sizes) - sizes, sizes))).astype(np.uint32)
    p = eng.sa2pos(a[hit], rows, lns[rid[hit]])
    found = np.zeros(lns.size, bool)
    m = (p == pos0[rid[hit]]) & (a[hit] == st0[rid[hit]])
    found[rid[hit][m]] = True
    assert found.all(), np.nonzero(~found)[0][:10]


def test_errors(golden_dir):
    eng = E.Engine(0)
    g = os.path.join(golden_dir, "g1m")
    eng.load_index_files(g)
    with pytest.raises(E.IbwaError):  # no SA loaded
        eng.sa2pos(np.ones(1, np.uint8), np.ones(1, np.uint32), np.ones(1, np.uint32))
    with pytest.raises(E.IbwaError):  # .rsa does not belong to .bwt (bwtio.c:37)
        E._chk(E.lib().ibwa_ctx_load_sa_file(eng.h, 0, (g + ".rsa").encode()))
    eng.load_sa_files(g)
    n = eng.bwt_info(0)[1][3]
    with pytest.raises(E.IbwaError):  # row past seq_len
        eng.sa2pos(np.ones(1, np.uint8), np.array([n + 1], np.uint32), np.ones(1, np.uint32))
    assert eng.sa2pos(np.zeros(0, np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint32)).size == 0
    eng.close()
