"""Parity at sizes the golden fixtures do not reach (31 Mb genome built on device).

* round trip: reads copied exactly from the genome must all be found by
  `aln -n 0`, on the strand they were drawn from (strand 0 = forward);
* GPU == CPU restatement on seeded reads for default gapped options, -n 0,
  and a 150 bp / 2 % error set, including the overflow-retry path.
"""
import ctypes

import numpy as np
import pytest

import oracle
from ibwa_amd import _native
from ibwa_amd import engine as E

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mid_genome():
    L = _native.lib()
    lens = (ctypes.c_uint64 * 24)()
    tot = L.ibwa_synth_grch37_lengths(1, 100, lens)
    ascii_ = np.empty(tot, dtype=np.uint8)
    L.ibwa_synth_genome(77, 24, lens, 0.45, 0.01, 120, ascii_.ctypes.data, 8)
    codes = np.empty(tot, dtype=np.uint8)
    L.ibwa_pack_nt4_mt(ascii_.ctypes.data, tot, codes.ctypes.data, 8)
    eng = E.Engine(0)
    eng.build_index(codes)
    p0, l0, w0 = eng.export_bwt(0)
    p1, l1, w1 = eng.export_bwt(1)
    b0 = oracle.Bwt(primary=p0, L2=l0, words=w0)
    b1 = oracle.Bwt(primary=p1, L2=l1, words=w1)
    yield ascii_, [int(x) for x in lens], eng, b0, b1
    eng.close()


def reads(ascii_, lens, seed, n, ln, sub, indel):
    L = _native.lib()
    c_lens = (ctypes.c_uint64 * 24)(*lens)
    raw = np.empty(n * ln, dtype=np.uint8)
    pos = np.empty(n, dtype=np.uint64)
    strand = np.empty(n, dtype=np.uint8)
    L.ibwa_synth_reads(seed, ascii_.ctypes.data, ascii_.size, 24, c_lens, n, ln, sub, indel, raw.ctypes.data,
                       pos.ctypes.data, strand.ctypes.data, 8)
    seq = np.empty(n * ln, dtype=np.uint8)
    off = np.empty(n, dtype=np.uint64)
    lns = np.empty(n, dtype=np.uint32)
    L.ibwa_encode_reads_fixed(raw.ctypes.data, n, ln, seq.ctypes.data, off.ctypes.data, lns.ctypes.data, 8)
    return seq, off, lns, strand, raw


def eopt(argv):
    o, _ = oracle.parse_aln_args(argv)
    e = E.GapOpt()
    for f, _ in E.GapOpt._fields_:
        setattr(e, f, getattr(o, f))
    return o, e


def test_device_built_index_uses_the_jump(mid_genome):
    ascii_, lens, eng, _, _ = mid_genome
    seq, off, lns, _, _ = reads(ascii_, lens, 3, 1000, 100, 0.0, 0.0)
    _, e = eopt(["-n", "0"])
    eng.aln(seq, off, lns, e)
    assert eng.stats().path == 3


def test_exact_reads_round_trip(mid_genome):
    ascii_, lens, eng, _, _ = mid_genome
    seq, off, lns, strand, raw = reads(ascii_, lens, 11, 200_000, 100, 0.0, 0.0)
    has_n = (seq.reshape(-1, 100) > 3).any(axis=1)
    _, e = eopt(["-n", "0"])
    n_aln, alns = eng.aln(seq, off, lns, e)
    assert (n_aln[~has_n] >= 1).all()
    first = np.concatenate([[0], np.cumsum(n_aln)[:-1]])
    a = (alns["info"] >> 24) & 1
    # the drawing strand is always among the hits: strand 0 = forward = a 0
    ok = np.zeros(len(n_aln), bool)
    for j in range(2):
        sel = n_aln > j
        ok[sel] |= a[first[sel] + j] == strand[sel]
    assert ok[~has_n].all()


@pytest.mark.parametrize("argv,ln,sub,n,tune", [
    ([], 100, 0.01, 30_000, {}), (["-n", "0"], 100, 0.01, 100_000, {}),
    ([], 150, 0.02, 8_000, {}), (["-n", "3", "-o", "2", "-e", "3"], 100, 0.02, 8_000, {}),
    ([], 150, 0.02, 8_000, {"gap_lw_min_waves": 12}),  # 150 bp through the first pass without LDS widths
    # small static regions: many reads take pages from their workgroup pool, some exhaust it
    ([], 100, 0.02, 20_000, {"gap_cap1": 256, "gap_pages_per_block": 2}),
    (["-n", "0"], 100, 0.01, 20_000, {"exact_path": 0}),
    (["-n", "0"], 100, 0.01, 100_000, {"exact_jump": 0}),
    (["-n", "0"], 150, 0.0, 50_000, {}), (["-n", "0"], 36, 0.0, 50_000, {}),
    ([], 100, 0.01, 4_000, {"gapped_v2": 0}),
    # every read past one first-pass iteration goes to the wave-cooperative kernel (coop.hip) ...
    ([], 100, 0.01, 30_000, {"gap_iter_budget": 1}), ([], 150, 0.02, 8_000, {"gap_iter_budget": 1}),
    (["-n", "3", "-o", "2", "-e", "3"], 100, 0.02, 8_000, {"gap_iter_budget": 1}),
    # ... including reads cut off by max_entries (bwtgap.c:138), which it resolves itself ...
    (["-m", "300"], 100, 0.02, 8_000, {"gap_iter_budget": 1}),
    (["-m", "2000"], 150, 0.02, 4_000, {"gap_iter_budget": 1}),
    # ... with level 0 run by k_coop_roots (the default) or by k_coop itself, under other options
    ([], 100, 0.01, 30_000, {"gap_iter_budget": 1, "coop_roots": 0}),
    (["-m", "300"], 100, 0.02, 8_000, {"gap_iter_budget": 1, "coop_roots": 0}),
    (["-N", "-n", "2"], 100, 0.01, 4_000, {"gap_iter_budget": 1}), (["-L"], 100, 0.02, 8_000, {"gap_iter_budget": 1}),
    (["-c"], 100, 0.02, 8_000, {"gap_iter_budget": 1}), (["-l", "20", "-k", "1"], 100, 0.02, 8_000, {"gap_iter_budget": 1}),
    (["-n", "1"], 100, 0.01, 8_000, {"gap_iter_budget": 1}), (["-i", "0", "-d", "0"], 70, 0.02, 8_000, {"gap_iter_budget": 1}),
    # ... or, with it off, to the sequential wide kernel
    ([], 100, 0.01, 8_000, {"gap_iter_budget": 1, "gap_coop": 0}),
    # early hand-offs that leave their search state at the next score-level boundary: the cooperative
    # pass resumes them (gap_resume), under the options above, with paged first-pass stacks and with a
    # state buffer too small for some of them (those start over); the LDS-width first pass, which
    # leaves the states, takes reads up to ~100 bp (its LDS records) with max_diff <= 6
    ([], 100, 0.01, 30_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    ([], 90, 0.02, 8_000, {"gap_resume_iters": 60, "gap_resume_entries": 16}),
    (["-n", "3", "-o", "2", "-e", "3"], 100, 0.02, 8_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    (["-m", "300"], 100, 0.02, 8_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    (["-m", "2000"], 100, 0.03, 4_000, {"gap_resume_iters": 40, "gap_resume_entries": 8}),
    (["-N", "-n", "2"], 100, 0.01, 4_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    (["-L"], 100, 0.02, 8_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    (["-c"], 100, 0.02, 8_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    (["-l", "20", "-k", "1"], 100, 0.02, 8_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    (["-n", "1"], 100, 0.01, 8_000, {"gap_resume_iters": 5, "gap_resume_entries": 2}),
    (["-i", "0", "-d", "0"], 70, 0.02, 8_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    ([], 100, 0.01, 30_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "coop_roots": 0}),
    ([], 100, 0.02, 20_000, {"gap_resume_iters": 100, "gap_resume_entries": 50, "gap_cap1": 256,
                             "gap_pages_per_block": 8}),
    ([], 100, 0.01, 30_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "gap_resume_records": 20_000}),
    # 150 bp (and 120 bp) reads: the LDS-width first pass in 64-lane workgroups, with resume states
    ([], 150, 0.02, 8_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    ([], 120, 0.02, 8_000, {"gap_resume_iters": 40, "gap_resume_entries": 8}),
    (["-n", "3", "-o", "2", "-e", "3"], 150, 0.02, 4_000, {"gap_resume_iters": 20, "gap_resume_entries": 4}),
    # every read past 5 iterations in the launch's tail (here: from the start) leaves its state
    ([], 100, 0.01, 30_000, {"gap_tail_lanes": 64, "gap_tail_iters": 5}),
    (["-n", "3", "-o", "2", "-e", "3"], 100, 0.02, 8_000, {"gap_tail_lanes": 64, "gap_tail_iters": 1}),
    # a 1 GiB page pool: resumed reads that run out of pages start over in the later passes
    ([], 100, 0.01, 30_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "coop_pool_gb": 1}),
    # pools of a few pages: the reads out of pages run again in launches of their own, then go on to
    # the wide kernel
    ([], 100, 0.02, 4_000, {"gap_iter_budget": 1, "coop_pool_pages": 48}),
    ([], 100, 0.01, 30_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "coop_pool_pages": 256}),
    ([], 100, 0.01, 8_000, {"gap_early_iters": 20, "gap_early_entries": 4, "gap_resume": 0}),
    # several first-pass chunks, each followed by the cooperative pass over its resumed reads (the
    # state buffer and its fill counter reused chunk after chunk), under several options and a state
    # buffer too small for some states
    ([], 100, 0.01, 30_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "gap_reads_per_chunk": 10_000}),
    ([], 150, 0.02, 12_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "gap_reads_per_chunk": 4_000}),
    (["-n", "3", "-o", "2", "-e", "3"], 100, 0.02, 12_000, {"gap_resume_iters": 20, "gap_resume_entries": 4,
                                                           "gap_reads_per_chunk": 3_000}),
    (["-m", "300"], 100, 0.02, 12_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "gap_reads_per_chunk": 4_000}),
    ([], 100, 0.01, 30_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "gap_reads_per_chunk": 7_500,
                             "gap_resume_records": 8_000}),
    ([], 100, 0.01, 30_000, {"gap_resume_iters": 20, "gap_resume_entries": 4, "gap_reads_per_chunk": 7_500,
                             "coop_pool_gb": 1}),
    # the first pass with its shallow nodes stored by their strings (level tables, gap_tab_k): alone,
    # with resume states that carry such entries to the cooperative pass (converted to intervals), with
    # gaps, seeds, long deletions, 150 bp, and every read leaving its state in the launch's tail
    ([], 100, 0.01, 30_000, {"gap_tab_k": 12}),
    ([], 100, 0.02, 20_000, {"gap_tab_k": 12, "gap_resume_iters": 20, "gap_resume_entries": 4}),
    (["-n", "3", "-o", "2", "-e", "3"], 100, 0.02, 8_000, {"gap_tab_k": 10, "gap_resume_iters": 20,
                                                          "gap_resume_entries": 4}),
    (["-l", "20", "-k", "1"], 100, 0.02, 8_000, {"gap_tab_k": 8, "gap_resume_iters": 20, "gap_resume_entries": 4}),
    (["-L", "-d", "30"], 100, 0.02, 8_000, {"gap_tab_k": 11, "gap_resume_iters": 20, "gap_resume_entries": 4}),
    ([], 150, 0.02, 8_000, {"gap_tab_k": 13, "gap_resume_iters": 20, "gap_resume_entries": 4}),
    ([], 100, 0.02, 8_000, {"gap_tab_k": 14, "gap_resume_iters": 20, "gap_resume_entries": 4}),
    ([], 100, 0.01, 30_000, {"gap_tab_k": 12, "gap_tail_lanes": 64, "gap_tail_iters": 5})])
def test_gpu_equals_oracle(mid_genome, argv, ln, sub, n, tune):
    ascii_, lens, eng, b0, b1 = mid_genome
    seq, off, lns, _, _ = reads(ascii_, lens, 5 + n, n, ln, sub, 0.05)
    o, e = eopt(argv)
    defaults = {"gap_cap1": 8192, "gap_pages_per_block": 384, "exact_path": 1, "gapped_v2": 1, "exact_jump": 1,
                "gap_iter_budget": 8000, "gap_coop": 1, "coop_roots": 1, "gap_early_iters": 3000,
                "gap_early_entries": 1000, "gap_resume": 1, "gap_resume_records": 0, "gap_resume_iters": 2000,
                "gap_resume_entries": 300, "coop_pool_gb": 0, "gap_tail_lanes": 16, "gap_tail_iters": 200,
                "gap_lw_min_waves": 8, "coop_pool_pages": 0, "gap_reads_per_chunk": 16 << 20, "gap_tab_k": -1}
    try:
        for k, v in tune.items():
            eng.set_option(k, v)
        n_aln, alns = eng.aln(seq, off, lns, e)
        st = eng.stats()
        hpop = eng.handoff_pops()
        ids, ps = eng.retry_info()
    finally:
        for k in tune:
            eng.set_option(k, defaults[k])
    if "-m" in argv:
        assert st.n_heavy > 0 and st.n_coop == st.n_heavy  # nothing handed on to the sequential kernel
    if ("gap_resume_iters" in tune or "gap_tail_lanes" in tune) and tune.get("gap_resume", 1):
        assert st.n_resumed > 0  # the resume path ran
        if "gap_resume_records" in tune:
            assert st.resume_records > tune["gap_resume_records"]  # ... and some states did not fit
    ost = np.zeros(len(lns), dtype=oracle.STATS_DTYPE)
    rn, ra, _ = oracle.cal_sa_reg_gap(b0, b1, seq, off, lns, o, n_threads=8, stats=ost)
    assert (n_aln == rn).all()
    assert alns.tobytes() == ra.tobytes()
    # the pops a resumed read made before its hand-off (the bench's touch split): every read the
    # cooperative pass resumed has them, and the reference's search went on past them
    res = ids[ps == 4]
    assert (hpop[res] > 0).all()
    assert (hpop[res] < ost["pops"][res]).all()
    if st.n_resumed == 0:
        assert not hpop.any()
