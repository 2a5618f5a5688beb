"""GPU parity: the HIP engine (through the C ABI) against the reference's goldens.

Bit-exact for every .sai of the option matrix (tools/make_golden.py) and for
bwt_occ4 KATs; plus engine-vs-oracle on larger seeded read sets.
"""
import os

import numpy as np
import pytest

import oracle
from ibwa_amd import engine as E

pytestmark = pytest.mark.gpu


def _eopt(o):
    e = E.GapOpt()
    for f, _ in E.GapOpt._fields_:
        setattr(e, f, getattr(o, f))
    return e


def test_occ4_kats_gpu(golden_dir, gpu_engine):
    for s, which in enumerate(["bwt", "rbwt"]):
        rows = [list(map(int, l.split())) for l in open(os.path.join(golden_dir, f"kat_occ4_{which}.tsv"))]
        ks = np.array([r[0] for r in rows], dtype=np.uint32)
        got = gpu_engine.occ4(s, ks)
        assert (got == np.array([r[1:] for r in rows], dtype=np.uint32)).all(), which


@pytest.mark.parametrize("exact_path,gapped_v2", [(1, 1), (0, 1), (1, 0), (0, 0)])
def test_sai_goldens_gpu(golden_dir, sai_manifest, gpu_engine, exact_path, gapped_v2):
    """exact_path=0 forces -n 0 through the gapped search too; gapped_v2=0 selects the
    general (retry-pass) kernels for every gapped option set."""
    gpu_engine.set_option("exact_path", exact_path)
    gpu_engine.set_option("gapped_v2", gapped_v2)
    bad = []
    for key, m in sorted(sai_manifest.items()):
        opt, _ = oracle.parse_aln_args(m["argv"])
        recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
        seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
        n_aln, alns = gpu_engine.aln(seqs, offs, lens, _eopt(opt))
        got = oracle.sai_bytes(opt, n_aln, alns)
        exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
        if not oracle.sai_body_equal(got, exp):
            bad.append(key)
        if m["argv"] == ["-n", "0"]:
            # a file-loaded index gets the jump arrays derived from its BWT (path 3)
            assert gpu_engine.stats().path == (3 if exact_path else 2 if gapped_v2 else 0), key
        elif gapped_v2 and gpu_engine.stats().path != 2:
            bad.append(key + ":path")
    gpu_engine.set_option("exact_path", 1)
    gpu_engine.set_option("gapped_v2", 1)
    assert not bad, bad


@pytest.mark.parametrize("tab_k", [12, 6, 0])
def test_sai_goldens_level_tables(golden_dir, sai_manifest, gpu_engine, tab_k):
    """The first pass with its shallow nodes stored by their strings and expanded from the level
    tables (GapArgs::ltab, gap_tab_k; 0: off, every node by its interval): every golden .sai of the
    option matrix, bit for bit."""
    gpu_engine.set_option("gap_tab_k", tab_k)
    bad = []
    try:
        for key, m in sorted(sai_manifest.items()):
            opt, _ = oracle.parse_aln_args(m["argv"])
            recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
            seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
            n_aln, alns = gpu_engine.aln(seqs, offs, lens, _eopt(opt))
            got = oracle.sai_bytes(opt, n_aln, alns)
            if not oracle.sai_body_equal(got, open(os.path.join(golden_dir, key + ".sai"), "rb").read()):
                bad.append(key)
    finally:
        gpu_engine.set_option("gap_tab_k", -1)
    assert not bad, bad


def test_fetch_sai_equals_fetch(golden_dir, sai_manifest, gpu_engine):
    """ibwa_batch_fetch_sai (the CLI's writer input: records serialised by host threads into the
    caller's buffer) == the .sai body built from ibwa_batch_fetch, == the reference's golden; a buffer
    too small is left untouched and reports the size."""
    import ctypes as c
    for key in ("r100.default", "mixed.N", "r150.m50"):
        m = sai_manifest[key]
        opt, _ = oracle.parse_aln_args(m["argv"])
        recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
        seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
        gpu_engine.stage(seqs, offs, lens)
        gpu_engine.run(_eopt(opt))
        body = gpu_engine.fetch_sai()
        n_aln, alns = gpu_engine.fetch()
        assert body == oracle.sai_bytes(opt, n_aln, alns)[64:], key
        exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
        assert body == exp[64:], key
        small = c.create_string_buffer(b"\x5a" * 16, 16)
        need = c.c_uint64()
        assert E.lib().ibwa_batch_fetch_sai(gpu_engine.h, small, 16, c.byref(need), None) == 0
        assert need.value == len(body) and small.raw == b"\x5a" * 16


@pytest.mark.parametrize("width_jump,width_tab", [(0, 1), (2, 1), (1, 0), (0, 0)])
def test_sai_goldens_width_jump(golden_dir, sai_manifest, gpu_engine, width_jump, width_tab):
    """k_width with (2: SA / text derived from the loaded BWT) and without (0) one-row steps from
    the text, with and without its leading steps from the level tables (width_tab): every gapped
    golden, in the first pass and (budget 1) through the heavy-read pass."""
    bad = []
    try:
        gpu_engine.set_option("width_jump", width_jump)
        gpu_engine.set_option("width_tab", width_tab)
        for budget in (8000, 1):
            gpu_engine.set_option("gap_iter_budget", budget)
            for key, m in sorted(sai_manifest.items()):
                if m["argv"] == ["-n", "0"]:
                    continue
                opt, _ = oracle.parse_aln_args(m["argv"])
                recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
                seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
                n_aln, alns = gpu_engine.aln(seqs, offs, lens, _eopt(opt))
                exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
                if not oracle.sai_body_equal(oracle.sai_bytes(opt, n_aln, alns), exp):
                    bad.append(f"{key}:budget {budget}")
    finally:
        gpu_engine.set_option("width_jump", 1)
        gpu_engine.set_option("width_tab", 1)
        gpu_engine.set_option("gap_iter_budget", 8000)
    assert not bad, bad


def _edge_records(golden_dir, seed=7):
    """Reads from the first and last bases of the golden reference (and its middle), forward and
    reverse-complemented, exact and with one or two substitutions, 100 / 36 / 20 / 12 bp."""
    codes, l_pac = oracle.read_pac(os.path.join(golden_dir, "g1m"))
    rng = np.random.default_rng(seed)
    recs = []
    for L in (100, 36, 20, 12):
        for start in (0, 1, 5, 17, l_pac // 2, l_pac - L - 3, l_pac - L):
            ref = codes[start:start + L].astype(np.int64)
            for nm in (0, 1, 2):
                t = ref.copy()
                for p in rng.choice(L, size=nm, replace=False):
                    t[p] = (t[p] + 1 + rng.integers(3)) % 4
                for rc in (False, True):
                    u = 3 - t[::-1] if rc else t
                    recs.append((f"e{len(recs)}", "".join("ACGT"[c] for c in u).encode(), b"I" * L))
            # an N where k_width's table prefix reads (the read's last bases: bwa_seq_t.seq is reversed)
            for q in (L - 1, L - 4, L - 15, L - 17):
                if 0 <= q < L:
                    u = bytearray("".join("ACGT"[c] for c in ref).encode())
                    u[q] = ord("N")
                    recs.append((f"e{len(recs)}", bytes(u), b"I" * L))
    return recs


@pytest.mark.parametrize("width_jump,budget", [(1, 8000), (2, 8000), (2, 1), (0, 1)])
def test_reference_edge_reads(golden_dir, gpu_engine, width_jump, budget):
    """Reads at the reference's ends: k_width's level-table prefix and its text windows as the
    suffix position nears 0 (width_jump 2 derives the SA / text of the loaded index), the level
    tables' short-read rule (12 / 20 bp reads keep intervals), in the first pass and (budget 1)
    through the heavy-read pass -- hits equal to the oracle's."""
    recs = _edge_records(golden_dir)
    opt, _ = oracle.parse_aln_args([])
    seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
    try:
        gpu_engine.set_option("width_jump", width_jump)
        gpu_engine.set_option("gap_iter_budget", budget)
        n_aln, alns = gpu_engine.aln(seqs, offs, lens, _eopt(opt))
    finally:
        gpu_engine.set_option("width_jump", 1)
        gpu_engine.set_option("gap_iter_budget", 8000)
    b0 = oracle.Bwt(os.path.join(golden_dir, "g1m.bwt"))
    b1 = oracle.Bwt(os.path.join(golden_dir, "g1m.rbwt"))
    rn, ra, _ = oracle.cal_sa_reg_gap(b0, b1, seqs, offs, lens, opt)
    assert (n_aln == rn).all() and alns.tobytes() == ra.tobytes()
    assert int(rn.sum()) > len(recs) // 2  # most of them align


@pytest.mark.parametrize("coop", [1, 0])
def test_sai_goldens_heavy_pass(golden_dir, sai_manifest, gpu_engine, coop):
    """An iteration budget of 1 hands every gapped read to the heavy-read pass: the
    wave-cooperative kernel (coop.hip), or with coop=0 the sequential wide kernel."""
    bad = []
    try:
        gpu_engine.set_option("gap_iter_budget", 1)
        gpu_engine.set_option("gap_coop", coop)
        for key, m in sorted(sai_manifest.items()):
            if m["argv"] == ["-n", "0"]:
                continue
            opt, _ = oracle.parse_aln_args(m["argv"])
            recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
            seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
            n_aln, alns = gpu_engine.aln(seqs, offs, lens, _eopt(opt))
            exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
            if not oracle.sai_body_equal(oracle.sai_bytes(opt, n_aln, alns), exp):
                bad.append(key)
            st = gpu_engine.stats()
            if st.path == 2 and (st.n_heavy == 0 or (coop and st.n_coop == 0)):
                bad.append(key + f":heavy {st.n_heavy} coop {st.n_coop}")
            # max_entries cut-offs (-m) are resolved inside the cooperative kernel
            if coop and "-m" in m["argv"] and max(lens) <= 256 and st.n_coop != st.n_heavy:
                bad.append(key + f":coop resolved {st.n_coop} of {st.n_heavy}")
    finally:
        gpu_engine.set_option("gap_iter_budget", 8000)
        gpu_engine.set_option("gap_coop", 1)
    assert not bad, bad


@pytest.mark.parametrize("stack_cap,aln_cap,v2", [(16, 1, 0), (64, 2, 0), (16, 1, 1), (64, 2, 1)])
def test_overflow_retry_is_exact(golden_dir, sai_manifest, gpu_engine, stack_cap, aln_cap, v2):
    """Tiny per-lane capacities force most reads through the large-capacity retry pass
    (v2: tiny primary regions, an extension pool of 4 regions, tiny hit arrays)."""
    try:
        gpu_engine.set_tuning(stack_cap=stack_cap, aln_cap=aln_cap)
        gpu_engine.set_option("gapped_v2", v2)
        gpu_engine.set_option("gap_cap1", stack_cap)
        gpu_engine.set_option("gap_pages_per_block", 1)
        gpu_engine.set_option("gap_hit_slots", aln_cap)
        for key in ["r150.default", "mixed.N", "r100.default"]:
            m = sai_manifest[key]
            opt, _ = oracle.parse_aln_args(m["argv"])
            recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
            seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
            n_aln, alns = gpu_engine.aln(seqs, offs, lens, _eopt(opt))
            assert gpu_engine.stats().n_retry > 0
            exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
            assert oracle.sai_body_equal(oracle.sai_bytes(opt, n_aln, alns), exp), key
    finally:
        gpu_engine.set_tuning(stack_cap=4096, aln_cap=8)
        for k, v in [("gapped_v2", 1), ("gap_cap1", 8192), ("gap_pages_per_block", 384), ("gap_hit_slots", 256)]:
            gpu_engine.set_option(k, v)


@pytest.mark.parametrize("stream_min", [1, 64, 700])
def test_hit_stream_overflow_is_exact(golden_dir, sai_manifest, gpu_engine, stream_min):
    """A first-pass hit stream smaller than the batch's hits: reads past its end are flagged and
    re-run, and the fetch copies only the records the stream holds (the fill counter
    runs past the stream's end on overflow)."""
    try:
        gpu_engine.set_option("gap_stream_per_read", 0)
        gpu_engine.set_option("gap_stream_min", stream_min)
        for key in ["r100.default", "mixed.N", "r100.N"]:
            if key not in sai_manifest:
                continue
            m = sai_manifest[key]
            opt, _ = oracle.parse_aln_args(m["argv"])
            recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
            seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
            n_aln, alns = gpu_engine.aln(seqs, offs, lens, _eopt(opt))
            st = gpu_engine.stats()
            assert st.path == 2, (key, st.path)
            if int(n_aln.sum()) > stream_min:  # more hits than the stream holds: some reads overflowed
                assert st.n_aln_overflow > 0, (key, st.n_aln_overflow)
            exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
            assert oracle.sai_body_equal(oracle.sai_bytes(opt, n_aln, alns), exp), key
    finally:
        gpu_engine.set_option("gap_stream_per_read", 4)
        gpu_engine.set_option("gap_stream_min", 1 << 20)


def test_exact_path_without_jump(golden_dir, sai_manifest, gpu_engine):
    """-n 0 goldens with the jump arrays not derived (path 1), then derived again (path 3)."""
    for derive, path in [(0, 1), (1, 3)]:
        eng = E.Engine(0)
        try:
            eng.load_index_files(os.path.join(golden_dir, "g1m"))
            eng.set_option("jump_derive", derive)
            for key, m in sorted(sai_manifest.items()):
                if m["argv"] != ["-n", "0"]:
                    continue
                opt, _ = oracle.parse_aln_args(m["argv"])
                recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
                seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
                n_aln, alns = eng.aln(seqs, offs, lens, _eopt(opt))
                assert eng.stats().path == path, (key, derive)
                exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
                assert oracle.sai_body_equal(oracle.sai_bytes(opt, n_aln, alns), exp), (key, derive)
        finally:
            eng.close()


@pytest.mark.parametrize("prefix", ["g1m", "tandem", "idx_quirks"])
def test_sampled_sa_derived_from_bwt(golden_dir, prefix):
    """The sampled SA derived on the device from .bwt / .rbwt alone (LF walks between marked rows
    + list ranking) equals the reference-built .sa / .rsa byte for byte."""
    eng = E.Engine(0)
    try:
        eng.load_index_files(os.path.join(golden_dir, prefix))
        eng.derive_sa(32)
        for s, ext in [(0, ".sa"), (1, ".rsa")]:
            raw = np.fromfile(os.path.join(golden_dir, prefix + ext), dtype=np.uint32)
            intv = int(raw[5])
            assert intv == 32
            got = eng.export_sa(s, 32)
            assert got[0] == 0xFFFFFFFF and (got[1:] == raw[7:]).all(), (prefix, ext)
    finally:
        eng.close()


def test_empty_batch(gpu_engine):
    n_aln, alns = gpu_engine.aln(np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                                 E.default_opt())
    assert n_aln.size == 0 and alns.size == 0


def test_rejects_zero_penalty(gpu_engine):
    o = E.default_opt()
    o.s_gapo = 0  # the reference aborts on -O 0
    with pytest.raises(E.IbwaError):
        gpu_engine.aln(np.zeros(36, np.uint8), np.zeros(1, np.uint64), np.full(1, 36, np.uint32), o)


@pytest.mark.parametrize("gap_lw", [1, 0])
def test_sai_goldens_lds_widths(golden_dir, sai_manifest, gpu_engine, gap_lw):
    """The first pass with its width bounds in LDS (gapped.hip LW: clamped bids, equality bits,
    ring of bucket heads; used when the options and the LDS budget allow) and without them: every
    gapped golden .sai either way (150 bp reads and the -M 1 -O 3 -E 1 penalties also exercise the
    fallback's selection)."""
    gpu_engine.set_option("gap_lw", gap_lw)
    bad = []
    for key, m in sorted(sai_manifest.items()):
        if m["argv"] == ["-n", "0"]:
            continue
        opt, _ = oracle.parse_aln_args(m["argv"])
        recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
        seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
        n_aln, alns = gpu_engine.aln(seqs, offs, lens, _eopt(opt))
        if not oracle.sai_body_equal(oracle.sai_bytes(opt, n_aln, alns), open(os.path.join(golden_dir, key + ".sai"), "rb").read()):
            bad.append(key)
    gpu_engine.set_option("gap_lw", 1)
    assert not bad, bad


def test_shared_index_is_frozen(golden_dir, sai_manifest):
    """ibwa_ctx_share_index: a context borrowing another's index aligns the goldens bit-exact, and
    while the index is shared neither side may rebuild or replace it (borrowed buffers would be
    written in place under the other context, or could not grow): option kmer_k and load_bwt fail
    with IBWA_EINVAL on both; once the borrower is gone the source may again."""
    src = E.Engine(0)
    src.load_index_files(os.path.join(golden_dir, "g1m"))
    m = sai_manifest["r100.default"]
    opt, _ = oracle.parse_aln_args(m["argv"])
    src.prepare(_eopt(opt))
    dst = E.Engine(0)
    dst.share_index(src)
    recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
    seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
    n_aln, alns = dst.aln(seqs, offs, lens, _eopt(opt))
    assert oracle.sai_body_equal(oracle.sai_bytes(opt, n_aln, alns), open(os.path.join(golden_dir, "r100.default.sai"), "rb").read())
    for eng in (dst, src):
        with pytest.raises(E.IbwaError, match="share"):
            eng.set_option("kmer_k", 5)
        with pytest.raises(E.IbwaError, match="share"):
            eng.load_index_files(os.path.join(golden_dir, "g1m"))
    with pytest.raises(E.IbwaError, match="share"):
        E.Engine(0).share_index(dst)
    dst.close()
    src.set_option("kmer_k", 5)
    n2, a2 = src.aln(seqs, offs, lens, _eopt(opt))
    assert (n2 == n_aln).all() and a2.tobytes() == alns.tobytes()
    src.close()


_ARENA_SCRIPT = r"""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import oracle
from ibwa_amd import engine as E
L = E.lib()
gold = sys.argv[2]
recs = oracle.read_fastq_records(os.path.join(gold, "reads_r100.fq"))[:300]
opt, _ = oracle.parse_aln_args([])
seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
assert L.ibwa_reserve(0, 4 << 30) == 0, L.ibwa_last_error()
def run():
    eng = E.Engine(0)
    eng.load_index_files(os.path.join(gold, "g1m"))
    n_aln, alns = eng.aln(seqs, offs, lens, E.default_opt())
    return eng, n_aln, alns
eng, n1, a1 = run()
used = ctypes.c_uint64()
L.ibwa_arena_stats(0, None, ctypes.byref(used), None)
assert used.value > 0
# buffers are still carved: the arena cannot go
assert L.ibwa_release(0) != 0 and b"destroy the contexts" in L.ibwa_last_error()
eng.close()
assert L.ibwa_release(0) == 0, L.ibwa_last_error()
# a new arena after the release, and the same hits from contexts carved from it
assert L.ibwa_reserve(0, 4 << 30) == 0, L.ibwa_last_error()
eng, n2, a2 = run()
assert (n1 == n2).all() and a1.tobytes() == a2.tobytes()
eng.close()
assert L.ibwa_release(0) == 0, L.ibwa_last_error()
print("arena ok")
"""


def test_arena_release_refused_while_carved(golden_dir, tmp_path):
    """ibwa_release: refused while a context still holds buffers carved from the arena
    (they would point into freed HBM), allowed once the contexts are destroyed; a new arena can then be
    reserved and gives the same hits.  Its own process: the arena is process-wide."""
    import subprocess
    import sys
    s = tmp_path / "arena.py"
    s.write_text(_ARENA_SCRIPT)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, str(s), root, golden_dir], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "arena ok" in r.stdout, r.stderr[-3000:]
