"""The CPU restatement (oracle/) against the compiled reference's own outputs.

Pins the oracle before it is trusted: every golden .sai (option matrix x read
sets, tools/make_golden.py) must be byte-identical after masking the
n_threads header field, and bwt_occ4 must match the reference's KATs.
"""
import os

import numpy as np
import pytest

import oracle


def test_occ4_kats(golden_dir, oracle_index):
    for which, b in zip(["bwt", "rbwt"], oracle_index):
        for line in open(os.path.join(golden_dir, f"kat_occ4_{which}.tsv")):
            k, *cnt = map(int, line.split())
            assert b.occ4(k) == tuple(cnt), (which, k)


def _load(golden_dir, m):
    opt, _ = oracle.parse_aln_args(m["argv"])
    recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
    return opt, oracle.encode_reads(recs, opt.mode, opt.trim_qual)


@pytest.mark.parametrize("threads", [1, 3])
def test_sai_goldens(golden_dir, sai_manifest, oracle_index, threads):
    b0, b1 = oracle_index
    for key, m in sorted(sai_manifest.items()):
        opt, (seqs, offs, lens) = _load(golden_dir, m)
        n_aln, alns, _ = oracle.cal_sa_reg_gap(b0, b1, seqs, offs, lens, opt, n_threads=threads)
        got = oracle.sai_bytes(opt, n_aln, alns)
        exp = open(os.path.join(golden_dir, key + ".sai"), "rb").read()
        assert oracle.sai_body_equal(got, exp), key


def test_maxdiff_table():
    # bwtaln.c:317-324 prints these breakpoints for the default fnr 0.04
    L = oracle.lib()
    md = [L.or_cal_maxdiff(l, 0.02, 0.04) for l in range(17, 251)]
    assert md[0] == 2 and md[100 - 17] == 5 and md[150 - 17] == 6 and md[37 - 17] == 2 and md[38 - 17] == 3


def test_touch_counts_positive(golden_dir, sai_manifest, oracle_index):
    b0, b1 = oracle_index
    opt, (seqs, offs, lens) = _load(golden_dir, sai_manifest["r100.n0"])
    _, _, t = oracle.cal_sa_reg_gap(b0, b1, seqs, offs, lens, opt, touches=True)
    # -n 0 on 100 bp: 2 full + 2 seed widths (264 steps) plus exact tails
    assert 250 < t.mean() < 500


def test_sw_restatement_matches_reference_vectors(golden_dir):
    """aln_local_core restated (oracle) == the reference's outputs on 2 520 pairs."""
    vecs = oracle.read_sw_vectors(os.path.join(golden_dir, "sw_vectors.tsv"))
    assert len(vecs) > 2000
    bad = []
    for k, (ref, rd, score, pl, start, end, cig) in enumerate(vecs):
        got = oracle.sw_local(oracle.nt4(ref), oracle.nt4(rd))
        if got != (score, pl, start, end, cig):
            bad.append((k, got, (score, pl, start, end, cig)))
    assert not bad, bad[:5]


def test_sw_restatement_matches_reference_ties(golden_dir):
    """... and on 1 080 score-tie pairs (tools/make_sw_ties_golden.py): tandem copies, periods
    1-5 / 31-33, N runs -- the first maximum in row-major order."""
    vecs = oracle.read_sw_vectors(os.path.join(golden_dir, "sw_ties.tsv"))
    assert len(vecs) > 1000
    bad = []
    for k, (ref, rd, score, pl, start, end, cig) in enumerate(vecs):
        got = oracle.sw_local(oracle.nt4(ref), oracle.nt4(rd))
        if got != (score, pl, start, end, cig):
            bad.append((k, got, (score, pl, start, end, cig)))
    assert not bad, bad[:5]


def test_sa2pos_restatement_matches_reference_vectors(golden_dir):
    """bwt_sa (bwt.c:69) + bwtdb_sa2seq (dbset.c:240) restated == the reference on 10 755 rows."""
    g = os.path.join(golden_dir, "g1m")
    b0 = oracle.Bwt(g + ".bwt").load_sa(g + ".sa")
    b1 = oracle.Bwt(g + ".rbwt").load_sa(g + ".rsa")
    s, k, ln, sa, pos = oracle.read_sa2pos_vectors(os.path.join(golden_dir, "sa2pos_vectors.tsv"))
    assert len(k) > 10000 and b0.sa_intv == 32
    got, steps = oracle.sa2seq(b0, b1, s, k, ln, steps=True)
    assert (got == pos).all()
    assert all((b0 if s[i] else b1).bwt_sa(int(k[i])) == sa[i] for i in range(0, len(k), 7))
    assert steps.max() > 64  # walks well past one sampling interval are covered


@pytest.mark.parametrize("name", ["std100", "std150", "solid50"])
def test_paired_sw_restatement_matches_reference(golden_dir, name):
    """bwa_paired_sw (bwasw.c:145-304) restated == the reference's own outputs (tools/make_psw_golden.py)."""
    import json
    m = json.load(open(os.path.join(golden_dir, "psw_manifest.json")))[name]
    pac, l_pac = oracle.read_pac(os.path.join(golden_dir, "g1m"))
    pin, pout = oracle.read_psw(golden_dir, name)
    cnt = oracle.paired_sw(pin, m["type"], m["avg"], m["std"], m["ap_prior"], pac, l_pac)
    assert cnt == [m["mated_singletons"], m["singletons"], m["fixed"], m["discordant"]]
    bad = [(i, k) for i, (p, q) in enumerate(zip(pin, pout)) for k in (0, 1)
           if oracle.psw_row(p[k]) != tuple(q[k][f] for f in oracle.PSW_OUT)]
    assert not bad, bad[:5]


def test_global_core_restatement_matches_reference_vectors(golden_dir):
    """aln_global_core with aln_param_bwa (band 50, gap_end 5; refine_gapped_core) restated ==
    the reference on 3 006 pairs (tools/make_gsw_golden.py)."""
    vecs = oracle.read_gsw_vectors(os.path.join(golden_dir, "gsw_vectors.tsv"))
    assert len(vecs) > 3000
    bad = [k for k, (a, b, sc, pl, cg) in enumerate(vecs)
           if oracle.global_core(oracle.nt4(a), oracle.nt4(b)) != (sc, pl, cg)]
    assert not bad, bad[:5]
