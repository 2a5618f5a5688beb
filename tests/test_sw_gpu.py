"""GPU parity of the batched Smith-Waterman.

ibwa_sw_batch (sw.hip, through the C ABI) against the reference's own
aln_local_core outputs (tests/golden/sw_vectors.tsv: 2 520 pairs made by the
compiled reference, tools/make_sw_golden.py) and against the CPU restatement
on seeded random pairs of many shapes: score, path length, start and end
coordinates and CIGAR, bit-exact.
"""
import os
import random

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def test_sw_golden_vectors(golden_dir, gpu_engine):
    vecs = oracle.read_sw_vectors(os.path.join(golden_dir, "sw_vectors.tsv"))
    got = gpu_engine.sw([oracle.nt4(v[0]) for v in vecs], [oracle.nt4(v[1]) for v in vecs])
    bad = [(k, g, v[2:]) for k, (g, v) in enumerate(zip(got, vecs)) if g != tuple(v[2:])]
    assert not bad, bad[:5]


def test_sw_random_shapes_vs_oracle(gpu_engine):
    rng = random.Random(99)
    refs, reads = [], []
    for _ in range(3000):
        l1 = rng.choice([1, 5, 20, 64, 150, 333, 510, 800])
        l2 = rng.choice([1, 7, 20, 36, 100, 150, 251])
        ref = np.array([rng.choice([0, 1, 2, 3, 3, 2, 4] if rng.random() < 0.1 else [0, 1, 2, 3])
                        for _ in range(l1)], np.uint8)
        if rng.random() < 0.6 and l1 > 10:
            a = rng.randrange(0, l1)
            rd = ref[a:a + l2].copy()
            for k in range(len(rd)):
                if rng.random() < 0.05:
                    rd[k] = rng.randrange(5)
            rd = np.concatenate([rd, np.array([rng.randrange(4) for _ in range(max(0, l2 - len(rd)))], np.uint8)])
        else:
            rd = np.array([rng.randrange(4) for _ in range(l2)], np.uint8)
        refs.append(ref)
        reads.append(rd)
    got = gpu_engine.sw(refs, reads)
    bad = []
    for k, (a, b) in enumerate(zip(refs, reads)):
        exp = oracle.sw_local(a, b)
        if got[k] != exp:
            bad.append((k, got[k], exp))
    assert not bad, bad[:5]


def test_sw_tie_vectors(golden_dir, gpu_engine):
    """The reference's outputs on 1 080 score-tie pairs (tools/make_sw_ties_golden.py)."""
    vecs = oracle.read_sw_vectors(os.path.join(golden_dir, "sw_ties.tsv"))
    got = gpu_engine.sw([oracle.nt4(v[0]) for v in vecs], [oracle.nt4(v[1]) for v in vecs])
    bad = [(k, g, v[2:]) for k, (g, v) in enumerate(zip(got, vecs)) if g != tuple(v[2:])]
    assert not bad, (len(bad), bad[:5])


def test_sw_adversarial_ties(gpu_engine):
    """Inputs whose best local score is reached by many cells: tandem copies of the read in the
    window (equal maxima in different rows and strips), homopolymers and short-period repeats
    (equal maxima along diagonals, across the 32-column strip edges), N runs, and reads that match
    two windows places equally.  The reference keeps the first maximum in row-major order
    (stdaln.c:615-626, `if (h > score_f)`); the strip-mined forward pass must find the same cell."""
    rng = random.Random(2024)
    refs, reads = [], []

    def push(ref, rd):
        refs.append(np.array(ref, np.uint8))
        reads.append(np.array(rd, np.uint8))

    for _ in range(400):
        l2 = rng.choice([7, 16, 31, 32, 33, 36, 64, 100, 150])
        rd = [rng.randrange(4) for _ in range(l2)]
        k = rng.choice([2, 3, 4])
        gap = [rng.randrange(4) for _ in range(rng.choice([0, 1, 5, 31, 32, 33]))]
        ref = []
        for _c in range(k):
            ref += rd + gap
        push(ref[:800], rd)
        # the read's halves swapped in the window: two equal partial maxima
        h = l2 // 2
        push(rd[h:] + gap + rd[:h] + gap + rd[h:], rd)
    for period in (1, 2, 3, 4, 5, 31, 32, 33):
        unit = [rng.randrange(4) for _ in range(period)]
        for l1, l2 in ((64, 36), (510, 150), (300, 100), (33, 33), (96, 64)):
            ref = (unit * (l1 // period + 1))[:l1]
            rd = (unit * (l2 // period + 2))[rng.randrange(period):][:l2]
            push(ref, rd)
            rd2 = list(rd)
            rd2[l2 // 2] = (rd2[l2 // 2] + 1) % 4  # one mismatch: many equal-score local hits
            push(ref, rd2)
    for _ in range(200):  # N runs in the window and the read
        l1, l2 = rng.choice([(510, 150), (200, 100), (64, 36)])
        ref = [rng.randrange(4) for _ in range(l1)]
        a0 = rng.randrange(0, l1 - l2)
        rd = ref[a0:a0 + l2]
        for _n in range(rng.randrange(1, 6)):
            q = rng.randrange(l2)
            for t in range(q, min(l2, q + rng.randrange(1, 8))):
                rd[t] = 4
        q = rng.randrange(l1)
        for t in range(q, min(l1, q + rng.randrange(1, 40))):
            ref[t] = 4
        push(ref, rd)
    got = gpu_engine.sw(refs, reads)
    bad = [(k, got[k], exp) for k, (a, b) in enumerate(zip(refs, reads)) if got[k] != (exp := oracle.sw_local(a, b))]
    assert not bad, (len(bad), bad[:3])


def test_sw_rejects_overflowing_lengths(gpu_engine):
    from ibwa_amd import engine as E
    with pytest.raises(E.IbwaError):
        gpu_engine.sw([np.zeros(3000, np.uint8)], [np.zeros(3000, np.uint8)])


def test_sw_core_batch_vs_oracle(gpu_engine):
    """bwa_sw_core (a13): pre-checks, SW, acceptance, soft clips, counts -- GPU batch == restatement."""
    from tests.synth_util import golden_genome_ascii
    genome, _, _ = golden_genome_ascii()
    g = oracle.nt4(genome)
    rng = random.Random(7)
    reads, wins, regl, begs = [], [], [], []
    for k in range(1500):
        ln = rng.choice([36, 100, 150])
        p = rng.randrange(0, g.size - 700)
        reglen = rng.choice([10, 19, 20, 2 * ln + 210, 600])
        beg = p
        w = g[p:p + reglen].copy()
        off = rng.randrange(-40, max(1, reglen - ln + 40))
        src = g[max(0, p + off):max(0, p + off) + ln].copy()
        if src.size < ln:
            src = np.concatenate([src, np.zeros(ln - src.size, np.uint8)])
        for q in range(ln):
            if rng.random() < 0.02:
                src[q] = rng.randrange(4)
        if k % 50 == 0:
            src[: ln // 3] = 4  # too many N
        reads.append(src)
        wins.append(w)
        regl.append(reglen)
        begs.append(beg)
    l_pac = int(g.size)
    got = gpu_engine.sw_core(reads, wins, regl, begs, l_pac)
    exp = [oracle.sw_core(r, w, rg, b, l_pac) for r, w, rg, b in zip(reads, wins, regl, begs)]
    exp = [None if e is None else (e[0], e[1], e[2]) for e in exp]
    bad = [(k, a, b) for k, (a, b) in enumerate(zip(got, exp)) if a != b]
    assert not bad, bad[:5]
    assert sum(e is not None for e in exp) > 500


def test_global_golden_vectors(golden_dir, gpu_engine):
    """Batched aln_global_core (bwa_refine_gapped's band 50, gap_end 5) == the reference."""
    vecs = oracle.read_gsw_vectors(os.path.join(golden_dir, "gsw_vectors.tsv"))
    got = gpu_engine.global_align([oracle.nt4(v[0]) for v in vecs], [oracle.nt4(v[1]) for v in vecs], 50, 5)
    bad = [(k, g, v[2:]) for k, (g, v) in enumerate(zip(got, vecs)) if g != tuple(v[2:])]
    assert not bad, bad[:3]


def test_global_gap_end_negative_vs_oracle(gpu_engine):
    """gap_end < 0 (the local core's path fill) and other bands on random shapes vs the restatement."""
    rng = np.random.default_rng(3)
    refs, reads = [], []
    for _ in range(400):
        n1, n2 = int(rng.integers(1, 160)), int(rng.integers(1, 160))
        refs.append(rng.integers(0, 5, n1).astype(np.uint8))
        reads.append(rng.integers(0, 5, n2).astype(np.uint8))
    for band, ge in ((50, -1), (5, 5), (20, -1)):
        got = gpu_engine.global_align(refs, reads, band, ge)
        exp = [oracle.global_core(a, b, band, ge) for a, b in zip(refs, reads)]
        assert got == exp, (band, ge, [k for k in range(len(got)) if got[k] != exp[k]][:5])
