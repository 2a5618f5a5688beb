"""Synthetic inputs for tests and fixtures (wraps ibwa_amd's synth.cpp)."""
import ctypes
import os

import numpy as np

from ibwa_amd import _native

GOLDEN_SEED = 1
# ~1 Mb golden genome: GRCh37 contig proportions scaled by 1/3100
GOLDEN_SCALE = (1, 3100)


def genome_ascii(seed, num, den, repeat_frac=0.45, n_frac=0.01, n_families=40, threads=8):
    L = _native.lib()
    lens = (ctypes.c_uint64 * 24)()
    tot = L.ibwa_synth_grch37_lengths(num, den, lens)
    buf = np.empty(tot, dtype=np.uint8)
    L.ibwa_synth_genome(seed, 24, lens, repeat_frac, n_frac, n_families, buf.ctypes.data, threads)
    return buf, [int(x) for x in lens]


def golden_genome_ascii():
    buf, lens = genome_ascii(GOLDEN_SEED, *GOLDEN_SCALE)
    names = [f"chr{i}" for i in range(1, 23)] + ["chrX", "chrY"]
    return buf.tobytes().decode(), names, lens


def synth_reads(genome, lens, seed, n, ln, sub, indel, threads=8):
    L = _native.lib()
    g = np.frombuffer(genome.encode() if isinstance(genome, str) else genome, dtype=np.uint8)
    c_lens = (ctypes.c_uint64 * len(lens))(*lens)
    seqs = np.empty(n * ln, dtype=np.uint8)
    pos = np.empty(n, dtype=np.uint64)
    strand = np.empty(n, dtype=np.uint8)
    L.ibwa_synth_reads(seed, g.ctypes.data, g.size, len(lens), c_lens, n, ln, sub, indel,
                       seqs.ctypes.data, pos.ctypes.data, strand.ctypes.data, threads)
    raw = seqs.tobytes().decode()
    return [raw[i * ln:(i + 1) * ln] for i in range(n)]


def write_fastq(path, recs):
    with open(path, "w") as f:
        for nm, s, q in recs:
            f.write(f"@{nm}\n{s}\n+\n{q}\n")
