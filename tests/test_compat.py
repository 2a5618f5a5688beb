"""The drop-in boundary in the reference's own types (include/ibwa_bwa_compat.h).

* layout: every member offset and the sizes of the mirrored bwt_t / bwa_seq_t /
  gap_opt_t / bwt_aln1_t equal the reference's (compile-time checks against the
  reference headers; runs only where /root/reference exists -- this container);
* drop-in parity (GPU): bwa_cal_sa_reg_gap called exactly as bwa_aln_core calls
  it -- reference-layout bwt_t from the .bwt/.rbwt files, a bwa_seq_t array
  with malloc'd seq/rseq/qual/name -- reproduces the golden .sai bytes and
  performs the reference's side effects (seq/rseq/qual/name freed and NULL,
  sa = 0, type = NO_MATCH, c1 = c2 = 0).
"""
import ctypes as c
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
from ibwa_amd import _native
from ibwa_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


class RefBwt(c.Structure):  # bwt_t (bwt.h:41-53)
    _fields_ = [("primary", c.c_uint32), ("L2", c.c_uint32 * 5), ("seq_len", c.c_uint32),
                ("bwt_size", c.c_uint32), ("bwt", c.POINTER(c.c_uint32)), ("cnt_table", c.c_uint32 * 256),
                ("sa_intv", c.c_int), ("n_sa", c.c_uint32), ("sa", c.POINTER(c.c_uint32))]


RefSeq = E.RefSeq  # bwa_seq_t (bwtaln.h:62-93)


LAYOUT_C = r"""
#include <stddef.h>
#include "bwtaln.h"
#include "bwapair.h"
#include "dbset.h"
#include "ibwa_bwa_compat.h"
#define SAME(R, M, F) _Static_assert(offsetof(R, F) == offsetof(M, F), #R "." #F); \
                      _Static_assert(sizeof(((R *)0)->F) == sizeof(((M *)0)->F), #R "." #F " size");
#define SIZE(R, M) _Static_assert(sizeof(R) == sizeof(M), #R " size");
SIZE(bwt_t, ibwa_ref_bwt_t)
SAME(bwt_t, ibwa_ref_bwt_t, primary) SAME(bwt_t, ibwa_ref_bwt_t, L2) SAME(bwt_t, ibwa_ref_bwt_t, seq_len)
SAME(bwt_t, ibwa_ref_bwt_t, bwt_size) SAME(bwt_t, ibwa_ref_bwt_t, bwt) SAME(bwt_t, ibwa_ref_bwt_t, cnt_table)
SAME(bwt_t, ibwa_ref_bwt_t, sa_intv) SAME(bwt_t, ibwa_ref_bwt_t, n_sa) SAME(bwt_t, ibwa_ref_bwt_t, sa)
SIZE(bwa_seq_t, ibwa_ref_seq_t)
SAME(bwa_seq_t, ibwa_ref_seq_t, name) SAME(bwa_seq_t, ibwa_ref_seq_t, seq) SAME(bwa_seq_t, ibwa_ref_seq_t, rseq)
SAME(bwa_seq_t, ibwa_ref_seq_t, qual) SAME(bwa_seq_t, ibwa_ref_seq_t, score) SAME(bwa_seq_t, ibwa_ref_seq_t, clip_len)
SAME(bwa_seq_t, ibwa_ref_seq_t, n_aln) SAME(bwa_seq_t, ibwa_ref_seq_t, aln) SAME(bwa_seq_t, ibwa_ref_seq_t, n_multi)
SAME(bwa_seq_t, ibwa_ref_seq_t, multi) SAME(bwa_seq_t, ibwa_ref_seq_t, sa) SAME(bwa_seq_t, ibwa_ref_seq_t, pos)
SAME(bwa_seq_t, ibwa_ref_seq_t, remapped_pos) SAME(bwa_seq_t, ibwa_ref_seq_t, dbidx)
SAME(bwa_seq_t, ibwa_ref_seq_t, remapped_dbidx) SAME(bwa_seq_t, ibwa_ref_seq_t, remapped_seqid)
SAME(bwa_seq_t, ibwa_ref_seq_t, remap_identical) SAME(bwa_seq_t, ibwa_ref_seq_t, n_cigar)
SAME(bwa_seq_t, ibwa_ref_seq_t, cigar) SAME(bwa_seq_t, ibwa_ref_seq_t, tid) SAME(bwa_seq_t, ibwa_ref_seq_t, bc)
SAME(bwa_seq_t, ibwa_ref_seq_t, md)
SIZE(bwt_multi1_t, ibwa_ref_multi1_t)
SIZE(gap_opt_t, ibwa_gap_opt_t)
SAME(gap_opt_t, ibwa_gap_opt_t, s_mm) SAME(gap_opt_t, ibwa_gap_opt_t, mode) SAME(gap_opt_t, ibwa_gap_opt_t, fnr)
SAME(gap_opt_t, ibwa_gap_opt_t, max_diff) SAME(gap_opt_t, ibwa_gap_opt_t, seed_len)
SAME(gap_opt_t, ibwa_gap_opt_t, max_top2) SAME(gap_opt_t, ibwa_gap_opt_t, trim_qual)
SIZE(bwt_aln1_t, ibwa_aln1_t)
SAME(bwt_aln1_t, ibwa_aln1_t, k) SAME(bwt_aln1_t, ibwa_aln1_t, l) SAME(bwt_aln1_t, ibwa_aln1_t, score)
SIZE(pe_opt_t, ibwa_ref_pe_opt_t)
SAME(pe_opt_t, ibwa_ref_pe_opt_t, max_isize) SAME(pe_opt_t, ibwa_ref_pe_opt_t, n_threads)
SAME(pe_opt_t, ibwa_ref_pe_opt_t, type) SAME(pe_opt_t, ibwa_ref_pe_opt_t, is_sw)
SAME(pe_opt_t, ibwa_ref_pe_opt_t, remapping) SAME(pe_opt_t, ibwa_ref_pe_opt_t, ap_prior)
SIZE(isize_info_t, ibwa_ref_isize_info_t)
SAME(isize_info_t, ibwa_ref_isize_info_t, avg) SAME(isize_info_t, ibwa_ref_isize_info_t, std)
SAME(isize_info_t, ibwa_ref_isize_info_t, ap_prior) SAME(isize_info_t, ibwa_ref_isize_info_t, low)
SAME(isize_info_t, ibwa_ref_isize_info_t, high) SAME(isize_info_t, ibwa_ref_isize_info_t, high_bayesian)
SIZE(bntann1_t, ibwa_ref_bntann1_t) SAME(bntann1_t, ibwa_ref_bntann1_t, offset) SAME(bntann1_t, ibwa_ref_bntann1_t, gi)
SAME(bntann1_t, ibwa_ref_bntann1_t, name) SAME(bntann1_t, ibwa_ref_bntann1_t, anno)
SIZE(bntamb1_t, ibwa_ref_bntamb1_t) SAME(bntamb1_t, ibwa_ref_bntamb1_t, amb)
SIZE(bntseq_t, ibwa_ref_bntseq_t) SAME(bntseq_t, ibwa_ref_bntseq_t, l_pac) SAME(bntseq_t, ibwa_ref_bntseq_t, n_seqs)
SAME(bntseq_t, ibwa_ref_bntseq_t, anns) SAME(bntseq_t, ibwa_ref_bntseq_t, n_holes) SAME(bntseq_t, ibwa_ref_bntseq_t, ambs)
SAME(bntseq_t, ibwa_ref_bntseq_t, fp_pac)
SIZE(seq_t, ibwa_ref_seqt_t) SAME(seq_t, ibwa_ref_seqt_t, bns) SAME(seq_t, ibwa_ref_seqt_t, data)
SAME(seq_t, ibwa_ref_seqt_t, remap) SAME(seq_t, ibwa_ref_seqt_t, mappings)
SIZE(bwtdb_t, ibwa_ref_bwtdb_t) SAME(bwtdb_t, ibwa_ref_bwtdb_t, prefix) SAME(bwtdb_t, ibwa_ref_bwtdb_t, bwt)
SAME(bwtdb_t, ibwa_ref_bwtdb_t, bwtcache) SAME(bwtdb_t, ibwa_ref_bwtdb_t, offset) SAME(bwtdb_t, ibwa_ref_bwtdb_t, bns)
SAME(bwtdb_t, ibwa_ref_bwtdb_t, ntbns)
SIZE(dbset_t, ibwa_ref_dbset_t) SAME(dbset_t, ibwa_ref_dbset_t, count) SAME(dbset_t, ibwa_ref_dbset_t, color_space)
SAME(dbset_t, ibwa_ref_dbset_t, preload) SAME(dbset_t, ibwa_ref_dbset_t, db) SAME(dbset_t, ibwa_ref_dbset_t, bns)
SAME(dbset_t, ibwa_ref_dbset_t, ntbns) SAME(dbset_t, ibwa_ref_dbset_t, l_pac)
SAME(dbset_t, ibwa_ref_dbset_t, total_bwt_seq_len)
int main(void) { return 0; }
"""


@pytest.mark.skipif(not os.path.isdir(REF) or not shutil.which("gcc"), reason="reference headers absent")
def test_layout_matches_reference_headers(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    r = subprocess.run(["gcc", "-std=gnu11", "-fsyntax-only", f"-I{REF}", f"-I{os.path.join(ROOT, 'include')}",
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_python_mirror_sizes():
    # the ctypes mirrors used below agree with the C header's (x86-64 SysV) sizes
    assert c.sizeof(RefBwt) == 4 * 8 + 8 + 1024 + 8 + 8
    assert c.sizeof(RefSeq) % 8 == 0 and RefSeq.bc.offset + 16 <= c.sizeof(RefSeq)


def _load_ref_bwt(path, keep):
    raw = np.fromfile(path, dtype=np.uint32)
    words = np.ascontiguousarray(raw[5:])
    keep.append(words)
    b = RefBwt()
    b.primary = int(raw[0])
    for j in range(4):
        b.L2[j + 1] = int(raw[1 + j])
    b.seq_len = b.L2[4]
    b.bwt_size = words.size
    b.bwt = words.ctypes.data_as(c.POINTER(c.c_uint32))
    return b


def _dropin_run(L, libc, bw, golden_dir, sai_manifest, key):
    """bwa_cal_sa_reg_gap on the golden reads of `key` -> (.sai bytes, expected bytes)."""
    m = sai_manifest[key]
    opt, _ = oracle.parse_aln_args(m["argv"])
    recs = oracle.read_fastq_records(os.path.join(golden_dir, m["reads"]))
    seqs, offs, lens = oracle.encode_reads(recs, opt.mode, opt.trim_qual)
    n = lens.size
    arr = (RefSeq * n)()
    for i in range(n):
        s = seqs[int(offs[i]):int(offs[i]) + int(lens[i])]
        p = libc.malloc(max(1, s.size))
        c.memmove(p, s.ctypes.data, s.size)
        arr[i].seq = p
        arr[i].rseq = libc.malloc(max(1, s.size))  # content unused by the engine; freed by it
        arr[i].qual = libc.malloc(8)
        arr[i].name = libc.malloc(8)
        arr[i].len = int(lens[i])
        arr[i].tid = -1
        arr[i].sa = 7
        arr[i].type = 3
    eo = E.GapOpt()
    for f, _ in E.GapOpt._fields_:
        setattr(eo, f, getattr(opt, f))
    L.bwa_cal_sa_reg_gap(0, bw, n, arr, c.byref(eo))
    n_aln = np.array([arr[i].n_aln for i in range(n)], dtype=np.int32)
    parts = [c.string_at(arr[i].aln, 16 * arr[i].n_aln) for i in range(n)]
    alns = np.frombuffer(b"".join(parts), dtype=oracle.ALN_DTYPE)
    assert all(arr[i].seq is None and arr[i].rseq is None and arr[i].qual is None and arr[i].name is None
               for i in range(n))
    assert all(arr[i].sa == 0 and arr[i].type == 0 and arr[i].c1 == 0 and arr[i].c2 == 0 for i in range(n))
    for i in range(n):
        libc.free(c.c_void_p(arr[i].aln))
    return oracle.sai_bytes(opt, n_aln, alns), open(os.path.join(golden_dir, key + ".sai"), "rb").read()


def _dropin_setup(golden_dir, keep):
    L = c.CDLL(_native.LIB_PATH)
    libc = c.CDLL(None)
    libc.malloc.restype = c.c_void_p
    libc.malloc.argtypes = [c.c_size_t]
    libc.free.argtypes = [c.c_void_p]
    b0 = _load_ref_bwt(os.path.join(golden_dir, "g1m.bwt"), keep)
    b1 = _load_ref_bwt(os.path.join(golden_dir, "g1m.rbwt"), keep)
    keep += [b0, b1]
    bw = (c.POINTER(RefBwt) * 2)(c.pointer(b0), c.pointer(b1))
    L.ibwa_gpu_init.argtypes = [c.c_void_p, c.c_int]
    L.ibwa_gpu_init_ex.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int]
    L.bwa_cal_sa_reg_gap.argtypes = [c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.POINTER(E.GapOpt)]
    L.bwa_cal_sa_reg_gap.restype = None
    return L, libc, bw


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["r100.default", "mixed.default", "mixed.n0", "r150.default", "mixed.c"])
def test_dropin_matches_golden_sai(golden_dir, sai_manifest, key):
    keep = []
    L, libc, bw = _dropin_setup(golden_dir, keep)
    assert L.ibwa_gpu_init(bw, 1) == 0
    try:
        got, exp = _dropin_run(L, libc, bw, golden_dir, sai_manifest, key)
        assert oracle.sai_body_equal(got, exp), key
    finally:
        L.ibwa_gpu_destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("slices,min_slice", [(3, 16), (5, 32), (4, 400)])
def test_dropin_sliced_batch(golden_dir, sai_manifest, slices, min_slice):
    """configs[3]'s split on one GPU: the drop-in cuts a batch into `slices` contiguous slices
    (concurrent engines on device 0).  reads_mixed (17-250 bp) gives every slice its own max
    length, so the .sai matches the golden only if each slice keeps the batch-level max_len
    clamps of bwtaln.c:86-93 (max_gapo, the stack size); -n 0 takes the exact path (and its
    derived jump arrays) per slice."""
    keep = []
    L, libc, bw = _dropin_setup(golden_dir, keep)
    assert L.ibwa_gpu_init_ex(bw, 1, slices, min_slice) == 0
    try:
        bad = []
        for key in ["mixed.default", "mixed.n3o2e3", "mixed.N", "mixed.n0", "mixed.l1000", "mixed.q15",
                    "r100.default", "r150.default"]:
            got, exp = _dropin_run(L, libc, bw, golden_dir, sai_manifest, key)
            if not oracle.sai_body_equal(got, exp):
                bad.append(key)
        assert not bad, bad
    finally:
        L.ibwa_gpu_destroy()
