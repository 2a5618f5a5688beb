"""Python binding (ctypes) of the C ABI in include/ibwa_aln.h.

This is plumbing for tests and bench.py; the product interface is the C ABI
and the `ibwa-amd aln` CLI.  Every call goes to libibwa_amd.so on a gfx950
device; there is no CPU path here -- if the library or the device is missing
the call raises.
"""
import ctypes
import os
import struct

import numpy as np

from . import _native

c = ctypes


class GapOpt(c.Structure):
    """gap_opt_t (bwtaln.h:105-115) == ibwa_gap_opt_t; also the 64-byte .sai header."""
    _fields_ = [(n, c.c_int) for n in ("s_mm", "s_gapo", "s_gape", "mode", "indel_end_skip",
                                       "max_del_occ", "max_entries")] + \
               [("fnr", c.c_float)] + \
               [(n, c.c_int) for n in ("max_diff", "max_gapo", "max_gape", "max_seed_diff",
                                       "seed_len", "n_threads", "max_top2", "trim_qual")]


class RunStats(c.Structure):
    _fields_ = [("ms_width", c.c_double), ("ms_search", c.c_double), ("ms_retry", c.c_double),
                ("ms_total", c.c_double), ("n_retry", c.c_int64), ("n_launch_width", c.c_int64),
                ("n_launch_search", c.c_int64), ("path", c.c_int), ("kmer_k", c.c_int),
                ("n_stack_overflow", c.c_int64), ("n_aln_overflow", c.c_int64), ("n_heavy", c.c_int64), ("ms_sw", c.c_double),
                ("n_coop", c.c_int64), ("ms_coop", c.c_double), ("ms_sa2pos", c.c_double),
                ("sa2pos_full", c.c_int), ("ms_coop_width", c.c_double), ("ms_coop_roots", c.c_double),
                ("n_resumed", c.c_int64), ("resume_records", c.c_int64),
                ("resume_records_peak", c.c_int64), ("resume_records_cap", c.c_int64),
                ("coop_pages_peak", c.c_int64), ("coop_pages_cap", c.c_int64), ("ms_alloc", c.c_double)]


class RefSeq(c.Structure):
    """bwa_seq_t (bwtaln.h:62-93) == ibwa_ref_seq_t (ibwa_bwa_compat.h)"""
    _fields_ = [("name", c.c_void_p), ("seq", c.c_void_p), ("rseq", c.c_void_p), ("qual", c.c_void_p),
                ("len", c.c_uint32, 20), ("strand", c.c_uint32, 1), ("type", c.c_uint32, 2),
                ("dummy", c.c_uint32, 1), ("extra_flag", c.c_uint32, 8),
                ("n_mm", c.c_uint32, 8), ("n_gapo", c.c_uint32, 8), ("n_gape", c.c_uint32, 8),
                ("mapQ", c.c_uint32, 8), ("score", c.c_int), ("clip_len", c.c_int), ("n_aln", c.c_int),
                ("aln", c.c_void_p), ("n_multi", c.c_int), ("multi", c.c_void_p), ("sa", c.c_uint32),
                ("pos", c.c_uint64), ("remapped_pos", c.c_uint64), ("dbidx", c.c_uint32),
                ("remapped_dbidx", c.c_uint32), ("remapped_seqid", c.c_int32), ("remap_identical", c.c_int),
                ("c1", c.c_uint64, 28), ("c2", c.c_uint64, 28), ("seQ", c.c_uint64, 8), ("n_cigar", c.c_int),
                ("cigar", c.c_void_p), ("tid", c.c_int), ("bc", c.c_char * 16),
                ("full_len", c.c_uint32, 20), ("nm", c.c_uint32, 12), ("md", c.c_void_p)]


class PeOpt(c.Structure):
    """pe_opt_t (bwtaln.h:120-128) == ibwa_ref_pe_opt_t"""
    _fields_ = [(n, c.c_int) for n in ("max_isize", "force_isize", "max_occ", "n_multi", "N_multi", "n_threads",
                                       "type", "is_sw", "is_preload", "remapping")] + [("ap_prior", c.c_double)]


class IsizeInfo(c.Structure):
    """isize_info_t (bwapair.h:8-11) == ibwa_ref_isize_info_t"""
    _fields_ = [("avg", c.c_double), ("std", c.c_double), ("ap_prior", c.c_double), ("low", c.c_uint32),
                ("high", c.c_uint32), ("high_bayesian", c.c_uint32)]


assert c.sizeof(GapOpt) == 64
ALN_DTYPE = np.dtype([("info", "<u4"), ("k", "<u4"), ("l", "<u4"), ("score", "<i4")])  # bwt_aln1_t

MODE_GAPE, MODE_COMPREAD, MODE_LOGGAP, MODE_NONSTOP = 0x01, 0x02, 0x04, 0x10
MODE_BAM, MODE_BAM_SE, MODE_BAM_READ1, MODE_BAM_READ2, MODE_IL13 = 0x20, 0x40, 0x80, 0x100, 0x200

# every exported symbol declared in include/ibwa_aln.h: name -> (restype, argtypes)
_vp, _i, _i64, _u32, _u64 = c.c_void_p, c.c_int, c.c_int64, c.c_uint32, c.c_uint64
CAPI = {
    "ibwa_last_error": (c.c_char_p, []),
    "ibwa_free": (None, [_vp]),
    "ibwa_gap_init_opt": (None, [c.POINTER(GapOpt)]),
    "ibwa_cal_maxdiff": (_i, [_i, c.c_double, c.c_double]),
    "ibwa_ctx_create": (_i, [_i, c.POINTER(_vp)]),
    "ibwa_device_count": (_i, [c.POINTER(_i)]),
    "ibwa_device_bytes": (_i, [c.POINTER(c.c_int64), c.POINTER(c.c_int64)]),
    "ibwa_device_memory": (_i, [_i, c.POINTER(c.c_uint64), c.POINTER(c.c_uint64)]),
    "ibwa_reserve": (_i, [_i, c.c_uint64]),
    "ibwa_arena_stats": (_i, [_i, c.POINTER(c.c_uint64), c.POINTER(c.c_uint64), c.POINTER(c.c_uint64)]),
    "ibwa_fq_parse": (_i, [_vp, _vp, c.c_uint64, _i, _i, c.POINTER(c.c_int64), c.POINTER(c.c_uint64), c.POINTER(_i),
                           _vp, _vp, c.c_int64]),
    "ibwa_fq_stats": (_i, [_vp, c.POINTER(c.c_int64), c.POINTER(c.c_double)]),
    "ibwa_fq_offset": (_i, [_vp, c.c_int64, c.POINTER(c.c_uint64)]),
    "ibwa_fq_share_scratch": (_i, [_vp, _vp]),
    "ibwa_release": (_i, [_i]),
    "ibwa_batch_fetch_sai": (_i, [_vp, _vp, c.c_uint64, c.POINTER(c.c_uint64), c.POINTER(c.c_int64)]),
    "ibwa_batch_stage_fq": (_i, [_vp, _vp, c.c_int64, c.c_int64, _i]),
    "ibwa_host_alloc": (_i, [c.c_uint64, c.POINTER(_vp)]),
    "ibwa_host_free": (_i, [_vp]),
    "ibwa_ctx_destroy": (None, [_vp]),
    "ibwa_ctx_load_bwt": (_i, [_vp, _i, _u32, c.POINTER(_u32), _vp, _u64]),
    "ibwa_ctx_load_bwt_file": (_i, [_vp, _i, c.c_char_p]),
    "ibwa_ctx_clone_index": (_i, [_vp, _vp]),
    "ibwa_ctx_share_index": (_i, [_vp, _vp]),
    "ibwa_aln_batch": (_i, [_vp, c.POINTER(GapOpt), _i64, _vp, _vp, _vp, _i, _vp, c.POINTER(_vp),
                            c.POINTER(_i64)]),
    "ibwa_batch_stage": (_i, [_vp, _i64, _vp, _vp, _vp]),
    "ibwa_batch_run": (_i, [_vp, c.POINTER(GapOpt), _i]),
    "ibwa_batch_fetch": (_i, [_vp, _vp, c.POINTER(_vp), c.POINTER(_i64)]),
    "ibwa_batch_stats": (_i, [_vp, c.POINTER(RunStats)]),
    "ibwa_ctx_set_tuning": (_i, [_vp, _i, _i, _i]),
    "ibwa_aln_parse_args": (_i, [_i, c.POINTER(c.c_char_p), c.POINTER(GapOpt), c.POINTER(_i), c.POINTER(c.c_char_p)]),
    "ibwa_batch_retry_info": (_i, [_vp, _vp, _vp, _i64, c.POINTER(_i64)]),
    "ibwa_batch_diag": (_i, [_vp, _i, _vp, _u64]),
    "ibwa_ctx_set_option": (_i, [_vp, c.c_char_p, c.c_long]),
    "ibwa_build_id": (c.c_char_p, []),
    "ibwa_occ4": (_i, [_vp, _i, _i64, _vp, _vp]),
    "ibwa_ctx_load_sa": (_i, [_vp, _i, _u32, _vp, _u64]),
    "ibwa_ctx_load_sa_file": (_i, [_vp, _i, c.c_char_p]),
    "ibwa_ctx_expand_sa": (_i, [_vp]),
    "ibwa_ctx_prepare": (_i, [_vp, c.POINTER(GapOpt)]),
    "ibwa_ctx_derive_sa": (_i, [_vp, _u32]),
    "ibwa_sa2pos": (_i, [_vp, _i64, _vp, _vp, _vp, _u64, _vp]),
    "ibwa_ctx_build_index": (_i, [_vp, _vp, _u64, _i]),
    "ibwa_ctx_bwt_info": (_i, [_vp, _i, c.POINTER(_u32), c.POINTER(_u32), c.POINTER(_u64)]),
    "ibwa_ctx_export_bwt": (_i, [_vp, _i, _vp, _u64]),
    "ibwa_ctx_export_sa": (_i, [_vp, _i, _vp, _u64]),
    "ibwa_sw_batch": (_i, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, c.POINTER(c.c_void_p),
                           c.POINTER(_i64)]),
    "ibwa_global_batch": (_i, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, c.POINTER(c.c_void_p),
                               c.POINTER(_i64)]),
    "ibwa_paired_sw": (_i, [_vp, _i, c.POINTER(c.POINTER(RefSeq)), c.POINTER(PeOpt), c.POINTER(IsizeInfo), _vp,
                            _u64, c.POINTER(_u64), c.POINTER(_u64)]),
    "ibwa_paired_sw_dbs": (_i, [_vp, _i, c.POINTER(c.POINTER(RefSeq)), c.POINTER(PeOpt), c.POINTER(IsizeInfo), _i, _vp,
                                _vp, _vp, c.POINTER(_u64), c.POINTER(_u64)]),
    "ibwa_sw_core_batch": (_i, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp,
                                c.POINTER(c.c_void_p)]),
}


def declare(L):
    import os
    older = bool(os.environ.get("IBWA_LIB"))  # an A/B build (tools/) may predate newer entry points
    for name, (res, args) in CAPI.items():
        if older and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


_declared = False


def lib():
    global _declared
    L = _native.lib()
    if not _declared:
        declare(L)
        _declared = True
    return L


class IbwaError(RuntimeError):
    pass


def _chk(rc):
    if rc != 0:
        raise IbwaError(f"ibwa error {rc}: {lib().ibwa_last_error().decode()}")


def default_opt():
    o = GapOpt()
    lib().ibwa_gap_init_opt(c.byref(o))
    return o


def parse_aln_args(args):
    """The product's own `aln` option parser (ibwa_aln_parse_args: bwtaln.c:249-284) -> GapOpt."""
    argv = [b"aln"] + [a.encode() for a in args]
    arr = (c.c_char_p * len(argv))(*argv)
    o = GapOpt()
    rc = lib().ibwa_aln_parse_args(len(argv), arr, c.byref(o), None, None)
    if rc < 0:
        raise IbwaError(f"bad aln options {args}")
    if rc != len(argv):
        raise IbwaError(f"unexpected positional arguments in {args}")
    return o


def read_bwt_file(path):
    """bwt_restore_bwt (bwtio.c:51-70): -> (primary, L2[1..4], words uint32)."""
    with open(path, "rb") as f:
        primary, = struct.unpack("<I", f.read(4))
        L2 = struct.unpack("<4I", f.read(16))
        words = np.frombuffer(f.read(), dtype=np.uint32)
    return primary, L2, words


class Engine:
    """One device context (one GPU) with both FM-indexes resident in HBM."""

    def __init__(self, device=0):
        L = lib()
        h = c.c_void_p()
        _chk(L.ibwa_ctx_create(device, c.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib().ibwa_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_index_files(self, prefix):
        _chk(lib().ibwa_ctx_load_bwt_file(self.h, 0, (prefix + ".bwt").encode()))
        _chk(lib().ibwa_ctx_load_bwt_file(self.h, 1, (prefix + ".rbwt").encode()))

    def load_index(self, strand, primary, L2, words):
        words = np.ascontiguousarray(words, dtype=np.uint32)
        arr = (c.c_uint32 * 4)(*[int(x) for x in L2])
        _chk(lib().ibwa_ctx_load_bwt(self.h, strand, int(primary), arr, words.ctypes.data, words.size))

    def share_index(self, src):
        """Borrow src's resident index (ibwa_ctx_share_index); src must outlive this engine."""
        _chk(lib().ibwa_ctx_share_index(self.h, src.h))
        self._share_src = src

    def set_tuning(self, stack_cap=0, aln_cap=0, block=0):
        _chk(lib().ibwa_ctx_set_tuning(self.h, stack_cap, aln_cap, block))

    def set_option(self, key, value):
        _chk(lib().ibwa_ctx_set_option(self.h, key.encode(), int(value)))

    def stage(self, seqs, offs, lens):
        self._keep = (np.ascontiguousarray(seqs, dtype=np.uint8), np.ascontiguousarray(offs, dtype=np.uint64),
                      np.ascontiguousarray(lens, dtype=np.uint32))
        s, o, l = self._keep
        _chk(lib().ibwa_batch_stage(self.h, l.size, s.ctypes.data, o.ctypes.data, l.ctypes.data))
        self.n = l.size

    def run(self, opt, batch_max_len=0):
        _chk(lib().ibwa_batch_run(self.h, c.byref(opt), batch_max_len))

    def fetch(self):
        n_aln = np.zeros(self.n, dtype=np.int32)
        ptr = c.c_void_p()
        tot = c.c_int64()
        _chk(lib().ibwa_batch_fetch(self.h, n_aln.ctypes.data, c.byref(ptr), c.byref(tot)))
        buf = c.string_at(ptr.value, tot.value * 16)
        lib().ibwa_free(ptr)
        return n_aln, np.frombuffer(buf, dtype=ALN_DTYPE).copy()

    def fetch_sai(self):
        """The batch's .sai records (ibwa_batch_fetch_sai): per read int32 n_aln + n_aln records."""
        need = c.c_uint64()
        _chk(lib().ibwa_batch_fetch_sai(self.h, None, 0, c.byref(need), None))
        buf = c.create_string_buffer(max(need.value, 1))
        _chk(lib().ibwa_batch_fetch_sai(self.h, buf, need.value, c.byref(need), None))
        return buf.raw[:need.value]

    def retry_info(self):
        """(read ids, pass) of the reads the last run's first pass handed on; pass 1 = coop,
        2 = sequential wide, 3 = general kernels, 4 = coop resuming the first pass's state."""
        n = c.c_int64()
        _chk(lib().ibwa_batch_retry_info(self.h, None, None, 0, c.byref(n)))
        ids = np.zeros(n.value, np.int64)
        ps = np.zeros(n.value, np.uint8)
        _chk(lib().ibwa_batch_retry_info(self.h, ids.ctypes.data, ps.ctypes.data, n.value, c.byref(n)))
        return ids, ps

    def diag(self):
        """(first-pass iterations uint32[n], k_width features uint16[n, 4]) of the last run (option diag=1)."""
        it = np.zeros(self.n, np.uint32)
        ft = np.zeros((self.n, 4), np.uint16)
        _chk(lib().ibwa_batch_diag(self.h, 0, it.ctypes.data, it.nbytes))
        _chk(lib().ibwa_batch_diag(self.h, 1, ft.ctypes.data, ft.nbytes))
        return it, ft

    def handoff_pops(self):
        """Per read: pops the first pass made before leaving its resume state (0: none), ibwa_batch_diag 2."""
        hp = np.zeros(self.n, np.uint32)
        _chk(lib().ibwa_batch_diag(self.h, 2, hp.ctypes.data, hp.nbytes))
        return hp

    @staticmethod
    def device_bytes():
        """(bytes held now, high-water mark) of the library's device buffers, all contexts of the process."""
        now, peak = c.c_int64(), c.c_int64()
        _chk(lib().ibwa_device_bytes(c.byref(now), c.byref(peak)))
        return now.value, peak.value

    def stats(self):
        st = RunStats()
        _chk(lib().ibwa_batch_stats(self.h, c.byref(st)))
        return st

    def aln(self, seqs, offs, lens, opt, batch_max_len=0):
        """bwa_cal_sa_reg_gap over one batch -> (n_aln[n], alns ALN_DTYPE)."""
        self.stage(seqs, offs, lens)
        self.run(opt, batch_max_len)
        return self.fetch()

    def build_index(self, codes, sa_intv=0):
        """On-device `bwa index` (BWT part) from 2-bit codes (uint8, N already replaced)."""
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        _chk(lib().ibwa_ctx_build_index(self.h, codes.ctypes.data, codes.size, sa_intv))

    def bwt_info(self, strand):
        p = c.c_uint32()
        L2 = (c.c_uint32 * 4)()
        sz = c.c_uint64()
        _chk(lib().ibwa_ctx_bwt_info(self.h, strand, c.byref(p), L2, c.byref(sz)))
        return p.value, tuple(L2), sz.value

    def export_bwt(self, strand):
        """-> (primary, L2[1..4], words) in the reference .bwt layout."""
        primary, L2, sz = self.bwt_info(strand)
        words = np.zeros(sz, dtype=np.uint32)
        _chk(lib().ibwa_ctx_export_bwt(self.h, strand, words.ctypes.data, sz))
        return primary, L2, words

    def export_sa(self, strand, intv):
        n = self.bwt_info(strand)[1][3]
        out = np.zeros((n + intv) // intv, dtype=np.uint32)
        _chk(lib().ibwa_ctx_export_sa(self.h, strand, out.ctypes.data, out.size))
        return out

    def load_sa_files(self, prefix):
        """bwt_restore_sa (bwtio.c:29) of prefix.sa / prefix.rsa onto the device."""
        _chk(lib().ibwa_ctx_load_sa_file(self.h, 0, (prefix + ".sa").encode()))
        _chk(lib().ibwa_ctx_load_sa_file(self.h, 1, (prefix + ".rsa").encode()))

    def load_sa(self, strand, sa, intv):
        sa = np.ascontiguousarray(sa, dtype=np.uint32)
        _chk(lib().ibwa_ctx_load_sa(self.h, strand, int(intv), sa.ctypes.data, sa.size))

    def derive_sa(self, intv=32):
        """Sampled SA of both strands derived on the device from the resident BWT alone."""
        _chk(lib().ibwa_ctx_derive_sa(self.h, intv))

    def expand_sa(self):
        _chk(lib().ibwa_ctx_expand_sa(self.h))

    def prepare(self, opt):
        """The per-index device structures the first run with `opt` needs (ibwa_ctx_prepare)."""
        _chk(lib().ibwa_ctx_prepare(self.h, c.byref(opt)))

    def sa2pos(self, strand, k, lens, offset=0):
        """bwtdb_sa2seq (dbset.c:240-246) for arrays of hits -> uint64 positions."""
        strand = np.ascontiguousarray(strand, dtype=np.uint8)
        k = np.ascontiguousarray(k, dtype=np.uint32)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        pos = np.zeros(k.size, dtype=np.uint64)
        _chk(lib().ibwa_sa2pos(self.h, k.size, strand.ctypes.data, k.ctypes.data, lens.ctypes.data, int(offset),
                               pos.ctypes.data))
        return pos

    def paired_sw(self, seqs0, seqs1, pe_opt, ii, pac, l_pac):
        """bwa_paired_sw (bwasw.c:270) over two RefSeq arrays (mutated in place);
        pac = the packed .pac bytes.  Returns [mated singletons, singletons, fixed, discordant]."""
        arr = (c.POINTER(RefSeq) * 2)(c.cast(seqs0, c.POINTER(RefSeq)), c.cast(seqs1, c.POINTER(RefSeq)))
        pac = np.ascontiguousarray(pac, dtype=np.uint8)
        tot = (c.c_uint64 * 2)()
        mapped = (c.c_uint64 * 2)()
        _chk(lib().ibwa_paired_sw(self.h, len(seqs0), arr, c.byref(pe_opt), c.byref(ii), pac.ctypes.data, int(l_pac),
                                  tot, mapped))
        return [mapped[1], tot[1], mapped[0], tot[0]]

    def global_align(self, refs, reads, band=50, gap_end=5):
        """Batched aln_global_core (stdaln.c:345) with aln_param_bwa scores -> list of
        (score, path_len, cigar str) per pair."""
        n = len(refs)
        o1 = np.zeros(n, np.uint64)
        o2 = np.zeros(n, np.uint64)
        l1 = np.array([len(x) for x in refs], np.uint32)
        l2 = np.array([len(x) for x in reads], np.uint32)
        if n:
            o1[1:] = np.cumsum(l1[:-1])
            o2[1:] = np.cumsum(l2[:-1])
        s1 = np.concatenate([np.asarray(x, np.uint8) for x in refs] + [np.zeros(1, np.uint8)])
        s2 = np.concatenate([np.asarray(x, np.uint8) for x in reads] + [np.zeros(1, np.uint8)])
        score = np.zeros(n, np.int32)
        plen = np.zeros(n, np.int32)
        ncig = np.zeros(n, np.int32)
        ptr = c.c_void_p()
        tot = c.c_int64()
        _chk(lib().ibwa_global_batch(self.h, n, s1.ctypes.data, o1.ctypes.data, l1.ctypes.data, s2.ctypes.data,
                                     o2.ctypes.data, l2.ctypes.data, band, gap_end, score.ctypes.data,
                                     plen.ctypes.data, ncig.ctypes.data, c.byref(ptr), c.byref(tot)))
        cig = np.frombuffer(c.string_at(ptr.value, 4 * max(tot.value, 0)), dtype=np.uint32).copy()
        lib().ibwa_free(ptr)
        out, q = [], 0
        for p in range(n):
            out.append((int(score[p]), int(plen[p]),
                        "".join(f"{x >> 4}{'MIDS'[x & 0xf]}" for x in cig[q:q + ncig[p]])))
            q += ncig[p]
        return out

    def sw(self, refs, reads):
        """Batched aln_local_core (stdaln.c:529) over code arrays.  Returns a list of
        (score, path_len, start (i, j) | None, end (i, j) | None, cigar str | None)."""
        n = len(refs)
        o1 = np.zeros(n, np.uint64)
        o2 = np.zeros(n, np.uint64)
        l1 = np.array([len(x) for x in refs], np.uint32)
        l2 = np.array([len(x) for x in reads], np.uint32)
        if n:
            o1[1:] = np.cumsum(l1[:-1])
            o2[1:] = np.cumsum(l2[:-1])
        s1 = np.concatenate([np.asarray(x, np.uint8) for x in refs] + [np.zeros(1, np.uint8)])
        s2 = np.concatenate([np.asarray(x, np.uint8) for x in reads] + [np.zeros(1, np.uint8)])
        score = np.zeros(n, np.int32)
        plen = np.zeros(n, np.int32)
        ends = np.zeros((n, 4), np.int32)
        ncig = np.zeros(n, np.int32)
        ptr = c.c_void_p()
        tot = c.c_int64()
        _chk(lib().ibwa_sw_batch(self.h, n, s1.ctypes.data, o1.ctypes.data, l1.ctypes.data, s2.ctypes.data,
                                 o2.ctypes.data, l2.ctypes.data, score.ctypes.data, plen.ctypes.data,
                                 ends.ctypes.data, ncig.ctypes.data, c.byref(ptr), c.byref(tot)))
        cig = np.frombuffer(c.string_at(ptr.value, 4 * max(tot.value, 0)), dtype=np.uint32).copy()
        lib().ibwa_free(ptr)
        out, q = [], 0
        for p in range(n):
            if score[p] >= 0 and plen[p] > 0:
                cs = "".join(f"{x >> 4}{'MIDS'[x & 0xf]}" for x in cig[q:q + ncig[p]])
                out.append((int(score[p]), int(plen[p]), (int(ends[p, 0]), int(ends[p, 1])),
                            (int(ends[p, 2]), int(ends[p, 3])), cs))
            else:
                out.append((int(score[p]), int(plen[p]), None, None, None))
            q += ncig[p]
        return out

    def sw_core(self, reads, windows, reglen, beg, l_pac):
        """bwa_sw_core (bwasw.c:29-112) per mate rescue, batched.  Returns a list of
        None (rejected) or (beg, [bwa_cigar_t ...], cnt)."""
        n = len(reads)
        off = np.zeros(n, np.uint64)
        roff = np.zeros(n, np.uint64)
        ln = np.array([len(x) for x in reads], np.uint32)
        rl = np.array([len(x) for x in windows], np.uint32)
        if n:
            off[1:] = np.cumsum(ln[:-1])
            roff[1:] = np.cumsum(rl[:-1])
        s = np.concatenate([np.asarray(x, np.uint8) for x in reads] + [np.zeros(1, np.uint8)])
        r = np.concatenate([np.asarray(x, np.uint8) for x in windows] + [np.zeros(1, np.uint8)])
        rg = np.ascontiguousarray(reglen, np.int32)
        bg = np.ascontiguousarray(beg, np.int64).copy()
        nc = np.zeros(n, np.int32)
        cnt = np.zeros(n, np.uint32)
        ptr = c.c_void_p()
        _chk(lib().ibwa_sw_core_batch(self.h, n, s.ctypes.data, off.ctypes.data, ln.ctypes.data, r.ctypes.data,
                                      roff.ctypes.data, rl.ctypes.data, rg.ctypes.data, bg.ctypes.data, int(l_pac),
                                      nc.ctypes.data, cnt.ctypes.data, c.byref(ptr)))
        tot = int(nc.sum())
        cig = np.frombuffer(c.string_at(ptr.value, 4 * tot), dtype=np.uint32).copy() if tot else np.zeros(0, np.uint32)
        lib().ibwa_free(ptr)
        out, q = [], 0
        for p in range(n):
            if nc[p]:
                out.append((int(bg[p]), [int(x) for x in cig[q:q + nc[p]]], int(cnt[p])))
            else:
                out.append(None)
            q += nc[p]
        return out

    def occ4(self, strand, ks):
        ks = np.ascontiguousarray(ks, dtype=np.uint32)
        out = np.zeros((ks.size, 4), dtype=np.uint32)
        _chk(lib().ibwa_occ4(self.h, strand, ks.size, ks.ctypes.data, out.ctypes.data))
        return out
