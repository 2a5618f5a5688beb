"""oracle -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference `ibwa aln` hot path, used by tests/,
``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg as the checker
(or the timed CPU baseline).  The shipped product (ibwa_amd/, include/) never
imports it.  Parity of this restatement is pinned against golden vectors made
by the compiled reference (tests/golden/, tools/make_golden.py).
"""
import ctypes
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "liboracle.so")
REF_BIN = os.path.join(HERE, "_ref", "ibwa_ref")
REF_LIB = os.path.join(HERE, "_ref", "libibwa_ref.so")

MODE_GAPE, MODE_COMPREAD, MODE_LOGGAP, MODE_NONSTOP = 0x01, 0x02, 0x04, 0x10
MODE_BAM, MODE_BAM_SE, MODE_BAM_READ1, MODE_BAM_READ2, MODE_IL13 = 0x20, 0x40, 0x80, 0x100, 0x200


class GapOpt(ctypes.Structure):
    """gap_opt_t (bwtaln.h:105-115) -- also the 64-byte .sai header."""
    _fields_ = [(n, ctypes.c_int) for n in ("s_mm", "s_gapo", "s_gape", "mode", "indel_end_skip",
                                            "max_del_occ", "max_entries")] + \
               [("fnr", ctypes.c_float)] + \
               [(n, ctypes.c_int) for n in ("max_diff", "max_gapo", "max_gape", "max_seed_diff",
                                            "seed_len", "n_threads", "max_top2", "trim_qual")]


assert ctypes.sizeof(GapOpt) == 64

ALN_DTYPE = np.dtype([("info", "<u4"), ("k", "<u4"), ("l", "<u4"), ("score", "<i4")])  # bwtaln.h:34-38


def build(quiet=True):
    """Compile the restatement (gcc) -- building the checker, not using it."""
    kw = {"stdout": subprocess.DEVNULL} if quiet else {}
    subprocess.run(["make", "-C", HERE, "oracle"], check=True, **kw)


def build_ref(quiet=True):
    """Compile the reference from /root/reference into oracle/_ref (build container only)."""
    if not os.path.isdir("/root/reference"):
        return False
    kw = {"stdout": subprocess.DEVNULL, "stderr": subprocess.DEVNULL} if quiet else {}
    subprocess.run(["make", "-C", HERE, "ref", "-j8"], check=True, **kw)
    return True


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c = ctypes
        L.or_bwt_load.restype = c.c_void_p
        L.or_bwt_load.argtypes = [c.c_char_p]
        L.or_bwt_wrap.restype = c.c_void_p
        L.or_bwt_wrap.argtypes = [c.c_uint32, c.POINTER(c.c_uint32), c.c_void_p, c.c_uint64]
        L.or_bwt_free.argtypes = [c.c_void_p]
        L.or_occ.restype = c.c_uint32
        L.or_occ.argtypes = [c.c_void_p, c.c_uint32, c.c_int]
        L.or_occ4.argtypes = [c.c_void_p, c.c_uint32, c.POINTER(c.c_uint32)]
        L.or_cal_maxdiff.restype = c.c_int
        L.or_cal_maxdiff.argtypes = [c.c_int, c.c_double, c.c_double]
        L.or_gap_init_opt.argtypes = [c.POINTER(GapOpt)]
        L.or_cal_sa_reg_gap.restype = c.c_int64
        L.or_cal_sa_reg_gap.argtypes = [c.c_void_p, c.c_void_p, c.c_int64, c.c_void_p, c.c_void_p,
                                        c.c_void_p, c.POINTER(GapOpt), c.c_int, c.c_void_p,
                                        c.POINTER(c.c_void_p), c.c_void_p]
        L.or_free.argtypes = [c.c_void_p]
        L.or_set_stats.argtypes = [c.c_void_p]
        L.or_set_width_touches.argtypes = [c.c_void_p]
        L.or_set_touch_split.argtypes = [c.c_void_p, c.c_void_p]
        L.or_push_kinds.argtypes = [c.c_void_p]
        L.or_depth_hist.argtypes = [c.c_void_p]
        L.or_exact_touches.argtypes = [c.c_void_p, c.c_void_p, c.c_int64, c.c_void_p, c.c_void_p, c.c_void_p,
                                       c.c_int, c.c_int, c.c_int, c.c_void_p]
        L.or_aln_local_core.restype = c.c_int
        L.or_aln_local_core.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p,
                                        c.POINTER(c.c_int), c.c_int, c.c_void_p]
        L.or_path2cigar32.restype = c.c_int
        L.or_path2cigar32.argtypes = [c.c_void_p, c.c_int, c.c_void_p]
        L.or_bwt_info.argtypes = [c.c_void_p, c.POINTER(c.c_uint32), c.POINTER(c.c_uint32)]
        L.or_sa_load.restype = c.c_void_p
        L.or_sa_load.argtypes = [c.c_char_p, c.c_void_p, c.POINTER(c.c_uint32), c.POINTER(c.c_uint64)]
        L.or_bwt_sa.restype = c.c_uint32
        L.or_bwt_sa.argtypes = [c.c_void_p, c.c_void_p, c.c_uint32, c.c_uint32, c.c_void_p]
        L.or_sa2seq_batch.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint32, c.c_int64,
                                      c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p]
        _lib = L
    return _lib


class Bwt:
    """An index loaded by the restatement of bwt_restore_bwt (bwtio.c:51)."""

    def __init__(self, path=None, primary=None, L2=None, words=None):
        L = lib()
        if path is not None:
            self.h = L.or_bwt_load(path.encode())
            if not self.h:
                raise IOError(path)
            self._keep = None
        else:
            self._keep = np.ascontiguousarray(words, dtype=np.uint32)
            arr = (ctypes.c_uint32 * 4)(*[int(x) for x in L2])
            self.h = L.or_bwt_wrap(int(primary), arr, self._keep.ctypes.data, self._keep.size)

    def info(self):
        p, n = ctypes.c_uint32(), ctypes.c_uint32()
        lib().or_bwt_info(self.h, ctypes.byref(p), ctypes.byref(n))
        return p.value, n.value

    def primary(self):
        return self.info()[0]

    def seq_len(self):
        return self.info()[1]

    def load_sa(self, path):
        """bwt_restore_sa (bwtio.c:29-49): keeps sa[0..n_sa) (sa[0] = -1) and sa_intv on this index."""
        intv, n = ctypes.c_uint32(), ctypes.c_uint64()
        p = lib().or_sa_load(path.encode(), self.h, ctypes.byref(intv), ctypes.byref(n))
        if not p:
            raise IOError(path)
        self.sa = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)), shape=(n.value,)).copy()
        lib().or_free(p)
        self.sa_intv = intv.value
        return self

    def set_sa(self, sa, intv):
        self.sa = np.ascontiguousarray(sa, dtype=np.uint32)
        self.sa_intv = int(intv)
        return self

    def bwt_sa(self, k):
        """bwt_sa (bwt.c:69-79)"""
        return lib().or_bwt_sa(self.h, self.sa.ctypes.data, self.sa_intv, k & 0xFFFFFFFF, None)

    def occ4(self, k):
        out = (ctypes.c_uint32 * 4)()
        lib().or_occ4(self.h, k & 0xFFFFFFFF, out)
        return tuple(out)

    def __del__(self):
        try:
            lib().or_bwt_free(self.h)
        except Exception:
            pass


def sa2seq(bwt0, bwt1, strand, k, lens, steps=False):
    """bwtdb_sa2seq (dbset.c:240-246, db offset 0) over arrays; both indexes need load_sa/set_sa.
    steps=True also returns the LF-walk length of each row (bwt_sa's loop, bwt.c:72-75)."""
    strand = np.ascontiguousarray(strand, dtype=np.uint8)
    k = np.ascontiguousarray(k, dtype=np.uint32)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    assert bwt0.sa_intv == bwt1.sa_intv
    pos = np.empty(k.size, dtype=np.uint64)
    st = np.zeros(k.size, dtype=np.uint32) if steps else None
    lib().or_sa2seq_batch(bwt0.h, bwt0.sa.ctypes.data, bwt1.h, bwt1.sa.ctypes.data, bwt0.sa_intv, k.size,
                          strand.ctypes.data, k.ctypes.data, lens.ctypes.data, pos.ctypes.data,
                          st.ctypes.data if steps else None)
    return (pos, st) if steps else pos


def read_sa2pos_vectors(path):
    """tests/golden/sa2pos_vectors.tsv -> (strand, k, len, bwt_sa, pos) arrays"""
    a = np.loadtxt(path, dtype=np.uint64, comments="#", ndmin=2)
    return (a[:, 0].astype(np.uint8), a[:, 1].astype(np.uint32), a[:, 2].astype(np.uint32),
            a[:, 3].astype(np.uint32), a[:, 4])


def default_opt():
    o = GapOpt()
    lib().or_gap_init_opt(ctypes.byref(o))
    return o


def parse_aln_args(argv):
    """Restates bwa_aln's getopt loop (bwtaln.c:249-284).  Returns (opt, rest)."""
    import getopt
    o = default_opt()
    opte = -1
    opts, rest = getopt.getopt(argv, "n:o:e:i:d:l:k:cLR:m:t:NM:O:E:q:f:b012IB:")
    for k, v in opts:
        if k == "-n":
            if "." in v:
                o.fnr, o.max_diff = float(v), -1
            else:
                o.max_diff, o.fnr = int(v), -1.0
        elif k == "-o": o.max_gapo = int(v)
        elif k == "-e": opte = int(v)
        elif k == "-M": o.s_mm = int(v)
        elif k == "-O": o.s_gapo = int(v)
        elif k == "-E": o.s_gape = int(v)
        elif k == "-d": o.max_del_occ = int(v)
        elif k == "-i": o.indel_end_skip = int(v)
        elif k == "-l": o.seed_len = int(v)
        elif k == "-k": o.max_seed_diff = int(v)
        elif k == "-m": o.max_entries = int(v)
        elif k == "-t": o.n_threads = int(v)
        elif k == "-L": o.mode |= MODE_LOGGAP
        elif k == "-R": o.max_top2 = int(v)
        elif k == "-q": o.trim_qual = int(v)
        elif k == "-c": o.mode &= ~MODE_COMPREAD
        elif k == "-N": o.mode |= MODE_NONSTOP; o.max_top2 = 0x7fffffff
        elif k == "-b": o.mode |= MODE_BAM
        elif k == "-0": o.mode |= MODE_BAM_SE
        elif k == "-1": o.mode |= MODE_BAM_READ1
        elif k == "-2": o.mode |= MODE_BAM_READ2
        elif k == "-I": o.mode |= MODE_IL13
        elif k == "-B": o.mode |= int(v) << 24
    if opte > 0:
        o.max_gape = opte
        o.mode &= ~MODE_GAPE
    return o, rest


_NT4 = np.full(256, 4, dtype=np.uint8)
for _c, _v in zip(b"ACGTacgt", [0, 1, 2, 3, 0, 1, 2, 3]):
    _NT4[_c] = _v
_NT4[ord("-")] = 5  # bntseq.c:39-56


def read_fastq_records(path):
    """Minimal kseq_read (kseq.h:156): name = first token, seq/qual printable chars."""
    recs = []
    with open(path, "rb") as f:
        lines = f.read().split(b"\n")
    i = 0
    while i < len(lines):
        h = lines[i]
        if not h or h[:1] not in (b"@", b">"):
            i += 1
            continue
        name = h[1:].split()[0].decode()
        seq = lines[i + 1].strip()
        qual = b""
        i += 2
        if i < len(lines) and lines[i][:1] == b"+":
            qual = lines[i + 1].strip()
            i += 2
        recs.append((name, seq, qual))
    return recs


def encode_reads(recs, mode, trim_qual):
    """Restates bwa_read_seq (bwaseqio.c:145-208) for FASTQ input.

    Returns (seq_concat uint8, offsets uint64, lens uint32): seq is the
    bwa_seq_t.seq array -- codes of the (trimmed) read, reversed.
    """
    is_64 = mode & MODE_IL13
    l_bc = (mode >> 24) & 0xff
    out, offs, lens = [], [], []
    off = 0
    for name, seq, qual in recs:
        if is_64 and qual:
            qual = bytes(q - 31 for q in qual)
        if len(seq) <= l_bc:
            continue
        if l_bc:
            seq = seq[l_bc:]
            if qual:
                qual = qual[l_bc:]
        codes = _NT4[np.frombuffer(seq, dtype=np.uint8)]
        L = len(codes)
        if qual and trim_qual >= 1:  # bwa_trim_read (bwaseqio.c:74-87)
            s = mx = 0
            max_l = L - 1
            for l in range(L - 1, 35 - 2, -1):  # l >= BWA_MIN_RDLEN - 1
                s += trim_qual - (qual[l] - 33)
                if s < 0:
                    break
                if s > mx:
                    mx, max_l = s, l
            L = max_l + 1
        out.append(codes[:L][::-1].copy())
        offs.append(off)
        lens.append(L)
        off += L
    seqs = np.concatenate(out) if out else np.zeros(0, np.uint8)
    return seqs, np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint32)


STATS_DTYPE = np.dtype([("pushes", "<u4"), ("pops", "<u4"), ("peak_entries", "<u4"), ("peak_bucket", "<u4"),
                        ("n_aln", "<u4"), ("touches", "<u4"), ("peak_real", "<u4"), ("tails", "<u4"),
                        ("tail_steps", "<u4"), ("pruned_m", "<u4"), ("pruned_w", "<u4"), ("expansions", "<u4"),
                        ("hits", "<u4"), ("distinct_exp", "<u4"), ("chains", "<u4"), ("rounds", "<u4"),
                        ("rounds_g4", "<u4"), ("rounds_g16", "<u4"), ("rounds_lvl", "<u4")])


def cal_sa_reg_gap(bwt0, bwt1, seqs, offs, lens, opt, n_threads=1, touches=False, stats=None, width_touches=None,
                   split_pops=None, split_touches=None):
    """Run the restated bwa_cal_sa_reg_gap.  Returns (n_aln int32[n], alns ALN_DTYPE[...], touches).
    `stats`: optional STATS_DTYPE[n] array filled with per-read search statistics.
    `width_touches`: optional uint32[n] array filled with the touches of each read's bwt_cal_width
    calls (bwtaln.c:123-130) alone; touches - width_touches are bwt_match_gap's.
    `split_pops` / `split_touches`: optional uint32[n] arrays; split_touches[r] gets the touches counted
    before pop split_pops[r] + 1 of read r (its total if split_pops[r] is 0 or never reached) -- the
    GPU first pass's share of a read that left its resume state after that many pops."""
    L = lib()
    n = len(lens)
    if split_pops is not None:
        assert split_pops.dtype == np.uint32 and split_pops.size >= n and split_pops.flags.c_contiguous
        assert split_touches.dtype == np.uint32 and split_touches.size >= n and split_touches.flags.c_contiguous
        L.or_set_touch_split(ctypes.c_void_p(split_pops.ctypes.data), ctypes.c_void_p(split_touches.ctypes.data))
    if width_touches is not None:
        assert width_touches.dtype == np.uint32 and width_touches.size >= n and width_touches.flags.c_contiguous
        L.or_set_width_touches(ctypes.c_void_p(width_touches.ctypes.data))
    if stats is not None:
        assert stats.dtype == STATS_DTYPE and stats.size >= n and stats.flags.c_contiguous
        L.or_set_stats(ctypes.c_void_p(stats.ctypes.data))
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    n_aln = np.zeros(n, dtype=np.int32)
    tch = np.zeros(n, dtype=np.uint32) if touches else None
    ptr = ctypes.c_void_p()
    tot = L.or_cal_sa_reg_gap(bwt0.h, bwt1.h, n, seqs.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                              ctypes.byref(opt), n_threads, n_aln.ctypes.data, ctypes.byref(ptr),
                              tch.ctypes.data if touches else None)
    buf = ctypes.string_at(ptr.value, max(tot, 0) * 16)
    L.or_free(ptr)
    alns = np.frombuffer(buf, dtype=ALN_DTYPE).copy()
    return n_aln, alns, tch


PUSH_KINDS = ("root", "ins_open", "del_open", "ins_ext", "del_ext", "mismatch", "match")


def push_kinds(reset=False):
    """Instrumentation: {kind: (pushes, pops, expansions)} summed over the restated bwt_match_gap
    calls since the last reset (which this call does after reading, with reset=True)."""
    L = lib()
    out = np.zeros(3 * len(PUSH_KINDS), dtype=np.uint64)
    L.or_push_kinds(out.ctypes.data)
    if reset:
        L.or_push_kinds_reset()
    n = len(PUSH_KINDS)
    return {k: (int(out[i]), int(out[n + i]), int(out[2 * n + i])) for i, k in enumerate(PUSH_KINDS)}


DEP_N = 64


def depth_hist(reset=False):
    """Instrumentation: by depth d (BWT steps from the root; the last bin holds d >= DEP_N - 1) the
    expansions (one bwt_2occ4 each), the pops and the exact-tail steps (one bwt_2occ each) of the
    restated bwt_match_gap calls since the last push_kinds(reset=True) (or this call's reset)."""
    L = lib()
    out = np.zeros(4 * DEP_N + 3, dtype=np.uint64)
    L.or_depth_hist(out.ctypes.data)
    if reset:
        L.or_push_kinds_reset()
    return {"expansions": out[:DEP_N].copy(), "pops": out[DEP_N:2 * DEP_N].copy(),
            "tail_steps": out[2 * DEP_N:3 * DEP_N].copy(), "match_child_pops": out[3 * DEP_N:4 * DEP_N].copy(),
            "unique_pops": int(out[4 * DEP_N]), "unique_match_child_pops": int(out[4 * DEP_N + 1]),
            "unique_tail_steps": int(out[4 * DEP_N + 2])}


def exact_touches(bwt0, bwt1, seqs, offs, lens, mode, K=0, jump=False):
    """Per-read touches of the exact-match path (max_diff == 0) the GPU runs; with a
    K-mer table the first K steps of a chain count as one (table) touch; with `jump`
    the rest of a chain whose interval is one row costs SA + text (+ ISA on a match)."""
    seqs = np.ascontiguousarray(seqs, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    out = np.zeros(lens.size, dtype=np.uint32)
    lib().or_exact_touches(bwt0.h, bwt1.h, lens.size, seqs.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                           int(mode), int(K), int(bool(jump)), out.ctypes.data)
    return out


def sai_bytes(opt, n_aln, alns, batch=0x40000):
    """bwtaln.c:192,227-231: 64 B gap_opt_t header, then per read int32 n_aln + n_aln x 16 B."""
    parts = [bytes(opt)]
    p = 0
    for n in n_aln:
        parts.append(struct.pack("<i", int(n)))
        if n:
            parts.append(alns[p:p + n].tobytes())
            p += n
    return b"".join(parts)


def sai_body_equal(a, b):
    """Compare .sai files, masking header bytes 52..55 (gap_opt_t.n_threads)."""
    return a[:52] == b[:52] and a[56:64] == b[56:64] and a[64:] == b[64:]


class PathT(ctypes.Structure):
    """path_t (stdaln.h:97-101)."""
    _fields_ = [("i", ctypes.c_int), ("j", ctypes.c_int), ("ctype", ctypes.c_ubyte)]


def sw_local(ref_codes, read_codes):
    """aln_local_core(ref, read, aln_param_bwa, thres 1) restated (stdaln.c:529) + path2cigar32.
    Returns (score, path_len, (start_i, start_j), (end_i, end_j), cigar string) -- the fields of
    tests/golden/sw_vectors.tsv; start/end/cigar are None without a path."""
    L = lib()
    a = np.ascontiguousarray(ref_codes, dtype=np.uint8)
    b = np.ascontiguousarray(read_codes, dtype=np.uint8)
    path = (PathT * (a.size + b.size + 2))()
    pl = ctypes.c_int(0)
    sc = L.or_aln_local_core(a.ctypes.data, a.size, b.ctypes.data, b.size, path, ctypes.byref(pl), 1, None)
    if sc < 0 or pl.value == 0:
        return sc, pl.value, None, None, None
    cig = (ctypes.c_uint32 * (pl.value + 1))()
    n = L.or_path2cigar32(path, pl.value, cig)
    cs = "".join(f"{cig[k] >> 4}{'MIDS'[cig[k] & 0xf]}" for k in range(n))
    return sc, pl.value, (path[pl.value - 1].i, path[pl.value - 1].j), (path[0].i, path[0].j), cs


def read_sw_vectors(path):
    """tests/golden/sw_vectors.tsv -> list of (ref, read, score, path_len, start, end, cigar)."""
    out = []
    for line in open(path):
        if line.startswith("#"):
            continue
        f = line.rstrip("\n").split("\t")
        start = tuple(map(int, f[4].split(","))) if f[4] else None
        end = tuple(map(int, f[5].split(","))) if f[5] else None
        out.append((f[0], f[1], int(f[2]), int(f[3]), start, end, f[6] or None))
    return out


def nt4(s):
    """nst_nt4_table (bntseq.c:39-56) over a str."""
    return _NT4[np.frombuffer(s.encode(), dtype=np.uint8)] if s else np.zeros(0, np.uint8)


def sw_core(read, window, reglen, beg, l_pac):
    """bwa_sw_core (bwasw.c:29-112) restated over sw_local: None when rejected, else
    (beg, [bwa_cigar_t op << 29 | len ...], cnt = n_mm << 16 | n_gapo << 8 | n_gape)."""
    read = np.asarray(read, np.uint8)
    window = np.asarray(window, np.uint8)
    L = read.size
    if reglen < 20 or l_pac - beg < L:
        return None
    x = int((read >= 4).sum())
    if L == 0 or np.float32(x) / np.float32(L) >= np.float32(0.25) or L - x < 20:
        return None
    score, pl, start, end, cig = sw_local(window, read)
    if score < 0 or not cig:
        return None
    import re
    ops = [(int(n), "MIDS".index(t)) for n, t in re.findall(r"(\d+)([MIDS])", cig)]
    xx = sum(n for n, t in ops if t in (0, 2))
    yy = sum(n for n, t in ops if t in (0, 1))
    if xx < 20 or yy < 20:
        return None
    c = [t << 29 | n for n, t in ops]
    beg += (start[0] or 1) - 1
    st = (start[1] or 1) - 1
    if st:
        c.insert(0, 3 << 29 | st)
    if end[1] < L:
        c.append(3 << 29 | (L - end[1]))
    n_mm = n_gapo = n_gape = 0
    rx = start[0] - 1 if start[0] else 0
    ry = start[1] - 1 if start[1] else 0
    for v in c:
        t, n = v >> 29, v & 0x1FFFFFFF
        if t == 0:
            a, b = window[rx:rx + n], read[ry:ry + n]
            n_mm += int(((a < 4) & (b < 4) & (a != b)).sum())
            rx += n
            ry += n
        elif t == 2:
            rx += n
            n_gapo += 1
            n_gape += n - 1
        elif t == 1:
            ry += n
            n_gapo += 1
            n_gape += n - 1
    return beg, c, n_mm << 16 | n_gapo << 8 | n_gape


# ---------------------------------------------------------------- bwa_paired_sw

PSW_IN = ("read", "strand", "type", "mapQ", "seQ", "extra_flag", "n_mm", "n_gapo", "n_gape", "pos")
PSW_OUT = ("type", "strand", "pos", "remapped_pos", "dbidx", "remapped_dbidx", "mapQ", "seQ", "n_mm", "n_gapo",
           "n_gape", "extra_flag", "n_cigar", "cigar")


def read_psw(golden_dir, name):
    """tests/golden/psw_<name>.{in,out}.tsv -> (pairs, expected): lists of [end0, end1] dicts."""
    def parse(line, keys):
        out = []
        for half in line.rstrip("\n").split("\t"):
            f = half.split()
            d = {}
            for k, v in zip(keys, f):
                d[k] = v if k in ("read", "cigar") else int(v)
            out.append(d)
        return out
    pin = [parse(l, PSW_IN) for l in open(os.path.join(golden_dir, f"psw_{name}.in.tsv")) if l.strip()]
    pout = [parse(l, PSW_OUT) for l in open(os.path.join(golden_dir, f"psw_{name}.out.tsv")) if l.strip()]
    return pin, pout


def read_pac(prefix):
    """The packed reference (bntseq.c bns_dump / bns_pac, 4 bases per byte MSB first) unpacked
    to one code per base, and l_pac from the .ann header (bntseq.c:100)."""
    with open(prefix + ".ann") as f:
        l_pac = int(f.readline().split()[0])
    raw = np.fromfile(prefix + ".pac", dtype=np.uint8)
    codes = np.stack([(raw >> 6) & 3, (raw >> 4) & 3, (raw >> 2) & 3, raw & 3], axis=1).reshape(-1)
    return codes[:l_pac].copy(), l_pac


def _seq_rev(x, comp):
    """seq_reverse (bwaseqio.c:55-72)"""
    y = x[::-1].copy()
    if comp:
        m = y < 4
        y[m] = 3 - y[m]
    return y


def paired_sw(pairs, pe_type, avg, std, ap_prior, pac, l_pac):
    """bwa_paired_sw / bwa_paired_sw_thread (bwasw.c:145-304) restated over the ends of
    read_psw (db offset 0, one database): mutates the end dicts like the reference mutates
    bwa_seq_t (type, pos, strand, mapQ, seQ, n_mm/gapo/gape, extra_flag, cigar) and returns
    the counters [mated singletons, singletons, fixed, discordant] of its stderr summary."""
    import math
    SAM_FPP, NO_MATCH, MATESW, STD, SOLID = 2, 0, 3, 1, 2
    n_tot, n_mapped = [0, 0], [0, 0]
    for p in pairs:
        for e in p:
            e.setdefault("remapped_pos", e["pos"])
            e.setdefault("dbidx", 0)
            e.setdefault("remapped_dbidx", 0)
            e.setdefault("cigar_list", [])
            c = nt4(e["read"])
            e["_seq"] = _seq_rev(c, False)   # bwa_seq_t.seq (bwaseqio.c:191)
            e["_rseq"] = _seq_rev(c, True)   # bwa_seq_t.rseq (bwaseqio.c:192)
        if not ((p[0]["mapQ"] >= 17 or p[1]["mapQ"] >= 17) and (p[0]["extra_flag"] & SAM_FPP) == 0):
            continue
        mq_adjust = [255, 255]
        single = 1 if (p[0]["type"] == NO_MATCH or p[1]["type"] == NO_MATCH) else 0
        n_tot[single] += 1
        cig, beg, cnt = [None, None], [0, 0], [0, 0]
        if pe_type not in (STD, SOLID):
            continue
        for k in (0, 1):
            ref, mate = p[1 - k], p[k]
            if ref["type"] == NO_MATCH:
                continue
            L = len(mate["read"])

            def right():  # set_right_coordinate (bwasw.c:114-129), double arithmetic then truncation
                b = int(ref["remapped_pos"] + avg - 3 * std - L * 1.5)
                e = int(b + 6 * std + 2 * L)
                if b < ref["remapped_pos"] + len(ref["read"]):
                    b = ref["remapped_pos"] + len(ref["read"])
                if e > l_pac:
                    e = l_pac
                return b, e

            def left():  # set_left_coordinate (bwasw.c:131-143)
                b = int(ref["remapped_pos"] + len(ref["read"]) - avg - 3 * std - L * 0.5)
                e = int(b + 6 * std + 2 * L)
                if b < 0:
                    b = 0
                if e > ref["remapped_pos"]:
                    e = ref["remapped_pos"]
                return b, e
            if pe_type == STD:
                if ref["strand"] == 0:
                    b, e = right()
                    seq = mate["_rseq"]
                else:
                    b, e = left()
                    seq = _seq_rev(mate["_seq"], False)
            else:
                if ref["strand"] == 0:
                    b, e = left() if k == 0 else right()
                    seq = _seq_rev(mate["_rseq"], False)
                else:
                    b, e = right() if k == 0 else left()
                    seq = mate["_seq"]
            beg[k] = b
            reglen = int(np.int32(e - b))
            win = pac[b:b + reglen] if 0 <= b < l_pac and reglen > 0 else np.zeros(0, np.uint8)
            r = sw_core(seq, win, reglen, b, l_pac)
            if r is not None:
                beg[k], cig[k], cnt[k] = r
            if cig[k] is not None and mate["type"] != NO_MATCH:  # bwasw.c:222-236
                clip = 0
                if cig[k][0] >> 29 == 3:
                    clip += cig[k][0] & 0x1FFFFFFF
                if cig[k][-1] >> 29 == 3:
                    clip += cig[k][-1] & 0x1FFFFFFF
                s_old = int((mate["n_mm"] * 9 + mate["n_gapo"] * 13 + mate["n_gape"] * 2) / 3. * 8. + .499)
                s_new = int(((cnt[k] >> 16) * 9 + (cnt[k] >> 8 & 0xff) * 13 + (cnt[k] & 0xff) * 2 + clip * 3)
                            / 3. * 8. + .499)
                s_old = int(s_old + -4.343 * math.log(ap_prior / l_pac))
                s_new += int(-4.343 * math.log(.5 * math.erfc(math.sqrt(0.5) * 1.5) + .499))
                if s_old < s_new:
                    mq_adjust[k] = s_new - s_old
                    cig[k] = None
                else:
                    mq_adjust[k] = s_old - s_new
        k, mapQ = -1, 0
        if cig[0] is not None and cig[1] is not None:
            k = 0 if p[0]["mapQ"] < p[1]["mapQ"] else 1
            mapQ = abs(p[1]["mapQ"] - p[0]["mapQ"])
        elif cig[0] is not None:
            k, mapQ = 0, p[1]["mapQ"]
        elif cig[1] is not None:
            k, mapQ = 1, p[0]["mapQ"]
        if k >= 0 and p[k]["pos"] != beg[k]:
            n_mapped[single] += 1
            fx, rf = p[k], p[1 - k]
            tmp = rf["mapQ"] - fx["mapQ"] // 2 - 8
            if tmp <= 0:
                tmp = 1
            if mapQ > tmp:
                mapQ = tmp
            fx["mapQ"] = rf["mapQ"] = mapQ & 0xff
            sq = rf["seQ"] if rf["seQ"] < mapQ else mapQ
            fx["seQ"] = rf["seQ"] = sq & 0xff
            if fx["mapQ"] > mq_adjust[k]:
                fx["mapQ"] = mq_adjust[k] & 0xff
            if fx["seQ"] > mq_adjust[k]:
                fx["seQ"] = mq_adjust[k] & 0xff
            fx["cigar_list"] = cig[k]
            # __set_fixed (bwasw.c:167-178)
            fx["type"] = MATESW
            fx["pos"] = fx["remapped_pos"] = beg[k]
            fx["dbidx"] = fx["remapped_dbidx"] = 0
            fx["seQ"] = rf["seQ"]
            fx["strand"] = 1 - rf["strand"] if pe_type == STD else rf["strand"]
            fx["n_mm"], fx["n_gapo"], fx["n_gape"] = (cnt[k] >> 16) & 0xff, cnt[k] >> 8 & 0xff, cnt[k] & 0xff
            fx["extra_flag"] |= SAM_FPP
            rf["extra_flag"] |= SAM_FPP
    return [n_mapped[1], n_tot[1], n_mapped[0], n_tot[0]]


def psw_row(e):
    """an end in the field order of psw_<set>.out.tsv"""
    cg = e.get("cigar_list") or []
    cs = "".join(f"{v & 0x1FFFFFFF}{'MIDS'[v >> 29]}" for v in cg) or "*"
    return (e["type"], e["strand"], e["pos"], e.get("remapped_pos", e["pos"]), e.get("dbidx", 0),
            e.get("remapped_dbidx", 0), e["mapQ"], e["seQ"], e["n_mm"], e["n_gapo"], e["n_gape"], e["extra_flag"],
            len(cg), cs)


def global_core(ref_codes, read_codes, band=50, gap_end=5):
    """aln_global_core (stdaln.c:345-525) restated, aln_param_bwa scores, + path -> CIGAR.
    Returns (score, path_len, cigar str) -- the fields of tests/golden/gsw_vectors.tsv."""
    L = lib()
    if not hasattr(L.or_aln_global_core, "_typed"):
        L.or_aln_global_core.restype = ctypes.c_int
        L.or_aln_global_core.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.or_aln_global_core._typed = True
    a = np.ascontiguousarray(ref_codes, dtype=np.uint8)
    b = np.ascontiguousarray(read_codes, dtype=np.uint8)
    path = (PathT * (a.size + b.size + 2))()
    pl = ctypes.c_int(0)
    sc = L.or_aln_global_core(a.ctypes.data, a.size, b.ctypes.data, b.size, band, gap_end, path, ctypes.byref(pl))
    if pl.value <= 0:
        return sc, pl.value, ""
    cig = (ctypes.c_uint32 * (pl.value + 1))()
    n = L.or_path2cigar32(path, pl.value, cig)
    return sc, pl.value, "".join(f"{cig[k] >> 4}{'MIDS'[cig[k] & 0xf]}" for k in range(n))


def read_gsw_vectors(path):
    """tests/golden/gsw_vectors.tsv -> list of (ref, read, score, path_len, cigar)"""
    out = []
    for line in open(path):
        if line.startswith("#"):
            continue
        f = line.rstrip("\n").split("\t")
        out.append((f[0], f[1], int(f[2]), int(f[3]), f[4] if len(f) > 4 else ""))
    return out
