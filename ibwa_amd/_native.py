"""Loader for the in-tree native library ``ibwa_amd/lib/libibwa_amd.so``.

The library is built by ``__graft_entry__.build()`` (hipcc, gfx950).  There is
no fallback: if it is missing, importing the compute API raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# IBWA_LIB: another build of the same library (same-box A/B measurements in tools/)
LIB_PATH = os.environ.get("IBWA_LIB") or os.path.join(_HERE, "lib", "libibwa_amd.so")
BIN_PATH = os.path.join(_HERE, "bin", "ibwa-amd")
_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def lib():
    """Return the loaded ctypes handle (raises NativeLibraryMissing if absent)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _declare(L)
        if not os.environ.get("IBWA_LIB"):
            check_build_id(L)
        _lib = L
    return _lib


def source_digest():
    """The digest the Makefile bakes into ibwa_build_id(), from the sources in this tree
    (None when the sources are not next to the library)."""
    import glob
    import hashlib
    csrc = os.path.join(_HERE, "csrc")
    inc = os.path.join(os.path.dirname(_HERE), "include")
    if not os.path.isdir(csrc):
        return None
    files = sorted((f for pat in ("*.cpp", "*.h", "*.hip") for f in glob.glob(os.path.join(csrc, pat))),
                   key=lambda f: os.path.basename(f).encode())
    files += sorted(glob.glob(os.path.join(inc, "*.h")), key=lambda f: os.path.basename(f).encode())
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def check_build_id(L):
    """Refuse a library built from other sources than the ones in this tree (a stale prebuilt
    .so shipped to a GPU box)."""
    want = source_digest()
    got = L.ibwa_build_id().decode()
    if want is not None and got != want:
        raise NativeLibraryMissing(
            f"{LIB_PATH} was built from other sources (build id {got}, sources {want}); rebuild with "
            "`python -c 'import __graft_entry__ as g; g.build()'`")


def _declare(L):
    c = ctypes
    L.ibwa_build_id.restype = c.c_char_p
    L.ibwa_build_id.argtypes = []
    u64p = c.POINTER(c.c_uint64)
    L.ibwa_synth_grch37_lengths.restype = c.c_uint64
    L.ibwa_synth_grch37_lengths.argtypes = [c.c_uint64, c.c_uint64, u64p]
    L.ibwa_synth_genome.restype = None
    L.ibwa_synth_genome.argtypes = [c.c_uint64, c.c_int, u64p, c.c_double, c.c_double, c.c_int,
                                    c.c_void_p, c.c_int]
    L.ibwa_pack_nt4.restype = c.c_uint64
    L.ibwa_pack_nt4.argtypes = [c.c_void_p, c.c_uint64, c.c_void_p]
    L.ibwa_synth_reads.restype = None
    L.ibwa_synth_reads.argtypes = [c.c_uint64, c.c_void_p, c.c_uint64, c.c_int, u64p, c.c_uint64,
                                   c.c_int, c.c_double, c.c_double, c.c_void_p, c.c_void_p,
                                   c.c_void_p, c.c_int]
    declare_host_helpers(L)


def declare_host_helpers(L):
    c = ctypes
    L.ibwa_pack_nt4_mt.restype = c.c_uint64
    L.ibwa_pack_nt4_mt.argtypes = [c.c_void_p, c.c_uint64, c.c_void_p, c.c_int]
    L.ibwa_synth_write_fastq.restype = c.c_int
    L.ibwa_synth_write_fastq.argtypes = [c.c_char_p, c.c_void_p, c.c_uint64, c.c_uint64, c.c_int, c.c_int]
    L.ibwa_synth_write_fastq_gz.restype = c.c_int
    L.ibwa_synth_write_fastq_gz.argtypes = [c.c_char_p, c.c_void_p, c.c_uint64, c.c_uint64, c.c_int, c.c_int, c.c_int,
                                            c.c_int, c.c_int]
    L.ibwa_sai_diff.restype = c.c_int64
    L.ibwa_sai_diff.argtypes = [c.c_char_p, c.c_uint64, c.c_void_p, c.c_void_p]
    L.ibwa_encode_reads_fixed.restype = None
    L.ibwa_encode_reads_fixed.argtypes = [c.c_void_p, c.c_uint64, c.c_int, c.c_void_p, c.c_void_p, c.c_void_p,
                                          c.c_int]
