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
        _lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _declare(_lib)
    return _lib


def _declare(L):
    c = ctypes
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
    L.ibwa_encode_reads_fixed.restype = None
    L.ibwa_encode_reads_fixed.argtypes = [c.c_void_p, c.c_uint64, c.c_int, c.c_void_p, c.c_void_p, c.c_void_p,
                                          c.c_int]
