"""The POSIX 48-bit generators restated in the host code -- Drand48 and Lrand48 of sam_common.h
(samse/sampe hit choice, bwase.c:43-46 / bwape.c:317-319, seeded from .ann; the index's N fill,
bns_fasta2bntseq bntseq.c:224) -- against glibc's own drand48 / lrand48 on this host.  CPU only:
a small C++ program is compiled from the repo's headers."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = r'''
#include <stdio.h>
#include "sam_common.h"
int main(int argc, char **argv) {
  const long seed = atol(argv[1]);
  ibwa_sam::Drand48 d;
  d.seed(seed);
  for (int i = 0; i < 1000; ++i) printf("%.17g\n", d.next());
  ibwa_sam::Lrand48 l;
  l.seed(seed);
  for (int i = 0; i < 1000; ++i) printf("%ld\n", l.next());
  return 0;
}
'''


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    d = tmp_path_factory.mktemp("rng")
    src = d / "rng.cpp"
    src.write_text(SRC)
    exe = str(d / "rng")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I",
                    os.path.join(ROOT, "ibwa_amd", "csrc"), str(src), "-o", exe, "-lz", "-pthread"], check=True)
    return exe


@pytest.mark.parametrize("seed", [11, 0, 1, 12345, 2 ** 31 - 1])
def test_drand48_lrand48_match_glibc(prog, seed):
    libc = ctypes.CDLL("libc.so.6")
    libc.drand48.restype = ctypes.c_double
    libc.lrand48.restype = ctypes.c_long
    libc.srand48(ctypes.c_long(seed))
    want_d = [libc.drand48() for _ in range(1000)]
    libc.srand48(ctypes.c_long(seed))
    want_l = [libc.lrand48() for _ in range(1000)]
    out = subprocess.run([prog, str(seed)], check=True, capture_output=True, text=True).stdout.split()
    got_d = [float(x) for x in out[:1000]]
    got_l = [int(x) for x in out[1000:]]
    assert got_d == want_d
    assert got_l == want_l
