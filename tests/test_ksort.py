"""klib's ks_introsort as sampe restates it (ibwa_amd/csrc/ksort.h; the reference's klib
ksort.h:142-219) is not stable, and which of two equal positions find_optimal_pair sees first
follows from it (bwapair.c:188).  sampe_main.cpp sorts a pair's positions through 24-byte keys
(remapped_pos, pos, index) and gathers the records after: the permutation must be the one that
sorting the records themselves gives, ties included.  Checked here on the CPU by a small C++ driver
compiled against the header: many ties, all the size regimes (pairs, insertion sort, quicksort
partitions, the depth-limit combsort); and the LSD radix sort sampe uses when no two keys tie
(radix_sort_u64) against a stable sort."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r'''
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <random>
#include "ksort.h"
using namespace ibwa_sam;
struct Rec { uint64_t pos, rpos; uint32_t tag; int pad[9]; };
struct Key { uint64_t rp, p; uint32_t idx; };
int main() {
  std::mt19937_64 g(7);
  long bad = 0, cases = 0;
  for (int n : {1, 2, 3, 5, 16, 17, 33, 100, 1000, 5000, 70000}) {
    for (int rep = 0; rep < 20; ++rep) {
      const uint64_t span = rep % 4 == 0 ? 3 : rep % 4 == 1 ? 50 : rep % 4 == 2 ? 1000000 : 1;
      std::vector<Rec> a(n);
      for (int i = 0; i < n; ++i) {
        a[i].rpos = g() % span; a[i].pos = rep % 2 ? g() % 4 : a[i].rpos; a[i].tag = (uint32_t)i;
      }
      if (rep == 5) for (int i = 0; i < n; ++i) a[i].rpos = a[i].pos = (uint64_t)(n - i) / 3;  // descending runs
      std::vector<Rec> b = a;
      ks_introsort(a.size(), a.data(), [](const Rec &x, const Rec &y) {
        return x.rpos == y.rpos ? x.pos < y.pos : x.rpos < y.rpos; });
      std::vector<Key> k(n);
      for (int i = 0; i < n; ++i) k[i] = {b[i].rpos, b[i].pos, (uint32_t)i};
      ks_introsort(k.size(), k.data(), [](const Key &x, const Key &y) { return x.rp == y.rp ? x.p < y.p : x.rp < y.rp; });
      for (int i = 0; i < n; ++i) bad += b[k[i].idx].tag != a[i].tag;
      ++cases;
    }
  }
  // radix_sort_u64: a stable sort of the keys (payloads follow), any key range
  long rbad = 0;
  std::vector<uint64_t> tk;
  std::vector<uint32_t> tv;
  for (int n : {2, 3, 300, 5000, 100000}) {
    for (int rep = 0; rep < 6; ++rep) {
      const int sh = rep * 11;
      std::vector<uint64_t> k(n);
      std::vector<uint32_t> v(n);
      for (int i = 0; i < n; ++i) { k[i] = (g() % (rep % 2 ? 7 : 1000000)) << sh; v[i] = (uint32_t)i; }
      std::vector<std::pair<uint64_t, uint32_t>> e(n);
      for (int i = 0; i < n; ++i) e[i] = {k[i], v[i]};
      std::stable_sort(e.begin(), e.end(), [](const std::pair<uint64_t, uint32_t> &x, const std::pair<uint64_t, uint32_t> &y) {
        return x.first < y.first; });
      radix_sort_u64(n, k.data(), v.data(), tk, tv);
      for (int i = 0; i < n; ++i) rbad += k[i] != e[i].first || v[i] != e[i].second;
      ++cases;
    }
  }
  printf("%ld %ld\n", cases, bad + rbad);
  return bad + rbad != 0;
}
'''


def test_key_sort_permutation_equals_record_sort(tmp_path):
    src = tmp_path / "ks.cpp"
    src.write_text(DRIVER)
    exe = tmp_path / "ks"
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "ibwa_amd", "csrc"), str(src), "-o", str(exe)],
                       capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        pytest.fail(r.stderr[-2000:])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    cases, bad = map(int, r.stdout.split())
    assert cases == 250 and bad == 0
