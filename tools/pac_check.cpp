// pac_check.cpp -- CPU check of the .pac extraction samse/sampe use for MD/NM, refinement and
// mate-rescue windows (sam_common.h extract, dbset_extract_sequence dbset.c:306-325): the
// four-codes-per-byte unpacking against bns_pac base by base, for one reference and for several read
// back to back, at random starts and lengths including ranges that run past the end.
// usage: pac_check <seed> [time]
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <random>
#include <vector>

#include "sam_common.h"

using namespace ibwa_sam;

static uint32_t slow(const Dbs &d, uint64_t beg, uint32_t len, uint8_t *out) {
  uint32_t total = 0;
  while (total < len && beg < d.l_pac) {
    const RefDb &r = d.db[d.coord2idx((int64_t)beg)];
    uint64_t pos = beg - r.offset;
    while (pos < (uint64_t)r.bns.l_pac && total < len) out[total++] = pac_at(r.bns, pos++);
    beg = pos + r.offset;
  }
  return total;
}

int main(int argc, char **argv) {
  std::mt19937_64 g(argc > 1 ? strtoull(argv[1], nullptr, 10) : 1);
  if (argc > 2) {  // timing: 150-base windows at random in a 256 Mbp reference
    Bns b;
    b.l_pac = (int64_t)1 << 28;
    b.pac.resize(b.l_pac / 4 + 1);
    for (auto &x : b.pac) x = (uint8_t)g();
    std::vector<uint8_t> o(160);
    unsigned long long sum = 0;
    for (int pass = 0; pass < 2; ++pass) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < 2000000; ++k) {
        const uint64_t at = g() % (uint64_t)b.l_pac;
        uint32_t n;
        if (pass == 0) {
          n = 0;
          for (uint64_t x = at; n < 150 && x < (uint64_t)b.l_pac; ++x) o[n++] = pac_at(b, x);
        } else {
          n = extract(b, at, 150, o.data());
        }
        sum += o[0] + n;
      }
      printf("%s: %.1f ns per 150-base window (%llu)\n", pass ? "unpack" : "per base",
             std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 2e6 * 1e9, sum);
    }
    return 0;
  }
  for (int refs = 1; refs <= 3; ++refs) {
    Dbs d;
    d.db.resize(refs);
    for (int r = 0; r < refs; ++r) {
      RefDb &x = d.db[r];
      x.bns.l_pac = 1 + (int64_t)(g() % 700);
      x.bns.pac.resize(x.bns.l_pac / 4 + 1);
      for (auto &c : x.bns.pac) c = (uint8_t)g();
      x.offset = d.l_pac;
      d.l_pac += (uint64_t)x.bns.l_pac;
    }
    std::vector<uint8_t> a(1200), b(1200);
    for (int k = 0; k < 20000; ++k) {
      const uint64_t beg = g() % (d.l_pac + 20);
      const uint32_t len = (uint32_t)(g() % 1100);
      const uint32_t na = extract(d, beg, len, a.data()), nb = slow(d, beg, len, b.data());
      if (na != nb || memcmp(a.data(), b.data(), na)) {
        printf("refs %d beg %llu len %u: %u vs %u bases\n", refs, (unsigned long long)beg, len, na, nb);
        return 1;
      }
      if (refs == 1) {
        const RefDb &r = d.db[0];
        const uint32_t n1 = extract(r.bns, beg, len, a.data());
        uint32_t n2 = 0;
        for (uint64_t x = beg; n2 < len && x < (uint64_t)r.bns.l_pac; ++x) b[n2++] = pac_at(r.bns, x);
        if (n1 != n2 || memcmp(a.data(), b.data(), n1)) {
          printf("one reference, beg %llu len %u: %u vs %u bases\n", (unsigned long long)beg, len, n1, n2);
          return 1;
        }
      }
    }
  }
  printf("OK\n");
  return 0;
}
