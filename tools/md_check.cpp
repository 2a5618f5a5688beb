// md_check.cpp -- CPU check of sam_common.h cal_md1 (bwa_cal_md1, bwase.c:243-295) against a
// base-by-base restatement of the same function: random references (one or several), reads with
// substitutions and N's, with and without a CIGAR (M / I / D / S runs), at random positions
// including windows that run past the end of the packed reference.
// usage: md_check <seed>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <string>
#include <vector>

#include "sam_common.h"

using namespace ibwa_sam;

// bwa_cal_md1 base by base (the restatement cal_md1 replaced)
static std::string slow_md(const Read &s, uint64_t pos, const uint8_t *seq, const Dbs &b, int *nm_out) {
  std::string str;
  uint64_t x = pos, y = 0;
  int u = 0, nm = 0;
  uint8_t c = 0;
  auto base = [&](uint64_t at, bool &ok) -> uint8_t {
    uint8_t o = 0;
    ok = at < b.l_pac && extract(b, at, 1, &o) == 1;
    return o;
  };
  if (s.has_cigar) {
    for (uint32_t cg : s.cigar) {
      const int l = (int)cig_len(cg);
      const uint32_t op = cig_op(cg);
      if (op == FROM_M) {
        for (int z = 0; z < l; ++z) {
          bool ok;
          const uint8_t r = base(x + z, ok);
          if (!ok) break;
          c = r;
          if (c > 3 || seq[y + z] > 3 || c != seq[y + z]) {
            str += std::to_string(u);
            str += "ACGTN"[c];
            ++nm;
            u = 0;
          } else {
            ++u;
          }
        }
        x += l; y += l;
      } else if (op == FROM_I || op == FROM_S) {
        y += l;
        if (op == FROM_I) nm += l;
      } else if (op == FROM_D) {
        str += std::to_string(u);
        str += '^';
        for (int z = 0; z < l; ++z) {
          bool ok;
          const uint8_t r = base(x + z, ok);
          if (!ok) break;
          c = r;
          str += "ACGT"[c];
        }
        u = 0;
        x += l; nm += l;
      }
    }
  } else {
    for (int z = 0; z < s.len; ++z) {
      bool ok;
      const uint8_t r = base(x + z, ok);
      if (ok) c = r;
      if (c > 3 || seq[y + z] > 3 || c != seq[y + z]) {
        str += std::to_string(u);
        str += "ACGTN"[c];
        ++nm;
        u = 0;
      } else {
        ++u;
      }
    }
  }
  str += std::to_string(u);
  *nm_out = nm;
  return str;
}

int main(int argc, char **argv) {
  std::mt19937_64 g(argc > 1 ? strtoull(argv[1], nullptr, 10) : 1);
  for (int refs = 1; refs <= 3; ++refs) {
    Dbs d;
    d.db.resize(refs);
    for (int r = 0; r < refs; ++r) {
      RefDb &x = d.db[r];
      x.bns.l_pac = 200 + (int64_t)(g() % 2000);
      x.bns.pac.resize(x.bns.l_pac / 4 + 1);
      for (auto &c : x.bns.pac) c = (uint8_t)g();
      x.offset = d.l_pac;
      d.l_pac += (uint64_t)x.bns.l_pac;
    }
    for (int k = 0; k < 20000; ++k) {
      Read s;
      s.len = 1 + (int)(g() % 180);
      const uint64_t pos = g() % (d.l_pac + 30);
      // the read: the reference there (where there is one) with substitutions and N's
      std::vector<uint8_t> ref(s.len + 64, 0);
      extract(d, pos, (uint32_t)s.len, ref.data());
      s.seq.resize(s.len);
      for (int z = 0; z < s.len; ++z) {
        const uint64_t r = g() % 100;
        s.seq[z] = r < 3 ? (uint8_t)(g() % 4) : r < 4 ? 4 : ref[z];
      }
      if (g() % 2) {
        // a CIGAR whose read length is s.len: M / I / D / S runs
        int left = s.len;
        while (left > 0) {
          const uint32_t op = (uint32_t)(g() % 6);
          const int l = 1 + (int)(g() % std::max(1, std::min(left, 40)));
          if (op == 2) { s.cigar.push_back(cig_make(FROM_D, (uint32_t)l)); continue; }
          const uint32_t o = op == 3 ? FROM_I : op == 4 ? FROM_S : FROM_M;
          const int ll = std::min(l, left);
          s.cigar.push_back(cig_make(o, (uint32_t)ll));
          left -= ll;
        }
        s.has_cigar = true;
      }
      int nm1 = 0, nm2 = 0;
      const std::string a = cal_md1(s, pos, s.seq.data(), d, &nm1), b = slow_md(s, pos, s.seq.data(), d, &nm2);
      if (a != b || nm1 != nm2) {
        printf("refs %d read %d (len %d, pos %llu, cigar %d): '%s' nm %d vs '%s' nm %d\n", refs, k, s.len,
               (unsigned long long)pos, (int)s.has_cigar, a.c_str(), nm1, b.c_str(), nm2);
        return 1;
      }
    }
  }
  printf("OK\n");
  return 0;
}
