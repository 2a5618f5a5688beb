// host_check.cpp -- the CLI's host-only code (readers.h, sam_common.h) driven without a GPU, for
// the sanitizer builds of tests/test_host_sanitizers.py (ASan/UBSan and TSan on the
// host code; the GPU code is not instrumented).
//
//   host_check reads <file> <mode> <trim_qual> [bam_which]
//       next_read (bwa_read_seq / bwa_read_bam, bwaseqio.c:89-208) over the whole input, parsed on a
//       Background thread one batch ahead, as the CLIs do; every read printed as an unmapped SAM
//       line by print_parallel (parallel_chunks over the host threads).  Exit 3 on a truncated
//       or corrupt record (BamReader::read() == -2).
//   host_check bns <prefix>
//       bns_restore (.ann/.amb/.pac), then coor_pac2real / pac_at over a grid of positions.
//   host_check chunks <n> <threads>
//       parallel_chunks coverage: every index visited exactly once.
//   host_check remap < cases
//       remap.h (the -R remapping of sampe) on one case per line, one result line each:
//         H <header>                               read_mapping_extract
//         R <cigar> <pos> <seqlen>                 remap_cigar
//         I <cigar> <exact> <start> <len>          is_remapped_sequence_identical
//         T <cigar> <start> <read cigar|-> <len>   translate_cigar (read CIGAR as text, - for none)
//         L <file> <n_seqs>                        load_remappings
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <string>
#include <vector>

#include "readers.h"
#include "sam_common.h"
#include "remap.h"

using namespace ibwa_sam;

namespace {

template <class Reader>
int drain(Reader &rd, int mode, int trim) {
  const int kBatch = 1000;  // small batches: many hand-overs between the parser and the printer
  Out o{stdout, {}};
  Dbs none;  // unmapped reads only: no reference is consulted
  std::vector<Read> cur, nxt;
  bool done = false;  // the reader has ended (end of input or a bad record): do not read on
  auto fill = [&](std::vector<Read> &b) {
    b.clear();
    Read r;
    while (!done && (int)b.size() < kBatch) {
      if (!next_read(rd, mode, trim, r)) done = true;
      else b.push_back(std::move(r));
    }
  };
  fill(cur);
  while (!cur.empty()) {
    Background bg;
    bg.start([&]() { fill(nxt); });
    print_parallel(o, (int64_t)cur.size(), [&](Out &ob, int64_t i) { print_sam1(ob, none, cur[i], nullptr, mode, 30, nullptr); });
    bg.wait();
    cur.swap(nxt);
  }
  o.flush();
  fflush(stdout);
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  init_tables();
  if (argc >= 5 && !strcmp(argv[1], "reads")) {
    const int mode = atoi(argv[3]), trim = atoi(argv[4]);
    if (argc >= 6) {
      ibwa_cli::BamReader rd;
      if (!rd.open(argv[2], atoi(argv[5]))) return 2;
      drain(rd, mode, trim);
      // next_read stops at -1 (end) and -2 (truncated); tell them apart
      return rd.last == -2 ? 3 : 0;
    }
    ibwa_cli::SeqReader rd;
    if (!rd.open(argv[2])) return 2;
    return drain(rd, mode, trim);
  }
  if (argc >= 3 && !strcmp(argv[1], "bns")) {
    Bns b;
    if (!bns_restore(argv[2], b)) return 2;
    uint64_t h = 1469598103934665603ull;
    for (int64_t x = 0; x < b.l_pac; x += 997) {
      int32_t id = -1;
      const int nn = coor_pac2real(b, x, 50, &id);
      h = (h ^ (uint64_t)(pac_at(b, (uint64_t)x) + 4 * id + 64 * nn)) * 1099511628211ull;
    }
    printf("%lld %zu %zu %016llx\n", (long long)b.l_pac, b.anns.size(), b.ambs.size(), (unsigned long long)h);
    return 0;
  }
  if (argc >= 4 && !strcmp(argv[1], "chunks")) {
    const int64_t n = atoll(argv[2]);
    std::vector<std::atomic<int>> seen(n);
    for (auto &x : seen) x = 0;
    parallel_chunks(n, [&](int64_t lo, int64_t hi, int) {
      for (int64_t i = lo; i < hi; ++i) seen[i]++;
    }, atoi(argv[3]));
    for (int64_t i = 0; i < n; ++i)
      if (seen[i] != 1) return 1;
    printf("ok %lld\n", (long long)n);
    return 0;
  }
  if (argc >= 2 && !strcmp(argv[1], "remap")) {
    char buf[4096];
    while (fgets(buf, sizeof buf, stdin)) {
      char kind = buf[0], a[1024] = "", b[1024] = "", c[1024] = "";
      long x = 0, y = 0, z = 0;
      if (kind == 'H' && sscanf(buf + 2, "%1023[^\n]", a) >= 0) {
        Mapping m;
        if (read_mapping_extract(a, m)) printf("%s %d %u %u\n", m.seqname.c_str(), m.exact, m.start, m.stop);
        else printf("fail\n");
      } else if (kind == 'R' && sscanf(buf + 2, "%1023s %ld %ld", a, &x, &y) == 3) {
        uint32_t r = 0;
        const int ok = remap_cigar(a[0] == '-' ? "" : a, &r, (uint32_t)x, (uint32_t)y);
        if (ok) printf("%u\n", r);
        else printf("fail\n");
      } else if (kind == 'I' && sscanf(buf + 2, "%1023s %ld %ld %ld", a, &x, &y, &z) == 4) {
        Mapping m;
        m.cigar = a[0] == '-' ? "" : a;
        m.exact = (int)x;
        printf("%d\n", is_remapped_sequence_identical(m, (uint32_t)y, (uint32_t)z));
      } else if (kind == 'T' && sscanf(buf + 2, "%1023s %ld %1023s %ld", a, &x, b, &y) == 4) {
        std::vector<uint32_t> rc;  // the read CIGAR as bwa_cigar_t runs, then one zero run of slack
        for (const char *p = b; *p && *p != '-';) {
          char *e;
          const uint32_t n = (uint32_t)strtoul(p, &e, 10);
          rc.push_back((uint32_t)(strchr("MIDSN", *e) - "MIDSN") << 29 | n);
          p = e + 1;
        }
        const int n_rc = (int)rc.size();
        rc.push_back(0);
        std::vector<uint32_t> out;
        if (!translate_cigar(a[0] == '-' ? std::string() : std::string(a), (uint32_t)x, b[0] == '-' ? nullptr : rc.data(),
                             n_rc, (int)y, out)) {
          printf("fail\n");
        } else {
          for (uint32_t v : out) printf("%u%c", v & 0x1fffffffu, "MIDSN"[v >> 29]);
          printf("\n");
        }
      } else if (kind == 'L' && sscanf(buf + 2, "%1023s %ld", c, &x) == 2) {
        std::vector<std::unique_ptr<Mapping>> maps;
        const int rv = load_remappings(c, (int)x, maps);
        printf("%d", rv);
        if (rv == 1)
          for (auto &m : maps)
            if (m) printf(" [%s %d %u %u %s %d]", m->seqname.c_str(), m->exact, m->start, m->stop, m->cigar.c_str(), m->n_gapo);
            else printf(" []");
        printf("\n");
      } else {
        printf("?\n");
      }
    }
    return 0;
  }
  fprintf(stderr, "usage: host_check reads <file> <mode> <trim> [bam_which] | bns <prefix> | chunks <n> <threads>\n");
  return 1;
}
