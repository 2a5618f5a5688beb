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
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <string>
#include <vector>

#include "readers.h"
#include "sam_common.h"

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
  fprintf(stderr, "usage: host_check reads <file> <mode> <trim> [bam_which] | bns <prefix> | chunks <n> <threads>\n");
  return 1;
}
