// gz_check.cpp -- CPU harness for gzsrc.h (tests/test_gzsrc.py).
//   gz_check stream <file> <read size>    ByteStream reads of <read size> bytes to stdout
//   gz_check source <file> <cap>          GzSource::read in <cap>-byte calls to stdout; "failed at N"
//                                          or "eof at N" on stderr
//   gz_check gzread <file> <read size>    zlib's gzread (the reference's reader) to stdout
//   gz_check bench <file> [cap]           inflate the whole file with GzSource: GB/s on stderr
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../ibwa_amd/csrc/gzsrc.h"

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  const char *mode = argv[1], *fn = argv[2];
  const uint64_t sz = argc > 3 ? strtoull(argv[3], nullptr, 10) : (64u << 20);
  std::vector<uint8_t> buf(sz ? sz : 1);
  if (!strcmp(mode, "stream")) {
    ibwa_cli::ByteStream in;
    if (!in.open(fn)) return 1;
    for (;;) {
      const int64_t r = in.read(buf.data(), sz);
      if (r < 0) { fprintf(stderr, "error\n"); break; }
      if (r == 0) break;
      fwrite(buf.data(), 1, (size_t)r, stdout);
    }
    return 0;
  }
  if (!strcmp(mode, "gzread")) {
    gzFile f = gzopen(fn, "r");
    if (!f) return 1;
    for (;;) {
      const int r = gzread(f, buf.data(), (unsigned)sz);
      if (r < 0) { fprintf(stderr, "error\n"); break; }
      if (r == 0) break;
      fwrite(buf.data(), 1, (size_t)r, stdout);
    }
    gzclose(f);
    return 0;
  }
  if (!strcmp(mode, "source") || !strcmp(mode, "bench")) {
    ibwa_cli::GzSource s;
    if (!s.open(fn)) return 1;
    const bool bench = !strcmp(mode, "bench");
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t tot = 0;
    while (!s.eof() && !s.failed()) {
      const uint64_t r = s.read(buf.data(), sz);
      tot += r;
      if (!bench) fwrite(buf.data(), 1, (size_t)r, stdout);
    }
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "%s at %llu\n", s.failed() ? "failed" : "eof", (unsigned long long)s.offset());
    if (bench)
      fprintf(stderr, "%s%s: %.3f GB in %.3f s = %.2f GB/s inflated (%.3f GB compressed, hint %.3f GB)\n",
              s.bgzf() ? "bgzf" : "gzip", "", tot / 1e9, sec, tot / 1e9 / sec, s.compressed_size() / 1e9,
              s.size_hint() / 1e9);
    return 0;
  }
  return 2;
}
