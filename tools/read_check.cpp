// read_check.cpp -- CPU check of samse/sampe's read path (sam_common.h): batches taken by
// take_reads (the bulk FASTQ parser's records converted by rec_to_read on host threads, then the
// serial reader from the first record the bulk parser does not take) against next_read alone
// (bwa_read_seq, bwaseqio.c:145-208) record by record, as Read objects: name, sequence, quality,
// reverse complement, lengths and barcode.  The batch's buffers are reused from batch to batch as
// sampe's reader reuses them.
// usage: read_check <file> <mode> <trim_qual> <batch> <threads> [time]
//   mode: the .sai header's mode word (barcode length << 24 | IBWA_MODE_IL13 | IBWA_MODE_COMPREAD)
//   time: only the bulk path, timed: prints records/s
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "sam_common.h"

using namespace ibwa_sam;

static std::string dump(const Read &r) {
  std::string s = r.name + "\t";
  for (uint8_t c : r.seq) s += (char)('0' + c);
  s += "\t" + r.qual + "\t";
  for (uint8_t c : r.rseq) s += (char)('0' + c);
  s += "\t" + std::to_string(r.len) + "," + std::to_string(r.full_len) + "," + std::to_string(r.clip_len) + "," +
       std::to_string((int)r.has_qual) + "\t" + r.bc;
  return s;
}

int main(int argc, char **argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: read_check <file> <mode> <trim_qual> <batch> <threads> [time]\n");
    return 2;
  }
  init_tables();
  const int mode = (int)strtol(argv[2], nullptr, 0), trim = atoi(argv[3]);
  const size_t batch = (size_t)atoll(argv[4]);
  const int nt = atoi(argv[5]);
  const bool timed = argc > 6;
  ibwa_cli::SeqReader a;
  if (!a.open(argv[1])) return 2;
  ibwa_cli::FastqBulk fb(a);
  std::vector<Read> got;
  long n = 0;
  if (timed) {
    const auto t0 = std::chrono::steady_clock::now();
    unsigned long long sum = 0;
    for (;;) {
      take_reads(&fb, mode, trim, got, batch, nt, [&](Read &r) { return next_read(a, mode, trim, r); });
      if (got.empty()) break;
      for (const Read &r : got) sum = sum * 31 + (unsigned)r.len + r.seq[0];
      n += (long)got.size();
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("%ld records in %.3f s: %.2f M records/s (checksum %llu)\n", n, s, n / s * 1e-6, sum);
    return 0;
  }
  ibwa_cli::SeqReader b;
  if (!b.open(argv[1])) return 2;
  Read want;
  for (;;) {
    take_reads(&fb, mode, trim, got, batch, nt, [&](Read &r) { return next_read(a, mode, trim, r); });
    for (size_t i = 0; i < got.size(); ++i, ++n) {
      if (!next_read(b, mode, trim, want)) {
        printf("record %ld: the serial reader ended first\n", n);
        return 1;
      }
      const std::string x = dump(got[i]), y = dump(want);
      if (x != y) {
        printf("record %ld differs:\n batch  %s\n serial %s\n", n, x.c_str(), y.c_str());
        return 1;
      }
    }
    if (got.size() < batch) break;
  }
  if (next_read(b, mode, trim, want)) {
    printf("record %ld: the batches ended first\n", n);
    return 1;
  }
  printf("OK %ld\n", n);
  return 0;
}
