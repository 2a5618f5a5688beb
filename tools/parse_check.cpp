// parse_check.cpp -- CPU check of the CLI's bulk FASTQ parser (readers.h FastqBulk) against the
// serial kseq-semantics reader (SeqReader::read): both read <file> (FASTQ/FASTA, .gz or plain)
// and print one line per record "<seq>\t<qual>" (bulk records first, then the serial reader
// from where the bulk parser stopped), so the two outputs must be identical.
// usage: parse_check serial|bulk|serialcount|bulkcount <file> [chunk_bytes] [threads]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../ibwa_amd/csrc/readers.h"

int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: parse_check serial|bulk <file> [chunk_bytes] [threads]\n");
    return 2;
  }
  ibwa_cli::SeqReader rd;
  if (!rd.open(argv[2])) return 2;
  const bool bulk = strncmp(argv[1], "bulk", 4) == 0;
  const bool quiet = strstr(argv[1], "count") != nullptr;  // timing: a checksum instead of the records
  unsigned long long sum = 0;
  long n = 0;
  if (bulk) {
    ibwa_cli::FastqBulk fb(rd);
    if (argc > 3) fb.chunk = (size_t)atoll(argv[3]);
    const int nt = argc > 4 ? atoi(argv[4]) : 4;
    auto par = [](int k, const std::function<void(int)> &g) {
      std::vector<std::thread> th;
      for (int t = 1; t < k; ++t) th.emplace_back(g, t);
      g(0);
      for (auto &x : th) x.join();
    };
    while (fb.more(nt, par)) {
      for (; fb.qi < fb.recs.size(); ++fb.qi, ++n) {
        const auto &r = fb.recs[fb.qi];
        if (quiet) {
          sum = sum * 31 + r.len + (unsigned char)fb.blk[r.s] + (unsigned char)fb.blk[r.q + r.len - 1];
          continue;
        }
        fwrite(fb.blk.data() + r.s, 1, r.len, stdout);
        fputc('\t', stdout);
        fwrite(fb.blk.data() + r.q, 1, r.len, stdout);
        fputc('\n', stdout);
      }
    }
    fprintf(stderr, "bulk records %ld, serial from byte offset of the rest\n", n);
  }
  int l;
  while ((l = rd.read()) >= 0) {
    ++n;
    if (quiet) {
      sum = sum * 31 + (unsigned)l + (unsigned char)rd.seq[0] + (unsigned char)rd.qual.back();
      continue;
    }
    printf("%s\t%s\n", rd.seq.c_str(), rd.qual.c_str());
  }
  printf("#end %d records %ld\n", l, n);
  if (quiet) printf("#sum %llu\n", sum);
  return 0;
}
