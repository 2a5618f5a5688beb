// readers.h -- read input of the CLI commands (aln_main.cpp, samse_main.cpp): FASTQ/FASTA
// (.gz) with kseq_read's record semantics and unaligned BAM with bwa_read_bam's selection.
#pragma once
#include <ctype.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <string>
#include <vector>

namespace ibwa_cli {

// Buffered gz reader with the record semantics of kseq_read (kseq.h:156-195).
struct SeqReader {
  gzFile fp = nullptr;
  std::vector<char> buf = std::vector<char>(1 << 20);
  int begin = 0, end = 0;
  bool eof = false;
  int last_char = 0;
  std::string name, seq, qual;
  // kseq's comment buffer (index): once allocated it keeps the last comment read, and a header
  // without one leaves it as it was (kseq_read only resets its length)
  bool keep_comment = false, comment_alloc = false;
  std::string comment;

  bool open(const char *fn) {
    fp = strcmp(fn, "-") ? gzopen(fn, "r") : gzdopen(fileno(stdin), "r");
    if (fp) gzbuffer(fp, 1 << 20);
    return fp != nullptr;
  }
  ~SeqReader() {
    if (fp) gzclose(fp);
  }
  int getc_() {
    if (!fill()) return -1;
    return (unsigned char)buf[begin++];
  }
  bool fill() {
    if (begin < end) return true;
    if (eof) return false;
    end = gzread(fp, buf.data(), (unsigned)buf.size());
    begin = 0;
    if (end <= 0) { eof = true; end = 0; return false; }
    return true;
  }
  // byte classes for the sequence scan: 0 skipped (not isgraph), 1 kept, 2 ends the sequence
  static const uint8_t *seq_class() {
    static uint8_t t[256];
    static bool init = false;
    if (!init) {
      for (int c = 0; c < 256; ++c) t[c] = isgraph(c) ? 1 : 0;
      t[(int)'>'] = t[(int)'+'] = t[(int)'@'] = 2;
      init = true;
    }
    return t;
  }
  // returns seq length, -1 at EOF, -2 on a truncated quality string.  Byte-for-byte the loops of
  // kseq_read, run over the buffer in bulk (runs of kept bytes are appended at once).
  int read() {
    int c = -1;
    if (last_char == 0) {  // jump to the next header line
      for (;;) {
        if (!fill()) return -1;
        const char *p = buf.data() + begin, *e = buf.data() + end, *q = p;
        while (q < e && *q != '>' && *q != '@') ++q;
        if (q < e) { last_char = (unsigned char)*q; begin = (int)(q + 1 - buf.data()); break; }
        begin = end;
      }
    }
    name.clear(); seq.clear(); qual.clear();
    bool got = false;
    for (;;) {  // name: up to the first isspace
      if (!fill()) { c = -1; break; }
      const char *p = buf.data() + begin, *e = buf.data() + end, *q = p;
      while (q < e && !isspace((unsigned char)*q)) ++q;
      if (q > p) { name.append(p, q); got = true; }
      if (q < e) { c = (unsigned char)*q; begin = (int)(q + 1 - buf.data()); break; }
      begin = end;
    }
    if (c == -1 && !got) return -1;
    if (c != '\n' && c != -1) {  // comment: the rest of the line
      if (keep_comment) { comment.clear(); comment_alloc = true; }
      for (;;) {
        if (!fill()) { c = -1; break; }
        const char *p = buf.data() + begin, *e = buf.data() + end;
        const char *q = (const char *)memchr(p, '\n', (size_t)(e - p));
        if (keep_comment) comment.append(p, q ? q : e);
        if (q) { c = '\n'; begin = (int)(q + 1 - buf.data()); break; }
        begin = end;
      }
    }
    const uint8_t *cls = seq_class();
    c = -1;
    for (;;) {  // sequence: kept bytes up to '>', '+' or '@'
      if (!fill()) break;
      const unsigned char *p = (const unsigned char *)buf.data() + begin, *e = (const unsigned char *)buf.data() + end;
      bool stop = false;
      while (p < e) {
        const unsigned char *q = p;
        while (q < e && cls[*q] == 1) ++q;
        if (q > p) seq.append((const char *)p, (const char *)q);
        if (q == e) { p = q; break; }
        if (cls[*q] == 2) { c = *q; p = q + 1; stop = true; break; }
        p = q + 1;
      }
      begin = (int)((const char *)p - buf.data());
      if (stop) break;
    }
    if (c == '>' || c == '@') last_char = c;
    if (c != '+') return (int)seq.size();
    for (;;) {  // the rest of the '+' line
      if (!fill()) return -2;
      const char *p = buf.data() + begin, *e = buf.data() + end;
      const char *q = (const char *)memchr(p, '\n', (size_t)(e - p));
      if (q) { begin = (int)(q + 1 - buf.data()); break; }
      begin = end;
    }
    // quality: bytes 33..127 until it is as long as the sequence; like kseq, the byte read when
    // it is full is consumed too
    for (;;) {
      if (!fill()) break;
      const unsigned char *p = (const unsigned char *)buf.data() + begin, *e = (const unsigned char *)buf.data() + end;
      bool done = false;
      while (p < e) {
        if (qual.size() >= seq.size()) { ++p; done = true; break; }
        const size_t need = seq.size() - qual.size();
        const unsigned char *q = p;
        while (q < e && (size_t)(q - p) < need && *q >= 33 && *q <= 127) ++q;
        if (q > p) { qual.append((const char *)p, (const char *)q); p = q; continue; }
        ++p;  // a byte outside 33..127 is consumed and dropped
      }
      begin = (int)((const char *)p - buf.data());
      if (done) break;
    }
    last_char = 0;
    if (seq.size() != qual.size()) return -2;
    return (int)seq.size();
  }
};

// BAM input: bam_header_read / bam_read1 (bamlite.c:34-116) over gzread (a BGZF file is a
// series of gzip members), and the record selection and decoding of bwa_read_bam
// (bwaseqio.c:89-143): `which` bit 1 = read 1, 2 = read 2, 4 = neither (bwtaln.c:159-171);
// 4-bit bases -> A/C/G/T/N, reverse-strand records reverse-complemented back, qualities
// +33 capped at 126.  The record is handed on as FASTQ-like strings.
struct BamReader {
  gzFile fp = nullptr;
  int which = 7;
  std::string name, seq, qual;
  std::vector<uint8_t> data;
  bool readn(void *p, int n) { return gzread(fp, p, (unsigned)n) == n; }
  bool open(const char *fn, int w) {
    which = w;
    fp = strcmp(fn, "-") ? gzopen(fn, "r") : gzdopen(fileno(stdin), "r");
    if (!fp) return false;
    gzbuffer(fp, 1 << 20);
    char magic[4];
    if (!readn(magic, 4) || memcmp(magic, "BAM\1", 4) != 0) {
      fprintf(stderr, "[bam_header_read] invalid BAM binary header (this is not a BAM file).\n");
      return false;
    }
    int32_t l_text = 0, n_ref = 0;
    if (!readn(&l_text, 4)) return false;
    std::vector<char> text(l_text > 0 ? l_text : 0);
    if (l_text > 0 && !readn(text.data(), l_text)) return false;
    if (!readn(&n_ref, 4)) return false;
    for (int32_t i = 0; i < n_ref; ++i) {
      int32_t l_name = 0;
      uint32_t l_ref = 0;
      if (!readn(&l_name, 4) || l_name < 0) return false;
      std::vector<char> nm(l_name);
      if ((l_name && !readn(nm.data(), l_name)) || !readn(&l_ref, 4)) return false;
    }
    return true;
  }
  ~BamReader() {
    if (fp) gzclose(fp);
  }
  int last = 0;  // what the last read() returned
  // seq length of the next selected record, -1 at EOF, -2 on a truncated or corrupt record
  int read() { return last = read_record(); }
  int read_record() {
    static const char nt16[] = "NACNGNNNTNNNNNNN";  // bam_nt16_nt4_table (bwaseqio.c:11) as bases
    for (;;) {
      int32_t block_len = 0;
      const int got = gzread(fp, &block_len, 4);
      if (got == 0) return -1;
      if (got != 4 || block_len < 32) return -2;
      uint32_t x[8];
      if (!readn(x, 32)) return -2;
      const int l_qname = x[2] & 0xff, flag = x[3] >> 16, n_cigar = x[3] & 0xffff, l_qseq = (int)x[4];
      data.resize(block_len - 32);
      if (!data.empty() && !readn(data.data(), (int)data.size())) return -2;
      int go = 0;
      if ((which & 1) && (flag & 0x40)) go = 1;
      if ((which & 2) && (flag & 0x80)) go = 1;
      if ((which & 4) && !(flag & 0x40) && !(flag & 0x80)) go = 1;
      if (!go) continue;
      // the variable-length fields must lie inside the record (a corrupt or truncated BAM
      // would otherwise be read past the block)
      if (l_qseq < 0 || (uint64_t)l_qname + 4ull * n_cigar + ((uint64_t)l_qseq + 1) / 2 + (uint64_t)l_qseq > data.size())
        return -2;
      const uint8_t *sq = data.data() + l_qname + 4 * n_cigar, *q = sq + (l_qseq + 1) / 2;
      name.assign((const char *)data.data(), strnlen((const char *)data.data(), (size_t)l_qname));
      seq.resize(l_qseq);
      qual.resize(l_qseq);
      for (int i = 0; i < l_qseq; ++i) {
        seq[i] = nt16[(sq[i >> 1] >> ((~i & 1) << 2)) & 0xf];
        qual[i] = (char)(q[i] + 33 < 126 ? q[i] + 33 : 126);
      }
      if (flag & 0x10) {  // seq_reverse(len, seq, 1) / seq_reverse(len, qual, 0)
        std::reverse(seq.begin(), seq.end());
        std::reverse(qual.begin(), qual.end());
        for (auto &ch : seq) ch = ch == 'A' ? 'T' : ch == 'C' ? 'G' : ch == 'G' ? 'C' : ch == 'T' ? 'A' : ch;
      }
      return l_qseq;
    }
  }
};

}  // namespace ibwa_cli
