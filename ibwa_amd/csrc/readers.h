// readers.h -- read input of the CLI commands (aln_main.cpp, samse_main.cpp): FASTQ/FASTA
// (.gz) with kseq_read's record semantics and unaligned BAM with bwa_read_bam's selection.  Bytes
// come from a ByteStream (gzsrc.h): gzip files inflated on all host threads ahead of the parse,
// anything else through gzread as the reference reads it.
#pragma once
#include <ctype.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "gzsrc.h"

namespace ibwa_cli {

// Buffered reader with the record semantics of kseq_read (kseq.h:156-195).
struct SeqReader {
  ByteStream in;
  std::vector<char> buf = std::vector<char>(1 << 20);
  int begin = 0, end = 0;
  bool eof = false;
  int last_char = 0;
  std::string name, seq, qual;
  // kseq's comment buffer (index): once allocated it keeps the last comment read, and a header
  // without one leaves it as it was (kseq_read only resets its length)
  bool keep_comment = false, comment_alloc = false;
  std::string comment;

  bool open(const char *fn) { return in.open(fn); }
  int getc_() {
    if (!fill()) return -1;
    return (unsigned char)buf[begin++];
  }
  // bytes handed back by FastqBulk when it stops (read before the rest of the stream)
  std::vector<char> pending;
  size_t pend_pos = 0;
  bool fill() {
    if (begin < end) return true;
    if (pend_pos < pending.size()) {
      const size_t n = std::min(buf.size(), pending.size() - pend_pos);
      memcpy(buf.data(), pending.data() + pend_pos, n);
      pend_pos += n;
      begin = 0;
      end = (int)n;
      return true;
    }
    if (eof) return false;
    end = (int)in.read(buf.data(), buf.size());
    begin = 0;
    if (end <= 0) { eof = true; end = 0; return false; }
    return true;
  }
  // byte classes for the sequence scan: 0 skipped (not isgraph), 1 kept, 2 ends the sequence
  static const uint8_t *seq_class() {
    static const struct Tab {  // built once, thread-safely (readers run on several threads)
      uint8_t t[256];
      Tab() {
        for (int c = 0; c < 256; ++c) t[c] = isgraph(c) ? 1 : 0;
        t[(int)'>'] = t[(int)'+'] = t[(int)'@'] = 2;
      }
    } tab;
    return tab.t;
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

// Strict 4-line FASTQ in bulk (aln's input in the common case).  Whole records -- "@header\n", a
// line of sequence bytes (isgraph, none of '>', '+', '@'), a line starting with '+', a line of
// quality bytes 33..127 exactly as long as the sequence -- are split and checked by several
// threads over a large block.  On such a record kseq_read (SeqReader::read) returns exactly that
// sequence and quality and stops right after the quality line's newline.  At the first record
// of any other shape (FASTA, multi-line, CRLF, a short or long quality line, a truncated tail)
// the rest of the input goes to the serial reader, whose state there -- after a record's last
// byte, looking for the next '@' or '>' -- is the one kseq_read would be in.
struct FastqBulk {
  struct Rec {
    uint64_t h, s, q;  // offsets of the header (its '@'), the sequence and the quality lines in blk
    uint32_t len;
  };
  SeqReader &rd;
  struct Buf {  // raw bytes, not zero-filled, kept across blocks (no page faults after the first)
    std::unique_ptr<char[]> p;
    size_t cap = 0;
    char *data() const { return p.get(); }
    const char &operator[](size_t i) const { return p[i]; }
  } blk;
  size_t pos = 0, end = 0;  // unparsed bytes [pos, end)
  bool eof = false;         // the stream is drained into blk
  bool on = true;           // false from the first record the bulk parser does not take
  bool handed = false;      // the rest went to the serial reader
  std::vector<Rec> recs;    // parsed, not yet taken
  size_t qi = 0;
  size_t chunk = (size_t)32 << 20;
  explicit FastqBulk(SeqReader &r) : rd(r) {}

  // bytes of the record at p (> 0), 0 when the data ends inside it, -1 when it is not strict
  static int64_t rec_at(const char *p, const char *e, bool at_eof, const char *base, Rec &r) {
    if (p >= e) return 0;
    if (*p != '@') return -1;
    const char *h = (const char *)memchr(p, '\n', (size_t)(e - p));
    if (!h) return at_eof ? -1 : 0;
    const char *sq = h + 1;
    const char *se = (const char *)memchr(sq, '\n', (size_t)(e - sq));
    if (!se) return at_eof ? -1 : 0;
    const int64_t L = se - sq;
    if (L < 1 || L > (1 << 24)) return -1;
    // no exit per byte: the checks run branch-free over the line (and vectorise).  seq_class() == 1
    // is isgraph() in the C locale, 33..126, but for '>', '+' and '@'
    uint8_t bad = 0;
    for (const char *x = sq; x < se; ++x) {
      const uint8_t c = (uint8_t)*x;
      bad |= (uint8_t)((c < 33) | (c > 126) | (c == '>') | (c == '+') | (c == '@'));
    }
    if (bad) return -1;
    const char *pl = se + 1;
    if (pl >= e) return at_eof ? -1 : 0;
    if (*pl != '+') return -1;
    const char *pe = (const char *)memchr(pl, '\n', (size_t)(e - pl));
    if (!pe) return at_eof ? -1 : 0;
    const char *u = pe + 1;
    if (e - u < L + 1) return at_eof ? -1 : 0;
    uint8_t qbad = 0;
    for (int64_t k = 0; k < L; ++k) {
      const uint8_t c = (uint8_t)u[k];
      qbad |= (uint8_t)((c < 33) | (c > 127));
    }
    if (qbad) return -1;
    if (u[L] != '\n') return -1;
    r.h = (uint64_t)(p - base);
    r.s = (uint64_t)(sq - base);
    r.q = (uint64_t)(u - base);
    r.len = (uint32_t)L;
    return u + L + 1 - p;
  }
  // all taken: keep the unparsed tail, read the next block of the stream behind it
  void refill() {
    recs.clear();
    qi = 0;
    const size_t tail = end - pos;
    if (blk.cap < tail + chunk) {
      std::unique_ptr<char[]> q(new char[tail + chunk]);
      if (tail) memcpy(q.get(), blk.data() + pos, tail);
      blk.p.swap(q);
      blk.cap = tail + chunk;
    } else if (pos) {
      memmove(blk.data(), blk.data() + pos, tail);
    }
    pos = 0;
    end = tail;
    if (eof) return;
    while (end < blk.cap) {
      const size_t want = std::min<size_t>(blk.cap - end, (size_t)1 << 26);
      const int64_t got = rd.in.read(blk.data() + end, want);
      if (got <= 0) { eof = true; break; }
      end += (size_t)got;
    }
  }
  // the records of [pos, end), nt threads from record starts spread over the block
  template <class Par>
  void parse(int nt, Par par) {
    const char *base = blk.data(), *p0 = base + pos, *e = base + end;
    const size_t n = end - pos;
    if (!n) return;
    nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, n >> 20));
    std::vector<const char *> st(nt + 1, e);
    st[0] = p0;
    for (int t = 1; t < nt; ++t) {  // the first strict record at a line start after the split point
      const char *x = p0 + n * t / nt;
      st[t] = e;
      while (x < e) {
        const char *nl = (const char *)memchr(x, '\n', (size_t)(e - x));
        if (!nl) break;
        x = nl + 1;
        Rec r;
        if (x < e && *x == '@' && rec_at(x, e, eof, base, r) > 0) { st[t] = x; break; }
      }
      if (st[t] < st[t - 1]) st[t] = st[t - 1];
    }
    std::vector<std::vector<Rec>> out(nt);
    std::vector<const char *> stop(nt);
    std::vector<int> code(nt, 1);  // 1: reached the next start, 0: data ends, -1: not strict
    par(nt, [&](int t) {
      const char *p = st[t];
      while (p < st[t + 1]) {
        Rec r;
        const int64_t k = rec_at(p, e, eof, base, r);
        if (k <= 0) { code[t] = (int)k; break; }
        out[t].push_back(r);
        p += k;
      }
      stop[t] = p;
    });
    const char *P = p0;
    for (int t = 0; t < nt; ++t) {
      if (st[t] != P) break;  // the previous segment did not end on this start: parse on from P next time
      recs.insert(recs.end(), out[t].begin(), out[t].end());
      P = stop[t];
      if (code[t] < 0) { on = false; break; }
      if (code[t] == 0 || P != st[t + 1]) break;
    }
    pos = (size_t)(P - base);
  }
  // the serial reader continues at pos
  void handoff() {
    on = false;
    handed = true;
    rd.pending.assign(blk.data() + pos, blk.data() + end);
    rd.pend_pos = 0;
    rd.begin = rd.end = 0;
    rd.last_char = 0;
    rd.eof = false;  // pending first, then the stream (at its end if eof)
    blk.p.reset();
    blk.cap = 0;
    pos = end = 0;
  }
  // records available to take (parses the next block when all are taken); false: bulk is over
  template <class Par>
  bool more(int nt, Par par) {
    if (qi < recs.size()) return true;
    if (!on) {
      if (!handed) handoff();
      return false;
    }
    for (int tries = 0; tries < 4 && on; ++tries) {
      refill();
      parse(nt, par);
      if (!recs.empty()) return true;
      if (eof && pos == end) return false;  // the input is exhausted in bulk
      if (on && !eof) { chunk *= 2; continue; }  // a record longer than the block
      break;
    }
    handoff();
    return false;
  }
};

// BAM input: bam_header_read / bam_read1 (bamlite.c:34-116) over the inflated BGZF stream (a BGZF
// file is a series of gzip members: ByteStream inflates them on all threads), and the record
// selection and decoding of bwa_read_bam
// (bwaseqio.c:89-143): `which` bit 1 = read 1, 2 = read 2, 4 = neither (bwtaln.c:159-171);
// 4-bit bases -> A/C/G/T/N, reverse-strand records reverse-complemented back, qualities
// +33 capped at 126.  The record is handed on as FASTQ-like strings.
struct BamReader {
  ByteStream in;
  int which = 7;
  std::string name, seq, qual;
  std::vector<uint8_t> data;
  bool readn(void *p, int n) { return in.read(p, (uint64_t)n) == n; }
  bool open(const char *fn, int w) {
    which = w;
    if (!in.open(fn)) return false;
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
  int last = 0;  // what the last read() returned
  // seq length of the next selected record, -1 at EOF, -2 on a truncated or corrupt record
  int read() { return last = read_record(); }
  int read_record() {
    static const char nt16[] = "NACNGNNNTNNNNNNN";  // bam_nt16_nt4_table (bwaseqio.c:11) as bases
    for (;;) {
      int32_t block_len = 0;
      const int64_t got = in.read(&block_len, 4);
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
