// remap.h -- iBWA's compound-sequence remapping (`sampe -R`) and the multi-reference database set
// of `sampe <pri> <1.sai> <2.sai> <1.fq> <2.fq> [<alt> <a1.sai> <a2.sai> ...]`, host side:
//   * the .remap table of an alternate reference (load_remappings / read_mapping_extract,
//     bwaremap.cpp:42-127): per alternate sequence, its target sequence in the primary, the
//     1-based region it replaces (or `exact`) and the alt-vs-primary CIGAR;
//   * position projection (remap_cigar, bwa_remap_position[_with_seqid], bwaremap.cpp:170-311)
//     and the "identical remapping" test (is_remapped_sequence_identical, :129-168);
//   * CIGAR projection of a read aligned to an alternate sequence (translate_cigar,
//     translate_cigar.cpp:1-356);
//   * the database set: references concatenated at their offsets (dbset_restore, dbset.c:135-176),
//     coord2idx / dbset_extract_sequence / dbset_extract_remapped / dbset_coor_pac2real
//     (dbset.c:17-39, :248-325).
// Reference quirks are kept, including the fatal errors (message + abort, as err_fatal).
#ifndef IBWA_REMAP_H
#define IBWA_REMAP_H
#include <errno.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ibwa_sam {

[[noreturn]] inline void err_fatal(const char *header, const char *fmt, ...) {  // utils.c:67-76
  va_list args;
  va_start(args, fmt);
  fprintf(stderr, "[%s] ", header);
  vfprintf(stderr, fmt, args);
  fprintf(stderr, " Abort!\n");
  va_end(args);
  abort();
}

// read_mapping_t (bwaremap.h:10-17)
struct Mapping {
  std::string seqname;
  int exact = 0;
  uint32_t start = 0, stop = 0;
  std::string cigar;
  bool has_cigar = false;
  int n_gapo = 0;
};

// can_remap (bwaremap.cpp:17-26): exactly one '-' and two '|'
inline bool can_remap(const char *str) {
  int ndash = 0, npipe = 0;
  for (; *str; ++str) {
    if (*str == '-') ++ndash;
    if (*str == '|') ++npipe;
  }
  return ndash == 1 && npipe == 2;
}

// read_mapping_extract (bwaremap.cpp:102-141): "name-target|start|stop" or "name-target|exact..."
inline bool read_mapping_extract(const char *str, Mapping &m) {
  m.exact = 0;
  if (!can_remap(str)) return false;
  const char *beg = strchr(str, '-');
  if (!beg) return false;
  ++beg;
  const char *end = strchr(beg, '|');
  if (beg == end || !end) return false;
  m.seqname.assign(beg, end);
  beg = end + 1;
  if (strncmp("exact", beg, 5) == 0) {
    m.exact = 1;
    m.start = m.stop = 0;
    m.has_cigar = false;
    return true;
  }
  char *e = nullptr;
  m.start = (uint32_t)strtoul(beg, &e, 10);
  if (e == beg || *e != '|') return false;
  --m.start;
  beg = e + 1;
  m.stop = (uint32_t)strtoul(beg, &e, 10) + 1;  // one past the last base
  if (e == beg || *e != '\0') return false;
  return true;
}

// load_remappings (bwaremap.cpp:42-100): -1 error, 0 no file, 1 loaded.  Entries are assigned to
// the sequences in file order (the i-th entry is sequence i's mapping).  The std::getline /
// eof() loop is emulated exactly: a last header line without a newline is not read.
inline int load_remappings(const std::string &path, int n_seqs, std::vector<std::unique_ptr<Mapping>> &maps) {
  FILE *fp = fopen(path.c_str(), "r");
  if (!fp) {
    fprintf(stderr, "No remapping file %s: (%s)\n", path.c_str(), strerror(errno));
    return 0;
  }
  std::string data;
  {
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, fp)) > 0) data.append(buf, n);
    fclose(fp);
  }
  maps.clear();
  maps.resize(n_seqs);
  size_t at = 0;
  bool eofbit = false;
  auto getline = [&](std::string &out) -> bool {  // std::getline on an ifstream
    out.clear();
    if (at >= data.size()) {
      eofbit = true;
      return false;  // nothing extracted: failbit
    }
    const size_t e = data.find('\n', at);
    if (e == std::string::npos) {
      out = data.substr(at);
      at = data.size();
      eofbit = true;
      return true;
    }
    out = data.substr(at, e - at);
    at = e + 1;
    return true;
  };
  std::string line;
  if (!getline(line)) {
    fprintf(stderr, "Empty remapping file '%s'\n", path.c_str());
    return -1;
  }
  long lineNum = 0;
  int i = 0;
  while (!eofbit) {
    ++lineNum;
    const char c0 = line.empty() ? '\0' : line[0];
    if (c0 != '>') {
      fprintf(stderr, "Unexpected character '%c' at start of line %ld in file '%s'. Expected '>'.\n", c0, lineNum,
              path.c_str());
      return -1;
    }
    if (i >= n_seqs) {  // the reference writes past its array here
      fprintf(stderr, "More remappings than sequences in '%s'\n", path.c_str());
      return -1;
    }
    maps[i].reset(new Mapping);
    if (!read_mapping_extract(line.c_str() + 1, *maps[i])) {
      fprintf(stderr, "Failed to extract read mapping from string '%s' in file %s, line %ld\n", line.c_str() + 1,
              path.c_str(), lineNum);
      return -1;
    }
    std::string cigar;
    while (getline(line) && !(!line.empty() && line[0] == '>')) {
      ++lineNum;
      cigar += line;
    }
    maps[i]->cigar = cigar;  // also for `exact` entries (an empty string)
    maps[i]->has_cigar = true;
    ++lineNum;
    int go = 0;
    for (char ch : cigar) go += ch == 'I' || ch == 'D' || ch == 'N';  // cigar_gap_opens (bwaremap.cpp:28-36)
    maps[i]->n_gapo = go;
    ++i;
  }
  return 1;
}

// is_remapped_sequence_identical (bwaremap.cpp:129-168)
inline int is_remapped_sequence_identical(const Mapping &m, uint32_t start, uint32_t len) {
  uint32_t pos = 0, last_len = 0;
  const char *cigar = m.cigar.c_str();
  char last_op = 0;
  if (m.exact) return 1;
  while (pos <= start && *cigar) {
    char *end;
    last_len = (uint32_t)strtoul(cigar, &end, 10);
    if (end == cigar) {
      fprintf(stderr, "[remap_coordinates] expected number in cigar string '%s' at pos %ld\n", m.cigar.c_str(),
              (long)(cigar - m.cigar.c_str()));
      return 0;
    }
    cigar = end;
    last_op = *cigar;
    switch (last_op) {
      case 'M': case 'X': case '=': case 'N': case 'D': pos += last_len; break;
      case 'I': break;
      default: fprintf(stderr, "invalid cigar character '%c'\n", last_op); return 0;
    }
    cigar++;
  }
  if (pos > start) return (last_op == 'M' || last_op == '=') && last_len - start > len;
  if (pos == last_len) {
    fprintf(stderr, "failed to parse cigar string '%s'\n", m.cigar.c_str());
    return 0;
  }
  return 0;
}

// remap_cigar (bwaremap.cpp:170-238): the target offset of alternate position pos
inline int remap_cigar(const char *cigar, uint32_t *result, uint32_t pos, uint32_t seqlen) {
  const char *p = cigar;
  uint32_t altpos = 0, refpos = 0, last_len = 0;
  char last_op = 0;
  if (pos >= seqlen) {
    fprintf(stderr, "[remap_coordinates] requested pos %u > sequence length %u\n", pos, seqlen);
    return 0;
  }
  while (altpos <= pos && *p) {
    char *end;
    last_len = (uint32_t)strtoul(p, &end, 10);
    if (end == p) {
      fprintf(stderr, "[remap_coordinates] expected number in cigar string '%s' at pos %ld\n", cigar, (long)(p - cigar));
      return 0;
    }
    p = end;
    last_op = *p;
    switch (last_op) {
      case 'M': case 'X': case '=': refpos += last_len; altpos += last_len; break;
      case 'N': case 'D': refpos += last_len; break;
      case 'I': altpos += last_len; break;
      default: fprintf(stderr, "invalid cigar character '%c'\n", last_op); return 0;
    }
    p++;
  }
  if (altpos > seqlen) {
    fprintf(stderr, "[remap_coordinates] cigar '%s' string implies length > read mapping (%u vs %u)\n", cigar, altpos,
            seqlen);
    return 0;
  }
  if (altpos == pos) {
    *result = refpos;
    return 1;
  } else if (altpos > pos) {
    switch (last_op) {
      case 'M': case 'X': case '=': *result = refpos - (altpos - pos); break;
      case 'I': *result = refpos; break;
      default: fprintf(stderr, "Error remapping cigar string %s:, pos=%u\n", cigar, pos); return 0;
    }
  } else {
    fprintf(stderr, "failed to parse cigar string '%s'\n", cigar);
    return 0;
  }
  return 1;
}

// ---------------------------------------------------------------- translate_cigar (translate_cigar.cpp)
// A read's CIGAR against an alternate sequence (starting at `start` on it) composed with the
// alternate's CIGAR against the primary.  bwa_cigar_t: op << 29 | len, ops M I D S N = 0..4.
class CigarTranslator {
 public:
  CigarTranslator(const char *seq_cigar, uint32_t start_pos, const uint32_t *read_cigar, int n_cigar, int total_read_len)
      : seq_cigar_(seq_cigar), p_(seq_cigar), start_pos_(start_pos), rc_(read_cigar), n_(n_cigar),
        total_read_len_(total_read_len) {
    seq_advance();
    read_advance();
  }
  std::vector<uint32_t> out;

  void exec() {
    find_start_pos();
    if (!rc_) {
      int len = 0;
      while (len < total_read_len_ && !eos()) {
        const int dist = total_read_len_ - len;
        if (seq_len_ < dist) {
          push(tr_seqop(seq_op_), seq_len_);
          len += seq_len_;
          seq_advance();
        } else {
          push(tr_seqop(seq_op_), dist);
          break;
        }
      }
      return;
    }
    while (!eor() && !eos()) {
      if (seq_len_ == 0) seq_advance();
      if (read_len_ == 0) read_advance();
      if (OPS[read_op_] == 'S') {
        push(read_op_, read_len_);
        read_len_ = 0;
        if (!eor()) read_advance();
        continue;
      }
      switch (seq_op_) {
        case '=': case 'M': case 'X': in_match(); break;
        case 'I': in_insertion(); break;
        case 'N': case 'D': in_deletion(); break;
        default: throw std::runtime_error(std::string("Invalid cigar character: ") + seq_op_);
      }
    }
    while (!eor()) {
      if (read_len_ == 0) read_advance();
      if (OPS[read_op_] == 'M' || OPS[read_op_] == 'I' || OPS[read_op_] == 'S') push(tr_seqop('S'), read_len_);
      read_len_ = 0;
    }
  }

 private:
  static constexpr const char *OPS = "MIDSN";
  const char *seq_cigar_, *p_;
  uint32_t start_pos_;
  const uint32_t *rc_;
  int rci_ = 0, n_;
  int total_read_len_;
  uint32_t cpos_ = 0;
  char seq_op_ = 0;
  int seq_len_ = 0, read_op_ = 0, read_len_ = 0;

  void push(int op, int len) {  // CigarBuilder::push: merges a run with the previous one
    const uint32_t c = (uint32_t)op << 29 | (uint32_t)len;
    if (!out.empty() && (out.back() >> 29) == (uint32_t)op)
      out.back() = (uint32_t)op << 29 | ((out.back() & 0x1fffffffu) + (uint32_t)len);
    else
      out.push_back(c);
  }
  static int tr_seqop(char op) {
    switch (op) {
      case 'M': return 0;
      case 'I': return 1;
      case 'D': return 2;
      case 'S': return 3;
      case 'N': return 4;
      default: throw std::runtime_error(std::string("Unknown cigar operation: ") + op);
    }
  }
  void in_match() {
    switch (OPS[read_op_]) {
      case 'M': case 'N': case 'D':
        if (seq_len_ >= read_len_) {
          push(read_op_, read_len_);
          seq_len_ -= read_len_;
          read_len_ = 0;
        } else {
          push(read_op_, seq_len_);
          read_len_ -= seq_len_;
          seq_len_ = 0;
        }
        break;
      case 'I':
        push(read_op_, read_len_);
        read_len_ = 0;
        break;
      default: throw std::runtime_error("Unknown cigar op in read");
    }
  }
  void in_insertion() {
    switch (OPS[read_op_]) {
      case 'M':
        if (seq_len_ < read_len_) {
          push(1, seq_len_);
          read_len_ -= seq_len_;
          seq_len_ = 0;
        } else {
          push(1, read_len_);
          seq_len_ -= read_len_;
          read_len_ = 0;
        }
        break;
      case 'I':
        push(read_op_, read_len_);
        read_len_ = 0;
        break;
      case 'N': case 'D':
        if (seq_len_ > read_len_) {
          seq_len_ -= read_len_;
          read_len_ = 0;
        } else {
          read_len_ -= seq_len_;
          seq_len_ = 0;
        }
        break;
      default: throw std::runtime_error("Unknown cigar op in read");
    }
  }
  void in_deletion() {
    switch (OPS[read_op_]) {
      case 'M':
        push(tr_seqop(seq_op_), seq_len_);
        seq_advance();
        break;
      case 'I':
        push(tr_seqop(seq_op_), seq_len_);
        seq_advance();
        push(read_op_, read_len_);
        read_advance();
        break;
      case 'N': case 'D':
        push(tr_seqop(seq_op_), seq_len_);
        seq_len_ = 0;
        break;
      default: throw std::runtime_error("Unknown cigar op in read");
    }
  }
  void find_start_pos() {
    while (cpos_ < start_pos_ && !eos()) {
      if (seq_len_ == 0) seq_advance();
      const int dist = (int)(start_pos_ - cpos_);
      switch (seq_op_) {
        case '=': case 'M': case 'X': case 'I':
          if (seq_len_ > dist) {
            seq_len_ -= (int)(start_pos_ - cpos_);
            cpos_ = start_pos_;
          } else {
            cpos_ += (uint32_t)seq_len_;
            seq_len_ = 0;
          }
          break;
        case 'N': case 'D': seq_len_ = 0; break;
        default: throw std::runtime_error(std::string("Invalid cigar character: ") + seq_op_);
      }
    }
    if (cpos_ < start_pos_)
      throw std::runtime_error("Failed to seek to position " + std::to_string(start_pos_) + " in cigar string '" +
                               std::string(seq_cigar_) + "'");
  }
  bool eos() const { return seq_len_ == 0 && *p_ == 0; }
  bool eor() const { return read_len_ == 0 && rci_ >= n_; }
  void seq_advance() {
    char *end;
    seq_len_ = (int)strtoul(p_, &end, 10);
    p_ = end;
    seq_op_ = *p_;
    if (*p_) ++p_;  // the reference steps past the terminating NUL too (never read again)
  }
  void read_advance() {
    if (!rc_) return;
    read_len_ = (int)(rc_[rci_] & 0x1fffffffu);
    read_op_ = (int)(rc_[rci_++] >> 29);
  }
};

// translate_cigar (translate_cigar.cpp:342-356): false (message printed) when the translation fails
inline bool translate_cigar(const std::string &seq_cigar, uint32_t start, const uint32_t *read_cigar, int n_cigar,
                            int read_len, std::vector<uint32_t> &out) {
  CigarTranslator ct(seq_cigar.c_str(), start, read_cigar, n_cigar, read_len);
  try {
    ct.exec();
    out.swap(ct.out);
    return true;
  } catch (const std::exception &e) {
    fprintf(stderr, "Error translating cigar string: %s\n", e.what());
    out.clear();
    return false;
  }
}

}  // namespace ibwa_sam
#endif
