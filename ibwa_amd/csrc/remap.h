// remap.h -- iBWA's compound-sequence remapping (`sampe -R`), host side:
//   * the .remap table of an alternate reference (load_remappings / read_mapping_extract,
//     bwaremap.cpp:42-141): per alternate sequence, its target sequence in the primary, the
//     1-based region it replaces (or `exact`) and the alternate-vs-primary CIGAR;
//   * a walk over that CIGAR, run by run (walk_alt), which serves the position projection
//     (remap_cigar, bwaremap.cpp:170-238) and the "identical remapping" test
//     (is_remapped_sequence_identical, :129-168);
//   * the CIGAR projection of a read aligned to an alternate sequence (translate_cigar,
//     translate_cigar.cpp:342-356), a table-driven merge of the two CIGARs.
// The reference's observable behaviour is kept, quirks included (noted where they occur), and its
// fatal errors (message + abort, as err_fatal).
#ifndef IBWA_REMAP_H
#define IBWA_REMAP_H
#include <errno.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
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

// The header of a .remap entry, "<name>-<target>|<start>|<stop>" or "<name>-<target>|exact..."
// (bwaremap.cpp:16-26, :102-141): the text must hold exactly one '-' and two '|'; the target runs
// from after the '-' to the first '|' and may not be empty; start / stop are 1-based inclusive
// (read with strtoul, so leading blanks and a sign pass as there) and end the text.
inline bool read_mapping_extract(const char *str, Mapping &m) {
  m.exact = 0;
  const std::string h(str);
  if (std::count(h.begin(), h.end(), '-') != 1 || std::count(h.begin(), h.end(), '|') != 2) return false;
  const size_t t0 = h.find('-') + 1, t1 = h.find('|', t0);
  if (t1 == std::string::npos || t1 == t0) return false;
  m.seqname = h.substr(t0, t1 - t0);
  const char *f = str + t1 + 1;  // the fields after the target
  if (strncmp(f, "exact", 5) == 0) {
    m.exact = 1;
    m.start = m.stop = 0;
    m.has_cigar = false;
    return true;
  }
  // two numeric fields, the first closed by '|', the second by the end of the text
  uint32_t v[2];
  const char closer[2] = {'|', '\0'};
  for (int q = 0; q < 2; ++q) {
    char *e = nullptr;
    v[q] = (uint32_t)strtoul(f, &e, 10);
    if (e == f || *e != closer[q]) return false;
    f = e + 1;
  }
  m.start = v[0] - 1;  // 0-based first base
  m.stop = v[1] + 1;   // one past the last base
  return true;
}

// load_remappings (bwaremap.cpp:42-100): -1 error, 0 no file, 1 loaded.  The file is a FASTA-like
// list: a header per alternate sequence, in sequence order, then its CIGAR over any number of lines.
// The reference reads it with std::getline and stops at end-of-file, so a header is taken only when
// a newline ends it (a last header without one is ignored); a last CIGAR line counts either way.
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
  if (data.empty()) {
    fprintf(stderr, "Empty remapping file '%s'\n", path.c_str());
    return -1;
  }
  // the lines, and whether a newline ends each
  std::vector<std::pair<std::string, bool>> lines;
  for (size_t at = 0; at < data.size();) {
    const size_t e = data.find('\n', at);
    const bool nl = e != std::string::npos;
    lines.emplace_back(data.substr(at, (nl ? e : data.size()) - at), nl);
    at = nl ? e + 1 : data.size();
  }
  auto is_header = [](const std::string &x) { return !x.empty() && x[0] == '>'; };
  int n = 0;
  for (size_t h = 0; h < lines.size() && lines[h].second;) {  // h: a header line
    const std::string &hdr = lines[h].first;
    if (!is_header(hdr)) {
      fprintf(stderr, "Unexpected character '%c' at start of line %zu in file '%s'. Expected '>'.\n",
              hdr.empty() ? '\0' : hdr[0], h + 1, path.c_str());
      return -1;
    }
    if (n >= n_seqs) {  // the reference writes past its array here
      fprintf(stderr, "More remappings than sequences in '%s'\n", path.c_str());
      return -1;
    }
    Mapping *m = new Mapping;
    maps[n].reset(m);
    if (!read_mapping_extract(hdr.c_str() + 1, *m)) {
      fprintf(stderr, "Failed to extract read mapping from string '%s' in file %s, line %zu\n", hdr.c_str() + 1,
              path.c_str(), h + 1);
      return -1;
    }
    size_t nx = h + 1;  // the CIGAR: every line up to the next header
    for (; nx < lines.size() && !is_header(lines[nx].first); ++nx) m->cigar += lines[nx].first;
    m->has_cigar = true;  // also for `exact` entries (an empty string)
    m->n_gapo = (int)std::count_if(m->cigar.begin(), m->cigar.end(),
                                   [](char ch) { return ch == 'I' || ch == 'D' || ch == 'N'; });  // cigar_gap_opens
    ++n;
    h = nx;
  }
  return 1;
}

// ---------------------------------------------------------------- the alternate's CIGAR against the primary
// Its text is read run by run ("<digits><op>", strtoul), lazily as the reference's loops read it: a
// malformed run is an error only for a walk that gets to it.  Each op moves the position on the
// alternate, on the primary, or both.
enum : int { ADV_ALT = 1, ADV_PRI = 2 };
inline int run_moves(char op) {
  switch (op) {
    case 'M': case 'X': case '=': return ADV_ALT | ADV_PRI;
    case 'I': return ADV_ALT;
    case 'N': case 'D': return ADV_PRI;
    default: return -1;
  }
}

// The runs of `text` taken while keep(walk) holds before a run (bwaremap.cpp:140-166, :180-207):
// positions after them, and the last run taken.  error: a run did not parse (message printed).
struct AltWalk {
  uint32_t alt = 0, pri = 0, last_len = 0;
  char last_op = 0;
  bool error = false;
};
template <class Keep>
inline AltWalk walk_alt(const char *text, Keep keep) {
  AltWalk w;
  for (const char *p = text; *p && keep(w);) {
    char *e;
    const uint32_t n = (uint32_t)strtoul(p, &e, 10);
    const int mv = e == p ? 0 : run_moves(*e);
    if (e == p) fprintf(stderr, "[remap_coordinates] expected number in cigar string '%s' at pos %ld\n", text, (long)(p - text));
    else if (mv < 0) fprintf(stderr, "invalid cigar character '%c'\n", *e);
    if (mv <= 0) {
      w.error = true;
      return w;
    }
    w.last_len = n;
    w.last_op = *e;
    if (mv & ADV_ALT) w.alt += n;
    if (mv & ADV_PRI) w.pri += n;
    p = e + 1;
  }
  return w;
}

// is_remapped_sequence_identical (bwaremap.cpp:129-168): whether the alternate is the primary
// unchanged over the read -- an exact remapping, or the run reaching past `start` on the primary
// is a match run with last_len - start > len (the reference's own test, unsigned, kept as is)
inline int is_remapped_sequence_identical(const Mapping &m, uint32_t start, uint32_t len) {
  if (m.exact) return 1;
  const AltWalk w = walk_alt(m.cigar.c_str(), [&](const AltWalk &x) { return x.pri <= start; });
  if (w.error || w.pri <= start) return 0;
  return (w.last_op == 'M' || w.last_op == '=') && w.last_len - start > len;
}

// remap_cigar (bwaremap.cpp:170-238): the primary offset of alternate position pos
inline int remap_cigar(const char *cigar, uint32_t *result, uint32_t pos, uint32_t seqlen) {
  if (pos >= seqlen) {
    fprintf(stderr, "[remap_coordinates] requested pos %u > sequence length %u\n", pos, seqlen);
    return 0;
  }
  const AltWalk w = walk_alt(cigar, [&](const AltWalk &x) { return x.alt <= pos; });
  if (w.error) return 0;
  if (w.alt > seqlen) {
    fprintf(stderr, "[remap_coordinates] cigar '%s' string implies length > read mapping (%u vs %u)\n", cigar, w.alt,
            seqlen);
    return 0;
  }
  if (w.alt < pos) {
    fprintf(stderr, "failed to parse cigar string '%s'\n", cigar);
    return 0;
  }
  if (w.alt == pos) {
    *result = w.pri;
    return 1;
  }
  // pos lies inside the last run: a match run maps it base for base, an insertion to where it starts
  const int mv = run_moves(w.last_op);
  if (mv == (ADV_ALT | ADV_PRI)) *result = w.pri - (w.alt - pos);
  else if (mv == ADV_ALT) *result = w.pri;
  else {
    fprintf(stderr, "Error remapping cigar string %s:, pos=%u\n", cigar, pos);
    return 0;
  }
  return 1;
}

// ---------------------------------------------------------------- translate_cigar (translate_cigar.cpp:342-356)
// A read's CIGAR (bwa_cigar_t: op << 29 | len, ops M I D S N = 0..4) against an alternate sequence,
// from `start` on it, composed with the alternate's CIGAR against the primary.  The two are merged
// run against run by the table below; what the reference does past either end (a zero-length run
// of the last op, deletions counted against an ungapped read's length, the read cursor stepped
// after an insertion without a bound check) is reproduced, since the SAM output shows it.
namespace xlat {
enum Act : uint8_t {
  EMIT_READ_MIN,   // emit the read's op over min(both); both consume it
  EMIT_READ_ALL,   // emit the read's op (an insertion) over the read run; the read run ends
  EMIT_INS_MIN,    // emit an insertion over min(both); both consume it
  SKIP_MIN,        // both consume min(both), nothing emitted
  EMIT_ALT_NEXT,   // emit the alternate's op over its run; the next alternate run
  EMIT_ALT_NEXT_I, // the same, then the read run as an insertion; the next read run
  EMIT_ALT_END,    // emit the alternate's op over its run; the alternate run ends
  BAD
};
// [alternate run: 0 match (M = X), 1 insertion (I), 2 deletion (D N)][read op M I D S N]; S never
// reaches the table (a read clip is emitted before)
constexpr Act ACT[3][5] = {
    {EMIT_READ_MIN, EMIT_READ_ALL, EMIT_READ_MIN, BAD, EMIT_READ_MIN},
    {EMIT_INS_MIN, EMIT_READ_ALL, SKIP_MIN, BAD, SKIP_MIN},
    {EMIT_ALT_NEXT, EMIT_ALT_NEXT_I, EMIT_ALT_END, BAD, EMIT_ALT_END},
};
inline int alt_class(char op) { return op == 'M' || op == '=' || op == 'X' ? 0 : op == 'I' ? 1 : op == 'N' || op == 'D' ? 2 : -1; }
inline int op_code(char op) {  // a CIGAR letter as a bwa_cigar_t op; -1 for '=' / 'X' and others
  const char *c = strchr("MIDSN", op);
  return op && c ? (int)(c - "MIDSN") : -1;
}
}  // namespace xlat

inline bool translate_cigar(const std::string &seq_cigar, uint32_t start, const uint32_t *read_cigar, int n_cigar,
                            int read_len, std::vector<uint32_t> &out) {
  using namespace xlat;
  out.clear();
  std::string err;
  auto emit = [&](int op, int n) {  // runs of one op merge (the length within its 29 bits)
    if (!out.empty() && (int)(out.back() >> 29) == op)
      out.back() = (uint32_t)op << 29 | (((out.back() & 0x1fffffffu) + (uint32_t)n) & 0x1fffffffu);
    else
      out.push_back((uint32_t)op << 29 | (uint32_t)n);
  };
  // the alternate's runs: op '\0' and length 0 once its text is used up
  const char *ap = seq_cigar.c_str();
  char a_op = 0;
  int a_left = 0;
  auto a_next = [&]() {
    char *e;
    a_left = (int)strtoul(ap, &e, 10);
    ap = e;
    a_op = *ap;
    if (*ap) ++ap;
  };
  auto a_done = [&]() { return a_left == 0 && *ap == 0; };
  // the read's runs (the reference reads the next one without a bound check)
  int r_i = 0, r_op = 0, r_left = 0;
  auto r_next = [&]() {
    if (!read_cigar) return;
    r_left = (int)(read_cigar[r_i] & 0x1fffffffu);
    r_op = (int)(read_cigar[r_i++] >> 29);
  };
  auto r_done = [&]() { return r_left == 0 && r_i >= n_cigar; };
  auto fail = [&](const std::string &why) {
    fprintf(stderr, "Error translating cigar string: %s\n", why.c_str());
    out.clear();
    return false;
  };
  a_next();
  r_next();
  // 1. the alternate's runs up to `start` (an insertion on it counts, a deletion does not)
  uint32_t at = 0;
  while (at < start && !a_done()) {
    if (a_left == 0) a_next();
    const int cl = alt_class(a_op);
    if (cl < 0) return fail(std::string("Invalid cigar character: ") + a_op);
    if (cl == 2) {
      a_left = 0;
    } else if ((uint32_t)a_left > start - at) {
      a_left -= (int)(start - at);
      at = start;
    } else {
      at += (uint32_t)a_left;
      a_left = 0;
    }
  }
  if (at < start)
    return fail("Failed to seek to position " + std::to_string(start) + " in cigar string '" + seq_cigar + "'");
  // 2a. an ungapped read: the alternate's runs over the read length
  if (!read_cigar) {
    for (int len = 0; len < read_len && !a_done();) {
      const int op = op_code(a_op);
      if (op < 0) return fail(std::string("Unknown cigar operation: ") + a_op);
      const int take = a_left < read_len - len ? a_left : read_len - len;
      emit(op, take);
      if (take < a_left) break;
      len += a_left;
      a_next();
    }
    return !out.empty();
  }
  // 2b. both CIGARs run against each other
  while (!r_done() && !a_done()) {
    if (a_left == 0) a_next();
    if (r_left == 0) r_next();
    if (r_op == 3) {  // a clip of the read passes through
      emit(3, r_left);
      r_left = 0;
      if (!r_done()) r_next();
      continue;
    }
    const int cl = alt_class(a_op);
    if (cl < 0) return fail(std::string("Invalid cigar character: ") + a_op);
    const Act act = r_op >= 0 && r_op < 5 ? ACT[cl][r_op] : BAD;
    const int mn = a_left < r_left ? a_left : r_left;
    switch (act) {
      case EMIT_READ_MIN: emit(r_op, mn); a_left -= mn; r_left -= mn; break;
      case EMIT_READ_ALL: emit(r_op, r_left); r_left = 0; break;
      case EMIT_INS_MIN: emit(1, mn); a_left -= mn; r_left -= mn; break;
      case SKIP_MIN: a_left -= mn; r_left -= mn; break;
      case EMIT_ALT_NEXT: emit(op_code(a_op), a_left); a_next(); break;
      case EMIT_ALT_NEXT_I: emit(op_code(a_op), a_left); a_next(); emit(r_op, r_left); r_next(); break;
      case EMIT_ALT_END: emit(op_code(a_op), a_left); a_left = 0; break;
      default: return fail("Unknown cigar op in read");
    }
  }
  // 3. what is left of the read is clipped (its deletions dropped)
  while (!r_done()) {
    if (r_left == 0) r_next();
    if (r_op == 0 || r_op == 1 || r_op == 3) emit(3, r_left);
    r_left = 0;
  }
  return !out.empty();  // an empty translation is the reference's NULL as well
}

}  // namespace ibwa_sam
#endif
