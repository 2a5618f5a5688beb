// samse_main.cpp -- `ibwa-amd samse [-n max_occ] [-f out.sam] [-r RG] <prefix> <in.sai> <in.fq>`:
// the reference's samse (bwa_sai2sam_se, bwase.c:643-740) for one reference database, with
// its two compute steps on the GPU:
//   * SA -> coordinate of every chosen hit and every XA hit (bwa_cal_pac_pos, bwase.c:137-165)
//     is one ibwa_sa2pos launch per batch over the resident (full) suffix array;
//   * the banded global alignments of bwa_refine_gapped (refine_gapped_core, bwase.c:167-241)
//     are one ibwa_global_batch launch per batch.
// Everything else is the reference's host logic in its order: bwa_aln2seq_core (bwase.c:29-104,
// hit choice with the POSIX drand48 stream seeded from .ann, bwase.c:662), the approximate
// mapQ (:111-126), the CIGAR end fix-ups, MD/NM (bwa_cal_md1 :243-295), trimmed-read
// correction (:297-331) and bwa_print_sam1 (:451-581).  Reference quirks are kept: samse
// never sets remapped_pos, so MD/NM are computed at pac position 0 (bwase.c:401) and every
// mapped read carries a ZR tag (bwase.c:556-563).  Color-space input (.sai written with -c)
// needs the .nt index and is rejected.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "ibwa_aln.h"
#include "readers.h"

namespace {

constexpr int TYPE_NO_MATCH = 0, TYPE_UNIQUE = 1, TYPE_REPEAT = 2, TYPE_MATESW = 3;  // bwtaln.h:7-10
constexpr int SAM_FSU = 4, SAM_FSR = 16;                                             // bwtaln.h:11-20
constexpr int FROM_M = 0, FROM_I = 1, FROM_D = 2, FROM_S = 3;
constexpr int kMinRdLen = 35;  // BWA_MIN_RDLEN

inline uint32_t cig_op(uint32_t c) { return c >> 29; }         // bwtaln.h:44-49
inline uint32_t cig_len(uint32_t c) { return c & 0x1fffffffu; }
inline uint32_t cig_make(uint32_t op, uint32_t len) { return op << 29 | len; }

// ---------------------------------------------------------------- reference metadata (bntseq.c)
struct Ann {
  uint32_t gi = 0;
  std::string name;
  int64_t offset = 0;
  int32_t len = 0, n_ambs = 0;
};
struct Amb {
  int64_t offset = 0;
  int32_t len = 0;
};
struct Bns {
  int64_t l_pac = 0;
  int32_t n_seqs = 0;
  uint32_t seed = 0;
  std::vector<Ann> anns;
  std::vector<Amb> ambs;
  std::vector<uint8_t> pac;  // seq_load_pac (dbset.c:103-108): l_pac / 4 + 1 bytes
};

// bns_restore_core (bntseq.c:88-140) + seq_load_pac
bool bns_restore(const std::string &prefix, Bns &b) {
  FILE *fp = fopen((prefix + ".ann").c_str(), "r");
  if (!fp) return false;
  long long xx = 0;
  if (fscanf(fp, "%lld%d%u", &xx, &b.n_seqs, &b.seed) != 3) { fclose(fp); return false; }
  b.l_pac = xx;
  b.anns.resize(b.n_seqs);
  std::vector<char> str(65536);
  for (auto &a : b.anns) {
    if (fscanf(fp, "%u%65535s", &a.gi, str.data()) != 2) { fclose(fp); return false; }
    a.name = str.data();
    int c;
    while ((c = fgetc(fp)) != '\n' && c != EOF) {}
    if (fscanf(fp, "%lld%d%d", &xx, &a.len, &a.n_ambs) != 3) { fclose(fp); return false; }
    a.offset = xx;
  }
  fclose(fp);
  fp = fopen((prefix + ".amb").c_str(), "r");
  if (!fp) return false;
  int32_t n_seqs = 0, n_holes = 0;
  if (fscanf(fp, "%lld%d%d", &xx, &n_seqs, &n_holes) != 3 || xx != b.l_pac || n_seqs != b.n_seqs) {
    fclose(fp);
    fprintf(stderr, "[bns_restore_core] inconsistent .ann and .amb files.\n");
    return false;
  }
  b.ambs.resize(n_holes);
  for (auto &h : b.ambs) {
    if (fscanf(fp, "%lld%d%65535s", &xx, &h.len, str.data()) != 3) { fclose(fp); return false; }
    h.offset = xx;
  }
  fclose(fp);
  fp = fopen((prefix + ".pac").c_str(), "rb");
  if (!fp) return false;
  b.pac.assign(b.l_pac / 4 + 1, 0);
  const size_t got = fread(b.pac.data(), 1, b.pac.size(), fp);
  fclose(fp);
  (void)got;
  return true;
}

inline uint8_t pac_at(const Bns &b, uint64_t x) { return (b.pac[x >> 2] >> ((~x & 3) << 1)) & 3; }  // bns_pac

// dbset_extract_sequence (dbset.c:306-325), one database at offset 0
uint32_t extract(const Bns &b, uint64_t beg, uint32_t len, uint8_t *out) {
  uint32_t t = 0;
  while (t < len && beg < (uint64_t)b.l_pac) out[t++] = pac_at(b, beg++);
  return t;
}

// bns_seq_for_pos (bntseq.c:278-294)
int32_t seq_for_pos(const Bns &b, int64_t pac_coor) {
  if (pac_coor >= b.l_pac) {
    fprintf(stderr, "[bns_seq_for_pos] bug! Coordinate is longer than sequence (%lld>=%lld).\n",
            (long long)pac_coor, (long long)b.l_pac);
    exit(1);
  }
  int32_t left = 0, mid = 0, right = b.n_seqs;
  while (left < right) {
    mid = (left + right) >> 1;
    if (pac_coor >= b.anns[mid].offset) {
      if (mid == b.n_seqs - 1) break;
      if (pac_coor < b.anns[mid + 1].offset) break;
      left = mid + 1;
    } else {
      right = mid;
    }
  }
  return mid;
}

// bns_coor_pac2real (bntseq.c:296-318): the sequence holding pac_coor and the N overlap of [pac_coor, +len)
int coor_pac2real(const Bns &b, int64_t pac_coor, int len, int32_t *seqid) {
  *seqid = seq_for_pos(b, pac_coor);
  int32_t left = 0, right = (int32_t)b.ambs.size(), nn = 0;
  while (left < right) {
    const int64_t mid = (left + right) >> 1;
    const Amb &h = b.ambs[mid];
    if (pac_coor >= h.offset + h.len) left = (int32_t)mid + 1;
    else if (pac_coor + len <= h.offset) right = (int32_t)mid;
    else {
      if (pac_coor >= h.offset) nn += h.offset + h.len < pac_coor + len ? (int)(h.offset + h.len - pac_coor) : len;
      else nn += h.offset + h.len < pac_coor + len ? h.len : (int)(len - (h.offset - pac_coor));
      break;
    }
  }
  return nn;
}

// POSIX drand48 / srand48 (glibc: X' = 0x5DEECE66D X + 0xB mod 2^48, the result is X' / 2^48)
struct Drand48 {
  uint64_t x = 0x1234ABCD330Eull;
  void seed(long s) { x = ((uint64_t)(uint32_t)s << 16) | 0x330Eu; }
  double next() {
    x = (0x5DEECE66Dull * x + 0xBu) & ((1ull << 48) - 1);
    return ldexp((double)x, -48);
  }
};

// ---------------------------------------------------------------- reads (bwa_seq_t)
struct Multi {  // bwt_multi1_t (bwtaln.h:51-60)
  uint64_t pos = 0;
  int gap = 0, mm = 0, strand = 0;
  std::vector<uint32_t> cigar;
  bool has_cigar = false;
};
struct Read {
  std::string name, qual;
  bool has_qual = false;
  std::vector<uint8_t> seq;   // the read in input order (bwa_seq_t.seq after bwa_refine_gapped's reversal)
  std::vector<uint8_t> rseq;  // reverse complement of its first len bases, zero-padded to full_len
  int len = 0, full_len = 0, clip_len = 0;
  char bc[16] = {0};
  int type = TYPE_NO_MATCH, strand = 0, n_mm = 0, n_gapo = 0, n_gape = 0, score = 0;
  uint32_t sa = 0;
  uint64_t pos = 0, remapped_pos = 0;
  uint32_t c1 = 0, c2 = 0;
  int seQ = 0, mapQ = 0, nm = 0;
  std::vector<uint32_t> cigar;
  bool has_cigar = false;
  std::vector<Multi> multi;
  std::string md;
  bool has_md = false;
};

// bwa_trim_read (bwaseqio.c:74-87)
int trim_read(int trim_qual, Read &p) {
  if (trim_qual < 1 || !p.has_qual) return 0;
  int s = 0, mx = 0, max_l = p.len - 1;
  for (int l = p.len - 1; l >= kMinRdLen - 1; --l) {
    s += trim_qual - ((unsigned char)p.qual[l] - 33);
    if (s < 0) break;
    if (s > mx) { mx = s; max_l = l; }
  }
  p.clip_len = p.len = max_l + 1;
  return p.full_len - p.len;
}

unsigned char nt4[256];

// bwa_read_seq (bwaseqio.c:145-208) / bwa_read_bam (:89-143) for one record
template <class Reader>
bool next_read(Reader &rd, int mode, int trim_qual, Read &p) {
  const bool bam = std::is_same<Reader, ibwa_cli::BamReader>::value;
  const bool is_comp = mode & IBWA_MODE_COMPREAD;
  const bool is_64 = !bam && (mode & IBWA_MODE_IL13);
  const int l_bc = bam ? 0 : (int)((unsigned)mode >> 24);
  for (;;) {
    const int l = rd.read();
    if (l < 0) return false;
    std::string s = rd.seq, q = rd.qual;
    if (is_64 && !q.empty())
      for (auto &ch : q) ch = (char)(ch - 31);
    if (!bam && (int)s.size() <= l_bc) continue;
    p = Read();
    if (l_bc) {
      for (int i = 0; i < l_bc; ++i)
        p.bc[i] = (!q.empty() && q[i] - 33 < 13) ? (char)tolower(s[i]) : (char)toupper(s[i]);
      p.bc[l_bc] = 0;
      s.erase(0, l_bc);
      if (!q.empty()) q.erase(0, l_bc);
    }
    p.full_len = p.clip_len = p.len = (int)s.size();
    p.seq.resize(p.full_len);
    for (int i = 0; i < p.full_len; ++i) p.seq[i] = nt4[(unsigned char)s[i]];
    if (!q.empty() || bam) {
      p.qual = q;
      p.has_qual = true;
      if (trim_qual >= 1) trim_read(trim_qual, p);
    }
    p.rseq.assign(p.full_len, 0);
    for (int i = 0; i < p.len; ++i) {
      const uint8_t c = p.seq[p.len - 1 - i];
      p.rseq[i] = is_comp && c < 4 ? 3 - c : c;
    }
    p.name = rd.name;
    if (!bam) {  // trim /[12]$
      const size_t t = p.name.size();
      if (t > 2 && p.name[t - 2] == '/' && (p.name[t - 1] == '1' || p.name[t - 1] == '2')) p.name.resize(t - 2);
    }
    return true;
  }
}

// bwa_aln2seq_core (bwase.c:29-104) with set_main = 1
void aln2seq(int n_aln, const ibwa_aln1_t *aln, Read &s, int n_multi, Drand48 &rnd) {
  if (n_aln == 0) {
    s.type = TYPE_NO_MATCH;
    s.c1 = s.c2 = 0;
    return;
  }
  int i, cnt;
  const int best = aln[0].score;
  for (i = cnt = 0; i < n_aln; ++i) {
    const ibwa_aln1_t *p = aln + i;
    if (p->score > best) break;
    if (rnd.next() * (double)(uint32_t)(p->l - p->k + 1 + (uint32_t)cnt) > (double)cnt) {
      s.n_mm = p->n_mm; s.n_gapo = p->n_gapo; s.n_gape = p->n_gape; s.strand = p->a;
      s.score = p->score;
      s.sa = p->k + (uint32_t)((double)(uint32_t)(p->l - p->k + 1) * rnd.next());
    }
    cnt += (int)(p->l - p->k + 1);
  }
  s.c1 = (uint32_t)cnt & 0xfffffffu;
  for (; i < n_aln; ++i) cnt += (int)(aln[i].l - aln[i].k + 1);
  s.c2 = ((uint32_t)cnt - s.c1) & 0xfffffffu;
  s.type = s.c1 > 1 ? TYPE_REPEAT : TYPE_UNIQUE;
  if (n_multi) {
    int n_occ = 0;
    for (int k = 0; k < n_aln; ++k) n_occ += (int)(aln[k].l - aln[k].k + 1);
    s.multi.clear();
    if (n_occ > n_multi + 1) return;  // too many hits: none of them
    // every hit fits (rest = n_occ), so the reference's sampling branch is never taken
    for (int k = 0; k < n_aln; ++k) {
      const ibwa_aln1_t *q = aln + k;
      for (uint32_t l = q->k; l <= q->l; ++l) {
        Multi m;
        m.pos = l;
        m.gap = (q->n_gapo + q->n_gape) & 0xff;
        m.mm = q->n_mm;
        m.strand = q->a;
        s.multi.push_back(m);
      }
    }
    std::vector<Multi> kept;
    for (auto &m : s.multi)
      if (m.pos != s.sa) kept.push_back(m);
    if ((int)kept.size() > n_multi) kept.resize(n_multi);
    s.multi.swap(kept);
  }
}

int g_log_n[256];

// bwa_approx_mapQ (bwase.c:111-126)
int approx_mapQ(const Read &p, int mm) {
  if (p.c1 == 0) return 23;
  if (p.c1 > 1) return 0;
  if (p.n_mm == mm) return 25;
  if (p.c2 == 0) return 37;
  const int n = p.c2 >= 255 ? 255 : (int)p.c2;
  return 23 < g_log_n[n] ? 0 : 23 - g_log_n[n];
}

// bwa_cal_md1 (bwase.c:243-295)
std::string cal_md1(const Read &s, uint64_t pos, const uint8_t *seq, const Bns &b, int *nm_out) {
  std::string str;
  char buf[32];
  uint64_t x = pos, y = 0;
  const uint64_t l_pac = (uint64_t)b.l_pac;
  int u = 0, nm = 0;
  uint8_t c = 0;
  if (s.has_cigar) {
    for (uint32_t cg : s.cigar) {
      const int l = (int)cig_len(cg);
      const uint32_t op = cig_op(cg);
      if (op == FROM_M) {
        for (int z = 0; z < l && x + z < l_pac; ++z) {
          extract(b, x + z, 1, &c);
          if (c > 3 || seq[y + z] > 3 || c != seq[y + z]) {
            snprintf(buf, sizeof buf, "%d", u);
            str += buf;
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
        snprintf(buf, sizeof buf, "%d", u);
        str += buf;
        str += '^';
        for (int z = 0; z < l && x + z < l_pac; ++z) {
          extract(b, x + z, 1, &c);
          str += "ACGT"[c];
        }
        u = 0;
        x += l; nm += l;
      }
    }
  } else {
    for (int z = 0; z < s.len; ++z) {
      extract(b, x + z, 1, &c);  // past l_pac nothing is written: c keeps its value (as the reference)
      if (c > 3 || seq[y + z] > 3 || c != seq[y + z]) {
        snprintf(buf, sizeof buf, "%d", u);
        str += buf;
        str += "ACGTN"[c];
        ++nm;
        u = 0;
      } else {
        ++u;
      }
    }
  }
  snprintf(buf, sizeof buf, "%d", u);
  str += buf;
  *nm_out = nm;
  return str;
}

// bwa_correct_trimmed (bwase.c:297-331)
void correct_trimmed(Read &s) {
  if (s.len == s.full_len) return;
  const uint32_t clip = cig_make(FROM_S, (uint32_t)(s.full_len - s.len));
  if (s.strand == 0) {
    if (s.has_cigar && cig_op(s.cigar.back()) == FROM_S) {
      s.cigar.back() += (uint32_t)(s.full_len - s.len);
    } else {
      if (!s.has_cigar) {
        s.cigar.assign(1, cig_make(FROM_M, (uint32_t)s.len));
        s.has_cigar = true;
      }
      s.cigar.push_back(clip);
    }
  } else {
    if (s.has_cigar && cig_op(s.cigar[0]) == FROM_S) {
      s.cigar[0] += (uint32_t)(s.full_len - s.len);
    } else {
      if (!s.has_cigar) {
        s.cigar.assign(1, cig_make(FROM_M, (uint32_t)s.len));
        s.has_cigar = true;
      }
      s.cigar.insert(s.cigar.begin(), clip);
    }
  }
  s.len = s.full_len;
}

int64_t pos_end(const Read &p) {  // bwase.c:418-429
  if (!p.has_cigar) return (int64_t)p.pos + p.len;
  int64_t x = (int64_t)p.pos;
  for (uint32_t c : p.cigar)
    if (cig_op(c) == 0 || cig_op(c) == 2) x += cig_len(c);
  return x;
}
int64_t pos_end_multi(const Multi &q, int len) {  // bwase.c:431-442
  if (!q.has_cigar) return (int64_t)q.pos + len;
  int64_t x = (int64_t)q.pos;
  for (uint32_t c : q.cigar)
    if (cig_op(c) == 0 || cig_op(c) == 2) x += cig_len(c);
  return x;
}

// ---------------------------------------------------------------- refine_gapped_core (bwase.c:167-241)
struct Refine {
  int64_t ref_start = 0;
  uint32_t l = 0;
  int ext = 0;
  Read *s = nullptr;
  Multi *q = nullptr;  // null: the read's own hit
};

// the window of one refinement; fills the job's reference / read slices
bool refine_prepare(const Bns &b, Read &s, uint64_t pos, int ext, Refine &j, std::vector<uint8_t> &rbuf,
                    std::vector<uint64_t> &roff, std::vector<uint32_t> &rlen) {
  if (pos > (uint64_t)b.l_pac) {
    fprintf(stderr, "[refine_gapped_core] position=%llu > l_pac=%llu\n", (unsigned long long)pos,
            (unsigned long long)b.l_pac);
    return false;
  }
  const int64_t p = (int64_t)pos;
  int64_t ref_len = s.len + abs(ext), ref_start;
  if (ext > 0) {
    ref_start = p;
  } else {
    const int64_t x = p + s.len;  // is_end_correct = 1
    ref_start = x - ref_len > 0 ? x - ref_len : 0;
    ref_len = x - ref_start;
  }
  const size_t o = rbuf.size();
  rbuf.resize(o + (size_t)ref_len);
  j.l = extract(b, (uint64_t)ref_start, (uint32_t)ref_len, rbuf.data() + o);
  rbuf.resize(o + j.l);
  j.ref_start = ref_start;
  j.ext = ext;
  roff.push_back(o);
  rlen.push_back(j.l);
  return true;
}

// the CIGAR and position fix-ups after the alignment (bwase.c:200-223, no remapping)
void refine_finish(const Refine &j, const uint32_t *c32, int n32, uint64_t *pos, std::vector<uint32_t> &cigar) {
  cigar.clear();
  for (int k = 0; k < n32; ++k) cigar.push_back(cig_make(c32[k] & 0xf, c32[k] >> 4));  // bwa_aln_path2cigar
  int64_t p = (int64_t)*pos;
  if (j.ext < 0) {  // is_end_correct: fix the coordinate of a forward-strand read
    int64_t l = 0;
    for (uint32_t c : cigar) {
      if (cig_op(c) == FROM_D) l -= cig_len(c);
      else if (cig_op(c) == FROM_I) l += cig_len(c);
    }
    p += l;
  }
  if (!cigar.empty() && cig_op(cigar[0]) == FROM_D) {  // deletion at the 5'-end
    p += cig_len(cigar[0]);
    cigar.erase(cigar.begin());
  }
  if (!cigar.empty() && cig_op(cigar.back()) == FROM_D) cigar.pop_back();  // at the 3'-end
  if (!cigar.empty() && cig_op(cigar.back()) == FROM_I) cigar.back() = cig_make(FROM_S, cig_len(cigar.back()));
  if (!cigar.empty() && cig_op(cigar[0]) == FROM_I) cigar[0] = cig_make(FROM_S, cig_len(cigar[0]));
  *pos = (uint64_t)p;
}

// ---------------------------------------------------------------- SAM output (bwa_print_sam1, bwase.c:451-581)
struct Out {
  FILE *fp;
  std::string b;
  void flush() {
    if (!b.empty()) fwrite(b.data(), 1, b.size(), fp);
    b.clear();
  }
  Out &s(const char *x) { b += x; return *this; }
  Out &s(const std::string &x) { b += x; return *this; }
  Out &c(char x) { b += x; return *this; }
  Out &i(long long v) {
    char t[32];
    snprintf(t, sizeof t, "%lld", v);
    b += t;
    return *this;
  }
};

void print_cigar(Out &o, const std::vector<uint32_t> &cg) {
  for (uint32_t c : cg) o.i((long long)cig_len(c)).c("MIDSN"[cig_op(c)]);
}

void print_sam1(Out &o, const Bns &b, Read &p, int mode, int max_top2, const char *rg_id) {
  if (p.type != TYPE_NO_MATCH) {
    int32_t seqid = 0;
    int flag = 0;
    int j = (int)(pos_end(p) - (int64_t)p.pos);
    int nn = coor_pac2real(b, (int64_t)p.pos, j, &seqid);
    if ((int64_t)p.pos + j - b.anns[seqid].offset > b.anns[seqid].len) flag |= SAM_FSU;
    if (p.strand) flag |= SAM_FSR;
    o.s(p.name).c('\t').i(flag).c('\t').s(b.anns[seqid].name).c('\t');
    o.i((int)((int64_t)p.pos - b.anns[seqid].offset + 1)).c('\t').i(p.mapQ).c('\t');
    if (p.has_cigar) print_cigar(o, p.cigar);
    else o.i(p.len).c('M');
    o.s("\t*\t0\t0\t");
    if (p.strand == 0)
      for (int k = 0; k < p.full_len; ++k) o.c("ACGTN"[p.seq[k]]);
    else
      for (int k = 0; k < p.full_len; ++k) o.c("TGCAN"[p.seq[p.full_len - 1 - k]]);
    o.c('\t');
    if (p.has_qual) {
      if (p.strand) std::reverse(p.qual.begin(), p.qual.begin() + std::min<size_t>(p.len, p.qual.size()));
      o.s(p.qual.c_str());
    } else {
      o.c('*');
    }
    if (rg_id) o.s("\tRG:Z:").s(rg_id);
    if (p.bc[0]) o.s("\tBC:Z:").s(p.bc);
    if (p.clip_len < p.full_len) o.s("\tXC:i:").i(p.clip_len);
    char XT = "NURM"[p.type];
    if (nn > 10) XT = 'N';
    o.s("\tXT:A:").c(XT).c('\t').s((mode & IBWA_MODE_COMPREAD) ? "NM" : "CM").s(":i:").i(p.nm);
    if (nn) o.s("\tXN:i:").i(nn);
    if (p.type != TYPE_MATESW) {
      o.s("\tX0:i:").i(p.c1);
      if ((long long)p.c1 <= max_top2) o.s("\tX1:i:").i(p.c2);
    }
    o.s("\tXM:i:").i(p.n_mm).s("\tXO:i:").i(p.n_gapo).s("\tXG:i:").i(p.n_gapo + p.n_gape);
    if (p.has_md) o.s("\tMD:Z:").s(p.md);
    if (!p.multi.empty()) {
      o.s("\tXA:Z:");
      for (const Multi &q : p.multi) {
        j = (int)(pos_end_multi(q, p.len) - (int64_t)q.pos);
        nn = coor_pac2real(b, (int64_t)q.pos, j, &seqid);
        o.s(b.anns[seqid].name).c(',').c(q.strand ? '-' : '+');
        o.i((int)((int64_t)q.pos - b.anns[seqid].offset + 1)).c(',');
        if (q.has_cigar) print_cigar(o, q.cigar);
        else o.i(p.len).c('M');
        o.c(',').i(q.gap + q.mm).c(';');
      }
    }
    if (p.pos != p.remapped_pos) {
      int32_t rs = 0;
      coor_pac2real(b, (int64_t)p.remapped_pos, j, &rs);
      o.s("\tZR:Z:").s(b.anns[rs].name).c(',').i((int)((int64_t)p.remapped_pos - b.anns[rs].offset + 1));
    }
    o.c('\n');
  } else {
    const std::vector<uint8_t> &s = p.strand ? p.rseq : p.seq;
    o.s(p.name).c('\t').i(SAM_FSU).s("\t*\t0\t0\t*\t*\t0\t0\t");
    for (int k = 0; k < p.len; ++k) o.c("ACGTN"[s[k]]);
    o.c('\t');
    if (p.has_qual) {
      if (p.strand) std::reverse(p.qual.begin(), p.qual.begin() + std::min<size_t>(p.len, p.qual.size()));
      o.s(p.qual.c_str());
    } else {
      o.c('*');
    }
    if (rg_id) o.s("\tRG:Z:").s(rg_id);
    if (p.bc[0]) o.s("\tBC:Z:").s(p.bc);
    if (p.clip_len < p.full_len) o.s("\tXC:i:").i(p.clip_len);
    o.c('\n');
  }
}

// bwa_escape / bwa_set_rg (bwase.c:608-641)
bool set_rg(const char *s, std::string &line, std::string &id) {
  if (strstr(s, "@RG") != s) return false;
  line.clear();
  for (const char *p = s; *p; ++p) {
    if (*p == '\\') {
      ++p;
      if (*p == 't') line += '\t';
      else if (*p == 'n') line += '\n';
      else if (*p == 'r') line += '\r';
      else if (*p == '\\') line += '\\';
      if (!*p) break;
    } else {
      line += *p;
    }
  }
  const size_t t = line.find("\tID:");
  if (t == std::string::npos) return false;
  size_t e = t + 4;
  while (e < line.size() && line[e] != '\t' && line[e] != '\n') ++e;
  id = line.substr(t + 4, e - t - 4);
  return true;
}

int die(const char *what) {
  fprintf(stderr, "[ibwa-amd samse] %s: %s\n", what, ibwa_last_error());
  return 1;
}

template <class Reader>
int run_samse(Reader &rd, FILE *fp_sa, const ibwa_gap_opt_t &opt, const std::string &prefix, int n_occ, FILE *out,
              const std::string &rg_line, const std::string &rg_id) {
  Bns b;
  if (!bns_restore(prefix, b)) {
    fprintf(stderr, "[ibwa-amd samse] cannot read %s.ann / .amb / .pac\n", prefix.c_str());
    return 1;
  }
  ibwa_ctx_t *ctx = nullptr;
  if (ibwa_ctx_create(0, &ctx)) return die("ibwa_ctx_create");
  if (ibwa_ctx_load_bwt_file(ctx, 0, (prefix + ".bwt").c_str()) ||
      ibwa_ctx_load_bwt_file(ctx, 1, (prefix + ".rbwt").c_str()))
    return die("load .bwt / .rbwt");
  if (ibwa_ctx_load_sa_file(ctx, 0, (prefix + ".sa").c_str()) || ibwa_ctx_load_sa_file(ctx, 1, (prefix + ".rsa").c_str()))
    return die("load .sa / .rsa");
  if (ibwa_ctx_expand_sa(ctx)) return die("expand SA");
  Drand48 rnd;
  rnd.seed((long)b.seed);  // srand48(bns->seed), bwase.c:662
  Out o{out, {}};
  for (const Ann &a : b.anns) o.s("@SQ\tSN:").s(a.name).s("\tLN:").i(a.len).c('\n');  // dbset_print_sam_SQ
  if (!rg_line.empty()) o.s(rg_line).c('\n');
  o.s("@PG\tID:bwa\tPN:bwa\tVN:ibwa-amd\n");  // bwa_print_sam_PG (main.cpp:31-34) names this program
  o.flush();
  const char *rgid = rg_id.empty() ? nullptr : rg_id.c_str();
  std::vector<ibwa_aln1_t> aln;
  long tot = 0;
  for (;;) {
    std::vector<Read> seqs;
    seqs.reserve(0x40000);
    Read r;
    while ((int)seqs.size() < 0x40000 && next_read(rd, opt.mode, opt.trim_qual, r)) seqs.push_back(std::move(r));
    if (seqs.empty()) break;
    tot += (long)seqs.size();
    // ---- read alignment (bwase.c:671-682)
    for (Read &p : seqs) {
      int32_t n_aln = 0;
      if (fread(&n_aln, 4, 1, fp_sa) != 1) n_aln = 0;
      aln.resize(std::max(n_aln, 1));
      if (n_aln > 0 && fread(aln.data(), sizeof(ibwa_aln1_t), n_aln, fp_sa) != (size_t)n_aln) {
        fprintf(stderr, "[ibwa-amd samse] truncated .sai\n");
        return 1;
      }
      aln2seq(n_aln, aln.data(), p, n_occ, rnd);
    }
    // ---- SA -> coordinate (bwa_cal_pac_pos, bwase.c:128-165): one launch for the batch
    std::vector<uint8_t> hs;
    std::vector<uint32_t> hk, hl;
    for (const Read &p : seqs) {
      if (p.type == TYPE_UNIQUE || p.type == TYPE_REPEAT) {
        hs.push_back((uint8_t)p.strand); hk.push_back(p.sa); hl.push_back((uint32_t)p.len);
      }
      for (const Multi &q : p.multi) {
        hs.push_back((uint8_t)q.strand); hk.push_back((uint32_t)q.pos); hl.push_back((uint32_t)p.len);
      }
    }
    std::vector<uint64_t> pos(hk.size());
    if (!hk.empty() && ibwa_sa2pos(ctx, (int64_t)hk.size(), hs.data(), hk.data(), hl.data(), 0, pos.data()))
      return die("sa2pos");
    size_t x = 0;
    for (Read &p : seqs) {
      if (p.type == TYPE_UNIQUE || p.type == TYPE_REPEAT) {
        p.pos = pos[x++];
        const int max_diff = opt.fnr > 0.0 ? ibwa_cal_maxdiff(p.len, 0.02, opt.fnr) : opt.max_diff;
        p.seQ = p.mapQ = approx_mapQ(p, max_diff) & 0xff;
      }
      for (Multi &q : p.multi) q.pos = pos[x++];
    }
    // ---- refine gapped alignments (bwa_refine_gapped, bwase.c:333-416): one global-alignment launch
    std::vector<Refine> jobs;
    std::vector<uint8_t> rbuf, qbuf;
    std::vector<uint64_t> roff, qoff;
    std::vector<uint32_t> rlen, qlen;
    auto add_job = [&](Read &p, Multi *q, uint64_t ps, int ext, int strand) -> bool {
      Refine j;
      j.s = &p;
      j.q = q;
      if (!refine_prepare(b, p, ps, ext, j, rbuf, roff, rlen)) return false;
      const std::vector<uint8_t> &sq = strand ? p.rseq : p.seq;
      qoff.push_back(qbuf.size());
      qlen.push_back((uint32_t)p.len);
      qbuf.insert(qbuf.end(), sq.begin(), sq.begin() + p.len);
      jobs.push_back(j);
      return true;
    };
    for (Read &p : seqs) {
      for (Multi &q : p.multi) {
        if (q.gap == 0) continue;
        if (!add_job(p, &q, q.pos, (q.strand ? 1 : -1) * q.gap, q.strand)) return 1;
      }
      if (p.type == TYPE_NO_MATCH || p.type == TYPE_MATESW || p.n_gapo == 0) continue;
      if (!add_job(p, nullptr, p.pos, (p.strand ? 1 : -1) * (p.n_gapo + p.n_gape), p.strand)) return 1;
    }
    if (!jobs.empty()) {
      rbuf.push_back(0);
      qbuf.push_back(0);
      const int64_t m = (int64_t)jobs.size();
      std::vector<int32_t> sc(m), pl(m), nc(m);
      uint32_t *c32 = nullptr;
      int64_t tc = 0;
      if (ibwa_global_batch(ctx, m, rbuf.data(), roff.data(), rlen.data(), qbuf.data(), qoff.data(), qlen.data(), 50, 5,
                            sc.data(), pl.data(), nc.data(), &c32, &tc))
        return die("global alignment");
      int64_t q0 = 0;
      for (int64_t k = 0; k < m; ++k) {
        Refine &j = jobs[k];
        if (j.q) {
          refine_finish(j, c32 + q0, nc[k], &j.q->pos, j.q->cigar);
          j.q->has_cigar = true;
        } else {
          refine_finish(j, c32 + q0, nc[k], &j.s->pos, j.s->cigar);
          j.s->has_cigar = true;
        }
        q0 += nc[k];
      }
      ibwa_free(c32);
    }
    // ---- MD / NM at remapped_pos (0 here, bwase.c:401), trimmed-read correction
    for (Read &p : seqs) {
      if (p.type != TYPE_NO_MATCH) {
        p.md = cal_md1(p, p.remapped_pos, p.strand ? p.rseq.data() : p.seq.data(), b, &p.nm);
        p.nm &= 0xfff;
        p.has_md = true;
      }
    }
    for (Read &p : seqs) correct_trimmed(p);
    // ---- print
    for (Read &p : seqs) {
      print_sam1(o, b, p, opt.mode, opt.max_top2, rgid);
      if (o.b.size() > (1u << 20)) o.flush();
    }
    o.flush();
    fprintf(stderr, "[bwa_aln_core] %ld sequences have been processed.\n", tot);
  }
  ibwa_ctx_destroy(ctx);
  return 0;
}

}  // namespace

int samse_main(int argc, char *argv[]) {
  memset(nt4, 4, sizeof nt4);  // nst_nt4_table (bntseq.c:39-56)
  nt4[(int)'A'] = nt4[(int)'a'] = 0;
  nt4[(int)'C'] = nt4[(int)'c'] = 1;
  nt4[(int)'G'] = nt4[(int)'g'] = 2;
  nt4[(int)'T'] = nt4[(int)'t'] = 3;
  nt4[(int)'-'] = 5;
  for (int i = 1; i != 256; ++i) g_log_n[i] = (int)(4.343 * log(i) + 0.5);  // bwase_initialize
  int c, n_occ = 3;
  const char *fn_out = nullptr;
  std::string rg_line, rg_id;
  optind = 1;
  while ((c = getopt(argc, argv, "hn:f:r:")) >= 0) {  // bwa_sai2sam_se (bwase.c:710-740)
    switch (c) {
      case 'h': break;
      case 'r':
        if (!set_rg(optarg, rg_line, rg_id)) {
          fprintf(stderr, "[bwa_sai2sam_se] malformated @RG line\n");
          return 1;
        }
        break;
      case 'n': n_occ = atoi(optarg); break;
      case 'f': fn_out = optarg; break;
      default: return 1;
    }
  }
  if (optind + 3 > argc) {
    fprintf(stderr, "Usage: ibwa-amd samse [-n max_occ] [-f out.sam] [-r RG] <prefix> <in.sai> <in.fq>\n");
    return 1;
  }
  const std::string prefix = argv[optind];
  FILE *fp_sa = fopen(argv[optind + 1], "rb");
  if (!fp_sa) {
    fprintf(stderr, "[ibwa-amd samse] cannot open %s\n", argv[optind + 1]);
    return 1;
  }
  ibwa_gap_opt_t opt;
  if (fread(&opt, sizeof opt, 1, fp_sa) != 1) {
    fprintf(stderr, "[ibwa-amd samse] %s: no .sai header\n", argv[optind + 1]);
    return 1;
  }
  if (!(opt.mode & IBWA_MODE_COMPREAD)) {
    fprintf(stderr, "[ibwa-amd samse] color-space alignments (aln -c) need the .nt index: not supported\n");
    return 1;
  }
  FILE *out = fn_out ? fopen(fn_out, "w") : stdout;
  if (!out) {
    fprintf(stderr, "[ibwa-amd samse] cannot write %s\n", fn_out);
    return 1;
  }
  int rc;
  if (opt.mode & IBWA_MODE_BAM) {  // bwa_open_reads (bwtaln.c:159-171)
    int which = 0;
    if (opt.mode & IBWA_MODE_BAM_SE) which |= 4;
    if (opt.mode & IBWA_MODE_BAM_READ1) which |= 1;
    if (opt.mode & IBWA_MODE_BAM_READ2) which |= 2;
    if (which == 0) which = 7;
    ibwa_cli::BamReader rd;
    if (!rd.open(argv[optind + 2], which)) return 1;
    rc = run_samse(rd, fp_sa, opt, prefix, n_occ, out, rg_line, rg_id);
  } else {
    ibwa_cli::SeqReader rd;
    if (!rd.open(argv[optind + 2])) {
      fprintf(stderr, "[ibwa-amd samse] cannot open %s\n", argv[optind + 2]);
      return 1;
    }
    rc = run_samse(rd, fp_sa, opt, prefix, n_occ, out, rg_line, rg_id);
  }
  fclose(fp_sa);
  if (out != stdout) fclose(out);
  return rc;
}
