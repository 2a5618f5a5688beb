// sam_common.h -- the host side shared by `ibwa-amd samse` and `ibwa-amd sampe`: reference
// metadata (.ann/.amb/.pac, bntseq.c), the read record (bwa_seq_t, bwtaln.h:62-93) and its
// ingestion (bwaseqio.c), the POSIX drand48 stream, approximate mapQ, refine_gapped_core's
// window / fix-ups around the GPU global alignment, MD/NM, and SAM printing (bwase.c).
#ifndef IBWA_SAM_COMMON_H
#define IBWA_SAM_COMMON_H
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "ibwa_aln.h"
#include "readers.h"
#include "remap.h"

namespace ibwa_sam {

// ---------------------------------------------------------------- host parallelism and timing
// Host threads for the per-read steps that do not touch the RNG stream (MD/NM, SAM formatting):
// OMP_NUM_THREADS when set (the GPU box sets it to its CPU share), else the hardware's, at most 32.
inline int host_threads() {
  const char *e = getenv("OMP_NUM_THREADS");
  int n = e ? atoi(e) : (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 32));
}
// f(begin, end, chunk) over [0, n) in contiguous chunks, one per thread
inline void parallel_chunks(int64_t n, const std::function<void(int64_t, int64_t, int)> &f, int nt = 0) {
  if (nt <= 0) nt = host_threads();
  nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n / 256 + 1));
  if (nt == 1) {
    f(0, n, 0);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back(f, n * t / nt, n * (t + 1) / nt, t);
  for (auto &x : th) x.join();
}
// Messages of per-read steps: printed at once, or inside parallel_ordered collected per chunk and
// printed after the join in chunk order -- the stderr a sequential loop gives
inline std::string *&msg_sink() {
  static thread_local std::string *sink = nullptr;
  return sink;
}
// The stderr of one sampe batch (-G workers): collected while a worker runs the batch and printed
// when its SAM is written, in file order -- the reference's sequential order of batch messages
inline std::string *&batch_log() {
  static thread_local std::string *log = nullptr;
  return log;
}
inline void emit(const char *s) {
  if (std::string *b = batch_log()) b->append(s);
  else fputs(s, stderr);
}
inline void elog(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
inline void elog(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  emit(buf);
}
inline void msg(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
inline void msg(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (std::string *s = msg_sink()) s->append(buf);
  else emit(buf);
}
// f(begin, end, thread) over [0, n) in chunks of `grain` claimed dynamically by the host threads
// (a few costly items do not hold one thread's whole share back), with msg() output kept in the
// order of a sequential loop: each chunk's messages are printed after the join, chunk by chunk
inline void parallel_ordered(int64_t n, const std::function<void(int64_t, int64_t, int)> &f, int nt = 0,
                             int64_t grain = 256) {
  if (n <= 0) return;
  if (nt <= 0) nt = host_threads();
  const int64_t nch = (n + grain - 1) / grain;
  nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, nch));
  std::vector<std::string> out(nch);
  std::atomic<int64_t> next{0};
  auto work = [&](int t) {
    for (;;) {
      const int64_t ch = next.fetch_add(1);
      if (ch >= nch) break;
      msg_sink() = &out[ch];
      f(ch * grain, std::min(n, (ch + 1) * grain), t);
      msg_sink() = nullptr;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
  for (const std::string &x : out)
    if (!x.empty()) emit(x.c_str());
}
// a thread joined when it goes out of scope (the next batch's parser, on every return path)
struct Background {
  std::thread t;
  template <class F> void start(F &&f) { t = std::thread(std::forward<F>(f)); }
  void wait() { if (t.joinable()) t.join(); }
  ~Background() { wait(); }
};
// wall-clock seconds per named phase, printed to stderr at the end of a command
// (IBWA_PHASE_CPU=1: also the process's CPU seconds, all threads, per phase -- a worker's own only
// when it is the only one running)
struct Phases {
  std::vector<std::pair<const char *, double>> acc, cpu;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double c0 = cpu_now();
  static double cpu_now() {
    timespec ts;
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
  }
  static void add(std::vector<std::pair<const char *, double>> &v, const char *name, double dt) {
    for (auto &a : v)
      if (!strcmp(a.first, name)) { a.second += dt; return; }
    v.push_back({name, dt});
  }
  void mark(const char *name) {
    const auto t = std::chrono::steady_clock::now();
    add(acc, name, std::chrono::duration<double>(t - t0).count());
    t0 = t;
    static const bool want_cpu = getenv("IBWA_PHASE_CPU") != nullptr;
    if (want_cpu) {
      const double c = cpu_now();
      add(cpu, name, c - c0);
      c0 = c;
    }
  }
  void print(const char *who) const {
    fprintf(stderr, "[%s] wall s:", who);
    for (auto &a : acc) fprintf(stderr, " %s %.2f", a.first, a.second);
    fprintf(stderr, "\n");
    if (cpu.empty()) return;
    fprintf(stderr, "[%s] cpu s:", who);
    for (auto &a : cpu) fprintf(stderr, " %s %.2f", a.first, a.second);
    fprintf(stderr, "\n");
  }
};


constexpr int TYPE_NO_MATCH = 0, TYPE_UNIQUE = 1, TYPE_REPEAT = 2, TYPE_MATESW = 3;  // bwtaln.h:7-10
constexpr int SAM_FPD = 1, SAM_FPP = 2, SAM_FSU = 4, SAM_FMU = 8, SAM_FSR = 16, SAM_FMR = 32,  // bwtaln.h:12-20
              SAM_FR1 = 64, SAM_FR2 = 128;
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
// 2 MiB-aligned memory advised for transparent huge pages before it is first touched: the .pac is
// read at random (MD/NM, refinement and mate-rescue windows), and with 4 KiB pages most of those
// reads also miss the TLB
template <class T>
struct HugeAlloc {
  using value_type = T;
  HugeAlloc() = default;
  template <class U>
  HugeAlloc(const HugeAlloc<U> &) {}
  T *allocate(size_t n) {
    const size_t huge = (size_t)2 << 20, bytes = (n * sizeof(T) + huge - 1) / huge * huge;
    void *p = aligned_alloc(huge, bytes);
    if (!p) throw std::bad_alloc();
    madvise(p, bytes, MADV_HUGEPAGE);
    return static_cast<T *>(p);
  }
  void deallocate(T *p, size_t) { free(p); }
  template <class U>
  bool operator==(const HugeAlloc<U> &) const { return true; }
  template <class U>
  bool operator!=(const HugeAlloc<U> &) const { return false; }
};

struct Bns {
  int64_t l_pac = 0;
  int32_t n_seqs = 0;
  uint32_t seed = 0;
  std::vector<Ann> anns;
  std::vector<Amb> ambs;
  std::vector<uint8_t, HugeAlloc<uint8_t>> pac;  // seq_load_pac (dbset.c:103-108): l_pac / 4 + 1 bytes
};

// bns_restore_core (bntseq.c:88-140) + seq_load_pac
inline bool bns_restore(const std::string &prefix, Bns &b) {
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

// codes [x, x + n) of a 2-bit packed sequence (base x at bits 7-6 of byte x / 4 down to bits 1-0):
// pac_at base by base, a whole byte's four codes at once where x is byte-aligned
inline void unpack_pac(const uint8_t *pac, uint64_t x, uint64_t n, uint8_t *out) {
  static const struct Lut {
    uint32_t w[256];
    Lut() {
      for (int b = 0; b < 256; ++b) {
        const uint8_t c[4] = {(uint8_t)(b >> 6 & 3), (uint8_t)(b >> 4 & 3), (uint8_t)(b >> 2 & 3), (uint8_t)(b & 3)};
        memcpy(&w[b], c, 4);
      }
    }
  } lut;
  uint64_t t = 0;
  for (; t < n && (x & 3); ++t, ++x) *out++ = (pac[x >> 2] >> ((~x & 3) << 1)) & 3;
  for (const uint8_t *q = pac + (x >> 2); t + 4 <= n; t += 4, x += 4, out += 4) memcpy(out, &lut.w[*q++], 4);
  for (; t < n; ++t, ++x) *out++ = (pac[x >> 2] >> ((~x & 3) << 1)) & 3;
}

// dbset_extract_sequence (dbset.c:306-325), one database at offset 0
inline uint32_t extract(const Bns &b, uint64_t beg, uint32_t len, uint8_t *out) {
  if (beg >= (uint64_t)b.l_pac) return 0;
  const uint32_t t = (uint32_t)std::min<uint64_t>(len, (uint64_t)b.l_pac - beg);
  unpack_pac(b.pac.data(), beg, t, out);
  return t;
}

// bns_seq_for_pos (bntseq.c:278-294)
inline int32_t seq_for_pos(const Bns &b, int64_t pac_coor) {
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
inline int coor_pac2real(const Bns &b, int64_t pac_coor, int len, int32_t *seqid) {
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

// ---------------------------------------------------------------- the database set (dbset.c)
// sampe's references concatenated at their offsets (dbset_restore, dbset.c:135-176): the primary
// first, then the alternates; an alternate may carry a .remap table (remap.h).  samse and a
// single-reference sampe use a set of one.
struct RefDb {
  Bns bns;
  uint64_t offset = 0;
  int remap = 0;
  std::vector<std::unique_ptr<Mapping>> mappings;  // per sequence, when remap
};
struct Dbs {
  std::vector<RefDb> db;
  uint64_t l_pac = 0;  // sum of the references' l_pac
  // coord2idx (dbset.c:17-39)
  int coord2idx(int64_t pos) const {
    const int count = (int)db.size();
    int left = 0, right = count, mid = 0;
    if (pos > (int64_t)l_pac) return -1;
    while (left < right) {
      mid = (left + right) >> 1;
      if (pos > (int64_t)db[mid].offset) {
        if (mid == count - 1) break;
        if (pos < (int64_t)db[mid + 1].offset) break;
        left = mid + 1;
      } else if (pos < (int64_t)db[mid].offset) {
        right = mid;
      } else {
        break;
      }
    }
    return mid;
  }
};

// dbset_extract_sequence (dbset.c:306-325): the references read back to back
inline uint32_t extract(const Dbs &d, uint64_t beg, uint32_t len, uint8_t *out) {
  uint32_t total = 0;
  while (total < len) {
    if (beg >= d.l_pac) break;
    const int idx = d.coord2idx((int64_t)beg);
    const RefDb &r = d.db[idx];
    uint64_t pos = beg - r.offset;
    if (pos < (uint64_t)r.bns.l_pac) {
      const uint64_t k = std::min<uint64_t>(len - total, (uint64_t)r.bns.l_pac - pos);
      unpack_pac(r.bns.pac.data(), pos, k, out + total);
      total += (uint32_t)k;
      pos += k;
    }
    beg = pos + r.offset;
  }
  return total;
}

// dbset_coor_pac2real (dbset.c:248-255): the sequence (and reference) holding pac_coor
inline int coor_pac2real(const Dbs &d, int64_t pac_coor, int len, int32_t *seqid, int *dbi) {
  const int idx = d.coord2idx(pac_coor);
  if (idx < 0) err_fatal("bns_seq_for_pos", "bug! Coordinate is longer than sequence (%lld>=%lld).", (long long)pac_coor,
                         (long long)d.l_pac);
  *dbi = idx;
  return coor_pac2real(d.db[idx].bns, pac_coor - (int64_t)d.db[idx].offset, len, seqid);
}

// bns_seq_by_name (bntseq.c:269-276)
inline int32_t seq_by_name(const Bns &b, const std::string &name) {
  for (int32_t i = 0; i < b.n_seqs; ++i)
    if (b.anns[i].name == name) return i;
  return -1;
}

// bwa_remap_position_with_seqid (bwaremap.cpp:252-311): an alternate position (relative to its
// reference) -> the target position in the primary; *status 1 on success
inline uint64_t remap_position_with_seqid(const RefDb &r, const Bns &target, uint64_t pac_coor, int32_t seqid, int *status) {
  *status = 0;
  const Mapping *m = seqid >= 0 && seqid < (int32_t)r.mappings.size() ? r.mappings[seqid].get() : nullptr;
  if (!m) err_fatal("bwa_remap_position_with_seqid", "No read mapping for sequence id %d\n", seqid);
  const int32_t target_idx = seq_by_name(target, m->seqname);
  if (target_idx < 0) err_fatal("bwa_remap_position_with_seqid", "Failed to locate remapping target: %s\n", m->seqname.c_str());
  uint32_t rv = 0;
  if (!m->exact) {
    uint32_t offset = 0;
    const uint32_t altpos = (uint32_t)(pac_coor - (uint64_t)r.bns.anns[seqid].offset);
    if (!remap_cigar(m->cigar.c_str(), &offset, altpos, (uint32_t)r.bns.anns[seqid].len)) {
      msg("Failed to remap coordinates to %s (coord=%lu)", r.bns.anns[seqid].name.c_str(), (unsigned long)pac_coor);
      return 0;
    }
    rv = m->start + offset;
  } else {
    rv = (uint32_t)(pac_coor - (uint64_t)r.bns.anns[seqid].offset);
  }
  if (!m->exact && (rv < m->start || rv > m->stop))
    err_fatal("bwa_remap_position_with_seqid", "remapped position out of range (%u should be in [%u, %u])\n", rv, m->start,
              m->stop);
  *status = 1;
  return rv + (uint64_t)target.anns[target_idx].offset;
}

// __remap (bwape.c:201-219, filter_alignments.cpp:15-34) for a hit at global position pos on
// reference dbidx: its position in the primary (pos itself when the reference has no table)
inline uint64_t remap_pos(const Dbs &d, int dbidx, uint64_t pos, uint64_t len, uint32_t gap, int32_t *seqid, int *identical,
                          int *status) {
  const RefDb &r = d.db[dbidx];
  if (!r.remap) {
    *seqid = -1;
    *status = 1;
    return pos;
  }
  const uint64_t rel = pos - r.offset;
  *seqid = seq_for_pos(r.bns, (int64_t)rel);  // bwa_remap_position (bwaremap.cpp:244-249)
  const uint64_t x = remap_position_with_seqid(r, d.db[0].bns, rel, *seqid, status);
  const Mapping &m = *r.mappings[*seqid];
  const uint64_t relpos = rel - (uint64_t)r.bns.anns[*seqid].offset;
  *identical = is_remapped_sequence_identical(m, (uint32_t)(relpos > gap ? relpos - gap : 0), (uint32_t)(len + gap));
  return x;
}

// dbset_extract_remapped (dbset.c:257-304): a window of an alternate sequence, continued on the
// primary before its start and after its end
inline uint32_t extract_remapped(const Dbs &d, int dbidx, int32_t seqid, uint64_t beg, uint32_t len, uint8_t *out) {
  const RefDb &r = d.db[dbidx];
  if (seqid < 0 || !r.remap) return extract(d, beg, len, out);
  const Ann &ann = r.bns.anns[seqid];
  const uint64_t seq_begin = r.offset + (uint64_t)ann.offset;
  uint32_t total = 0;
  int status = 0;
  if (beg < seq_begin) {
    const uint64_t remapped_begin = remap_position_with_seqid(r, d.db[0].bns, (uint64_t)ann.offset, seqid, &status);
    const uint64_t sublen = seq_begin - beg;
    const uint64_t offset = remapped_begin - sublen;
    if (sublen > remapped_begin || status == 0) err_fatal("dbset_extract_remapped", "request too far ahead of remapped region");
    total += extract(d, offset, (uint32_t)sublen, out + total);
  }
  if (total < len) {
    uint32_t sublen = len - total;
    if (sublen > (uint32_t)ann.len) sublen = (uint32_t)ann.len;
    total += extract(d, beg, sublen, out + total);
  }
  if (total < len) {
    const uint64_t remapped_end =
        remap_position_with_seqid(r, d.db[0].bns, (uint64_t)ann.offset + ann.len - 1, seqid, &status) + 1;
    if (status == 0) err_fatal("dbset_extract_remapped", "request too far ahead of remapped region");
    total += extract(d, remapped_end, len - total, out + total);
  }
  if (total != len)
    err_fatal("dbset_extract_remapped", "logic error: got %lu bases instead of %lu\n", (unsigned long)total, (unsigned long)len);
  return total;
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

// POSIX lrand48 on the same generator (bns_fasta2bntseq's N fill, bntseq.c:224): X' >> 17
struct Lrand48 {
  uint64_t x = 0;
  void seed(long s) { x = ((uint64_t)(uint32_t)s << 16) | 0x330Eu; }
  long next() {
    x = (0x5DEECE66Dull * x + 0xBu) & ((1ull << 48) - 1);
    return (long)(x >> 17);
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
  int type = TYPE_NO_MATCH, strand = 0, n_mm = 0, n_gapo = 0, n_gape = 0, score = 0, extra_flag = 0;
  uint32_t sa = 0;
  uint64_t pos = 0, remapped_pos = 0;
  int dbidx = 0, remapped_dbidx = 0, remapped_seqid = 0, remap_identical = 0;  // sampe's database set
  uint32_t c1 = 0, c2 = 0;
  int seQ = 0, mapQ = 0, nm = 0;
  std::vector<uint32_t> cigar;
  bool has_cigar = false;
  std::vector<Multi> multi;
  std::string md;
  bool has_md = false;
};

// bwa_trim_read (bwaseqio.c:74-87)
inline int trim_read(int trim_qual, Read &p) {
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

inline unsigned char nt4[256];  // nst_nt4_table (bntseq.c:39-56)

// bwa_read_seq (bwaseqio.c:145-208) / bwa_read_bam (:89-143) for one record
template <class Reader>
inline bool next_read(Reader &rd, int mode, int trim_qual, Read &p) {
  const bool bam = std::is_same<Reader, ibwa_cli::BamReader>::value;
  const bool is_comp = mode & IBWA_MODE_COMPREAD;
  const bool is_64 = !bam && (mode & IBWA_MODE_IL13);
  const int l_bc = bam ? 0 : (int)((unsigned)mode >> 24);
  for (;;) {
    const int l = rd.read();
    if (l < 0) return false;
    std::string s = std::move(rd.seq), q = std::move(rd.qual);  // the reader refills them
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
      p.qual = std::move(q);
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

// a Read back to its defaults, keeping its strings' and vectors' buffers (a batch's reads are
// refilled in place: no allocation per read in the steady state)
inline void reset_read(Read &p) {
  Read t;
  t.name.swap(p.name); t.qual.swap(p.qual); t.seq.swap(p.seq); t.rseq.swap(p.rseq);
  t.cigar.swap(p.cigar); t.multi.swap(p.multi); t.md.swap(p.md);
  t.name.clear(); t.qual.clear(); t.seq.clear(); t.rseq.clear(); t.cigar.clear(); t.multi.clear(); t.md.clear();
  p = std::move(t);
}

// next_read's record (bwa_read_seq, bwaseqio.c:145-208) from a strict FASTQ record of the bulk
// parser: false for a record bwa_read_seq skips (not longer than the barcode)
inline bool rec_to_read(const char *base, const ibwa_cli::FastqBulk::Rec &r, int mode, int trim_qual, Read &p) {
  const bool is_comp = mode & IBWA_MODE_COMPREAD;
  const bool is_64 = mode & IBWA_MODE_IL13;
  const int l_bc = (int)((unsigned)mode >> 24);
  const int L = (int)r.len;
  if (L <= l_bc) return false;
  const char *s = base + r.s, *q = base + r.q;
  reset_read(p);
  auto qv = [&](int i) { return is_64 ? (char)(q[i] - 31) : q[i]; };
  if (l_bc) {
    for (int i = 0; i < l_bc; ++i) p.bc[i] = qv(i) - 33 < 13 ? (char)tolower(s[i]) : (char)toupper(s[i]);
    p.bc[l_bc] = 0;
  }
  const int n = L - l_bc;
  p.full_len = p.clip_len = p.len = n;
  p.seq.resize(n);
  p.qual.resize(n);
  p.rseq.resize(n);
  uint8_t *sq = p.seq.data(), *rs = p.rseq.data();
  const char *src = s + l_bc;
  if (is_64) {
    for (int i = 0; i < n; ++i) p.qual[i] = qv(l_bc + i);
  } else {
    memcpy(&p.qual[0], q + l_bc, (size_t)n);
  }
  p.has_qual = true;
  if (trim_qual >= 1) {
    for (int i = 0; i < n; ++i) sq[i] = nt4[(unsigned char)src[i]];
    trim_read(trim_qual, p);
    memset(rs, 0, (size_t)n);
    for (int i = 0; i < p.len; ++i) {
      const uint8_t c = sq[p.len - 1 - i];
      rs[i] = is_comp && c < 4 ? 3 - c : c;
    }
  } else {  // untrimmed: the codes and their reverse complement in one pass
    for (int i = 0; i < n; ++i) {
      const uint8_t c = nt4[(unsigned char)src[i]];
      sq[i] = c;
      rs[n - 1 - i] = is_comp && c < 4 ? 3 - c : c;
    }
  }
  // kseq's name: the header up to its first white space; then /[12]$ trimmed
  const char *h = base + r.h + 1, *e = h;
  while (*e != '\n' && !isspace((unsigned char)*e)) ++e;
  size_t t = (size_t)(e - h);
  if (t > 2 && h[t - 2] == '/' && (h[t - 1] == '1' || h[t - 1] == '2')) t -= 2;
  p.name.assign(h, t);
  return true;
}

// A batch of reads into out (its elements, from a batch before, refilled in place) up to n_max:
// the bulk parser's strict FASTQ records converted on nt host threads, then record by record
// through next(Read &) (the serial reader, from the first record the bulk parser did not take):
// the same reads in the same order as next() alone.
template <class NextFn>
inline void take_reads(ibwa_cli::FastqBulk *fb, int mode, int trim_qual, std::vector<Read> &out, size_t n_max, int nt,
                       NextFn next) {
  auto par = [](int k, const std::function<void(int)> &g) {
    std::vector<std::thread> th;
    for (int t = 1; t < k; ++t) th.emplace_back(g, t);
    g(0);
    for (auto &x : th) x.join();
  };
  size_t have = 0;
  while (fb && have < n_max && fb->more(nt, par)) {
    const size_t i0 = fb->qi, m = std::min(fb->recs.size() - i0, n_max - have);
    if (out.size() < have + m) out.resize(have + m);
    std::vector<uint8_t> keep(m);
    const char *base = fb->blk.data();
    parallel_chunks((int64_t)m, [&](int64_t lo, int64_t hi, int) {
      for (int64_t k = lo; k < hi; ++k) keep[k] = rec_to_read(base, fb->recs[i0 + k], mode, trim_qual, out[have + k]);
    }, nt);
    size_t w = have;
    for (size_t k = 0; k < m; ++k)
      if (keep[k]) {
        if (w != have + k) std::swap(out[w], out[have + k]);
        ++w;
      }
    have = w;
    fb->qi = i0 + m;
  }
  Read r;
  while (have < n_max && next(r)) {
    if (have < out.size()) out[have] = std::move(r);
    else out.push_back(std::move(r));
    ++have;
  }
  out.resize(have);
}

// bwa_aln2seq_core (bwase.c:29-104) with set_main = 1
inline void aln2seq(int n_aln, const ibwa_aln1_t *aln, Read &s, int n_multi, Drand48 &rnd) {
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

inline int g_log_n[256];  // bwase.c g_log_n

// bwa_approx_mapQ (bwase.c:111-126)
inline int approx_mapQ(const Read &p, int mm) {
  if (p.c1 == 0) return 23;
  if (p.c1 > 1) return 0;
  if (p.n_mm == mm) return 25;
  if (p.c2 == 0) return 37;
  const int n = p.c2 >= 255 ? 255 : (int)p.c2;
  return 23 < g_log_n[n] ? 0 : 23 - g_log_n[n];
}

// bwa_cal_md1 (bwase.c:243-295)
inline std::string cal_md1(const Read &s, uint64_t pos, const uint8_t *seq, const Dbs &b, int *nm_out) {
  // the reference bases of a CIGAR run are extracted at once (extract(x, n) == n one-base extracts:
  // both stop at l_pac and cross references the same way), the numbers formatted in place; built in a
  // per-thread buffer and returned as one string (most MD strings fit the string's inline storage:
  // no allocation per read)
  thread_local std::string str;
  str.clear();
  auto put_int = [](int v) {
    char t[12];
    char *e = t + sizeof t, *q = e;
    unsigned u = (unsigned)v;
    do {
      *--q = (char)('0' + u % 10);
      u /= 10;
    } while (u);
    str.append(q, (size_t)(e - q));
  };
  thread_local std::vector<uint8_t> rb;
  uint64_t x = pos, y = 0;
  const uint64_t l_pac = b.l_pac;
  int u = 0, nm = 0;
  uint8_t c = 0;
  auto run = [&](uint64_t at, int l) -> int {  // the bases of [at, at + l) before l_pac, into rb
    if ((int)rb.size() < l) rb.resize((size_t)l);
    if (at >= l_pac || l <= 0) return 0;
    const uint64_t n = std::min<uint64_t>((uint64_t)l, l_pac - at);
    return (int)extract(b, at, (uint32_t)n, rb.data());
  };
  // bases [0, n) of rb against seq[y, y + n): the mismatches into the MD string; eight equal bytes at a
  // time are eight matches (extracted codes are 0-3, so equal bytes exclude an N); c ends as rb[n - 1]
  auto md_run = [&](int n, uint64_t yy) {
    int z = 0;
    while (z < n) {
      if (z + 8 <= n) {
        uint64_t ra, sb;
        memcpy(&ra, rb.data() + z, 8);
        memcpy(&sb, seq + yy + z, 8);
        if (ra == sb) {
          u += 8;
          z += 8;
          continue;
        }
      }
      c = rb[z];
      if (c > 3 || seq[yy + z] > 3 || c != seq[yy + z]) {
        put_int(u);
        str += "ACGTN"[c];
        ++nm;
        u = 0;
      } else {
        ++u;
      }
      ++z;
    }
    if (n > 0) c = rb[n - 1];
  };
  if (s.has_cigar) {
    for (uint32_t cg : s.cigar) {
      const int l = (int)cig_len(cg);
      const uint32_t op = cig_op(cg);
      if (op == FROM_M) {
        const int n = run(x, l);
        md_run(n, y);
        x += l; y += l;
      } else if (op == FROM_I || op == FROM_S) {
        y += l;
        if (op == FROM_I) nm += l;
      } else if (op == FROM_D) {
        put_int(u);
        str += '^';
        const int n = run(x, l);
        for (int z = 0; z < n; ++z) {
          c = rb[z];
          str += "ACGT"[c];
        }
        u = 0;
        x += l; nm += l;
      }
    }
  } else {
    // past l_pac nothing is extracted: c keeps the last base's value (as the reference)
    const int n = run(x, s.len);
    md_run(n, y);
    for (int z = n; z < s.len; ++z) {
      if (c > 3 || seq[y + z] > 3 || c != seq[y + z]) {
        put_int(u);
        str += "ACGTN"[c];
        ++nm;
        u = 0;
      } else {
        ++u;
      }
    }
  }
  put_int(u);
  *nm_out = nm;
  return std::string(str);
}

// bwa_correct_trimmed (bwase.c:297-331)
inline void correct_trimmed(Read &s) {
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

inline int64_t pos_end(const Read &p) {  // bwase.c:418-429
  if (!p.has_cigar) return (int64_t)p.pos + p.len;
  int64_t x = (int64_t)p.pos;
  for (uint32_t c : p.cigar)
    if (cig_op(c) == 0 || cig_op(c) == 2) x += cig_len(c);
  return x;
}
inline int64_t pos_end_multi(const Multi &q, int len) {  // bwase.c:431-442
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
  int dbidx = 0, seqid = -1;  // the hit's reference and (remapped references) its sequence
  Read *s = nullptr;
  Multi *q = nullptr;  // null: the read's own hit
};

// the window of one refinement (dbset_extract_remapped on a remapped reference); fills the
// job's reference / read slices
inline bool refine_prepare(const Dbs &b, Read &s, uint64_t pos, int ext, Refine &j, std::vector<uint8_t> &rbuf,
                           std::vector<uint64_t> &roff, std::vector<uint32_t> &rlen) {
  if (pos > b.l_pac) return false;  // the caller reports it (bwase.c:175-178)
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
  j.l = extract_remapped(b, j.dbidx, j.seqid, (uint64_t)ref_start, (uint32_t)ref_len, rbuf.data() + o);
  rbuf.resize(o + j.l);
  j.ref_start = ref_start;
  j.ext = ext;
  roff.push_back(o);
  rlen.push_back(j.l);
  return true;
}

// the CIGAR and position fix-ups after the alignment (bwase.c:200-240): ends, then the CIGAR of a
// hit on an alternate sequence translated onto the primary (translate_cigar)
inline void refine_finish(const Dbs &b, const Refine &j, const uint32_t *c32, int n32, int len, uint64_t *pos,
                          std::vector<uint32_t> &cigar, bool *has_cigar) {
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
  *has_cigar = true;
  const RefDb &r = b.db[j.dbidx];
  if (r.remap && j.seqid >= 0 && j.seqid < (int)r.mappings.size() && r.mappings[j.seqid] && r.mappings[j.seqid]->has_cigar) {
    const uint64_t start = *pos - r.offset - (uint64_t)r.bns.anns[j.seqid].offset;
    std::vector<uint32_t> t;
    // a failed translation leaves no CIGAR (the reference's NULL)
    *has_cigar = translate_cigar(r.mappings[j.seqid]->cigar, (uint32_t)start, cigar.data(), (int)cigar.size(), len, t);
    cigar.swap(t);
  }
}

// bwa_refine_gapped (bwase.c:333-416) over a set of reads: the banded global alignment of every
// gapped hit (refine_gapped_core, bwase.c:167-241) in one ibwa_global_batch launch, then MD/NM at
// each read's remapped_pos as the reference has it at that point (bwase.c:401) and the
// trimmed-read correction.  Returns 0, 1 on a bad position (message printed), -1 on a GPU error.
inline int refine_gapped(ibwa_ctx_t *ctx, const Dbs &b, std::vector<Read *> &reads) {
  // the jobs in read order, gathered in contiguous read ranges on the host threads and concatenated
  struct Part {
    std::vector<Refine> jobs;
    std::vector<uint8_t> rbuf, qbuf;
    std::vector<uint64_t> roff, qoff;
    std::vector<uint32_t> rlen, qlen;
    int64_t bad = -1;  // the first read whose window is out of range
    uint64_t bad_pos = 0;
  };
  const int nt = std::max(1, std::min<int>(host_threads(), (int)(reads.size() / 1024) + 1));
  std::vector<Part> part(nt);
  parallel_chunks((int64_t)reads.size(), [&](int64_t lo, int64_t hi, int t) {
    Part &P = part[t];
    auto add_job = [&](Read &p, Multi *q, uint64_t ps, int ext, int strand, int dbidx, int seqid) -> bool {
      Refine j;
      j.s = &p;
      j.q = q;
      j.dbidx = dbidx;
      j.seqid = seqid;
      if (ps > b.l_pac) {
        P.bad_pos = ps;
        return false;
      }
      if (!refine_prepare(b, p, ps, ext, j, P.rbuf, P.roff, P.rlen)) return false;
      const std::vector<uint8_t> &sq = strand ? p.rseq : p.seq;
      P.qoff.push_back(P.qbuf.size());
      P.qlen.push_back((uint32_t)p.len);
      P.qbuf.insert(P.qbuf.end(), sq.begin(), sq.begin() + p.len);
      P.jobs.push_back(j);
      return true;
    };
    for (int64_t i = lo; i < hi && P.bad < 0; ++i) {
      Read &p = *reads[i];
      // remapped sequences can also have gaps (bwase.c:341-347)
      int remapped_gapo = 0;
      const RefDb &r = b.db[p.dbidx];
      if (r.remap && p.remapped_seqid >= 0 && p.remapped_seqid < (int)r.mappings.size() && r.mappings[p.remapped_seqid])
        remapped_gapo += r.mappings[p.remapped_seqid]->n_gapo;
      bool ok = true;
      for (Multi &q : p.multi) {  // bwt_multi1_t.dbidx / remapped_seqid are 0 (select_sai_multi)
        if (q.gap == 0) continue;
        if (!(ok = add_job(p, &q, q.pos, (q.strand ? 1 : -1) * q.gap, q.strand, 0, 0))) break;
      }
      if (ok && !(p.type == TYPE_NO_MATCH || p.type == TYPE_MATESW || (p.n_gapo == 0 && remapped_gapo == 0)))
        ok = add_job(p, nullptr, p.pos, (p.strand ? 1 : -1) * (p.n_gapo + p.n_gape), p.strand, p.dbidx, p.remapped_seqid);
      if (!ok) P.bad = i;
    }
  }, nt);
  for (const Part &P : part)
    if (P.bad >= 0) {
      fprintf(stderr, "[refine_gapped_core] position=%llu > l_pac=%llu\n", (unsigned long long)P.bad_pos,
              (unsigned long long)b.l_pac);
      return 1;
    }
  std::vector<Refine> jobs;
  std::vector<uint8_t> rbuf, qbuf;
  std::vector<uint64_t> roff, qoff;
  std::vector<uint32_t> rlen, qlen;
  for (Part &P : part) {
    const uint64_t rb = rbuf.size(), qb = qbuf.size();
    jobs.insert(jobs.end(), P.jobs.begin(), P.jobs.end());
    for (uint64_t x : P.roff) roff.push_back(rb + x);
    for (uint64_t x : P.qoff) qoff.push_back(qb + x);
    rlen.insert(rlen.end(), P.rlen.begin(), P.rlen.end());
    qlen.insert(qlen.end(), P.qlen.begin(), P.qlen.end());
    rbuf.insert(rbuf.end(), P.rbuf.begin(), P.rbuf.end());
    qbuf.insert(qbuf.end(), P.qbuf.begin(), P.qbuf.end());
    P = Part();
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
      return -1;
    // the fix-ups on the host threads (each job writes its own read's or multi hit's fields)
    std::vector<int64_t> q0(m + 1, 0);
    for (int64_t k = 0; k < m; ++k) q0[k + 1] = q0[k] + nc[k];
    parallel_chunks(m, [&](int64_t lo, int64_t hi, int) {
      for (int64_t k = lo; k < hi; ++k) {
        Refine &j = jobs[k];
        if (j.q) refine_finish(b, j, c32 + q0[k], nc[k], j.s->len, &j.q->pos, j.q->cigar, &j.q->has_cigar);
        else refine_finish(b, j, c32 + q0[k], nc[k], j.s->len, &j.s->pos, j.s->cigar, &j.s->has_cigar);
      }
    });
    ibwa_free(c32);
  }
  parallel_chunks((int64_t)reads.size(), [&](int64_t lo, int64_t hi, int) {
    for (int64_t t = lo; t < hi; ++t) {
      Read &p = *reads[t];
      if (p.type != TYPE_NO_MATCH) {
        p.md = cal_md1(p, p.remapped_pos, p.strand ? p.rseq.data() : p.seq.data(), b, &p.nm);
        p.nm &= 0xfff;
        p.has_md = true;
      }
      correct_trimmed(p);
    }
  });
  return 0;
}

// ---------------------------------------------------------------- SAM output (bwa_print_sam1, bwase.c:451-581)
struct Out {
  FILE *fp;
  std::string b;
  std::thread w;  // print_parallel's write-behind of a batch's lines
  // print_parallel's per-thread line buffers, handed back by the writer with their capacity: a batch's
  // lines go into memory the previous batch already faulted in (a fresh ~0.2 GB per batch, allocated,
  // faulted in and freed, cost about as much as formatting into it)
  std::vector<std::string> spare;
  void wait() {
    if (w.joinable()) w.join();
  }
  void flush() {
    wait();
    if (!b.empty()) fwrite(b.data(), 1, b.size(), fp);
    b.clear();
  }
  ~Out() { wait(); }
  Out &s(const char *x) { b += x; return *this; }
  Out &s(const std::string &x) { b += x; return *this; }
  Out &c(char x) { b += x; return *this; }
  // n bases of s as letters (codes 0-4), or the reverse complement of s[0, n)
  Out &bases(const uint8_t *q, int n, bool rc) {
    const size_t o0 = b.size();
    b.resize(o0 + (size_t)(n > 0 ? n : 0));
    char *w = &b[o0];
    if (!rc)
      for (int k = 0; k < n; ++k) w[k] = "ACGTN"[q[k]];
    else
      for (int k = 0; k < n; ++k) w[k] = "TGCAN"[q[n - 1 - k]];
    return *this;
  }
  Out &i(long long v) {  // %lld
    char t[24];
    char *e = t + sizeof t, *q = e;
    unsigned long long u = v < 0 ? 0ull - (unsigned long long)v : (unsigned long long)v;
    do {
      *--q = (char)('0' + u % 10);
      u /= 10;
    } while (u);
    if (v < 0) *--q = '-';
    b.append(q, (size_t)(e - q));
    return *this;
  }
};

inline void print_cigar(Out &o, const std::vector<uint32_t> &cg) {
  for (uint32_t c : cg) o.i((long long)cig_len(c)).c("MIDSN"[cig_op(c)]);
}

// bwa_print_sam1 (bwase.c:451-581).  `mate` is null for samse.  As the reference, an unmapped read
// with a mapped mate takes the mate's position and strand, and the quality string is reversed in
// place for a reverse-strand read.
inline int64_t pos_5(const Read &p) { return p.type != TYPE_NO_MATCH ? (p.strand ? pos_end(p) : (int64_t)p.pos) : -1; }

inline void print_sam1(Out &o, const Dbs &d, Read &p, const Read *mate, int mode, int max_top2, const char *rg_id) {
  if (p.type != TYPE_NO_MATCH || (mate && mate->type != TYPE_NO_MATCH)) {
    int32_t seqid = 0;
    int flag = p.extra_flag, am = 0, j, dbi = 0;
    if (p.type == TYPE_NO_MATCH) {
      p.pos = mate->pos;
      p.remapped_pos = mate->remapped_pos;
      p.strand = mate->strand;
      flag |= SAM_FSU;
      j = 1;
    } else {
      j = (int)(pos_end(p) - (int64_t)p.pos);  // the reference length of the alignment
    }
    // dbset_coor_pac2real: the sequence, and the reference (bns, offset) it belongs to
    int nn = coor_pac2real(d, (int64_t)p.pos, j, &seqid, &dbi);
    const Bns *bns = &d.db[dbi].bns;
    int64_t bnsoffset = (int64_t)d.db[dbi].offset;
    if (p.type != TYPE_NO_MATCH && (int64_t)p.pos + j - (bns->anns[seqid].offset + bnsoffset) > bns->anns[seqid].len)
      flag |= SAM_FSU;
    if (p.strand) flag |= SAM_FSR;
    if (mate) {
      if (mate->type != TYPE_NO_MATCH) {
        if (mate->strand) flag |= SAM_FMR;
      } else {
        flag |= SAM_FMU;
      }
    }
    o.s(p.name).c('\t').i(flag).c('\t').s(bns->anns[seqid].name).c('\t');
    o.i((int)((int64_t)p.pos - (bns->anns[seqid].offset + bnsoffset) + 1)).c('\t').i(p.mapQ).c('\t');
    if (p.has_cigar) print_cigar(o, p.cigar);
    else if (p.type == TYPE_NO_MATCH) o.c('*');
    else o.i(p.len).c('M');
    if (mate && mate->type != TYPE_NO_MATCH) {
      int32_t m_seqid = 0;
      int m_dbi = 0;
      am = mate->seQ < p.seQ ? mate->seQ : p.seQ;  // the smaller single-end mapping quality
      coor_pac2real(d, (int64_t)mate->pos, mate->len, &m_seqid, &m_dbi);
      const int64_t m_bnsoffset = (int64_t)d.db[m_dbi].offset;
      bns = &d.db[m_dbi].bns;  // as the reference, bns now names the mate's reference
      const bool same = seqid == m_seqid && bnsoffset == m_bnsoffset;
      o.c('\t').s(same ? std::string("=") : bns->anns[m_seqid].name).c('\t');
      long long isize = same ? pos_5(*mate) - pos_5(p) : 0;
      if (p.type == TYPE_NO_MATCH) isize = 0;
      o.i((int)((int64_t)mate->pos - (bns->anns[m_seqid].offset + m_bnsoffset) + 1)).c('\t').i(isize).c('\t');
    } else if (mate) {
      o.s("\t=\t").i((int)((int64_t)p.pos - (bns->anns[seqid].offset + bnsoffset) + 1)).s("\t0\t");
    } else {
      o.s("\t*\t0\t0\t");
    }
    o.bases(p.seq.data(), p.full_len, p.strand != 0);
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
    if (p.type != TYPE_NO_MATCH) {
      char XT = "NURM"[p.type];
      if (nn > 10) XT = 'N';
      o.s("\tXT:A:").c(XT).c('\t').s((mode & IBWA_MODE_COMPREAD) ? "NM" : "CM").s(":i:").i(p.nm);
      if (nn) o.s("\tXN:i:").i(nn);
      if (mate) o.s("\tSM:i:").i(p.seQ).s("\tAM:i:").i(am);
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
          int q_dbi = 0;
          coor_pac2real(d, (int64_t)q.pos, j, &seqid, &q_dbi);
          const Bns &qb = d.db[q_dbi].bns;
          const int64_t qoff = (int64_t)d.db[q_dbi].offset;
          o.s(qb.anns[seqid].name).c(',').c(q.strand ? '-' : '+');
          o.i((int)((int64_t)q.pos - (qb.anns[seqid].offset + qoff) + 1)).c(',');
          if (q.has_cigar) print_cigar(o, q.cigar);
          else o.i(p.len).c('M');
          o.c(',').i(q.gap + q.mm).c(';');
        }
      }
    }
    if (p.pos != p.remapped_pos) {
      int32_t rs = 0;
      int r_dbi = 0;
      coor_pac2real(d, (int64_t)p.remapped_pos, j, &rs, &r_dbi);
      const Bns &rb = d.db[r_dbi].bns;
      o.s("\tZR:Z:").s(rb.anns[rs].name).c(',');
      o.i((int)((int64_t)p.remapped_pos - (rb.anns[rs].offset + (int64_t)d.db[r_dbi].offset) + 1));
    }
    o.c('\n');
  } else {
    const std::vector<uint8_t> &s = p.strand ? p.rseq : p.seq;
    int flag = p.extra_flag | SAM_FSU;
    if (mate && mate->type == TYPE_NO_MATCH) flag |= SAM_FMU;
    o.s(p.name).c('\t').i(flag).s("\t*\t0\t0\t*\t*\t0\t0\t");
    o.bases(s.data(), p.len, false);
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

// SAM lines of items [0, n) formatted on host threads into per-chunk buffers, written in order
inline void print_parallel(Out &o, int64_t n, const std::function<void(Out &, int64_t)> &fmt) {
  o.flush();  // (joins the previous batch's writer: o.spare holds its buffers)
  const int nt = host_threads();
  std::vector<std::string> bufs = std::move(o.spare);
  o.spare.clear();
  bufs.resize(nt);
  for (auto &x : bufs) x.clear();  // (a small batch leaves some unused: none may write old lines)
  parallel_chunks(n, [&](int64_t lo, int64_t hi, int t) {
    Out ob{nullptr, std::move(bufs[t])};
    for (int64_t i = lo; i < hi; ++i) fmt(ob, i);
    bufs[t] = std::move(ob.b);
  }, nt);
  // written while the next batch is worked on (Out::flush / the next call / ~Out wait for it), then
  // handed back for the next batch
  Out *op = &o;
  o.w = std::thread([op, fp = o.fp, bufs = std::move(bufs)]() mutable {
    for (auto &x : bufs)
      if (!x.empty()) fwrite(x.data(), 1, x.size(), fp);
    op->spare = std::move(bufs);
  });
}

// bwa_escape / bwa_set_rg (bwase.c:608-641)
inline bool set_rg(const char *s, std::string &line, std::string &id) {
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

// nst_nt4_table (bntseq.c:39-56) and g_log_n (bwase_initialize)
inline void init_tables() {
  memset(nt4, 4, sizeof nt4);
  nt4[(int)'A'] = nt4[(int)'a'] = 0;
  nt4[(int)'C'] = nt4[(int)'c'] = 1;
  nt4[(int)'G'] = nt4[(int)'g'] = 2;
  nt4[(int)'T'] = nt4[(int)'t'] = 3;
  nt4[(int)'-'] = 5;
  for (int i = 1; i != 256; ++i) g_log_n[i] = (int)(4.343 * log(i) + 0.5);
}

}  // namespace ibwa_sam
#endif
