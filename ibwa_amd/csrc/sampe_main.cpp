// sampe_main.cpp -- `ibwa-amd sampe [options] <prefix> <in1.sai> <in2.sai> <in1.fq> <in2.fq>`: the
// reference's sampe (bwa_sai2sam_pe_core, bwape.c:436-540) for one reference database, with its
// compute steps on the GPU:
//   * SA -> coordinate (bwtdb_sa2seq, dbset.c:240-246) of every primary hit and of every row of
//     every SA interval both ends have (compute_seq_coords_and_counts, filter_alignments.cpp:53-140):
//     one ibwa_sa2pos launch per batch for each of the two passes;
//   * the mate rescue (bwa_paired_sw, bwasw.c:270-304): ibwa_paired_sw, one local-SW launch;
//   * bwa_refine_gapped's banded global alignments (bwase.c:333-416): one launch for both ends.
// The host runs the reference's logic in its order and with its quirks: select_sai_ibwa's hit
// choice (bwape.c:281-358) on the POSIX drand48 stream seeded from .ann, infer_isize (bwape.c:91-198,
// including the std accumulator that starts at -1), the per-pair position array sorted by klib's
// introsort (not stable, so its exact algorithm is restated), find_optimal_pair (bwapair.c:166-279)
// with its look-ahead one element past the array, select_sai_multi (saiset.c:124-163), and the
// (k,l)-keyed position cache of bwtcache.c for intervals of >= 1000 rows, whose key ignores the
// strand and the read length.
//
// Several references (`sampe <pri> <1.sai> <2.sai> <1.fq> <2.fq> [<alt> <a1.sai> <a2.sai> ...]`,
// pe_inputs_parse, bwape.c:548-581) are concatenated at their offsets (dbset_restore); each has its
// own index on the GPU for SA -> coordinate, and the hits of all references are merged per read
// (alngrp_create, saiset.c:45-76, with klib's unstable introsort when there are several).  With -R
// a reference that has a .remap table is a set of alternate sequences: hits on them are projected
// onto the primary (remap.h), pairing runs on the projected positions, refinement translates the
// CIGAR of gapped hits, and the SAM prints the projected position with ZR:Z: the original.
// Without -R the reference's select_sai_ibwa never sees a successful remap status and leaves every
// read unmapped ("Failed to select primary alignment"); that is reproduced.
//
// `-G N` shards the batch loop (bwape.c:476-536) over N workers, worker w on GPU w mod the visible
// devices (several on one device share its index): a worker takes the next batch of 0x40000 pairs
// in file order and runs it whole.  What the reference carries from batch to batch is settled in
// that order when the batch is taken -- the drand48 draws of its hit choice and the first use of each
// wide interval (whose strand and read length the cached positions keep) -- or waited for: a batch
// whose insert size cannot be inferred takes the previous batch's (bwape.c:410-411), and the SAM is
// written batch by batch in file order.  The output does not depend on N.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ibwa_bwa_compat.h"
#include "ksort.h"
#include "sam_common.h"

using namespace ibwa_sam;

namespace {

constexpr uint32_t kMinHashWidth = 1000;  // MIN_HASH_WIDTH (bwape.c:46, filter_alignments.cpp:10)

struct PeOpt {  // pe_opt_t defaults (bwa_init_pe_opt, bwape.c:68-84)
  int max_isize = 500, force_isize = 0, max_occ = 100000, n_multi = 3, N_multi = 10, type = IBWA_PET_STD;
  int is_sw = 1, is_preload = 0, remapping = 0, n_threads = 1;
  double ap_prior = 1e-5;
};

struct Isize {  // isize_info_t (bwapair.h:8-11)
  double avg = -1.0, std = -1.0, ap_prior = 0.0;
  uint32_t low = 0, high = 0, high_bayesian = 0;
};

int die(const char *what) {
  fprintf(stderr, "[ibwa-amd sampe] %s: %s\n", what, ibwa_last_error());
  return 1;
}

// ---------------------------------------------------------------- pairing (bwapair.c)
struct Position {  // position_t (bwapair.h:13-25)
  uint64_t pos = 0, remapped_pos = 0;
  uint32_t idx_and_end = 0;
  int dbidx = 0, remapped_dbidx = 0, remapped_seqid = 0, remap_identical = 0;
  int n_gapo = 0, n_gape = 0, len = 0, score = 0;
};
struct PosKey {  // a position's sort key (position_lt's fields) and its index
  uint64_t rp, p;
  uint32_t idx;
};
inline bool position_lt(const Position &a, const Position &b) {  // bwapair.c:22-28
  if (a.remapped_pos == b.remapped_pos) return a.pos < b.pos;
  return a.remapped_pos < b.remapped_pos;
}

// kvec-style position array reused for every pair of a batch (bwape.c:244, filter_alignments.cpp:62):
// find_optimal_pair's look-ahead (bwapair.c:204) reads the slot past the last position, which
// holds whatever an earlier pair left there.
struct PosArr {
  std::vector<Position> a;  // capacity slots; a.size() == kvec m
  size_t n = 0;
  void clear() { n = 0; }
  void push(const Position &p) {
    if (n == a.size()) a.resize(a.empty() ? 2 : a.size() << 1);  // kv_push growth
    a[n++] = p;
  }
  const Position &at(size_t i) const {
    static const Position zero;
    return i < a.size() ? a[i] : zero;
  }
};

// One pair's position array as find_optimal_pair sees it when the batch's pairs share one kvec in
// pair order (the reference's single-threaded loop): slots [0, n) are this pair's, a slot past them
// holds what the most recent earlier pair with more positions left there -- found by walking the
// nearest-previous-greater chain of the pairs' counts -- and a slot no pair wrote is zero.
struct PosView {
  const Position *const *arr;  // every pair's final array (sorted when find_optimal_pair ran)
  const uint32_t *cnt;         // every pair's count
  const int32_t *pg;           // nearest earlier pair with a larger count (-1: none)
  int64_t i;                   // this pair
  size_t n;
  const Position *a;
  PosView(const Position *const *arr_, const uint32_t *cnt_, const int32_t *pg_, int64_t i_)
      : arr(arr_), cnt(cnt_), pg(pg_), i(i_), n(cnt_[i_]), a(arr_[i_]) {}
  const Position &at(size_t idx) const {
    static const Position zero;
    if (idx < n) return a[idx];
    int64_t j = pg[i];
    while (j >= 0 && cnt[j] <= idx) j = pg[j];
    return j >= 0 ? arr[j][idx] : zero;
  }
};

inline uint64_t hash_64(uint64_t key) {  // bwapair.c:31-41
  key += ~(key << 32);
  key ^= (key >> 22);
  key += ~(key << 13);
  key ^= (key >> 8);
  key += (key << 3);
  key ^= (key >> 15);
  key += ~(key << 27);
  key ^= (key >> 31);
  return key;
}

struct Aln {  // alignment_t (saiset.h:9-14)
  ibwa_aln1_t aln;
  int dbidx;
};

// one read's alignments: a slice of the batch's flat array
struct AlnSpan {
  const Aln *p = nullptr;
  size_t n = 0;
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const Aln &operator[](size_t i) const { return p[i]; }
  const Aln *begin() const { return p; }
  const Aln *end() const { return p + n; }
};

struct PairCtx {
  Read *p[2];
  const AlnSpan *aln[2];
  const PeOpt *opt;
  const Isize *ii;
  int s_mm;
  const int *pen;  // pairing_aux's insert-size penalty per l <= ii->high_bayesian (with ii->high)
  const ibwa_aln1_t &al(const Position &x) const {
    // a position left by an earlier pair (PosView) may index past this pair's alignments: the
    // reference reads whatever lies there; here a zero record
    static const ibwa_aln1_t none = {};
    const AlnSpan &s = *aln[x.idx_and_end & 1];
    const size_t k = x.idx_and_end >> 1;
    return k < s.size() ? s[k].aln : none;
  }
};

struct Pint {  // pairing_internals_t (bwapair.c:8-17)
  int o_n = 0, subo_n = 0, cnt_chg = 0, max_len = 0;
  Position last_pos[2][2];
  Position o_pos[2];
  uint64_t subo_score = ~0ull, o_score = ~0ull;
};

// pairing_aux (bwapair.c:92-140)
void pairing_aux(const PairCtx &c, Pint &pi, const Position &u, const Position &v, int n_optimal) {
  uint32_t l;
  // both remapped onto the same alternate sequence: the insert size on it
  if (u.remapped_pos != u.pos && v.remapped_pos != v.pos && u.dbidx == v.dbidx && u.remapped_seqid == v.remapped_seqid)
    l = (uint32_t)(v.pos + (uint64_t)c.p[v.idx_and_end & 1]->len - u.pos);
  else
    l = (uint32_t)(v.remapped_pos + (uint64_t)c.p[v.idx_and_end & 1]->len - u.remapped_pos);
  if (u.remapped_pos != ~0ull && v.remapped_pos > u.remapped_pos && l >= (uint32_t)pi.max_len &&
      ((c.ii->high && l <= c.ii->high_bayesian) || (c.ii->high == 0 && l <= (uint32_t)c.opt->max_isize))) {
    uint64_t s = (uint64_t)(int64_t)(c.al(v).score + c.al(u).score);
    s *= 10;
    if (c.ii->high) s += c.pen[l];  // (int)(-4.343 * log(.5 * erfc(M_SQRT1_2 * |l - avg| / std)) + .499)
    s = s << 32 | (uint32_t)hash_64(u.remapped_pos << 32 | v.remapped_pos);
    if (s >> 32 == pi.o_score >> 32) {
      pi.o_n += n_optimal;
    } else if (s >> 32 < pi.o_score >> 32) {
      pi.subo_n += pi.o_n;
      pi.o_n = n_optimal;
    } else {
      ++pi.subo_n;
    }
    if (s < pi.o_score) {
      pi.subo_score = pi.o_score;
      pi.o_score = s;
      pi.o_pos[u.idx_and_end & 1] = u;
      pi.o_pos[v.idx_and_end & 1] = v;
    } else if (s < pi.subo_score) {
      pi.subo_score = s;
    }
  }
}

// pairing_aux2 (bwapair.c:142-158)
void pairing_aux2(const PairCtx &c, Pint &pi, Read &r, const Position &pos) {
  const ibwa_aln1_t &a = c.al(pos);
  r.extra_flag |= SAM_FPP;
  if (r.pos != pos.pos || r.strand != (int)a.a) {
    r.n_mm = a.n_mm; r.n_gapo = a.n_gapo; r.n_gape = a.n_gape; r.strand = a.a;
    r.score = a.score;
    r.pos = pos.pos;
    r.dbidx = pos.dbidx;
    r.remapped_pos = pos.remapped_pos;
    r.remapped_seqid = pos.remapped_seqid;
    if (r.mapQ > 0) ++pi.cnt_chg;
  }
}

// select_mapping (bwapair.c:64-90): the first lowest-score position of a run that maps to the same
// place, skipping a remapped position identical to a primary one already seen (the set is seeded
// from the array's first element, as the reference does)
const Position &select_mapping(const PairCtx &c, const PosView &arr, size_t begin, size_t end) {
  const Position *best = &arr.at(begin);
  std::vector<uint64_t> seen;
  auto has = [&](uint64_t x) { return std::find(seen.begin(), seen.end(), x) != seen.end(); };
  if (arr.at(0).pos == arr.at(0).remapped_pos) seen.push_back(arr.at(0).pos);
  for (size_t i = begin + 1; i <= end; ++i) {
    const Position &p = arr.at(i);
    if (p.pos == p.remapped_pos) {
      if (!has(p.pos)) seen.push_back(p.pos);
    } else if (has(p.remapped_pos) && p.remap_identical) {
      continue;
    }
    if (c.al(p).score < c.al(*best).score) best = &p;
  }
  return *best;
}

// find_optimal_pair (bwapair.c:166-279), BWA_PET_STD, on the pair's array already sorted by
// ks_introsort (bwapair.c:188)
int find_optimal_pair(const PairCtx &c, const PosView &arr) {
  Read **p = (Read **)c.p;
  Pint pi;
  pi.max_len = std::max(p[0]->full_len, p[1]->full_len);
  for (int j = 0; j < 2; ++j)
    for (int t = 0; t < 2; ++t) pi.last_pos[j][t].pos = pi.last_pos[j][t].remapped_pos = ~0ull;
  // mappings_overlap (bwapair.c:43-62)
  auto overlap = [](const Position &a, const Position &b) {
    if (a.pos == ~0ull || b.pos == ~0ull) return false;
    return a.remapped_pos == b.remapped_pos && (a.idx_and_end & 1) == (b.idx_and_end & 1);
  };
  size_t i = 0;
  while (i < arr.n) {
    Position pos = arr.a[i];
    const int strand = c.al(arr.a[i]).a;
    const int n_optimal = 1;
    if (i < arr.n - 1) {
      size_t k = i;
      while (overlap(pos, arr.at(k + 1))) ++k;
      if (k > i) {
        pos = select_mapping(c, arr, i, k);
        i = k;
      }
    }
    const int e = pos.idx_and_end & 1;
    if (strand == 1) {
      pairing_aux(c, pi, pi.last_pos[1 - e][1], pos, n_optimal);
      pairing_aux(c, pi, pi.last_pos[1 - e][0], pos, n_optimal);
    } else {
      pi.last_pos[e][0] = pi.last_pos[e][1];
      pi.last_pos[e][1] = pos;
    }
    ++i;
  }
  if (pi.o_score != ~0ull) {
    int mapQ_p = 0;  // the maximum mapping quality when one end is moved
    if (pi.o_n == 1) {
      if (pi.subo_score == ~0ull) {
        mapQ_p = 29;
      } else if ((pi.subo_score >> 32) - (pi.o_score >> 32) > (uint64_t)(int64_t)(c.s_mm * 10)) {
        mapQ_p = 23;
      } else {
        const int n = pi.subo_n > 255 ? 255 : pi.subo_n;
        mapQ_p = (int)(((pi.subo_score >> 32) - (pi.o_score >> 32)) / 2 - (uint64_t)(int64_t)g_log_n[n]);
        if (mapQ_p < 0) mapQ_p = 0;
      }
    }
    const int rr0 = c.al(pi.o_pos[0]).a, rr1 = c.al(pi.o_pos[1]).a;
    const bool keep0 = p[0]->remapped_pos == pi.o_pos[0].remapped_pos && p[0]->strand == rr0;
    const bool keep1 = p[1]->remapped_pos == pi.o_pos[1].remapped_pos && p[1]->strand == rr1;
    if (keep0 && keep1) {
      if (p[0]->mapQ > 0 && p[1]->mapQ > 0) {
        int mapQ = p[0]->mapQ + p[1]->mapQ;
        if (mapQ > 60) mapQ = 60;
        p[0]->mapQ = p[1]->mapQ = mapQ;
      } else {
        if (p[0]->mapQ == 0) p[0]->mapQ = (mapQ_p + 7 < p[1]->mapQ) ? mapQ_p + 7 : p[1]->mapQ;
        if (p[1]->mapQ == 0) p[1]->mapQ = (mapQ_p + 7 < p[0]->mapQ) ? mapQ_p + 7 : p[0]->mapQ;
      }
    } else if (keep0) {
      p[1]->seQ = 0;
      p[1]->mapQ = p[0]->mapQ;
      if (p[1]->mapQ > mapQ_p) p[1]->mapQ = mapQ_p;
    } else if (keep1) {
      p[0]->seQ = 0;
      p[0]->mapQ = p[1]->mapQ;
      if (p[0]->mapQ > mapQ_p) p[0]->mapQ = mapQ_p;
    } else {
      p[0]->seQ = p[1]->seQ = 0;
      mapQ_p -= 20;
      if (mapQ_p < 0) mapQ_p = 0;
      p[0]->mapQ = p[1]->mapQ = mapQ_p;
    }
    p[0]->mapQ &= 0xff;
    p[1]->mapQ &= 0xff;
    pairing_aux2(c, pi, *p[0], pi.o_pos[0]);
    pairing_aux2(c, pi, *p[1], pi.o_pos[1]);
  }
  return pi.cnt_chg;
}

// ---------------------------------------------------------------- insert size (infer_isize, bwape.c:91-198)
int infer_isize(const std::vector<Read> &s0, const std::vector<Read> &s1, Isize &ii, double ap_prior, int64_t L) {
  const int n_seqs = (int)s0.size();
  ii = Isize();
  ii.avg = ii.std = -1.0;
  std::vector<uint64_t> isizes;
  int max_len = 1;
  int n_rej = 0;
  for (int i = 0; i < n_seqs; ++i) {
    const Read *p[2] = {&s0[i], &s1[i]};
    const uint64_t x = p[0]->pos < p[1]->pos ? p[1]->pos + p[1]->len - p[0]->pos : p[0]->pos + p[0]->len - p[1]->pos;
    if (p[0]->mapQ >= 20 && p[1]->mapQ >= 20 && x < 100000) isizes.push_back(x);
    else ++n_rej;
    max_len = std::max(max_len, std::max(p[0]->len, p[1]->len));
  }
  elog("[infer_isize]  total rejected pairs: %d\n", n_rej);
  const int tot = (int)isizes.size();
  if (tot < 20) {
    elog("[infer_isize] fail to infer insert size: too few good pairs\n");
    return -1;
  }
  {  // sorted by counting (every kept size is < 100000): the order the sums below need
    std::vector<uint32_t> cnt(100000, 0);
    for (uint64_t v : isizes) ++cnt[v];
    size_t q = 0;
    for (uint32_t v = 0; v < 100000; ++v)
      for (uint32_t c = cnt[v]; c; --c) isizes[q++] = v;
  }
  const int p25 = (int)isizes[(int)(tot * 0.25 + 0.5)];
  const int p50 = (int)isizes[(int)(tot * 0.50 + 0.5)];
  const int p75 = (int)isizes[(int)(tot * 0.75 + 0.5)];
  const int tmp = (int)(p25 - 2.0 * (p75 - p25) + .499);  // OUTLIER_BOUND
  ii.low = (uint32_t)(tmp > max_len ? tmp : max_len);
  ii.high = (uint32_t)(int)(p75 + 2.0 * (p75 - p25) + .499);
  uint64_t x = 0;
  int n = 0;
  for (int i = 0; i < tot; ++i)
    if (isizes[i] >= ii.low && isizes[i] <= ii.high) ++n, x += isizes[i];
  ii.avg = (double)x / n;
  for (int i = 0; i < tot; ++i)
    if (isizes[i] >= ii.low && isizes[i] <= ii.high) ii.std += (isizes[i] - ii.avg) * (isizes[i] - ii.avg);
  ii.std = sqrt(ii.std / n);
  double y;
  for (y = 1.0; y < 10.0; y += 0.01)
    if (.5 * erfc(y / M_SQRT2) < ap_prior / L * (y * ii.std + ii.avg)) break;
  ii.high_bayesian = (uint32_t)(y * ii.std + ii.avg + .499);
  uint64_t n_ap = 0;
  for (int i = 0; i < tot; ++i)
    if (isizes[i] > ii.high_bayesian) ++n_ap;
  ii.ap_prior = .01 * (n_ap + .01) / tot;
  if (ii.ap_prior < ap_prior) ii.ap_prior = ap_prior;
  elog("[infer_isize] (25, 50, 75) percentile: (%d, %d, %d)\n", p25, p50, p75);
  if (std::isnan(ii.std) || p75 > 100000) {
    ii.low = ii.high = ii.high_bayesian = 0;
    ii.avg = ii.std = -1.0;
    elog("[infer_isize] fail to infer insert size: weird pairing\n");
    return -1;
  }
  for (y = 1.0; y < 10.0; y += 0.01)
    if (.5 * erfc(y / M_SQRT2) < ap_prior / L * (y * ii.std + ii.avg)) break;
  ii.high_bayesian = (uint32_t)(y * ii.std + ii.avg + .499);
  elog("[infer_isize] inferred external isize from %d pairs: %.3lf +/- %.3lf\n", n, ii.avg, ii.std);
  elog("[infer_isize] inferred maximum insert size: %u (%.2lf sigma)\n", ii.high_bayesian, y);
  return 0;
}

// ---------------------------------------------------------------- read sources (bwa_open_reads, bwtaln.c:159-171)
struct Source {
  std::unique_ptr<ibwa_cli::SeqReader> fq;
  std::unique_ptr<ibwa_cli::FastqBulk> fb;  // strict FASTQ records in bulk, before the serial reader
  std::unique_ptr<ibwa_cli::BamReader> bam;
  int mode = 0, trim_qual = 0;
  bool open(const char *fn, const ibwa_gap_opt_t &opt) {
    mode = opt.mode;
    trim_qual = opt.trim_qual;
    if (mode & IBWA_MODE_BAM) {
      int which = 0;
      if (mode & IBWA_MODE_BAM_SE) which |= 4;
      if (mode & IBWA_MODE_BAM_READ1) which |= 1;
      if (mode & IBWA_MODE_BAM_READ2) which |= 2;
      if (which == 0) which = 7;
      bam.reset(new ibwa_cli::BamReader);
      return bam->open(fn, which);
    }
    fq.reset(new ibwa_cli::SeqReader);
    if (!fq->open(fn)) return false;
    if (!getenv("IBWA_SAMPE_SERIAL_READ")) fb.reset(new ibwa_cli::FastqBulk(*fq));
    return true;
  }
  bool next(Read &r) { return bam ? next_read(*bam, mode, trim_qual, r) : next_read(*fq, mode, trim_qual, r); }
  // reads appended to out up to n_max: the bulk parser's records on nt threads, then record by
  // record (the same reads in the same order as next() alone)
  void take(std::vector<Read> &out, size_t n_max, int nt) {
    take_reads(fb.get(), mode, trim_qual, out, n_max, nt, [this](Read &r) { return next(r); });
  }
};

// ---------------------------------------------------------------- the batch loop (bwa_sai2sam_pe_core)
// a host thread's buffers for the positions pass
struct PosScratch {
  PosArr arr;
  std::vector<std::pair<uint64_t, int>> ps;
  std::vector<PosKey> pk;
  std::vector<uint64_t> kk, tk;
  std::vector<uint32_t> ki, tv;
};

// One shard of the batch loop (-G): its GPU contexts, one per reference, and what its batches work
// in, kept from batch to batch.
struct Worker {
  std::vector<ibwa_ctx_t *> ctx;  // per reference: its index, SA -> coordinate
  // every pair's positions, per host thread; kept across batches (a batch holds ~10 M positions,
  // 0.5 GB: allocating, faulting in and freeing that each batch cost about as much as filling it)
  std::vector<std::vector<Position>> pstore;
  std::vector<PosScratch> pscr;  // per host thread
  std::unique_ptr<ibwa_ref_seq_t[]> sw_ref[2];  // paired_sw's bwa_seq_t mirrors per end (capacity kept)
  std::unique_ptr<uint8_t[]> sw_rev[2];
  size_t sw_ref_cap[2] = {0, 0}, sw_rev_cap[2] = {0, 0};
  Phases ph;
};

// A batch of pairs (bwa_read_seq twice, bwape.c:466-468) with its .sai records and what its place
// in the file settles: the drand48 decisions and the first uses of its wide intervals.
struct Batch {
  int64_t idx = 0;
  std::vector<Read> seqs[2];
  std::vector<Aln> flat[2];       // every read's alignments, one flat array per end
  std::vector<size_t> offs[2];    // read i's at flat[offs[i] .. offs[i + 1])
  std::vector<int> midx;          // select_rng per (pair, end) at 2 i + j: the main alignment
  std::vector<double> rcache;     // and the draw that picks its row
  // per reference: each interval of >= kMinHashWidth rows the batch uses -> (strand << 32 | read
  // length) of its first use in the run (the cached positions are computed with those)
  std::vector<std::unordered_map<uint64_t, uint64_t>> wide;
  bool ok[2] = {true, true};  // the .sai records were read whole
};

struct Sampe {
  // bwtcache (bwtcache.c:27-45), one per reference and shared by the -G workers: positions of an
  // interval of >= 1000 rows, keyed by (k, l) only, computed with the strand and read length of the
  // interval's first use in the run (Batch::wide settles those in file order, so every worker that
  // computes an interval gets the same positions)
  std::vector<std::unordered_map<uint64_t, std::shared_ptr<const std::vector<uint64_t>>>> wide_cache;
  std::mutex wide_mu;
  Dbs dbs;
  std::vector<Worker> W;  // -G workers (at least one)
  std::vector<std::vector<const char *>> sai_fn;  // per reference: end 1, end 2
  PeOpt popt;
  ibwa_gap_opt_t gopt[2];
  std::vector<FILE *> fp_sai[2];  // per end, per reference
  std::vector<ibwa_aln1_t> sai_tmp[2];  // per end (the ends are read on two threads)
  Drand48 rnd;
  // per reference: each wide interval's first use so far (in batch order, when a batch is taken)
  std::vector<std::unordered_map<uint64_t, uint64_t>> first_use;
  const char *rg_id = nullptr;
  // batch-to-batch order between the workers: the insert size each batch settled on (for the next
  // batch's fallback), the next batch to print, a failure anywhere
  std::mutex mu;
  std::condition_variable cv;
  std::map<int64_t, Isize> ii_done;
  int64_t printed = 0;
  long tot = 0;
  bool failed = false;

  int max_diff_of(const Read &r) const {
    return gopt[1].fnr > 0.0 ? ibwa_cal_maxdiff(r.len, 0.02, gopt[1].fnr) : gopt[1].max_diff;
  }

  // alngrp_create (saiset.c:45-76): the read's records of every reference; with several
  // references sorted by score (klib's introsort, not stable) and cut at best + s_mm
  // a .sai read in 16 MiB blocks (one fread per block, not two per read)
  struct SaiIn {
    FILE *fp = nullptr;
    std::vector<char> b;
    size_t p = 0, e = 0;
    size_t read(void *dst, size_t n) {  // bytes copied (< n: the file ended)
      size_t got = 0;
      char *d = static_cast<char *>(dst);
      while (got < n) {
        if (p == e) {
          if (b.empty()) b.resize((size_t)16 << 20);
          p = 0;
          e = fread(b.data(), 1, b.size(), fp);
          if (e == 0) break;
        }
        const size_t k = std::min(n - got, e - p);
        memcpy(d + got, b.data() + p, k);
        p += k;
        got += k;
      }
      return got;
    }
  };
  std::vector<SaiIn> sai_in[2];  // per end, per reference: over fp_sai

  bool read_alns(int j, std::vector<Aln> &flat) {
    const size_t first = flat.size();
    std::vector<Aln> &v = flat;
    if (sai_in[j].size() != fp_sai[j].size()) {
      sai_in[j].resize(fp_sai[j].size());
      for (size_t d = 0; d < fp_sai[j].size(); ++d) sai_in[j][d].fp = fp_sai[j][d];
    }
    for (size_t d = 0; d < fp_sai[j].size(); ++d) {
      uint32_t count = 0;
      if (sai_in[j][d].read(&count, 4) != 4) continue;  // past the end: nothing
      const size_t o = v.size();
      v.resize(o + count);
      sai_tmp[j].resize(count);  // the read's records in one read
      if (count && sai_in[j][d].read(sai_tmp[j].data(), sizeof(ibwa_aln1_t) * count) != sizeof(ibwa_aln1_t) * count) {
        fprintf(stderr, "[ibwa-amd sampe] truncated .sai\n");
        return false;
      }
      for (uint32_t t = 0; t < count; ++t) {
        v[o + t].aln = sai_tmp[j][t];
        v[o + t].dbidx = (int)d;
      }
    }
    if (fp_sai[j].size() > 1 && v.size() > first) {
      Aln *a = v.data() + first;
      const size_t m = v.size() - first;
      ks_introsort(m, a, [](const Aln &x, const Aln &y) { return x.aln.score < y.aln.score; });
      const int best = a[0].aln.score;
      for (size_t t = 0; t < m; ++t)
        if (a[t].aln.score > best + gopt[0].s_mm) {
          v.resize(first + t);
          break;
        }
    }
    return true;
  }

  static void unmap(Read &s) {  // UNMAP_READ (bwape.c:48-56)
    s.type = TYPE_NO_MATCH;
    s.pos = s.remapped_pos = s.sa = s.c1 = s.c2 = 0;
    s.cigar.clear();
    s.has_cigar = false;
  }

  // SA rows -> positions (bwtdb_sa2seq, dbset.c:240-246), one launch per reference
  int sa2pos(Worker &w, const std::vector<int> &db, const std::vector<uint8_t> &st, const std::vector<uint32_t> &k,
             const std::vector<uint32_t> &len, std::vector<uint64_t> &pos) {
    const std::vector<ibwa_ctx_t *> &ctx = w.ctx;
    pos.assign(k.size(), 0);
    if (ctx.size() == 1) {  // one reference: the lists as they are
      if (!k.empty() && ibwa_sa2pos(ctx[0], (int64_t)k.size(), st.data(), k.data(), len.data(), dbs.db[0].offset, pos.data()))
        return die("sa2pos");
      return 0;
    }
    for (size_t d = 0; d < ctx.size(); ++d) {
      std::vector<size_t> idx;
      for (size_t t = 0; t < k.size(); ++t)
        if (db[t] == (int)d) idx.push_back(t);
      if (idx.empty()) continue;
      std::vector<uint8_t> s2(idx.size());
      std::vector<uint32_t> k2(idx.size()), l2(idx.size());
      std::vector<uint64_t> p2(idx.size());
      for (size_t t = 0; t < idx.size(); ++t) { s2[t] = st[idx[t]]; k2[t] = k[idx[t]]; l2[t] = len[idx[t]]; }
      if (ibwa_sa2pos(ctx[d], (int64_t)idx.size(), s2.data(), k2.data(), l2.data(), dbs.db[d].offset, p2.data()))
        return die("sa2pos");
      for (size_t t = 0; t < idx.size(); ++t) pos[idx[t]] = p2[t];
    }
    return 0;
  }

  // remap (bwape.c:223-235) of a hit at pos on reference dbidx; status untouched without -R
  template <class T>
  void remap(T &p, uint64_t pos, int dbidx, uint64_t len, uint32_t gap, int *status) {
    p.dbidx = dbidx;
    p.remapped_dbidx = 0;
    if (popt.remapping) {
      p.remapped_pos = remap_pos(dbs, dbidx, pos, len, gap, &p.remapped_seqid, &p.remap_identical, status);
    } else {
      p.remapped_pos = pos;
      p.remapped_seqid = -1;
    }
  }

  // select_sai_ibwa (bwape.c:299-369) up to the coordinate: the RNG decisions, the main alignment
  // and the first SA row to try; returns false when the read is unmapped without a try.
  struct Pick {
    int main_idx = 0;
    uint32_t start = 0, num = 0;
  };
  // the drand48 decisions of select_sai_ibwa (bwape.c:305-318): the main alignment and the draw
  // that picks its row.  The only sequential part of the hit choice.
  void select_rng(const AlnSpan &ag, int &main_idx, double &rng_cache) {
    main_idx = 0;
    rng_cache = 0.0;
    if (ag.empty()) return;
    const int best = ag[0].aln.score;
    int cnt = 0;
    for (int i = 0; i < (int)ag.size(); ++i) {
      const ibwa_aln1_t &p = ag[i].aln;
      if (p.score > best) break;
      if (rnd.next() * (double)(uint32_t)(p.l - p.k + 1 + (uint32_t)cnt) > (double)cnt) {
        main_idx = i;
        rng_cache = rnd.next();
      }
      cnt += (int)(p.l - p.k + 1);
    }
  }
  // the rest of select_sai_ibwa up to the coordinate (bwape.c:319-335): counts, type, the main
  // alignment's fields and first SA row; false when the read is unmapped without a try
  bool select_sai(const AlnSpan &ag, Read &s, Pick &pk, int main_idx, double rng_cache) {
    if (ag.empty()) {
      unmap(s);
      return false;
    }
    int i, cnt;
    const int best = ag[0].aln.score;
    for (i = cnt = 0; i < (int)ag.size(); ++i) {
      const ibwa_aln1_t &p = ag[i].aln;
      if (p.score > best) break;
      cnt += (int)(p.l - p.k + 1);
    }
    s.c1 = (uint32_t)cnt & 0xfffffffu;
    for (int t = i; t < (int)ag.size(); ++t) cnt += (int)(ag[t].aln.l - ag[t].aln.k + 1);
    s.c2 = ((uint32_t)cnt - s.c1) & 0xfffffffu;
    if (s.c1 != 0) s.type = s.c1 > 1 ? TYPE_REPEAT : TYPE_UNIQUE;
    const ibwa_aln1_t &p = ag[main_idx].aln;
    const uint32_t num = p.l - p.k + 1;
    const uint32_t start = (uint32_t)(rng_cache * num);
    s.n_mm = p.n_mm; s.n_gapo = p.n_gapo; s.n_gape = p.n_gape; s.strand = p.a;
    s.score = p.score;
    if (!popt.remapping) {  // remap() never reports success: every row, then UNMAP_READ
      s.sa = p.k + (start == 0 ? num - 1 : start - 1);
      s.dbidx = ag[main_idx].dbidx;
      s.remapped_dbidx = 0;
      s.remapped_seqid = -1;
      unmap(s);
      msg("Failed to select primary alignment for %s\n", s.name.c_str());
      return false;
    }
    s.sa = p.k + start;
    pk.main_idx = main_idx;
    pk.start = start;
    pk.num = num;
    return true;
  }

  // The batches of 0x40000 pairs (bwa_read_seq twice, bwape.c:466-468) with their .sai records, end
  // 1 and end 2 on two threads, read ahead by a reader thread into a queue of up to `depth` batches:
  // the first ones while the index loads, later ones while the batches before them are processed
  // (with several workers one batch ahead left a worker waiting whenever two finished close together).
  size_t batch_pairs = 0x40000;  // IBWA_SAMPE_BATCH: other sizes are for tests (the SAM depends on it)
  size_t depth = 2;              // IBWA_SAMPE_READ_AHEAD
  double rd_s[2][2] = {{0, 0}, {0, 0}};  // per end: seconds reading reads, reading .sai records
  std::mutex rq_mu;
  std::condition_variable rq_cv;
  std::deque<std::unique_ptr<Batch>> ready;  // read, in file order; an empty or failed one ends it
  std::vector<std::unique_ptr<Batch>> spare;  // taken and done: buffers for the reader to refill
  bool stop_reading = false;
  std::thread reader;
  void read_into(Source *src, Batch &nb) {
    auto rd = [this, src, &nb](int j) {
      const auto t0 = std::chrono::steady_clock::now();
      nb.seqs[j].reserve(batch_pairs);
      src[j].take(nb.seqs[j], batch_pairs, std::max(1, host_threads() / 2));
      const auto t1 = std::chrono::steady_clock::now();
      // alngrp_create per read, in read order (saiset.c:45-76)
      const size_t n = nb.seqs[j].size();
      nb.flat[j].clear();
      nb.flat[j].reserve(n + n / 4);
      nb.offs[j].assign(n + 1, 0);
      nb.ok[j] = true;
      for (size_t i = 0; i < n && nb.ok[j]; ++i) {
        nb.offs[j][i] = nb.flat[j].size();
        nb.ok[j] = read_alns((int)j, nb.flat[j]);
        nb.offs[j][i + 1] = nb.flat[j].size();
      }
      const auto t2 = std::chrono::steady_clock::now();
      rd_s[j][0] += std::chrono::duration<double>(t1 - t0).count();
      rd_s[j][1] += std::chrono::duration<double>(t2 - t1).count();
    };
    std::thread t1(rd, 1);
    rd(0);
    t1.join();
  }
  void start_reading(Source *src) {
    reader = std::thread([this, src]() {
      for (;;) {
        std::unique_ptr<Batch> nb;
        {
          std::unique_lock<std::mutex> l(rq_mu);
          rq_cv.wait(l, [&] { return stop_reading || ready.size() < depth; });
          if (stop_reading) return;
          if (!spare.empty()) {
            nb = std::move(spare.back());
            spare.pop_back();
          } else {
            nb.reset(new Batch);
          }
        }
        read_into(src, *nb);
        const bool last = nb->seqs[0].empty() || !nb->ok[0] || !nb->ok[1];
        {
          std::lock_guard<std::mutex> l(rq_mu);
          ready.push_back(std::move(nb));
        }
        rq_cv.notify_all();
        if (last) return;
      }
    });
  }
  ~Sampe() { stop_reader(); }
  void stop_reader() {
    {
      std::lock_guard<std::mutex> l(rq_mu);
      stop_reading = true;
    }
    rq_cv.notify_all();
    if (reader.joinable()) reader.join();
  }

  // The next batch in file order into b (b's previous batch goes back to the reader), with the
  // decisions the reference makes in batch order; one worker at a time.  1: a batch, 0: the end, -1:
  // an error.
  int take(Worker &w, std::unique_ptr<Batch> &bp, int64_t idx) {
    {
      std::unique_lock<std::mutex> l(rq_mu);
      if (bp) spare.push_back(std::move(bp));
      rq_cv.wait(l, [&] { return !ready.empty(); });
      const Batch &f = *ready.front();
      if (f.seqs[0].empty()) return 0;  // left in the queue: the end for every worker
      if (!f.ok[0] || !f.ok[1]) return -1;
      bp = std::move(ready.front());
      ready.pop_front();
    }
    rq_cv.notify_all();
    w.ph.mark("read (wait)");
    Batch &b = *bp;
    if (b.seqs[1].size() != b.seqs[0].size()) {
      fprintf(stderr, "[ibwa-amd sampe] the two read files hold different numbers of reads\n");
      return -1;
    }
    b.idx = idx;
    const int n = (int)b.seqs[0].size();
    auto span = [&b](int j, int i) { return AlnSpan{b.flat[j].data() + b.offs[j][i], b.offs[j][i + 1] - b.offs[j][i]}; };
    b.midx.resize(2 * (size_t)n);
    b.rcache.resize(2 * (size_t)n);
    for (int i = 0; i < n; ++i)  // the drand48 stream, in pair order
      for (int j = 0; j < 2; ++j) select_rng(span(j, i), b.midx[2 * i + j], b.rcache[2 * i + j]);
    w.ph.mark("hit choice: drand48");
    b.wide.resize(dbs.db.size());
    for (auto &m : b.wide) m.clear();
    if (popt.remapping) {  // the wide intervals' first uses in (pair, end, alignment) order
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < 2; ++j)
          for (const Aln &al : span(j, i)) {
            const ibwa_aln1_t &a = al.aln;
            if (a.l - a.k + 1 < kMinHashWidth) continue;
            const uint64_t key = (uint64_t)a.k << 32 | a.l;
            const uint64_t use = (uint64_t)a.a << 32 | (uint32_t)b.seqs[j][i].len;
            b.wide[al.dbidx].emplace(key, first_use[al.dbidx].emplace(key, use).first->second);
          }
      w.ph.mark("rows: first uses");
    }
    return 1;
  }

  // the batch-to-batch waits: false when a worker failed
  bool wait_ii(int64_t idx, Isize &ii) {
    if (idx < 0) {
      ii = Isize();
      return true;
    }
    std::unique_lock<std::mutex> l(mu);
    cv.wait(l, [&] { return failed || ii_done.count(idx) != 0; });
    if (failed) return false;
    ii = ii_done[idx];
    return true;
  }
  void publish_ii(int64_t idx, const Isize &ii) {
    std::lock_guard<std::mutex> l(mu);
    ii_done[idx] = ii;  // kept: a slower worker's batch idx + 1 may ask for it late
    cv.notify_all();
  }
  bool wait_turn(int64_t idx) {
    std::unique_lock<std::mutex> l(mu);
    cv.wait(l, [&] { return failed || printed == idx; });
    return !failed;
  }
  void end_turn(int n) {
    std::lock_guard<std::mutex> l(mu);
    tot += n;
    if (std::string *b = batch_log()) {  // the batch's messages, in file order with the SAM
      fputs(b->c_str(), stderr);
      b->clear();
    }
    fprintf(stderr, "[bwa_sai2sam_pe_core] %ld sequences have been processed.\n", tot);
    ++printed;
    cv.notify_all();
  }
  void fail() {
    std::lock_guard<std::mutex> l(mu);
    failed = true;
    cv.notify_all();
  }

  int run(FILE *out) {
    Out o{out, {}};
    std::mutex take_mu;
    bool end = false;
    int64_t n_taken = 0;
    std::vector<int> rcs(W.size(), 0);
    auto work = [&](int wi) {
      Worker &w = W[wi];
      std::unique_ptr<Batch> b;  // the batch in hand (its buffers go back to the reader)
      for (;;) {
        {
          std::lock_guard<std::mutex> l(take_mu);
          if (end) return;
          {
            std::lock_guard<std::mutex> l2(mu);
            if (failed) return;
          }
          const int t = take(w, b, n_taken);
          if (t == 0) {
            end = true;
            return;
          }
          if (t < 0) {
            rcs[wi] = 1;
            end = true;
            fail();
            return;
          }
          ++n_taken;
        }
        std::string log;  // this batch's stderr, printed with its SAM (end_turn)
        batch_log() = &log;
        const int brc = batch(w, *b, o);
        batch_log() = nullptr;
        if (!log.empty()) fputs(log.c_str(), stderr);  // an error return: what the batch said so far
        if (int rc = brc) {
          rcs[wi] = rc;
          fail();
          return;
        }
      }
    };
    std::vector<std::thread> th;
    for (size_t wi = 1; wi < W.size(); ++wi) th.emplace_back(work, (int)wi);
    work(0);
    for (auto &t : th) t.join();
    stop_reader();
    for (int rc : rcs)
      if (rc) return rc;
    o.flush();
    for (size_t wi = 0; wi < W.size(); ++wi) {
      char who[48];
      if (W.size() == 1) snprintf(who, sizeof who, "ibwa-amd sampe");
      else snprintf(who, sizeof who, "ibwa-amd sampe worker %zu", wi);
      W[wi].ph.print(who);
    }
    fprintf(stderr, "[ibwa-amd sampe] read-ahead thread s: end 1 reads %.2f .sai %.2f, end 2 reads %.2f .sai %.2f\n",
            rd_s[0][0], rd_s[0][1], rd_s[1][0], rd_s[1][1]);
    return 0;
  }

  int batch(Worker &wk, Batch &bt, Out &o) {
    Phases &ph = wk.ph;
    std::vector<Read> *seqs = bt.seqs;
    const int n = (int)seqs[0].size();
    // every read's alignments in one flat array per end (alns[j][i] slices it), read with the batch
    std::vector<AlnSpan> alns[2];
    // ---- SE (bwa_cal_pac_pos_pe, bwape.c:366-385): hit choice in pair order (the drand48 stream),
    // one SA->pos launch per reference, then remap() on the host threads; the main alignment's other
    // rows for the reads whose remap failed, in one more launch per reference
    std::vector<Pick> pick[2];
    std::vector<uint8_t> chosen[2];
    for (int j = 0; j < 2; ++j) {
      pick[j].assign(n, Pick());
      chosen[j].assign(n, 0);
    }
    for (int j = 0; j < 2; ++j) {
      alns[j].resize(n);
      for (int i = 0; i < n; ++i)
        alns[j][i] = AlnSpan{bt.flat[j].data() + bt.offs[j][i], bt.offs[j][i + 1] - bt.offs[j][i]};
    }
    {
      const std::vector<int> &midx = bt.midx;  // the drand48 decisions, made when the batch was taken
      const std::vector<double> &rcache = bt.rcache;
      parallel_ordered(n, [&](int64_t lo, int64_t hi_, int) {
        for (int64_t i = lo; i < hi_; ++i)
          for (int j = 0; j < 2; ++j) {
            Read &p = seqs[j][i];
            p.multi.clear();
            p.extra_flag |= SAM_FPD | (j == 0 ? SAM_FR1 : SAM_FR2);
            chosen[j][i] = select_sai(alns[j][i], p, pick[j][i], midx[2 * i + j], rcache[2 * i + j]) ? 1 : 0;
          }
      }, 0, 1024);
      ph.mark("hit choice: select");
    }
    std::vector<int> hd;
    std::vector<uint8_t> hs;
    std::vector<uint32_t> hk, hl;
    std::vector<int> hi;  // (pair, end) as 2 i + j
    {
      // the chosen hits in (pair, end) order: counts per thread's range of pairs, then filled in place
      // (parallel_chunks splits [0, n) the same way both times)
      const int nt = host_threads();
      std::vector<int64_t> c0(nt + 1, 0);
      parallel_chunks(n, [&](int64_t lo, int64_t hi_, int t) {
        int64_t c = 0;
        for (int64_t i = lo; i < hi_; ++i) c += chosen[0][i] + chosen[1][i];
        c0[t + 1] = c;
      }, nt);
      for (int t = 0; t < nt; ++t) c0[t + 1] += c0[t];
      hd.resize(c0[nt]); hs.resize(c0[nt]); hk.resize(c0[nt]); hl.resize(c0[nt]); hi.resize(c0[nt]);
      parallel_chunks(n, [&](int64_t lo, int64_t hi_, int t) {
        int64_t o = c0[t];
        for (int64_t i = lo; i < hi_; ++i)
          for (int j = 0; j < 2; ++j)
            if (chosen[j][i]) {
              const Read &p = seqs[j][i];
              hd[o] = alns[j][i][pick[j][i].main_idx].dbidx;
              hs[o] = (uint8_t)p.strand; hk[o] = p.sa; hl[o] = (uint32_t)p.len;
              hi[o++] = (int)(2 * i + j);
            }
      }, nt);
    }
    ph.mark("hit choice: row lists");
    std::vector<uint64_t> pos;
    if (int rc = sa2pos(wk, hd, hs, hk, hl, pos)) return rc;
    ph.mark("sa2pos: kernel");
    std::vector<uint8_t> ok(hi.size(), 0);
    auto remap_main = [&](size_t t) {
      const int i = hi[t] >> 1, j = hi[t] & 1;
      Read &p = seqs[j][i];
      const Aln &ma = alns[j][i][pick[j][i].main_idx];
      int status = 0;
      p.pos = pos[t];
      remap(p, p.pos, ma.dbidx, (uint64_t)p.len, (uint32_t)(p.n_gapo + p.n_gape), &status);
      ok[t] = status == 1;
    };
    parallel_ordered((int64_t)hi.size(), [&](int64_t lo, int64_t hi_, int) {
      for (int64_t t = lo; t < hi_; ++t) remap_main((size_t)t);
    });
    ph.mark("sa2pos: remap");
    // the other rows of the main alignment, cyclically from the chosen one (bwape.c:336-357), for
    // the reads whose remap failed: their rows in one launch per reference (bounded per launch)
    {
      std::vector<size_t> fail;
      for (size_t t = 0; t < hi.size(); ++t)
        if (!ok[t] && pick[hi[t] & 1][hi[t] >> 1].num > 1) fail.push_back(t);
      size_t f0 = 0;
      while (f0 < fail.size()) {
        std::vector<int> d1;
        std::vector<uint8_t> s1;
        std::vector<uint32_t> k1, l1;
        std::vector<size_t> first;
        size_t f1 = f0;
        for (; f1 < fail.size() && (f1 == f0 || k1.size() < ((size_t)1 << 22)); ++f1) {
          const int i = hi[fail[f1]] >> 1, j = hi[fail[f1]] & 1;
          const Read &p = seqs[j][i];
          const Pick &pk = pick[j][i];
          const Aln &ma = alns[j][i][pk.main_idx];
          first.push_back(k1.size());
          for (uint32_t step = 1; step < pk.num; ++step) {
            d1.push_back(ma.dbidx); s1.push_back((uint8_t)p.strand);
            k1.push_back(ma.aln.k + (pk.start + step) % pk.num); l1.push_back((uint32_t)p.len);
          }
        }
        std::vector<uint64_t> p1;
        if (int rc = sa2pos(wk, d1, s1, k1, l1, p1)) return rc;
        parallel_ordered((int64_t)(f1 - f0), [&](int64_t lo, int64_t hi_, int) {
          for (int64_t u = lo; u < hi_; ++u) {
            const size_t t = fail[f0 + u];
            const int i = hi[t] >> 1, j = hi[t] & 1;
            Read &p = seqs[j][i];
            const Pick &pk = pick[j][i];
            const Aln &ma = alns[j][i][pk.main_idx];
            int status = 0;
            for (uint32_t step = 1; status != 1 && step < pk.num; ++step) {
              p.sa = ma.aln.k + (pk.start + step) % pk.num;
              p.pos = p1[first[u] + step - 1];
              remap(p, p.pos, ma.dbidx, (uint64_t)p.len, (uint32_t)(p.n_gapo + p.n_gape), &status);
            }
            ok[t] = status == 1;
          }
        });
        f0 = f1;
      }
    }
    parallel_ordered((int64_t)hi.size(), [&](int64_t lo, int64_t hi_, int) {
      for (int64_t t = lo; t < hi_; ++t) {
        Read &p = seqs[hi[t] & 1][hi[t] >> 1];
        if (!ok[t]) {
          unmap(p);
          msg("Failed to select primary alignment for %s\n", p.name.c_str());
          continue;
        }
        p.seQ = p.mapQ = approx_mapQ(p, max_diff_of(p)) & 0xff;
      }
    }, 0, 4096);
    ph.mark("sa2pos");
    // ---- insert size
    Isize ii;
    infer_isize(seqs[0], seqs[1], ii, popt.ap_prior, (int64_t)dbs.l_pac);
    if (ii.avg < 0.0) {  // the previous batch's, as it ended up (bwape.c:410-411)
      Isize last_ii;
      if (!wait_ii(bt.idx - 1, last_ii)) return 1;
      if (last_ii.avg > 0.0) ii = last_ii;
    }
    if (popt.force_isize) {
      elog("[bwa_cal_pac_pos_pe] discard insert size estimate as user's request.\n");
      ii.low = ii.high = 0;
      ii.avg = ii.std = -1.0;
    }
    publish_ii(bt.idx, ii);
    ph.mark("isize");
    // ---- every row of every interval (compute_seq_coords_and_counts): one SA->pos launch per
    // reference.  Rows of intervals narrower than kMinHashWidth are computed per (read, alignment);
    // wider ones come from the reference's cache, filled on first use with that caller's strand
    // and read length.
    std::vector<int64_t> row0[2];  // per (pair, end): first alignment slot in aslot
    std::vector<int64_t> aslot;    // per alignment: first row in rows (-1: cached)
    hd.clear(); hs.clear(); hk.clear(); hl.clear();
    std::vector<std::pair<std::pair<int, uint64_t>, int64_t>> fill;  // new cache keys -> first row
    // this batch's wide intervals (per reference) -> their positions in the shared cache
    std::vector<std::unordered_map<uint64_t, std::shared_ptr<const std::vector<uint64_t>>>> bc(wide_cache.size());
    if (popt.remapping) {
      // alignment slots in (pair, end, alignment) order; the narrow intervals' rows at offsets from
      // per-pair counts, filled on the host threads; then the wide ones in pair order (the first use
      // of an interval fills the cache), behind them
      for (int j = 0; j < 2; ++j) row0[j].assign(n + 1, 0);
      int64_t na = 0;
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < 2; ++j) {
          row0[j][i] = na;
          na += (int64_t)alns[j][i].size();
        }
      aslot.assign(na, -1);
      std::vector<int64_t> r0(n + 1, 0);
      parallel_chunks(n, [&](int64_t lo, int64_t hi_, int) {
        for (int64_t i = lo; i < hi_; ++i) {
          int64_t c = 0;
          for (int j = 0; j < 2; ++j)
            for (const Aln &al : alns[j][i]) {
              const uint32_t w = al.aln.l - al.aln.k + 1;
              if (w < kMinHashWidth) c += w;
            }
          r0[i + 1] = c;
        }
      });
      for (int i = 0; i < n; ++i) r0[i + 1] += r0[i];
      hd.resize(r0[n]); hs.resize(r0[n]); hk.resize(r0[n]); hl.resize(r0[n]);
      parallel_chunks(n, [&](int64_t lo, int64_t hi_, int) {
        for (int64_t i = lo; i < hi_; ++i) {
          int64_t o = r0[i];
          for (int j = 0; j < 2; ++j) {
            const AlnSpan &ag = alns[j][i];
            for (size_t k = 0; k < ag.size(); ++k) {
              const ibwa_aln1_t &a = ag[k].aln;
              const uint32_t w = a.l - a.k + 1;
              if (w >= kMinHashWidth) continue;
              aslot[row0[j][i] + (int64_t)k] = o;
              for (uint32_t r = 0; r < w; ++r, ++o) {
                hd[o] = ag[k].dbidx; hs[o] = (uint8_t)a.a; hk[o] = a.k + r; hl[o] = (uint32_t)seqs[j][i].len;
              }
            }
          }
        }
      });
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < 2; ++j)
          for (const Aln &al : alns[j][i]) {
            const ibwa_aln1_t &a = al.aln;
            const uint32_t w = a.l - a.k + 1;
            if (w < kMinHashWidth) continue;
            const uint64_t key = (uint64_t)a.k << 32 | a.l;
            if (bc[al.dbidx].count(key)) continue;
            {
              std::lock_guard<std::mutex> l(wide_mu);
              auto it = wide_cache[al.dbidx].find(key);
              if (it != wide_cache[al.dbidx].end()) {
                bc[al.dbidx][key] = it->second;
                continue;
              }
            }
            fill.push_back({{al.dbidx, key}, (int64_t)hk.size()});
            bc[al.dbidx][key];  // reserve: later uses in this batch share it
            const uint64_t use = bt.wide[al.dbidx].at(key);  // the run's first use: its strand, read length
            for (uint32_t r = 0; r < w; ++r) {
              hd.push_back(al.dbidx); hs.push_back((uint8_t)(use >> 32)); hk.push_back(a.k + r);
              hl.push_back((uint32_t)use);
            }
          }
    }
    ph.mark("rows");
    if (int rc = sa2pos(wk, hd, hs, hk, hl, pos)) return rc;
    ph.mark("rows: sa2pos kernel");
    for (auto &f : fill) {
      const uint32_t k = (uint32_t)(f.first.second >> 32), l = (uint32_t)f.first.second;
      auto v = std::make_shared<const std::vector<uint64_t>>(pos.begin() + f.second, pos.begin() + f.second + (l - k + 1));
      std::lock_guard<std::mutex> lk(wide_mu);
      // a worker that missed the same interval meanwhile computed the same positions (the first use
      // fixes strand and length): the first one stored is kept
      bc[f.first.first][f.first.second] = wide_cache[f.first.first].emplace(f.first.second, std::move(v)).first->second;
    }
    ph.mark("rows: cache");
    // ---- select_sai_multi's rows that the -R pass did not compute (no -R, or a cached interval):
    // for every read that can take the multi list (n_occ <= max(n, N) + 1), in one launch
    std::vector<int64_t> mfirst[2];
    std::vector<uint64_t> mpos;
    if (popt.N_multi || popt.n_multi) {
      const int cap = std::max(popt.n_multi, popt.N_multi) + 1;
      hd.clear(); hs.clear(); hk.clear(); hl.clear();
      for (int j = 0; j < 2; ++j) {
        mfirst[j].assign(n, -1);
        for (int i = 0; i < n; ++i) {
          const AlnSpan &ag = alns[j][i];
          int n_occ = 0;
          for (const Aln &q : ag) n_occ += (int)(q.aln.l - q.aln.k + 1);
          if (ag.empty() || n_occ > cap) continue;
          mfirst[j][i] = (int64_t)hk.size();
          const int64_t slot0 = row0[j].empty() ? -1 : row0[j][i];
          for (size_t k = 0; k < ag.size(); ++k) {
            if (slot0 >= 0 && aslot[slot0 + (int64_t)k] >= 0) continue;
            const ibwa_aln1_t &q = ag[k].aln;
            for (uint32_t r = 0; r < q.l - q.k + 1; ++r) {
              hd.push_back(ag[k].dbidx); hs.push_back((uint8_t)q.a); hk.push_back(q.k + r);
              hl.push_back((uint32_t)seqs[j][i].len);
            }
          }
        }
      }
      if (int rc = sa2pos(wk, hd, hs, hk, hl, mpos)) return rc;
    }
    ph.mark("multi rows");
    // ---- PE (bwa_cal_pac_pos_pe_thread, bwape.c:238-297) on the host threads, in three passes so
    // that find_optimal_pair's look-ahead past a pair's positions sees what the reference's one
    // shared array holds there: (A) every pair's positions, counts and sort; (B) each pair's nearest
    // earlier pair with more positions; (C) the pairing itself and select_sai_multi.
    const int nth = host_threads();
    std::vector<std::vector<Position>> &pstore = wk.pstore;  // every pair's positions, per host thread
    pstore.resize(std::max<size_t>(pstore.size(), (size_t)nth));
    for (auto &v : pstore) v.clear();
    std::vector<uint32_t> pcnt(n, 0);
    std::vector<uint64_t> poff(n, 0);
    std::vector<int> pth(n, 0);
    std::vector<uint8_t> paired(n, 0);
    static const bool pstats = getenv("IBWA_SAMPE_STATS") != nullptr;
    const bool fit32 = dbs.l_pac < (1ull << 32);  // positions (and remapped ones) in 32 bits: radix keys
    std::atomic<int64_t> t_pos{0}, t_cnt{0}, t_sort{0};  // ns in the rows' remap, the c1 / c2 count, the sort
    auto now_ns = []() {
      return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    wk.pscr.resize(std::max(wk.pscr.size(), (size_t)nth));
    parallel_ordered(n, [&](int64_t lo, int64_t hi_, int th) {
      // this host thread's scratch, kept across chunks and batches (a pair of a repeat holds up to
      // ~160 k positions: fresh buffers per chunk were page-faulted in again and again)
      PosScratch &sc = wk.pscr[th];
      PosArr &arr = sc.arr;
      std::vector<std::pair<uint64_t, int>> &ps = sc.ps;
      std::vector<PosKey> &pk = sc.pk;
      std::vector<uint64_t> &kk = sc.kk, &tk = sc.tk;
      std::vector<uint32_t> &ki = sc.ki, &tv = sc.tv;
      int64_t a_pos = 0, a_cnt = 0, a_sort = 0;
      for (int64_t i = lo; i < hi_; ++i) {
        Read *p[2] = {&seqs[0][i], &seqs[1][i]};
        arr.clear();
        int64_t t0 = pstats ? now_ns() : 0;
        if (popt.remapping) {
          for (int j = 0; j < 2; ++j) {
            // compute_seq_coords_and_counts (filter_alignments.cpp:53-140): positions inside their
            // reference, remapped; per distinct remapped position the lowest score seen there; c1 / c2
            // count the positions whose lowest score is / is not the best
            ps.clear();
            int min_score = INT32_MAX;
            const AlnSpan &ag = alns[j][i];
            // one alignment on a reference without a remapping table: its rows' positions are distinct
            // (distinct suffixes) and unmoved, and all score the same -- c1 = the positions kept, c2 = 0,
            // no sort (the repeats' long lists are mostly such ends)
            const bool one = ag.size() == 1 && !dbs.db[ag[0].dbidx].remap;
            size_t n_one = 0;
            for (size_t k = 0; k < ag.size(); ++k) {
              const ibwa_aln1_t &a = ag[k].aln;
              const int d = ag[k].dbidx;
              const RefDb &rdb = dbs.db[d];
              min_score = std::min(min_score, a.score);
              const uint32_t w = a.l - a.k + 1;
              const int64_t slot = aslot[row0[j][i] + (int64_t)k];
              const uint64_t *pp = slot < 0 ? bc[d].find((uint64_t)a.k << 32 | a.l)->second->data() : pos.data() + slot;
              for (uint32_t r = 0; r < w; ++r) {
                const uint64_t x = pp[r];
                if (x < rdb.offset || x >= rdb.offset + (uint64_t)rdb.bns.l_pac) continue;
                Position ap;
                ap.pos = x;
                ap.len = p[j]->len;
                ap.n_gape = a.n_gape;
                ap.n_gapo = a.n_gapo;
                ap.score = a.score;
                int status = 0;
                remap(ap, x, d, (uint64_t)ap.len, (uint32_t)(ap.n_gapo + ap.n_gape), &status);
                if (!status) continue;
                ap.idx_and_end = (uint32_t)k << 1 | (uint32_t)j;
                arr.push(ap);
                if (one) ++n_one;
                else ps.push_back({ap.remapped_pos, a.score});
              }
            }
            const int64_t t1 = pstats ? now_ns() : 0;
            if (pstats) a_pos += t1 - t0;
            // c1 / c2 below need the positions grouped, each group's lowest score first: a sort
            // by (remapped position, score), on one 64-bit key when the values fit
            size_t c[2] = {n_one, 0};
            if (!one) {
              bool sc20 = true;
              for (const auto &x : ps) sc20 = sc20 && (unsigned)x.second < (1u << 20);
              if (ps.size() > 256 && fit32 && sc20) {
                kk.resize(ps.size());
                for (size_t t = 0; t < ps.size(); ++t) kk[t] = ps[t].first << 20 | (uint64_t)(ps[t].second & 0xFFFFF);
                radix_sort_u64(kk.size(), kk.data(), nullptr, tk, tv);
                for (size_t t = 0; t < ps.size(); ++t) ps[t] = {kk[t] >> 20, (int)(kk[t] & 0xFFFFF)};
              } else {
                std::sort(ps.begin(), ps.end());
              }
              for (size_t t = 0; t < ps.size(); ++t)
                if (t == 0 || ps[t].first != ps[t - 1].first) ++c[ps[t].second == min_score ? 0 : 1];
            }
            p[j]->c1 = (uint32_t)c[0] & 0xfffffffu;
            p[j]->c2 = (uint32_t)c[1] & 0xfffffffu;
            if (p[j]->c1 != 0) p[j]->type = p[j]->c1 > 1 ? TYPE_REPEAT : TYPE_UNIQUE;
            if (pstats) {
              const int64_t t2 = now_ns();
              a_cnt += t2 - t1;
              t0 = t2;
            }
          }
        }
        for (int j = 0; j < 2; ++j)
          if (p[j]->c1 || p[j]->c2) p[j]->seQ = p[j]->mapQ = approx_mapQ(*p[j], max_diff_of(*p[j])) & 0xff;
        const bool m0 = p[0]->type == TYPE_UNIQUE || p[0]->type == TYPE_REPEAT;
        const bool m1 = p[1]->type == TYPE_UNIQUE || p[1]->type == TYPE_REPEAT;
        paired[i] = m0 && m1;
        // the pair's positions go to this thread's store, sorted for find_optimal_pair when paired:
        // gathered there in sorted order through a permutation when one is computed
        std::vector<Position> &st = pstore[th];
        const uint32_t *perm = nullptr;
        if (paired[i]) {  // find_optimal_pair's sort
          bool done = false;
          if (arr.n > 256 && fit32) {
            // no two positions with the same (remapped position, position): then the sorted order is
            // unique and a radix sort gives the introsort's; with such ties the introsort decides.
            // Without remapping (every remapped position == its position) the key is the position
            // alone: the same order and the same ties, in half the radix passes.
            bool plain = true;
            for (size_t t = 0; t < arr.n && plain; ++t) plain = arr.a[t].remapped_pos == arr.a[t].pos;
            kk.resize(arr.n);
            ki.resize(arr.n);
            for (size_t t = 0; t < arr.n; ++t) {
              kk[t] = plain ? arr.a[t].pos : arr.a[t].remapped_pos << 32 | arr.a[t].pos;
              ki[t] = (uint32_t)t;
            }
            radix_sort_u64(arr.n, kk.data(), ki.data(), tk, tv);
            done = true;
            for (size_t t = 1; t < arr.n && done; ++t) done = kk[t] != kk[t - 1];
            if (done) perm = ki.data();
          }
          if (done) {
          } else if (arr.n > 32) {
            // on 24-byte keys with the positions' indices: the introsort's moves depend only on the
            // comparisons, so the permutation -- ties included -- is the one of the positions themselves
            pk.resize(arr.n);
            for (size_t t = 0; t < arr.n; ++t) pk[t] = {arr.a[t].remapped_pos, arr.a[t].pos, (uint32_t)t};
            ks_introsort(arr.n, pk.data(), [](const PosKey &a, const PosKey &b) {
              return a.rp == b.rp ? a.p < b.p : a.rp < b.rp;
            });
            ki.resize(arr.n);
            for (size_t t = 0; t < arr.n; ++t) ki[t] = pk[t].idx;
            perm = ki.data();
          } else {
            ks_introsort(arr.n, arr.a.data(), position_lt);
          }
        }
        if (pstats) a_sort += now_ns() - t0;
        pth[i] = th;
        poff[i] = st.size();
        pcnt[i] = (uint32_t)arr.n;
        if (perm) {
          if (st.capacity() < st.size() + arr.n) st.reserve(std::max(st.size() + arr.n, 2 * st.capacity()));
          for (size_t t = 0; t < arr.n; ++t) st.push_back(arr.a[perm[t]]);
        } else {
          st.insert(st.end(), arr.a.begin(), arr.a.begin() + arr.n);
        }
      }
      t_pos += a_pos;
      t_cnt += a_cnt;
      t_sort += a_sort;
    }, nth);
    ph.mark("pairing: positions");
    std::vector<const Position *> parr(n);
    for (int i = 0; i < n; ++i) parr[i] = pstore[pth[i]].data() + poff[i];
    // `sampe -t T`: the reference's thread t (threadblock_exec, bwape.c:249-253) takes pairs t, t+T,
    // t+2T, ... into its own position array, so the slots past a pair's positions hold what the
    // earlier pairs of its residue class mod T left there: one nearest-greater chain per class
    std::vector<int32_t> pg(n, -1);
    {
      const int T = popt.n_threads > 1 ? popt.n_threads : 1;
      std::vector<int32_t> st;
      for (int c = 0; c < T && c < n; ++c) {
        st.clear();
        for (int i = c; i < n; i += T) {
          while (!st.empty() && pcnt[st.back()] <= pcnt[i]) st.pop_back();
          pg[i] = st.empty() ? -1 : st.back();
          st.push_back(i);
        }
      }
    }
    if (getenv("IBWA_SAMPE_STATS")) {
      uint64_t tot = 0, mx = 0;
      for (int i = 0; i < n; ++i) { tot += pcnt[i]; mx = std::max<uint64_t>(mx, pcnt[i]); }
      elog("[ibwa-amd sampe] batch of %d pairs: %llu positions (max %llu per pair), %zu rows computed; "
              "positions pass thread-ms: rows %.0f, c1/c2 %.0f, sort %.0f\n", n, (unsigned long long)tot,
              (unsigned long long)mx, pos.size(), t_pos * 1e-6, t_cnt * 1e-6, t_sort * 1e-6);
    }
    // pairing_aux's penalty depends on l alone: once per batch for every l it can be asked for
    std::vector<int> pen;
    if (ii.high) {
      pen.resize((size_t)ii.high_bayesian + 1);
      for (uint32_t l = 0; l <= ii.high_bayesian; ++l)
        pen[l] = (int)(-4.343 * log(.5 * erfc(M_SQRT1_2 * fabs(l - ii.avg) / ii.std)) + .499);
    }
    std::vector<int> chg(nth, 0);
    parallel_ordered(n, [&](int64_t lo, int64_t hi_, int th) {
      for (int64_t i = lo; i < hi_; ++i) {
        Read *p[2] = {&seqs[0][i], &seqs[1][i]};
        if (paired[i]) {
          PairCtx c{{p[0], p[1]}, {&alns[0][i], &alns[1][i]}, &popt, &ii, gopt[1].s_mm, pen.data()};
          chg[th] += find_optimal_pair(c, PosView(parr.data(), pcnt.data(), pg.data(), i));
        }
        if (popt.N_multi || popt.n_multi) {
          for (int j = 0; j < 2; ++j) {
            if (p[j]->type == TYPE_NO_MATCH) continue;
            int max_multi = popt.n_multi;
            if (!(p[j]->extra_flag & SAM_FPP) && p[1 - j]->type != TYPE_NO_MATCH)
              max_multi = (int)(p[j]->c1 + p[j]->c2) - 1 > popt.N_multi ? popt.n_multi : popt.N_multi;
            const uint64_t *mrow = mfirst[j][i] >= 0 ? mpos.data() + mfirst[j][i] : nullptr;
            select_sai_multi(alns[j][i], *p[j], max_multi, row0[j].empty() ? -1 : row0[j][i], aslot, pos, mrow);
          }
        }
      }
    }, nth);
    int cnt_chg = 0;
    for (int x : chg) cnt_chg += x;
    elog("[bwa_sai2sam_pe_core] changing coordinates of %d alignments.\n", cnt_chg);
    ph.mark("pairing");
    // ---- mate rescue (bwa_paired_sw) over the concatenated references
    if (int rc = paired_sw(wk, seqs, n, ii)) return rc;
    ph.mark("paired SW");
    // ---- refine gapped alignments of both ends, MD/NM, trimmed reads; then remap()
    std::vector<Read *> rp;
    for (int j = 0; j < 2; ++j)
      for (Read &r : seqs[j]) rp.push_back(&r);
    if (int rc = refine_gapped(wk.ctx[0], dbs, rp)) return rc == 1 ? 1 : die("global alignment");
    ph.mark("refine");
    for (int j = 0; j < 2; ++j)
      parallel_ordered(n, [&](int64_t lo, int64_t hi_, int) {
        for (int64_t i = lo; i < hi_; ++i) {
          Read &r = seqs[j][i];
          int status = 0;
          remap(r, r.pos, r.dbidx, (uint64_t)r.len, (uint32_t)(r.n_gapo + r.n_gape), &status);
          if (status == 0) {
            msg("Failed to remap read %s after refining gaps.\n", r.name.c_str());
            unmap(r);
          }
        }
      }, 0, 4096);
    ph.mark("remap after refine");
    // ---- print: with -R the remapped (primary) coordinates, the original ones as ZR; batch by batch
    // in file order
    if (!wait_turn(bt.idx)) return 1;
    print_parallel(o, n, [&](Out &ob, int64_t i) {
      Read *p[2] = {&seqs[0][i], &seqs[1][i]};
      if (p[0]->bc[0] || p[1]->bc[0]) {
        strncat(p[0]->bc, p[1]->bc, sizeof p[0]->bc - strlen(p[0]->bc) - 1);
        memcpy(p[1]->bc, p[0]->bc, sizeof p[1]->bc);
      }
      if (popt.remapping) {
        std::swap(p[0]->pos, p[0]->remapped_pos);
        std::swap(p[1]->pos, p[1]->remapped_pos);
      } else {
        p[0]->remapped_pos = p[0]->pos;
        p[1]->remapped_pos = p[1]->pos;
      }
      print_sam1(ob, dbs, *p[0], p[1], gopt[1].mode, gopt[1].max_top2, rg_id);
      print_sam1(ob, dbs, *p[1], p[0], gopt[1].mode, gopt[1].max_top2, rg_id);
    });
    end_turn(n);
    ph.mark("print");
    return 0;
  }

  // select_sai_multi (saiset.c:124-163): every hit when there are at most n_multi + 1 of them
  // (positions as bwtdb_sa2seq gives them: not remapped)
  int select_sai_multi(const AlnSpan &ag, Read &s, int n_multi, int64_t slot0, const std::vector<int64_t> &aslot,
                       const std::vector<uint64_t> &pos, const uint64_t *mrow) {
    int n_occ = 0;
    for (const Aln &q : ag) n_occ += (int)(q.aln.l - q.aln.k + 1);
    s.multi.clear();
    if (n_occ > n_multi + 1) return 0;
    std::vector<Multi> all;
    for (size_t k = 0; k < ag.size(); ++k) {
      const ibwa_aln1_t &q = ag[k].aln;
      const uint32_t w = q.l - q.k + 1;
      const uint64_t *pp = nullptr;
      const int64_t slot = slot0 >= 0 ? aslot[slot0 + (int64_t)k] : -1;
      if (slot >= 0) {
        pp = pos.data() + slot;
      } else {  // not on hand (no -R pass, or a cached interval): this read's rows of the batch's
                // one bwtdb_sa2seq launch for select_sai_multi (mrow, alignment by alignment)
        pp = mrow;
        mrow += w;
      }
      for (uint32_t r = 0; r < w; ++r) {
        Multi m;
        m.pos = pp[r];
        m.gap = (q.n_gapo + q.n_gape) & 0xff;
        m.mm = q.n_mm;
        m.strand = q.a;
        all.push_back(m);
      }
    }
    for (const Multi &m : all)
      if (m.pos != s.pos) s.multi.push_back(m);
    if ((int)s.multi.size() > n_multi) s.multi.resize(std::max(n_multi, 0));
    return 0;
  }

  // bwa_paired_sw through the C-ABI (compat.cpp) on bwa_seq_t mirrors of the batch
  int paired_sw(Worker &wk, std::vector<Read> seqs[2], int n, const Isize &ii) {
    Phases &ph = wk.ph;
    if (!popt.is_sw || ii.avg < 0.0) return 0;
    // the mirrors are filled in parallel below, in buffers kept across batches (allocating, faulting
    // in and freeing a batch's worth each time cost ~25 ms per batch)
    std::unique_ptr<ibwa_ref_seq_t[]> *ref = wk.sw_ref;
    std::unique_ptr<uint8_t[]> *rev = wk.sw_rev;
    size_t *sw_ref_cap_ = wk.sw_ref_cap, *sw_rev_cap_ = wk.sw_rev_cap;
    for (int j = 0; j < 2; ++j) {
      if (sw_ref_cap_[j] < (size_t)std::max(n, 1)) {
        sw_ref_cap_[j] = (size_t)std::max(n, 1);
        ref[j].reset(new ibwa_ref_seq_t[sw_ref_cap_[j]]);
      }
      std::vector<size_t> ro(n + 1, 0);
      for (int i = 0; i < n; ++i) ro[i + 1] = ro[i] + (size_t)seqs[j][i].len;
      if (sw_rev_cap_[j] < ro[n] + 1) {
        sw_rev_cap_[j] = ro[n] + 1;
        rev[j].reset(new uint8_t[sw_rev_cap_[j]]);
      }
      parallel_chunks(n, [&](int64_t lo, int64_t hi, int) {
        for (int64_t i = lo; i < hi; ++i) {
          Read &r = seqs[j][i];
          ibwa_ref_seq_t &t = ref[j][i];
          memset(&t, 0, sizeof t);
          // the sequences of pairs bwa_paired_sw looks at (bwasw.c:157-159: an end with mapQ >= 17, end 1
          // not properly paired -- its first test, before any sequence is read); the others' are never read
          const bool looked_at = (seqs[0][i].mapQ >= 17 || seqs[1][i].mapQ >= 17) && (seqs[0][i].extra_flag & SAM_FPP) == 0;
          if (looked_at)
            std::reverse_copy(r.seq.begin(), r.seq.begin() + r.len, rev[j].get() + ro[i]);  // bwa_seq_t.seq: reversed
          t.seq = rev[j].get() + ro[i];
          t.rseq = r.rseq.data();
          t.len = (uint32_t)r.len;
          t.full_len = (uint32_t)r.full_len;
          t.strand = (uint32_t)r.strand;
          t.type = (uint32_t)r.type;
          t.extra_flag = (uint32_t)r.extra_flag;
          t.n_mm = (uint32_t)r.n_mm; t.n_gapo = (uint32_t)r.n_gapo; t.n_gape = (uint32_t)r.n_gape;
          t.mapQ = (uint32_t)r.mapQ;
          t.seQ = (uint64_t)r.seQ;
          t.pos = r.pos;
          t.remapped_pos = r.remapped_pos;
          t.dbidx = (uint32_t)r.dbidx;
          t.remapped_dbidx = (uint32_t)r.remapped_dbidx;
          t.c1 = r.c1; t.c2 = r.c2;
        }
      });
    }
    ph.mark("paired SW: mirrors");
    ibwa_ref_pe_opt_t po;
    memset(&po, 0, sizeof po);
    po.max_isize = popt.max_isize; po.force_isize = popt.force_isize; po.max_occ = popt.max_occ;
    po.n_multi = popt.n_multi; po.N_multi = popt.N_multi; po.n_threads = 1;
    po.type = popt.type; po.is_sw = popt.is_sw; po.is_preload = popt.is_preload; po.remapping = popt.remapping;
    po.ap_prior = popt.ap_prior;
    ibwa_ref_isize_info_t ri{ii.avg, ii.std, ii.ap_prior, ii.low, ii.high, ii.high_bayesian};
    ibwa_ref_seq_t *sp[2] = {ref[0].get(), ref[1].get()};
    uint64_t n_tot[2], n_mapped[2];
    std::vector<const uint8_t *> pacs;
    std::vector<uint64_t> offs, lens;
    for (const RefDb &r : dbs.db) {
      pacs.push_back(r.bns.pac.data());
      offs.push_back(r.offset);
      lens.push_back((uint64_t)r.bns.l_pac);
    }
    if (ibwa_paired_sw_dbs(wk.ctx[0], n, sp, &po, &ri, (int)pacs.size(), pacs.data(), offs.data(), lens.data(), n_tot,
                           n_mapped))
      return die("paired SW");
    ph.mark("paired SW: windows+SW+fix-up");
    elog("[bwa_paired_sw] %llu out of %llu Q17 singletons are mated.\n", (unsigned long long)n_mapped[1],
            (unsigned long long)n_tot[1]);
    elog("[bwa_paired_sw] %llu out of %llu Q17 discordant pairs are fixed.\n", (unsigned long long)n_mapped[0],
            (unsigned long long)n_tot[0]);
    for (int j = 0; j < 2; ++j) {
      parallel_chunks(n, [&](int64_t lo, int64_t hi, int) {
        for (int64_t i = lo; i < hi; ++i) {
          Read &r = seqs[j][i];
          ibwa_ref_seq_t &t = ref[j][i];
          r.type = t.type;
          r.strand = t.strand;
          r.extra_flag = t.extra_flag;
          r.n_mm = t.n_mm; r.n_gapo = t.n_gapo; r.n_gape = t.n_gape;
          r.mapQ = t.mapQ;
          r.seQ = (int)t.seQ;
          r.pos = t.pos;
          r.remapped_pos = t.remapped_pos;
          r.dbidx = (int)t.dbidx;
          r.remapped_dbidx = (int)t.remapped_dbidx;
          if (t.cigar) {
            r.cigar.assign(t.cigar, t.cigar + t.n_cigar);
            r.has_cigar = true;
            free(t.cigar);
          }
        }
      });
    }
    return 0;
  }
};

}  // namespace

int sampe_main(int argc, char *argv[]) {
  init_tables();
  Source src[2];  // before S: the background reader S holds uses it until S is gone
  Sampe S;
  int c;
  const char *fn_out = nullptr;
  std::string rg_line, rg_id;
  int n_workers = 1;
  optind = 1;
  while ((c = getopt(argc, argv, "a:o:sPn:N:c:f:ARr:t:G:")) >= 0) {  // bwa_sai2sam_pe (bwape.c:583-610) + -G
    switch (c) {
      case 'r':
        if (!set_rg(optarg, rg_line, rg_id)) {
          fprintf(stderr, "[bwa_sai2sam_pe] malformated @RG line\n");
          return 1;
        }
        break;
      case 'a': S.popt.max_isize = atoi(optarg); break;
      case 'o': S.popt.max_occ = atoi(optarg); break;
      case 's': S.popt.is_sw = 0; break;
      case 'P': S.popt.is_preload = 1; break;
      case 'n': S.popt.n_multi = atoi(optarg); break;
      case 'N': S.popt.N_multi = atoi(optarg); break;
      case 't': S.popt.n_threads = atoi(optarg); break;
      case 'c': S.popt.ap_prior = atof(optarg); break;
      case 'f': fn_out = optarg; break;
      case 'A': S.popt.force_isize = 1; break;
      case 'R': S.popt.remapping = 1; break;
      case 'G': n_workers = atoi(optarg); break;
      default: return 1;
    }
  }
  if (optind + 5 > argc) {
    fprintf(stderr, "Usage: ibwa-amd sampe [-a INT] [-o INT] [-n INT] [-N INT] [-c FLOAT] [-f out.sam] [-r RG] [-G INT] [-sAR]\n"
                    "                      <prefix> <in1.sai> <in2.sai> <in1.fq> <in2.fq> [<prefix2> <in1.sai> <in2.sai> ...]\n");
    return 1;
  }
  // pe_inputs_parse (bwape.c:548-581)
  std::vector<std::string> prefixes{argv[optind]};
  std::vector<std::pair<const char *, const char *>> sais{{argv[optind + 1], argv[optind + 2]}};
  const char *fq[2] = {argv[optind + 3], argv[optind + 4]};
  for (int i = optind + 5; i < argc; i += 3) {
    if (argc - i < 3) {
      fprintf(stderr, "[pe_inputs_parse] insufficient arguments\n");
      return 1;
    }
    prefixes.push_back(argv[i]);
    sais.push_back({argv[i + 1], argv[i + 2]});
  }
  const int count = (int)prefixes.size();
  for (int j = 0; j < 2; ++j) {  // saiset_create (saiset.c:15-33): the last reference's header holds
    for (int d = 0; d < count; ++d) {
      const char *fn = j == 0 ? sais[d].first : sais[d].second;
      FILE *fp = fopen(fn, "rb");
      if (fp) setvbuf(fp, nullptr, _IOFBF, 1 << 22);
      if (!fp || fread(&S.gopt[j], sizeof S.gopt[j], 1, fp) != 1) {
        fprintf(stderr, "[ibwa-amd sampe] cannot read the .sai header of %s\n", fn);
        return 1;
      }
      S.fp_sai[j].push_back(fp);
    }
    if (!(S.gopt[j].mode & IBWA_MODE_COMPREAD)) {
      fprintf(stderr, "[ibwa-amd sampe] color-space alignments (aln -c) need the .nt index: not supported\n");
      return 1;
    }
  }
  for (int j = 0; j < 2; ++j) {
    if (!src[j].open(fq[j], S.gopt[j])) {
      fprintf(stderr, "[ibwa-amd sampe] cannot open %s\n", fq[j]);
      return 1;
    }
  }
  if (const char *e = getenv("IBWA_SAMPE_BATCH")) S.batch_pairs = (size_t)std::max(1L, atol(e));
  if (const char *e = getenv("IBWA_SAMPE_READ_AHEAD")) S.depth = (size_t)std::max(1L, atol(e));
  S.start_reading(src);
  // dbset_restore (dbset.c:135-176): references at cumulative offsets, each with its index on the
  // GPU, and (-R) its .remap table when it has one
  S.dbs.db.resize(count);
  if (n_workers < 1) n_workers = 1;
  S.W.resize(n_workers);
  S.wide_cache.resize(count);
  S.first_use.resize(count);
  int n_dev = 0;
  if (ibwa_device_count(&n_dev) || n_dev < 1) return die("no HIP device");
  if (n_workers > n_dev)
    fprintf(stderr, "[ibwa-amd sampe] -G %d on %d visible device(s): worker w runs on device w mod %d\n", n_workers, n_dev, n_dev);
  // the host side (.ann / .amb / .pac, .remap tables) on a thread while the GPUs take the indexes
  std::vector<int> host_ok(count, 0);
  std::thread host_side([&]() {
    for (int d = 0; d < count; ++d) {
      RefDb &r = S.dbs.db[d];
      if (!bns_restore(prefixes[d], r.bns)) return;
      host_ok[d] = 1;
      if (S.popt.remapping)  // seq_restore (dbset.c:81-101)
        r.remap = load_remappings(prefixes[d] + ".remap", r.bns.n_seqs, r.mappings);
      host_ok[d] = 2;
    }
  });
  // the first worker on each device loads the indexes there (the devices in parallel); the others
  // share them
  const int n_load = std::min(n_workers, n_dev);
  std::vector<int> gpu_rcs(n_load, 0);
  auto load = [&](int w) {
    int &rc = gpu_rcs[w];
    for (int d = 0; d < count && !rc; ++d) {
      const std::string &prefix = prefixes[d];
      ibwa_ctx_t *cx = nullptr;
      if (ibwa_ctx_create(w, &cx)) { rc = 1; break; }
      S.W[w].ctx.push_back(cx);
      if (ibwa_ctx_load_bwt_file(cx, 0, (prefix + ".bwt").c_str()) || ibwa_ctx_load_bwt_file(cx, 1, (prefix + ".rbwt").c_str()))
        rc = 2;
      else if (ibwa_ctx_load_sa_file(cx, 0, (prefix + ".sa").c_str()) || ibwa_ctx_load_sa_file(cx, 1, (prefix + ".rsa").c_str()))
        rc = 3;
      else if (ibwa_ctx_expand_sa(cx))
        rc = 4;
    }
  };
  {
    std::vector<std::thread> lt;
    for (int w = 1; w < n_load; ++w) lt.emplace_back(load, w);
    load(0);
    for (auto &t : lt) t.join();
  }
  int gpu_rc = 0;
  for (int x : gpu_rcs) gpu_rc = gpu_rc ? gpu_rc : x;
  for (int w = n_load; w < n_workers && !gpu_rc; ++w)
    for (int d = 0; d < count && !gpu_rc; ++d) {
      ibwa_ctx_t *cx = nullptr;
      if (ibwa_ctx_create(w % n_dev, &cx)) { gpu_rc = 1; break; }
      S.W[w].ctx.push_back(cx);
      if (ibwa_ctx_share_index(cx, S.W[w % n_dev].ctx[d])) gpu_rc = 5;
    }
  host_side.join();
  if (gpu_rc == 1) return die("ibwa_ctx_create");
  if (gpu_rc == 2) return die("load .bwt / .rbwt");
  if (gpu_rc == 3) return die("load .sa / .rsa");
  if (gpu_rc == 4) return die("expand SA");
  if (gpu_rc == 5) return die("share index");
  for (int d = 0; d < count; ++d) {
    RefDb &r = S.dbs.db[d];
    const std::string &prefix = prefixes[d];
    if (host_ok[d] < 1) {
      fprintf(stderr, "[ibwa-amd sampe] cannot read %s.ann / .amb / .pac\n", prefix.c_str());
      return 1;
    }
    r.offset = S.dbs.l_pac;
    S.dbs.l_pac += (uint64_t)r.bns.l_pac;
    if (S.popt.remapping) {
      if (r.remap < 0) {
        fprintf(stderr, "Fatal error loading sequence mappings from %s\n", (prefix + ".remap").c_str());
        return 1;
      } else if (r.remap) {
        fprintf(stderr, " - Remapping enabled for sequence %s\n", prefix.c_str());
      }
    }
  }
  S.rnd.seed((long)S.dbs.db[0].bns.seed);  // srand48(dbs->db[0]->bns->bns->seed), bwape.c:471
  S.rg_id = rg_id.empty() ? nullptr : rg_id.c_str();
  FILE *out = fn_out ? fopen(fn_out, "w") : stdout;
  if (!out) {
    fprintf(stderr, "[ibwa-amd sampe] cannot write %s\n", fn_out);
    return 1;
  }
  // @SQ lines of every sequence that is not remapped (dbset_print_sam_SQ, dbset.c:327-339), @RG, @PG
  std::string head;
  for (const RefDb &r : S.dbs.db)
    for (int32_t t = 0; t < r.bns.n_seqs; ++t)
      if (!r.remap || t >= (int32_t)r.mappings.size() || !r.mappings[t])
        head += "@SQ\tSN:" + r.bns.anns[t].name + "\tLN:" + std::to_string(r.bns.anns[t].len) + "\n";
  if (!rg_line.empty()) head += rg_line + "\n";
  head += "@PG\tID:bwa\tPN:bwa\tVN:ibwa-amd\n";
  fwrite(head.data(), 1, head.size(), out);
  S.W[0].ph.mark("load index (first batch read meanwhile)");
  const int rc = S.run(out);
  S.stop_reader();  // batches read ahead on an error return
  for (int j = 0; j < 2; ++j)
    for (FILE *fp : S.fp_sai[j]) fclose(fp);
  if (out != stdout) fclose(out);
  for (size_t w = S.W.size(); w-- > 0;)  // the sharing contexts before the ones they borrow from
    for (ibwa_ctx_t *cx : S.W[w].ctx) ibwa_ctx_destroy(cx);
  return rc;
}
