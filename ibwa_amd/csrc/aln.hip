// aln.hip -- the aln hot path on gfx950: one read per lane.
//
// Why a lane, not a wavefront, per read: every backward-search step is a
// dependent random 64 B fetch into a 1.5 GB table, so throughput is set by
// the number of independent chains in flight (Little's law: ~8 TB/s x ~2 us
// / 64 B = ~250k outstanding fetches).  One read per wave would give 8k
// chains on 256 CUs; one read per lane gives 64x that.
//
//   k_width  : bwt_cal_width x4 per read (bwtaln.c:54-78, called :123-130),
//              the two strands (and the two seeds) advanced in lockstep so
//              each lane keeps two fetches in flight.
//   k_search : bwt_match_gap (bwtgap.c:104-264) with the bucketed LIFO
//              priority stack of bwtgap.c:13-79 kept per lane in HBM as
//              per-bucket linked lists.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "engine.h"
#include "occ.h"

namespace ibwa {

namespace {

constexpr int MODE_GAPE = 0x01, MODE_COMPREAD = 0x02, MODE_LOGGAP = 0x04, MODE_NONSTOP = 0x10;
constexpr int STATE_M = 0, STATE_I = 1, STATE_D = 2;

// All six 16 B loads of a rank-query pair are issued unconditionally so that
// the compiler can put every fetch of a step in flight before the first wait.
struct Fetch {
  uint4 ck, bk, sk, cl, bl, sl;
  uint32_t offk, offl;
  bool kneg;
};

__device__ __forceinline__ void fetch_pair(const IndexView &ix, uint32_t k, uint32_t l, Fetch &f) {
  f.kneg = (k == 0xFFFFFFFFu);
  uint32_t kk = f.kneg ? 0u : bwt_kk(ix, k);
  uint32_t ll = bwt_kk(ix, l);
  const uint4 *pk = ix.blk + (size_t)(kk >> 7) * 4;
  const uint4 *pl = ix.blk + (size_t)(ll >> 7) * 4;
  f.offk = kk & 127;
  f.offl = ll & 127;
  f.ck = pk[0];
  f.bk = pk[1 + (f.offk >> 6)];
  f.sk = pk[3];
  f.cl = pl[0];
  f.bl = pl[1 + (f.offl >> 6)];
  f.sl = pl[3];
}

// Predicated fetch: no loads when !run; the l-end reuses the k-end block's
// counts when both ends fall in one 128-symbol block (bwt.c:125's fast path).
__device__ __forceinline__ void fetch_pair_p(const IndexView &ix, uint32_t k, uint32_t l, bool run, Fetch &f) {
  f.kneg = (k == 0xFFFFFFFFu);
  uint32_t kk = f.kneg ? 0u : bwt_kk(ix, k);
  uint32_t ll = bwt_kk(ix, l);
  const bool same = !f.kneg && (kk >> 7) == (ll >> 7);
  const uint4 *pk = ix.blk + (size_t)(kk >> 7) * 4;
  const uint4 *pl = ix.blk + (size_t)(ll >> 7) * 4;
  f.offk = kk & 127;
  f.offl = ll & 127;
  if (run && !f.kneg) {
    f.ck = pk[0];
    f.bk = pk[1 + (f.offk >> 6)];
    f.sk = pk[3];
  }
  if (run) f.bl = pl[1 + (f.offl >> 6)];
  if (run && !same) {
    f.cl = pl[0];
    f.sl = pl[3];
  }
  if (same) {
    f.cl = f.ck;
    f.sl = f.sk;
  }
}

// Single-symbol rank pair: per end only the 16 B that bwt_2occ needs --
// C[c], the 32-symbol chunk (8 B) and its sub-count word -- 3 loads, 4 VGPRs.
struct Fetch1 {
  uint32_t ck, sk, cl, sl;
  uint2 wk, wl;
  uint32_t offk, offl;
  bool kneg;
};

__device__ __forceinline__ void fetch1(const IndexView &ix, uint32_t k, uint32_t l, uint32_t c, bool run,
                                       Fetch1 &f) {
  f.kneg = (k == 0xFFFFFFFFu);
  const uint32_t kk = f.kneg ? 0u : bwt_kk(ix, k);
  const uint32_t ll = bwt_kk(ix, l);
  const uint32_t *pk = reinterpret_cast<const uint32_t *>(ix.blk + (size_t)(kk >> 7) * 4);
  const uint32_t *pl = reinterpret_cast<const uint32_t *>(ix.blk + (size_t)(ll >> 7) * 4);
  f.offk = kk & 127;
  f.offl = ll & 127;
  const uint32_t qk = f.offk >> 5, ql = f.offl >> 5;
  if (run && !f.kneg) {
    f.ck = pk[c];
    f.wk = *reinterpret_cast<const uint2 *>(pk + 4 + 2 * qk);
    f.sk = pk[11 + (qk ? qk : 1)];
  }
  if (run) {
    f.cl = pl[c];
    f.wl = *reinterpret_cast<const uint2 *>(pl + 4 + 2 * ql);
    f.sl = pl[11 + (ql ? ql : 1)];
  }
}

__device__ __forceinline__ uint32_t occ1_end(uint32_t cnt, uint32_t sub, uint2 w, uint32_t off, uint32_t c) {
  const uint32_t q = off >> 5;
  uint32_t m0, m1;
  chunk_masks(off & 31, m0, m1);
  return cnt + (q ? (sub >> (8 * c)) & 0xFFu : 0u) + count1(w.x, w.y, m0, m1, c);
}

__device__ __forceinline__ void occ2_from1(const Fetch1 &f, uint32_t c, uint32_t &ok, uint32_t &ol) {
  ok = f.kneg ? 0u : occ1_end(f.ck, f.sk, f.wk, f.offk, c);
  ol = occ1_end(f.cl, f.sl, f.wl, f.offl, c);
}

__device__ __forceinline__ uint32_t occ_c(const uint4 &cnt, const uint4 &bs, const uint4 &sb, uint32_t off,
                                          uint32_t c) {
  uint32_t q = off >> 5, w0, w1, m0, m1;
  chunk_words(bs, q, w0, w1);
  chunk_masks(off & 31, m0, m1);
  return sel4(cnt, c) + sub_byte(sb, q, c) + count1(w0, w1, m0, m1, c);
}

// bwt_2occ(k-1, l, c) from a fetch made with (k-1, l)
__device__ __forceinline__ void occ2_from(const Fetch &f, uint32_t c, uint32_t &ok, uint32_t &ol) {
  ok = f.kneg ? 0u : occ_c(f.ck, f.bk, f.sk, f.offk, c);
  ol = occ_c(f.cl, f.bl, f.sl, f.offl, c);
}

__device__ __forceinline__ void occ4x2_from(const Fetch &f, uint32_t ck[4], uint32_t cl[4]) {
  if (f.kneg) {
    ck[0] = ck[1] = ck[2] = ck[3] = 0;
  } else {
    occ4_from(f.ck, f.bk, f.sk, f.offk, ck);
  }
  occ4_from(f.cl, f.bl, f.sl, f.offl, cl);
}

__device__ __forceinline__ uint32_t strand_base(uint32_t c, int a, bool comp) {
  // seq[1] = rseq = complement of seq under COMPREAD (bwaseqio.c:189-192)
  return (a == 1 && comp && c < 4) ? 3u - c : c;
}

// The compact record's byte stream (engine.h AlnArgs::cw) as width_pair produces it: byte `off` of
// the stream goes to bits 8 * (off & 3) of word off >> 2; the accumulator carries a partial word from
// the full-length chains into the seed chains.
struct RecOut {
  uint32_t *words;  // the record's width bytes (word 1 + cw_rw of the record)
  uint32_t off, acc;
  __device__ __forceinline__ void put(uint32_t byte) {
    acc |= byte << (8 * (off & 3));
    if ((off & 3) == 3) {
      words[off >> 2] = acc;
      acc = 0;
    }
    ++off;
  }
  __device__ __forceinline__ void flush() {
    if (off & 3) words[off >> 2] = acc;
    acc = 0;
  }
};

// one position's byte: per strand the bid clamped to `clamp` and "width equals the previous
// position's", at bit offsets 0 and nb (full: 3 + 1 bits per strand, seed: 2 + 1)
__device__ __forceinline__ uint32_t rec_byte(uint2 a, uint2 b, uint32_t pa, uint32_t pb, bool first, uint32_t clamp,
                                             int nb) {
  const uint32_t ea = !first && a.x == pa, eb = !first && b.x == pb;
  return (a.y < clamp ? a.y : clamp) | ea << (nb - 1) | ((b.y < clamp ? b.y : clamp) | eb << (nb - 1)) << nb;
}

// One bwt_cal_width step (bwtaln.c:54-78) of a chain, with one-row intervals stepped from the
// text: row k with k == l has the suffix at q = SA[k], BWT[k] = text[q-1], and stepping with c
// stays on one row (suffix at q-1) exactly when q > 0 and text[q-1] == c; otherwise the interval
// is empty and the reference resets it.  Mode 0: Occ steps; 1: the interval became one row at
// the last step -- this step is an Occ step that also loads SA[k]; 2: text steps (suffix at t)
// from a window of two 2-bit text words (32 symbols).  Every mode issues its loads in the same
// round trip as the other chain's and the other lanes' (the chains stay in lockstep), and the text
// windows are refilled at the 16-position blocks' first step (`refresh`), for the block's 16 steps at
// once: text-mode lanes then load in the same steps, so the wave waits once per block for them
// instead of at almost every step (a lane entering text mode inside a block loads its window then).
struct WChain {
  uint32_t k, l, bid;
  uint32_t mode, t, wi, w, w2;  // text mode: suffix position, window's first word index, its two words
};

struct WLoad {
  Fetch1 f;
  uint32_t q, w, w2, wi;
  bool tl;
};

// text position p is in the chain's window
__device__ __forceinline__ bool win_has(const WChain &h, uint32_t p) {
  return h.wi != 0xFFFFFFFFu && p >= 16u * h.wi && p - 16u * h.wi < 32u;
}

// the step's loads (issued for both chains before either is consumed: one round trip)
__device__ __forceinline__ void wchain_load(const IndexView &ix, const uint32_t *sa, const uint32_t *tx,
                                            const WChain &h, uint32_t c, WLoad &x, bool refresh) {
  fetch1(ix, h.k - 1, h.l, c & 3, c < 4 && h.mode != 2, x.f);
  x.q = 0;
  if (h.mode == 1) x.q = sa[h.k];
  // the next 16 steps read text positions p, p - 1, ..., p - 15 (p = t - 1): a window from word
  // (p - 15) / 16 holds them all
  const uint32_t p = h.t - 1u;
  x.tl = h.mode == 2 && h.t > 0 && (!win_has(h, p) || (refresh && !win_has(h, p >= 15u ? p - 15u : 0u)));
  x.wi = (p >= 15u ? p - 15u : 0u) >> 4;
  x.w = h.w;
  x.w2 = h.w2;
  if (x.tl) {
    x.w = tx[x.wi];
    x.w2 = tx[x.wi + 1];
  }
}

__device__ __forceinline__ void wchain_step(const IndexView &ix, bool jump, WChain &h, uint32_t c, const WLoad &x) {
  if (h.mode == 2) {
    if (x.tl) { h.w = x.w; h.w2 = x.w2; h.wi = x.wi; }
    const uint32_t p = h.t - 1u;
    const uint32_t tw = p - 16u * h.wi < 16u ? h.w : h.w2;
    if (h.t > 0 && c < 4 && ((tw >> (2 * (p & 15))) & 3u) == c) {
      --h.t;  // still one row: k == l stays, width 1
    } else {
      h.k = 0; h.l = ix.seq_len; ++h.bid; h.mode = 0;
    }
    return;
  }
  bool reset = c > 3;
  if (c < 4) {
    uint32_t ok, ol;
    occ2_from1(x.f, c, ok, ol);
    h.k = l2of(ix, c) + ok + 1;
    h.l = l2of(ix, c) + ol;
    reset = h.k > h.l;
  }
  if (reset) { h.k = 0; h.l = ix.seq_len; ++h.bid; }
  if (h.mode == 1) {
    // the step from the one row with its suffix at q succeeded (suffix at q - 1) or emptied it
    h.mode = reset ? 0u : 2u;
    h.t = x.q - 1u;
    h.wi = 0xFFFFFFFFu;
  } else if (jump && !reset && h.k == h.l) {
    h.mode = 1;
  }
}

// two bwt_cal_width chains in lockstep (bwtaln.c:54-78): str on ixa -> wa, strand-1 str on
// ixb -> wb.  The entries of 16 steps are kept in
// registers and stored back to back (a lane's 128 B of widths leave in consecutive instructions,
// so the L2 merges them into whole lines instead of 16 partial writes far apart).
// With sa0/sa1 and tx0/tx1 (the exact path's full SA and 2-bit text per strand) one-row
// intervals step from the text (wchain_step).
__device__ __forceinline__ void width_pair(const IndexView ixa, const IndexView ixb, int L, const uint8_t *s, bool comp,
                                           uint2 *wa, uint2 *wb, uint32_t *lw = nullptr, RecOut *rec = nullptr,
                                           uint32_t clamp = 0, int nb = 4, uint32_t *rd = nullptr,
                                           const uint32_t *sa0 = nullptr, const uint32_t *sa1 = nullptr,
                                           const uint32_t *tx0 = nullptr, const uint32_t *tx1 = nullptr,
                                           const uint2 *lta = nullptr, const uint2 *ltb = nullptr, int tdep = 0) {
  WChain A{0u, ixa.seq_len, 0u, 0u, 0u, 0xFFFFFFFFu, 0u, 0u};
  WChain B{0u, ixb.seq_len, 0u, 0u, 0u, 0xFFFFFFFFu, 0u, 0u};
  uint32_t lwa = 0, lwb = 0;  // sum of log2(width) over the positions (diagnostics)
  uint32_t pa = 0, pb = 0;    // previous positions' widths (record)
  // The first min(L, tdep) steps of both chains from the level tables (AlnArgs::ltab): the interval
  // after d symbols is the table entry of their string, so those steps' loads are independent -- one
  // round trip for all of them instead of a chain of dependent Occ steps.  A chain takes table steps
  // up to its first N or empty interval (the steps from there reset it as before).
  constexpr int TMAX = 15;
  uint2 ta[TMAX], tb[TMAX];
  int da = 0, db = 0;
  if (tdep > 0) {
    const int D = L < tdep ? L : tdep;
    uint32_t xa = 0, xb = 0;
    int dn = D;  // steps before the first N
#pragma unroll
    for (int d = 0; d < TMAX; ++d) {
      ta[d] = tb[d] = make_uint2(1u, 0u);
      if (d < dn) {
        const uint32_t ca = s[d];
        if (ca > 3) {
          dn = d;
        } else {
          const uint32_t cb = strand_base(ca, 1, comp);
          xa = xa << 2 | ca;
          xb = xb << 2 | cb;
          ta[d] = lta[ltab_off((uint32_t)d + 1u) + xa];
          tb[d] = ltb[ltab_off((uint32_t)d + 1u) + xb];
        }
      }
    }
    // the nonempty prefix (the intervals along a string only narrow)
#pragma unroll
    for (int d = 0; d < TMAX; ++d) {
      da += (d < dn && ta[d].x <= ta[d].y) ? 1 : 0;
      db += (d < dn && tb[d].x <= tb[d].y) ? 1 : 0;
    }
  }
  // one block of 16 steps; the first block (the only one with table steps) peeled so that the table
  // registers are dead before the others
  auto block = [&](int base, auto first) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(first)::value;
    uint2 ba[16], bb[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int i = base + t;
      if (i < L) {
        uint32_t ca = s[i];
        uint32_t cb = strand_base(ca, 1, comp);
        const bool tA = FIRST && t < TMAX && t < da, tB = FIRST && t < TMAX && t < db;
        WLoad xa, xb;
        if (!tA) wchain_load(ixa, sa0, tx0, A, ca, xa, t == 0);
        if (!tB) wchain_load(ixb, sa1, tx1, B, cb, xb, t == 0);
        if (FIRST && t < TMAX && tA) {
          A.k = ta[t < TMAX ? t : 0].x;
          A.l = ta[t < TMAX ? t : 0].y;
          if (t == da - 1 && sa0 != nullptr && A.k == A.l) A.mode = 1;  // as an Occ step to one row would
        } else {
          wchain_step(ixa, sa0 != nullptr, A, ca, xa);
        }
        if (FIRST && t < TMAX && tB) {
          B.k = tb[t < TMAX ? t : 0].x;
          B.l = tb[t < TMAX ? t : 0].y;
          if (t == db - 1 && sa1 != nullptr && B.k == B.l) B.mode = 1;
        } else {
          wchain_step(ixb, sa1 != nullptr, B, cb, xb);
        }
        ba[t] = make_uint2(A.l - A.k + 1, A.bid);
        lwa += 31 - __builtin_clz(A.l - A.k + 1);
        bb[t] = make_uint2(B.l - B.k + 1, B.bid);
        lwb += 31 - __builtin_clz(B.l - B.k + 1);
      }
    }
#pragma unroll
    for (int t = 0; t < 16; ++t)
      if (base + t < L) wa[base + t] = ba[t];
#pragma unroll
    for (int t = 0; t < 16; ++t)
      if (base + t < L) wb[base + t] = bb[t];
    if (rec) {
      uint32_t x = 0;
#pragma unroll
      for (int t = 0; t < 16; ++t)
        if (base + t < L) {
          rec->put(rec_byte(ba[t], bb[t], pa, pb, base + t == 0, clamp, nb));
          pa = ba[t].x;
          pb = bb[t].x;
          x |= ((uint32_t)s[base + t] & 3u) << (2 * t);
        }
      if (rd) rd[base >> 4] = x;
    }
  };
  if (L > 0) block(0, std::true_type{});
  for (int base = 16; base < L; base += 16) block(base, std::false_type{});
  wa[L] = make_uint2(0u, A.bid + 1);
  wb[L] = make_uint2(0u, B.bid + 1);
  if (rec) rec->put(rec_byte(wa[L], wb[L], pa, pb, L == 0, clamp, nb));
  if (lw) {
    lw[0] = lwa;
    lw[1] = lwb;
    lw[2] = A.bid;
    lw[3] = B.bid;
  }
}

__global__ void __launch_bounds__(256) k_width(AlnArgs A) {
  const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= A.n) return;
  const int64_t r = A.ids ? A.ids[lane] : lane;
  const int L = (int)A.len[r];
  const uint8_t *s = A.seq + A.off[r];
  const bool comp = A.o.mode & MODE_COMPREAD;
  const uint32_t *sa0 = A.jsa[0], *sa1 = A.jsa[1], *tx0 = A.jtxt[0], *tx1 = A.jtxt[1];
  const int tdep = A.ltab[0] ? (int)min(A.tab_k + 1u, 15u) : 0;  // leading steps from the level tables
  uint2 *w0 = A.wbuf + (uint64_t)lane * A.wstride;
  uint2 *w1 = w0 + A.wlen1;
  uint2 *sw0 = w1 + A.wlen1;
  uint2 *sw1 = sw0 + (A.o.seed_len + 1);
  if (A.nN) {
    uint32_t nN = 0;
    for (int j = 0; j < L; ++j) nN += s[j] > 3;
    A.nN[lane] = (uint16_t)(nN > 0xFFFFu ? 0xFFFFu : nN);
  }
  if (A.feat) {
    // search-cost features: sum of log2(width) over both full-length chains, and the seed's
    uint32_t f[4] = {0, 0, 0, 0}, g[4] = {0, 0, 0, 0};
    width_pair(A.ix[0], A.ix[1], L, s, comp, w0, w1, f);
    if (L > A.o.seed_len) width_pair(A.ix[0], A.ix[1], A.o.seed_len, s + (L - A.o.seed_len), comp, sw0, sw1, g);
    A.feat[lane * 4 + 0] = (uint16_t)(f[0] + f[1]);
    A.feat[lane * 4 + 1] = (uint16_t)(g[0] + g[1]);
    A.feat[lane * 4 + 2] = (uint16_t)(f[2] < f[3] ? f[2] : f[3]);
    A.feat[lane * 4 + 3] = (uint16_t)(g[2] < g[3] ? g[2] : g[3]);
    return;
  }
  if (A.cw) {
    // the compact record (engine.h AlnArgs::cw), built from the chains' registers
    uint32_t *rec = A.cw + (uint64_t)lane * A.cw_words;
    uint32_t nN = 0;
    for (int j = 0; j < L; ++j) nN += s[j] > 3;
    const int md = A.o.fnr_pos ? (int)A.maxdiff_tab[L] : A.o.max_diff;
    rec[0] = (uint32_t)L | (nN < 255u ? nN : 255u) << 16 | (uint32_t)md << 24;
    RecOut ro{rec + 1 + A.cw_rw, 0u, 0u};
    width_pair(A.ix[0], A.ix[1], L, s, comp, w0, w1, nullptr, &ro, (uint32_t)md + 1u, 4, rec + 1, sa0, sa1, tx0, tx1,
               A.ltab[0], A.ltab[1], tdep);
    while (ro.off < A.wlen1) ro.put(0u);  // positions past this read's length
    if (L > A.o.seed_len)
      width_pair(A.ix[0], A.ix[1], A.o.seed_len, s + (L - A.o.seed_len), comp, sw0, sw1, nullptr, &ro,
                 (uint32_t)A.o.max_seed_diff + 1u, 3, nullptr, sa0, sa1, tx0, tx1, A.ltab[0], A.ltab[1], tdep);
    ro.flush();
    return;
  }
  width_pair(A.ix[0], A.ix[1], L, s, comp, w0, w1, nullptr, nullptr, 0, 4, nullptr, sa0, sa1, tx0, tx1, A.ltab[0],
             A.ltab[1], tdep);
  if (L > A.o.seed_len)
    width_pair(A.ix[0], A.ix[1], A.o.seed_len, s + (L - A.o.seed_len), comp, sw0, sw1, nullptr, nullptr, 0, 4,
               nullptr, sa0, sa1, tx0, tx1, A.ltab[0], A.ltab[1], tdep);
}

__device__ __forceinline__ int int_log2(uint32_t v) {  // bwtgap.c:93-102
  return v ? 31 - __builtin_clz(v) : 0;
}

// bwt_match_exact_alt (bwt.c:235-250) over str[0..i-1] from (k, l)
__device__ __forceinline__ bool match_exact_alt(const IndexView &ix, int i, const uint8_t *s, int a, bool comp,
                                                uint32_t &k0, uint32_t &l0) {
  uint32_t k = k0, l = l0;
  for (int j = i - 1; j >= 0; --j) {
    uint32_t c = strand_base(s[j], a, comp);
    if (c > 3) return false;
    Fetch1 f;
    fetch1(ix, k - 1, l, c, true, f);
    uint32_t ok, ol;
    occ2_from1(f, c, ok, ol);
    k = l2of(ix, c) + ok + 1;
    l = l2of(ix, c) + ol;
    if (k > l) return false;
  }
  k0 = k;
  l0 = l;
  return true;
}

__global__ void __launch_bounds__(256) k_search(AlnArgs A) {
  const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= A.n) return;
  const AlnOpt o = A.o;
  const IndexView ixv0 = A.ix[0], ixv1 = A.ix[1];
  const int64_t r = A.ids ? A.ids[lane] : lane;
  const int len = (int)A.len[r];
  const uint8_t *s = A.seq + A.off[r];
  const bool comp = o.mode & MODE_COMPREAD;
  uint2 *wbase = A.wbuf + (uint64_t)lane * A.wstride;
  uint2 *const W0 = wbase, *const W1 = wbase + A.wlen1;
  const uint2 *const SW0 = wbase + 2 * A.wlen1, *const SW1 = wbase + 2 * A.wlen1 + (o.seed_len + 1);
  const bool seeded = len > o.seed_len;  // bwtaln.c:127,132
  uint32_t *heads = A.heads + (uint64_t)lane * o.n_stacks;
  uint4 *ent = A.ent + (uint64_t)lane * A.cap;
  uint32_t *prv = A.prev + (uint64_t)lane * A.cap;
  uint4 *out = A.aln + (uint64_t)lane * A.aln_cap;
  uint32_t status = 0;
  int n_aln = 0;

  // per-read local_opt (bwtaln.c:125-126)
  const int opt_max_diff = o.fnr_pos ? (int)A.maxdiff_tab[len] : o.max_diff;
  const int seed_len = o.seed_len;  // only read when seeded
  int best_score = (opt_max_diff + 1) * o.s_mm + (o.max_gapo + 1) * o.s_gapo + (o.max_gape + 1) * o.s_gape;
  int max_diff = opt_max_diff;
  int best_cnt = 0;

  // bwtgap.c:116-122: too many N
  {
    int nN = 0;
    for (int j = 0; j < len; ++j) nN += s[j] > 3;
    if (nN > max_diff) {
      A.n_aln[lane] = 0;
      A.status[lane] = 0;
      return;
    }
  }
  for (int b = 0; b < o.n_stacks; ++b) heads[b] = NIL;
  int best = o.n_stacks, n_entries = 0;
  uint32_t bump = 0, free_head = NIL;  // slots: bump allocator + free list threaded through prv[]
  bool dead = false;

  auto push = [&](int a, int i, uint32_t k, uint32_t l, int n_mm, int n_gapo, int n_gape, int state, int ldp) {
    n_mm &= 0xff; n_gapo &= 0xff; n_gape &= 0xff;  // 8-bit fields (bwtgap.h:9)
    int score = n_mm * o.s_mm + n_gapo * o.s_gapo + n_gape * o.s_gape;
    if (score < 0 || score >= o.n_stacks) { status |= ST_BAD_SCORE; dead = true; return; }
    uint32_t slot;
    if (free_head != NIL) {
      slot = free_head;
      free_head = prv[slot];
    } else {
      if (bump >= A.cap) { status |= ST_STACK_OVERFLOW; dead = true; return; }
      slot = bump++;
    }
    ent[slot] = make_uint4(k, l, (uint32_t)(i & 0xffff) | ((uint32_t)ldp << 16),
                           (uint32_t)a | (uint32_t)state << 1 | (uint32_t)n_mm << 8 | (uint32_t)n_gapo << 16 |
                               (uint32_t)n_gape << 24);
    prv[slot] = heads[score];
    heads[score] = slot;
    ++n_entries;
    if (best > score) best = score;
  };

  push(0, len, 0, ixv0.seq_len, 0, 0, 0, STATE_M, 0);
  push(1, len, 0, ixv0.seq_len, 0, 0, 0, STATE_M, 0);

  while (n_entries && !dead) {
    if (n_entries > o.max_entries) break;
    // gap_pop (bwtgap.c:66-79): top of the lowest non-empty bucket
    uint32_t slot = heads[best];
    const uint4 e = ent[slot];
    const uint32_t pv = prv[slot];
    heads[best] = pv;
    if (slot + 1 == bump) {
      bump = slot;
    } else {
      prv[slot] = free_head;
      free_head = slot;
    }
    --n_entries;
    if (pv == NIL) {
      if (n_entries) {
        int b = best + 1;
        while (b < o.n_stacks && heads[b] == NIL) ++b;
        best = b;
      } else {
        best = o.n_stacks;
      }
    }
    uint32_t k = e.x, l = e.y;
    int i = (int)(e.z & 0xffff), ldp = (int)(e.z >> 16);
    const int a = (int)(e.w & 1), state = (int)((e.w >> 1) & 3);
    const int e_mm = (int)((e.w >> 8) & 0xff), e_go = (int)((e.w >> 16) & 0xff), e_ge = (int)(e.w >> 24);
    const int e_score = (e_mm * o.s_mm + e_go * o.s_gapo + e_ge * o.s_gape) & 0x7ff;  // info>>21
    if (!(o.mode & MODE_NONSTOP) && (uint32_t)e_score > (uint32_t)(best_score + o.s_mm)) break;

    int m = max_diff - (e_mm + e_go);
    if (o.mode & MODE_GAPE) m -= e_ge;
    if (m < 0) continue;
    const IndexView ix = a ? ixv0 : ixv1;
    uint2 *width = a ? W1 : W0;
    const uint2 *sw = a ? SW1 : SW0;
    int m_seed = 0;
    if (seeded) {
      m_seed = o.max_seed_diff - (e_mm + e_go);
      if (o.mode & MODE_GAPE) m_seed -= e_ge;
    }
    if (i > 0 && m < (int)width[i - 1].y) continue;

    bool hit = false;
    if (i == 0) {
      hit = true;
    } else if (m == 0 && (state == STATE_M || (o.mode & MODE_GAPE) || e_ge == o.max_gape)) {
      if (match_exact_alt(ix, i, s, a, comp, k, l)) hit = true;
      else continue;
    }
    if (hit) {
      const int score = e_mm * o.s_mm + e_go * o.s_gapo + e_ge * o.s_gape;
      bool do_add = true;
      if (n_aln == 0) {
        best_score = score;
        int best_diff = e_mm + e_go;
        if (o.mode & MODE_GAPE) best_diff += e_ge;
        if (!(o.mode & MODE_NONSTOP)) max_diff = (best_diff + 1 > opt_max_diff) ? opt_max_diff : best_diff + 1;
      }
      if (score == best_score) best_cnt = (int)((uint32_t)best_cnt + (l - k + 1));
      else if (best_cnt > o.max_top2) break;
      if (e_go) {
        for (int j = 0; j < n_aln && j < (int)A.aln_cap; ++j) {
          uint4 h = out[j];
          if (h.y == k && h.z == l) { do_add = false; break; }
        }
      }
      if (do_add) {
        // gap_shadow (bwtgap.c:81-91) on this strand's width array
        const uint32_t x = l - k + 1, mx = ix.seq_len;
        uint32_t jj = 0;
        for (int q = 0; q < ldp; ++q) {
          uint2 w = width[q];
          if (w.x > x) { w.x -= x; width[q] = w; }
          else if (w.x == x) { ++jj; width[q] = make_uint2(mx - jj, 1u); }
        }
        if (n_aln >= (int)A.aln_cap) { status |= ST_ALN_OVERFLOW; dead = true; break; }
        out[n_aln++] = make_uint4((uint32_t)e_mm | (uint32_t)e_go << 8 | (uint32_t)e_ge << 16 | (uint32_t)a << 24, k,
                                  l, (uint32_t)score);
      }
      continue;
    }

    --i;
    uint32_t cnt_k[4], cnt_l[4];
    {
      Fetch f;
      fetch_pair(ix, k - 1, l, f);
      occ4x2_from(f, cnt_k, cnt_l);
    }
    const uint32_t occ = l - k + 1;
    bool allow_diff = true, allow_M = true;
    if (i > 0) {
      const uint2 w_im1 = width[i - 1], w_i = width[i];
      const int ii = i - (len - seed_len);
      if ((int)w_im1.y > m - 1) allow_diff = false;
      else if ((int)w_im1.y == m - 1 && (int)w_i.y == m - 1 && w_im1.x == w_i.x) allow_M = false;
      if (seeded && ii > 0) {
        const uint2 s_im1 = sw[ii - 1], s_i = sw[ii];
        if ((int)s_im1.y > m_seed - 1) allow_diff = false;
        else if ((int)s_im1.y == m_seed - 1 && (int)s_i.y == m_seed - 1 && s_im1.x == s_i.x) allow_M = false;
      }
    }
    const int tmp = (o.mode & MODE_LOGGAP) ? int_log2((uint32_t)(e_ge + e_go)) / 2 + 1 : e_go + e_ge;
    if (allow_diff && i >= o.indel_end_skip + tmp && len - i >= o.indel_end_skip + tmp) {
      if (state == STATE_M) {
        if (e_go < o.max_gapo) {
          push(a, i, k, l, e_mm, e_go + 1, e_ge, STATE_I, i);
          for (int j = 0; j != 4; ++j) {
            uint32_t kk = l2of(ix, j) + cnt_k[j] + 1, ll = l2of(ix, j) + cnt_l[j];
            if (kk <= ll) push(a, i + 1, kk, ll, e_mm, e_go + 1, e_ge, STATE_D, i + 1);
          }
        }
      } else if (state == STATE_I) {
        if (e_ge < o.max_gape) push(a, i, k, l, e_mm, e_go, e_ge + 1, STATE_I, i);
      } else if (state == STATE_D) {
        if (e_ge < o.max_gape) {
          if (e_ge + e_go < max_diff || occ < (uint32_t)o.max_del_occ) {
            for (int j = 0; j != 4; ++j) {
              uint32_t kk = l2of(ix, j) + cnt_k[j] + 1, ll = l2of(ix, j) + cnt_l[j];
              if (kk <= ll) push(a, i + 1, kk, ll, e_mm, e_go, e_ge + 1, STATE_D, i + 1);
            }
          }
        }
      }
    }
    const uint32_t ci = strand_base(s[i], a, comp);
    if (allow_diff && allow_M) {
      for (int j = 1; j <= 4; ++j) {
        const uint32_t c = (ci + j) & 3;
        const int is_mm = (j != 4 || ci > 3);
        uint32_t kk = l2of(ix, c) + cnt_k[c] + 1, ll = l2of(ix, c) + cnt_l[c];
        if (kk <= ll) push(a, i, kk, ll, e_mm + is_mm, e_go, e_ge, STATE_M, is_mm ? i : ldp);
      }
    } else if (ci < 4) {
      const uint32_t c = ci & 3;
      uint32_t kk = l2of(ix, c) + cnt_k[c] + 1, ll = l2of(ix, c) + cnt_l[c];
      if (kk <= ll) push(a, i, kk, ll, e_mm, e_go, e_ge, STATE_M, ldp);
    }
  }
  A.n_aln[lane] = n_aln;
  A.status[lane] = status;
}

__global__ void __launch_bounds__(256) k_occ4(IndexView ix, int64_t n, const uint32_t *k, uint32_t *cnt) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint32_t o[4];
  occ4(ix, k[t], o);
  cnt[4 * t + 0] = o[0];
  cnt[4 * t + 1] = o[1];
  cnt[4 * t + 2] = o[2];
  cnt[4 * t + 3] = o[3];
}

}  // namespace

hipError_t launch_width(const AlnArgs &a, int block, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  uint64_t grid = (a.n + block - 1) / block;
  hipLaunchKernelGGL(k_width, dim3((unsigned)grid), dim3(block), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_search(const AlnArgs &a, int block, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  uint64_t grid = (a.n + block - 1) / block;
  hipLaunchKernelGGL(k_search, dim3((unsigned)grid), dim3(block), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_occ4(const IndexView &ix, int64_t n, const uint32_t *k, uint32_t *cnt, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_occ4, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ix, n, k, cnt);
  return hipGetLastError();
}

}  // namespace ibwa
