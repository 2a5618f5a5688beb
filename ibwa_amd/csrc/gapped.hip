// gapped.hip -- bwt_match_gap (bwtgap.c:104-264) as a persistent, one-read-
// per-lane state machine in which every loop iteration is exactly one memory
// round trip for every lane.
//
// The reference pops the top of the lowest non-empty score bucket (bucketed
// LIFO, bwtgap.c:45-79).  Here each lane keeps, per bucket, a LIFO linked
// list of 16 B entries in HBM with the list heads in LDS, and keeps the NEXT
// entry to pop ("candidate" C = head of the lowest non-empty bucket) in
// registers.  A pop therefore costs no memory round trip; the entry that
// becomes the next candidate is loaded in the same iteration as the popped
// entry's rank-query blocks, its width bounds and its read symbol.  Pushes
// are fire-and-forget stores; a push into a bucket <= the candidate's simply
// replaces the candidate (it is the new LIFO top / new minimum).
//
// The rank-query blocks (occ64.hip, all four symbols of the k-1 and l rows)
// are fetched speculatively together with the width bound the pop must
// pass (`m < width[i-1].bid`, bwtgap.c:155): measured, fewer than 5 % of
// pops fail it (tools/dfs stats in DESIGN.md), so one round trip per pop
// beats a dependent load.  The same blocks serve the first step of
// bwt_match_exact_alt when the entry goes down the exact path.
//
// Entry (uint4): {k, l, i | last_diff_pos << 16,
//                 prev(16) | n_mm(5) << 16 | n_gapo(3) << 21 | n_gape(4) << 24 | a << 28 | state << 29}
// last_diff_pos: a non-diff push inherits the parent's.
// Stack slots: a per-lane region of CAP1 slots, then one extension region
// from a per-launch pool; a read that needs more (or options that do not fit
// the bit fields) is re-run by the general kernels (aln.hip), exactly.
// Slots are bump-allocated; a popped slot below the bump pointer goes on a
// small per-lane free stack in LDS and is reused by the next pushes, so the
// slots in use track the live entries (the reference's stack size).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "engine.h"
#include "occ.h"

namespace ibwa {

namespace {

constexpr int MODE_GAPE = 0x01, MODE_COMPREAD = 0x02, MODE_LOGGAP = 0x04, MODE_NONSTOP = 0x10;
constexpr int STATE_M = 0, STATE_I = 1, STATE_D = 2;
constexpr int GAP_CHUNK = 64;
constexpr int FREE_DEPTH = 8;  // per-lane LDS stack of popped slots awaiting reuse

// The 64-row bit-plane block (occ64.hip): v[c] = {C[c], 0, P_lo[c], P_hi[c]}.  Four named
// uint4 members, not an array: an array indexed by a runtime symbol is placed in scratch.
struct Blk {
  uint4 v0, v1, v2, v3;
};

__device__ __forceinline__ void load_blk(const uint4 *o, uint32_t row, bool run, Blk &b) {
  if (run) {
    const uint4 *p = o + (size_t)(row >> 6) * 4;
    b.v0 = p[0];
    b.v1 = p[1];
    b.v2 = p[2];
    b.v3 = p[3];
  }
}

__device__ __forceinline__ uint32_t occ_of(const uint4 &v, uint32_t row) {
  const uint32_t o = row & 63;
  const uint32_t mlo = o >= 31 ? 0xFFFFFFFFu : ((2u << o) - 1u);
  const uint32_t mhi = o < 32 ? 0u : (o == 63 ? 0xFFFFFFFFu : ((2u << (o - 32)) - 1u));
  return v.x + (uint32_t)__builtin_popcount(v.z & mlo) + (uint32_t)__builtin_popcount(v.w & mhi);
}

// all four Occ(c, row) from a block; pick one by a runtime symbol with scalar selects
// (a select chain over vector aggregates is lowered to an indexed scratch access)
__device__ __forceinline__ uint4 occ4_of(const Blk &b, uint32_t row) {
  return make_uint4(occ_of(b.v0, row), occ_of(b.v1, row), occ_of(b.v2, row), occ_of(b.v3, row));
}

__device__ __forceinline__ uint32_t pick4(uint4 v, uint32_t c) {
  const uint32_t x = v.x, y = v.y, z = v.z, w = v.w;
  const uint32_t lo = (c & 1) ? y : x, hi = (c & 1) ? w : z;
  return (c & 2) ? hi : lo;
}

__device__ __forceinline__ int int_log2(uint32_t v) { return v ? 31 - __builtin_clz(v) : 0; }

// Entry packing.  Narrow (first pass): 16-bit slot links, i and last_diff_pos 16 bits each.
// Wide (retry pass, reads < 4096 bp): 24-bit links, the top 8 bits in z above 12-bit i / ldp.
template <bool WIDE> struct Ent {
  using Head = typename std::conditional<WIDE, uint32_t, uint16_t>::type;
  static constexpr uint32_t NIL = WIDE ? 0xFFFFFFu : 0xFFFFu;
  static __device__ __forceinline__ uint4 make(uint32_t k, uint32_t l, int i, int ldp, uint32_t prev, int n_mm,
                                               int n_gapo, int n_gape, int a, int state) {
    const uint32_t w = (prev & 0xffffu) | (uint32_t)n_mm << 16 | (uint32_t)n_gapo << 21 | (uint32_t)n_gape << 24 |
                       (uint32_t)a << 28 | (uint32_t)state << 29;
    const uint32_t z = WIDE ? ((uint32_t)i & 0xfffu) | ((uint32_t)ldp & 0xfffu) << 12 | (prev >> 16) << 24
                            : ((uint32_t)i & 0xffffu) | (uint32_t)ldp << 16;
    return make_uint4(k, l, z, w);
  }
  static __device__ __forceinline__ int i(const uint4 &e) { return (int)(WIDE ? e.z & 0xfffu : e.z & 0xffffu); }
  static __device__ __forceinline__ int ldp(const uint4 &e) { return (int)(WIDE ? (e.z >> 12) & 0xfffu : e.z >> 16); }
  static __device__ __forceinline__ uint32_t prev(const uint4 &e) {
    return WIDE ? (e.w & 0xffffu) | (e.z >> 24) << 16 : e.w & 0xffffu;
  }
};

}  // namespace

// lane -> LDS heads: heads[b * blockDim + tid] (bank-friendly: lanes of a wave hit consecutive u16)
template <bool WIDE>
__global__ void __launch_bounds__(256) k_gapped(GapArgs A, unsigned long long *counter) {
  using E = Ent<WIDE>;
  using H = typename E::Head;
  constexpr uint32_t NILH = E::NIL;
  extern __shared__ uint4 lds_raw[];
  H *const lds_heads = reinterpret_cast<H *>(lds_raw);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  const int NB = blockDim.x;
  const AlnOpt o = A.o;
  const IndexView ixv0 = A.ix[0], ixv1 = A.ix[1];
  const bool comp = o.mode & MODE_COMPREAD;
  const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + tid;
  uint4 *const ent1 = A.ent + gtid * A.cap1;  // primary slot region
  uint4 *ent2 = nullptr;                      // extension region (lazy)

  int64_t cur = 0, cend = 0;
  bool more = true;
  // ---- lane state
  int st = 0;  // 0 idle, 1 search (C valid or empty), 2 exact sub-search
  int64_t r = 0;
  int len = 0, opt_max_diff = 0, max_diff = 0, best_score = 0, n_aln = 0;
  int best_cnt = 0, n_entries = 0;
  uint32_t bump = 0, status = 0, n_free = 0;
  H *const free_slots = lds_heads + o.n_stacks * NB;  // free_slots[j * NB + tid]
  bool seeded = false;
  const uint8_t *s = nullptr;
  const uint2 *W0 = nullptr, *W1 = nullptr, *SW0 = nullptr, *SW1 = nullptr;
  uint4 C = make_uint4(0, 0, 0, 0);
  uint32_t C_slot = 0;
  int C_b = 0;
  bool C_valid = false;
  bool C_load = false;  // C's data arrives with this iteration's loads (slot C_slot)
  // exact sub-search state
  uint32_t xk = 0, xl = 0;
  int xj = 0, xa = 0;
  uint4 xe = make_uint4(0, 0, 0, 0);  // the entry that went down the exact path

  auto slot_ptr = [&](uint32_t slot) __attribute__((always_inline)) -> uint4 * {
    return slot < A.cap1 ? ent1 + slot : ent2 + (slot - A.cap1);
  };

  for (;;) {
    // ------------------------------------------------ claim + init new reads
    unsigned long long need = __ballot(st == 0);
    while (need && more) {
      if (cur >= cend) {
        int64_t base = 0;
        if (lane == 0) base = (int64_t)atomicAdd(counter, (unsigned long long)GAP_CHUNK);
        base = __shfl(base, 0);
        if (base >= A.n) { more = false; break; }
        cur = base;
        cend = base + GAP_CHUNK < A.n ? base + GAP_CHUNK : A.n;
      }
      const int rank = __popcll(need & lt_mask);
      const int64_t avail = cend - cur;
      if (st == 0 && rank < avail) {
        r = cur + rank;
        const int64_t rr = A.ids ? A.ids[r] : r;
        len = (int)A.len[rr];
        s = A.seq + A.off[rr];
        opt_max_diff = o.fnr_pos ? (int)A.maxdiff_tab[len] : o.max_diff;
        max_diff = opt_max_diff;
        best_score = (opt_max_diff + 1) * o.s_mm + (o.max_gapo + 1) * o.s_gapo + (o.max_gape + 1) * o.s_gape;
        best_cnt = 0;
        n_aln = 0;
        status = 0;
        seeded = len > o.seed_len;
        const uint2 *wb = A.wbuf + (uint64_t)r * A.wstride;
        W0 = wb;
        W1 = wb + A.wlen1;
        SW0 = wb + 2 * A.wlen1;
        SW1 = SW0 + (o.seed_len + 1);
        if ((int)A.nN[r] > max_diff) {  // bwtgap.c:116-122
          A.n_aln[r] = 0;
          A.status[r] = 0;
        } else {
          for (int b = 0; b < o.n_stacks; ++b) lds_heads[b * NB + tid] = (H)NILH;
          // roots (bwtgap.c:126-127): strand 0 then strand 1, both score 0 -> C = strand 1
          ent1[0] = E::make(0u, ixv0.seq_len, len, 0, NILH, 0, 0, 0, 0, STATE_M);
          C = E::make(0u, ixv0.seq_len, len, 0, 0u, 0, 0, 0, 1, STATE_M);
          ent1[1] = C;
          lds_heads[0 * NB + tid] = 1;
          bump = 2;
          n_free = 0;
          n_entries = 2;
          C_slot = 1;
          C_b = 0;
          C_valid = true;
          C_load = false;
          st = 1;
        }
      }
      const int64_t cnt = __popcll(need);
      cur += avail < cnt ? avail : cnt;
      need = __ballot(st == 0);
    }
    if (__ballot(st != 0) == 0ull) break;

    // ------------------------------------------------ decide this iteration's work
    // search lanes pop C; exact lanes advance one symbol
    bool do_pop = false, finish = false;
    uint4 e = make_uint4(0, 0, 0, 0);
    int a = 0, i = 0, ldp = 0, e_mm = 0, e_go = 0, e_ge = 0, state = 0, m = 0, m_seed = 0;
    if (st == 1) {
      if (n_entries == 0 || n_entries > o.max_entries) {
        finish = true;
      } else {
        e = C;
        a = (int)((e.w >> 28) & 1);
        i = E::i(e);
        ldp = E::ldp(e);
        e_mm = (int)((e.w >> 16) & 31);
        e_go = (int)((e.w >> 21) & 7);
        e_ge = (int)((e.w >> 24) & 15);
        state = (int)((e.w >> 29) & 3);
        const int e_score = (e_mm * o.s_mm + e_go * o.s_gapo + e_ge * o.s_gape) & 0x7ff;
        if (!(o.mode & MODE_NONSTOP) && (uint32_t)e_score > (uint32_t)(best_score + o.s_mm)) {
          finish = true;  // bwtgap.c:143 (after the pop; nothing else observes the stack)
        } else {
          do_pop = true;
          m = max_diff - (e_mm + e_go);
          if (o.mode & MODE_GAPE) m -= e_ge;
          if (seeded) {
            m_seed = o.max_seed_diff - (e_mm + e_go);
            if (o.mode & MODE_GAPE) m_seed -= e_ge;
          }
        }
      }
    }
    // pop bookkeeping (no memory round trip): unlink C, choose the next candidate
    uint32_t load_slot = 0;
    if (do_pop) {
      const uint32_t prev = E::prev(e);
      lds_heads[C_b * NB + tid] = (H)prev;
      --n_entries;
      if (C_slot + 1 == bump) {
        bump = C_slot;
      } else if (n_free < FREE_DEPTH) {
        free_slots[n_free * NB + tid] = (H)C_slot;
        ++n_free;
      }
      if (prev != NILH) {
        load_slot = prev;
        C_load = true;
      } else {
        int b = C_b + 1;
        while (b < o.n_stacks && lds_heads[b * NB + tid] == NILH) ++b;
        if (b < o.n_stacks) {
          load_slot = lds_heads[b * NB + tid];
          C_b = b;
          C_load = true;
        } else {
          C_load = false;
        }
      }
      C_valid = false;
      if (C_load) C_slot = load_slot;
    }

    // ------------------------------------------------ issue every load of this iteration
    const bool srch = do_pop && m >= 0;
    const IndexView ix = a ? ixv0 : ixv1;  // strand a searches bwt[1-a]
    const uint4 *ob = a ? A.o64[0] : A.o64[1];
    uint32_t k = e.x, l = e.y;
    // exact lanes query (xk-1, xl) on bwt[1-xa]
    const IndexView ixq = st == 2 ? (xa ? ixv0 : ixv1) : ix;
    const uint4 *obq = st == 2 ? (xa ? A.o64[0] : A.o64[1]) : ob;
    const uint32_t qk = st == 2 ? xk : k, ql = st == 2 ? xl : l;
    const bool qrun = (srch && i > 0) || (st == 2 && xj >= 0);
    const bool qkneg = qk == 0;
    const bool qshare = !qkneg && ((qk - 1) >> 6) == (ql >> 6);
    Blk bk, bl;
    load_blk(obq, ql, qrun, bl);
    load_blk(obq, qk - 1, qrun && !qkneg && !qshare, bk);
    // width bounds of strand a at positions i-2, i-1 and the seed pair
    const uint2 *Wa = a ? W1 : W0;
    const uint2 *SWa = a ? SW1 : SW0;
    uint2 w_im1 = make_uint2(0, 0), w_im2 = make_uint2(0, 0), sw_lo = make_uint2(0, 0), sw_hi = make_uint2(0, 0);
    const int ii = (i - 1) - (len - o.seed_len);
    if (srch && i > 0) w_im1 = Wa[i - 1];
    if (srch && i > 1) w_im2 = Wa[i - 2];
    if (srch && i > 1 && seeded && ii > 0) {
      sw_lo = SWa[ii - 1];
      sw_hi = SWa[ii];
    }
    // read symbol str[i-1] (search) or str[xj] (exact); strand 1 = complement under COMPREAD
    uint32_t sym = 0;
    if (srch && i > 0) sym = s[i - 1];
    if (st == 2 && xj >= 0) sym = s[xj];
    // next candidate
    uint4 Cn = make_uint4(0, 0, 0, 0);
    if (do_pop && C_load) Cn = *slot_ptr(load_slot);

    // ------------------------------------------------ consume
    if (do_pop && C_load) {
      C = Cn;
      C_valid = true;
    }
    if (finish) {
      A.n_aln[r] = n_aln;
      A.status[r] = status;
      st = 0;
      continue;
    }
    const uint32_t csym = (st == 2 ? xa : a) == 1 && comp && sym < 4 ? 3u - sym : sym;

    if (st == 2) {
      // one step of bwt_match_exact_alt (bwt.c:240-247)
      bool fail = false;
      if (xj >= 0) {
        if (csym > 3) {
          fail = true;
        } else {
          const uint32_t ok = qkneg ? 0u : pick4(occ4_of(qshare ? bl : bk, qk - 1), csym);
          const uint32_t ol = pick4(occ4_of(bl, ql), csym);
          const uint32_t base = l2of(ixq, csym);
          xk = base + ok + 1;
          xl = base + ol;
          if (xk > xl) fail = true;
          --xj;
        }
      }
      if (fail) {
        st = 1;  // no hit (bwtgap.c:162): back to popping
      } else if (xj < 0) {
        // exact path succeeded: hit with the refined interval; fall through to hit handling
        st = 1;
        e = xe;
        a = xa;
        k = xk;
        l = xl;
        ldp = E::ldp(e);
        e_mm = (int)((e.w >> 16) & 31);
        e_go = (int)((e.w >> 21) & 7);
        e_ge = (int)((e.w >> 24) & 15);
        goto hit;
      }
      continue;
    }
    if (!do_pop) continue;
    if (m < 0) continue;                                   // bwtgap.c:147
    if (i > 0 && m < (int)w_im1.y) continue;              // bwtgap.c:155
    if (i == 0) goto hit;                                  // bwtgap.c:159
    if (m == 0 && (state == STATE_M || (o.mode & MODE_GAPE) || e_ge == o.max_gape)) {
      // bwt_match_exact_alt over str[0..i-1] (bwtgap.c:160-163): the first step uses this
      // iteration's blocks; the rest run in sub-state 2
      if (csym > 3) continue;
      const uint32_t ok = qkneg ? 0u : pick4(occ4_of(qshare ? bl : bk, qk - 1), csym);
      const uint32_t ol = pick4(occ4_of(bl, ql), csym);
      const uint32_t base = l2of(ix, csym);
      xk = base + ok + 1;
      xl = base + ol;
      if (xk > xl) continue;
      xj = i - 2;
      xa = a;
      xe = e;
      if (xj >= 0) {
        st = 2;
        continue;
      }
      k = xk;
      l = xl;
      goto hit;
    }
    {
      // ---- expansion (bwtgap.c:200-258)
      const int ni = i - 1;
      // counts as uint4 + select: a dynamically indexed array would live in scratch
      const uint4 ck4 = qkneg ? make_uint4(0, 0, 0, 0)
                              : make_uint4(occ_of(qshare ? bl.v0 : bk.v0, qk - 1),
                                           occ_of(qshare ? bl.v1 : bk.v1, qk - 1),
                                           occ_of(qshare ? bl.v2 : bk.v2, qk - 1),
                                           occ_of(qshare ? bl.v3 : bk.v3, qk - 1));
      const uint4 cl4 = make_uint4(occ_of(bl.v0, ql), occ_of(bl.v1, ql), occ_of(bl.v2, ql), occ_of(bl.v3, ql));
      const uint32_t occ = l - k + 1;
      bool allow_diff = true, allow_M = true;
      if (ni > 0) {
        // width[ni-1] = w_im2, width[ni] = w_im1
        if ((int)w_im2.y > m - 1) allow_diff = false;
        else if ((int)w_im2.y == m - 1 && (int)w_im1.y == m - 1 && w_im2.x == w_im1.x) allow_M = false;
        if (seeded && ii > 0) {
          if ((int)sw_lo.y > m_seed - 1) allow_diff = false;
          else if ((int)sw_lo.y == m_seed - 1 && (int)sw_hi.y == m_seed - 1 && sw_lo.x == sw_hi.x) allow_M = false;
        }
      }
      // push: link into bucket `sc`, keep C = head of the lowest non-empty bucket
      auto push = [&](int pi, uint32_t pk, uint32_t pl, int n_mm, int n_gapo, int n_gape, int pstate,
                      int pldp) __attribute__((always_inline)) {
        const int sc = n_mm * o.s_mm + n_gapo * o.s_gapo + n_gape * o.s_gape;
        if (sc >= o.n_stacks) { status |= ST_BAD_SCORE; return; }
        if (n_mm > 31 || n_gapo > 7 || n_gape > 15) { status |= ST_STACK_OVERFLOW; return; }
        uint32_t slot;
        if (n_free) {
          --n_free;
          slot = free_slots[n_free * NB + tid];
        } else {
          if (bump >= A.cap1 + A.cap2 || bump >= NILH) { status |= ST_STACK_OVERFLOW; return; }
          if (bump >= A.cap1 && ent2 == nullptr) {
            unsigned long long x = atomicAdd(A.pool_next, 1ull);
            if (x >= A.pool_n) { status |= ST_STACK_OVERFLOW; return; }
            ent2 = A.pool + x * A.cap2;
          }
          slot = bump++;
        }
        const uint32_t hd = lds_heads[sc * NB + tid];
        const uint4 ne = E::make(pk, pl, pi, pldp, hd, n_mm, n_gapo, n_gape, a, pstate);
        *slot_ptr(slot) = ne;
        lds_heads[sc * NB + tid] = (H)slot;
        ++n_entries;
        if (!C_valid || sc <= C_b) {
          C = ne;
          C_slot = slot;
          C_b = sc;
          C_valid = true;
        }
      };
      const int tmp = (o.mode & MODE_LOGGAP) ? int_log2((uint32_t)(e_ge + e_go)) / 2 + 1 : e_go + e_ge;
      if (allow_diff && ni >= o.indel_end_skip + tmp && len - ni >= o.indel_end_skip + tmp) {
        if (state == STATE_M) {
          if (e_go < o.max_gapo) {
            push(ni, k, l, e_mm, e_go + 1, e_ge, STATE_I, ni);
            for (int j = 0; j != 4; ++j) {
              const uint32_t kk = l2of(ix, j) + pick4(ck4, j) + 1, ll = l2of(ix, j) + pick4(cl4, j);
              if (kk <= ll) push(ni + 1, kk, ll, e_mm, e_go + 1, e_ge, STATE_D, ni + 1);
            }
          }
        } else if (state == STATE_I) {
          if (e_ge < o.max_gape) push(ni, k, l, e_mm, e_go, e_ge + 1, STATE_I, ni);
        } else if (state == STATE_D) {
          if (e_ge < o.max_gape && (e_ge + e_go < max_diff || occ < (uint32_t)o.max_del_occ)) {
            for (int j = 0; j != 4; ++j) {
              const uint32_t kk = l2of(ix, j) + pick4(ck4, j) + 1, ll = l2of(ix, j) + pick4(cl4, j);
              if (kk <= ll) push(ni + 1, kk, ll, e_mm, e_go, e_ge + 1, STATE_D, ni + 1);
            }
          }
        }
      }
      if (allow_diff && allow_M) {
        for (int j = 1; j <= 4; ++j) {
          const uint32_t c = (csym + j) & 3;
          const int is_mm = (j != 4 || csym > 3);
          const uint32_t kk = l2of(ix, c) + pick4(ck4, c) + 1, ll = l2of(ix, c) + pick4(cl4, c);
          if (kk <= ll) push(ni, kk, ll, e_mm + is_mm, e_go, e_ge, STATE_M, is_mm ? ni : ldp);
        }
      } else if (csym < 4) {
        const uint32_t c = csym;
        const uint32_t kk = l2of(ix, c) + pick4(ck4, c) + 1, ll = l2of(ix, c) + pick4(cl4, c);
        if (kk <= ll) push(ni, kk, ll, e_mm, e_go, e_ge, STATE_M, ldp);
      }
      if (status) {  // overflow / bad score: give the read to the general kernels
        A.n_aln[r] = 0;
        A.status[r] = status;
        st = 0;
      }
      continue;
    }
  hit : {
    // ---- hit (bwtgap.c:165-197)
    const int score = e_mm * o.s_mm + e_go * o.s_gapo + e_ge * o.s_gape;
    bool do_add = true;
    if (n_aln == 0) {
      best_score = score;
      int best_diff = e_mm + e_go;
      if (o.mode & MODE_GAPE) best_diff += e_ge;
      if (!(o.mode & MODE_NONSTOP)) max_diff = (best_diff + 1 > opt_max_diff) ? opt_max_diff : best_diff + 1;
    }
    uint4 *out = A.aln + (uint64_t)r * A.aln_cap;
    if (score == best_score) {
      best_cnt = (int)((uint32_t)best_cnt + (l - k + 1));
    } else if (best_cnt > o.max_top2) {
      A.n_aln[r] = n_aln;
      A.status[r] = 0;
      st = 0;
      continue;
    }
    if (e_go) {
      for (int j = 0; j < n_aln; ++j) {
        const uint4 h = out[j];
        if (h.y == k && h.z == l) { do_add = false; break; }
      }
    }
    if (do_add) {
      // gap_shadow (bwtgap.c:81-91) on this strand's width array
      uint2 *width = const_cast<uint2 *>(a ? W1 : W0);
      const uint32_t x = l - k + 1, mx = ix.seq_len;
      uint32_t jj = 0;
      for (int q = 0; q < ldp; ++q) {
        uint2 w = width[q];
        if (w.x > x) { w.x -= x; width[q] = w; }
        else if (w.x == x) { ++jj; width[q] = make_uint2(mx - jj, 1u); }
      }
      if (n_aln >= (int)A.aln_cap) {
        A.n_aln[r] = 0;
        A.status[r] = ST_ALN_OVERFLOW;
        st = 0;
        continue;
      }
      out[n_aln++] = make_uint4((uint32_t)e_mm | (uint32_t)e_go << 8 | (uint32_t)e_ge << 16 | (uint32_t)a << 24, k, l,
                                (uint32_t)score);
    }
    continue;
  }
  }
}

size_t gapped_lds_bytes(int n_stacks, int block, bool wide) {
  return (size_t)(n_stacks + FREE_DEPTH) * block * (wide ? 4 : 2);
}

hipError_t launch_gapped(const GapArgs &g, unsigned long long *d_counter, int blocks, int block, bool wide,
                         hipStream_t st) {
  if (g.n <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(d_counter, 0, 2 * sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  const size_t lds = gapped_lds_bytes(g.o.n_stacks, block, wide);
  if (wide)
    hipLaunchKernelGGL(k_gapped<true>, dim3(blocks), dim3(block), lds, st, g, d_counter);
  else
    hipLaunchKernelGGL(k_gapped<false>, dim3(blocks), dim3(block), lds, st, g, d_counter);
  return hipGetLastError();
}

}  // namespace ibwa
