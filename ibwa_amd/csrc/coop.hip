// coop.hip -- bwt_match_gap (bwtgap.c:104-264) for the heavy reads: one read per
// wavefront, its search spread over the 64 lanes, results bit-identical to the
// sequential search.
//
// Why the search parallelises exactly.  The reference pops the top of the
// lowest non-empty score bucket (bucketed LIFO, bwtgap.c:45-79).  Every child
// of an entry scores at least its parent (penalties are positive; the engine
// rejects others) and only the match child (pushed last, bwtgap.c:244-258)
// scores the same, so:
//   * the search visits score levels in increasing order, and nothing is ever
//     pushed into the level being processed except match children;
//   * a match child is popped right after its parent's expansion.
// So a level is a fixed list of entries (the bucket at the time the level
// starts, popped from the top), and each entry starts a "match chain": the
// entry, its match child, that one's match child, ..., ending in a prune
// (bwtgap.c:147,155), an expansion without a match child, a hit at i == 0
// (:159) or an exact tail (bwt_match_exact_alt, :160-163).  Between two hits
// the only state a chain reads is fixed (max_diff, best_score, the width arrays
// gap_shadow rewrites, :81-91), so the chains of a level are independent: the
// lanes run them concurrently, each writing its children, in the reference's
// push order, to a private staging ring.  A reorder buffer of chain records
// (LDS) commits finished chains strictly in pop order: their children are
// appended to the target buckets by a wave prefix sum, which reproduces the
// reference's bucket contents and order exactly.  A chain that ends in a hit
// is a barrier: chains after it were run with stale state, so they are
// discarded (their staging rolled back) and re-run once the hit (top-2 rule,
// dedup, gap_shadow, max_diff) has been applied.
//
// Reasons a read is handed on (status bits 8-15, diagnostics): 1 read too long / seed
// too long / too many buckets / staging too small, 3 page pool empty, 4 a bucket past
// COOP_MAXP pages, 5 runaway guard.  Such reads go to the sequential kernel
// (gapped.hip, wide).
//
// The max_entries check before each pop (bwtgap.c:138) is exact.  Inside a
// chain the stack size before pop t is (size before the chain's first pop) +
// (children the chain staged before pop t): each consumed match child was
// pushed and popped.  Staged counts only grow, so the largest of these is the
// count at the chain's last pop, which the chain record carries.  The commit
// knows the size before each chain's first pop (prefix sum over the chains
// before it), so it finds the first chain whose last pop would see more than
// max_entries: the reference breaks before that pop, so neither that chain
// (whose only possible hit is its last pop) nor anything after it counts, and
// the read ends with the hits committed so far.
//
// Storage per wave: LDS holds the read's two strands, its width arrays (so
// gap_shadow and the pruning tests are LDS work), bucket sizes, the page
// directories of the level and its three target buckets, and the chain
// records.  Buckets live in 128 KiB pages of a global pool (per-wave free
// stack, global bump pointer); staging rings are per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine.h"
#include "occ.h"

namespace ibwa {

namespace {

constexpr int MODE_GAPE = 0x01, MODE_COMPREAD = 0x02, MODE_LOGGAP = 0x04, MODE_NONSTOP = 0x10;
constexpr int STATE_M = 0, STATE_I = 1, STATE_D = 2;
// Gap group: a gap-opening expansion stages its insertion child with its deletion children pending
// (ldp field = their symbols; the group's ldp is its i) as one entry in STATE_G.  95 % of gap-open
// children on a GRCh37-sized genome are never popped, so the deletions are spelled out only when
// the group's level is reached (expand_groups); until then the group counts as all its entries in
// the stack size (bwtgap.c:138).
constexpr int STATE_G = 3;
constexpr int RREC = COOP_RREC;      // chain records in flight (ring)
constexpr int MAXP = COOP_MAXP;      // pages per bucket
constexpr int NSTK = COOP_NSTK;      // buckets
constexpr uint32_t NONE = 0xFFFFFFFFu;

// lane states
constexpr int L_IDLE = 0, L_FETCH = 1, L_EXP = 2, L_TAIL = 3;
// prologue chain records: the root chain ended in a hit / did not run (read not for this kernel)
constexpr uint32_t PRO_HIT = 1, PRO_SKIP = 2;

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

__device__ __forceinline__ uint32_t pick4(uint4 v, uint32_t c) {
  const uint32_t lo = (c & 1) ? v.y : v.x, hi = (c & 1) ? v.w : v.z;
  return (c & 2) ? hi : lo;
}

__device__ __forceinline__ int int_log2(uint32_t v) { return v ? 31 - __builtin_clz(v) : 0; }

// wave-wide exclusive prefix sum and total (64 lanes, all active): DPP row shifts within the rows
// of 16 lanes, then the row broadcasts of lanes 15 and 31 -- six VALU steps instead of six
// ds_bpermute round trips through the LDS crossbar
__device__ __forceinline__ uint32_t wave_excl(uint32_t v, int lane, uint32_t &total) {
  (void)lane;
  uint32_t x = v;
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  return x - v;
}

// wave-wide minimum (64 lanes, all active), the same DPP steps as wave_excl; lane 63 ends with it
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
  const int NO = -1;  // 0xFFFFFFFF: the identity for lanes with no source
  auto mn = [](uint32_t a, int b) __attribute__((always_inline)) { return a < (uint32_t)b ? a : (uint32_t)b; };
  v = mn(v, __builtin_amdgcn_update_dpp(NO, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
  v = mn(v, __builtin_amdgcn_update_dpp(NO, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
  v = mn(v, __builtin_amdgcn_update_dpp(NO, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
  v = mn(v, __builtin_amdgcn_update_dpp(NO, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
  v = mn(v, __builtin_amdgcn_update_dpp(NO, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = mn(v, __builtin_amdgcn_update_dpp(NO, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// entry (uint4): {k, l, i | ldp << 10 | rank << 20, n_mm | n_gapo << 8 | n_gape << 16 | a << 24 | state << 25
//                  | cat << 27}
// i, ldp <= COOP_MAXLEN < 1024.  rank / cat: a staged child's target bucket (0..2 = mismatch, gap
// extension, gap open, merged when penalties coincide) and its index among the chain's children of
// that bucket -- so a commit can place every child independently.
__device__ __forceinline__ uint4 mk_ent(uint32_t k, uint32_t l, int i, int ldp, int n_mm, int n_gapo, int n_gape,
                                        int a, int state, uint32_t cat = 0, uint32_t rank = 0) {
  return make_uint4(k, l, (uint32_t)i | (uint32_t)ldp << 10 | rank << 20,
                    (uint32_t)n_mm | (uint32_t)n_gapo << 8 | (uint32_t)n_gape << 16 | (uint32_t)a << 24 |
                        (uint32_t)state << 25 | cat << 27);
}

// A node of a match chain (a popped entry, or the match child that continues the chain).
struct Node {
  uint32_t k, l;
  int i, ldp, e_mm, e_go, e_ge, a, state;
};

// The widths an expansion at read position ni reads (bwtgap.c:205-214): width[ni-1], width[ni] and
// the seed widths at ii-1, ii (ii = ni - (len - seed_len)); {w, bid}.
struct ExpW {
  uint2 im2, im1, slo, shi;
};

// bwtgap.c:200-258 for node nd with the Occ blocks of rows k-1 (bk) and l (bl) loaded (k_coop_roots;
// k_coop runs the same steps inline): stages the children other than the match child, in the
// reference's push order, each tagged with its target bucket category and its rank among the
// chain's children of that category; returns whether the match child exists (it continues the
// chain: its interval in mk, ml).  csym: the read symbol at i-1; w: the widths it tests.
__device__ __forceinline__ bool expand_node(const AlnOpt &o, uint4 L2, const Blk &bl, Blk bk, bool qkneg,
                                            bool qshare, const Node &nd, int max_diff, bool seeded, int len,
                                            uint32_t csym, const ExpW &w, int t0, int t1, int q1, int q2, uint4 *stg,
                                            uint32_t &stg_w, uint32_t smask, uint32_t &cnt0, uint32_t &cnt1,
                                            uint32_t &cnt2, uint32_t &cex, uint32_t &cgq, uint32_t &mk, uint32_t &ml) {
  const bool gape = o.mode & MODE_GAPE;
  const uint32_t qk = nd.k, ql = nd.l;
  if (qshare) bk = bl;
  uint4 KK, LL;
  {
    const uint4 cl4 = make_uint4(occ_of(bl.v0, ql), occ_of(bl.v1, ql), occ_of(bl.v2, ql), occ_of(bl.v3, ql));
    const uint4 ck4 = qkneg ? make_uint4(0, 0, 0, 0)
                            : make_uint4(occ_of(bk.v0, qk - 1), occ_of(bk.v1, qk - 1), occ_of(bk.v2, qk - 1),
                                         occ_of(bk.v3, qk - 1));
    KK = make_uint4(L2.x + ck4.x + 1, L2.y + ck4.y + 1, L2.z + ck4.z + 1, L2.w + ck4.w + 1);
    LL = make_uint4(L2.x + cl4.x, L2.y + cl4.y, L2.z + cl4.z, L2.w + cl4.w);
  }
  const int e_mm = nd.e_mm, e_go = nd.e_go, e_ge = nd.e_ge, state = nd.state;
  int m = max_diff - (e_mm + e_go);
  if (gape) m -= e_ge;
  int m_seed = 0;
  if (seeded) {
    m_seed = o.max_seed_diff - (e_mm + e_go);
    if (gape) m_seed -= e_ge;
  }
  const int ni = nd.i - 1;
  const uint32_t occ = nd.l - nd.k + 1;
  bool allow_diff = true, allow_M = true;
  if (ni > 0) {
    const int ii = ni - (len - o.seed_len);
    if ((int)w.im2.y > m - 1) allow_diff = false;
    else if ((int)w.im2.y == m - 1 && (int)w.im1.y == m - 1 && w.im2.x == w.im1.x) allow_M = false;
    if (seeded && ii > 0) {
      if ((int)w.slo.y > m_seed - 1) allow_diff = false;
      else if ((int)w.slo.y == m_seed - 1 && (int)w.shi.y == m_seed - 1 && w.slo.x == w.shi.x) allow_M = false;
    }
  }
  const uint32_t ne4 = (KK.x <= LL.x ? 1u : 0u) | (KK.y <= LL.y ? 2u : 0u) | (KK.z <= LL.z ? 4u : 0u) |
                       (KK.w <= LL.w ? 8u : 0u);
  const int tmp = (o.mode & MODE_LOGGAP) ? int_log2((uint32_t)(e_ge + e_go)) / 2 + 1 : e_go + e_ge;
  uint32_t vm = 0;
  if (allow_diff && ni >= o.indel_end_skip + tmp && len - ni >= o.indel_end_skip + tmp) {
    if (state == STATE_M) {
      if (e_go < o.max_gapo) vm = 1u | ne4 << 1;
    } else if (state == STATE_I) {
      if (e_ge < o.max_gape) vm = 1u;
    } else if (state == STATE_D) {
      if (e_ge < o.max_gape && (e_ge + e_go < max_diff || occ < (uint32_t)o.max_del_occ)) vm = ne4 << 1;
    }
  }
  const uint32_t rot = (csym + 1) & 3;
  const uint32_t ner = ((ne4 >> rot) | (ne4 << (4 - rot))) & 15u;
  if (allow_diff && allow_M) vm |= ner << 5;
  else if (csym < 4) vm |= ner & 8u ? 1u << 8 : 0u;
  // bit 8 with csym < 4 is the match child: it continues the chain instead of being staged
  const bool match = (vm >> 8) & 1u && csym < 4;
  if (match) vm &= ~(1u << 8);
  const int sc_base = e_mm * o.s_mm + e_go * o.s_gapo + e_ge * o.s_gape;
  const int sc_gap = state == STATE_M ? o.s_gapo : o.s_gape;
  // a gap-opening expansion's deletions ride on its insertion child (gap group)
  const uint32_t gdm = state == STATE_M && (vm & 1u) ? (vm >> 1) & 15u : 0u;
  vm &= ~(gdm << 1);
  while (vm) {
    const uint32_t j = (uint32_t)__builtin_ctz(vm);
    vm &= vm - 1;
    const bool is_ins = j == 0, is_del = j - 1 < 4, is_sym = j >= 5;
    const uint32_t cc = is_del ? j - 1 : (csym + j - 4) & 3;
    const uint32_t pk = is_ins ? nd.k : pick4(KK, cc);
    const uint32_t pl = is_ins ? nd.l : pick4(LL, cc);
    const bool open = !is_sym && state == STATE_M;
    const int n_mm = e_mm + (is_sym ? 1 : 0);  // staged symbol children are mismatches
    const int n_gapo = e_go + (open ? 1 : 0), n_gape = e_ge + (!is_sym && !open ? 1 : 0);
    const int pi = is_del ? ni + 1 : ni;
    const int pstate = is_ins ? STATE_I : is_del ? STATE_D : STATE_M;
    const int sc = sc_base + (is_sym ? o.s_mm : sc_gap);
    const int q = sc == t0 ? 0 : sc == t1 ? q1 : q2;
    const uint32_t rk = q == 0 ? cnt0++ : q == 1 ? cnt1++ : cnt2++;
    const bool grp = is_ins && gdm;
    stg[(stg_w++) & smask] = mk_ent(pk, pl, pi, grp ? (int)gdm : pi, n_mm, n_gapo, n_gape, nd.a, grp ? STATE_G : pstate,
                                    (uint32_t)q, rk);
    if (grp) {
      cex += (uint32_t)__builtin_popcount(gdm);
      cgq |= 1u << q;
    }
  }
  if (match) {
    mk = pick4(KK, csym);
    ml = pick4(LL, csym);
  }
  return match;
}

// Level start with gap groups (bucket s, N entries on the pages of dirc0): spell each group out as
// the reference pushed it (bwtgap.c:221-227: the insertion, then the deletions A..T, bottom to top)
// into new pages, whose ids go to dir_s (the bucket's global directory row) and dirc0.  The
// deletions' intervals are the symbol steps of the group's own (k, l).  Returns {entries, n_free},
// entries >= GRP_FAIL | why on a page shortage.  Out of line: inlined into k_coop its registers
// spilled into the chain loop (k_coop +40 %, same-box A/B); it runs once per such level.
constexpr uint32_t GRP_FAIL = 0xFFFFFFF0u;

__device__ __noinline__ uint2 expand_groups(uint4 *pool, const uint4 *o0, const uint4 *o1, uint4 L2, uint32_t *dir_s,
                                            uint32_t *dirc0, uint32_t *freel, uint32_t n_free, uint32_t freecap,
                                            uint32_t *pool_next, uint32_t pool_pages, uint32_t N, uint32_t old_np,
                                            int lane) {
  auto ent_at = [&](uint32_t j) -> uint4 {
    return pool[((uint64_t)dirc0[j >> COOP_PG_LOG2] << COOP_PG_LOG2) + (j & (COOP_PG - 1))];
  };
  auto size_of = [](const uint4 &e) -> uint32_t {
    return ((e.w >> 25) & 3u) == (uint32_t)STATE_G ? 1u + (uint32_t)__builtin_popcount((e.z >> 10) & 15u) : 1u;
  };
  uint32_t nvt = 0;
  for (uint32_t b0 = 0; b0 < N; b0 += 64) {
    const uint32_t j = b0 + (uint32_t)lane;
    uint32_t t = 0;
    wave_excl(j < N ? size_of(ent_at(j)) : 0u, lane, t);
    nvt += t;
  }
  const uint32_t npv = (nvt + COOP_PG - 1) >> COOP_PG_LOG2;
  if (npv > MAXP) return make_uint2(GRP_FAIL | 4u, n_free);
  for (uint32_t pq = 0; pq < npv; ++pq) {  // the new pages: the wave's free stack, else the global pool
    uint32_t p;
    if (n_free) {
      p = freel[--n_free];
    } else {
      uint32_t q = 0;
      if (lane == 0) q = atomicAdd(pool_next, 1u);
      q = __shfl(q, 0);
      if (q >= pool_pages) return make_uint2(GRP_FAIL | 3u, n_free);
      p = q;
    }
    if (lane == 0) dir_s[pq] = p;
  }
  __threadfence_block();
  __syncthreads();
  auto put = [&](uint32_t vpos, const uint4 &x) {
    pool[((uint64_t)dir_s[vpos >> COOP_PG_LOG2] << COOP_PG_LOG2) + (vpos & (COOP_PG - 1))] = x;
  };
  uint32_t vbase = 0;
  for (uint32_t b0 = 0; b0 < N; b0 += 64) {
    const uint32_t j = b0 + (uint32_t)lane;
    const uint4 e = j < N ? ent_at(j) : make_uint4(0, 0, 0, 0);
    const bool grp = j < N && ((e.w >> 25) & 3u) == (uint32_t)STATE_G;
    uint32_t t = 0;
    const uint32_t vo = vbase + wave_excl(j < N ? size_of(e) : 0u, lane, t);
    vbase += t;
    if (j < N && !grp) put(vo, e);
    if (grp) {
      const uint4 *ob = (e.w >> 24) & 1u ? o0 : o1;  // strand a searches bwt[1-a]
      const uint32_t gi = e.z & 0x3ffu, dm = (e.z >> 10) & 15u;
      // the insertion child: the group itself, its deletions spelled out
      put(vo, make_uint4(e.x, e.y, gi | gi << 10, (e.w & ~(3u << 25)) | (uint32_t)STATE_I << 25));
      uint32_t r = 1;
      for (uint32_t cc = 0; cc < 4; ++cc) {
        if (dm & (1u << cc)) {
          const uint32_t l2 = pick4(L2, cc);
          const uint32_t dl = l2 + occ_of(ob[(size_t)(e.y >> 6) * 4 + cc], e.y);
          uint32_t dk = l2 + 1u;
          if (e.x != 0) dk += occ_of(ob[(size_t)((e.x - 1) >> 6) * 4 + cc], e.x - 1);
          put(vo + r, make_uint4(dk, dl, (gi + 1) | (gi + 1) << 10, (e.w & ~(3u << 25)) | (uint32_t)STATE_D << 25));
          ++r;
        }
      }
    }
  }
  __threadfence_block();
  __syncthreads();
  // the old pages back (beyond the free stack's room they are dropped), the new directory in
  const uint32_t room = freecap - n_free, nf = old_np < room ? old_np : room;
  for (uint32_t j = lane; j < nf; j += 64) freel[n_free + j] = dirc0[j];
  n_free += nf;
  __syncthreads();
  for (uint32_t j = lane; j < npv; j += 64) dirc0[j] = dir_s[j];
  return make_uint2(nvt, n_free);
}

struct Shm {
  uint4 recA[RREC];   // {staging start, cnt0 | cnt1 << 16, cnt2 | ring << 16 | hit << 24 | gap-group categories << 25,
                      //  done (1) | stack growth before the chain's last pop << 1 (16 bits) |
                      //  deletions pending in its gap groups << 17}
  uint32_t dirc[4][MAXP];  // page ids of the level's bucket and of its (up to) three target buckets
  uint32_t nb[NSTK];       // entries per bucket
  uint16_t np[NSTK];       // pages per bucket (<= MAXP)
  // width arrays (bwt_width_t {w, bid}) of strands 0 / 1 and the seed widths, split so that the
  // bids (<= COOP_MAXLEN + 1) take 16 bits: with the 128-record ring the wave's LDS fits 12 waves
  // per CU
  uint32_t Ww[2][COOP_MAXLEN + 1];
  uint32_t SWw[2][COOP_SEEDMAX + 1];
  uint16_t Wb[2][COOP_MAXLEN + 2];
  uint16_t SWb[2][COOP_SEEDMAX + 1];
  uint8_t str[COOP_MAXLEN];      // bwa_seq_t.seq; strand 1 reads it complemented (COMPREAD)
  uint32_t gm[NSTK / 32];        // buckets holding gap groups
  uint32_t gq;                   // target categories (bit q) that this level's commits gave gap groups
  uint32_t head[64];             // per-lane staging ring: first uncommitted slot
  uint32_t rb[64];               // per-lane staging rollback point (discarded chains)
};

// Resume a read from the first pass's state at a level boundary (GapArgs::rdump): {entries, hits,
// lowest score, stack size}, {best_score, best_cnt, max_diff}, the live entries in slot order (per
// bucket bottom to top), the hits in the order they were added.  gap_shadow (bwtgap.c:81-91) of
// each hit is replayed, in order, on widths k_width computed afresh (replay; else the widths are
// the first pass's own, already shadowed); each entry goes to the top of its bucket.  Out of line: k_coop's chain loop keeps its registers.
struct ResumeOut {
  int s, best_score, best_cnt, max_diff, n_aln;
  uint32_t n_live, status, n_free;
};
__device__ __noinline__ ResumeOut resume_state(const uint4 *rs, Shm *S, uint4 *pool, uint32_t *dir, uint4 *hitv,
                                               uint32_t hcap, uint32_t *freel, uint32_t n_free, uint32_t *pool_next,
                                               uint32_t pool_pages, uint32_t seq_len, int s_mm, int s_gapo, int s_gape,
                                               int n_stacks, int lane, bool replay) {
  ResumeOut R;
  __syncthreads();
  const uint4 h0 = rs[0], h1 = rs[1];
  const uint32_t ne = h0.x, nh = h0.y;
  R.s = (int)h0.z;
  R.n_live = h0.w;
  R.best_score = (int)h1.x;
  R.best_cnt = (int)h1.y;
  R.max_diff = (int)h1.z;
  R.status = 0;
  for (uint32_t j = 0; j < nh && j < hcap; ++j) {
    const uint4 h = rs[RD_HDR + ne + j];
    const int h_a = (int)((h.x >> 24) & 1u), h_ldp = replay ? (int)(h.w >> 16) : 0;
    const uint32_t x = h.z - h.y + 1u;
    uint32_t jrun = 0;
    for (int base = 0; base < h_ldp; base += 64) {
      const int q = base + lane;
      uint2 w = q < h_ldp ? make_uint2(S->Ww[h_a][q], S->Wb[h_a][q]) : make_uint2(0, 0);
      const bool eq = q < h_ldp && w.x == x;
      const unsigned long long em = __ballot(eq);
      if (q < h_ldp) {
        if (w.x > x) {
          S->Ww[h_a][q] = w.x - x;
        } else if (eq) {
          S->Ww[h_a][q] = seq_len - (jrun + (uint32_t)__popcll(em & ((1ull << lane) - 1ull)) + 1u);
          S->Wb[h_a][q] = 1u;
        }
      }
      jrun += (uint32_t)__popcll(em);
    }
    if (lane == 0) hitv[j] = make_uint4(h.x, h.y, h.z, h.w & 0xFFFFu);
  }
  R.n_aln = (int)nh;
  if (nh > hcap) R.status = ST_ALN_OVERFLOW;
  // a bucket's page ids also in LDS (S->dirc, free until the levels start: 8 pages of 8192 entries
  // per bucket cover the first pass's 64 k slots)
  uint32_t *const pc8 = &S->dirc[0][0];
  for (uint32_t b0 = 0; b0 < ne && R.status == 0; b0 += 64) {
    const uint32_t j = b0 + (uint32_t)lane;
    uint4 ce = make_uint4(0, 0, 0, 0);
    int b = -1;
    bool grp = false;
    if (j < ne) {
      const uint4 e = rs[RD_HDR + j];
      const int e_mm = (int)((e.w >> 16) & 31u), e_go = (int)((e.w >> 21) & 7u), e_ge = (int)((e.w >> 24) & 15u);
      const int est = (int)((e.w >> 29) & 3u);
      ce = mk_ent(e.x, e.y, (int)(e.z & 0xFFFFu), (int)(e.z >> 16), e_mm, e_go, e_ge, (int)((e.w >> 28) & 1u), est);
      b = e_mm * s_mm + e_go * s_gapo + e_ge * s_gape;
      grp = est == STATE_G;
      if (b >= n_stacks) b = NSTK;  // not from the first pass; fails below
    }
    unsigned long long pend = __ballot(b >= 0);
    while (pend) {
      const int bb = __shfl(b, (int)__builtin_ctzll(pend));
      const unsigned long long mm = __ballot(b == bb);
      pend &= ~mm;
      if (bb >= n_stacks) {
        R.status = ST_STACK_OVERFLOW | 1u << 8;
        break;
      }
      const uint32_t base = S->nb[bb], tot = (uint32_t)__popcll(mm);
      const uint32_t need_p = (base + tot + COOP_PG - 1u) >> COOP_PG_LOG2;
      uint32_t npb = S->np[bb];
      while (npb < need_p) {
        uint32_t p = NONE;
        if (npb < 8u) {
          if (n_free) {
            --n_free;
            p = freel[n_free];
          } else {
            uint32_t q = 0;
            if (lane == 0) q = atomicAdd(pool_next, 1u);
            q = __shfl(q, 0);
            p = q < pool_pages ? q : NONE;
          }
        }
        if (p == NONE) {
          R.status = ST_STACK_OVERFLOW | 3u << 8;
          break;
        }
        if (lane == 0) {
          pc8[bb * 8 + npb] = p;
          dir[bb * MAXP + npb] = p;
        }
        ++npb;
      }
      __syncthreads();
      if (R.status) break;
      if (b == bb) {
        const uint32_t pos = base + (uint32_t)__popcll(mm & ((1ull << lane) - 1ull));
        pool[((uint64_t)pc8[bb * 8 + (pos >> COOP_PG_LOG2)] << COOP_PG_LOG2) + (pos & (COOP_PG - 1u))] = ce;
      }
      const bool g = __ballot(b == bb && grp) != 0ull;
      __syncthreads();
      if (lane == 0) {
        S->np[bb] = (uint16_t)npb;
        S->nb[bb] = base + tot;
        if (g) S->gm[(uint32_t)bb >> 5] |= 1u << (bb & 31);
      }
      __syncthreads();
    }
  }
  __threadfence_block();
  __syncthreads();
  R.n_free = n_free;
  return R;
}

}  // namespace

template <bool PROF>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) k_coop(CoopArgs A,
                                                                                     unsigned long long *counter) {
  __shared__ Shm S;
  const int lane = threadIdx.x;
  const uint64_t wave = blockIdx.x;
  const AlnOpt o = A.o;
  const bool comp = o.mode & MODE_COMPREAD;
  // read symbol x of strand a: strand 1 is the complement under COMPREAD
  auto sym_of = [&](int a, int x) __attribute__((always_inline)) -> uint32_t {
    const uint32_t c = S.str[x];
    return a && comp && c < 4 ? 3u - c : c;
  };
  const bool gape = o.mode & MODE_GAPE;
  const IndexView ixv0 = A.ix[0];  // L2 only: the same for both strands (checked at launch)
  uint4 *const stg_base = A.stg + ((wave * 64) << A.stg_log2);
  uint4 *const stg = stg_base + ((uint64_t)lane << A.stg_log2);
  const uint32_t SMASK = (1u << A.stg_log2) - 1u;
  const uint32_t STG = 1u << A.stg_log2;
  uint32_t *const dir = A.dir + wave * (uint64_t)NSTK * MAXP;
  uint32_t *const freel = A.freel + wave * (uint64_t)A.freecap;
  uint4 *const hitv = A.hits + wave * (uint64_t)A.hcap;
  uint32_t n_free = 0;  // pages on this wave's free stack (kept across reads)
  // diagnostics (A.prof): wave cycles per phase -- 0 hit barriers, 1 commits, 2 claims,
  // 3 loads + consume, 4 level set-up / teardown, 5 read set-up; 6 iterations, 7 commits, 8 levels
  const bool prof = PROF && A.prof != nullptr;
  // 9..11: lanes running a chain / fetching its entry / in an exact tail, summed over iterations
  // 12..15: idle lanes per iteration waiting on a hit barrier / with the level's chains all claimed /
  // held by the chain ring / short of staging room; 16 chains per level (sum of N); 17 chains
  // discarded at barriers; 18 barriers; 19 children committed
  // 20..24 iterations in levels of N <= 2, <= 16, <= 64, <= 256, > 256 chains; 25..29 running lanes
  // summed over those iterations; 30/31 lane-steps expanding / in an exact tail at a one-row
  // interval; 32..35 chains of < 4, < 16, < 64, >= 64 steps, 36..39 their steps
  __shared__ unsigned long long pc[40];  // LDS: no registers taken from the hot loop
  if (prof) {
    if (lane < 40) pc[lane] = 0;
    __syncthreads();
  }
  auto now = []() __attribute__((always_inline)) -> uint64_t { return __builtin_amdgcn_s_memtime(); };
  uint64_t t_mark = prof ? now() : 0;
  if (prof && A.wave_t && lane == 0) A.wave_t[2 * wave] = t_mark;
  auto lap = [&](int ph) __attribute__((always_inline)) {
    if (prof) {
      const uint64_t t = now();
      if (lane == 0) pc[ph] += t - t_mark;
      t_mark = t;
    }
  };

  // take a page: this wave's free stack, else the global pool (NONE when exhausted)
  auto alloc_page = [&]() __attribute__((always_inline)) -> uint32_t {
    uint32_t p = NONE;
    if (n_free) {
      --n_free;
      p = freel[n_free];
    } else {
      uint32_t q = 0;
      if (lane == 0) q = atomicAdd(A.pool_next, 1u);
      q = __shfl(q, 0);
      p = q < A.pool_pages ? q : NONE;
    }
    return p;
  };
  // give back the pages of bucket b (dirc slot ds holds its directory)
  auto free_pages = [&](uint32_t npg, const uint32_t *d) __attribute__((always_inline)) {
    const uint32_t room = A.freecap - n_free;
    const uint32_t nf = npg < room ? npg : room;  // beyond the stack's room pages are dropped
    for (uint32_t j = lane; j < nf; j += 64) freel[n_free + j] = d[j];
    n_free += nf;
  };

  for (;;) {
    // ------------------------------------------------ claim a read
    int64_t r = 0;
    if (lane == 0) r = (int64_t)atomicAdd(counter, 1ull);
    r = __shfl(r, 0);
    if (r >= A.n) break;
    const int64_t rr = A.ids ? A.ids[r] : r;
    const int64_t ro = A.out_by_id ? rr : r;
    const int len = (int)A.len[rr];
    const uint8_t *sq = A.seq + A.off[rr];
    const int opt_max_diff = o.fnr_pos ? (int)A.maxdiff_tab[len] : o.max_diff;
    uint32_t status = 0;
    int n_aln = 0;
    uint32_t n_iter = 0;
    if (len > COOP_MAXLEN || o.n_stacks > NSTK || (1u << A.stg_log2) < 9u * (uint32_t)(len + 1) + 16u ||
        (len > o.seed_len && o.seed_len > COOP_SEEDMAX)) {
      status = ST_STACK_OVERFLOW | 1u << 8;  // not for this kernel: the sequential kernel takes it
    } else if ((int)A.nN[A.wb_base >= 0 ? rr - A.wb_base : r] > opt_max_diff) {
      // bwtgap.c:116-122: no hit
    } else {
      // ---------------------------------------------- per-read setup
      const bool seeded = len > o.seed_len;
      // a first-pass search state to resume from (GapArgs::rdump), 1 + its offset
      const uint64_t rof = A.roff ? A.roff[rr] : 0ull;
      // level 0 done by k_coop_roots: the records of its two chains (A.proot[2 r], [2 r + 1])
      bool pro = !rof && A.proot && (A.proot[2 * r].w & 0xFFu) == 0u && (A.proot[2 * r + 1].w & 0xFFu) == 0u;
      const uint2 *wb = A.wbuf + (uint64_t)(A.wb_base >= 0 ? rr - A.wb_base : r) * A.wstride;
      for (int j = lane; j < len; j += 64) {
        const uint32_t c = sq[j];
        S.str[j] = (uint8_t)c;
      }
      for (int j = lane; j <= len; j += 64) {
        const uint2 w0 = wb[j], w1 = wb[A.wlen1 + j];
        S.Ww[0][j] = w0.x; S.Wb[0][j] = (uint16_t)w0.y;
        S.Ww[1][j] = w1.x; S.Wb[1][j] = (uint16_t)w1.y;
      }
      if (seeded)
        for (int j = lane; j <= o.seed_len; j += 64) {
          const uint2 w0 = wb[2 * A.wlen1 + j], w1 = wb[2 * A.wlen1 + o.seed_len + 1 + j];
          S.SWw[0][j] = w0.x; S.SWb[0][j] = (uint16_t)w0.y;
          S.SWw[1][j] = w1.x; S.SWb[1][j] = (uint16_t)w1.y;
        }
      for (int b = lane; b < NSTK; b += 64) {
        S.nb[b] = 0;
        S.np[b] = 0;
      }
      S.head[lane] = 0;
      S.rb[lane] = NONE;
      if (lane == 0) S.gq = 0;
      for (int j = lane; j < RREC; j += 64) S.recA[j].w = 0;
      if (pro && lane < 2) {
        // the finished chains 0 and 1 of level 0: staging start = their offset in A.pstore (ring 64)
        const uint4 q = A.proot[2 * r + lane];
        S.recA[lane] = make_uint4(q.x, q.y, (q.z & 0xffffu) | 64u << 16 | ((q.w >> 24) & 7u) << 25,
                                  1u | (q.z >> 16) << 1 | ((q.w >> 8) & 0xFFFFu) << 17);
      }
      __syncthreads();
      // roots (bwtgap.c:126-127): strand 0 then strand 1, both in bucket 0
      if (!rof) {
        const uint32_t p = alloc_page();
        if (p == NONE) {
          status = ST_STACK_OVERFLOW | 3u << 8;
        } else {
          if (lane == 0) {
            dir[0] = p;
            S.np[0] = 1;
            S.nb[0] = 2;
            uint4 *pg = A.pool + ((uint64_t)p << COOP_PG_LOG2);
            pg[0] = mk_ent(0u, ixv0.seq_len, len, 0, 0, 0, 0, 0, STATE_M);
            pg[1] = mk_ent(0u, ixv0.seq_len, len, 0, 0, 0, 0, 1, STATE_M);
          }
          __syncthreads();
        }
      }
      int best_score = (opt_max_diff + 1) * o.s_mm + (o.max_gapo + 1) * o.s_gapo + (o.max_gape + 1) * o.s_gape;
      int max_diff = opt_max_diff, best_cnt = 0;
      // buckets holding gap groups: bit b of S.gm[b >> 5]
      if (lane < 4) S.gm[lane] = 0;
      uint32_t n_live = 2;  // entries on the stack (bwtgap.c n_entries)
      uint32_t stg_w = 0;   // this lane's staging write counter
      int s = 0;            // level (score bucket)
      if (rof) {
        const ResumeOut ro_ = resume_state(A.rdump + (rof - 1), &S, A.pool, dir, hitv, A.hcap, freel, n_free, A.pool_next,
                                           A.pool_pages, ixv0.seq_len, o.s_mm, o.s_gapo, o.s_gape, o.n_stacks, lane,
                                           A.wb_base < 0);
        s = ro_.s;
        n_live = ro_.n_live;
        best_score = ro_.best_score;
        best_cnt = ro_.best_cnt;
        max_diff = ro_.max_diff;
        n_aln = ro_.n_aln;
        status = ro_.status;
        n_free = ro_.n_free;
      }
      bool done = status != 0;
      lap(5);
      // ---------------------------------------------- levels
      while (!done) {
        while (s < o.n_stacks && S.nb[s] == 0) ++s;
        if (s >= o.n_stacks) break;                                              // stack empty
        if (n_live > (uint32_t)o.max_entries) break;                            // :138, before the level's first pop
        if (!(o.mode & MODE_NONSTOP) && s > best_score + o.s_mm) break;         // :143
        uint32_t N = S.nb[s];
        // targets: mismatch, gap extension, gap open (deduplicated when penalties coincide)
        const int t0 = s + o.s_mm;
        const int t1 = s + o.s_gape;
        const int t2 = s + o.s_gapo;
        const int q1 = t1 == t0 ? 0 : 1;
        const int q2 = t2 == t0 ? 0 : (t2 == t1 ? q1 : 2);
        auto tg = [&](int q) __attribute__((always_inline)) { return q == 0 ? t0 : q == 1 ? t1 : t2; };
        // directories into LDS
        for (uint32_t j = lane; j < S.np[s]; j += 64) S.dirc[0][j] = dir[s * MAXP + j];
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (tg(q) < o.n_stacks)
            for (uint32_t j = lane; j < S.np[tg(q)]; j += 64) S.dirc[1 + q][j] = dir[tg(q) * MAXP + j];
        __syncthreads();
        {
          if ((S.gm[(uint32_t)s >> 5] >> (s & 31)) & 1u) {
            // the level holds gap groups: spell them out first
            const uint2 g = expand_groups(A.pool, A.o64[0], A.o64[1],
                                          make_uint4(ixv0.L2[0], ixv0.L2[1], ixv0.L2[2], ixv0.L2[3]), dir + s * MAXP,
                                          S.dirc[0], freel, n_free, A.freecap, A.pool_next, A.pool_pages, N, S.np[s], lane);
            n_free = g.y;
            if (g.x >= GRP_FAIL) {
              status = ST_STACK_OVERFLOW | (g.x & 15u) << 8;
              done = true;
              break;
            }
            if (lane == 0) {
              S.np[s] = (uint16_t)((g.x + COOP_PG - 1) >> COOP_PG_LOG2);
              S.nb[s] = g.x;
            }
            N = g.x;
            __syncthreads();
          }
        }
        const int nbk = N <= 2 ? 0 : N <= 16 ? 1 : N <= 64 ? 2 : N <= 256 ? 3 : 4;
        if (prof && lane == 0) {
          ++pc[8];
          pc[16] += N;
        }
        lap(4);
        uint32_t next_c = 0, cp = 0, barrier = NONE;
        // lane chain state
        int lst = L_IDLE;
        uint32_t c = 0, cstart = 0, cnt0 = 0, cnt1 = 0, cnt2 = 0;
        uint32_t mpre = 0;  // stack growth (children staged, a group counting all) before the chain's latest pop
        uint32_t k = 0, l = 0;
        int i = 0, ldp = 0;  // an exact tail steps k, l, i down to the hit
        // the node's entry word, fields unpacked where used (registers are the loop's limit):
        // n_mm | n_gapo << 8 | n_gape << 16 | a << 24 | state << 25
        uint32_t ew = 0;
        uint32_t ent_page = 0, ent_off = 0;
        // Entry window: lane x holds the entry of chain wh (wh = x mod 64), loaded with an earlier
        // iteration's round trip, so a chain claimed inside the window starts expanding in the
        // iteration that claims it instead of spending one on fetching its entry.
        uint32_t wh = (uint32_t)lane;
        uint4 wen = make_uint4(0, 0, 0, 0);
        bool wld = false, wreq = wh < N;
        if (pro) {
          // level 0 ran in the prologue: its two chains are finished (records in place) and commit below
          pro = false;
          next_c = 2;
          wreq = false;
        }
        uint32_t hit_c = NONE;  // chain this lane ended with a hit in the last iteration
        uint32_t csteps = 0;    // (prof) steps of the lane's chain
        // end the lane's chain: its record (hit or not) goes to the reorder buffer
        auto end_chain = [&](bool hit, uint32_t hk, uint32_t hl) __attribute__((always_inline)) {
          const uint32_t slot = c & (RREC - 1);
          if (prof) {
            const int b = csteps < 4 ? 0 : csteps < 16 ? 1 : csteps < 64 ? 2 : 3;
            atomicAdd(&pc[32 + b], 1ull);
            atomicAdd(&pc[36 + b], (unsigned long long)csteps);
            csteps = 0;
          }
          if (hit) {  // the hit record {k, l, n_mm | n_gapo << 8 | n_gape << 16 | a << 24, ldp}: global,
                      // agent-scope (L2) accesses, read once by the whole wave at the barrier
            uint32_t *hr = reinterpret_cast<uint32_t *>(A.recb + wave * RREC + slot);
            __hip_atomic_store(hr + 0, hk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(hr + 1, hl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(hr + 2, ew & 0x1FFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(hr + 3, (uint32_t)ldp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          S.recA[slot] = make_uint4(cstart, cnt0 | cnt1 << 16,
                                    (cnt2 & 0xFFFFu) | (uint32_t)lane << 16 | (hit ? 1u << 24 : 0u) | (cnt2 >> 28) << 25,
                                    1u | mpre << 1 | ((cnt2 >> 16) & 0xFFFu) << 17);
          if (hit) hit_c = c;
          lst = L_IDLE;
        };
        auto take_entry = [&](const uint4 &ent) __attribute__((always_inline)) {
          k = ent.x;
          l = ent.y;
          i = (int)(ent.z & 0x3ff);
          ldp = (int)((ent.z >> 10) & 0x3ff);
          ew = ent.w & 0x7FFFFFFu;
        };
        // the pops of bwtgap.c:139-163 for the node in registers: prune, hit, tail or expand
        auto pop_node = [&]() __attribute__((always_inline)) {
          mpre = cnt0 + cnt1 + (cnt2 & 0xFFFFu) + ((cnt2 >> 16) & 0xFFFu);
          const int e_mm = (int)(ew & 0xffu), e_go = (int)((ew >> 8) & 0xffu), e_ge = (int)((ew >> 16) & 0xffu);
          const int a = (int)((ew >> 24) & 1u), state = (int)((ew >> 25) & 3u);
          int m = max_diff - (e_mm + e_go);
          if (gape) m -= e_ge;
          // one end_chain call site: with several, the calls were merged across the lambdas before
          // inlining and the chain state went to scratch
          int end = 0;  // 1 no hit, 2 hit
          if (m < 0) end = 1;                                                                // :147
          else if (i > 0 && m < (int)S.Wb[a][i - 1]) end = 1;                                // :155
          else if (i == 0) end = 2;                                                          // :159
          else if (m == 0 && (state == STATE_M || gape || e_ge == o.max_gape)) {             // :160
            --i;  // the tail's next symbol
            if (sym_of(a, i) > 3) end = 1;
            else lst = L_TAIL;
          } else {
            lst = L_EXP;
          }
          if (end) end_chain(end == 2, k, l);
        };

        for (;;) {
          if (++n_iter > A.max_iters) {  // runaway guard: hand the read to the sequential kernel
            status = ST_STACK_OVERFLOW | 5u << 8;
            done = true;
            break;
          }
          // ============================================ uniform control
          // (a) hits of chains that ended last iteration: the earliest becomes the barrier, and
          //     every chain after it (running or finished) is discarded
          {
            uint32_t newb = NONE;
            if (__ballot(hit_c != NONE)) newb = wave_min(hit_c);
            hit_c = NONE;
            if (newb < barrier) {
              if (prof) {
                const unsigned long long dr = __ballot(lst != L_IDLE && c > newb);
                if (lane == 0) {
                  pc[17] += __popcll(dr);
                  ++pc[18];
                }
              }
              if (lst != L_IDLE && c > newb) {
                S.rb[lane] = S.rb[lane] < cstart ? S.rb[lane] : cstart;
                lst = L_IDLE;
              }
              __syncthreads();
              for (uint32_t base = newb + 1; base < next_c; base += 64) {
                const uint32_t cc = base + lane;
                if (cc < next_c) {
                  const uint32_t slot = cc & (RREC - 1);
                  const uint4 ra = S.recA[slot];
                  if (ra.w) {
                    const uint32_t rl = (ra.z >> 16) & 127;
                    if (rl < 64) atomicMin(&S.rb[rl], ra.x);  // (a prologue chain is never rolled back)
                    S.recA[slot].w = 0;
                  }
                }
              }
              __syncthreads();
              if (S.rb[lane] != NONE) {
                stg_w = S.rb[lane];
                S.rb[lane] = NONE;
              }
              barrier = newb;
              next_c = newb + 1;
              // the window restarts at the rolled-back claim point
              const uint32_t nh = next_c + (((uint32_t)lane - next_c) & 63u);
              if (nh != wh) {
                wh = nh;
                wld = false;
                wreq = wh < N;
              }
            }
          }
          lap(0);
          if (prof && lane == 0) {
            ++pc[6];
            ++pc[20 + nbk];
          }
          // finished chains from cp on, in pop order
          uint32_t ndone = 0;
          for (uint32_t base = cp; base < next_c; base += 64) {
            const uint32_t cc = base + lane;
            const bool dn = cc < next_c && S.recA[cc & (RREC - 1)].w != 0u;
            const unsigned long long dm = __ballot(dn);
            const uint32_t run = dm == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~dm);
            ndone += run;
            if (run < 64) break;
          }
          // (b) commit the finished prefix (in pop order): at least 32 chains, or all there is
          const unsigned long long active = __ballot(lst != L_IDLE);
          uint32_t lim = ndone;
          if (barrier != NONE && lim > barrier + 1 - cp) lim = barrier + 1 - cp;
          const bool at_barrier = barrier != NONE && cp + lim == barrier + 1;
          if (lim && (lim >= 32 || active == 0ull || at_barrier)) {
            if (prof && lane == 0) ++pc[7];
            __threadfence_block();  // staging stores of earlier iterations are visible
            for (uint32_t base = 0; base < lim && !done; base += 64) {
              const uint32_t cc = cp + base + lane;
              const bool v = base + lane < lim;
              const uint4 ra = v ? S.recA[cc & (RREC - 1)] : make_uint4(0, 0, 0, 0);
              const uint32_t n0 = ra.y & 0xffffu, n1 = ra.y >> 16, n2 = ra.z & 0xffffu;
              const uint32_t tot = n0 + n1 + n2;  // entries staged (a gap group is one)
              // stack size before this chain's first pop; its largest before any of its pops is
              // nc + (its stack growth before its last pop) (bwtgap.c:138); a gap group counts all
              // its entries
              uint32_t dsum = 0, vsum = 0;
              const uint32_t pre = wave_excl(v ? tot : 0u, lane, dsum);
              const uint32_t vpre = wave_excl(v ? tot + (ra.w >> 17) : 0u, lane, vsum);
              const uint32_t nc = n_live + vpre - (uint32_t)lane;  // each earlier chain popped one entry
              if (__ballot(v && nc + ((ra.w >> 1) & 0xFFFFu) > (uint32_t)o.max_entries)) {
                done = true;  // the search breaks inside the first such chain: the hits so far stand
                break;
              }
              const uint32_t nv = (lim - base) < 64 ? (lim - base) : 64;
              n_live = n_live + vsum - nv;
              // target categories that now hold gap groups (buckets marked at the level's end)
              if (v && ((ra.z >> 25) & 7u)) atomicOr(&S.gq, (ra.z >> 25) & 7u);
              if (prof && lane == 0) pc[19] += dsum;
              uint32_t T0 = 0, T1 = 0, T2 = 0;
              const uint32_t o0 = wave_excl(n0, lane, T0);
              const uint32_t o1 = wave_excl(n1, lane, T1);
              const uint32_t o2 = wave_excl(n2, lane, T2);
              auto Tq = [&](int q) __attribute__((always_inline)) { return q == 0 ? T0 : q == 1 ? T1 : T2; };
              // pages for the targets
              bool bad = false;
              uint32_t why = 0;
              for (int q = 0; q < 3; ++q) {
                if (!Tq(q)) continue;
                const int tb = tg(q);
                if (tb >= o.n_stacks) { bad = true; continue; }
                const uint32_t need = (S.nb[tb] + Tq(q) + COOP_PG - 1) >> COOP_PG_LOG2;
                if (need > MAXP) { bad = true; why = 4; continue; }
                for (uint32_t pq = S.np[tb]; pq < need; ++pq) {
                  const uint32_t p = alloc_page();
                  if (p == NONE) { bad = true; why = 3; break; }
                  if (lane == 0) {
                    S.dirc[1 + q][pq] = p;
                    dir[tb * MAXP + pq] = p;
                  }
                  S.np[tb] = pq + 1;  // same value from every lane
                }
              }
              if (bad) {
                // a score past the last bucket is an option error; the rest is storage
                status = (T0 && t0 >= o.n_stacks) || (T1 && t1 >= o.n_stacks) || (T2 && t2 >= o.n_stacks)
                             ? ST_BAD_SCORE : ST_STACK_OVERFLOW | why << 8;
                done = true;
                break;
              }
              __syncthreads();
              // copy: the batch's children, flattened, 64 per round trip and two round trips'
              // loads in flight (four spill registers); child g belongs to chain j with pre_j <= g < pre_j + tot_j
              // (binary search over the lanes' prefixes) and goes to its category's bucket at
              // (bucket size) + (chain's offset in the batch) + (its rank in the chain)
              {
                const uint32_t my_rl = (ra.z >> 16) & 127, my_st = ra.x;
                const uint32_t nb0 = S.nb[t0], nb1 = t1 < o.n_stacks ? S.nb[t1] : 0u,
                               nb2 = t2 < o.n_stacks ? S.nb[t2] : 0u;
                for (uint32_t g0 = 0; g0 < dsum; g0 += 64u * 2) {
                  uint4 e[2];
                  uint32_t f0[2], f1[2], f2[2];
#pragma unroll
                  for (int u = 0; u < 2; ++u) {
                    const uint32_t g = g0 + 64u * u + (uint32_t)lane;
                    int j = 0;
#pragma unroll
                    for (int step = 32; step >= 1; step >>= 1) {
                      const uint32_t pm = __shfl(pre, j + step);
                      if (pm <= g) j += step;
                    }
                    const uint32_t x = g - __shfl(pre, j);
                    const uint32_t rl = __shfl(my_rl, j), st0 = __shfl(my_st, j);
                    f0[u] = nb0 + __shfl(o0, j);
                    f1[u] = nb1 + __shfl(o1, j);
                    f2[u] = nb2 + __shfl(o2, j);
                    e[u] = make_uint4(0, 0, 0, 0);
                    if (g < dsum)
                      e[u] = rl < 64 ? stg_base[((uint64_t)rl << A.stg_log2) + ((st0 + x) & SMASK)] : A.pstore[st0 + x];
                  }
#pragma unroll
                  for (int u = 0; u < 2; ++u) {
                    if (g0 + 64u * u + (uint32_t)lane < dsum) {
                      const uint32_t q = (e[u].w >> 27) & 3u, rk = e[u].z >> 20;
                      const uint32_t pos = (q == 0 ? f0[u] : q == 1 ? f1[u] : f2[u]) + rk;
                      const uint32_t pg = S.dirc[1 + q][pos >> COOP_PG_LOG2];
                      A.pool[((uint64_t)pg << COOP_PG_LOG2) + (pos & (COOP_PG - 1))] = e[u];
                    }
                  }
                }
                if (v && tot && my_rl < 64) atomicMax(&S.head[my_rl], my_st + tot);
              }
              if (v) S.recA[cc & (RREC - 1)].w = 0;
              __syncthreads();
              if (lane == 0) {
                S.nb[t0] += T0;
                if (q1 == 1) S.nb[t1] += T1;
                if (q2 == 2) S.nb[t2] += T2;
              }
              __syncthreads();
            }
            if (done) break;
            cp += lim;
            if (at_barrier) {
              // ---- the hit of chain `barrier` (bwtgap.c:165-197)
              uint4 hb;
              {
                __threadfence_block();
                uint32_t *hr = reinterpret_cast<uint32_t *>(A.recb + wave * RREC + (barrier & (RREC - 1)));
                hb.x = __hip_atomic_load(hr + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                hb.y = __hip_atomic_load(hr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                hb.z = __hip_atomic_load(hr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                hb.w = __hip_atomic_load(hr + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              const uint32_t hk = hb.x, hl = hb.y;
              const int h_mm = (int)(hb.z & 0xff), h_go = (int)((hb.z >> 8) & 0xff), h_ge = (int)((hb.z >> 16) & 0xff);
              const int h_a = (int)((hb.z >> 24) & 1), h_ldp = (int)hb.w;
              const int score = h_mm * o.s_mm + h_go * o.s_gapo + h_ge * o.s_gape;
              barrier = NONE;
              if (n_aln == 0) {
                best_score = score;
                int best_diff = h_mm + h_go;
                if (gape) best_diff += h_ge;
                if (!(o.mode & MODE_NONSTOP)) max_diff = (best_diff + 1 > opt_max_diff) ? opt_max_diff : best_diff + 1;
              }
              if (score == best_score) {
                best_cnt = (int)((uint32_t)best_cnt + (hl - hk + 1));
              } else if (best_cnt > o.max_top2) {
                done = true;  // :185
                break;
              }
              bool add = true;
              if (h_go) {
                bool dup = false;
                for (int j = lane; j < n_aln; j += 64) {
                  const uint4 h = hitv[j];
                  dup |= h.y == hk && h.z == hl;
                }
                add = __ballot(dup) == 0ull;
              }
              if (add) {
                // gap_shadow (bwtgap.c:81-91) on strand h_a's widths, 64 positions at a time
                const uint32_t x = hl - hk + 1, mx = ixv0.seq_len;
                uint32_t jrun = 0;
                for (int base = 0; base < h_ldp; base += 64) {
                  const int q = base + lane;
                  uint2 w = q < h_ldp ? make_uint2(S.Ww[h_a][q], S.Wb[h_a][q]) : make_uint2(0, 0);
                  const bool eq = q < h_ldp && w.x == x;
                  const unsigned long long em = __ballot(eq);
                  if (q < h_ldp) {
                    if (w.x > x) {
                      w.x -= x;
                      S.Ww[h_a][q] = w.x;
                    } else if (eq) {
                      const uint32_t jj = jrun + (uint32_t)__popcll(em & ((1ull << lane) - 1ull)) + 1u;
                      S.Ww[h_a][q] = mx - jj;
                      S.Wb[h_a][q] = 1u;
                    }
                  }
                  jrun += (uint32_t)__popcll(em);
                }
                if ((uint32_t)n_aln >= A.hcap) {
                  status = ST_ALN_OVERFLOW;
                  done = true;
                  break;
                }
                if (lane == 0)
                  hitv[n_aln] = make_uint4((uint32_t)h_mm | (uint32_t)h_go << 8 | (uint32_t)h_ge << 16 |
                                               (uint32_t)h_a << 24, hk, hl, (uint32_t)score);
                ++n_aln;
                __threadfence_block();
                __syncthreads();
              }
            }
          }
          lap(1);
          // (c) level finished
          if (cp == N && __ballot(lst != L_IDLE) == 0ull) break;
          // (d) claims: idle lanes take the next chains in pop order
          {
            const uint32_t ch_max = 9u * (uint32_t)(len + 1) + 16u;
            const bool want = lst == L_IDLE && barrier == NONE && STG - (stg_w - S.head[lane]) >= ch_max;
            const unsigned long long wm = __ballot(want);
            const uint32_t cap_c = cp + RREC < N ? cp + RREC : N;
            const uint32_t avail = cap_c > next_c ? cap_c - next_c : 0u;
            const uint32_t rank = (uint32_t)__popcll(wm & ((1ull << lane) - 1ull));
            if (prof) {
              const bool idle = lst == L_IDLE;
              const unsigned long long i_b = __ballot(idle && barrier != NONE),
                                       i_n = __ballot(idle && barrier == NONE && next_c >= N),
                                       i_r = __ballot(idle && barrier == NONE && next_c < N && next_c >= cap_c),
                                       i_s = __ballot(idle && barrier == NONE && !want);
              if (lane == 0) {
                pc[12] += __popcll(i_b);
                pc[13] += __popcll(i_n);
                pc[14] += __popcll(i_r);
                pc[15] += __popcll(i_s);
              }
            }
            if (wm) {
              // every lane takes part in the shuffles; the claim reads its chain's window slot
              const uint32_t cc = next_c + rank, src = cc & 63u;
              const uint32_t tag = __shfl(wld ? wh : NONE, (int)src);
              const uint4 ce = make_uint4(__shfl(wen.x, (int)src), __shfl(wen.y, (int)src), __shfl(wen.z, (int)src),
                                          __shfl(wen.w, (int)src));
              if (want && rank < avail) {
                c = cc;
                cstart = stg_w;
                csteps = 0;
                cnt0 = cnt1 = cnt2 = 0;
                if (tag == cc) {
                  take_entry(ce);
                  pop_node();
                } else {
                  const uint32_t idx = N - 1u - c;  // LIFO: chain 0 is the top of the bucket
                  ent_page = S.dirc[0][idx >> COOP_PG_LOG2];
                  ent_off = idx & (COOP_PG - 1);
                  lst = L_FETCH;
                }
              }
              const uint32_t nw = (uint32_t)__popcll(wm);
              next_c += nw < avail ? nw : avail;
              // window slots whose chain is now claimed move on to the chain 64 further
              while (wh < next_c) {
                wh += 64;
                wld = false;
                wreq = wh < N;
              }
            }
          }
          lap(2);
          // ============================================ loads of this iteration (one round trip)
          // L2 (symbol counts) is the same for bwt and rbwt -- one text, reversed (checked at launch):
          // the uniform copy keeps it out of the loop's vector registers
          const IndexView &ix = ixv0;
          const int a = (int)((ew >> 24) & 1u);
          const uint4 *ob = a ? A.o64[0] : A.o64[1];
          if (wreq) {
            const uint32_t widx = N - 1u - wh;
            wen = A.pool[((uint64_t)S.dirc[0][widx >> COOP_PG_LOG2] << COOP_PG_LOG2) + (widx & (COOP_PG - 1))];
            wld = true;
            wreq = false;
          }
          const bool exp = lst == L_EXP;
          const bool tail = lst == L_TAIL;
          if (prof) {
            const unsigned long long b_act = __ballot(lst != L_IDLE), b_f = __ballot(lst == L_FETCH),
                                     b_t = __ballot(tail);
            if (lane == 0) {
              pc[9] += __popcll(b_act);
              pc[10] += __popcll(b_f);
              pc[11] += __popcll(b_t);
              pc[25 + nbk] += __popcll(b_act);
            }
            const unsigned long long b_e1 = __ballot(exp && k == l), b_t1 = __ballot(tail && k == l);
            if (lane == 0) {
              pc[30] += __popcll(b_e1);
              pc[31] += __popcll(b_t1);
            }
            if (lst != L_IDLE) ++csteps;
          }
          const uint32_t qk = k, ql = l;
          const bool qkneg = qk == 0;
          const bool qshare = !qkneg && ((qk - 1) >> 6) == (ql >> 6);
          const uint32_t tsym = tail ? sym_of(a, i) : 0u;
          // One set of load registers: a lane fetches its chain's entry (bl.v0), takes an exact-tail
          // step (the tail symbol's Occ words of both rows: bl.v0, bk.v0) or expands (both whole
          // blocks) -- never two of these, so the round trip holds 8 uint4s, not 14
          Blk bk, bl;
          {
            const bool fetch = lst == L_FETCH;
            const bool kld = (exp || tail) && !qkneg && !qshare;
            const uint4 *pl = fetch ? A.pool + (((uint64_t)ent_page << COOP_PG_LOG2) + ent_off)
                                    : ob + ((size_t)(ql >> 6) * 4 + tsym);
            const uint4 *pk = ob + ((size_t)((qk - 1) >> 6) * 4 + tsym);
            if (fetch || exp || tail) bl.v0 = pl[0];
            if (exp) {
              bl.v1 = pl[1];
              bl.v2 = pl[2];
              bl.v3 = pl[3];
            }
            if (kld) bk.v0 = pk[0];
            if (exp && kld) {
              bk.v1 = pk[1];
              bk.v2 = pk[2];
              bk.v3 = pk[3];
            }
          }

          // ============================================ consume
          if (lst == L_FETCH) {
            take_entry(bl.v0);
            pop_node();
          } else if (tail) {
            // one step of bwt_match_exact_alt (bwt.c:240-247)
            const uint4 tvl = bl.v0;
            uint4 tvk = bk.v0;
            if (qshare) tvk = tvl;
            const uint32_t ok = qkneg ? 0u : occ_of(tvk, qk - 1), ol = occ_of(tvl, ql);
            const uint32_t base = l2of(ix, tsym);
            k = base + ok + 1;
            l = base + ol;
            if (k > l) {
              end_chain(false, 0, 0);
            } else if (--i < 0) {
              end_chain(true, k, l);
            } else if (sym_of(a, i) > 3) {
              end_chain(false, 0, 0);
            }
          } else if (exp) {
            // ---- expansion (bwtgap.c:200-258); the match child continues the chain.  The same steps as
            // expand_node (k_coop_roots), kept inline: through the function this loop's registers
            // spilled (16 -> 39 scratch accesses) and k_coop ran 10 % slower (same-box A/B)
            if (qshare) bk = bl;
            const int e_mm = (int)(ew & 0xffu), e_go = (int)((ew >> 8) & 0xffu), e_ge = (int)((ew >> 16) & 0xffu);
            const int state = (int)((ew >> 25) & 3u);
            uint4 KK, LL;
            {
              const uint4 cl4 = make_uint4(occ_of(bl.v0, ql), occ_of(bl.v1, ql), occ_of(bl.v2, ql), occ_of(bl.v3, ql));
              const uint4 ck4 = qkneg ? make_uint4(0, 0, 0, 0)
                                      : make_uint4(occ_of(bk.v0, qk - 1), occ_of(bk.v1, qk - 1), occ_of(bk.v2, qk - 1),
                                                   occ_of(bk.v3, qk - 1));
              KK = make_uint4(ix.L2[0] + ck4.x + 1, ix.L2[1] + ck4.y + 1, ix.L2[2] + ck4.z + 1, ix.L2[3] + ck4.w + 1);
              LL = make_uint4(ix.L2[0] + cl4.x, ix.L2[1] + cl4.y, ix.L2[2] + cl4.z, ix.L2[3] + cl4.w);
            }
            int m = max_diff - (e_mm + e_go);
            if (gape) m -= e_ge;
            int m_seed = 0;
            if (seeded) {
              m_seed = o.max_seed_diff - (e_mm + e_go);
              if (gape) m_seed -= e_ge;
            }
            const int ni = i - 1;
            const uint32_t csym = sym_of(a, ni);
            const uint32_t occ = l - k + 1;
            bool allow_diff = true, allow_M = true;
            if (ni > 0) {
              const uint2 w_im2 = make_uint2(S.Ww[a][ni - 1], S.Wb[a][ni - 1]),
                          w_im1 = make_uint2(S.Ww[a][ni], S.Wb[a][ni]);
              if ((int)w_im2.y > m - 1) allow_diff = false;
              else if ((int)w_im2.y == m - 1 && (int)w_im1.y == m - 1 && w_im2.x == w_im1.x) allow_M = false;
              const int ii = ni - (len - o.seed_len);
              if (seeded && ii > 0) {
                const uint2 sw_lo = make_uint2(S.SWw[a][ii - 1], S.SWb[a][ii - 1]),
                            sw_hi = make_uint2(S.SWw[a][ii], S.SWb[a][ii]);
                if ((int)sw_lo.y > m_seed - 1) allow_diff = false;
                else if ((int)sw_lo.y == m_seed - 1 && (int)sw_hi.y == m_seed - 1 && sw_lo.x == sw_hi.x) allow_M = false;
              }
            }
            const uint32_t ne4 = (KK.x <= LL.x ? 1u : 0u) | (KK.y <= LL.y ? 2u : 0u) | (KK.z <= LL.z ? 4u : 0u) |
                                 (KK.w <= LL.w ? 8u : 0u);
            const int tmp = (o.mode & MODE_LOGGAP) ? int_log2((uint32_t)(e_ge + e_go)) / 2 + 1 : e_go + e_ge;
            uint32_t vm = 0;
            if (allow_diff && ni >= o.indel_end_skip + tmp && len - ni >= o.indel_end_skip + tmp) {
              if (state == STATE_M) {
                if (e_go < o.max_gapo) vm = 1u | ne4 << 1;
              } else if (state == STATE_I) {
                if (e_ge < o.max_gape) vm = 1u;
              } else if (state == STATE_D) {
                if (e_ge < o.max_gape && (e_ge + e_go < max_diff || occ < (uint32_t)o.max_del_occ)) vm = ne4 << 1;
              }
            }
            const uint32_t rot = (csym + 1) & 3;
            const uint32_t ner = ((ne4 >> rot) | (ne4 << (4 - rot))) & 15u;
            if (allow_diff && allow_M) vm |= ner << 5;
            else if (csym < 4) vm |= ner & 8u ? 1u << 8 : 0u;
            // bit 8 with csym < 4 is the match child: it continues the chain instead of being staged
            const bool match = (vm >> 8) & 1u && csym < 4;
            if (match) vm &= ~(1u << 8);
            const int sc_base = e_mm * o.s_mm + e_go * o.s_gapo + e_ge * o.s_gape;
            const int sc_gap = state == STATE_M ? o.s_gapo : o.s_gape;
            // a gap-opening expansion's deletions ride on its insertion child (gap group)
            const uint32_t gdm = state == STATE_M && (vm & 1u) ? (vm >> 1) & 15u : 0u;
            vm &= ~(gdm << 1);
            while (vm) {
              const uint32_t j = (uint32_t)__builtin_ctz(vm);
              vm &= vm - 1;
              const bool is_ins = j == 0, is_del = j - 1 < 4, is_sym = j >= 5;
              const uint32_t cc = is_del ? j - 1 : (csym + j - 4) & 3;
              const uint32_t pk = is_ins ? k : pick4(KK, cc);
              const uint32_t pl = is_ins ? l : pick4(LL, cc);
              const bool open = !is_sym && state == STATE_M;
              const int n_mm = e_mm + (is_sym ? 1 : 0);  // staged symbol children are mismatches
              const int n_gapo = e_go + (open ? 1 : 0), n_gape = e_ge + (!is_sym && !open ? 1 : 0);
              const int pi = is_del ? ni + 1 : ni;
              const int pstate = is_ins ? STATE_I : is_del ? STATE_D : STATE_M;
              const int sc = sc_base + (is_sym ? o.s_mm : sc_gap);
              const int q = sc == t0 ? 0 : sc == t1 ? q1 : q2;
              const uint32_t rk = q == 0 ? cnt0++ : q == 1 ? cnt1++ : (cnt2++ & 0xFFFFu);
              const bool grp = is_ins && gdm;
              stg[(stg_w++) & SMASK] = mk_ent(pk, pl, pi, grp ? (int)gdm : pi, n_mm, n_gapo, n_gape, a,
                                              grp ? STATE_G : pstate, (uint32_t)q, rk);
              if (grp) cnt2 = (cnt2 + ((uint32_t)__builtin_popcount(gdm) << 16)) | 1u << (28 + q);
            }
            if (match) {
              k = pick4(KK, csym);
              l = pick4(LL, csym);
              i = ni;
              ew = (ew & ~(3u << 25)) | (uint32_t)STATE_M << 25;
              pop_node();
            } else {
              end_chain(false, 0, 0);
            }
          }
          lap(3);
        }
        if (done) break;
        // level s is consumed: its pages go back
        free_pages(S.np[s], S.dirc[0]);
        __syncthreads();
        if (lane == 0) {
          S.nb[s] = 0;
          S.np[s] = 0;
          for (int q = 0; q < 3; ++q)
            if ((S.gq >> q) & 1u) {
              const int b = q == 0 ? t0 : q == 1 ? t1 : t2;
              if (b < o.n_stacks) S.gm[(uint32_t)b >> 5] |= 1u << (b & 31);
            }
          S.gq = 0;
        }
        __syncthreads();
        ++s;
      }
      // every bucket's pages go back (termination leaves entries behind)
      for (int b = 0; b < o.n_stacks; ++b) {
        const uint32_t npg = S.np[b];
        if (npg) {
          const uint32_t room = A.freecap - n_free;
          const uint32_t nf = npg < room ? npg : room;
          for (uint32_t j = lane; j < nf; j += 64) freel[n_free + j] = dir[b * MAXP + j];
          n_free += nf;
        }
      }
      __syncthreads();
    }
    lap(4);
    // ------------------------------------------------ hits of the read to the stream
    int na = status ? 0 : n_aln;
    if (na) {
      unsigned long long pos = 0;
      if (lane == 0) pos = atomicAdd(A.aln_next, (unsigned long long)na);
      pos = __shfl(pos, 0);
      if (pos + (unsigned long long)na > A.aln_total) {
        status |= ST_ALN_OVERFLOW;
        na = 0;
      } else {
        __threadfence_block();
        for (int j = lane; j < na; j += 64) A.aln[pos + j] = hitv[j];
        if (lane == 0) A.aln_off[ro] = pos;
      }
    }
    if (lane == 0) {
      A.n_aln[ro] = na;
      A.status[r] = status;  // per launch read: the host collects the reads to re-run from it
      if (A.fix_status) {
        if (status == 0u) A.fix_status[rr] = 0u;
        else A.fix_roff[rr] = 0u;
      }
      if (A.iters) A.iters[r] = n_iter;
    }
    __syncthreads();
    lap(5);
  }
  if (prof && lane == 0)
    for (int q = 0; q < 40; ++q) atomicAdd(A.prof + q, (unsigned long long)pc[q]);
  if (prof && A.wave_t && lane == 0) A.wave_t[2 * wave + 1] = now();
}

// k_coop_roots -- level 0 of the heavy reads, before k_coop takes them.  Level 0 is the two root
// chains (strand 1 popped first, bwtgap.c:126-127): each walks the read from its end while the
// match child exists, staging the mismatch and gap children of every expansion.  They take about a
// tenth of k_coop's iterations with two lanes of 64 running, so here each lane runs one root chain
// on its own (chain u = 2 r + x of launch read r: x = 0 strand 1, x = 1 strand 0), from the read's
// initial state, widths and symbols from global memory.  The two chains are independent unless
// chain 0 ends in a hit (chain 1 would have to see it): then, or when the read is not for k_coop,
// the record says so and k_coop runs level 0 itself.  A chain's children are staged in the lane's
// ring (k_coop's staging rings, unused until it starts), then copied to the compact store pstore
// at an offset reserved when the chain ends; proot[u] = {offset, cnt0 | cnt1 << 16,
// cnt2 | stack growth before its last pop << 16, flag | deletions pending in its gap groups << 8 |
// categories holding a gap group << 24}.
__global__ void __launch_bounds__(64) k_coop_roots(CoopArgs A, unsigned long long *counter) {
  const int lane = threadIdx.x;
  const AlnOpt o = A.o;
  const bool comp = o.mode & MODE_COMPREAD;
  const IndexView ixv0 = A.ix[0], ixv1 = A.ix[1];
  const uint32_t SMASK = (1u << A.stg_log2) - 1u;
  uint4 *const ring = A.stg + (((uint64_t)blockIdx.x * 64 + lane) << A.stg_log2);
  const int t0 = o.s_mm, t1 = o.s_gape, t2 = o.s_gapo;  // the targets of level 0's children
  const int q1 = t1 == t0 ? 0 : 1;
  const int q2 = t2 == t0 ? 0 : (t2 == t1 ? q1 : 2);
  constexpr int L_COPY = 4, L_END = 5;
  int pst = L_IDLE;
  uint64_t u = 0;
  uint32_t pflag = 0, c0 = 0, c1 = 0, c2 = 0, pmpre = 0, pw = 0, ci = 0, pex = 0, pgq = 0;
  uint64_t off = 0;
  Node nd = {};
  int pa = 0, plen = 0, pmd = 0;
  bool pseed = false;
  const uint8_t *psq = nullptr;
  const uint2 *pwb = nullptr, *pswb = nullptr;
  uint32_t xk = 0, xl = 0, tcur = 0, snext = 0;
  int xj = 0;
  uint2 wim1 = make_uint2(0, 0);  // width[i-1] of the node about to be popped
  auto psym = [&](int x) __attribute__((always_inline)) -> uint32_t {
    const uint32_t c = psq[x];
    return pa && comp && c < 4 ? 3u - c : c;
  };
  auto record = [&]() __attribute__((always_inline)) {
    A.proot[u] = make_uint4((uint32_t)off, c0 | c1 << 16, c2 | pmpre << 16, pflag | pex << 8 | pgq << 24);
    pst = L_IDLE;
  };
  // the chain has ended without a hit: reserve its children's room in the store
  auto finish = [&]() __attribute__((always_inline)) {
    const uint32_t tot = c0 + c1 + c2;
    off = 0;
    if (tot) {
      off = atomicAdd(A.pstore_next, (unsigned long long)tot);
      if (off + tot > A.pstore_cap) pflag = PRO_SKIP;  // (cap < 2^32: offsets fit the record)
    }
    ci = 0;
    if (tot && pflag == 0) pst = L_COPY;
    else record();
  };
  // a pop of the chain (level 0: no differences, state M, m = max_diff; bwtgap.c:139-163)
  auto ppop = [&]() __attribute__((always_inline)) {
    pmpre = c0 + c1 + c2 + pex;  // the stack grew by the entries staged so far (a group counts all)
    if (nd.i > 0 && pmd < (int)wim1.y) { finish(); return; }  // :155
    if (nd.i == 0) { pflag = PRO_HIT; record(); return; }     // :159
    if (pmd == 0) {                                            // :160
      xj = nd.i - 1;
      xk = nd.k;
      xl = nd.l;
      tcur = snext;
      if (snext > 3) finish();
      else pst = L_TAIL;
      return;
    }
    pst = L_EXP;
  };
  for (;;) {
    // ---- idle lanes take the next chains (one atomic per wave)
    {
      const bool want = pst == L_IDLE;
      const unsigned long long wm = __ballot(want);
      if (wm) {
        unsigned long long base = 0;
        if (lane == (int)__builtin_ctzll(wm)) base = atomicAdd(counter, (unsigned long long)__popcll(wm));
        base = __shfl(base, (int)__builtin_ctzll(wm));
        if (want) {
          u = base + (uint64_t)__popcll(wm & ((1ull << lane) - 1ull));
          if (u >= 2ull * (uint64_t)A.n) {
            pst = L_END;
          } else {
            const int64_t r = (int64_t)(u >> 1);
            pa = (u & 1) ? 0 : 1;
            const int64_t rr = A.ids ? A.ids[r] : r;
            plen = (int)A.len[rr];
            psq = A.seq + A.off[rr];
            pmd = o.fnr_pos ? (int)A.maxdiff_tab[plen] : o.max_diff;
            pseed = plen > o.seed_len;
            const uint2 *wb = A.wbuf + (uint64_t)r * A.wstride;
            pwb = wb + (pa ? A.wlen1 : 0);
            pswb = wb + 2 * A.wlen1 + (pa ? o.seed_len + 1 : 0);
            c0 = c1 = c2 = pmpre = pw = off = pex = pgq = 0;
            if (plen < 1 || plen > COOP_MAXLEN || o.n_stacks > NSTK ||
                (1u << A.stg_log2) < 9u * (uint32_t)(plen + 1) + 16u ||
                (plen > o.seed_len && o.seed_len > COOP_SEEDMAX) || (int)A.nN[r] > pmd ||
                (A.roff && A.roff[rr])) {  // resumed reads start past level 0
              pflag = PRO_SKIP;
              record();
            } else {
              pflag = 0;
              nd = {0u, ixv0.seq_len, plen, 0, 0, 0, 0, pa, STATE_M};
              wim1 = pwb[plen - 1];
              snext = psym(plen - 1);
              pst = L_FETCH;  // the root's pop, once its width is in
            }
          }
        }
      }
    }
    if (__ballot(pst != L_END) == 0ull) break;
    // ---- loads (one round trip)
    const bool exp = pst == L_EXP, tail = pst == L_TAIL, copy = pst == L_COPY;
    const IndexView ix = pa ? ixv0 : ixv1;  // strand a searches bwt[1-a]
    const uint4 *ob = pa ? A.o64[0] : A.o64[1];
    const uint32_t qk = tail ? xk : nd.k, ql = tail ? xl : nd.l;
    const bool qkneg = qk == 0;
    const bool qshare = !qkneg && ((qk - 1) >> 6) == (ql >> 6);
    Blk bk, bl;
    load_blk(ob, ql, exp, bl);
    load_blk(ob, qk - 1, exp && !qkneg && !qshare, bk);
    uint4 tvl = make_uint4(0, 0, 0, 0), tvk = make_uint4(0, 0, 0, 0);
    if (tail) tvl = ob[(size_t)(ql >> 6) * 4 + tcur];
    if (tail && !qkneg && !qshare) tvk = ob[(size_t)((qk - 1) >> 6) * 4 + tcur];
    const int ni = nd.i - 1;
    ExpW w = {};
    uint32_t csym = 0, snx = 0;
    if (exp) {
      csym = psym(ni);
      if (ni > 0) {
        w.im2 = pwb[ni - 1];
        w.im1 = pwb[ni];
        snx = psym(ni - 1);
        const int ii = ni - (plen - o.seed_len);
        if (pseed && ii > 0) {
          w.slo = pswb[ii - 1];
          w.shi = pswb[ii];
        }
      }
    } else if (tail && xj > 0) {
      snx = psym(xj - 1);
    }
    uint4 cv[4];
    const uint32_t tot = c0 + c1 + c2;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (copy && ci + q < tot) cv[q] = ring[ci + q];
    // ---- consume
    if (pst == L_FETCH) {
      ppop();
    } else if (copy) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (ci + q < tot) A.pstore[off + ci + q] = cv[q];
      ci += 4;
      if (ci >= tot) record();
    } else if (tail) {
      // one step of bwt_match_exact_alt (bwt.c:240-247)
      if (qshare) tvk = tvl;
      const uint32_t ok = qkneg ? 0u : occ_of(tvk, qk - 1), ol = occ_of(tvl, ql);
      const uint32_t base = l2of(ix, tcur);
      xk = base + ok + 1;
      xl = base + ol;
      tcur = snx;
      if (xk > xl) finish();
      else if (--xj < 0) { pflag = PRO_HIT; record(); }
      else if (snx > 3) finish();
    } else if (exp) {
      uint32_t mk = 0, ml = 0;
      if (expand_node(o, make_uint4(ix.L2[0], ix.L2[1], ix.L2[2], ix.L2[3]), bl, bk, qkneg, qshare, nd, pmd, pseed,
                      plen, csym, w, t0, t1, q1, q2, ring, pw, SMASK,
                      c0, c1, c2, pex, pgq, mk, ml)) {
        nd.k = mk;
        nd.l = ml;
        nd.i = ni;
        wim1 = w.im2;  // width[ni - 1]
        snext = snx;
        ppop();
      } else {
        finish();
      }
    }
  }
}

hipError_t launch_coop_roots(const CoopArgs &g, unsigned long long *d_counter, int blocks, hipStream_t st) {
  if (g.n <= 0) return hipSuccess;
  hipError_t e = zero_async(d_counter, sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  e = zero_async(g.pstore_next, sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_coop_roots, dim3(blocks), dim3(64), 0, st, g, d_counter);
  return hipGetLastError();
}

hipError_t launch_coop(const CoopArgs &g, unsigned long long *d_counter, int blocks, hipStream_t st) {
  if (g.n <= 0) return hipSuccess;
  for (int c = 0; c < 5; ++c)  // the kernel takes L2 from ix[0] for both strands
    if (g.ix[0].L2[c] != g.ix[1].L2[c]) return hipErrorInvalidValue;
  hipError_t e = zero_async(d_counter, sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  e = zero_async(g.pool_next, sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  if (g.prof) hipLaunchKernelGGL(k_coop<true>, dim3(blocks), dim3(64), 0, st, g, d_counter);
  else hipLaunchKernelGGL(k_coop<false>, dim3(blocks), dim3(64), 0, st, g, d_counter);
  return hipGetLastError();
}

}  // namespace ibwa
