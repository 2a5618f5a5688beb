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
// Slot arena of a lane (16 B slots, addressed by a 16-bit (narrow) or 24-bit
// (wide) slot number): a static region of P0 slots -- its last H slots hold
// the read's hits, the rest the first stack entries -- followed by up to
// max_pages pages of PG slots taken, only when the stack grows that far, from
// its workgroup's page pool (a bitmap in LDS; pages go back when the read
// ends).  Measured on a GRCh37-sized genome the live entries of a 100 bp read
// have median 306, p99 14.5k, max 461k (tools/dfs_stats.py), so memory
// follows the reads actually running instead of the worst case.  Stack slots
// are bump-allocated; a popped slot below the bump pointer goes on a small
// per-lane free stack in LDS and is reused by the next pushes, so the slots in
// use track the live entries (the reference's stack size).  At read end the
// hits are appended to a compact per-batch stream (one atomic per read).  A
// read that needs more (or options that do not fit the bit fields) is re-run,
// exactly, by the retry pass -- or, past the early hand-off rule in the
// LDS-width variant, leaves its search state (dump_states: live stack, hits,
// best score) for the cooperative pass to continue from (coop.hip resume_state).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "engine.h"
#include "occ.h"

namespace ibwa {

namespace {

constexpr int MODE_GAPE = 0x01, MODE_COMPREAD = 0x02, MODE_LOGGAP = 0x04, MODE_NONSTOP = 0x10;
constexpr int STATE_M = 0, STATE_I = 1, STATE_D = 2;
// Gap group (first pass): a gap-opening expansion pushes the insertion child and then the non-empty
// deletion children into one bucket, consecutively (bwtgap.c:221-227), and measured on a
// GRCh37-sized genome 95 % of them are never popped (they score a gap open above the first hit).
// The group is stored as ONE entry: the insertion child with the deletions still pending (z bits
// 16-19 by symbol, ldp = i), in state STATE_G.  Popping it materializes its top deletion (T before G
// before C before A) from its own Occ blocks -- the deletions' intervals are the symbol steps of
// the group's (k, l) -- as the new candidate on top of the group, which keeps the rest; once none
// is left it is the plain insertion child.  Pop order and stack size (a group counts as all of its
// entries) are the reference's; a write per deletion is saved for every group never popped.
constexpr int STATE_G = 3;
// Slots: the first pass takes them from the bump region only (a popped slot is reused when it is the
// last one taken, as in a match chain), so an expansion's pushes land in consecutive slots; the
// retry pass, whose stacks can be large, also reuses popped slots (LDS free stack, free list).
// Same-box A/B at 10M reads: first-pass write requests 4.77G -> 3.63G, time unchanged.
// per-lane LDS stack of popped slots awaiting reuse (the retry pass's heavy reads get more)
constexpr int NARROW_FREE_DEPTH = 8;
constexpr int LW_FREE_DEPTH = 4;  // LDS-width variant: 8 B per lane
constexpr int MAX_BUCKETS = 128;  // non-empty-bucket bitmask: four 32-bit registers
// first pass: a read of <= 16 * RDW bases without N is kept 2-bit packed in LDS, so the read
// symbol of an iteration is an LDS access instead of one more HBM line request
constexpr int RDW = 8;

// Non-empty score buckets as a 128-bit mask in four named registers (no array: scratch).
struct BMask {
  uint32_t m0, m1, m2, m3;
};
__device__ __forceinline__ void bm_set(BMask &m, int b) {
  const uint32_t bit = 1u << (b & 31), w = (uint32_t)b >> 5;
  m.m0 |= w == 0 ? bit : 0u;
  m.m1 |= w == 1 ? bit : 0u;
  m.m2 |= w == 2 ? bit : 0u;
  m.m3 |= w == 3 ? bit : 0u;
}
__device__ __forceinline__ void bm_clr(BMask &m, int b) {
  const uint32_t bit = 1u << (b & 31), w = (uint32_t)b >> 5;
  m.m0 &= w == 0 ? ~bit : ~0u;
  m.m1 &= w == 1 ? ~bit : ~0u;
  m.m2 &= w == 2 ? ~bit : ~0u;
  m.m3 &= w == 3 ? ~bit : ~0u;
}
__device__ __forceinline__ bool bm_has(const BMask &m, int b) {
  const uint32_t w = (uint32_t)b >> 5;
  const uint32_t x = w == 0 ? m.m0 : w == 1 ? m.m1 : w == 2 ? m.m2 : m.m3;
  return (x >> (b & 31)) & 1u;
}
// lowest non-empty bucket >= from (MAX_BUCKETS if none)
__device__ __forceinline__ int bm_next(const BMask &m, int from) {
  const uint32_t w = (uint32_t)from >> 5, lo = ~0u << (from & 31);
  const uint32_t x0 = w > 0 ? 0u : m.m0 & lo;
  const uint32_t x1 = w > 1 ? 0u : (w == 1 ? m.m1 & lo : m.m1);
  const uint32_t x2 = w > 2 ? 0u : (w == 2 ? m.m2 & lo : m.m2);
  const uint32_t x3 = w > 3 ? 0u : (w == 3 ? m.m3 & lo : m.m3);
  return x0 ? __builtin_ctz(x0) : x1 ? 32 + __builtin_ctz(x1) : x2 ? 64 + __builtin_ctz(x2)
                                 : x3 ? 96 + __builtin_ctz(x3) : MAX_BUCKETS;
}

// LW: non-empty buckets of the head ring, bit (b & 15) of m0; the lowest non-empty bucket >= from
// (every live bucket lies in [from - 1, from + 14] when this is asked)
__device__ __forceinline__ int ring_next(uint32_t m, int from) {
  const uint32_t r = (uint32_t)from & (GAP_RING - 1);
  const uint32_t x = ((m >> r) | (m << (GAP_RING - r))) & ((1u << GAP_RING) - 1u);
  return x ? from + __builtin_ctz(x) : (1 << 30);
}

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

// LDS layout (per workgroup of NB lanes, lane-minor so a wave's accesses are consecutive):
//   heads[n_stacks][LN] (H), free[free_depth][LN] (H), ptab[max_pages][LN] (u16), bitmap[ceil(NPB/32)] (u32),
//   narrow only: reads[RDW][LN] (u32, 16 bases each)
// with LN = the block's lanes that run reads (block / 64 * lanes_per_wave)
size_t gapped_lds_bytes(int n_stacks, int block, bool wide, int max_pages, int pages_per_block, int lanes_per_wave,
                        int free_depth, int cw_words) {
  const size_t ln = (size_t)block / 64 * lanes_per_wave;
  if (cw_words > 0 && !wide)  // LDS widths: ring heads, a 4-slot free stack, bitmap, the records
    return (size_t)(GAP_RING + LW_FREE_DEPTH) * ln * 2 + (size_t)((pages_per_block + 31) / 32) * 4 +
           (size_t)cw_words * ln * 4;
  const int fd = wide ? free_depth : NARROW_FREE_DEPTH;
  size_t b = (size_t)(n_stacks + fd) * ln * (wide ? 4 : 2) + (size_t)max_pages * ln * 2;
  b = (b + 3) & ~(size_t)3;
  return b + (size_t)((pages_per_block + 31) / 32) * 4 + (wide ? 0 : (size_t)RDW * ln * 4);
}

// PROF: per-wave cycle accounting of the loop's phases into A.prof[] (diagnostics build of
// the same kernel): 0 claim, 1 pop, 2 wait for the loads, 3 rest; then wave-level event
// counts (the wave executes a block once for all its lanes in it): 4 exact steps, 5 push-loop
// trips, 6 hit blocks, 7 read ends, 8 expansions, 9 wave iterations, 10 read claims.
template <bool WIDE, bool PROF, bool LW, int NBL>
__device__ __forceinline__ void gapped_body(const GapArgs &A, unsigned long long *counter) {
  static_assert(!(WIDE && LW), "the LDS-width variant is a first-pass kernel");
  using E = Ent<WIDE>;
  // gap_shadow positions per iteration (st 5): 16 in the LDS-width first pass (the hot kernel), 8
  // elsewhere (one block register set: the other variants are at their register limit)
  constexpr int SHW = LW ? 16 : 8;
  using H = typename E::Head;
  constexpr bool REUSE = WIDE;
  constexpr uint32_t NILH = E::NIL;
  extern __shared__ uint4 lds_raw[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  const int NB = blockDim.x;
  // LDS lanes: the lanes that run reads; LDS index (x << nbl) + ltid (powers of two)
  // NBL > 0: log2 of the LDS lanes known at compile time (the LW first pass, one instantiation per
  // workgroup size), so a row's LDS address is the lane's plus an immediate offset
  const int LNB = NBL ? (1 << NBL) : (NB >> 6) * A.lanes_per_wave;
  const int nbl = NBL ? NBL : 31 - __builtin_clz(LNB);
  const int ltid = (tid >> 6) * A.lanes_per_wave + (lane < A.lanes_per_wave ? lane : 0);
  const AlnOpt o = A.o;
  H *const lds_heads = reinterpret_cast<H *>(lds_raw);
  // bucket heads: one per bucket, or (LW) a ring of GAP_RING -- every live entry scores within
  // [last popped score, last popped score + max penalty], so score & 15 names its bucket
  auto hidx = [&](int sc) __attribute__((always_inline)) -> uint32_t {
    return LW ? (((uint32_t)sc & (GAP_RING - 1)) << nbl) + ltid : ((uint32_t)sc << nbl) + ltid;
  };
  // free stack of popped slots: narrow, 8 (LW: 4) u16 per lane side by side (one LDS read per
  // expansion); wide (retry pass), lane-minor rows
  constexpr uint32_t NFREE = LW ? LW_FREE_DEPTH : NARROW_FREE_DEPTH;
  H *const free_slots = lds_heads + (LW ? GAP_RING : o.n_stacks) * LNB;
  auto fsi = [&](uint32_t j) __attribute__((always_inline)) -> uint32_t {
    return WIDE ? (j << nbl) + ltid : (uint32_t)ltid * NFREE + j;
  };
  const uint32_t FREE_DEPTH = WIDE ? (uint32_t)A.free_depth : NFREE;
  // page table of a lane: LDS rows ptab[((q) << nbl) + ltid], or (LW) global
  uint16_t *const ptab = reinterpret_cast<uint16_t *>(free_slots + FREE_DEPTH * LNB);
  uint32_t *const bitmap =
      reinterpret_cast<uint32_t *>(ptab + (LW ? 0 : ((A.max_pages * LNB + 1) & ~1)));  // 4-byte aligned, still LDS
  const int bm_words = (A.pages_per_block + 31) / 32;
  uint32_t *const rdl = bitmap + bm_words;  // narrow: the lane's read, rdl[(w << nbl) + ltid]
  // LW: the lane's k_width record (engine.h AlnArgs::cw), word w at cwl[(w << nbl) + ltid]
  uint32_t *const cwl = bitmap + bm_words;
  const uint32_t CWR = A.cw_rw;  // read words; the width bytes start at word 1 + CWR
  auto cw_byte = [&](uint32_t b) __attribute__((always_inline)) -> uint32_t {
    const uint32_t w = 1u + CWR + (b >> 2);
    return (cwl[(w << nbl) + ltid] >> (8 * (b & 3))) & 0xFFu;
  };
  for (int w = tid; w < bm_words; w += NB) {
    const int lo = w * 32, hi = lo + 32 < A.pages_per_block ? lo + 32 : A.pages_per_block;
    bitmap[w] = hi - lo >= 32 ? 0u : ~((1u << (hi - lo)) - 1u);  // bits past the pool stay taken
  }
  __syncthreads();
  const IndexView ixv0 = A.ix[0];  // L2 and seq_len of both strands (checked at launch)
  const bool comp = o.mode & MODE_COMPREAD;
  const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + tid;
  const uint32_t P0 = A.cap1;                  // static slots per lane
  const uint32_t HS = A.hit_slots;             // hits live in static slots [P0 - HS, P0)
  const uint32_t LG = A.page_log2;             // page = 2^LG slots
  // static region: one per lane that runs reads (lanes_per_wave of each wave)
  uint4 *const ent1 = A.ent + ((gtid >> 6) * (uint64_t)A.lanes_per_wave + (uint64_t)(lane < A.lanes_per_wave ? lane : 0)) * P0;
  uint4 *const pool = A.pool + (uint64_t)blockIdx.x * A.pages_per_block * (1ull << LG);
  // highest stack slot + 1 (slot NILH is the list terminator)
  const uint32_t slot_end = P0 + ((uint32_t)A.max_pages << LG) < NILH ? P0 + ((uint32_t)A.max_pages << LG) : NILH;

  int64_t cur = 0, cend = 0;
  bool more = true;
  // ---- lane state
  // 0 idle, 1 search (C valid or empty), 2 exact sub-search, 3 ended (retire), 4 (LW) record loading,
  // 5 gap_shadow of the lane's latest hit (16 width positions per iteration)
  int st = 0;
  uint32_t end_stat = 0;
  int64_t r = 0, ro = 0;  // read of this launch, its output index
  int len = 0, opt_max_diff = 0, max_diff = 0, best_score = 0, n_aln = 0;
  int best_cnt = 0, n_entries = 0;
  uint32_t bump = 0, status = 0, n_free = 0, n_pages = 0, n_iter = 0;
  uint32_t n_pops = 0;  // pops made (bwtgap.c:129): where a resume state splits the read's work
  // freed slots beyond the LDS stack: a list threaded through the slots themselves (x = next);
  // fl_next is the head's successor once known (loaded with an iteration's other loads)
  uint32_t fl_head = 0, fl_next = 0;
  bool fl_known = true;
  bool seeded = false;
  const uint8_t *s = nullptr;
  bool fastrd = false;  // the read's symbols are in LDS (rdl)
  // LW level tables (GapArgs::ltab): this read's nodes at depth <= TK are stored by their string; a read
  // so short that a hit could come at such a depth does not use them
  const uint32_t TK = LW ? A.tab_k : 0u;
  bool tabok = false;
  const uint2 *W0 = nullptr, *W1 = nullptr, *SW0 = nullptr, *SW1 = nullptr;
  BMask nonempty = {0u, 0u, 0u, 0u};
  uint4 C = make_uint4(0, 0, 0, 0);
  uint32_t C_slot = 0;
  int C_b = 0;
  bool C_valid = false;
  bool C_load = false;  // C's data arrives with this iteration's loads (slot C_slot)
  // Register cache of the stack top.  A push that becomes the candidate is not stored: it stays in
  // C ("dirty") and is written only if it is displaced twice.  The entry a push displaces from C
  // is kept in D (with its slot): it is exactly the next candidate once the pushed entry is popped
  // (it was the head of the pushed entry's bucket, or of the next non-empty one), so a match chain
  // -- pop, expand, pop the match child -- needs neither the candidate load nor the child's store.
  // Flags: bit 0 C dirty, bit 1 D valid, bit 2 D dirty.
  uint4 D = make_uint4(0, 0, 0, 0);
  uint32_t D_slot = 0, cfl = 0;
  // exact sub-search state
  uint32_t xk = 0, xl = 0;
  int xj = 0, xa = 0;
  uint4 xe = make_uint4(0, 0, 0, 0);  // the entry that went down the exact path
  // gap_shadow sub-state (st 5, bwtgap.c:81-91 after a hit is added): a lane is never in both
  // sub-states, so it reuses the exact sub-search's registers -- the interval size x of the hit,
  // the new width of the position before the chunk, the chunk's first position, the hit's strand,
  // and (xe) the widths equal to x so far and last_diff_pos
  uint32_t &sh_x = xk, &sh_prevx = xl;
  int &sh_q = xj, &sh_a = xa;
  uint32_t &sh_jj = xe.x, &sh_ldp = xe.y;

  // The per-read argument pointers are re-read from the kernel-argument segment where they are used
  // (read claim, read end) instead of staying live in SGPRs through the loop, where the compiler
  // spilled them into VGPR lanes and read them back in the hot path.
  typedef const __attribute__((address_space(4))) GapArgs KArgs;
  auto args = [&]() __attribute__((always_inline)) -> KArgs * {
    KArgs *p = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();  // A is the first kernel argument
    asm volatile("" : "+s"(p));
    return p;
  };
  auto ptab_at = [&](uint32_t q) __attribute__((always_inline)) -> uint16_t & {
    if (LW) return args()->ptab_g[gtid * GAP_MAX_PAGES + q];
    return ptab[((q) << nbl) + ltid];
  };
  auto slot_ptr = [&](uint32_t slot) __attribute__((always_inline)) -> uint4 * {
    if (slot < P0) return ent1 + slot;
    const uint32_t q = (slot - P0) >> LG;
    return pool + ((uint64_t)ptab_at(q) << LG) + ((slot - P0) & ((1u << LG) - 1u));
  };
  // the read is done: hits to the output stream, pages back to the pool
  uint64_t pf0 = 0, pf1 = 0, pf2 = 0, pf3 = 0, pf4 = 0, pf5 = 0, pf6 = 0, pf7 = 0, t_rest = 0;
  uint64_t pf8 = 0, pf9 = 0, pf10 = 0;
  // lane counts (PROF): block loads, second-block loads, width loads, seed-width loads, candidate loads, live lanes
  uint64_t pl11 = 0, pl12 = 0, pl13 = 0, pl14 = 0, pl15 = 0, pl16 = 0, pl17 = 0, pl18 = 0;
  auto pnow = []() __attribute__((always_inline)) -> uint64_t {
    uint64_t t = 0;
    if (PROF) __asm__ volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
  };
  auto pleader = [&]() __attribute__((always_inline)) -> bool {
    return PROF && lane == __builtin_ctzll(__builtin_amdgcn_read_exec());
  };
  // a free page of this workgroup's pool for the lane's next slots
  auto take_page = [&]() __attribute__((always_inline)) -> bool {
    for (int w = 0; w < bm_words; ++w) {
      uint32_t x = bitmap[w];
      while (x != 0xFFFFFFFFu) {
        const uint32_t bit = (uint32_t)__builtin_ctz(~x);
        const uint32_t old = atomicOr(&bitmap[w], 1u << bit);
        if (!(old & (1u << bit))) {
          ptab_at(n_pages) = (uint16_t)(w * 32 + bit);
          ++n_pages;
          return true;
        }
        x = old | (1u << bit);
      }
    }
    return false;
  };
  // (the room for its na hits was reserved at pos, and its first four hits hb.v3, v2, v1, v0 loaded,
  // in the iteration's round trip: see `ending` below)
  auto end_read = [&](uint32_t stat, uint32_t na, unsigned long long pos, const Blk &hb) __attribute__((always_inline)) {
    const bool pl_ = pleader();
    KArgs *ka = args();
    if (na) {
      if (pos + (unsigned long long)na > ka->aln_total) {
        stat |= ST_ALN_OVERFLOW;
        na = 0;
      } else {
        // the hit's last_diff_pos rides in bits 16-31 (resume states replay gap_shadow): masked off
        auto put = [&](uint32_t j, uint4 h) __attribute__((always_inline)) {
          h.w &= 0xFFFFu;
          ka->aln[pos + j] = h;
        };
        put(0, hb.v3);
        if (na > 1) put(1, hb.v2);
        if (na > 2) put(2, hb.v1);
        if (na > 3) put(3, hb.v0);
        for (uint32_t j = 4; j < na; ++j) put(j, ent1[P0 - 1 - j]);
        ka->aln_off[ro] = pos;
      }
    }
    ka->n_aln[ro] = na;
    ka->status[ro] = stat;
    if (ka->iters) ka->iters[ro] = n_iter;
    for (uint32_t q = 0; q < n_pages; ++q) {
      const uint32_t pg = ptab_at(q);
      atomicAnd(&bitmap[pg >> 5], ~(1u << (pg & 31)));
    }
    n_pages = 0;
    st = 0;
    if (pl_) ++pf7;
  };

  // Resume states (LW, GapArgs::rdump): the lanes in `me` are between two pops; the whole wave copies
  // each one's live stack, its hits and its search variables to the state buffer, and the lane hands
  // its read on.  C (score minsc, slot cs, link cp) is the top of the lowest non-empty bucket.  Pops
  // come in score order, so every stored entry scoring above minsc is live and every one below is
  // dead.  At minsc the live entries are C and the list below it: the ones that were in the bucket
  // when its level started, minus those popped from the top since, all in slots below any pushed
  // since (the bump region only grows past live slots) -- i.e. every entry at minsc in a slot <= cp
  // is live and every other one but C is dead.  So the state is the stored entries (after the dirty
  // register entries are written back) that pass that test, in slot order: per bucket bottom to top.
  auto dump_states = [&](bool me, int minsc, uint32_t cs, uint32_t cp) __attribute__((always_inline)) {
    if (me) {
      if (cfl & 1u) *slot_ptr(C_slot) = C;
      if ((cfl & 6u) == 6u) *slot_ptr(D_slot) = D;
    }
    __threadfence_block();
    KArgs *ka = args();
    unsigned long long dm = __ballot(me);
    while (dm) {
      const int src = __builtin_ctzll(dm);
      dm &= dm - 1;
      const uint32_t sbump = (uint32_t)__shfl((int)bump, src), sna = (uint32_t)__shfl(n_aln, src);
      const uint32_t sne = (uint32_t)__shfl(n_entries, src), spops = (uint32_t)__shfl((int)n_pops, src);
      const int smin = __shfl(minsc, src);
      const uint32_t scs = (uint32_t)__shfl((int)cs, src), scp = (uint32_t)__shfl((int)cp, src);
      // the first pass runs 64 reads per wave: lane x's static region is region gtid
      const uint64_t sg = gtid - (uint64_t)lane + (uint64_t)src;
      const uint4 *const se1 = A.ent + sg * P0;
      const uint16_t *const spt = ka->ptab_g + sg * GAP_MAX_PAGES;
      // two sweeps over the slots: count the live entries, then (room reserved) copy them
      auto sweep = [&](uint4 *out) __attribute__((always_inline)) -> uint32_t {
        uint32_t cnt = 0;
        for (uint32_t b0 = 0; b0 < sbump; b0 += 128) {
          const uint32_t s0 = b0 + (uint32_t)lane, s1 = s0 + 64u;
          const bool ok0 = s0 < sbump && (s0 < P0 - HS || s0 >= P0), ok1 = s1 < sbump && (s1 < P0 - HS || s1 >= P0);
          auto sp = [&](uint32_t x) __attribute__((always_inline)) -> const uint4 * {
            if (x < P0) return se1 + x;
            return pool + ((uint64_t)spt[(x - P0) >> LG] << LG) + ((x - P0) & ((1u << LG) - 1u));
          };
          uint4 e0 = make_uint4(0, 0, 0, 0), e1 = make_uint4(0, 0, 0, 0);
          if (ok0) e0 = *sp(s0);
          if (ok1) e1 = *sp(s1);
          // entries stored by their strings leave with their intervals (the cooperative pass expands from
          // Occ blocks: tables there measured no faster, profiles/r06_sweep_tab2.jsonl)
          auto by_interval = [&](uint4 &x) __attribute__((always_inline)) {
            if (LW && TK > 0 && out && x.y >= LTAB_MARK) {
              const uint2 *tb = ((x.w >> 28) & 1u) ? A.ltab[0] : A.ltab[1];
              const uint2 iv = tb[ltab_off(x.y & 0xFFu) + x.x];
              x.x = iv.x;
              x.y = iv.y;
            }
          };
          by_interval(e0);
          by_interval(e1);
          auto live = [&](const uint4 &x, uint32_t slot) __attribute__((always_inline)) {
            const int sc = (int)(((x.w >> 16) & 31u) * (uint32_t)o.s_mm + ((x.w >> 21) & 7u) * (uint32_t)o.s_gapo +
                                 ((x.w >> 24) & 15u) * (uint32_t)o.s_gape);
            return sc > smin || (sc == smin && (slot == scs || (scp != NILH && slot <= scp)));
          };
          const bool l0 = ok0 && live(e0, s0), l1 = ok1 && live(e1, s1);
          const unsigned long long m0 = __ballot(l0), m1 = __ballot(l1);
          if (out && l0) out[RD_HDR + cnt + (uint32_t)__popcll(m0 & lt_mask)] = e0;
          cnt += (uint32_t)__popcll(m0);
          if (out && l1) out[RD_HDR + cnt + (uint32_t)__popcll(m1 & lt_mask)] = e1;
          cnt += (uint32_t)__popcll(m1);
        }
        return cnt;
      };
      const uint32_t nlive = sweep(nullptr);
      const unsigned long long need = (unsigned long long)RD_HDR + nlive + sna;
      unsigned long long off = 0;
      if (lane == src) off = atomicAdd(ka->rd_next, need);
      off = __shfl(off, src);
      if (off + need <= ka->rd_cap) {
        uint4 *const out = ka->rdump + off;
        const uint32_t cnt = sweep(out);
        for (uint32_t j = (uint32_t)lane; j < sna; j += 64) out[RD_HDR + cnt + j] = se1[P0 - 1 - j];
        if (lane == src) {
          out[0] = make_uint4(cnt, sna, (uint32_t)smin, sne);
          out[1] = make_uint4((uint32_t)best_score, (uint32_t)best_cnt, (uint32_t)max_diff, spops);
          ka->roff[ro] = off + 1;
          if (ka->hpop) ka->hpop[ro] = spops;
          atomicAdd(ka->rd_next + 1, 1ull);  // states stored
        }
      }
    }
    if (me) {
      status |= ST_HEAVY | (uint32_t)(n_entries < 0xFFFF ? n_entries : 0xFFFF) << 16;
      n_entries = 0;
    }
  };

  for (;;) {
    uint64_t t_top = pnow();
    if (PROF && t_rest) pf3 += t_top - t_rest;
    // ------------------------------------------------ retire reads that ended last iteration
    // the search state of a claimed read whose length, max_diff and N count are set: the two roots
    // (bwtgap.c:126-127: strand 0 then strand 1, both score 0 -> C = strand 1)
    auto start_read = [&]() __attribute__((always_inline)) {
      max_diff = opt_max_diff;
      best_score = (opt_max_diff + 1) * o.s_mm + (o.max_gapo + 1) * o.s_gapo + (o.max_gape + 1) * o.s_gape;
      best_cnt = 0;
      n_aln = 0;
      status = 0;
      seeded = len > o.seed_len;
      // (a hit needs every read symbol consumed: depth >= len - the insertions, at most 7 + 15)
      tabok = LW && TK > 0 && len > (int)TK + 24;
      const uint32_t root_l = tabok ? LTAB_MARK : ixv0.seq_len;  // the root by its (empty) string
      ent1[0] = E::make(0u, root_l, len, 0, NILH, 0, 0, 0, 0, STATE_M);
      C = E::make(0u, root_l, len, 0, 0u, 0, 0, 0, 1, STATE_M);
      ent1[1] = C;
      // every bucket head starts empty (a pop that empties a bucket writes NIL back), so a
      // push reads its bucket's head without consulting the non-empty mask
      for (int b = 1; b < (LW ? GAP_RING : o.n_stacks); ++b) lds_heads[hidx(b)] = (H)NILH;
      lds_heads[hidx(0)] = 1;
      nonempty.m0 = 1u;
      nonempty.m1 = nonempty.m2 = nonempty.m3 = 0u;
      bump = 2;
      n_free = 0;
      fl_head = NILH;
      fl_known = true;
      n_pages = 0;
      n_iter = 0;
      n_pops = 0;
      n_entries = 2;
      C_slot = 1;
      C_b = 0;
      C_valid = true;
      C_load = false;
      cfl = 0;
      end_stat = 0;  // LW: bit 31 = leave a resume state at the next pop
      st = 1;
    };
    // LW: reads claimed last iteration -- their records reached LDS with that iteration's loads
    if (LW && __ballot(st == 4)) {
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (st == 4) {
        const uint32_t hdr = cwl[ltid];
        len = (int)(hdr & 0xFFFFu);
        opt_max_diff = (int)(hdr >> 24);
        const int nN = (int)((hdr >> 16) & 0xFFu);
        if (nN > opt_max_diff) {  // bwtgap.c:116-122
          KArgs *ka = args();
          ka->n_aln[ro] = 0;
          ka->status[ro] = 0;
          st = 0;
        } else {
          fastrd = nN == 0 && len <= 16 * (int)CWR;
          start_read();
        }
      }
    }
    // ------------------------------------------------ claim + init new reads
    // lanes_per_wave < 64 (retry pass): a wave runs that many heavy reads, so each
    // iteration executes only their paths
    const int lpw = A.lanes_per_wave;
    unsigned long long need = __ballot(st == 0 && lane < lpw);
    while (need && more) {
      if (cur >= cend) {
        int64_t base = 0;
        if (lane == 0) base = (int64_t)atomicAdd(counter, (unsigned long long)lpw);
        base = __shfl(base, 0);
        if (base >= A.n) { more = false; break; }
        cur = base;
        cend = base + lpw < A.n ? base + lpw : A.n;
      }
      const int rank = __popcll(need & lt_mask);
      const int64_t avail = cend - cur;
      if (st == 0 && rank < avail) {
        if (pleader()) ++pf10;
        r = cur + rank;
        KArgs *ka = args();
        const int64_t rr = ka->ids ? ka->ids[r] : r;
        ro = ka->out_by_id ? rr : r;
        s = ka->seq + ka->off[rr];
        const uint2 *wb = ka->wbuf + (uint64_t)r * ka->wstride;
        W0 = wb;
        W1 = wb + ka->wlen1;
        SW0 = wb + 2 * ka->wlen1;
        SW1 = SW0 + (o.seed_len + 1);
        if (LW) {
          // the read's k_width record straight into its LDS rows (no registers); it is used from
          // the next iteration on, after that iteration's loads have been waited for
          const uint32_t *src = ka->cw + (uint64_t)r * ka->cw_words;
          const uint32_t nw = ka->cw_words;
          __attribute__((address_space(3))) uint32_t *dst =
              (__attribute__((address_space(3))) uint32_t *)(cwl + (tid & ~63));
          for (uint32_t w = 0; w < nw; ++w)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + w),
                                             (__attribute__((address_space(3))) void *)(dst + (w << nbl)), 4, 0, 0);
          st = 4;
        } else {
          len = (int)ka->len[rr];
          opt_max_diff = o.fnr_pos ? (int)ka->maxdiff_tab[len] : o.max_diff;
          const int nN = (int)ka->nN[r];
          if (nN > opt_max_diff) {  // bwtgap.c:116-122
            ka->n_aln[ro] = 0;
            ka->status[ro] = 0;
          } else {
            fastrd = !WIDE && nN == 0 && len <= 16 * RDW;
            if (fastrd) {
              // 16 B loads from the aligned-down start (the staging buffer has 16 B of tail padding)
              const uint4 *q0 = reinterpret_cast<const uint4 *>(reinterpret_cast<uintptr_t>(s) & ~(uintptr_t)15);
              const int mis = (int)(reinterpret_cast<uintptr_t>(s) & 15);
              const int nq = (mis + len + 15) >> 4;
              uint32_t w = 0;
              for (int q = 0; q < nq; ++q) {
                const uint4 v = q0[q];
#pragma unroll
                for (int b = 0; b < 16; ++b) {
                  const uint32_t word = b < 4 ? v.x : b < 8 ? v.y : b < 12 ? v.z : v.w;
                  const int jj = q * 16 + b - mis;
                  if (jj >= 0 && jj < len) {
                    w |= ((word >> (8 * (b & 3))) & 3u) << (2 * (jj & 15));
                    if ((jj & 15) == 15 || jj == len - 1) {
                      rdl[((jj >> 4) << nbl) + ltid] = w;
                      w = 0;
                    }
                  }
                }
              }
            }
            start_read();
          }
        }
      }
      const int64_t cnt = __popcll(need);
      cur += avail < cnt ? avail : cnt;
      need = __ballot(st == 0 && lane < lpw);
    }
    if (__ballot(st != 0) == 0ull) break;
    uint64_t t_pop = pnow();
    pf0 += t_pop - t_top;

    ++n_iter;
    if (PROF && lane == 0) ++pf9;
    // ------------------------------------------------ decide this iteration's work
    // search lanes pop C; exact lanes advance one symbol
    bool do_pop = false, finish = false, do_mat = false, dump_now = false;
    const bool over_budget = A.max_iters && n_iter > A.max_iters;
    // the launch's tail: no read left to claim and few lanes of this wave still busy -- their reads
    // leave their states for the cooperative pass instead of holding the wave (and the launch) open
    const bool tail = LW && A.rdump && A.tail_lanes && !more && (uint32_t)__popcll(__ballot(st != 0)) <= A.tail_lanes &&
                      n_iter > A.tail_iters;
    if ((over_budget || tail || (A.early_iters && n_iter > A.early_iters && n_entries > (int)A.early_entries)) &&
        (st == 1 || st == 2)) {
      if (LW && A.rdump && !over_budget && st == 1) {
        // resume: the read leaves its search state at this pop (below)
        end_stat |= 0x80000000u;
      } else if (LW && A.rdump && !over_budget) {
        // resume: the exact sub-search ends first
      } else {
        // a long search: the retry pass re-runs it from the start; bits 16-31 keep the stack size
        // (the cooperative pass takes the biggest first, so its longest reads do not start last)
        status |= ST_HEAVY | (uint32_t)(n_entries < 0xFFFF ? n_entries : 0xFFFF) << 16;
        st = 1;
        n_entries = 0;
      }
    }
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
        } else if (LW && (end_stat >> 31)) {
          // resume state (dump_states): C is the top of the lowest non-empty bucket
          dump_now = true;
          m = e_score;
        } else if (!WIDE && state == STATE_G) {
          do_mat = true;  // a gap group: its top deletion is the entry the reference pops
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
    if (LW && __ballot(dump_now)) {
      dump_states(dump_now, m, C_slot, E::prev(C));
      if (dump_now) finish = true;  // handed on (status set), with or without a stored state
    }
    if (do_pop) {
      const uint32_t prev = E::prev(e);
      lds_heads[hidx(C_b)] = (H)prev;
      --n_entries;
      ++n_pops;
      if (C_slot + 1 == bump) {
        bump = C_slot;
      } else if (REUSE && n_free < FREE_DEPTH) {
        free_slots[fsi(n_free)] = (H)C_slot;
        ++n_free;
      } else if (REUSE) {
        reinterpret_cast<uint32_t *>(slot_ptr(C_slot))[0] = fl_head;
        fl_next = fl_head;
        fl_head = C_slot;
        fl_known = true;
      }
      if (prev != NILH) {
        load_slot = prev;
        C_load = true;
      } else {
        int b;
        if (LW) {
          nonempty.m0 &= ~(1u << (C_b & (GAP_RING - 1)));
          b = ring_next(nonempty.m0, C_b + 1);
        } else {
          bm_clr(nonempty, C_b);
          b = bm_next(nonempty, C_b + 1);
        }
        if (b < o.n_stacks) {
          load_slot = lds_heads[hidx(b)];
          C_b = b;
          C_load = true;
        } else {
          C_load = false;
        }
      }
      C_valid = false;
      if (C_load) {
        C_slot = load_slot;
        if ((cfl & 2u) && load_slot == D_slot) {  // the next candidate is the cached D: no load
          C = D;
          C_valid = true;
          C_load = false;
          cfl = (cfl >> 2) & 1u;  // C dirty = D dirty; D invalid
        } else {
          cfl &= ~1u;  // C arrives from memory
        }
      }
    }

    uint64_t t_issue = pnow();
    pf1 += t_issue - t_pop;
    // ------------------------------------------------ issue every load of this iteration
    const bool srch = do_pop && m >= 0;
    // strand a searches bwt[1-a]; the two BWTs have the same L2 and length (a text and its reverse,
    // checked at launch), so those are uniform: no per-lane select of an IndexView
    const uint4 *ob = a ? A.o64[0] : A.o64[1];
    uint32_t k = e.x, l = e.y;
    // exact lanes query (xk-1, xl) on bwt[1-xa]
    const uint4 *obq = st == 2 ? (xa ? A.o64[0] : A.o64[1]) : ob;
    const uint32_t qk = st == 2 ? xk : k, ql = st == 2 ? xl : l;
    const bool qrun = (srch && i > 0) || (st == 2 && xj >= 0) || do_mat;
    // a node stored by its string: its children's intervals from the level table (one 32 B load),
    // and for a deletion state its own interval (the max_del_occ test); no Occ blocks
    const bool shq = LW && TK > 0 && st == 1 && qrun && e.y >= LTAB_MARK;
    const uint32_t sdep = e.y & 0xFFu;
    const bool qkneg = qk == 0;
    const bool qshare = !qkneg && ((qk - 1) >> 6) == (ql >> 6);
    Blk bk, bl;
    // a shadowing lane loads 16 width positions of its hit's strand into the block registers
    const bool shd = st == 5;
    const uint4 *shp = reinterpret_cast<const uint4 *>((sh_a ? W1 : W0) + sh_q);
    // a lane whose read ended last iteration (st 3) reserves its hits' room in the output stream and
    // loads its first four hits (the last static slots) in this same round trip; the consume step
    // writes them (end_read) -- the wave no longer waits on the atomic and then on the hit loads
    const bool ending = st == 3;
    const uint32_t na_end = ending && !end_stat ? (uint32_t)n_aln : 0u;
    unsigned long long e_pos = 0;
    if (na_end) e_pos = atomicAdd(args()->aln_next, (unsigned long long)na_end);
    load_blk(shd ? shp : na_end ? ent1 + (P0 - 4) : obq, (shd || na_end) ? 0u : ql, (qrun && !shq) || shd || na_end, bl);
    load_blk(shd ? shp + 4 : obq, shd ? 0u : qk - 1, (qrun && !qkneg && !qshare && !shq) || (shd && SHW > 8), bk);
    if (shq) {
      const uint2 *tb = a ? A.ltab[0] : A.ltab[1];
      const uint4 *ch = reinterpret_cast<const uint4 *>(tb + ltab_off(sdep + 1) + ((uint64_t)e.x << 2));
      bl.v0 = ch[0];
      bl.v1 = ch[1];
      if (state == STATE_D) {
        const uint2 own = tb[ltab_off(sdep) + e.x];
        bl.v2.x = own.x;
        bl.v2.y = own.y;
      }
    }
    // width bounds of strand a at positions i-2, i-1 and the seed pair
    const uint2 *Wa = a ? W1 : W0;
    const uint2 *SWa = a ? SW1 : SW0;
    // as bids (bid1 = width[i-1].bid, bid2 = width[i-2].bid), "width[i-2] == width[i-1]" (eq12), and
    // the seed pair's (sb_lo, sb_hi, seq_hi); LW: from the LDS record (bids clamped where no test
    // can tell them apart, engine.h AlnArgs::cw)
    uint32_t bid1 = 0, bid2 = 0, sb_lo = 0, sb_hi = 0;
    bool eq12 = false, seq_hi = false;
    const int ii = (i - 1) - (len - o.seed_len);
    if (LW) {
      if (srch && i > 0) {
        const uint32_t n1 = cw_byte((uint32_t)(i - 1)) >> (4 * a);
        bid1 = n1 & 7u;
        eq12 = (n1 >> 3) & 1u;
      }
      if (srch && i > 1) bid2 = (cw_byte((uint32_t)(i - 2)) >> (4 * a)) & 7u;
      if (srch && i > 1 && seeded && ii > 0) {
        const uint32_t sbase = A.wlen1;
        sb_lo = (cw_byte(sbase + (uint32_t)(ii - 1)) >> (3 * a)) & 3u;
        const uint32_t nh = cw_byte(sbase + (uint32_t)ii) >> (3 * a);
        sb_hi = nh & 3u;
        seq_hi = (nh >> 2) & 1u;
      }
    } else {
      uint2 w_im1 = make_uint2(0, 0), w_im2 = make_uint2(0, 0), sw_lo = make_uint2(0, 0), sw_hi = make_uint2(0, 0);
      if (srch && i > 0) w_im1 = Wa[i - 1];
      if (srch && i > 1) w_im2 = Wa[i - 2];
      if (srch && i > 1 && seeded && ii > 0) {
        sw_lo = SWa[ii - 1];
        sw_hi = SWa[ii];
      }
      bid1 = w_im1.y;
      bid2 = w_im2.y;
      eq12 = w_im2.x == w_im1.x;
      sb_lo = sw_lo.y;
      sb_hi = sw_hi.y;
      seq_hi = sw_lo.x == sw_hi.x;
    }
    // read symbol str[i-1] (search) or str[xj] (exact); strand 1 = complement under COMPREAD
    uint32_t sym = 0;
    {
      const int sp = (srch && i > 0) ? i - 1 : (st == 2 && xj >= 0) ? xj : -1;
      if (sp >= 0)
        sym = fastrd ? ((LW ? cwl[((1u + ((uint32_t)sp >> 4)) << nbl) + ltid] : rdl[((sp >> 4) << nbl) + ltid]) >>
                        (2 * (sp & 15))) & 3u
                     : s[sp];
    }
    // next candidate
    uint4 Cn = make_uint4(0, 0, 0, 0);
    if (do_pop && C_load) Cn = *slot_ptr(load_slot);
    // successor of the free-list head, if a push took the previous head
    uint32_t fl_ld = 0;
    if (!fl_known) fl_ld = reinterpret_cast<const uint32_t *>(slot_ptr(fl_head))[0];
    if (PROF) {
      const unsigned long long b11 = __ballot(qrun), b12 = __ballot(qrun && !qkneg && !qshare),
                               b13 = __ballot(srch && i > 0), b14 = __ballot(srch && i > 1 && seeded && ii > 0),
                               b15 = __ballot(do_pop && C_load), b16 = __ballot(st != 0), b17 = __ballot(st == 2),
                               b18 = __ballot(st == 2 && xk == xl);
      if (lane == 0) {
        pl11 += __popcll(b11);
        pl12 += __popcll(b12);
        pl13 += __popcll(b13);
        pl14 += __popcll(b14);
        pl15 += __popcll(b15);
        pl16 += __popcll(b16);
        pl17 += __popcll(b17);
        pl18 += __popcll(b18);
      }
    }
    if (PROF) {
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      t_rest = pnow();
      pf2 += t_rest - t_issue;
    }

    // ------------------------------------------------ consume
    if (!fl_known) {
      fl_next = fl_ld;
      fl_known = true;
    }
    if (do_pop && C_load) {
      C = Cn;
      C_valid = true;
    }
    if (finish) {
      end_stat = status;
      st = 3;
      continue;
    }
    if (ending) {
      end_read(end_stat, na_end, e_pos, bl);
      continue;
    }
    if (shd) {
      // ---- gap_shadow (bwtgap.c:81-91) of positions sh_q .. sh_q + 15 (< ldp) of strand sh_a: the
      // hit's interval size is taken off every width above it, and a width equal to it becomes the
      // jj-th largest row with bid 1.  LW: the LDS nibbles follow (the bid, clamped, and "equals the
      // previous position's width" of every position up to ldp).
      uint2 *width = const_cast<uint2 *>(sh_a ? W1 : W0);
      const uint32_t mx = ixv0.seq_len, cf = (uint32_t)opt_max_diff + 1u;
      const int ldp_ = (int)sh_ldp;
      const uint4 wq[8] = {bl.v0, bl.v1, bl.v2, bl.v3, bk.v0, bk.v1, bk.v2, bk.v3};
#pragma unroll
      for (int u = 0; u < SHW; ++u) {
        const int pp = sh_q + u;
        const uint4 &h = wq[u >> 1];
        uint2 w = (u & 1) ? make_uint2(h.z, h.w) : make_uint2(h.x, h.y);
        if (pp < ldp_) {
          if (w.x > sh_x) {
            w.x -= sh_x;
            width[pp] = w;
          } else if (w.x == sh_x) {
            ++sh_jj;
            w = make_uint2(mx - sh_jj, 1u);
            width[pp] = w;
          }
          if (LW) {
            const uint32_t eq = pp > 0 && sh_prevx == w.x;
            const uint32_t wd = 1u + CWR + ((uint32_t)pp >> 2), sh = 8u * ((uint32_t)pp & 3u) + 4u * (uint32_t)sh_a;
            uint32_t &cell = cwl[(wd << nbl) + ltid];
            cell = (cell & ~(0xFu << sh)) | (((w.y < cf ? w.y : cf) | eq << 3) << sh);
          }
          sh_prevx = w.x;
        } else if (LW && pp == ldp_ && ldp_ > 0 && ldp_ <= len) {
          // the position after the shadowed ones: only its "equal to the previous width" bit
          const uint32_t wd = 1u + CWR + ((uint32_t)pp >> 2), sh = 8u * ((uint32_t)pp & 3u) + 4u * (uint32_t)sh_a;
          uint32_t &cell = cwl[(wd << nbl) + ltid];
          cell = (cell & ~(0x8u << sh)) | ((sh_prevx == w.x ? 1u : 0u) << 3 << sh);
        }
      }
      sh_q += SHW;
      if (sh_q > ldp_) st = 1;  // every position up to ldp seen: back to popping
      continue;
    }
    const uint32_t csym = (st == 2 ? xa : a) == 1 && comp && sym < 4 ? 3u - sym : sym;
    // this iteration's rank queries, all four symbols: the children intervals (KK[c], LL[c])
    // of (qk, ql) -- for the exact step, the exact first step and the expansion alike
    uint4 KK = make_uint4(0, 0, 0, 0), LL = make_uint4(0, 0, 0, 0);
    if (shq) {
      KK = make_uint4(bl.v0.x, bl.v0.z, bl.v1.x, bl.v1.z);
      LL = make_uint4(bl.v0.y, bl.v0.w, bl.v1.y, bl.v1.w);
    } else if (qrun) {
      const uint4 cl4 = occ4_of(bl, ql);
      const uint4 ck4 = qkneg ? make_uint4(0, 0, 0, 0)
                              : make_uint4(occ_of(qshare ? bl.v0 : bk.v0, qk - 1),
                                           occ_of(qshare ? bl.v1 : bk.v1, qk - 1),
                                           occ_of(qshare ? bl.v2 : bk.v2, qk - 1),
                                           occ_of(qshare ? bl.v3 : bk.v3, qk - 1));
      KK = make_uint4(ixv0.L2[0] + ck4.x + 1, ixv0.L2[1] + ck4.y + 1, ixv0.L2[2] + ck4.z + 1, ixv0.L2[3] + ck4.w + 1);
      LL = make_uint4(ixv0.L2[0] + cl4.x, ixv0.L2[1] + cl4.y, ixv0.L2[2] + cl4.z, ixv0.L2[3] + cl4.w);
    }

    // the children of a node stored by its string are stored by theirs too while their depth is <= TK
    const bool shch = shq && sdep + 1u <= TK;
    auto cxk = [&](uint32_t c) __attribute__((always_inline)) -> uint32_t { return shch ? (e.x << 2 | c) : pick4(KK, c); };
    auto cxl = [&](uint32_t c) __attribute__((always_inline)) -> uint32_t {
      return shch ? (LTAB_MARK | (sdep + 1u)) : pick4(LL, c);
    };

    if (st == 2) {
      // one step of bwt_match_exact_alt (bwt.c:240-247)
      const bool pl_ = pleader();
      bool fail = false;
      if (xj >= 0) {
        if (csym > 3) {
          fail = true;
        } else {
          xk = pick4(KK, csym);
          xl = pick4(LL, csym);
          if (xk > xl) fail = true;
          --xj;
        }
      }
      if (pl_) ++pf4;
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
    if (do_mat) {
      // ---- the top deletion of gap group C, from C's blocks: the new candidate, on top of the
      // group (kept in D with the deletions still pending); nothing is popped, the stack size stays
      const uint32_t dm = (e.z >> 16) & 15u;
      const uint32_t c = 31u - (uint32_t)__builtin_clz(dm);
      const uint32_t dmr = dm & ~(1u << c);
      // one slot: LDS free stack, free list (its successor is known here), else the bump region
      uint32_t slot = 0;
      if (REUSE && n_free) {
        --n_free;
        slot = (uint32_t)free_slots[fsi(n_free)];
      } else if (REUSE && fl_head != NILH) {
        slot = fl_head;
        fl_head = fl_next;
        fl_known = fl_head == NILH;
      } else {
        const uint32_t skip_at = P0 - HS;
        slot = bump == skip_at ? bump + HS : bump;  // the bump region skips the hit area
        const uint32_t b_end = slot + 1;
        if (b_end > slot_end || (b_end > P0 && ((b_end - 1 - P0) >> LG) >= n_pages && !take_page())) {
          end_stat = status | ST_STACK_OVERFLOW;
          st = 3;
          continue;
        }
        bump = b_end;
      }
      const uint32_t g_prev = E::prev(e);
      const uint4 del = E::make(cxk(c), cxl(c), i + 1, i + 1, C_slot, e_mm, e_go, e_ge, a, STATE_D);
      const uint4 grp = dmr ? E::make(k, l, i, (int)dmr, g_prev, e_mm, e_go, e_ge, a, STATE_G)
                            : E::make(k, l, i, i, g_prev, e_mm, e_go, e_ge, a, STATE_I);
      lds_heads[hidx(C_b)] = (H)slot;
      if ((cfl & 6u) == 6u) *slot_ptr(D_slot) = D;
      D = grp;  // memory holds the group with its old mask, if at all: dirty
      D_slot = C_slot;
      C = del;
      C_slot = slot;
      C_valid = true;
      cfl = 7u;  // C dirty, D valid and dirty
      continue;
    }
    if (!do_pop) continue;
    if (m < 0) continue;                                   // bwtgap.c:147
    if (i > 0 && m < (int)bid1) continue;                 // bwtgap.c:155
    if (i == 0) goto hit;                                  // bwtgap.c:159
    if (m == 0 && (state == STATE_M || (o.mode & MODE_GAPE) || e_ge == o.max_gape)) {
      // bwt_match_exact_alt over str[0..i-1] (bwtgap.c:160-163): the first step uses this
      // iteration's blocks; the rest run in sub-state 2
      if (csym > 3) continue;
      xk = pick4(KK, csym);
      xl = pick4(LL, csym);
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
      const bool pl_ = pleader();
      const int ni = i - 1;
      const uint32_t occ = shq ? bl.v2.y - bl.v2.x + 1 : l - k + 1;  // (by string: its own interval, loaded for STATE_D)
      bool allow_diff = true, allow_M = true;
      if (ni > 0) {
        // width[ni-1] = position i-2, width[ni] = position i-1
        if ((int)bid2 > m - 1) allow_diff = false;
        else if ((int)bid2 == m - 1 && (int)bid1 == m - 1 && eq12) allow_M = false;
        if (seeded && ii > 0) {
          if ((int)sb_lo > m_seed - 1) allow_diff = false;
          else if ((int)sb_lo == m_seed - 1 && (int)sb_hi == m_seed - 1 && seq_hi) allow_M = false;
        }
      }
      // children in the reference's push order (bwtgap.c:216-258), as bits of a mask:
      //   bit 0 insertion (open or extend), bits 1-4 deletion by A,C,G,T, bits 5-8 the
      //   mismatch / match children of symbols (str[i] + 1..4) & 3 (bit 8 = str[i] itself)
      const uint32_t ne4 = (KK.x <= LL.x ? 1u : 0u) | (KK.y <= LL.y ? 2u : 0u) | (KK.z <= LL.z ? 4u : 0u) |
                           (KK.w <= LL.w ? 8u : 0u);  // non-empty symbol children
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
      // symbol children: c_j = (csym + j) & 3 for j = 1..4 -> rotate ne4 so bit j-1 = c_j
      const uint32_t rot = (csym + 1) & 3;
      const uint32_t ner = ((ne4 >> rot) | (ne4 << (4 - rot))) & 15u;
      if (allow_diff && allow_M) vm |= ner << 5;
      else if (csym < 4) vm |= ner & 8u ? 1u << 8 : 0u;  // the match child only
      // a gap-opening expansion's deletions go into its insertion child's gap group (narrow)
      const uint32_t dmask = !WIDE && state == STATE_M && (vm & 1u) ? (vm >> 1) & 15u : 0u;
      // slots for all pushes of this expansion; one new page at most (popcount <= 9)
      if (vm) {
        const uint32_t npush = (uint32_t)__builtin_popcount(vm & ~(dmask << 1));
        const uint32_t reuse = REUSE ? n_free + (fl_head != NILH ? 1u : 0u) : 0u;  // fl_known holds here
        const uint32_t nb = npush > reuse ? npush - reuse : 0u;
        uint32_t b_end = bump + nb;
        if (bump <= P0 - HS && b_end > P0 - HS) b_end += HS;  // bump skips the hit area
        if (b_end > slot_end) {
          status |= ST_STACK_OVERFLOW;
          vm = 0;
        } else if (b_end > P0 && ((b_end - 1 - P0) >> LG) >= n_pages && !take_page()) {
          // the expansion reaches a new page and the workgroup's pool has none
          status |= ST_STACK_OVERFLOW;
          vm = 0;
        }
      }
      // push each child (bwtgap.c:216-258, in the reference's order): link it into its bucket and
      // keep C = head of the lowest non-empty bucket.  The children of one expansion go to at most
      // three buckets -- gaps (sc_base + open/extend penalty), mismatches (+ s_mm), the match child
      // (sc_base) -- so the limits, the slot allocation and the non-empty mask are settled once per
      // expansion and each trip of the loop is branch-free.
      if (vm) {
        const int sc_base = e_mm * o.s_mm + e_go * o.s_gapo + e_ge * o.s_gape;
        const int sc_gap = state == STATE_M ? o.s_gapo : o.s_gape;
        const int scG = sc_base + sc_gap, scMM = sc_base + o.s_mm;
        const bool has_match = (vm & 0x100u) && csym < 4;
        const uint32_t vm_mm = vm & (has_match ? 0xE0u : 0x1E0u);  // mismatch children
        const bool has_gap = (vm & 0x1Fu) != 0, has_mm = vm_mm != 0;
        const bool open = state == STATE_M;
        if ((has_gap && scG >= o.n_stacks) || (has_mm && scMM >= o.n_stacks) || (has_match && sc_base >= o.n_stacks)) {
          status |= ST_BAD_SCORE;
          vm = 0;
        } else if ((has_mm && e_mm + 1 > 31) || (has_gap && open && e_go + 1 > 7) || (has_gap && !open && e_ge + 1 > 15)) {
          status |= ST_STACK_OVERFLOW;
          vm = 0;
        }
        const uint32_t npush = (uint32_t)__builtin_popcount(vm & ~(dmask << 1));
        const uint32_t n_fs = !REUSE ? 0u : npush < n_free ? npush : n_free;  // from the LDS free stack, top down
        const bool use_fl = REUSE && npush > n_fs && fl_head != NILH;    // one slot of the free list (fl_known)
        const uint32_t fs_top = n_free, fl_slot = fl_head, b0 = bump, skip_at = P0 - HS;
        const uint32_t fl_n = use_fl ? 1u : 0u;
        // narrow: the lane's whole free stack in one LDS read
        uint4 fsr = make_uint4(0, 0, 0, 0);
        if (LW && n_fs) {
          const uint2 f2 = *reinterpret_cast<const uint2 *>(free_slots + fsi(0));
          fsr.x = f2.x;
          fsr.y = f2.y;
        } else if (!WIDE && n_fs) {
          fsr = *reinterpret_cast<const uint4 *>(free_slots + fsi(0));
        }
        // slot of the t-th push: free stack, then the free list's head, then the bump region
        // (skipping the hit area)
        auto slot_at = [&](uint32_t t) __attribute__((always_inline)) -> uint32_t {
          const uint32_t fj = t < n_fs ? fs_top - 1 - t : 0u;
          uint32_t fsv;
          if (WIDE) {
            fsv = (uint32_t)free_slots[fsi(fj)];
          } else {
            const uint32_t wlo = (fj & 2) ? fsr.y : fsr.x, whi = (fj & 2) ? fsr.w : fsr.z;
            fsv = (((fj & 4) ? whi : wlo) >> (16 * (fj & 1))) & 0xffffu;
          }
          uint32_t bs = b0 + (t - n_fs - fl_n);
          bs += (b0 <= skip_at && bs >= skip_at) ? HS : 0u;
          return t < n_fs ? fsv : (t == n_fs && use_fl) ? fl_slot : bs;
        };
        // a taking group puts its last child in C (stored, clean); what C and D held is stored
        // first if memory lacks it, and D is dropped (the next candidate after C is loaded)
        auto group_take = [&](bool tk, uint4 last, uint32_t last_slot, int sc) __attribute__((always_inline)) {
          if (tk && C_valid && (cfl & 1u)) *slot_ptr(C_slot) = C;
          if (tk && (cfl & 6u) == 6u) *slot_ptr(D_slot) = D;
          if (tk) {
            C = last;
            C_slot = last_slot;
            C_b = sc;
            C_valid = true;
            cfl = 0;
          }
        };
        uint32_t t = 0;
        // the three target buckets' heads, read together (one LDS wait, not one per group); the
        // gap and mismatch buckets coincide when their penalties do, the match child's never does
        const uint32_t vg = vm & 0x1Fu & ~(dmask << 1);  // with a gap group: the group entry alone
        const uint32_t vmm = vm & vm_mm;
        const bool has_match_ch = has_match && vm;
        const uint32_t hG = vg ? (uint32_t)lds_heads[hidx(scG)] : 0u;
        uint32_t hM = vmm ? (uint32_t)lds_heads[hidx(scMM)] : 0u;
        const uint32_t hB = has_match_ch ? (uint32_t)lds_heads[hidx(sc_base)] : 0u;
        // ---- gap children (bit 0 insertion, bits 1-4 deletion by A..T): bucket scG, stored in order,
        // each linked to the one before
        if (vg) {
          if (pleader()) ++pf5;
          const bool tk = !C_valid || scG <= C_b;
          uint32_t link = hG;
          const int n_gapo = e_go + (open ? 1 : 0), n_gape = e_ge + (open ? 0 : 1);
          uint4 last = make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            if (vg & (1u << j)) {
              const uint32_t slot = slot_at(t++);
              const uint32_t pk = j == 0 ? k : cxk((uint32_t)j - 1u);
              const uint32_t pl = j == 0 ? l : cxl((uint32_t)j - 1u);
              const int pi = j == 0 ? ni : ni + 1;
              const bool grp = j == 0 && dmask;
              last = E::make(pk, pl, pi, grp ? (int)dmask : pi, link, e_mm, n_gapo, n_gape, a,
                             grp ? STATE_G : j == 0 ? STATE_I : STATE_D);
              *slot_ptr(slot) = last;
              link = slot;
            }
          }
          lds_heads[hidx(scG)] = (H)link;
          group_take(tk, last, link, scG);
          if (scMM == scG) hM = link;
        }
        // ---- mismatch children (bits 5-8 but the match child): bucket scMM
        if (vmm) {
          if (pleader()) ++pf5;
          const bool tk = !C_valid || scMM <= C_b;
          uint32_t link = hM;
          uint4 last = make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int j = 5; j < 9; ++j) {
            if (vmm & (1u << j)) {
              const uint32_t slot = slot_at(t++);
              const uint32_t c = (csym + (uint32_t)j - 4u) & 3u;
              last = E::make(cxk(c), cxl(c), ni, ni, link, e_mm + 1, e_go, e_ge, a, STATE_M);
              *slot_ptr(slot) = last;
              link = slot;
            }
          }
          lds_heads[hidx(scMM)] = (H)link;
          group_take(tk, last, link, scMM);
        }
        // ---- the match child (bucket sc_base <= C_b: always the new candidate): kept in C, not
        // stored; C moves to D, the old D is stored if memory lacks it
        if (has_match_ch) {
          const uint32_t slot = slot_at(t++);
          const uint32_t hd = hB;
          const uint4 ne = E::make(cxk(csym), cxl(csym), ni, ldp, hd, e_mm, e_go, e_ge, a, STATE_M);
          lds_heads[hidx(sc_base)] = (H)slot;
          if ((cfl & 6u) == 6u) *slot_ptr(D_slot) = D;
          D = C;
          D_slot = C_slot;
          cfl = (C_valid ? 2u : 0u) | (cfl & 1u) << 2 | 1u;
          C = ne;
          C_slot = slot;
          C_b = sc_base;
          C_valid = true;
        }
        if (t) {
          n_free -= n_fs;
          if (use_fl) {
            fl_head = fl_next;
            fl_known = fl_head == NILH;  // the next head's successor is loaded next iteration
          }
          const uint32_t nb = t - n_fs - fl_n;
          bump = b0 + nb + ((nb && b0 <= skip_at && b0 + nb > skip_at) ? HS : 0u);
          n_entries += (int)t + (vm ? __builtin_popcount(dmask) : 0);  // a group counts all its entries
          if (LW) {
            nonempty.m0 |= (has_match ? 1u << (sc_base & (GAP_RING - 1)) : 0u) |
                           (has_mm ? 1u << (scMM & (GAP_RING - 1)) : 0u) | (has_gap ? 1u << (scG & (GAP_RING - 1)) : 0u);
          } else {
            if (has_match) bm_set(nonempty, sc_base);
            if (has_mm) bm_set(nonempty, scMM);
            if (has_gap) bm_set(nonempty, scG);
          }
        }
      }
      if (pl_) ++pf8;
      if (status) {  // overflow / bad score: the retry pass re-runs the read
        end_stat = status;
        st = 3;
      }
      continue;
    }
  hit : {
    // ---- hit (bwtgap.c:165-197)
    const bool pl_ = pleader();
    if (pl_) ++pf6;
    const int score = e_mm * o.s_mm + e_go * o.s_gapo + e_ge * o.s_gape;
    bool do_add = true;
    if (n_aln == 0) {
      best_score = score;
      int best_diff = e_mm + e_go;
      if (o.mode & MODE_GAPE) best_diff += e_ge;
      if (!(o.mode & MODE_NONSTOP)) max_diff = (best_diff + 1 > opt_max_diff) ? opt_max_diff : best_diff + 1;
    }
    if (score == best_score) {
      best_cnt = (int)((uint32_t)best_cnt + (l - k + 1));
    } else if (best_cnt > o.max_top2) {
      
      end_stat = 0;
      st = 3;
      continue;
    }
    if (e_go) {
      for (int j = 0; j < n_aln; ++j) {
        const uint4 h = ent1[P0 - 1 - j];
        if (h.y == k && h.z == l) { do_add = false; break; }
      }
    }
    if (do_add) {
      if ((uint32_t)n_aln >= HS) {
        end_stat = ST_ALN_OVERFLOW;  // hit area full
        st = 3;
        continue;
      }
      ent1[P0 - 1 - n_aln] = make_uint4((uint32_t)e_mm | (uint32_t)e_go << 8 | (uint32_t)e_ge << 16 | (uint32_t)a << 24,
                                        k, l, (uint32_t)score | (uint32_t)ldp << 16);
      ++n_aln;
      // gap_shadow (bwtgap.c:81-91) on this strand's widths [0, ldp): a sub-state of the lane, 16
      // positions per iteration in the iteration's one round trip (st 5), so the wave does not wait
      // on a chain of width loads while its other lanes could pop; the lane pops again only once
      // every width is updated, as the reference does
      if (ldp > 0) {
        sh_x = l - k + 1;
        sh_prevx = 0;
        sh_q = 0;
        sh_a = a;
        sh_jj = 0;
        sh_ldp = (uint32_t)ldp;
        st = 5;
      }
    }
    
    continue;
  }
  }
  if (PROF && A.prof) {
    const uint64_t v[19] = {pf0, pf1, pf2, pf3, pf4, pf5, pf6, pf7, pf8, pf9, pf10, pl11, pl12, pl13, pl14, pl15, pl16, pl17, pl18};
#pragma unroll
    for (int q = 0; q < 19; ++q)
      if (v[q]) atomicAdd(A.prof + q, (unsigned long long)v[q]);
  }
}

// The search kernels hold 3 waves per SIMD (<= 168 VGPRs; the register allocator otherwise drifts
// a few registers past it); the PROF diagnostics build keeps its own allocation.
template <bool WIDE, bool LW, int NBL = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) k_gapped(GapArgs A, unsigned long long *counter) {
  gapped_body<WIDE, false, LW, NBL>(A, counter);
}
template <bool WIDE, bool LW, int NBL = 0>
__global__ void __launch_bounds__(256) k_gapped_prof(GapArgs A, unsigned long long *counter) {
  gapped_body<WIDE, true, LW, NBL>(A, counter);
}

hipError_t launch_gapped(const GapArgs &g, unsigned long long *d_counter, int blocks, int block, bool wide,
                         hipStream_t st) {
  if (g.n <= 0) return hipSuccess;
  for (int c = 0; c < 5; ++c)  // the kernel takes L2 and seq_len from ix[0] for both strands
    if (g.ix[0].L2[c] != g.ix[1].L2[c]) return hipErrorInvalidValue;
  if (g.ix[0].seq_len != g.ix[1].seq_len) return hipErrorInvalidValue;
  hipError_t e = zero_async(d_counter, sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  const bool lw = !wide && g.cw != nullptr;
  const size_t lds = gapped_lds_bytes(g.o.n_stacks, block, wide, g.max_pages, g.pages_per_block, g.lanes_per_wave,
                                      g.free_depth, lw ? (int)g.cw_words : 0);
  if (wide)
    hipLaunchKernelGGL((k_gapped<true, false>), dim3(blocks), dim3(block), lds, st, g, d_counter);
  else if (lw && g.lanes_per_wave != 64)
    return hipErrorInvalidValue;  // the LW first pass runs 64 reads per wave
  else if (lw && g.prof)
    hipLaunchKernelGGL((k_gapped_prof<false, true>), dim3(blocks), dim3(block), lds, st, g, d_counter);
  else if (lw && block == 256)
    hipLaunchKernelGGL((k_gapped<false, true, 8>), dim3(blocks), dim3(block), lds, st, g, d_counter);
  else if (lw && block == 128)
    hipLaunchKernelGGL((k_gapped<false, true, 7>), dim3(blocks), dim3(block), lds, st, g, d_counter);
  else if (lw && block == 64)
    hipLaunchKernelGGL((k_gapped<false, true, 6>), dim3(blocks), dim3(block), lds, st, g, d_counter);
  else if (lw)
    hipLaunchKernelGGL((k_gapped<false, true>), dim3(blocks), dim3(block), lds, st, g, d_counter);
  else if (g.prof)
    hipLaunchKernelGGL((k_gapped_prof<false, false>), dim3(blocks), dim3(block), lds, st, g, d_counter);
  else
    hipLaunchKernelGGL((k_gapped<false, false>), dim3(blocks), dim3(block), lds, st, g, d_counter);
  return hipGetLastError();
}

}  // namespace ibwa
