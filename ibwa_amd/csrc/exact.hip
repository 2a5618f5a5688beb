// exact.hip -- the exact-match path of `aln -n 0` (max_diff == 0).
//
// Why this path exists and is exact: with max_diff == 0 the search of
// bwtgap.c:104-264 never expands an entry.  The two root entries (strand 1
// popped first, LIFO) have m == 0, so each is either pruned by
// `m < width[len-1].bid` (:155) or resolved by bwt_match_exact_alt
// (:160-163).  width[len-1].bid == 0 exactly when the read occurs in the text
// -- the condition under which the exact search succeeds -- so the width
// pass (bwtaln.c:123-130) decides nothing the exact search does not, and
// gap_shadow is a no-op (last_diff_pos == 0).  Any N makes nN > max_diff
// (:116-122).  Hence: hits = [strand 1 exact, strand 0 exact] (each if
// found), each {0,0,0,a,k,l,score 0} -- verified bit-exact against the
// reference goldens and the CPU restatement (tests/).
//
// Two kernels:
//   k_pack_reads : streaming pre-pass, one read per lane: 2-bit codes, N flag,
//                  the two K-mer table indices and the first symbol word.
//   k_exact      : persistent; one read per lane, both strands advanced in
//                  lockstep; every loop iteration is exactly one memory round
//                  trip for every lane (rank queries, table lookups, the next
//                  16-symbol word and new read headers are all issued before
//                  the single wait), lanes refilled from a per-wave chunk.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "engine.h"
#include "occ.h"

namespace ibwa {

namespace {

constexpr int MODE_COMPREAD = 0x02;
constexpr int EXACT_CHUNK = 512;

// Record of read r at rec + r * stride (uint4 units):
//   [0] = {len | hasN << 16, kmer index strand 1, kmer index strand 0, first symbol word}
//   [1..] = 2-bit codes of bwa_seq_t.seq, 16 per dword, position p at bits 2*(p&15) of dword p>>4
// `first symbol word` is the dword holding position len-1-K (table used) or len-1.
// Pack one read: its bytes from `src` (16 B chunks, `mis` bytes before the read in the first chunk),
// the record to `R` (header) and `W` (2-bit words).  Called with LDS or global pointers.
__device__ __forceinline__ void pack_one(const uint4 *src, int mis, int L, int K, int comp, uint4 *R, uint32_t *W) {
  const bool use_tab = K > 0 && L >= K;
  const int p0 = use_tab ? L - 1 - K : L - 1;
  uint32_t nN = 0, xa = 0, xb = 0, w = 0, first = 0;
  const int nq = (mis + L + 15) >> 4;
  for (int q = 0; q < nq; ++q) {
    const uint4 v = src[q];
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const uint32_t word = b < 4 ? v.x : b < 8 ? v.y : b < 12 ? v.z : v.w;
      const uint32_t c = (word >> (8 * (b & 3))) & 0xffu;
      const int j = q * 16 + b - mis;
      if (j >= 0 && j < L) {
        nN += c > 3;
        const uint32_t c2 = c & 3;
        xa = (xa << 2) | (comp ? c2 ^ 3u : c2);
        xb = (xb << 2) | c2;
        w |= c2 << (2 * (j & 15));
        if ((j & 15) == 15 || j == L - 1) {
          W[j >> 4] = w;
          if (p0 >= 0 && (p0 >> 4) == (j >> 4)) first = w;
          w = 0;
        }
      }
    }
  }
  const uint32_t kmask = K >= 16 ? 0xFFFFFFFFu : ((1u << (2 * K)) - 1u);
  R[0] = make_uint4((uint32_t)L | (nN ? 1u << 16 : 0u), use_tab ? xa & kmask : 0u, use_tab ? xb & kmask : 0u, first);
}

// One wave packs 64 consecutive reads.  When their bytes form one span of at most `in_cap` bytes
// (reads staged back to back), the wave loads the span into LDS with coalesced 16 B loads, packs
// from LDS into an LDS copy of its 64 records, and stores those as one contiguous block -- the
// per-lane layout (lane i at byte 100 i) would otherwise make every load and store instruction
// touch 64 separate lines.  Other waves read and write per lane.
__global__ void __launch_bounds__(256) k_pack_reads(const uint8_t *__restrict__ seq, const uint64_t *__restrict__ off,
                                                    const uint32_t *__restrict__ len, int64_t n, uint4 *__restrict__ rec,
                                                    uint32_t stride, int K, int comp, uint32_t in_cap) {
  extern __shared__ uint4 lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * 64;
  const int nw = r0 >= n ? 0 : (int)(n - r0 < 64 ? n - r0 : 64);
  uint4 *in = lds + (size_t)wave * (in_cap / 16 + 64 * stride);
  uint4 *out = in + in_cap / 16;
  const int64_t r = r0 + lane;
  const bool act = lane < nw;
  const uint64_t o_r = act ? off[r] : 0;
  const int L = act ? (int)len[r] : 0;
  uint64_t start = 0, span = 0;
  bool fits = false;
  if (nw > 0) {
    start = off[r0] & ~(uint64_t)15;
    const uint64_t last = off[r0 + nw - 1] + len[r0 + nw - 1];
    span = ((last + 15) & ~(uint64_t)15) - start;
    const bool inside = !act || (o_r >= start && o_r + (uint64_t)L <= start + span);
    fits = span <= in_cap && __all(inside);
  }
  if (fits) {
    const uint4 *g = reinterpret_cast<const uint4 *>(seq + start);
    for (uint32_t c = lane; c < span / 16; c += 64) in[c] = g[c];
  }
  __syncthreads();
  if (act) {
    if (fits) {
      const uint64_t o = o_r - start;
      pack_one(in + (o >> 4), (int)(o & 15), L, K, comp, out + (size_t)lane * stride,
               reinterpret_cast<uint32_t *>(out + (size_t)lane * stride + 1));
    } else {
      // 16 B loads from the aligned-down start (the staging buffer has 16 B of tail padding)
      const uint8_t *sp = seq + o_r;
      const uint4 *q0 = reinterpret_cast<const uint4 *>(reinterpret_cast<uintptr_t>(sp) & ~(uintptr_t)15);
      uint4 *R = rec + (uint64_t)r * stride;
      pack_one(q0, (int)(reinterpret_cast<uintptr_t>(sp) & 15), L, K, comp, R, reinterpret_cast<uint32_t *>(R + 1));
    }
  }
  __syncthreads();
  if (fits) {
    uint4 *dst = rec + (uint64_t)r0 * stride;
    for (uint32_t c = lane; c < (uint32_t)nw * stride; c += 64) dst[c] = out[c];
  }
}

// bit-plane rank query (occ64.hip): {C[c], 0, P_lo[c], P_hi[c]} of the 64-row block of `row`
__device__ __forceinline__ uint4 load64(const uint4 *o, uint32_t row, uint32_t c, bool run) {
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (run) v = o[(size_t)(row >> 6) * 4 + c];
  return v;
}

__device__ __forceinline__ uint32_t occ64(const uint4 &v, uint32_t row) {
  const uint32_t o = row & 63;
  const uint32_t mlo = o >= 31 ? 0xFFFFFFFFu : ((2u << o) - 1u);
  const uint32_t mhi = o < 32 ? 0u : (o == 63 ? 0xFFFFFFFFu : ((2u << (o - 32)) - 1u));
  return v.x + (uint32_t)__builtin_popcount(v.z & mlo) + (uint32_t)__builtin_popcount(v.w & mhi);
}

// bwt_2occ + the interval update of bwt_match_exact_alt (bwt.c:243-245);
// `vk` is the k-1 end's block, or a copy of `vl` when both ends share it
__device__ __forceinline__ void extend64(const IndexView &ix, uint32_t &k, uint32_t &l, uint32_t c, const uint4 &vk,
                                         const uint4 &vl) {
  const uint32_t ok = k == 0 ? 0u : occ64(vk, k - 1);
  const uint32_t ol = occ64(vl, l);
  const uint32_t base = l2of(ix, c);
  k = base + ok + 1;
  l = base + ol;
}

__device__ __forceinline__ bool share_block(uint32_t k, uint32_t l) { return k != 0 && ((k - 1) >> 6) == (l >> 6); }

// Do the next min(32, left) read symbols (2-bit words rw0|rw1, positions t..t+31; complemented
// for strand 1 under COMPREAD) equal the text at positions tpos.. (words tw0..tw2 from tpos >> 4)?
__device__ __forceinline__ bool jump_cmp(uint32_t tw0, uint32_t tw1, uint32_t tw2, uint32_t rw0, uint32_t rw1,
                                         uint32_t tpos, int left, bool complement) {
  const uint32_t sh = 2 * (tpos & 15);
  const uint64_t lo = (uint64_t)tw1 << 32 | tw0;
  const uint64_t x = sh ? (lo >> sh) | ((uint64_t)tw2 << (64 - sh)) : lo;
  uint64_t rd = (uint64_t)rw1 << 32 | rw0;
  if (complement) rd = ~rd;
  const uint64_t mask = left >= 32 ? ~0ull : ((1ull << (2 * left)) - 1ull);
  return ((x ^ rd) & mask) == 0;
}

__global__ void __launch_bounds__(256) k_exact(ExactArgs A, const uint4 *__restrict__ rec, uint32_t stride,
                                               unsigned long long *counter) {
  const int lane = threadIdx.x & 63;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  const bool comp = A.mode & MODE_COMPREAD;
  const IndexView ix0 = A.ix[0], ix1 = A.ix[1];
  const int K = A.K;
  int64_t cur = 0, cend = 0;  // wave-uniform chunk cursor
  bool more = true;
  // lane state: 0 idle, 1 header requested, 2 running
  int st = 0;
  int64_t r = 0;
  int len = 0, p = 0;         // p: next position (both strands advance together)
  uint32_t ka = 0, la = 0, kb = 0, lb = 0, ia = 0, ib = 0, bw = 0;
  bool ra = false, rb = false, fa = false, fb = false, lk = false;
  // unique-interval jump per strand: 1 = SA[k] wanted, 2 = comparing the read's remaining
  // m symbols with the text before q = SA[k], 32 per iteration (t: compared so far)
  int ja = 0, jb = 0, ma = 0, mb = 0, tca = 0, tcb = 0;
  uint32_t qa = 0, qb = 0, isa_a = 0, isa_b = 0;
  for (;;) {
    // ---- claim reads for idle lanes (no memory traffic unless the chunk runs out)
    unsigned long long need = __ballot(st == 0);
    while (need && more) {
      if (cur >= cend) {
        int64_t base = 0;
        if (lane == 0) base = (int64_t)atomicAdd(counter, (unsigned long long)EXACT_CHUNK);
        base = __shfl(base, 0);
        if (base >= A.n) { more = false; break; }
        cur = base;
        cend = base + EXACT_CHUNK < A.n ? base + EXACT_CHUNK : A.n;
      }
      const int rank = __popcll(need & lt_mask);
      const int64_t avail = cend - cur;
      if (st == 0 && rank < avail) {
        r = cur + rank;
        st = 1;
      }
      const int64_t cnt = __popcll(need);
      cur += avail < cnt ? avail : cnt;
      need = __ballot(st == 0);
    }
    if (__ballot(st != 0) == 0ull) break;

    // ---- issue every load of this step
    const bool hdr = st == 1;
    const bool run = st == 2;
    const bool look_a = run && lk && ra, look_b = run && lk && rb;
    const bool step_a = run && !lk && ra && p >= 0, step_b = run && !lk && rb && p >= 0;
    const uint32_t c = (bw >> (2 * (p & 15))) & 3;  // symbol of seq at p (valid when running and !lk)
    const uint32_t ca = comp ? c ^ 3u : c, cb = c;
    uint4 h = make_uint4(0, 0, 0, 0);
    if (hdr) h = rec[(uint64_t)r * stride];
    uint2 ta = make_uint2(0, 0), tb = make_uint2(0, 0);
    if (look_a) ta = A.kt0[ia];
    if (look_b) tb = A.kt1[ib];
    const bool sha = share_block(ka, la), shb = share_block(kb, lb);
    const uint4 val = load64(A.o64[0], la, ca, step_a);
    const uint4 vbl = load64(A.o64[1], lb, cb, step_b);
    uint4 vak = load64(A.o64[0], ka - 1, ca, step_a && ka != 0 && !sha);
    uint4 vbk = load64(A.o64[1], kb - 1, cb, step_b && kb != 0 && !shb);
    // next symbol word: crossing into a new 16-symbol word on the next step
    uint32_t nbw = 0;
    const uint32_t *recw = reinterpret_cast<const uint32_t *>(rec + (uint64_t)r * stride + 1);
    const bool need_word = run && !lk && (ra || rb) && (p & 15) == 0 && p > 0;
    if (need_word) nbw = recw[(p - 1) >> 4];
    // jump loads: SA[k]; or 3 text words + 2 read words (+ ISA[q - m] on the first compare)
    uint32_t sa_ld_a = 0, sa_ld_b = 0, isa_ld_a = 0, isa_ld_b = 0;
    uint32_t twa0 = 0, twa1 = 0, twa2 = 0, rwa0 = 0, rwa1 = 0, twb0 = 0, twb1 = 0, twb2 = 0, rwb0 = 0, rwb1 = 0;
    if (run && ja == 1) sa_ld_a = A.sa[0][ka];
    if (run && jb == 1) sa_ld_b = A.sa[1][kb];
    if (run && ja == 2) {
      const uint32_t w = (qa - (uint32_t)ma + (uint32_t)tca) >> 4;
      twa0 = A.txt[0][w]; twa1 = A.txt[0][w + 1]; twa2 = A.txt[0][w + 2];
      rwa0 = recw[tca >> 4];
      if (((tca >> 4) + 1) * 16 < ma) rwa1 = recw[(tca >> 4) + 1];
      if (tca == 0) isa_ld_a = A.isa[0][qa - (uint32_t)ma];
    }
    if (run && jb == 2) {
      const uint32_t w = (qb - (uint32_t)mb + (uint32_t)tcb) >> 4;
      twb0 = A.txt[1][w]; twb1 = A.txt[1][w + 1]; twb2 = A.txt[1][w + 2];
      rwb0 = recw[tcb >> 4];
      if (((tcb >> 4) + 1) * 16 < mb) rwb1 = recw[(tcb >> 4) + 1];
      if (tcb == 0) isa_ld_b = A.isa[1][qb - (uint32_t)mb];
    }

    // ---- consume
    if (hdr) {
      len = (int)(h.x & 0xFFFF);
      const bool hasN = (h.x >> 16) & 1;
      ia = h.y;
      ib = h.z;
      bw = h.w;
      ka = kb = 0;
      la = ix0.seq_len;
      lb = ix1.seq_len;
      p = len - 1;
      fa = fb = hasN;  // nN > max_diff (= 0): no hit
      ra = rb = !hasN && len > 0;
      lk = ra && K > 0 && len >= K;
      st = 2;
    } else if (run) {
      // jumps in flight
      if (ja == 1) {
        qa = sa_ld_a;
        if (qa < (uint32_t)ma) { fa = true; ja = 0; } else { ja = 2; tca = 0; }
      } else if (ja == 2) {
        if (tca == 0) isa_a = isa_ld_a;
        if (jump_cmp(twa0, twa1, twa2, rwa0, rwa1, qa - (uint32_t)ma + (uint32_t)tca, ma - tca, comp)) {
          tca += 32;
          if (tca >= ma) { ka = la = isa_a; ja = 0; }
        } else {
          fa = true;
          ja = 0;
        }
      }
      if (jb == 1) {
        qb = sa_ld_b;
        if (qb < (uint32_t)mb) { fb = true; jb = 0; } else { jb = 2; tcb = 0; }
      } else if (jb == 2) {
        if (tcb == 0) isa_b = isa_ld_b;
        if (jump_cmp(twb0, twb1, twb2, rwb0, rwb1, qb - (uint32_t)mb + (uint32_t)tcb, mb - tcb, false)) {
          tcb += 32;
          if (tcb >= mb) { kb = lb = isa_b; jb = 0; }
        } else {
          fb = true;
          jb = 0;
        }
      }
      if (lk) {
        if (look_a) { ka = ta.x; la = ta.y; if (ka > la) { ra = false; fa = true; } }
        if (look_b) { kb = tb.x; lb = tb.y; if (kb > lb) { rb = false; fb = true; } }
        p -= K;
        lk = false;
      } else {
        if (step_a) {
          if (sha) vak = val;
          extend64(ix0, ka, la, ca, vak, val);
          if (ka > la) { ra = false; fa = true; }
        }
        if (step_b) {
          if (shb) vbk = vbl;
          extend64(ix1, kb, lb, cb, vbk, vbl);
          if (kb > lb) { rb = false; fb = true; }
        }
        if (need_word) bw = nbw;
        if (step_a || step_b) --p;
      }
      // a chain whose interval became one row jumps over its remaining p + 1 symbols:
      // stepping from row k succeeds exactly while the text before SA[k] spells them
      if (A.jump && !lk && p >= 0) {
        if (ra && ka == la) { ra = false; ja = 1; ma = p + 1; }
        if (rb && kb == lb) { rb = false; jb = 1; mb = p + 1; }
      }
    }
    if (st == 2 && ja == 0 && jb == 0 && (p < 0 || (!ra && !rb))) {
      // both chains finished: a chain that did not fail consumed every symbol
      uint4 *out = A.aln + (uint64_t)r * A.aln_cap;
      int nh = 0;
      if (!fa) out[nh++] = make_uint4(1u << 24, ka, la, 0u);
      if (!fb) out[nh++] = make_uint4(0u, kb, lb, 0u);
      A.n_aln[r] = nh;
      A.status[r] = 0;
      st = 0;
    }
  }
}

}  // namespace

uint32_t exact_record_stride(int max_len) {  // in uint4 units
  return 1u + (uint32_t)((max_len + 63) / 64);
}

hipError_t launch_exact(const AlnArgs &a, const uint4 *o64_0, const uint4 *o64_1, const uint2 *kt0,
                        const uint2 *kt1, int K, uint4 *rec, uint32_t stride, unsigned long long *d_counter,
                        int blocks, hipEvent_t ev_mid, const uint32_t *const jump[6], hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  const int comp = (a.o.mode & MODE_COMPREAD) ? 1 : 0;
  // LDS per wave: the span of 64 back-to-back reads of the batch's longest length, and 64 records
  uint32_t in_cap = (uint32_t)(((uint64_t)64 * std::max<uint32_t>(a.wlen1 - 1, 1) + 32 + 15) & ~15ull);
  if ((size_t)4 * (in_cap + 64 * stride * 16) > 64 * 1024) in_cap = 0;  // long reads: per-lane loads
  const size_t lds = (size_t)4 * (in_cap + 64 * stride * 16);
  hipLaunchKernelGGL(k_pack_reads, dim3((unsigned)((a.n + 255) / 256)), dim3(256), lds, st, a.seq, a.off, a.len, a.n,
                     rec, stride, K, comp, in_cap);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = zero_async(d_counter, sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  if (ev_mid && (e = hipEventRecord(ev_mid, st)) != hipSuccess) return e;  // pack | search boundary
  ExactArgs x;
  x.ix[0] = a.ix[0];
  x.ix[1] = a.ix[1];
  x.seq = a.seq;
  x.off = a.off;
  x.len = a.len;
  x.n = a.n;
  x.aln = a.aln;
  x.n_aln = a.n_aln;
  x.status = a.status;
  x.aln_cap = a.aln_cap;
  x.mode = a.o.mode;
  x.kt0 = kt0;
  x.kt1 = kt1;
  x.K = K;
  x.o64[0] = o64_0;
  x.o64[1] = o64_1;
  x.jump = jump != nullptr;
  for (int s = 0; s < 2; ++s) {
    x.sa[s] = jump ? jump[s] : nullptr;
    x.isa[s] = jump ? jump[2 + s] : nullptr;
    x.txt[s] = jump ? jump[4 + s] : nullptr;
  }
  hipLaunchKernelGGL(k_exact, dim3(blocks), dim3(256), 0, st, x, rec, stride, d_counter);
  return hipGetLastError();
}

}  // namespace ibwa
