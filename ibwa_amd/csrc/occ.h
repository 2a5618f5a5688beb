// occ.h -- FM-index rank queries on the MI355X HBM layout.
//
// The reference interleaves, per 128 BWT symbols, 4 cumulative counts and
// 8 words of 2-bit symbols: 48 B blocks (bwt.h:34,56-63; bwtmisc.c:122-144),
// so a random rank query straddles 64 B sectors and then popcounts up to
// 4 words per symbol (bwt.c:90-214).  Here every 128-symbol interval is one
// 64 B-aligned block, so one rank query = one 64 B HBM sector:
//
//   u32[0..3]   C[c]   occurrences of c in BWT'[0, 128b)   ($ removed, as the reference)
//   u32[4..11]  128 symbols, 2 bits each, MSB-first, 16 per word (same order as bwt.h:56)
//   u32[12..14] sub[j] byte c = occurrences of c in block symbols [0, 32(j+1))
//   u32[15]     0
//
// Occ(c,k) then needs C[c] + one sub-count byte + popcounts over at most one
// 32-symbol chunk (two words).  Semantics are exactly bwt_occ / bwt_occ4 /
// bwt_2occ / bwt_2occ4 (bwt.c:90-214), including k == (u32)-1 -> 0 and the
// `k >= primary -> k-1` removal of $; k == seq_len yields the total count,
// which is what bwt_occ's early return (bwt.c:95) returns.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ibwa {

struct IndexView {
  const uint4 *blk;  // 4 x uint4 per 128-symbol block
  uint32_t primary;
  uint32_t seq_len;
  uint32_t L2[5];
};

// L2[c] by selects: a dynamic index into the kernel-argument array would go through scratch
__device__ __forceinline__ uint32_t l2of(const IndexView &ix, uint32_t c) {
  return c == 0 ? ix.L2[0] : c == 1 ? ix.L2[1] : c == 2 ? ix.L2[2] : ix.L2[3];
}

__device__ __forceinline__ uint32_t bwt_kk(const IndexView &ix, uint32_t k) {
  return k >= ix.primary ? k - 1 : k;  // bwt.c:97
}

// masks keeping bases 0..r (inclusive) of the 32-base chunk held in (w0,w1)
__device__ __forceinline__ void chunk_masks(uint32_t r, uint32_t &m0, uint32_t &m1) {
  m0 = r >= 15 ? 0xFFFFFFFFu : (0xFFFFFFFFu << (2 * (15 - r)));
  m1 = r < 16 ? 0u : (0xFFFFFFFFu << (2 * (31 - r)));
}

// count of symbol c in the masked words
__device__ __forceinline__ uint32_t count1(uint32_t w0, uint32_t w1, uint32_t m0, uint32_t m1, uint32_t c) {
  const uint32_t pat = c * 0x55555555u;
  uint32_t x0 = w0 ^ pat, x1 = w1 ^ pat;
  uint32_t z0 = ~(x0 | (x0 >> 1)) & 0x55555555u & m0;
  uint32_t z1 = ~(x1 | (x1 >> 1)) & 0x55555555u & m1;
  return __builtin_popcount(z0) + __builtin_popcount(z1);
}

// counts of all four symbols in the masked words
__device__ __forceinline__ void count4(uint32_t w0, uint32_t w1, uint32_t m0, uint32_t m1, uint32_t n[4]) {
  uint32_t h0 = (w0 >> 1) & 0x55555555u & m0, l0 = w0 & 0x55555555u & m0;
  uint32_t h1 = (w1 >> 1) & 0x55555555u & m1, l1 = w1 & 0x55555555u & m1;
  uint32_t n3 = __builtin_popcount(h0 & l0) + __builtin_popcount(h1 & l1);
  uint32_t n2 = __builtin_popcount(h0 & ~l0) + __builtin_popcount(h1 & ~l1);
  uint32_t n1 = __builtin_popcount(l0 & ~h0) + __builtin_popcount(l1 & ~h1);
  uint32_t tot = __builtin_popcount(m0 & 0x55555555u) + __builtin_popcount(m1 & 0x55555555u);
  n[0] = tot - n1 - n2 - n3; n[1] = n1; n[2] = n2; n[3] = n3;
}

// words (w0,w1) of chunk q from the bases uint4s
__device__ __forceinline__ void chunk_words(const uint4 &b, uint32_t q, uint32_t &w0, uint32_t &w1) {
  // bases uint4 #1 holds words 4..7 (chunks 0,1); uint4 #2 holds words 8..11 (chunks 2,3)
  if (q & 1) { w0 = b.z; w1 = b.w; } else { w0 = b.x; w1 = b.y; }
}

__device__ __forceinline__ uint32_t sub_byte(const uint4 &s, uint32_t q, uint32_t c) {
  uint32_t v = q == 1 ? s.x : q == 2 ? s.y : s.z;
  return q == 0 ? 0u : (v >> (8 * c)) & 0xFFu;
}

__device__ __forceinline__ uint32_t sel4(const uint4 &v, uint32_t c) {
  return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}

// Occ(c, k) -- bwt_occ (bwt.c:90-113) for k in [-1, seq_len]
__device__ __forceinline__ uint32_t occ1(const IndexView &ix, uint32_t k, uint32_t c) {
  if (k == 0xFFFFFFFFu) return 0;
  uint32_t kk = bwt_kk(ix, k);
  const uint4 *p = ix.blk + (size_t)(kk >> 7) * 4;
  uint32_t off = kk & 127, q = off >> 5, r = off & 31;
  uint4 cnt = p[0], bs = p[1 + (q >> 1)], sb = p[3];
  uint32_t w0, w1, m0, m1;
  chunk_words(bs, q, w0, w1);
  chunk_masks(r, m0, m1);
  return sel4(cnt, c) + sub_byte(sb, q, c) + count1(w0, w1, m0, m1, c);
}

// bwt_2occ (bwt.c:116-151): Occ(c,k) and Occ(c,l), sharing the block when possible
__device__ __forceinline__ void occ2(const IndexView &ix, uint32_t k, uint32_t l, uint32_t c,
                                     uint32_t &ok, uint32_t &ol) {
  uint32_t kk = k == 0xFFFFFFFFu ? 0xFFFFFFFFu : bwt_kk(ix, k);
  uint32_t ll = bwt_kk(ix, l);
  if (k == 0xFFFFFFFFu || (kk >> 7) != (ll >> 7)) {
    ok = occ1(ix, k, c);
    ol = occ1(ix, l, c);
    return;
  }
  const uint4 *p = ix.blk + (size_t)(kk >> 7) * 4;
  uint32_t offk = kk & 127, qk = offk >> 5, offl = ll & 127, ql = offl >> 5;
  uint4 cnt = p[0], sb = p[3];
  uint4 bk = p[1 + (qk >> 1)];
  uint4 bl = ((qk >> 1) == (ql >> 1)) ? bk : p[1 + (ql >> 1)];
  uint32_t base = sel4(cnt, c), w0, w1, m0, m1;
  chunk_words(bk, qk, w0, w1);
  chunk_masks(offk & 31, m0, m1);
  ok = base + sub_byte(sb, qk, c) + count1(w0, w1, m0, m1, c);
  chunk_words(bl, ql, w0, w1);
  chunk_masks(offl & 31, m0, m1);
  ol = base + sub_byte(sb, ql, c) + count1(w0, w1, m0, m1, c);
}

__device__ __forceinline__ void occ4_from(const uint4 &cnt, const uint4 &bs, const uint4 &sb, uint32_t off,
                                          uint32_t o[4]) {
  uint32_t q = off >> 5, w0, w1, m0, m1, n[4];
  chunk_words(bs, q, w0, w1);
  chunk_masks(off & 31, m0, m1);
  count4(w0, w1, m0, m1, n);
  o[0] = cnt.x + sub_byte(sb, q, 0) + n[0];
  o[1] = cnt.y + sub_byte(sb, q, 1) + n[1];
  o[2] = cnt.z + sub_byte(sb, q, 2) + n[2];
  o[3] = cnt.w + sub_byte(sb, q, 3) + n[3];
}

// bwt_occ4 (bwt.c:157-174)
__device__ __forceinline__ void occ4(const IndexView &ix, uint32_t k, uint32_t o[4]) {
  if (k == 0xFFFFFFFFu) { o[0] = o[1] = o[2] = o[3] = 0; return; }
  uint32_t kk = bwt_kk(ix, k);
  const uint4 *p = ix.blk + (size_t)(kk >> 7) * 4;
  uint32_t off = kk & 127;
  occ4_from(p[0], p[1 + ((off >> 5) >> 1)], p[3], off, o);
}

// bwt_2occ4 (bwt.c:177-214)
__device__ __forceinline__ void occ4x2(const IndexView &ix, uint32_t k, uint32_t l, uint32_t ck[4],
                                       uint32_t cl[4]) {
  uint32_t kk = k == 0xFFFFFFFFu ? 0xFFFFFFFFu : bwt_kk(ix, k);
  uint32_t ll = bwt_kk(ix, l);
  if (k == 0xFFFFFFFFu || (kk >> 7) != (ll >> 7)) {
    occ4(ix, k, ck);
    occ4(ix, l, cl);
    return;
  }
  const uint4 *p = ix.blk + (size_t)(kk >> 7) * 4;
  uint32_t offk = kk & 127, offl = ll & 127;
  uint4 cnt = p[0], sb = p[3];
  uint4 bk = p[1 + (offk >> 6)];
  uint4 bl = ((offk >> 6) == (offl >> 6)) ? bk : p[1 + (offl >> 6)];
  occ4_from(cnt, bk, sb, offk, ck);
  occ4_from(cnt, bl, sb, offl, cl);
}

}  // namespace ibwa
