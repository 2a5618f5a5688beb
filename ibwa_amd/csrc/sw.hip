// sw.hip -- batched local alignment with path: aln_local_core (stdaln.c:529-760)
// with aln_param_bwa (gap open 26, extend 9, aln_sm_maq, band 50; stdaln.c:206-227)
// and _thres = 1, exactly as bwa_sw_core (bwasw.c:51) calls it per mate rescue,
// followed by aln_global_core (stdaln.c:345-525, gap_end = -1) for the path and
// aln_path2cigar32 (stdaln.c:1010-1040) for the CIGAR.
//
// One alignment per lane, persistent grid with per-wave claiming.  The forward
// pass and the global fill are strip-mined (a strip's columns of the row above in
// registers, one boundary per row through scratch); the reverse pass walks its
// lane-major eh row by aligned 32-word blocks (whole 128 B lines); all three are branch free per cell.
// Scratch that the lanes touch in step (strip boundaries, packed reference codes,
// traceback bytes) is interleaved lane-minor inside each wave, so a wave's access
// is one contiguous segment.  The passes are integer VALU work (roofline: VALU,
// cells/s); the 32000-point rebasing of the reference (stdaln.c:581-598) is
// unreachable because the host rejects min(len1, len2) * 11 > 32000.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "engine.h"

namespace ibwa {

namespace {

constexpr int Q = 26, R = 9, QR = Q + R, BAND = 50, MAXSC = 11;
constexpr int STRIP = 32;  // forward-pass columns held in registers
constexpr int GS = 16;      // global-fill columns held in registers (strip width; 32: 296 VGPRs)
// traceback bytes per row: whole strips, so a strip's junk columns past len1 stay in their row
__host__ __device__ inline uint32_t sw_tb_width(int max_len1) { return (uint32_t)((max_len1 + GS) / GS * GS); }
// the reverse pass walks its eh row by aligned blocks of RB words (16: 64 B, 32: whole 128 B lines)
#ifndef IBWA_SW_RB
#define IBWA_SW_RB 32
#endif
constexpr int RB = IBWA_SW_RB;
static_assert(RB == 16 || RB == 32, "reverse-pass block of 16 or 32 words");
// the reverse pass's eh row per lane: eh[0 .. l1+1] in whole blocks
__host__ __device__ inline uint32_t sw_eh_words(int max_len1) { return (uint32_t)((max_len1 + 2 + RB - 1) / RB * RB); }
constexpr int NEG_INF = -1073741823;  // MINOR_INF (stdaln.h:84)
constexpr int FM = 0, FI = 1, FD = 2;  // FROM_M / FROM_I / FROM_D

// aln_sm_maq score of codes x (row) and y (column): 11 match, -19 mismatch, -13 with an N
__device__ __forceinline__ int sm(uint32_t x, uint32_t y) {
  return (x > 3 || y > 3) ? -13 : (x == y ? 11 : -19);
}

// Per-wave scratch.  What the lanes touch in step with each other (the forward pass's reference
// words and strip boundaries, the global fill's M / I / D rows and traceback bytes: the lanes'
// alignments have the same shape, so a wave's access at one element is one contiguous segment) is
// lane-minor; the reverse pass's eh row, where each lane's adaptive band goes its own way, is
// lane-major, so a lane's consecutive cells share cache lines instead of each touching a line of
// its own (measured: reverse pass 89 -> 25 ms per 200 k rescues; the global fill lane-major was
// 4x slower).
struct Lane {
  uint32_t *w;   // lane-minor words: element e of lane at w[e * 64 + lane]
  uint32_t *wv;  // this lane's lane-major words
  uint8_t *tb;   // this wave's traceback bytes: dword e / 4 of lane at tb[(e / 4 * 64 + lane) * 4]
  int lane;
  __device__ __forceinline__ uint32_t &u(uint32_t e) const { return w[(uint64_t)e * 64 + lane]; }
  __device__ __forceinline__ uint32_t &v(uint32_t e) const { return wv[e]; }
  __device__ __forceinline__ uint4 &v4(uint32_t e4) const { return reinterpret_cast<uint4 *>(wv)[e4]; }
  __device__ __forceinline__ uint8_t &t(uint32_t e) const { return tb[((uint64_t)(e >> 2) * 64 + lane) * 4 + (e & 3)]; }
  __device__ __forceinline__ uint32_t &tw(uint32_t w) const {
    return reinterpret_cast<uint32_t *>(tb)[(uint64_t)w * 64 + lane];
  }
};

// banded global alignment (aln_global_core, stdaln.c:345-525).  gap_end < 0 (the local core's
// path fill): the set_end_* rules are set_*; gap_end >= 0 (bwa_refine_gapped's aln_param_bwa,
// stdaln.c:227): the extension penalty becomes gap_end in the set_end_I / set_end_D cells --
// row 0's deletions, cell 0's insertions, the last cell's insertion of a row clipped at len1,
// and every deletion of the last row (stdaln.c:392-470).
// seq1 = a[0..n1) along i (FROM_D steps i), seq2 = b[0..n2) along j (FROM_I steps j).
// Row j covers lo(j)..hi(j) with lo = 0 while j <= b2 (cell 0 takes an I from above) and j - b2
// after (a -inf boundary cell); the last cell takes an I from above only when the band was
// clipped at len1 (j + b1 - 1 > len1) -- the union of the reference's part 1-3 rows.
//
// Strip-mined like the forward pass: GS columns at a time for every row whose band meets them,
// the strip's M / I / D of the row above in registers, (M, I, D) of the strip's last column per
// row through scratch (eB) for the next strip, the traceback bytes of 4 cells in one dword.  A
// row's cells outside its band compute junk that no in-band cell reads (an in-band cell reads
// (j-1, i-1), (j-1, i) and (j, i-1), all inside row j-1's / row j's written range, except the
// above of an unclipped last cell, which the I rule ignores), and the junk traceback bytes lie
// off every path.  Returns the score; the path is traced into the CIGAR (reversed) and the
// start / end coordinates.
__device__ int global_fill(const Lane &L, uint32_t eB, uint32_t eT, uint32_t t_w, const uint8_t *a, int n1,
                           const uint8_t *b, int n2, int band, int gap_end, uint32_t *cig, int cap, int &n_cig,
                           int &path_len, int &si, int &sj) {
  const int RE = gap_end >= 0 ? gap_end : R;  // extension penalty of the set_end_* cells
  int b1, b2;
  if (n1 > n2) { b1 = n1 - n2 + band; b2 = band; } else { b1 = band; b2 = n2 - n1 + band; }
  if (b1 > n1) b1 = n1;
  if (b2 > n2) b2 = n2;
  auto T = [&](int j, int i) -> uint8_t & { return L.t(eT + (uint32_t)j * t_w + i); };
  // row 0: M(0,0) = 0, D(0,i) = -Q - i*RE for 0 < i < b1 (FROM_M at i = 1, FROM_D after)
  for (int i = 1; i < b1; ++i) T(0, i) = (uint8_t)((i == 1 ? FM : FD) << 4);
  auto row0 = [&](int i, int &m, int &iv, int &d) __attribute__((always_inline)) {
    m = i == 0 ? 0 : NEG_INF;
    iv = NEG_INF;
    d = i == 0 ? NEG_INF : -Q - i * RE;
  };
  int fm = 0, fi = 0, fd = 0;  // M / I / D of (n2, n1)
  for (int i0 = 0; i0 <= n1; i0 += GS) {
    int Mc[GS], Ic[GS], Dc[GS];  // the row above, columns i0 .. i0+GS-1
    uint32_t c6[GS / 4];         // 6 * column code (N: 24), 8 bits each
#pragma unroll
    for (int k = 0; k < GS / 4; ++k) c6[k] = 0;
#pragma unroll
    for (int k = 0; k < GS; ++k) {
      row0(i0 + k, Mc[k], Ic[k], Dc[k]);
      const int i = i0 + k;
      const uint32_t ca = i >= 1 ? a[(i <= n1 ? i : n1) - 1] : 0u;
      c6[k >> 2] |= (ca > 4 ? 24u : ca * 6u) << (8 * (k & 3));
    }
    const bool more = i0 + GS <= n1;  // a strip follows: keep the last column per row
    const int jlo = i0 - b1 + 1 > 1 ? i0 - b1 + 1 : 1;
    const int jhi = i0 + GS - 1 + b2 < n2 ? i0 + GS - 1 + b2 : n2;
    int dgm, dgi, dgd;  // (j-1, i0-1)
    if (i0 == 0) {
      dgm = dgi = dgd = NEG_INF;
    } else if (jlo == 1) {
      row0(i0 - 1, dgm, dgi, dgd);
    } else {
      dgm = (int)L.u(eB + 3 * (jlo - 1));
      dgi = (int)L.u(eB + 3 * (jlo - 1) + 1);
      dgd = (int)L.u(eB + 3 * (jlo - 1) + 2);
    }
    for (int j = jlo; j <= jhi; ++j) {
      const int lo = j <= b2 ? 0 : j - b2;
      const int hi = j + b1 - 1 < n1 ? j + b1 - 1 : n1;
      const bool clipped = j + b1 - 1 > n1;
      const int rd = j == n2 ? RE : R;
      const uint32_t cb = b[j - 1];
      // the row's score profile: 6-bit field 6*ca = sm(cb, ca) + 32
      const uint32_t rp = cb > 3 ? 19u * 0x1041041u : 13u * 0x41041u + (19u << 24) + (30u << (6 * cb));
      int lm = NEG_INF, li = NEG_INF, ld = NEG_INF;  // (j, i0-1)
      if (i0 > 0) {
        lm = (int)L.u(eB + 3 * j);
        li = (int)L.u(eB + 3 * j + 1);
        ld = (int)L.u(eB + 3 * j + 2);
      }
      int dm = dgm, di = dgi, dd = dgd;
      dgm = lm; dgi = li; dgd = ld;
      uint32_t tw = 0;
#pragma unroll
      for (int k = 0; k < GS; ++k) {
        const int i = i0 + k;
        const int um = Mc[k], ui = Ic[k], ud = Dc[k];
        int m, iv, dv;
        uint32_t tt;
        if (k == 0 && i0 == 0) {
          // cell 0: an I from above (set_end_I) while j <= b2; outside the band after
          const int x = um - Q;
          const bool c = x > ui;
          iv = (c ? x : ui) - RE;
          m = dv = NEG_INF;
          tt = (c ? (uint32_t)FM : (uint32_t)FI) << 2;
          if (lo > 0) iv = NEG_INF;
        } else {
          // set_M (stdaln.c:271-287) from the diagonal
          const int sc = (int)__builtin_amdgcn_ubfe(rp, (c6[k >> 2] >> (8 * (k & 3))) & 255u, 6) - 32;
          const bool c1 = dm >= di;
          const int b1v = c1 ? dm : di;
          const bool keep = b1v > dd || (c1 && b1v == dd);
          m = (keep ? b1v : dd) + sc;
          const uint32_t tm = keep ? (c1 ? (uint32_t)FM : (uint32_t)FI) : (uint32_t)FD;
          // set_I from above; the last cell only when the band was clipped at len1 (set_end_I)
          const bool inner = i < hi;
          const int x = um - Q;
          const bool ci = x > ui;
          iv = (ci ? x : ui) - (inner ? R : RE);
          uint32_t ti = ci ? (uint32_t)FM : (uint32_t)FI;
          if (!(inner || clipped)) {
            iv = NEG_INF;
            ti = FM;
          }
          // set_D from the left (set_end_D on the last row)
          const int y = lm - Q;
          const bool cd = y > ld;
          dv = (cd ? y : ld) - rd;
          const uint32_t td = cd ? (uint32_t)FM : (uint32_t)FD;
          tt = tm | ti << 2 | td << 4;
          if (i == lo) m = iv = dv = NEG_INF;  // the -inf boundary cell of a row past b2
        }
        tw |= tt << (8 * (k & 3));
        if ((k & 3) == 3) {
          L.tw((eT + (uint32_t)j * t_w + (uint32_t)(i - 3)) >> 2) = tw;
          tw = 0;
        }
        Mc[k] = m; Ic[k] = iv; Dc[k] = dv;
        lm = m; li = iv; ld = dv;
        dm = um; di = ui; dd = ud;
      }
      if (more) {
        L.u(eB + 3 * j) = (uint32_t)lm;
        L.u(eB + 3 * j + 1) = (uint32_t)li;
        L.u(eB + 3 * j + 2) = (uint32_t)ld;
      }
    }
    if (!more) {  // the strip of column n1; its last row was n2
#pragma unroll
      for (int k = 0; k < GS; ++k)
        if (i0 + k == n1) { fm = Mc[k]; fi = Ic[k]; fd = Dc[k]; }
    }
  }
  // traceback from (n1, n2) (stdaln.c:487-514); ops emitted end -> start, run-length encoded
  int best = fm, ctype = FM;
  uint8_t cell = T(n2, n1);
  int type = cell & 3;
  if (fi > best) { best = fi; type = (cell >> 2) & 3; ctype = FI; }
  if (fd > best) { best = fd; type = (cell >> 4) & 3; ctype = FD; }
  int i = n1, j = n2, n = 0;
  n_cig = 0;
  auto emit = [&](int op) {
    if (n_cig > 0 && (int)(cig[n_cig - 1] & 0xf) == op) cig[n_cig - 1] += 1u << 4;
    else if (n_cig < cap) cig[n_cig++] = 1u << 4 | (uint32_t)op;
  };
  int pi = i, pj = j;  // cell of the latest counted path entry
  emit(ctype);
  n = 1;
  for (;;) {
    if (ctype == FM) { --i; --j; } else if (ctype == FI) --j; else --i;
    ctype = type;
    if (i == 0 && j == 0) break;  // the (0,0) entry is not part of path_len
    if (i < 0 || j < 0) break;    // memory guard: a valid traceback never leaves the matrix
    cell = T(j, i);
    type = ctype == FM ? (cell & 3) : ctype == FI ? ((cell >> 2) & 3) : ((cell >> 4) & 3);
    emit(ctype);
    ++n;
    pi = i;
    pj = j;
  }
  path_len = n;
  si = pi;
  sj = pj;
  return best;
}

// One strip of the forward pass (stdaln.c:600-631): columns i0 .. i0+STRIP-1 for every row, the
// strip's H / E of the row above in registers, (H[j][i0-1], F) per row from / to scratch.  Branch
// free: sm() comes from a per-column profile (6-bit field 6*cb = sm(cb, column code) + 32), the
// F / E rules are selects, and the first maximum is found per row as the largest (h << 5 | 31-k)
// (the leftmost cell of the row's largest h), then compared with the running (score, j, i) in
// the reference's row-major order.  PART: the last strip is narrower than STRIP (its extra
// columns compute junk that nothing reads, and they are kept out of the maximum).
template <bool PART>
__device__ __forceinline__ void fwd_strip(const Lane &L, uint32_t eREF, uint32_t eBH, uint32_t eBF,
                                          const uint8_t *b, int n1, int n2, int i0, int &score_f, int &end_i,
                                          int &end_j) {
  const int wcols = n1 - i0 + 1;
  int Hc[STRIP], Ec[STRIP];  // H[j-1][i], E[j-1][i] of the strip's columns
  uint32_t cp[STRIP];        // column profiles
  uint32_t rc[STRIP / 8];
#pragma unroll
  for (int k = 0; k < STRIP / 8; ++k) rc[k] = L.u(eREF + (uint32_t)(i0 - 1) / 8 + k);
#pragma unroll
  for (int k = 0; k < STRIP; ++k) {
    const uint32_t ca = (rc[k >> 3] >> (4 * (k & 7))) & 15u;
    // fields cb = 0..3: 13 (mismatch) or 43 (match), field 4 (N): 19; an N column: 19 everywhere
    cp[k] = ca > 3 ? 19u * 0x1041041u : 13u * 0x41041u + (19u << 24) + (30u << (6 * ca));
    Hc[k] = Ec[k] = 0;
  }
  int diag_next = 0;  // H[j-1][i0-1]
  // the next row's read code and strip boundary are loaded one row ahead (row j+1's boundary
  // words are written by the previous strip; this strip writes row j's at the end of row j)
  uint32_t cb_n = b[0];
  int bh_n = 0, bf_n = 0;
  if (i0 > 1) {
    bh_n = (int)L.u(eBH + 1);
    bf_n = (int)L.u(eBF + 1);
  }
  for (int j = 1; j <= n2; ++j) {
    const uint32_t cb = cb_n > 4 ? 24u : cb_n * 6u;
    int last_h = bh_n, f = bf_n;  // H[j][i0-1] and the row's F state, from the previous strip
    if (j < n2) {
      cb_n = b[j];
      if (i0 > 1) {
        bh_n = (int)L.u(eBH + j + 1);
        bf_n = (int)L.u(eBF + j + 1);
      }
    }
    int diag = diag_next;
    diag_next = last_h;
    uint32_t rk = 0;
#pragma unroll
    for (int k = 0; k < STRIP; ++k) {
      const int above = Hc[k], e_old = Ec[k];
      const int hd = diag + (int)__builtin_amdgcn_ubfe(cp[k], cb, 6) - 32;
      const int fn = max(f - R, last_h - QR);
      const bool lp = last_h > 0;
      f = lp ? fn : f;
      const int fm = lp ? fn : 0;
      const int e = above > QR ? max(e_old - R, above - QR) : 0;
      const int h = max(max(hd, fm), e);  // >= 0: e is
      Ec[k] = e;
      Hc[k] = h;
      diag = above;
      last_h = h;
      uint32_t key = (uint32_t)h << 5 | (uint32_t)(31 - k);
      if (PART && k >= wcols) key = 0;
      rk = max(rk, key);
    }
    if (!PART && i0 + STRIP <= n1) {  // boundary for the next strip
      L.u(eBH + j) = (uint32_t)last_h;
      L.u(eBF + j) = (uint32_t)f;
    }
    const int rh = (int)(rk >> 5), ri = i0 + 31 - (int)(rk & 31);
    if (rh > score_f || (rh == score_f && rh > 0 && (j < end_j || (j == end_j && ri < end_i)))) {
      score_f = rh;
      end_i = ri;
      end_j = j;
    }
  }
}

}  // namespace

__global__ void __launch_bounds__(256) k_sw(SwArgs A, unsigned long long *counter) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  // lane-minor elements: ref4[(l1+31)/32*4], the forward pass's strip boundaries H / F per row, the
  // global fill's (M, I, D) per row; lane-major: eh[0..l1+1] (sw_words_per_lane in total)
  const uint32_t eREF = 0, eBH = eREF + (A.max_len1 + 31) / 32 * 4, eBF = eBH + A.max_len2 + 1;
  const uint32_t eB = eBF + A.max_len2 + 1;  // the global fill's (M, I, D) per row at a strip's end
  const uint32_t nminor = eB + 3 * (A.max_len2 + 1);
  const uint32_t t_w = sw_tb_width(A.max_len1);
  const uint32_t eEH = 0, nmajor = sw_eh_words(A.max_len1);
  Lane L;
  L.w = A.scratch + wave * A.words_per_lane * 64;
  L.wv = L.w + (uint64_t)nminor * 64 + (uint64_t)lane * nmajor;
  L.tb = A.tb + wave * A.tb_per_lane * 64;
  L.lane = lane;
  int64_t cur = 0, cend = 0;
  for (;;) {
    // one pair per lane, claimed per wave
    if (cur >= cend) {
      int64_t base = 0;
      if (lane == 0) base = (int64_t)atomicAdd(counter, 64ull);
      base = __shfl(base, 0);
      if (base >= A.n) break;
      cur = base;
      cend = base + 64 < A.n ? base + 64 : A.n;
    }
    const int64_t p = cur + lane;
    cur = cend;
    if (p >= cend) continue;
    const int n1 = (int)A.len1[p], n2 = (int)A.len2[p];
    const uint8_t *a = A.seq1 + A.off1[p];
    const uint8_t *b = A.seq2 + A.off2[p];
    uint32_t *cig = A.cigar + (uint64_t)p * A.cigar_cap;
    int score = -1, path_len = 0, n_cig = 0, s_i = 0, s_j = 0, e_i = 0, e_j = 0;
    if (A.global_band > 0) {
      // aln_global_core alone (bwa_refine_gapped, bwase.c:198): whole sequences, one band
      score = 0;
      if (n1 > 0 && n2 > 0) {
        int si = 0, sj = 0;
        score = global_fill(L, eB, 0, t_w, a, n1, b, n2, A.global_band, A.gap_end, cig,
                            A.cigar_cap, n_cig, path_len, si, sj);
        for (int k = 0; k < n_cig / 2; ++k) {
          const uint32_t t = cig[k];
          cig[k] = cig[n_cig - 1 - k];
          cig[n_cig - 1 - k] = t;
        }
        s_i = si; s_j = sj; e_i = n1; e_j = n2;
      }
    } else if (n1 > 0 && n2 > 0) {
      // ---- forward pass (stdaln.c:579-631): row j over seq2, columns i over seq1.
      // Strip-mined: STRIP columns at a time for all rows, the strip's H / E of the row
      // above in registers; between strips only (H[j][i0-1], F) per row goes through
      // scratch (fwd_strip).
      for (int w = 0; w < (n1 + 31) / 32 * 4; ++w) {
        uint32_t x = 0;
        for (int k = 0; k < 8 && w * 8 + k < n1; ++k) x |= (uint32_t)a[w * 8 + k] << (4 * k);
        L.u(eREF + w) = x;
      }
      int score_f = 0, end_i = 0, end_j = 0;
      for (int i0 = 1; i0 <= n1; i0 += STRIP) {
        if (n1 - i0 + 1 >= STRIP)
          fwd_strip<false>(L, eREF, eBH, eBF, b, n1, n2, i0, score_f, end_i, end_j);
        else
          fwd_strip<true>(L, eREF, eBH, eBF, b, n1, n2, i0, score_f, end_i, end_j);
      }
      score = score_f;
      if (score_f >= 1 && end_i > 0 && end_j > 0 && A.stop_after != 1) {
        // ---- reverse pass (stdaln.c:639-696) in the adaptive band
        // eh[0 .. end_i] = 0 by 16 B stores (up to 3 words past end_i as well: whole blocks of the
        // row, never read by a cell -- a cell i <= start < end_i reads eh[i] and eh[i + 1] only)
        for (int q = 0; q <= end_i / 4; ++q) L.v4((uint32_t)q) = make_uint4(0u, 0u, 0u, 0u);
        int score_r = sm(a[end_i - 1], b[end_j - 1]);
        int start_i = end_i, start_j = end_j;
        L.v(eEH + end_i) = (uint32_t)(QR + score_r) << 16;
        int start = end_i - 1, end = end_i - 3;
        if (end <= 0) end = 0;
        for (int j = end_j - 1; j != 0; --j) {
          const uint32_t cb = b[j - 1];
          // the row's score profile: 6-bit field 6*ca = sm(cb, ca) + 32
          const uint32_t rp = cb > 3 ? 19u * 0x1041041u : 13u * 0x41041u + (19u << 24) + (30u << (6 * cb));
          int last_h = 0, f = 0, i = start;
          bool found = false;
          int nxt = (int)L.v(eEH + i + 1);  // eh[i+1] of the row below (old value)
          // cells start, start-1, ..., end+1 (start > end >= 0 always) by aligned RB-word blocks of
          // the eh row: block q = eh[RB q .. RB q + RB-1] is loaded (RB / 4 x 16 B) before its cells
          // are updated (a cell writes eh[i+1] only, and cells go down, so every loaded value is
          // still the row below's) and stored back whole: cells outside [end+1, i], or after the
          // start was found, keep their word; cell RB q + RB-1 writes the next block's first word.
          // The block's reference codes are packed words of the forward pass's eREF (8 per word:
          // cell RB q + m reads a[RB q + m - 1]).
          constexpr int RW = RB / 8;  // eREF words per block
          while (i > end && !found) {
            const int q = i / RB;
            int blk[RB];
#pragma unroll
            for (int x = 0; x < RB / 4; ++x) {
              const uint4 v = L.v4((uint32_t)q * (RB / 4) + x);
              blk[4 * x] = (int)v.x; blk[4 * x + 1] = (int)v.y; blk[4 * x + 2] = (int)v.z; blk[4 * x + 3] = (int)v.w;
            }
            const uint32_t r0 = q > 0 ? L.u(eREF + RW * q - 1) : 0u;
            uint32_t rw[RW];
#pragma unroll
            for (int x = 0; x < RW; ++x) rw[x] = L.u(eREF + RW * q + x);
            uint32_t out[RB];
            out[0] = (uint32_t)blk[0];
            uint32_t top = 0;
            bool top_act = false;
            int ii = i;
#pragma unroll
            for (int m = RB - 1; m >= 0; --m) {
              const int ik = RB * q + m;
              const bool act = ik <= i && ik > end && !found;
              const int nx = m == RB - 1 ? nxt : blk[m + 1];
              const uint32_t code = m == 0 ? r0 >> 28 : (rw[(m - 1) >> 3] >> (4 * ((m - 1) & 7))) & 15u;
              const uint32_t ca = (code < 4u ? code : 4u) * 6u;
              const int hd = (nx >> 16) + (int)__builtin_amdgcn_ubfe(rp, ca, 6) - 32;
              const int fn = max(f - R, last_h - QR);
              const bool lp = last_h > 0;
              const int fc = lp ? fn : f, fm = lp ? fn : 0;
              const int above = blk[m] >> 16, e_old = nx & 0xffff;
              const int e = max(max(e_old - R, above - QR), 0);
              const int h = max(max(hd, fm), e);  // >= 0: e is
              const uint32_t val = (uint32_t)last_h << 16 | (uint32_t)e;
              if (m < RB - 1) {
                out[m + 1] = act ? val : (uint32_t)blk[m + 1];
              } else {
                top = val;
                top_act = act;
              }
              const bool upd = act && score_r < h;
              if (act) {
                f = fc;
                last_h = h;
              }
              if (upd) {
                score_r = h;
                start_i = ik;
                start_j = j;
              }
              found = found || (upd && h - QR == score_f);  // the start: stop here (j = 1; break)
              if (act && !found) ii = ik - 1;
            }
#pragma unroll
            for (int x = 0; x < RB / 4; ++x)
              L.v4((uint32_t)q * (RB / 4) + x) = make_uint4(out[4 * x], out[4 * x + 1], out[4 * x + 2], out[4 * x + 3]);
            if (top_act) L.v(eEH + (uint32_t)(RB * q + RB)) = top;
            nxt = blk[0];
            i = ii;
          }
          if (found) j = 1;
          L.v(eEH + i + 1) = (uint32_t)last_h << 16;
          if (((int)L.v(eEH + start) >> 16) <= QR) --start;
          if (start <= 0) start = 0;
          end = start_i - (start_j - j) - (score_r + (start_j - j) * MAXSC) / R - 1;
          if (end <= 0) end = 0;
        }
        score_r -= QR;
        if (A.stop_after == 2) goto done;
        // ---- path by banded global alignment, band doubling from 50 (stdaln.c:723-745)
        const int span = ((end_i - start_i > end_j - start_j) ? end_i - start_i : end_j - start_j) + 1;
        const int n1s = end_i - start_i + 1, n2s = end_j - start_j + 1;
        int score_g = 0, si = 0, sj = 0;
        for (int bw = BAND;; bw <<= 1) {
          score_g = global_fill(L, eB, 0, t_w, a + start_i - 1, n1s, b + start_j - 1, n2s,
                                bw, -1, cig, A.cigar_cap, n_cig, path_len, si, sj);
          if (score_g == score_r || score_f == score_g) break;
          if (bw > span) break;
        }
        score = (score_r > score_g && score_f > score_g) ? -1 : score_g;
        // reverse the CIGAR (traced end -> start) and convert the coordinates
        for (int k = 0; k < n_cig / 2; ++k) {
          const uint32_t t = cig[k];
          cig[k] = cig[n_cig - 1 - k];
          cig[n_cig - 1 - k] = t;
        }
        s_i = si + start_i - 1; s_j = sj + start_j - 1;
        e_i = n1s + start_i - 1; e_j = n2s + start_j - 1;
      }
    }
  done:
    A.score[p] = score;
    A.path_len[p] = path_len;
    A.n_cigar[p] = n_cig;
    A.ends[p] = make_int4(s_i, s_j, e_i, e_j);
  }
}

__global__ void __launch_bounds__(256) k_pack_cigar(const uint32_t *cig, int cap, const int32_t *n_cigar,
                                                    const uint64_t *first, int64_t n, uint32_t *out) {
  // one lane per CIGAR word slot of a row: a wave reads a row's words as one segment
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * 64; t += stride) {
    const int64_t p = t >> 6;
    const int w = (int)(t & 63);
    const int m = n_cigar[p];
    for (int x = w; x < m; x += 64) out[first[p] + x] = cig[(uint64_t)p * cap + x];
  }
}

hipError_t launch_pack_cigar(const uint32_t *cig, int cap, const int32_t *n_cigar, const uint64_t *first, int64_t n,
                             uint32_t *out, hipStream_t st) {
  const int64_t lanes = n * 64;
  const int blocks = (int)std::min<int64_t>((lanes + 255) / 256, 16384);
  hipLaunchKernelGGL(k_pack_cigar, dim3(blocks), dim3(256), 0, st, cig, cap, n_cigar, first, n, out);
  return hipGetLastError();
}

hipError_t launch_sw(const SwArgs &a, unsigned long long *d_counter, int blocks, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  hipError_t e = zero_async(d_counter, sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_sw, dim3(blocks), dim3(256), 0, st, a, d_counter);
  return hipGetLastError();
}

uint64_t sw_words_per_lane(int max_len1, int max_len2) {
  return (uint64_t)sw_eh_words(max_len1) + (uint64_t)(max_len1 + 31) / 32 * 4 + 5ull * (uint64_t)(max_len2 + 1);
}

uint64_t sw_tb_per_lane(int max_len1, int max_len2) {
  return (uint64_t)sw_tb_width(max_len1) * (uint64_t)(max_len2 + 1);
}

}  // namespace ibwa
