// sw.hip -- batched local alignment with path: aln_local_core (stdaln.c:529-760)
// with aln_param_bwa (gap open 26, extend 9, aln_sm_maq, band 50; stdaln.c:206-227)
// and _thres = 1, exactly as bwa_sw_core (bwasw.c:51) calls it per mate rescue,
// followed by aln_global_core (stdaln.c:345-525, gap_end = -1) for the path and
// aln_path2cigar32 (stdaln.c:1010-1040) for the CIGAR.
//
// One alignment per lane, persistent grid with per-wave claiming.  The DP
// vectors (packed h<<16|e of the local passes, the M/I/D rows of the global
// fill) and the traceback bytes live in per-lane HBM/L2 scratch interleaved
// lane-minor inside each wave, so a wave's accesses at the same column are
// one contiguous 256 B (or 64 B) segment; the reference window is re-packed 8
// codes per word so the forward pass loads one word per 8 cells.  The local
// passes are integer VALU work (roofline: VALU, cells/s); the 32000-point
// rebasing of the reference (stdaln.c:581-598) is unreachable because the
// host rejects min(len1, len2) * 11 > 32000.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine.h"

namespace ibwa {

namespace {

constexpr int Q = 26, R = 9, QR = Q + R, BAND = 50, MAXSC = 11;
constexpr int STRIP = 32;  // forward-pass columns held in registers
constexpr int RCHUNK = 16;  // reverse-pass cells whose loads are issued together
constexpr int GCH = 8;      // global-fill cells whose loads are issued together
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
  uint8_t *tb;   // this wave's traceback bytes, element e at tb[e * 64 + lane]
  int lane;
  __device__ __forceinline__ uint32_t &u(uint32_t e) const { return w[(uint64_t)e * 64 + lane]; }
  __device__ __forceinline__ uint32_t &v(uint32_t e) const { return wv[e]; }
  __device__ __forceinline__ uint8_t &t(uint32_t e) const { return tb[(uint64_t)e * 64 + lane]; }
};

// banded global alignment (aln_global_core, stdaln.c:345-525).  gap_end < 0 (the local core's
// path fill): the set_end_* rules are set_*; gap_end >= 0 (bwa_refine_gapped's aln_param_bwa,
// stdaln.c:227): the extension penalty becomes gap_end in the set_end_I / set_end_D cells --
// row 0's deletions, cell 0's insertions, the last cell's insertion of a row clipped at len1,
// and every deletion of the last row (stdaln.c:392-470).
// seq1 = a[0..n1) along i (FROM_D steps i), seq2 = b[0..n2) along j (FROM_I steps j).
// Rows are written generically: row j covers lo(j)..hi(j) with lo = 0 while j <= b2 (cell 0 takes
// an I from above) and j - b2 after (a -inf boundary cell); the last cell takes an I from above only
// when the band was clipped at len1 (j + b1 - 1 > len1) -- the union of the reference's part 1-3 rows.
// Returns the score; the path is traced into the CIGAR (reversed) and start/end coordinates.
__device__ int global_fill(const Lane &L, uint32_t eM, uint32_t eI, uint32_t eD, uint32_t eT, uint32_t t_w,
                           const uint8_t *a, int n1, const uint8_t *b, int n2, int band, int gap_end, uint32_t *cig,
                           int cap, int &n_cig, int &path_len, int &si, int &sj) {
  const int RE = gap_end >= 0 ? gap_end : R;  // extension penalty of the set_end_* cells
  int b1, b2;
  if (n1 > n2) { b1 = n1 - n2 + band; b2 = band; } else { b1 = band; b2 = n2 - n1 + band; }
  if (b1 > n1) b1 = n1;
  if (b2 > n2) b2 = n2;
  // two rows of {M, I, D} at eM/eI/eD + parity * (n1 + 1)
  auto M = [&](int par, int i) -> uint32_t & { return L.u(eM + par * (n1 + 1) + i); };
  auto I = [&](int par, int i) -> uint32_t & { return L.u(eI + par * (n1 + 1) + i); };
  auto D = [&](int par, int i) -> uint32_t & { return L.u(eD + par * (n1 + 1) + i); };
  auto T = [&](int j, int i) -> uint8_t & { return L.t(eT + (uint32_t)j * t_w + i); };
  // row 0
  M(0, 0) = 0;
  I(0, 0) = (uint32_t)NEG_INF;
  D(0, 0) = (uint32_t)NEG_INF;
  {
    int pm = 0, pd = NEG_INF;
    for (int i = 1; i < b1; ++i) {
      int d;
      uint8_t tt;
      if (pm - Q > pd) { d = pm - Q - RE; tt = FM; } else { d = pd - RE; tt = FD; }
      M(0, i) = (uint32_t)NEG_INF;
      I(0, i) = (uint32_t)NEG_INF;
      D(0, i) = (uint32_t)d;
      T(0, i) = (uint8_t)(tt << 4);
      pm = NEG_INF;
      pd = d;
    }
  }
  for (int j = 1; j <= n2; ++j) {
    const int cur = j & 1, prv = cur ^ 1;
    const int lo = j <= b2 ? 0 : j - b2;
    const int hi = j + b1 - 1 < n1 ? j + b1 - 1 : n1;
    const uint32_t cb = b[j - 1];
    int lm, li, ld;  // left cell (j, i-1)
    if (j <= b2) {
      const int um = (int)M(prv, 0), ui = (int)I(prv, 0);
      uint8_t tt;
      int iv;
      if (um - Q > ui) { iv = um - Q - RE; tt = FM; } else { iv = ui - RE; tt = FI; }
      M(cur, 0) = (uint32_t)NEG_INF;
      I(cur, 0) = (uint32_t)iv;
      D(cur, 0) = (uint32_t)NEG_INF;
      T(j, 0) = (uint8_t)(tt << 2);
      lm = NEG_INF; li = iv; ld = NEG_INF;
    } else {
      M(cur, lo) = I(cur, lo) = D(cur, lo) = (uint32_t)NEG_INF;
      lm = li = ld = NEG_INF;
    }
    // diagonal cell (j-1, i-1) starts at column lo
    int dm = (int)M(prv, lo), di = (int)I(prv, lo), dd = (int)D(prv, lo);
    // GCH cells at a time: the row above's values and the codes of the chunk are loaded together
    // before its cells are computed and stored (a cell stores into row `cur` only)
    for (int i0 = lo + 1; i0 <= hi; i0 += GCH) {
      int um_[GCH], ui_[GCH], ud_[GCH];
      uint32_t ca_[GCH];
#pragma unroll
      for (int q = 0; q < GCH; ++q) {
        const int i = i0 + q <= hi ? i0 + q : hi;
        um_[q] = (int)M(prv, i);
        ui_[q] = (int)I(prv, i);
        ud_[q] = (int)D(prv, i);
        ca_[q] = a[i - 1];
      }
#pragma unroll
      for (int q = 0; q < GCH; ++q) {
        const int i = i0 + q;
        if (i > hi) break;
        const int sc = sm(cb, ca_[q]);
        int m, iv, dv;
        uint8_t tm, ti, td;
        // set_M (stdaln.c:271-287)
        if (dm >= di) {
          if (dm >= dd) { m = dm + sc; tm = FM; } else { m = dd + sc; tm = FD; }
        } else {
          if (di > dd) { m = di + sc; tm = FI; } else { m = dd + sc; tm = FD; }
        }
        // above cell (j-1, i)
        const int um = um_[q], ui = ui_[q], ud = ud_[q];
        // set_I from above; the last cell only when the band was clipped at len1 (set_end_I)
        if (i < hi || j + b1 - 1 > n1) {
          const int ri = i < hi ? R : RE;
          if (um - Q > ui) { iv = um - Q - ri; ti = FM; } else { iv = ui - ri; ti = FI; }
        } else {
          iv = NEG_INF;
          ti = FM;
        }
        // set_D from the left (set_end_D on the last row)
        const int rd = j == n2 ? RE : R;
        if (lm - Q > ld) { dv = lm - Q - rd; td = FM; } else { dv = ld - rd; td = FD; }
        M(cur, i) = (uint32_t)m;
        I(cur, i) = (uint32_t)iv;
        D(cur, i) = (uint32_t)dv;
        T(j, i) = (uint8_t)(tm | ti << 2 | td << 4);
        lm = m; li = iv; ld = dv;
        dm = um; di = ui; dd = ud;
      }
    }
    (void)li;
  }
  // traceback from (n1, n2) (stdaln.c:487-514); ops emitted end -> start, run-length encoded
  const int par = n2 & 1;
  int best = (int)M(par, n1), ctype = FM;
  uint8_t cell = T(n2, n1);
  int type = cell & 3;
  if ((int)I(par, n1) > best) { best = (int)I(par, n1); type = (cell >> 2) & 3; ctype = FI; }
  if ((int)D(par, n1) > best) { best = (int)D(par, n1); type = (cell >> 4) & 3; ctype = FD; }
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
  for (int j = 1; j <= n2; ++j) {
    uint32_t cb = b[j - 1];
    cb = cb > 4 ? 24u : cb * 6u;
    int last_h = 0, f = 0;  // H[j][i0-1] and the row's F state, from the previous strip
    if (i0 > 1) {
      last_h = (int)L.u(eBH + j);
      f = (int)L.u(eBF + j);
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
  // lane-minor elements: ref4[(l1+31)/32*4], the strip boundaries H / F per row, two rows each of
  // M / I / D for the global fill; lane-major: eh[0..l1+1] (sw_words_per_lane in total)
  const uint32_t eREF = 0, eBH = eREF + (A.max_len1 + 31) / 32 * 4, eBF = eBH + A.max_len2 + 1;
  const uint32_t eM = eBF + A.max_len2 + 1, eI = eM + 2 * (A.max_len1 + 1), eD = eI + 2 * (A.max_len1 + 1);
  const uint32_t nminor = eD + 2 * (A.max_len1 + 1);
  const uint32_t eEH = 0, nmajor = A.max_len1 + 2;
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
        score = global_fill(L, eM, eI, eD, 0, (uint32_t)A.max_len1 + 1, a, n1, b, n2, A.global_band, A.gap_end, cig,
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
        for (int i = 0; i <= end_i; ++i) L.v(eEH + i) = 0;
        int score_r = sm(a[end_i - 1], b[end_j - 1]);
        int start_i = end_i, start_j = end_j;
        L.v(eEH + end_i) = (uint32_t)(QR + score_r) << 16;
        int start = end_i - 1, end = end_i - 3;
        if (end <= 0) end = 0;
        for (int j = end_j - 1; j != 0; --j) {
          const uint32_t cb = b[j - 1];
          int last_h = 0, f = 0, i = start;
          bool found = false;
          int nxt = (int)L.v(eEH + i + 1);  // eh[i+1] of the row below (old value)
          // cells start, start-1, ..., end+1 (start > end always), RCHUNK at a time: the
          // chunk's old eh values and codes are loaded together before its cells are updated
          // (a cell writes eh[i+1] only, so all loaded values are still the row below's)
          while (i != end && i > 0 && !found) {  // i > 0: memory guard, never binding
            int ab[RCHUNK];
            uint32_t cd[RCHUNK];
#pragma unroll
            for (int k = 0; k < RCHUNK; ++k) {
              const int ik = i - k;
              const bool ok = ik > end && ik > 0;
              ab[k] = ok ? (int)L.v(eEH + ik) : 0;
              cd[k] = ok ? a[ik - 1] : 0u;
            }
#pragma unroll
            for (int k = 0; k < RCHUNK; ++k) {
              if (i != end && i > 0 && !found) {
                int h = (nxt >> 16) + sm(cb, cd[k]);
                if (h < 0) h = 0;
                if (last_h > 0) {
                  f = (f > last_h - Q) ? f - R : last_h - QR;
                  if (h < f) h = f;
                }
                const int above = ab[k] >> 16, e_old = nxt & 0xffff;
                int e = (e_old > above - Q) ? e_old - R : above - QR;
                if (e < 0) e = 0;
                if (h < e) h = e;
                L.v(eEH + i + 1) = (uint32_t)last_h << 16 | (uint32_t)e;
                last_h = h;
                if (score_r < h) {
                  score_r = h; start_i = i; start_j = j;
                  if (score_r - QR == score_f) found = true;  // the start: stop here (j = 1; break)
                }
                if (!found) {
                  nxt = ab[k];
                  --i;
                }
              }
            }
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
          score_g = global_fill(L, eM, eI, eD, 0, (uint32_t)A.max_len1 + 1, a + start_i - 1, n1s, b + start_j - 1, n2s,
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

hipError_t launch_sw(const SwArgs &a, unsigned long long *d_counter, int blocks, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(d_counter, 0, sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_sw, dim3(blocks), dim3(256), 0, st, a, d_counter);
  return hipGetLastError();
}

uint64_t sw_words_per_lane(int max_len1, int max_len2) {
  return (uint64_t)(max_len1 + 2) + (uint64_t)(max_len1 + 31) / 32 * 4 + 6ull * (uint64_t)(max_len1 + 1) +
         2ull * (uint64_t)(max_len2 + 1);
}

uint64_t sw_tb_per_lane(int max_len1, int max_len2) {
  return (uint64_t)(max_len1 + 1) * (uint64_t)(max_len2 + 1);
}

}  // namespace ibwa
