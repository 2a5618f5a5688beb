// sa2pos.hip -- SA row -> text coordinate for a batch of hits:
// bwt_sa (bwt.c:69-79) inside bwtdb_sa2seq (dbset.c:240-246), as samse
// (bwase.c:133, :146, :157) and sampe (bwape.c:347, :400; saiset.c:136, :147)
// call it once per reported hit.
//
//   strand 1: pos = offset + bwt_sa(bwt[0], k)
//   strand 0: pos = offset + bwt[1].seq_len - (u32)(bwt_sa(bwt[1], k) + len)   (u64: wraps past 2^64
//             when the hit hangs off the end, as the reference's uint64_t expression does)
//
// bwt_sa walks the LF mapping bwt_invPsi (bwt.h:66-70) until the row is a
// multiple of the SA sampling interval and adds the walk length to the sampled
// value (sa[0] = (u32)-1, bwtio.c:45).  Two device forms, same results:
//
//   * full SA resident (intv == 1; the index builder keeps it when HBM allows,
//     or ibwa_ctx_expand_sa derives it): one 4 B gather per hit;
//   * sampled SA: the walk, one hit per lane.  Each step is one random 64 B
//     block of the occ.h layout (symbol word, block counts and sub-counts of
//     the same 128-row block), so the kernel is bound by random 64 B requests
//     like the aln kernels.  Lanes that finish take the next hit of their
//     grid-stride sequence at once, so a wave is not held by its longest walk
//     (walk lengths are geometric, mean ~intv, tail ~10 intv).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "engine.h"
#include "occ.h"

namespace ibwa {

namespace {

// symbol stored at position p of the $-removed BWT and Occ(c, k) from the same block
__device__ __forceinline__ uint32_t inv_psi(const IndexView &ix, uint32_t k) {
  if (k == ix.primary) return 0;                      // bwt.h:67
  const uint32_t p = k < ix.primary ? k : k - 1;      // bwt_B0(k) / bwt_B0(k - 1), bwt.h:68-70
  const uint4 *b = ix.blk + (size_t)(p >> 7) * 4;
  const uint32_t off = p & 127, q = off >> 5;
  const uint4 cnt = b[0], bs = b[1 + (q >> 1)], sb = b[3];
  uint32_t w0, w1, m0, m1;
  chunk_words(bs, q, w0, w1);
  const uint32_t r = off & 31;
  const uint32_t c = ((r < 16 ? w0 : w1) >> (2 * (15 - (r & 15)))) & 3u;
  chunk_masks(r, m0, m1);
  // bwt_occ(k, c) counts stored positions [0, p] (bwt.c:97 removes $)
  return l2of(ix, c) + sel4(cnt, c) + sub_byte(sb, q, c) + count1(w0, w1, m0, m1, c);
}

__device__ __forceinline__ uint64_t to_pos(const SaArgs &a, uint32_t strand, uint32_t sa, uint32_t len) {
  // dbset.c:241-245: (u64 offset + u32 seq_len) - u32 (sa + len), evaluated in u64
  return strand ? a.offset + sa : a.offset + a.ix[1].seq_len - (uint32_t)(sa + len);
}

__global__ void __launch_bounds__(256) k_sa2pos_full(SaArgs a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const uint32_t s = a.strand[i], k = a.k[i];
    const int x = s ? 0 : 1;  // strand 1 -> bwt[0], strand 0 -> bwt[1]
    const uint32_t v = k == 0 ? 0xFFFFFFFFu : a.sa[x][k];  // row 0 is sampled: sa[0] = -1
    a.pos[i] = to_pos(a, s, v, a.len[i]);
    if (a.steps) a.steps[i] = 0;
  }
}

__global__ void __launch_bounds__(256) k_sa2pos_walk(SaArgs a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  uint32_t s = a.strand[i], k = a.k[i], steps = 0;
  for (;;) {
    const int x = s ? 0 : 1;
    const uint32_t intv = a.intv[x];
    if (k % intv == 0) {  // bwt.c:72 loop condition failed: a sampled row
      const uint32_t v = steps + (k == 0 ? 0xFFFFFFFFu : a.sa[x][k / intv]);
      a.pos[i] = to_pos(a, s, v, a.len[i]);
      if (a.steps) a.steps[i] = steps;
      i += stride;
      if (i >= a.n) break;
      s = a.strand[i];
      k = a.k[i];
      steps = 0;
      continue;
    }
    ++steps;
    k = inv_psi(a.ix[x], k);
  }
}

// Full SA from the sampled one: the LF walk started at every sampled row visits the rows whose
// suffixes lie between that row's suffix and the previous sampled suffix in text order, and each
// row but row 0 is visited by exactly one walk.  A walk from sampled row k0 with value v gives the
// j-th row it visits the value v - j -- which is bwt_sa's result for that row, since bwt_sa walks
// the same chain down to the next sampled row (the walk from row 0 starts from seq_len, the true
// suffix, not the -1 the sampled array stores there).  Total work: seq_len steps.
__global__ void __launch_bounds__(256) k_expand_sa(IndexView ix, const uint32_t *__restrict__ sa_s, uint32_t intv,
                                                   uint64_t n_sa, uint32_t *__restrict__ full) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_sa; j += stride) {
    uint32_t k = (uint32_t)(j * intv);
    uint32_t v = j == 0 ? ix.seq_len : sa_s[j];
    full[k] = j == 0 ? 0xFFFFFFFFu : v;
    for (;;) {
      k = inv_psi(ix, k);
      --v;
      if (k % intv == 0) break;
      full[k] = v;
    }
  }
}

// ---- the unique-interval jump's SA / ISA / text for an index that arrives as .bwt files only
// (bwt_restore_bwt, bwtaln.c:184-189: `aln` never loads .sa or .pac).  Everything follows from
// the LF cycle: row 0 (suffix "$") -> seq_len - 1 -> ... -> primary (suffix 0) -> row 0.

// symbol of BWT row k (k != primary): the stored position bwt_kk(k) of the $-removed BWT
__device__ __forceinline__ uint32_t bwt_sym(const IndexView &ix, uint32_t k) {
  const uint32_t p = k < ix.primary ? k : k - 1;
  const uint4 *b = ix.blk + (size_t)(p >> 7) * 4;
  const uint32_t off = p & 127, q = off >> 5;
  uint32_t w0, w1;
  chunk_words(b[1 + (q >> 1)], q, w0, w1);
  const uint32_t r = off & 31;
  return ((r < 16 ? w0 : w1) >> (2 * (15 - (r & 15)))) & 3u;
}

// 1. marked rows j * intv: walk LF from each to the next marked row -> link and distance
__global__ void __launch_bounds__(256) k_sa_link(IndexView ix, uint32_t intv, uint64_t n_nodes,
                                                 uint32_t *__restrict__ next, uint32_t *__restrict__ dist) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_nodes; j += stride) {
    uint32_t k = (uint32_t)(j * intv), d = 0;
    do {
      k = inv_psi(ix, k);
      ++d;
    } while (k % intv);
    next[j] = k / intv;
    dist[j] = d;
  }
}

// 2. list ranking by pointer jumping (node 0 = row 0 is the sink): after the last round
//    rank[j] = LF steps from row j * intv to row 0 = SA[j * intv] + 1
__global__ void __launch_bounds__(256) k_sa_jump(uint64_t n_nodes, const uint32_t *__restrict__ nx,
                                                 const uint32_t *__restrict__ rk, uint32_t *__restrict__ nx2,
                                                 uint32_t *__restrict__ rk2, uint32_t *__restrict__ active) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t any = 0;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_nodes; j += stride) {
    const uint32_t a = nx[j];
    if (a != 0) {
      rk2[j] = rk[j] + rk[a];
      nx2[j] = nx[a];
      any |= nx[a] != 0;
    } else {
      rk2[j] = rk[j];
      nx2[j] = 0;
    }
  }
  if (__ballot(any) && (threadIdx.x & 63) == 0) atomicOr(active, 1u);
}

__global__ void __launch_bounds__(256) k_sa_sample(uint64_t n_nodes, const uint32_t *__restrict__ rk,
                                                   uint32_t *__restrict__ sa_s) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_nodes; j += stride)
    sa_s[j] = j == 0 ? 0xFFFFFFFFu : rk[j] - 1;  // bwtio.c:45 stores sa[0] = -1
}

// 3. ISA over text positions [0, seq_len] from the full SA (full[0] is the stored -1: row 0 is
//    the suffix at seq_len)
__global__ void __launch_bounds__(256) k_isa_from_sa(const uint32_t *__restrict__ full, uint64_t n_rows,
                                                     uint32_t seq_len, uint32_t *__restrict__ isa) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_rows; r += stride)
    isa[r == 0 ? seq_len : full[r]] = (uint32_t)r;
}

// 4. the 2-bit text (sa_build.hip's k_pack_text2 layout): T[p] is the BWT symbol of the row of
//    suffix p + 1
__global__ void __launch_bounds__(256) k_text_from_isa(IndexView ix, const uint32_t *__restrict__ isa,
                                                       uint64_t n_words, uint32_t *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t n = ix.seq_len;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_words; w += stride) {
    uint32_t x = 0;
    for (int k = 0; k < 16; ++k) {
      const uint64_t t = w * 16 + k;
      if (t < n) x |= bwt_sym(ix, isa[t + 1]) << (2 * k);
    }
    out[w] = x;
  }
}

}  // namespace

hipError_t derive_sampled_sa(const IndexView &ix, uint32_t intv, uint32_t *sa_s, uint32_t *tmp, hipStream_t st) {
  const uint64_t n_nodes = ((uint64_t)ix.seq_len + intv) / intv;  // rows 0 .. seq_len
  uint32_t *nx = tmp, *rk = tmp + n_nodes, *nx2 = tmp + 2 * n_nodes, *rk2 = tmp + 3 * n_nodes;
  uint32_t *active = tmp + 4 * n_nodes;
  const unsigned g = (unsigned)std::min<uint64_t>((n_nodes + 255) / 256, 65536);
  hipLaunchKernelGGL(k_sa_link, dim3(g), dim3(256), 0, st, ix, intv, n_nodes, nx, rk);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // sink: node 0
  e = zero_async(nx, 4, st);
  if (e == hipSuccess) e = zero_async(rk, 4, st);
  bool done = false;
  for (int round = 0; e == hipSuccess && !done && round < 40; ++round) {
    e = zero_async(active, 4, st);
    if (e != hipSuccess) break;
    hipLaunchKernelGGL(k_sa_jump, dim3(g), dim3(256), 0, st, n_nodes, nx, rk, nx2, rk2, active);
    e = hipGetLastError();
    std::swap(nx, nx2);
    std::swap(rk, rk2);
    uint32_t more = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&more, active, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    done = more == 0;
  }
  if (e != hipSuccess) return e;
  if (!done) return hipErrorUnknown;  // more than 2^40 nodes: cannot happen for a 32-bit index
  hipLaunchKernelGGL(k_sa_sample, dim3(g), dim3(256), 0, st, n_nodes, rk, sa_s);
  return hipGetLastError();
}

hipError_t derive_isa_text(const IndexView &ix, const uint32_t *full, uint32_t *isa, uint32_t *txt2, uint64_t txt_words,
                           hipStream_t st) {
  const uint64_t n_rows = (uint64_t)ix.seq_len + 1;
  const unsigned g = (unsigned)std::min<uint64_t>((n_rows + 255) / 256, 65536);
  hipLaunchKernelGGL(k_isa_from_sa, dim3(g), dim3(256), 0, st, full, n_rows, ix.seq_len, isa);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned gw = (unsigned)std::min<uint64_t>((txt_words + 255) / 256, 65536);
  hipLaunchKernelGGL(k_text_from_isa, dim3(gw), dim3(256), 0, st, ix, isa, txt_words, txt2);
  return hipGetLastError();
}

hipError_t launch_sa2pos(const SaArgs &a, bool full, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  int64_t g = (a.n + 255) / 256;
  if (!full && g > 8192) g = 8192;  // persistent-ish: lanes refill from their grid-stride sequence
  if (g > 1 << 20) g = 1 << 20;
  if (full) hipLaunchKernelGGL(k_sa2pos_full, dim3((unsigned)g), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(k_sa2pos_walk, dim3((unsigned)g), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t expand_sa(const IndexView &ix, const uint32_t *sa_s, uint32_t intv, uint32_t *full, hipStream_t st) {
  const uint64_t n_sa = ((uint64_t)ix.seq_len + intv) / intv;
  uint64_t g = (n_sa + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_expand_sa, dim3((unsigned)g), dim3(256), 0, st, ix, sa_s, intv, n_sa, full);
  return hipGetLastError();
}

}  // namespace ibwa
