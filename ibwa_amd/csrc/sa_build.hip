// sa_build.hip -- on-device FM-index construction.
//
// Produces exactly the BWT that `bwa index` writes (bwtindex.c:42-186): the
// suffix array of T$ ($ smallest, is.c:190-216), BWT[j] = T[SA[j]-1], the
// `primary` row where SA[j] == 0, and the $-removed string packed 16
// symbols per word (bwtmisc.c:56-98), for the text and for its reverse
// (.rpac, bwtmisc.c:160-185).  The Occ counts go straight into the 64 B
// block layout of occ.h.
//
// Algorithm (built for 288 GB of HBM rather than for a CPU cache): prefix
// doubling with LSD radix sort (rocPRIM).  Round 1 sorts every suffix by its
// first 21 symbols packed 3 bits each (0 = past the end, so a suffix shorter
// than 21 sorts before its extensions, as $ does).  Round r sorts only the
// suffixes still tied, by (rank[i], rank[i+h]) with h = 21 * 2^(r-1), the
// ranks being h-group start positions (Manber-Myers).  For a human-sized
// text the first round dominates: 3.1e9 (key, value) pairs, ~90 GB of HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <rocprim/rocprim.hpp>

#include "engine.h"

namespace ibwa {

namespace {

constexpr int KCHARS = 21;  // 3-bit symbols per 64-bit key

__global__ void k_init_keys(const uint8_t *__restrict__ T, uint64_t n, uint64_t N, uint64_t *__restrict__ key,
                            uint32_t *__restrict__ val) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = 0;
#pragma unroll
    for (int j = 0; j < KCHARS; ++j) {
      uint64_t p = i + j;
      uint64_t c = p < n ? (uint64_t)T[p] + 1 : 0;
      k = (k << 3) | c;
    }
    key[i] = k;
    val[i] = (uint32_t)i;
  }
}

// head flag as "j if group starts at j, else 0" for a max-scan
template <class K>
__global__ void k_heads(const K *__restrict__ key, uint64_t m, uint32_t *__restrict__ hs) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x)
    hs[j] = (j == 0 || key[j] != key[j - 1]) ? (uint32_t)j : 0u;
}

// round 1: rank[SA[j]] = group start; flag unsorted (group size > 1)
__global__ void k_rank1(const uint64_t *__restrict__ key, const uint32_t *__restrict__ sa,
                        const uint32_t *__restrict__ gstart, uint64_t m, uint32_t *__restrict__ rank,
                        uint32_t *__restrict__ flag) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
    rank[sa[j]] = gstart[j];
    bool head = j == 0 || key[j] != key[j - 1];
    bool next_head = j + 1 == m || key[j + 1] != key[j];
    flag[j] = (head && next_head) ? 0u : 1u;
  }
}

// later rounds: keys of the still-tied suffixes
__global__ void k_keys2(const uint32_t *__restrict__ V, uint64_t m, const uint32_t *__restrict__ rank, uint64_t h,
                        uint64_t *__restrict__ K) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t v = V[j];
    K[j] = (uint64_t)rank[v] << 32 | rank[(uint64_t)v + h];
  }
}

// later rounds: write back SA, new ranks (group start positions in SA), unsorted flags
__global__ void k_rank2(const uint64_t *__restrict__ K, const uint32_t *__restrict__ V, const uint32_t *__restrict__ P,
                        const uint32_t *__restrict__ gidx, uint64_t m, uint32_t *__restrict__ sa,
                        uint32_t *__restrict__ rank, uint32_t *__restrict__ flag) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
    sa[P[j]] = V[j];
    rank[V[j]] = P[gidx[j]];
    bool head = j == 0 || K[j] != K[j - 1];
    bool next_head = j + 1 == m || K[j + 1] != K[j];
    flag[j] = (head && next_head) ? 0u : 1u;
  }
}

// compaction of (P, V) by flag with exclusive-scanned offsets
__global__ void k_compact(const uint32_t *__restrict__ flag, const uint32_t *__restrict__ offs, uint64_t m,
                          const uint32_t *__restrict__ Pin, const uint32_t *__restrict__ Vin,
                          uint32_t *__restrict__ Pout, uint32_t *__restrict__ Vout) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
    if (flag[j]) {
      uint32_t o = offs[j];
      Pout[o] = Pin ? Pin[j] : (uint32_t)j;
      Vout[o] = Vin[j];
    }
  }
}

// $-removed BWT packed 16 symbols / word (bwtmisc.c:94-95) + per-block symbol counts
__global__ void k_bwt_pack(const uint8_t *__restrict__ T, const uint32_t *__restrict__ sa, uint64_t n,
                           uint32_t primary, uint32_t *__restrict__ words, uint64_t n_words) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_words;
       w += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = 0;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint64_t j = w * 16 + t;  // position in the $-removed string
      uint32_t c = 0;
      if (j < n) {
        uint64_t row = j < primary ? j : j + 1;
        uint32_t s = sa[row];
        c = T[s - 1];  // s > 0 for every row but `primary`
      }
      x |= c << ((15 - t) * 2);
    }
    words[w] = x;
  }
}

__global__ void k_block_counts(const uint32_t *__restrict__ words, uint64_t n, uint64_t n_blocks,
                               uint4 *__restrict__ cnt) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n_blocks;
       b += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t acc[4] = {0, 0, 0, 0};
    for (int q = 0; q < 8; ++q) {
      uint64_t w = b * 8 + q;
      uint64_t lo = w * 16;
      if (lo >= n) break;
      uint32_t valid = (uint32_t)((n - lo) < 16 ? (n - lo) : 16);
      uint32_t m = valid == 16 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (2 * valid));
      uint32_t nn[4];
      count4(words[w], 0u, m, 0u, nn);
      for (int c = 0; c < 4; ++c) acc[c] += nn[c];
    }
    cnt[b] = make_uint4(acc[0], acc[1], acc[2], acc[3]);
  }
}

__global__ void k_find_primary(const uint32_t *__restrict__ sa, uint64_t N, uint32_t *__restrict__ out) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < N; j += (uint64_t)gridDim.x * blockDim.x)
    if (sa[j] == 0) *out = (uint32_t)j;
}

__global__ void k_reverse(uint8_t *T, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t a = T[i], b = T[n - 1 - i];
    T[i] = b;
    T[n - 1 - i] = a;
  }
}

// inverse suffix array: isa[sa[r]] = r
__global__ void k_isa(const uint32_t *__restrict__ sa, uint64_t N, uint32_t *__restrict__ isa) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (uint64_t)gridDim.x * blockDim.x)
    isa[sa[r]] = (uint32_t)r;
}

// text codes -> 2 bits per base, base t at bits 2 (t & 15) of word t >> 4 (tail words zero)
__global__ void k_pack_text2(const uint8_t *__restrict__ T, uint64_t n, uint64_t n_words, uint32_t *__restrict__ out) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_words;
       w += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = 0;
    for (int k = 0; k < 16; ++k) {
      const uint64_t t = w * 16 + k;
      if (t < n) x |= (uint32_t)(T[t] & 3) << (2 * k);
    }
    out[w] = x;
  }
}

__global__ void k_sample_sa(const uint32_t *__restrict__ sa, uint64_t n_sa, uint32_t intv, uint32_t *__restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_sa; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = sa[i * intv];
}

struct Uint4Plus {
  __device__ __host__ uint4 operator()(const uint4 &a, const uint4 &b) const {
    return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
};

inline dim3 grid_for(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  if (g == 0) g = 1;
  return dim3((unsigned)g);
}

}  // namespace

// Scratch owned by the builder for one text of length n (N = n + 1 suffixes).
struct SaScratch {
  uint32_t *sa = nullptr, *rank = nullptr, *v1 = nullptr;
  uint64_t *k0 = nullptr, *k1 = nullptr;
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
};

#define HC(x)                          \
  do {                                 \
    hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return e_;   \
  } while (0)

// Suffix array of T[0..n) with the empty suffix at SA[0] (is.c:190 convention).
// On return S.sa[0..n] holds it.  `rounds` receives the number of sort rounds.
static hipError_t suffix_sort(const uint8_t *T, uint64_t n, SaScratch &S, hipStream_t st, int *rounds) {
  const uint64_t N = n + 1;
  // round 1
  hipLaunchKernelGGL(k_init_keys, grid_for(N), dim3(256), 0, st, T, n, N, S.k0, S.v1);
  HC(hipGetLastError());
  {
    rocprim::double_buffer<uint64_t> kb(S.k0, S.k1);
    rocprim::double_buffer<uint32_t> vb(S.v1, S.sa);
    size_t need = 0;
    HC(rocprim::radix_sort_pairs(nullptr, need, kb, vb, N, 0, 3 * KCHARS, st));
    if (need > S.tmp_bytes) return hipErrorOutOfMemory;
    HC(rocprim::radix_sort_pairs(S.tmp, need, kb, vb, N, 0, 3 * KCHARS, st));
    // make S.sa / S.k0 hold the sorted result
    if (vb.current() != S.sa) HC(hipMemcpyAsync(S.sa, vb.current(), N * 4, hipMemcpyDeviceToDevice, st));
    if (kb.current() != S.k0) HC(hipMemcpyAsync(S.k0, kb.current(), N * 8, hipMemcpyDeviceToDevice, st));
  }
  // group starts -> ranks; unsorted flags
  uint32_t *hs = reinterpret_cast<uint32_t *>(S.k1);      // N u32
  uint32_t *gst = hs + N;                                  // N u32 (k1 holds 2N u32)
  hipLaunchKernelGGL(k_heads<uint64_t>, grid_for(N), dim3(256), 0, st, S.k0, N, hs);
  {
    size_t need = 0;
    HC(rocprim::inclusive_scan(nullptr, need, hs, gst, N, rocprim::maximum<uint32_t>(), st));
    if (need > S.tmp_bytes) return hipErrorOutOfMemory;
    HC(rocprim::inclusive_scan(S.tmp, need, hs, gst, N, rocprim::maximum<uint32_t>(), st));
  }
  uint32_t *flag = hs;  // reuse
  hipLaunchKernelGGL(k_rank1, grid_for(N), dim3(256), 0, st, S.k0, S.sa, gst, N, S.rank, flag);
  HC(hipGetLastError());
  // compact unsorted: P (SA positions), V (suffix ids) into the k0 region (2N u32)
  uint32_t *offs = gst;
  {
    size_t need = 0;
    HC(rocprim::exclusive_scan(nullptr, need, flag, offs, 0u, N, rocprim::plus<uint32_t>(), st));
    if (need > S.tmp_bytes) return hipErrorOutOfMemory;
    HC(rocprim::exclusive_scan(S.tmp, need, flag, offs, 0u, N, rocprim::plus<uint32_t>(), st));
  }
  uint32_t last_off = 0, last_flag = 0;
  HC(hipMemcpyAsync(&last_off, offs + N - 1, 4, hipMemcpyDeviceToHost, st));
  HC(hipMemcpyAsync(&last_flag, flag + N - 1, 4, hipMemcpyDeviceToHost, st));
  HC(hipStreamSynchronize(st));
  uint64_t m = (uint64_t)last_off + last_flag;
  uint32_t *P = reinterpret_cast<uint32_t *>(S.k0), *V = P + N;
  hipLaunchKernelGGL(k_compact, grid_for(N), dim3(256), 0, st, flag, offs, N, (const uint32_t *)nullptr, S.sa, P, V);
  HC(hipGetLastError());
  int r = 1;
  uint64_t h = KCHARS;
  // later rounds: P, V in k0 (u32 x 2N); K in k1 (u64 x m); K2 in a fresh u64 x m buffer; V2 in v1
  uint64_t *K2 = nullptr;
  if (m > 0) HC(hipMalloc(&K2, m * 8));
  while (m > 0) {
    ++r;
    uint64_t *K = S.k1;
    uint32_t *V2 = S.v1;
    hipLaunchKernelGGL(k_keys2, grid_for(m), dim3(256), 0, st, V, m, S.rank, h, K);
    HC(hipGetLastError());
    {
      rocprim::double_buffer<uint64_t> kb(K, K2);
      rocprim::double_buffer<uint32_t> vb(V, V2);
      size_t need = 0;
      HC(rocprim::radix_sort_pairs(nullptr, need, kb, vb, m, 0, 64, st));
      if (need > S.tmp_bytes) return hipErrorOutOfMemory;
      HC(rocprim::radix_sort_pairs(S.tmp, need, kb, vb, m, 0, 64, st));
      if (kb.current() != K) HC(hipMemcpyAsync(K, kb.current(), m * 8, hipMemcpyDeviceToDevice, st));
      if (vb.current() != V) HC(hipMemcpyAsync(V, vb.current(), m * 4, hipMemcpyDeviceToDevice, st));
    }
    // group index within the compacted array: max-scan of heads
    uint32_t *hs2 = reinterpret_cast<uint32_t *>(K2);
    uint32_t *gidx = hs2 + m;
    hipLaunchKernelGGL(k_heads<uint64_t>, grid_for(m), dim3(256), 0, st, K, m, hs2);
    {
      size_t need = 0;
      HC(rocprim::inclusive_scan(nullptr, need, hs2, gidx, m, rocprim::maximum<uint32_t>(), st));
      if (need > S.tmp_bytes) return hipErrorOutOfMemory;
      HC(rocprim::inclusive_scan(S.tmp, need, hs2, gidx, m, rocprim::maximum<uint32_t>(), st));
    }
    uint32_t *flag2 = hs2;
    hipLaunchKernelGGL(k_rank2, grid_for(m), dim3(256), 0, st, K, V, P, gidx, m, S.sa, S.rank, flag2);
    HC(hipGetLastError());
    uint32_t *offs2 = gidx;
    {
      size_t need = 0;
      HC(rocprim::exclusive_scan(nullptr, need, flag2, offs2, 0u, m, rocprim::plus<uint32_t>(), st));
      if (need > S.tmp_bytes) return hipErrorOutOfMemory;
      HC(rocprim::exclusive_scan(S.tmp, need, flag2, offs2, 0u, m, rocprim::plus<uint32_t>(), st));
    }
    HC(hipMemcpyAsync(&last_off, offs2 + m - 1, 4, hipMemcpyDeviceToHost, st));
    HC(hipMemcpyAsync(&last_flag, flag2 + m - 1, 4, hipMemcpyDeviceToHost, st));
    HC(hipStreamSynchronize(st));
    uint64_t m2 = (uint64_t)last_off + last_flag;
    // compact in place via the v1 buffer as staging: P -> V2 ; V -> K region
    uint32_t *Pn = V2, *Vn = reinterpret_cast<uint32_t *>(K);
    hipLaunchKernelGGL(k_compact, grid_for(m), dim3(256), 0, st, flag2, offs2, m, P, V, Pn, Vn);
    HC(hipGetLastError());
    HC(hipMemcpyAsync(P, Pn, m2 * 4, hipMemcpyDeviceToDevice, st));
    V = P + m2;
    HC(hipMemcpyAsync(V, Vn, m2 * 4, hipMemcpyDeviceToDevice, st));
    m = m2;
    h *= 2;
    if (r > 40) { (void)hipFree(K2); return hipErrorUnknown; }  // LCP > 2^40: impossible for n < 2^32
  }
  if (K2) (void)hipFree(K2);
  if (rounds) *rounds = r;
  return hipSuccess;
}

// Build one strand's index from the device text T (codes 0..3, length n).
// out_blocks: ceil(n/128)+1 blocks of 64 B.  totals: symbol counts.
hipError_t build_strand(const uint8_t *T, uint64_t n, uint4 *out_blocks, uint32_t *primary, uint32_t totals[4],
                        uint32_t *sa_sample, uint32_t sa_intv, int *rounds, uint32_t *sa_full, uint32_t *isa_full,
                        hipStream_t st) {
  const uint64_t N = n + 1;
  SaScratch S;
  HC(hipMalloc(&S.sa, N * 4));
  HC(hipMalloc(&S.rank, N * 4));
  HC(hipMalloc(&S.v1, N * 4));
  HC(hipMalloc(&S.k0, N * 8));
  HC(hipMalloc(&S.k1, N * 8));
  // temp storage: the largest of the rocPRIM calls at size N
  {
    size_t a = 0, b = 0, c = 0;
    rocprim::double_buffer<uint64_t> kb(S.k0, S.k1);
    rocprim::double_buffer<uint32_t> vb(S.v1, S.sa);
    HC(rocprim::radix_sort_pairs(nullptr, a, kb, vb, N, 0, 64, st));
    HC(rocprim::inclusive_scan(nullptr, b, S.sa, S.v1, N, rocprim::maximum<uint32_t>(), st));
    HC(rocprim::exclusive_scan(nullptr, c, S.sa, S.v1, 0u, N, rocprim::plus<uint32_t>(), st));
    S.tmp_bytes = std::max(a, std::max(b, c)) + 4096;
    HC(hipMalloc(&S.tmp, S.tmp_bytes));
  }
  hipError_t e = suffix_sort(T, n, S, st, rounds);
  if (e == hipSuccess) {
    uint32_t *d_primary = S.rank;  // rank no longer needed
    hipLaunchKernelGGL(k_find_primary, grid_for(N), dim3(256), 0, st, S.sa, N, d_primary);
    e = hipMemcpyAsync(primary, d_primary, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  if (e == hipSuccess && sa_full) e = hipMemcpyAsync(sa_full, S.sa, N * 4, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess && isa_full) {
    hipLaunchKernelGGL(k_isa, grid_for(N), dim3(256), 0, st, S.sa, N, isa_full);
    e = hipGetLastError();
  }
  if (e == hipSuccess && sa_sample) {
    uint64_t n_sa = (n + sa_intv) / sa_intv;  // bwt.c:56
    hipLaunchKernelGGL(k_sample_sa, grid_for(n_sa), dim3(256), 0, st, S.sa, n_sa, sa_intv, sa_sample);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    const uint64_t n_words = (n + 15) / 16, n_blocks = (n + 127) / 128 + 1;
    uint32_t *words = reinterpret_cast<uint32_t *>(S.k0);
    uint4 *cnt = reinterpret_cast<uint4 *>(S.k1);
    uint4 *base = cnt + n_blocks;
    hipLaunchKernelGGL(k_bwt_pack, grid_for(n_words), dim3(256), 0, st, T, S.sa, n, *primary, words, n_words);
    hipLaunchKernelGGL(k_block_counts, grid_for(n_blocks), dim3(256), 0, st, words, n, n_blocks, cnt);
    size_t need = 0;
    e = rocprim::exclusive_scan(nullptr, need, cnt, base, make_uint4(0, 0, 0, 0), n_blocks, Uint4Plus(), st);
    if (e == hipSuccess && need <= S.tmp_bytes)
      e = rocprim::exclusive_scan(S.tmp, need, cnt, base, make_uint4(0, 0, 0, 0), n_blocks, Uint4Plus(), st);
    else if (e == hipSuccess)
      e = hipErrorOutOfMemory;
    if (e == hipSuccess) e = pack_blocks(words, n_words, base, n_blocks, out_blocks, st);
    uint4 tot;
    if (e == hipSuccess) e = hipMemcpyAsync(&tot, base + n_blocks - 1, 16, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) {
      totals[0] = tot.x; totals[1] = tot.y; totals[2] = tot.z; totals[3] = tot.w;
    }
  }
  (void)hipFree(S.sa); (void)hipFree(S.rank); (void)hipFree(S.v1);
  (void)hipFree(S.k0); (void)hipFree(S.k1); (void)hipFree(S.tmp);
  return e;
}

hipError_t pack_text2(const uint8_t *T, uint64_t n, uint32_t *out, uint64_t out_words, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_text2, grid_for(out_words), dim3(256), 0, st, T, n, out_words, out);
  return hipGetLastError();
}

hipError_t reverse_text(uint8_t *T, uint64_t n, hipStream_t st) {
  hipLaunchKernelGGL(k_reverse, grid_for(n / 2 + 1), dim3(256), 0, st, T, n);
  return hipGetLastError();
}

}  // namespace ibwa
