// kmer.hip -- K-mer -> SA-interval lookup table for the exact-match chains.
//
// An exact backward search (bwt_match_exact_alt, bwt.c:235-250) that has
// consumed the last K symbols of its string sits on a SA interval that depends
// only on those K symbols.  table[P] (P = the K-mer, first symbol most
// significant) holds that interval, or k > l if the search would already
// have failed inside those K steps (the reference returns "no match" at the
// first empty interval, so the outcome is the same).  One 8 B lookup thus
// replaces K dependent Occ fetches -- the dominant cost, since random HBM
// reads are request-rate bound on MI355X whatever their size (tools/membench).
//
// Built level by level on the device: level j+1 (4^(j+1) entries) extends
// every level-j interval by prepending symbol c with one rank-query pair.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine.h"
#include "occ.h"

namespace ibwa {

namespace {

__global__ void __launch_bounds__(256) k_kmer_level(IndexView ix, const uint2 *__restrict__ prev, uint2 *__restrict__ next,
                                                    int j) {
  const uint64_t n_next = 1ull << (2 * (j + 1));
  const uint64_t mask = (1ull << (2 * j)) - 1;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_next; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = (uint32_t)(t >> (2 * j));
    const uint2 iv = j == 0 ? make_uint2(0u, ix.seq_len) : prev[t & mask];
    uint2 out = make_uint2(1u, 0u);  // empty
    if (iv.x <= iv.y) {
      uint32_t ok, ol;
      occ2(ix, iv.x - 1, iv.y, c, ok, ol);
      const uint32_t k = l2of(ix, c) + ok + 1, l = l2of(ix, c) + ol;
      if (k <= l) out = make_uint2(k, l);
    }
    next[t] = out;
  }
}

// Level tables of the first pass (gapped.hip, GapArgs::ltab): every string of length d <= levels,
// its SA interval at entry ltab_off(d) + code, code = the string's symbols in the order the backward
// search reads them, the newest LEAST significant -- so the four children of node x at depth d are the
// 32 bytes at ltab_off(d + 1) + 4x.  Level d+1 from level d: entry 4x + c extends x by symbol c.
__global__ void __launch_bounds__(256) k_ltab_level(IndexView ix, uint2 *__restrict__ t, int d) {
  const uint64_t n_next = 1ull << (2 * (d + 1));
  const uint64_t o_prev = ltab_off(d), o_next = ltab_off(d + 1);
  for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n_next; x += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = (uint32_t)(x & 3);
    const uint2 iv = d == 0 ? make_uint2(0u, ix.seq_len) : t[o_prev + (x >> 2)];
    uint2 out = make_uint2(1u, 0u);  // empty
    if (iv.x <= iv.y) {
      uint32_t ok, ol;
      occ2(ix, iv.x - 1, iv.y, c, ok, ol);
      const uint32_t k = l2of(ix, c) + ok + 1, l = l2of(ix, c) + ol;
      if (k <= l) out = make_uint2(k, l);
    }
    t[o_next + x] = out;
  }
}

}  // namespace

// levels 0..levels of the first pass's level table into t (ltab_off(levels + 1) entries)
hipError_t build_level_tables(const IndexView &ix, int levels, uint2 *t, hipStream_t st) {
  const uint2 root = make_uint2(0u, ix.seq_len);
  hipError_t e = hipMemcpyAsync(t, &root, sizeof root, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return e;
  for (int d = 0; d < levels; ++d) {
    const uint64_t n_next = 1ull << (2 * (d + 1));
    uint64_t g = (n_next + 255) / 256;
    if (g > 65536) g = 65536;
    hipLaunchKernelGGL(k_ltab_level, dim3((unsigned)g), dim3(256), 0, st, ix, t, d);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipStreamSynchronize(st);  // (the root's copy reads host stack memory)
}

// table: 4^K uint2; tmp: 4^(K-1) uint2 (K >= 1)
hipError_t build_kmer_table(const IndexView &ix, int K, uint2 *table, uint2 *tmp, hipStream_t st) {
  uint2 *bufs[2];
  // the last level must land in `table`: alternate so that level K is written to it
  bufs[K & 1] = table;
  bufs[(K & 1) ^ 1] = tmp;
  for (int j = 0; j < K; ++j) {
    const uint64_t n_next = 1ull << (2 * (j + 1));
    uint64_t g = (n_next + 255) / 256;
    if (g > 65536) g = 65536;
    hipLaunchKernelGGL(k_kmer_level, dim3((unsigned)g), dim3(256), 0, st, ix, bufs[j & 1], bufs[(j + 1) & 1], j);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace ibwa
