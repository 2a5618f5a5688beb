// index.hip -- device residency of the .bwt / .rbwt FM-indexes (bwtio.c:51,
// bwt.h:42-63) in the 64 B-block HBM layout of occ.h.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "occ.h"
#include "engine.h"

namespace ibwa {

// One thread per 128-symbol block: copy the 4 counts and 8 symbol words of
// the reference's interleaved layout (bwtmisc.c:122-144) and add the three
// 32-symbol sub-counts.  Word reads past the end of the reference array
// (the last, partial block) read 0; those symbols lie beyond seq_len and are
// never counted by a query.
__global__ void __launch_bounds__(256) k_relayout(const uint32_t *__restrict__ ref, uint64_t n_words,
                                                  uint64_t n_blocks, uint4 *__restrict__ out) {
  uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_blocks) return;
  const uint64_t base = b * 12;
  uint32_t w[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) w[j] = base + j < n_words ? ref[base + j] : 0u;
  uint32_t sub[3];
  uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    uint32_t n[4];
    count4(w[4 + 2 * q], w[5 + 2 * q], 0xFFFFFFFFu, 0xFFFFFFFFu, n);
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] += n[c];
    sub[q] = acc[0] | acc[1] << 8 | acc[2] << 16 | acc[3] << 24;
  }
  uint4 *o = out + b * 4;
  o[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o[1] = make_uint4(w[4], w[5], w[6], w[7]);
  o[2] = make_uint4(w[8], w[9], w[10], w[11]);
  o[3] = make_uint4(sub[0], sub[1], sub[2], 0u);
}

// Same, from a packed $-removed BWT (16 symbols per word, MSB first) plus a
// per-block count prefix already computed: used by the on-device index
// builder (sa_build.hip).
__global__ void __launch_bounds__(256) k_pack_blocks(const uint32_t *__restrict__ sym_words, uint64_t n_sym_words,
                                                     const uint4 *__restrict__ block_base, uint64_t n_blocks,
                                                     uint4 *__restrict__ out) {
  uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_blocks) return;
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = b * 8 + j < n_sym_words ? sym_words[b * 8 + j] : 0u;
  uint32_t sub[3], acc[4] = {0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    uint32_t n[4];
    count4(w[2 * q], w[2 * q + 1], 0xFFFFFFFFu, 0xFFFFFFFFu, n);
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] += n[c];
    sub[q] = acc[0] | acc[1] << 8 | acc[2] << 16 | acc[3] << 24;
  }
  uint4 *o = out + b * 4;
  o[0] = block_base[b];
  o[1] = make_uint4(w[0], w[1], w[2], w[3]);
  o[2] = make_uint4(w[4], w[5], w[6], w[7]);
  o[3] = make_uint4(sub[0], sub[1], sub[2], 0u);
}

hipError_t relayout_reference_bwt(const uint32_t *d_ref, uint64_t n_words, uint64_t n_blocks, uint4 *d_out,
                                  hipStream_t st) {
  uint64_t grid = (n_blocks + 255) / 256;
  hipLaunchKernelGGL(k_relayout, dim3((unsigned)grid), dim3(256), 0, st, d_ref, n_words, n_blocks, d_out);
  return hipGetLastError();
}

hipError_t pack_blocks(const uint32_t *d_sym, uint64_t n_sym_words, const uint4 *d_block_base, uint64_t n_blocks,
                       uint4 *d_out, hipStream_t st) {
  uint64_t grid = (n_blocks + 255) / 256;
  hipLaunchKernelGGL(k_pack_blocks, dim3((unsigned)grid), dim3(256), 0, st, d_sym, n_sym_words, d_block_base,
                     n_blocks, d_out);
  return hipGetLastError();
}

}  // namespace ibwa
