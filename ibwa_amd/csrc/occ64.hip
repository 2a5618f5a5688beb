// occ64.hip -- one-hot "bit-plane" Occ layout for the exact-match path.
//
// Measured on MI355X (profiles/, tools/membench.hip): random reads are
// bound by per-lane line requests through the vector memory pipeline
// (~55 G requests/s chip-wide for 4..64 B reads) and every miss is a 128 B
// request.  So a rank query should be ONE 16 B load that carries everything,
// and the two ends of an interval should share it whenever they can.
// Trading HBM capacity for requests and instructions, this layout spends
// 1 byte per BWT row (2 x 3.1 GB for GRCh37):
//
//   block b = 64 rows of the BWT *including* the $ row, 64 B = 4 x uint4:
//     uint4[c] = {C[c], 0, P_lo[c], P_hi[c]}
//       C[c]  = occurrences of c in rows [0, 64b)   ($ excluded)
//       P[c]  = bit i set iff row 64b+i holds symbol c   (the $ row sets none)
//
//   Occ(c, k) = C[c] + popcount(P[c] & mask(k & 63)),   block k >> 6
//
// which is bwt_occ (bwt.c:90-113): occurrences of c in rows [0..k] with $
// removed -- no `k >= primary` correction, the $ row simply has no bit.
// The two ends k-1 and l of an interval share the load when they fall in
// one block (bwt_2occ's fast path, bwt.c:125-150, in spirit).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine.h"
#include "occ.h"

namespace ibwa {

namespace {

// symbol at position p of the $-removed BWT (occ.h layout)
__device__ __forceinline__ uint32_t sym_at(const IndexView &ix, uint32_t p) {
  const uint32_t *b = reinterpret_cast<const uint32_t *>(ix.blk + (size_t)(p >> 7) * 4);
  const uint32_t w = b[4 + ((p & 127) >> 4)];
  return (w >> (2 * (15 - (p & 15)))) & 3u;
}

__global__ void __launch_bounds__(256) k_occ64_build(IndexView ix, uint4 *__restrict__ out, uint64_t n_blk) {
  const uint64_t n_rows = (uint64_t)ix.seq_len + 1;  // BWT rows incl. $
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < n_blk; b += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t C[4] = {0, 0, 0, 0};
    if (b > 0) {
      const uint64_t last = b * 64 - 1;  // rows [0, 64b), $ removed (bwt.c:157)
      occ4(ix, (uint32_t)(last < ix.seq_len ? last : ix.seq_len), C);
    }
    uint64_t P[4] = {0, 0, 0, 0};
    for (int i = 0; i < 64; ++i) {
      const uint64_t row = b * 64 + i;
      if (row >= n_rows || row == ix.primary) continue;
      const uint32_t p = (uint32_t)(row < ix.primary ? row : row - 1);
      P[sym_at(ix, p)] |= 1ull << i;
    }
    uint4 *o = out + b * 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = make_uint4(C[c], 0u, (uint32_t)P[c], (uint32_t)(P[c] >> 32));
  }
}

}  // namespace

uint64_t occ64_blocks(uint32_t seq_len) { return ((uint64_t)seq_len + 1 + 63) / 64 + 1; }

hipError_t build_occ64(const IndexView &ix, uint4 *out, hipStream_t st) {
  const uint64_t nb = occ64_blocks(ix.seq_len);
  uint64_t g = (nb + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_occ64_build, dim3((unsigned)g), dim3(256), 0, st, ix, out, nb);
  return hipGetLastError();
}

}  // namespace ibwa
