// fastq.hip -- FASTQ records parsed and encoded on the device (§8f-4 read ingestion).
//
// bwa_read_seq (bwaseqio.c:145-208) reads each record with kseq_read (kseq.h:156-195) and turns
// it into bwa_seq_t.seq: barcode stripped (-B), -I qualities shifted, bwa_trim_read (:74-87) for
// -q, nst_nt4_table codes, and the sequence reversed (:197).  For the common input -- strict
// 4-line FASTQ: "@header\n", one line of sequence bytes (isgraph, none of '>', '+', '@'), a line
// starting with '+', one line of quality bytes 33..127 exactly as long as the sequence -- kseq_read
// returns exactly that sequence and quality, so a record is a fixed function of its four lines
// (readers.h FastqBulk::rec_at states the same shape on the host).  Here a raw block of the file
// goes to HBM and:
//   k_fq_count   newlines per 16 KiB tile (SWAR zero-byte count on 16 B loads)
//   (scan)       tile -> first line index
//   k_fq_lines   every newline's position, in order (block scan of per-thread counts)
//   k_fq_rec     one wavefront per record: the strict-shape checks over its lines, its kept length
//                (barcode / trim); the first record that is not strict ends the block's records
//   (scan)       kept-read rank and code offset of every record, one 64-bit key (32 bits each:
//                a block is < 4 GiB, so neither the rank nor the offset can overflow its half)
//   k_fq_encode  one wavefront per record: the reversed nt4 codes, coalesced stores
// The host hands the rest of the input, from the first record that is not strict, to the serial
// kseq-semantics reader, exactly as FastqBulk does; the kept reads of the block stay in HBM and
// are staged for the search passes device to device (engine.hip ibwa_batch_stage_fq).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <rocprim/rocprim.hpp>

#include "engine.h"

namespace ibwa {

namespace {

constexpr int FQ_BLOCK = 256;
constexpr uint32_t FQ_TILE = 16384;  // bytes per block in the newline kernels: 64 B per thread

__device__ __forceinline__ uint32_t nl_bytes(uint32_t w) {  // bytes of w equal to '\n'
  const uint32_t x = w ^ 0x0A0A0A0Au;
  const uint32_t t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
  return t;  // 0x80 in every byte that was '\n'
}

__global__ void __launch_bounds__(FQ_BLOCK) k_fq_count(const uint4 *buf, uint32_t *tile_cnt) {
  const uint4 *p = buf + ((size_t)blockIdx.x * FQ_TILE + threadIdx.x * 64u) / 16u;
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 v = p[q];
    c += __builtin_popcount(nl_bytes(v.x)) + __builtin_popcount(nl_bytes(v.y)) + __builtin_popcount(nl_bytes(v.z)) +
         __builtin_popcount(nl_bytes(v.w));
  }
  using BR = rocprim::block_reduce<uint32_t, FQ_BLOCK>;
  __shared__ typename BR::storage_type sr;
  uint32_t tot = 0;
  BR().reduce(c, tot, sr);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(FQ_BLOCK) k_fq_lines(const uint4 *buf, const uint32_t *tile_base, uint32_t n_tiles,
                                                      const uint32_t *tile_cnt, uint32_t *nl, uint32_t cap_lines,
                                                      uint32_t *n_lines) {
  const uint32_t t0 = blockIdx.x * FQ_TILE + threadIdx.x * 64u;
  const uint4 *p = buf + t0 / 16u;
  uint32_t w[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 v = p[q];
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
  uint32_t m[16], c = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    m[q] = nl_bytes(w[q]);
    c += __builtin_popcount(m[q]);
  }
  using BS = rocprim::block_scan<uint32_t, FQ_BLOCK>;
  __shared__ typename BS::storage_type ss;
  uint32_t before = 0;
  BS().exclusive_scan(c, before, 0u, ss);
  uint32_t k = tile_base[blockIdx.x] + before;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    uint32_t x = m[q];
    while (x) {
      const uint32_t b = (uint32_t)__builtin_ctz(x) >> 3;
      if (k < cap_lines) nl[k] = t0 + 4u * (uint32_t)q + b;
      ++k;
      x &= x - 1u;
    }
  }
  // lines past the table's capacity are not used: the block's records end before them
  if (blockIdx.x == n_tiles - 1 && threadIdx.x == 0) *n_lines = min(tile_base[blockIdx.x] + tile_cnt[blockIdx.x], cap_lines);
}

__device__ __forceinline__ uint32_t line_start(const uint32_t *nl, uint32_t L) { return L ? nl[L - 1] + 1u : 0u; }

// one wavefront per record: strict shape, kept length (-1: skipped, bwaseqio.c:162), sequence length
__global__ void __launch_bounds__(FQ_BLOCK) k_fq_rec(const uint8_t *buf, const uint32_t *nl, const uint32_t *n_lines,
                                                    FqOpt o, int32_t *rec_len, uint32_t *rec_L, uint32_t *bad) {
  const uint32_t n_rec = *n_lines / 4u;
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t r = wave; r < n_rec; r += n_waves) {
    const uint32_t h0 = line_start(nl, 4 * r), s0 = nl[4 * r] + 1u, s1 = nl[4 * r + 1];
    const uint32_t p0 = s1 + 1u, q0 = nl[4 * r + 2] + 1u, q1 = nl[4 * r + 3];
    const uint32_t L = s1 - s0;
    bool ok = buf[h0] == '@' && L >= 1u && L <= (1u << 24) && buf[p0] == '+' && q1 - q0 == L;
    if (ok) {
      bool lane_bad = false;
      for (uint32_t j = (uint32_t)lane; j < L; j += 64) {
        const uint8_t c = buf[s0 + j], q = buf[q0 + j];
        // isgraph and none of '>', '+', '@' (readers.h SeqReader::seq_class == 1); quality 33..127
        lane_bad |= c < 33 || c > 126 || c == '>' || c == '+' || c == '@' || q < 33 || q > 127;
      }
      ok = __ballot(lane_bad) == 0ull;
    }
    if (lane == 0) {
      int32_t len = -1;
      if (!ok) {
        atomicMin(bad, r);
      } else if ((int)L > o.l_bc) {
        len = (int)L - o.l_bc;
        if (o.trim_qual >= 1) {  // bwa_trim_read (bwaseqio.c:74-87) on the quality after the barcode
          const uint8_t *qq = buf + q0 + o.l_bc;
          int sc = 0, mx = 0, max_l = len - 1;
          for (int p = len - 1; p >= FQ_MIN_RDLEN - 1; --p) {
            const int c = o.is_64 ? (int)(uint8_t)(qq[p] - 31) : (int)qq[p];
            sc += o.trim_qual - (c - 33);
            if (sc < 0) break;
            if (sc > mx) { mx = sc; max_l = p; }
          }
          len = max_l + 1;
        }
      }
      rec_len[r] = len;
      rec_L[r] = ok ? L : 0u;
    }
  }
}

struct KeptKey {  // kept-read count << 32 | code bytes
  __host__ __device__ uint64_t operator()(int32_t len) const {
    return len >= 0 ? (1ull << 32) | (uint64_t)len : 0ull;
  }
};

// one wavefront per record: codes of the reversed read (bwaseqio.c:194-197), nst_nt4_table
__global__ void __launch_bounds__(FQ_BLOCK) k_fq_encode(const uint8_t *buf, const uint32_t *nl, const uint32_t *n_lines,
                                                       const uint32_t *bad, const int32_t *rec_len,
                                                       const uint64_t *rec_key, int l_bc, uint8_t *codes,
                                                       uint64_t *offk, uint32_t *lenk) {
  const uint32_t n_rec = min(*n_lines / 4u, *bad);
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t r = wave; r < n_rec; r += n_waves) {
    const int32_t len = rec_len[r];
    if (len < 0) continue;
    const uint64_t key = rec_key[r];
    const uint64_t kr = key >> 32, co = key & 0xFFFFFFFFull;
    if (lane == 0) {
      offk[kr] = co;
      lenk[kr] = (uint32_t)len;
    }
    const uint8_t *s = buf + nl[4 * r] + 1u + l_bc;
    for (int j = lane; j < len; j += 64) {
      const uint8_t c = s[len - 1 - j];
      const uint8_t u = c & 0xDF;  // upper case
      codes[co + j] = u == 'A' ? 0 : u == 'C' ? 1 : u == 'G' ? 2 : u == 'T' ? 3 : c == '-' ? 5 : 4;
    }
  }
}

}  // namespace

uint64_t fq_padded_bytes(uint64_t n) { return (n + FQ_TILE - 1) / FQ_TILE * FQ_TILE + FQ_TILE; }

hipError_t fq_parse_launch(const FqBufs &B, uint64_t n, const FqOpt &o, void *tmp, size_t *tmp_bytes, hipStream_t st,
                           const uint32_t *h_init) {
  const uint32_t n_tiles = (uint32_t)((n + FQ_TILE - 1) / FQ_TILE);
  const uint64_t max_rec = (uint64_t)B.cap_lines / 4 + 1;  // every record holds 4 newlines
  auto keys = rocprim::make_transform_iterator(B.rec_len, KeptKey());
  if (!tmp) {
    size_t a = 0, b = 0;
    hipError_t e = rocprim::exclusive_scan(nullptr, a, B.tile_cnt, B.tile_base, 0u, (size_t)n_tiles, rocprim::plus<uint32_t>(), st);
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan(nullptr, b, keys, B.rec_key, (uint64_t)0, (size_t)max_rec, rocprim::plus<uint64_t>(), st);
    *tmp_bytes = a > b ? a : b;
    return e;
  }
  hipError_t e = hipSuccess;
  if (h_init && B.bad == B.n_lines + 1) {
    e = hipMemcpyAsync(B.n_lines, h_init, 8, hipMemcpyHostToDevice, st);
  } else {
    e = hipMemsetAsync(B.n_lines, 0, 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(B.bad, 0xFF, 4, st);
  }
  if (e != hipSuccess) return e;
  if (n_tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_fq_count, dim3(n_tiles), dim3(FQ_BLOCK), 0, st, (const uint4 *)B.raw, B.tile_cnt);
  e = rocprim::exclusive_scan(tmp, *tmp_bytes, B.tile_cnt, B.tile_base, 0u, (size_t)n_tiles, rocprim::plus<uint32_t>(), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fq_lines, dim3(n_tiles), dim3(FQ_BLOCK), 0, st, (const uint4 *)B.raw, B.tile_base, n_tiles,
                     B.tile_cnt, B.nl, B.cap_lines, B.n_lines);
  const uint32_t grid = 4096;  // 16 k wavefronts, records claimed grid-stride
  hipLaunchKernelGGL(k_fq_rec, dim3(grid), dim3(FQ_BLOCK), 0, st, B.raw, B.nl, B.n_lines, o, B.rec_len, B.rec_L, B.bad);
  // records past the first bad one (and past the last complete one) do not count as kept
  e = rocprim::exclusive_scan(tmp, *tmp_bytes, keys, B.rec_key, (uint64_t)0, (size_t)max_rec, rocprim::plus<uint64_t>(), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fq_encode, dim3(grid), dim3(FQ_BLOCK), 0, st, B.raw, B.nl, B.n_lines, B.bad, B.rec_len, B.rec_key,
                     o.l_bc, B.codes, B.offk, B.lenk);
  return hipGetLastError();
}

}  // namespace ibwa
