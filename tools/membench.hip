// membench.hip -- calibrate random-access HBM rates on MI355X for the aln
// access pattern: independent random reads of S bytes (S-aligned) from a
// table far larger than the 256 MiB Infinity Cache.  Reports useful GB/s and
// reads/s; run under `rocprofv3 --pmc FETCH_SIZE` / `TCC_EA0_RDREQ_*` to
// relate the counters to known byte counts (MI355X_MICROARCH.md §HBM asks for
// exactly this calibration for non-streaming widths).
//
// usage: membench [table_GiB] [reads_per_lane]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}

// CHAINS independent reads in flight per lane; each read is S bytes (S/4 dwords)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// NT: non-temporal loads (global_load ... nt), to see whether the L2 then asks the fabric for
// less than a 128 B line per random read
template <int S, int CHAINS, bool NT = false>
__global__ void __launch_bounds__(256) k_rand(const uint32_t *__restrict__ t, uint64_t n_slots, int iters,
                                              uint32_t *__restrict__ out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t st[CHAINS];
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) st[c] = mix(tid * CHAINS + c + 1);
  for (int it = 0; it < iters; ++it) {
    uint32_t v[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      const uint32_t *p = t + (st[c] % n_slots) * (S / 4);
      uint32_t x = 0;
      if constexpr (S == 4) {
        x = p[0];
      } else if constexpr (S == 8) {
        uint2 a = *reinterpret_cast<const uint2 *>(p);
        x = a.x ^ a.y;
      } else {
#pragma unroll
        for (int q = 0; q < S / 16; ++q) {
          if constexpr (NT) {
            const v4u a = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p) + q);
            x ^= a.x ^ a.y ^ a.z ^ a.w;
          } else {
            uint4 a = reinterpret_cast<const uint4 *>(p)[q];
            x ^= a.x ^ a.y ^ a.z ^ a.w;
          }
        }
      }
      v[c] = x;
    }
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      acc += v[c];
      st[c] = mix(st[c] + v[c] + 0x9E3779B97F4A7C15ull);  // dependent: next address needs this read
    }
  }
  if (acc == 0x12345678u) out[tid] = acc;
}

template <int S, int CHAINS, bool NT = false>
void run(const uint32_t *t, uint64_t bytes, int iters, uint32_t *out, int blocks) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  uint64_t n_slots = bytes / S;
  hipLaunchKernelGGL((k_rand<S, CHAINS, NT>), dim3(blocks), dim3(256), 0, 0, t, n_slots, 4, out);  // warm
  CHK(hipEventRecord(a));
  hipLaunchKernelGGL((k_rand<S, CHAINS, NT>), dim3(blocks), dim3(256), 0, 0, t, n_slots, iters, out);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  double reads = (double)blocks * 256 * CHAINS * iters;
  printf("{\"nt\": %d, \"bytes\": %d, \"chains\": %d, \"blocks\": %d, \"ms\": %.3f, \"Greads_s\": %.2f, \"useful_GBs\": %.1f}\n", (int)NT, S,
         CHAINS, blocks, ms, reads / ms / 1e6, reads * S / ms / 1e6);
  fflush(stdout);
}

int main(int argc, char **argv) {
  double gib = argc > 1 ? atof(argv[1]) : 2.0;
  int iters = argc > 2 ? atoi(argv[2]) : 200;
  const bool nt_only = argc > 3 && argv[3][0] == 'n';
  uint64_t bytes = (uint64_t)(gib * (1ull << 30));
  uint32_t *t, *out;
  CHK(hipMalloc(&t, bytes));
  CHK(hipMemset(t, 1, bytes));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int blocks = cus * 8;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  if (nt_only) {  // one kernel per run, for PMC passes
    if (argv[3][1] == 't') run<16, 4, true>(t, bytes, iters, out, blocks);
    else run<16, 4, false>(t, bytes, iters, out, blocks);
    CHK(hipFree(t));
    CHK(hipFree(out));
    return 0;
  }
  run<16, 4, true>(t, bytes, iters, out, blocks);
  run<64, 4, true>(t, bytes, iters, out, blocks);
  run<4, 2>(t, bytes, iters, out, blocks);
  run<8, 2>(t, bytes, iters, out, blocks);
  run<16, 2>(t, bytes, iters, out, blocks);
  run<32, 2>(t, bytes, iters, out, blocks);
  run<64, 2>(t, bytes, iters, out, blocks);
  run<128, 2>(t, bytes, iters, out, blocks);
  run<64, 1>(t, bytes, iters, out, blocks);
  run<64, 4>(t, bytes, iters, out, blocks);
  run<32, 4>(t, bytes, iters, out, blocks);
  run<16, 4>(t, bytes, iters, out, blocks);
  run<64, 2>(t, bytes, iters, out, cus * 4);
  run<64, 2>(t, bytes, iters, out, cus * 16);
  CHK(hipFree(t));
  CHK(hipFree(out));
  return 0;
}
