// membench_w.hip -- random-write cost on MI355X HBM: is a partial-line write (16 B or 64 B of a
// 128 B line, as the gapped kernels' stack pushes and staging stores are) as cheap as a random
// read, or does it cost a read-modify-write?  Table far larger than the Infinity Cache.
//   k_rw<R, W, WS>: per lane-iteration R dependent random 16 B reads (4 independent chains) and
//   W random writes of WS bytes (addresses from the same hash stream; fire-and-forget).
// Prints requests/s of each kind.  usage: membench_w [table_GiB] [iters]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                   \
  do {                                                           \
    hipError_t e = (x);                                          \
    if (e != hipSuccess) {                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));     \
      exit(1);                                                   \
    }                                                            \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}

template <int R, int W, int WS>
__global__ void __launch_bounds__(256) k_rw(uint4 *__restrict__ t, uint64_t n16, int iters, uint32_t *__restrict__ out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t st[4];
  uint64_t ws = mix(tid * 977 + 13);
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) st[c] = mix(tid * 4 + c + 1);
  for (int it = 0; it < iters; ++it) {
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < R) {
        const uint4 a = t[st[c] % n16];
        v[c] = a.x ^ a.y ^ a.z ^ a.w;
      }
#pragma unroll
    for (int w = 0; w < W; ++w) {
      ws = mix(ws + 0x9E3779B97F4A7C15ull);
      constexpr uint64_t per = WS / 16;
      uint4 *p = t + (ws % (n16 / per)) * per;
#pragma unroll
      for (int q = 0; q < (int)per; ++q) p[q] = make_uint4((uint32_t)it, (uint32_t)w, (uint32_t)q, acc);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < R) {
        acc += v[c];
        st[c] = mix(st[c] + v[c] + 0x9E3779B97F4A7C15ull);
      }
  }
  if (acc == 0x12345678u) out[tid] = acc;
}

template <int R, int W, int WS>
void run(uint4 *t, uint64_t bytes, int iters, uint32_t *out, int blocks) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const uint64_t n16 = bytes / 16;
  hipLaunchKernelGGL((k_rw<R, W, WS>), dim3(blocks), dim3(256), 0, 0, t, n16, 4, out);
  CHK(hipEventRecord(a));
  hipLaunchKernelGGL((k_rw<R, W, WS>), dim3(blocks), dim3(256), 0, 0, t, n16, iters, out);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double li = (double)blocks * 256 * iters;
  printf("{\"reads_per_iter\": %d, \"writes_per_iter\": %d, \"write_bytes\": %d, \"ms\": %.3f, \"Greads_s\": %.2f, "
         "\"Gwrites_s\": %.2f}\n", R, W, WS, ms, li * R / ms / 1e6, li * W / ms / 1e6);
  fflush(stdout);
}

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const int iters = argc > 2 ? atoi(argv[2]) : 100;
  const uint64_t bytes = (uint64_t)(gib * (1ull << 30));
  uint4 *t;
  uint32_t *out;
  CHK(hipMalloc(&t, bytes));
  CHK(hipMemset(t, 1, bytes));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 8;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  run<4, 0, 16>(t, bytes, iters, out, blocks);   // reads alone
  run<0, 4, 16>(t, bytes, iters, out, blocks);   // 16 B writes alone
  run<0, 4, 64>(t, bytes, iters, out, blocks);   // 64 B writes alone
  run<0, 4, 128>(t, bytes, iters, out, blocks);  // whole-line writes alone
  run<4, 2, 16>(t, bytes, iters, out, blocks);   // the gapped kernels' mix
  run<4, 2, 128>(t, bytes, iters, out, blocks);
  CHK(hipFree(t));
  CHK(hipFree(out));
  return 0;
}
