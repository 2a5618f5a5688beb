// copy_under_load.hip -- how long do small / large copies and memsets on one non-blocking stream take
// while a persistent grid holds every CU on another stream (the CLI's ingest and fetch next to the
// searches)?  The spinning grid ends by wall clock (wall_clock64, 100 MHz) after SPIN_MS.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <unistd.h>
#include <chrono>

__global__ void __launch_bounds__(256) k_spin(unsigned long long ticks, unsigned *sink) {
  const unsigned long long t0 = wall_clock64();
  unsigned x = threadIdx.x;
  while (wall_clock64() - t0 < ticks) x = x * 1664525u + 1013904223u;
  if (x == 0x12345678u) sink[0] = x;
}

#define CK(e) do { hipError_t r_ = (e); if (r_ != hipSuccess) { printf("error %s line %d\n", hipGetErrorString(r_), __LINE__); return 1; } } while (0)

int main() {
  const double SPIN_MS = 1500;
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  unsigned *sink;
  CK(hipMalloc(&sink, 64));
  const size_t big = 64ull << 20, huge = 1ull << 30;
  char *d_big, *d_big2, *h_pin, *h_huge;
  CK(hipMalloc(&d_big, huge));
  CK(hipMalloc(&d_big2, big));
  CK(hipHostMalloc((void **)&h_pin, big, 0));
  CK(hipHostMalloc((void **)&h_huge, huge, 0));
  unsigned long long v = 0;
  auto now = []() { return std::chrono::steady_clock::now(); };
  auto ms = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
    return std::chrono::duration<double, std::milli>(y - x).count(); };
  const char *names[8] = {"hipMemcpy D2H 8 B", "hipMemcpyAsync D2H 8 B (pinned) + sync", "hipMemcpyAsync D2H 64 MB (pinned) + sync",
                          "hipMemcpyAsync H2D 1 GiB (pinned) + sync", "hipMemsetAsync 64 B + sync", "hipMemcpyAsync D2D 64 MB + sync",
                          "hipMemcpy D2H 64 MB (pageable)", "empty kernel on stream b + sync"};
  for (int load = 0; load < 2; ++load) {
    for (int t = 0; t < 8; ++t) {
      CK(hipDeviceSynchronize());
      if (load) {
        // 32 waves per CU (every wave slot: nothing else can start on any CU while it spins);
        // all of them resident at once, so the grid ends after one SPIN_MS
        hipLaunchKernelGGL(k_spin, dim3(cus * 8), dim3(256), 0, a, (unsigned long long)(SPIN_MS * 1e5), sink);
        CK(hipGetLastError());
        usleep(100000);  // the grid is resident
      }
      const auto t0 = now();
      switch (t) {
        case 0: CK(hipMemcpy(&v, sink, 8, hipMemcpyDeviceToHost)); break;
        case 1: CK(hipMemcpyAsync(h_pin, sink, 8, hipMemcpyDeviceToHost, b)); CK(hipStreamSynchronize(b)); break;
        case 2: CK(hipMemcpyAsync(h_pin, d_big, big, hipMemcpyDeviceToHost, b)); CK(hipStreamSynchronize(b)); break;
        case 3: CK(hipMemcpyAsync(d_big, h_huge, huge, hipMemcpyHostToDevice, b)); CK(hipStreamSynchronize(b)); break;
        case 4: CK(hipMemsetAsync(sink + 4, 0, 64 - 16, b)); CK(hipStreamSynchronize(b)); break;
        case 5: CK(hipMemcpyAsync(d_big2, d_big, big, hipMemcpyDeviceToDevice, b)); CK(hipStreamSynchronize(b)); break;
        case 6: { static char hp[64 << 20]; CK(hipMemcpy(hp, d_big, big, hipMemcpyDeviceToHost)); } break;
        case 7: hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, b, 0ull, sink); CK(hipStreamSynchronize(b)); break;
      }
      const auto t1 = now();
      CK(hipDeviceSynchronize());
      printf("%s  %-45s %9.2f ms\n", load ? "under load" : "idle      ", names[t], ms(t0, t1));
      fflush(stdout);
    }
  }
  return 0;
}
