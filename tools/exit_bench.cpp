// exit_bench.cpp -- what process exit costs with large pinned host buffers and device allocations
// (the `ibwa-amd aln` wall clock had ~0.7-0.9 s after its last phase).  The process allocates
// PIN_GB of pinned host memory (hipHostMalloc, touched) and DEV_GB of device memory (one hipMalloc),
// optionally frees them itself (FREE=1: hipHostFree / hipFree, timed), prints the time since start,
// and _exits; the parent times the whole process.
//   exit_bench PIN_GB DEV_GB FREE
// Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -o exit_bench exit_bench.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>

int main(int argc, char **argv) {
  const auto t0 = std::chrono::steady_clock::now();
  auto ms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  const double pin_gb = argc > 1 ? atof(argv[1]) : 0, dev_gb = argc > 2 ? atof(argv[2]) : 0;
  const int do_free = argc > 3 ? atoi(argv[3]) : 0;
  (void)hipFree(nullptr);
  const double t_init = ms();
  void *h = nullptr, *d = nullptr;
  const size_t hb = (size_t)(pin_gb * (1ull << 30)), db = (size_t)(dev_gb * (1ull << 30));
  if (hb && hipHostMalloc(&h, hb, hipHostMallocDefault) == hipSuccess) memset(h, 1, hb);
  const double t_pin = ms();
  if (db) (void)hipMalloc(&d, db);
  const double t_dev = ms();
  double t_free_h = 0, t_free_d = 0;
  if (do_free) {
    const double a = ms();
    if (h) (void)hipHostFree(h);
    t_free_h = ms() - a;
    const double b = ms();
    if (d) (void)hipFree(d);
    t_free_d = ms() - b;
  }
  printf("{\"pin_gb\": %.1f, \"dev_gb\": %.1f, \"free\": %d, \"init_ms\": %.0f, \"pin_ms\": %.0f, \"dev_ms\": %.0f, "
         "\"host_free_ms\": %.0f, \"dev_free_ms\": %.0f, \"before_exit_ms\": %.0f}\n",
         pin_gb, dev_gb, do_free, t_init, t_pin - t_init, t_dev - t_pin, t_free_h, t_free_d, ms());
  fflush(stdout);
  _exit(0);
}
