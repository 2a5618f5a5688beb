// alloc_bench.cpp -- what a hipMalloc costs right after another process released a lot of HBM
// (`aln` end 2 found single allocations taking 2.3-2.8 s after end 1 exited).
//   alloc_bench hold GB        allocate GB in 8 GiB blocks, write them, exit (the "previous process")
//   alloc_bench probe GB BLK   allocate GB in BLK-GiB blocks, report each block's time, then free
//                              them and allocate the same again (the same process's own frees)
// Prints one JSON line per run.  Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -o alloc_bench alloc_bench.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  const double gb = atof(argv[2]);
  const bool hold = !strcmp(argv[1], "hold");
  const double blk_gb = argc > 3 ? atof(argv[3]) : 8.0;
  const size_t blk = (size_t)(blk_gb * (1ull << 30));
  const int nb = (int)(gb / blk_gb + 0.5);
  std::string js = std::string("{\"mode\": \"") + argv[1] + "\", \"gb\": " + std::to_string(gb) + ", \"block_gb\": " +
                   std::to_string(blk_gb) + ", \"ms\": [";
  const auto t0 = std::chrono::steady_clock::now();
  (void)hipFree(nullptr);
  const double init_ms = ms_since(t0);
  std::vector<void *> p(nb, nullptr);
  double tot = 0;
  for (int i = 0; i < nb; ++i) {
    const auto t = std::chrono::steady_clock::now();
    if (hipMalloc(&p[i], blk) != hipSuccess) { fprintf(stderr, "hipMalloc %d failed\n", i); return 1; }
    const double ms = ms_since(t);
    tot += ms;
    js += (i ? ", " : "") + std::to_string((int)ms);
    if (hold) (void)hipMemset(p[i], 0x5a, blk);
  }
  (void)hipDeviceSynchronize();
  js += "], \"total_ms\": " + std::to_string((int)tot) + ", \"init_ms\": " + std::to_string((int)init_ms);
  if (!hold) {
    for (auto x : p) (void)hipFree(x);
    const auto t = std::chrono::steady_clock::now();
    for (auto &x : p) (void)hipMalloc(&x, blk);
    js += ", \"realloc_same_process_ms\": " + std::to_string((int)ms_since(t));
    for (auto x : p) (void)hipFree(x);
  }
  js += "}";
  printf("%s\n", js.c_str());
  return 0;
}
