// fileread_bench.cpp -- how fast can one process move a FASTQ file from the page cache to the GPU?
// (VERDICT r04 "file-read ceiling": the CLI's pread into pinned buffers ran at 4.4-5.4 GB/s on 16
// threads.)  Writes a file of --gb GiB under a directory (default $TMPDIR or /tmp), then times, each
// over the whole file:
//   pread_malloc   T threads pread() into a pre-faulted malloc'd buffer (1 GiB pieces)
//   pread_pinned   the same into hipHostMalloc'd memory (the CLI's path)
//   mmap_memcpy    mmap of the file, T threads memcpy into pinned memory
//   register_h2d   mmap + hipHostRegister of the mapping (read only) + one hipMemcpy to the device:
//                  the copy engine reads the page cache pages directly, no CPU copy
//   pinned_h2d     hipMemcpy of an already pinned buffer to the device (PCIe / SDMA ceiling)
//   odirect_pinned O_DIRECT pread into pinned memory (bypasses the page cache; may be refused)
// Prints one JSON line.  Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -o fileread_bench
// fileread_bench.cpp -pthread
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <unistd.h>

#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void par(int T, const std::function<void(int)> &f) {
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(f, t);
  f(0);
  for (auto &x : th) x.join();
}

static double pread_into(int fd, char *dst, uint64_t n, int T) {
  const double t0 = now();
  par(T, [&](int t) {
    uint64_t lo = n * t / T, hi = n * (t + 1) / T, p = lo;
    while (p < hi) {
      ssize_t r = pread(fd, dst + p, (size_t)std::min<uint64_t>(hi - p, 1ull << 30), (off_t)p);
      if (r <= 0) break;
      p += (uint64_t)r;
    }
  });
  return now() - t0;
}

int main(int argc, char **argv) {
  double gb = 8;
  int T = 16;
  std::string dir = getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp";
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--gb") && i + 1 < argc) gb = atof(argv[++i]);
    else if (!strcmp(argv[i], "--threads") && i + 1 < argc) T = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--dir") && i + 1 < argc) dir = argv[++i];
  }
  const uint64_t n = (uint64_t)(gb * (1ull << 30)) / 4096 * 4096;
  const std::string fn = dir + "/fileread_bench.dat";
  struct statfs sf;
  long fstype = statfs(dir.c_str(), &sf) == 0 ? (long)sf.f_type : -1;
  // write the file (FASTQ-like bytes), T threads
  {
    int fd = open(fn.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, (off_t)n) != 0) { perror("create"); return 1; }
    const double t0 = now();
    par(T, [&](int t) {
      std::vector<char> b(1 << 24);
      for (size_t i = 0; i < b.size(); ++i) b[i] = "ACGT\n@+I"[(i * 2654435761u >> 7) & 7];
      uint64_t lo = n * t / T / 4096 * 4096, hi = t == T - 1 ? n : n * (t + 1) / T / 4096 * 4096;
      for (uint64_t p = lo; p < hi;) {
        size_t m = (size_t)std::min<uint64_t>(hi - p, b.size());
        ssize_t w = pwrite(fd, b.data(), m, (off_t)p);
        if (w <= 0) break;
        p += (uint64_t)w;
      }
    });
    fprintf(stderr, "wrote %.1f GiB in %.2f s\n", n / 1073741824.0, now() - t0);
    close(fd);
  }
  int fd = open(fn.c_str(), O_RDONLY);
  std::string js = "{\"bytes\": " + std::to_string(n) + ", \"threads\": " + std::to_string(T) + ", \"fs_type\": \"0x" +
                   [&] { char b[32]; snprintf(b, sizeof b, "%lx", fstype); return std::string(b); }() + "\"";
  auto rec = [&](const char *k, double s) {
    char b[128];
    snprintf(b, sizeof b, ", \"%s_GBps\": %.2f", k, n / s / 1e9);
    js += b;
    fprintf(stderr, "%-16s %.3f s  %.2f GB/s\n", k, s, n / s / 1e9);
  };
  {  // pread -> malloc
    char *m = (char *)aligned_alloc(4096, n);
    par(T, [&](int t) { memset(m + n * t / T, 0, n * (t + 1) / T - n * t / T); });
    pread_into(fd, m, n, T);  // warm the page cache
    rec("pread_malloc", pread_into(fd, m, n, T));
    rec("pread_malloc_1thr", pread_into(fd, m, n, 1));
    free(m);
  }
  char *pin = nullptr;
  if (hipHostMalloc((void **)&pin, n, hipHostMallocDefault) != hipSuccess) { fprintf(stderr, "hipHostMalloc failed\n"); return 1; }
  rec("pread_pinned", pread_into(fd, pin, n, T));
  rec("pread_pinned_again", pread_into(fd, pin, n, T));
  {
    char *mp = (char *)mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    if (mp != MAP_FAILED) {
      double t0 = now();
      par(T, [&](int t) { memcpy(pin + n * t / T, mp + n * t / T, n * (t + 1) / T - n * t / T); });
      rec("mmap_memcpy", now() - t0);
      t0 = now();
      par(T, [&](int t) { memcpy(pin + n * t / T, mp + n * t / T, n * (t + 1) / T - n * t / T); });
      rec("mmap_memcpy_again", now() - t0);
      void *dv = nullptr;
      if (hipMalloc(&dv, n) == hipSuccess) {
        t0 = now();
        hipError_t e = hipHostRegister(mp, n, hipHostRegisterReadOnly);
        const double treg = now() - t0;
        if (e == hipSuccess) {
          const double t1 = now();
          e = hipMemcpy(dv, mp, n, hipMemcpyHostToDevice);
          const double tc = now() - t1;
          rec("register_h2d_total", now() - t0);
          rec("register_h2d_copy", tc);
          char b[96];
          snprintf(b, sizeof b, ", \"register_s\": %.3f, \"register_copy_ok\": %d", treg, e == hipSuccess);
          js += b;
          (void)hipHostUnregister(mp);
        } else {
          js += ", \"register_error\": \"" + std::string(hipGetErrorString(e)) + "\"";
          fprintf(stderr, "hipHostRegister: %s\n", hipGetErrorString(e));
        }
        t0 = now();
        (void)hipMemcpy(dv, pin, n, hipMemcpyHostToDevice);
        rec("pinned_h2d", now() - t0);
        (void)hipFree(dv);
      }
      munmap(mp, n);
    }
  }
  {
    int fdd = open(fn.c_str(), O_RDONLY | O_DIRECT);
    if (fdd >= 0) {
      const double s = pread_into(fdd, pin, n, T);
      rec("odirect_pinned", s);
      close(fdd);
    } else {
      js += ", \"odirect\": \"refused\"";
    }
  }
  (void)hipHostFree(pin);
  close(fd);
  unlink(fn.c_str());
  js += "}";
  printf("%s\n", js.c_str());
  return 0;
}
