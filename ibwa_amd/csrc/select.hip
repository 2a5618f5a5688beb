// select.hip -- the reads a search pass handed on, selected on the device.
//
// After the first gapped pass every read has a status word (0: done); the reads with a
// non-zero status go on to the cooperative / wide / general passes (bwa_cal_sa_reg_gap's results
// are per read, so which pass resolves a read changes nothing in its output).  Their ids, in
// input order, and their statuses are compacted here (rocPRIM select), so the host copies a few
// MB instead of two words per read of the batch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <rocprim/rocprim.hpp>

#include "engine.h"

namespace ibwa {

namespace {

struct NonZero {
  __host__ __device__ bool operator()(uint32_t s) const { return s != 0u; }
};
struct NonZero64 {
  __host__ __device__ bool operator()(uint64_t s) const { return s != 0u; }
};

// after a cooperative launch over resumed reads: a resolved read is done (status 0); one the pass
// handed on loses its state (the later passes run it from the start)
__global__ void k_resume_fixup(const uint32_t *r_status, const int64_t *ids, int64_t n, uint32_t *status,
                               uint64_t *roff) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = ids[i];
    if (r_status[i] == 0u) status[r] = 0u;
    else roff[r] = 0u;
  }
}

__global__ void k_gather_status(const uint32_t *status, const int64_t *ids, const unsigned long long *count,
                                uint32_t *out) {
  const unsigned long long m = *count;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = status[ids[i]];
}

__global__ void k_order_keys(const uint32_t *sel_status, unsigned long long n, uint32_t *keys, uint32_t *idx) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    keys[i] = 0xFFFFu - (sel_status[i] >> 16);  // ascending sort = largest stack first
    idx[i] = (uint32_t)i;
  }
}

__global__ void k_gather_ids(const int64_t *ids, const uint32_t *perm, unsigned long long n, int64_t *out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = ids[perm[i]];
}

}  // namespace

hipError_t select_resumed(const uint64_t *roff, int64_t base, int64_t n, const uint32_t *status, int64_t *ids,
                          uint32_t *sel_status, unsigned long long *d_count, void *tmp, size_t *tmp_bytes,
                          hipStream_t st) {
  auto in = rocprim::make_counting_iterator<int64_t>(base);
  auto flags = rocprim::make_transform_iterator(roff + base, NonZero64());
  if (!tmp) return rocprim::select(nullptr, *tmp_bytes, in, flags, ids, d_count, (size_t)n, st);
  hipError_t e = rocprim::select(tmp, *tmp_bytes, in, flags, ids, d_count, (size_t)n, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_gather_status, dim3(1024), dim3(256), 0, st, status, ids, d_count, sel_status);
  return hipGetLastError();
}

hipError_t resume_fixup(const uint32_t *r_status, const int64_t *ids, int64_t n, uint32_t *status, uint64_t *roff,
                        hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_resume_fixup, dim3(1024), dim3(256), 0, st, r_status, ids, n, status, roff);
  return hipGetLastError();
}

hipError_t order_heavy_first(const uint32_t *sel_status, const int64_t *ids, unsigned long long n, uint32_t *keys,
                             uint32_t *idx, int64_t *ids_out, void *tmp, size_t *tmp_bytes, hipStream_t st) {
  // keys / idx hold 2n entries each (double buffers); on return idx[0, n) is the order
  rocprim::double_buffer<uint32_t> kb(keys, keys + n), vb(idx, idx + n);
  if (!tmp) return rocprim::radix_sort_pairs(nullptr, *tmp_bytes, kb, vb, (size_t)n, 0, 16, st);
  hipLaunchKernelGGL(k_order_keys, dim3(1024), dim3(256), 0, st, sel_status, n, keys, idx);
  hipError_t e = rocprim::radix_sort_pairs(tmp, *tmp_bytes, kb, vb, (size_t)n, 0, 16, st);
  if (e != hipSuccess) return e;
  if (vb.current() != idx) e = hipMemcpyAsync(idx, vb.current(), n * 4, hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_gather_ids, dim3(1024), dim3(256), 0, st, ids, idx, n, ids_out);
  return hipGetLastError();
}

hipError_t select_handed_on(const uint32_t *status, int64_t n, int64_t *ids, uint32_t *sel_status,
                            unsigned long long *d_count, void *tmp, size_t *tmp_bytes, hipStream_t st) {
  auto in = rocprim::make_counting_iterator<int64_t>(0);
  auto flags = rocprim::make_transform_iterator(status, NonZero());
  if (!tmp) return rocprim::select(nullptr, *tmp_bytes, in, flags, ids, d_count, (size_t)n, st);
  hipError_t e = rocprim::select(tmp, *tmp_bytes, in, flags, ids, d_count, (size_t)n, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_gather_status, dim3(1024), dim3(256), 0, st, status, ids, d_count, sel_status);
  return hipGetLastError();
}

}  // namespace ibwa
