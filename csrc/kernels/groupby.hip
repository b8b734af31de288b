// O2 groupby_csr on the GPU: the job's transaction builder
// (machine-learning/main.py:195-207, polars group_by(pid).agg(list(track_name))) as
// radix sort of (key << 32 | value) composites → optional unique → per-key histogram → scan.
// Output = CSR with rows sorted and duplicate-free, identical to the host group_to_csr(dedup,
// sort_rows).  Worth it at the 100M-playlist scale (billions of rows); the host path stays the
// default for ds-sized inputs where the PCIe round trip dominates.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdexcept>
#include <string>

#include "kernels.hpp"

#define KMLS_HIP(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__));     \
  } while (0)

namespace kmls {
namespace kern {

namespace {

__global__ void k_compose(const int32_t* __restrict__ keys, const int32_t* __restrict__ vals,
                          int64_t n, unsigned long long* __restrict__ out) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr)
    out[i] = ((unsigned long long)(uint32_t)keys[i] << 32) | (uint32_t)vals[i];
}

__global__ void k_split_count(const unsigned long long* __restrict__ comp, const int64_t* n_ptr,
                              int32_t* __restrict__ vals_out, int64_t* __restrict__ key_count) {
  const int64_t n = *n_ptr;
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr) {
    const unsigned long long c = comp[i];
    vals_out[i] = (int32_t)(uint32_t)(c & 0xFFFFFFFFull);
    atomicAdd((unsigned long long*)&key_count[c >> 32], 1ull);
  }
}

int grid_of(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256)); }

}  // namespace

int64_t groupby_csr(const int32_t* d_keys, const int32_t* d_vals, int64_t n, int32_t n_keys,
                    bool dedup, int64_t* d_ptr, int32_t* d_idx, void* d_tmp, size_t tmp_bytes,
                    hipStream_t s) {
  // scratch layout: comp_in[n] | comp_out[n] | n_out | key_count[n_keys+1] | cub temp
  char* p = (char*)d_tmp;
  auto* comp_in = (unsigned long long*)p;
  p += ((size_t)n * 8 + 255) & ~(size_t)255;
  auto* comp_out = (unsigned long long*)p;
  p += ((size_t)n * 8 + 255) & ~(size_t)255;
  auto* n_out = (int64_t*)p;
  p += 256;
  auto* key_count = (int64_t*)p;
  p += ((size_t)(n_keys + 1) * 8 + 255) & ~(size_t)255;
  const size_t used = (size_t)(p - (char*)d_tmp);
  if (used > tmp_bytes) throw std::runtime_error("groupby_csr: scratch too small");
  void* cub_tmp = p;
  size_t cub_bytes = tmp_bytes - used;
  hipLaunchKernelGGL(k_compose, dim3(grid_of(n)), dim3(256), 0, s, d_keys, d_vals, n, comp_in);
  KMLS_HIP(hipGetLastError());
  KMLS_HIP(hipcub::DeviceRadixSort::SortKeys(cub_tmp, cub_bytes, comp_in, comp_out, (int)n, 0, 64, s));
  const unsigned long long* sorted = comp_out;
  if (dedup) {
    cub_bytes = tmp_bytes - used;
    KMLS_HIP(hipcub::DeviceSelect::Unique(cub_tmp, cub_bytes, comp_out, comp_in, n_out, (int)n, s));
    sorted = comp_in;
  } else {
    KMLS_HIP(hipMemcpyAsync(n_out, &n, 8, hipMemcpyHostToDevice, s));
  }
  KMLS_HIP(hipMemsetAsync(key_count, 0, (size_t)(n_keys + 1) * 8, s));
  hipLaunchKernelGGL(k_split_count, dim3(grid_of(n)), dim3(256), 0, s, sorted, n_out, d_idx, key_count);
  KMLS_HIP(hipGetLastError());
  cub_bytes = tmp_bytes - used;
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(cub_tmp, cub_bytes, key_count, d_ptr, (int)(n_keys + 1), s));
  int64_t total = 0;
  KMLS_HIP(hipMemcpyAsync(&total, d_ptr + n_keys, 8, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  return total;
}

size_t groupby_csr_temp_bytes(int64_t n, int32_t n_keys) {
  size_t a = 0, b = 0, c = 0;
  KMLS_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, a, (const unsigned long long*)nullptr,
                                             (unsigned long long*)nullptr, (int)n, 0, 64));
  KMLS_HIP(hipcub::DeviceSelect::Unique(nullptr, b, (const unsigned long long*)nullptr,
                                        (unsigned long long*)nullptr, (int64_t*)nullptr, (int)n));
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, c, (const int64_t*)nullptr, (int64_t*)nullptr,
                                            (int)(n_keys + 1)));
  const size_t fixed = 2 * (((size_t)n * 8 + 255) & ~(size_t)255) + 256 +
                       (((size_t)(n_keys + 1) * 8 + 255) & ~(size_t)255);
  return fixed + std::max(a, std::max(b, c)) + 256;
}

}  // namespace kern
}  // namespace kmls
