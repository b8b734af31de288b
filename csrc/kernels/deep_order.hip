// Level-3 task order of the deep miner on the device (csrc/host/deep_run.hip, assign = 1): the
// tasks sorted by estimated cost, largest first and stable in the task id, then dealt over the
// ranks in snake order.  Every rank computes the same order (a deterministic radix sort of a
// composite key), so the ranks' shares partition the tasks.  Replaces a host counting sort
// behind a device->host copy of the costs and a stream synchronisation on every call.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "kernels.hpp"
#include "kmls/common.hpp"

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

constexpr uint64_t kCostMask = 0xFFFFull;  // costs saturate at 65535 (class sizes are smaller)

// key = (kKeyMax - min(c, kKeyMax)) << 32 | t, c = by[t] (the cost, or a separate deal key):
// ascending keys = descending c, ascending t
constexpr uint64_t kKeyMax = 0xFFFFFFFFull;
__global__ void k_order_keys(const uint32_t* __restrict__ by, int64_t T, uint64_t* __restrict__ key) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < T;
       t += (int64_t)gridDim.x * blockDim.x)
    key[t] = ((kKeyMax - (uint64_t)by[t]) << 32) | (uint64_t)t;
}

// this rank's j-th task: sorted position q(j) = j * world + (j odd ? world - 1 - rank : rank)
__global__ void k_order_deal(const uint64_t* __restrict__ sorted, const uint32_t* __restrict__ cost,
                             int64_t T, int rank, int world, int64_t n,
                             int64_t* __restrict__ order, uint32_t* __restrict__ ocost) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = j * world + ((j & 1) ? world - 1 - rank : rank);
    const uint64_t t = sorted[q] & 0xFFFFFFFFull;
    order[j] = (int64_t)t;
    ocost[j] = std::min<uint32_t>(cost[t], (uint32_t)kCostMask);
  }
}

size_t cub_bytes(int64_t T) {
  size_t b = 0;
  KMLS_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, b, (const uint64_t*)nullptr,
                                             (uint64_t*)nullptr, (int)T, 0, 64));
  return b;
}

}  // namespace

int64_t deep_task_share(int64_t T, int rank, int world) {
  // q(j) is increasing (q(j + 1) >= (j + 1) * world > q(j)): count the positions below T
  int64_t n = 0;
  while (n * world + ((n & 1) ? world - 1 - rank : rank) < T) ++n;
  return n;
}

size_t deep_task_order_bytes(int64_t T) {
  return (size_t)std::max<int64_t>(T, 1) * 16 + cub_bytes(std::max<int64_t>(T, 1)) + 256;
}

int64_t deep_task_order(const uint32_t* cost, int64_t T, int rank, int world, void* tmp,
                        size_t tmp_bytes, int64_t* order, uint32_t* order_cost, hipStream_t s,
                        const uint32_t* key) {
  if (T <= 0) return 0;
  KMLS_CHECK(T < ((int64_t)1 << 32), "deep_task_order: task ids must fit 32 bits");
  KMLS_CHECK(tmp_bytes >= deep_task_order_bytes(T), "deep_task_order: scratch too small");
  uint64_t* keys = (uint64_t*)tmp;
  uint64_t* sorted = keys + T;
  void* cub = (void*)(((uintptr_t)(sorted + T) + 255) & ~(uintptr_t)255);
  size_t cb = cub_bytes(T);
  const unsigned g = (unsigned)std::min<int64_t>((T + 255) / 256, 2048);
  hipLaunchKernelGGL(k_order_keys, dim3(g), dim3(256), 0, s, key ? key : cost, T, keys);
  KMLS_HIP(hipGetLastError());
  // 64 key bits: the 32-bit task id and the 32-bit inverted cost / deal key
  KMLS_HIP(hipcub::DeviceRadixSort::SortKeys(cub, cb, keys, sorted, (int)T, 0, 64, s));
  const int64_t n = deep_task_share(T, rank, world);
  if (n > 0) {
    const unsigned g2 = (unsigned)std::min<int64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_order_deal, dim3(g2), dim3(256), 0, s, sorted, cost, T, rank, world, n,
                       order, order_cost);
    KMLS_HIP(hipGetLastError());
  }
  return n;
}

}  // namespace kern
}  // namespace kmls
