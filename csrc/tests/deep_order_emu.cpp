// The CPU wave emulator's stand-in for kern::deep_task_order (csrc/kernels/deep_order.hip, a
// hipCUB radix sort the emulator cannot compile): the same order — tasks by cost descending,
// stable in the task id, snake-dealt over the ranks — over the emulator's host-resident
// "device" memory.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <numeric>
#include <vector>

#include <hip/hip_runtime.h>

#include "../kernels/kernels.hpp"

namespace kmls {
namespace kern {

// stand-in for the popcount bit-GEMM (mine.hip): out[i][j] = |row i & row j| for i < j
void pair_gram_popcount(const uint64_t* bm, int64_t Wp, int64_t F, uint32_t* out, hipStream_t) {
  for (int64_t i = 0; i < F; ++i)
    for (int64_t j = i + 1; j < F; ++j) {
      uint32_t c = 0;
      for (int64_t w = 0; w < Wp; ++w) c += (uint32_t)__builtin_popcountll(bm[i * Wp + w] & bm[j * Wp + w]);
      out[i * F + j] = c;
    }
}

bool pair_gram_dev_needs_zero(int64_t, int64_t) { return false; }

int64_t deep_task_share(int64_t T, int rank, int world) {
  int64_t n = 0;
  while (n * world + ((n & 1) ? world - 1 - rank : rank) < T) ++n;
  return n;
}

size_t deep_task_order_bytes(int64_t T) { return (size_t)std::max<int64_t>(T, 1) * 8; }

int64_t deep_task_order(const uint32_t* cost, int64_t T, int rank, int world, void*, size_t,
                        int64_t* order, uint32_t* order_cost, hipStream_t, const uint32_t* by) {
  if (T <= 0) return 0;
  std::vector<int64_t> idx((size_t)T);
  std::iota(idx.begin(), idx.end(), 0);
  const uint32_t* k = by ? by : cost;  // the deal key (or the cost)
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return k[a] > k[b]; });
  const int64_t n = deep_task_share(T, rank, world);
  for (int64_t j = 0; j < n; ++j) {
    const int64_t q = j * world + ((j & 1) ? world - 1 - rank : rank);
    order[j] = idx[(size_t)q];
    order_cost[j] = std::min<uint32_t>(cost[idx[(size_t)q]], 0xFFFFu);
  }
  return n;
}

}  // namespace kern
}  // namespace kmls
