// Emit-mode node arena of the deep miner -> the product trie (parents before children).
//
// The deep miner (deep.hip, emit) writes every frequent itemset as a node (parent node id, item
// rank, support, size) at ids taken in per-wave chunks, so the arena has holes (size 0) and a
// child may hold a smaller id than its parent (a stolen frame's wave took its chunk earlier).
// The reference hands the mined itemsets to the rule-map loop and the artifacts
// (machine-learning/main.py:262-313); those consumers — and the ItemsetTrie of this package —
// want a dense trie whose parents precede their children.  Three passes turn the arena into one,
// entirely on the device:
//   1. count:   per unit of kTrieUnit consecutive ids (one wave), nodes per size (LDS histogram)
//               -> cnt[size][unit];
//   2. scan:    exclusive prefix of cnt in (size, unit) order (hipCUB) = the first new id of each
//               (size, unit) run: size-major, arena order inside a size (deterministic);
//   3. rank:    each wave re-walks its unit 64 ids at a time; the lanes of one size are ranked
//               by a ballot (wave-uniform loop over the sizes present in the 64 ids) -> new_id;
//   4. scatter: parent remapped through new_id, item rank -> original item id, support to u16,
//               size; written at new_id in the narrowest exact widths the host trie keeps.
// Sizes below min_depth are left out (a rank > 0 of a split exports only its share, sizes >= 3;
// its parents of size 2 keep their arena id, which is the same on every rank and equals their
// id in rank 0's export: levels 1-2 occupy ids [0, F + pairs) densely in size order).
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

constexpr int kTrieUnit = 8192;  // arena ids per wave unit
constexpr int kTrieWaves = 4;    // waves per 256-thread block
constexpr unsigned kNone = 0xffffffffu;

__global__ __launch_bounds__(256) void k_trie_count(const unsigned char* __restrict__ depth,
                                                    int64_t n, int min_depth, int nd,
                                                    int64_t n_units, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[kTrieWaves][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t u = (int64_t)blockIdx.x * kTrieWaves + wid;
  h[wid][lane] = 0u;
  __builtin_amdgcn_wave_barrier();
  if (u < n_units) {
    const int64_t i0 = u * kTrieUnit;
    const int64_t i1 = i0 + kTrieUnit < n ? i0 + kTrieUnit : n;
    for (int64_t i = i0 + lane; i < i1; i += 64) {
      const int d = depth[i];
      if (d >= min_depth && d < nd) atomicAdd(&h[wid][d], 1u);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < nd) cnt[(int64_t)lane * n_units + u] = h[wid][lane];
  }
}

__global__ __launch_bounds__(256) void k_trie_rank(const unsigned char* __restrict__ depth,
                                                   int64_t n, int min_depth, int nd,
                                                   int64_t n_units,
                                                   const uint32_t* __restrict__ first,
                                                   uint32_t* __restrict__ new_id) {
  __shared__ uint32_t base[kTrieWaves][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t u = (int64_t)blockIdx.x * kTrieWaves + wid;
  if (u >= n_units) return;  // (no block barrier below)
  if (lane < nd) base[wid][lane] = first[(int64_t)lane * n_units + u];
  __builtin_amdgcn_wave_barrier();
  const unsigned long long lanelt = (1ull << lane) - 1ull;
  const int64_t i0 = u * kTrieUnit;
  const int64_t i1 = i0 + kTrieUnit < n ? i0 + kTrieUnit : n;
  for (int64_t c = i0; c < i1; c += 64) {
    const int64_t i = c + lane;
    const int d = i < i1 ? (int)depth[i] : 0;
    const bool v = d >= min_depth && d < nd;
    unsigned long long rem = __ballot(v);
    unsigned id = kNone;
    while (rem) {  // one iteration per size present among these 64 ids (wave-uniform)
      const int d0 = __shfl(d, __builtin_ctzll(rem), 64);
      const unsigned long long m = __ballot(v && d == d0);
      const unsigned b0 = base[wid][d0];
      if (v && d == d0) id = b0 + (unsigned)__popcll(m & lanelt);
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) base[wid][d0] = b0 + (unsigned)__popcll(m);
      __builtin_amdgcn_wave_barrier();
      rem &= ~m;
    }
    if (i < i1) new_id[i] = id;
  }
}

template <typename ItemT>
__global__ __launch_bounds__(256) void k_trie_scatter(
    const unsigned* __restrict__ parent, const unsigned* __restrict__ item,
    const unsigned* __restrict__ count, const unsigned char* __restrict__ depth, int64_t n,
    const uint32_t* __restrict__ new_id, const int32_t* __restrict__ ids, int64_t base,
    int32_t* __restrict__ o_parent, ItemT* __restrict__ o_item, uint16_t* __restrict__ o_count,
    unsigned char* __restrict__ o_depth) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned v = new_id[i];
    if (v == kNone) continue;
    const unsigned p = parent[i];
    int32_t np = -1;
    if (p != kNone) {
      const unsigned q = new_id[p];
      np = q != kNone ? (int32_t)(base + (int64_t)q) : (int32_t)p;  // below min_depth: arena id
    }
    o_parent[v] = np;
    o_item[v] = (ItemT)ids[item[i]];
    o_count[v] = (uint16_t)count[i];
    o_depth[v] = depth[i];
  }
}

size_t scan_bytes(int64_t m) {
  size_t b = 0;
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const uint32_t*)nullptr,
                                            (uint32_t*)nullptr, (int)m));
  return b;
}

}  // namespace

int64_t deep_trie_units(int64_t n) { return (n + kTrieUnit - 1) / kTrieUnit; }

size_t deep_trie_scratch_bytes(int64_t n, int nd) {
  const int64_t m = std::max<int64_t>(deep_trie_units(n) * nd, 1);
  return (size_t)m * 8 + scan_bytes(m) + 512;
}

int64_t deep_trie_layout(const unsigned char* depth, int64_t n, int min_depth, int nd,
                         uint32_t* new_id, void* tmp, size_t tmp_bytes, hipStream_t s) {
  KMLS_CHECK(nd >= 1 && nd <= 64, "deep_trie_layout: sizes must be < 64");
  KMLS_CHECK(n < ((int64_t)1 << 32) - 1, "deep_trie_layout: 2^32 arena ids");
  KMLS_CHECK(tmp_bytes >= deep_trie_scratch_bytes(n, nd), "deep_trie_layout: scratch too small");
  if (n <= 0) return 0;
  const int64_t units = deep_trie_units(n);
  const int64_t m = units * nd;
  uint32_t* cnt = (uint32_t*)tmp;
  uint32_t* first = cnt + m;
  void* cub = (void*)(((uintptr_t)(first + m) + 255) & ~(uintptr_t)255);
  size_t cb = scan_bytes(m);
  const unsigned blocks = (unsigned)((units + kTrieWaves - 1) / kTrieWaves);
  hipLaunchKernelGGL(k_trie_count, dim3(blocks), dim3(256), 0, s, depth, n, min_depth, nd, units,
                     cnt);
  KMLS_HIP(hipGetLastError());
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(cub, cb, cnt, first, (int)m, s));
  hipLaunchKernelGGL(k_trie_rank, dim3(blocks), dim3(256), 0, s, depth, n, min_depth, nd, units,
                     first, new_id);
  KMLS_HIP(hipGetLastError());
  uint32_t last[2] = {0, 0};
  KMLS_HIP(hipMemcpyAsync(&last[0], first + m - 1, 4, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipMemcpyAsync(&last[1], cnt + m - 1, 4, hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  return (int64_t)last[0] + (int64_t)last[1];
}

void deep_trie_scatter(const unsigned* parent, const unsigned* item, const unsigned* count,
                       const unsigned char* depth, int64_t n, const uint32_t* new_id,
                       const int32_t* ids, int64_t base, int32_t* o_parent, void* o_item,
                       bool item16, uint16_t* o_count, unsigned char* o_depth, hipStream_t s) {
  if (n <= 0) return;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
  if (item16)
    hipLaunchKernelGGL(k_trie_scatter<uint16_t>, dim3(g), dim3(256), 0, s, parent, item, count,
                       depth, n, new_id, ids, base, o_parent, (uint16_t*)o_item, o_count, o_depth);
  else
    hipLaunchKernelGGL(k_trie_scatter<int32_t>, dim3(g), dim3(256), 0, s, parent, item, count,
                       depth, n, new_id, ids, base, o_parent, (int32_t*)o_item, o_count, o_depth);
  KMLS_HIP(hipGetLastError());
}

}  // namespace kern
}  // namespace kmls
