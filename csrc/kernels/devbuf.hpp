// Device-side building blocks shared by the sparse (CSR-driven) level kernels: grow-only device
// buffers, a hipCUB exclusive scan, wave-aggregated slot allocation, and the frequent-rank CSR
// filter (pairrows.hip builds it for the level-2 row count, hlevels.hip re-filters it).
#pragma once

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "kmls/common.hpp"

namespace kmls {
namespace kern {
namespace devbuf {

inline void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " at " + what);
}

template <typename T>
struct Buf {  // grow-only (25 % headroom), kept across calls
  T* p = nullptr;
  size_t cap = 0;
  void need(size_t n) {
    if (n <= cap) return;
    if (p) hip_ok(hipFree(p), "Buf free");
    p = nullptr;
    const size_t c = std::max<size_t>(n + (n >> 2), 1024);
    hip_ok(hipMalloc((void**)&p, c * sizeof(T)), "Buf alloc");
    cap = c;
  }
  Buf() = default;
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  ~Buf() {
    if (p) (void)hipFree(p);
  }
};

// exclusive prefix sum of m u32 values through a grow-only scratch buffer
inline void scan_u32(const uint32_t* in, uint32_t* out, int64_t m, Buf<uint8_t>& tmp, hipStream_t s) {
  KMLS_CHECK(m < (1ll << 31), "scan past 2^31 elements");
  size_t b = 0;
  hip_ok(hipcub::DeviceScan::ExclusiveSum(nullptr, b, in, out, (int)m), "scan size");
  tmp.need(b + 256);
  hip_ok(hipcub::DeviceScan::ExclusiveSum(tmp.p, b, in, out, (int)m, s), "scan");
}

inline void scan_u64(const unsigned long long* in, unsigned long long* out, int64_t m,
                     Buf<uint8_t>& tmp, hipStream_t s) {
  KMLS_CHECK(m < (1ll << 31), "scan past 2^31 elements");
  size_t b = 0;
  hip_ok(hipcub::DeviceScan::ExclusiveSum(nullptr, b, in, out, (int)m), "scan size");
  tmp.need(b + 256);
  hip_ok(hipcub::DeviceScan::ExclusiveSum(tmp.p, b, in, out, (int)m, s), "scan");
}

namespace {  // kernels and device helpers: one copy per translation unit

// Wave-aggregated slot allocation: one atomic per wave (and per call) for the active lanes that
// want a slot.  Every active lane must call it (it contains a ballot).
__device__ __forceinline__ unsigned long long wave_alloc(bool want, unsigned long long* ctr) {
  const unsigned long long m = __ballot(want);
  if (m == 0ull) return 0ull;
  const int lane = (int)(threadIdx.x & 63);
  const int leader = __builtin_ctzll(m);
  unsigned long long base = 0ull;
  if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(m));
  base = __shfl(base, leader, 64);
  return base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
}

// item id -> rank (16-bit, F <= 32768) for the ranks with keep[r] != 0 (keep == nullptr: all);
// the map starts at -1 (memset 0xFF)
__global__ void k_rank_map(const int32_t* __restrict__ ids, int64_t F, const uint8_t* __restrict__ keep,
                           int16_t* __restrict__ pr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < F && (keep == nullptr || keep[r])) pr[ids[r]] = (int16_t)r;
}

// Slots of a compacted CSR from ONE packed counter (transactions << 36 | items): a wave's rows
// and their items are reserved by the same atomic, so the item array stays in row order (row
// blocks own contiguous item ranges).  Every lane of the wave calls it.
constexpr int kPackShift = 36;
constexpr unsigned long long kPackMask = (1ull << kPackShift) - 1ull;
__device__ __forceinline__ void packed_alloc(bool want, uint32_t n, unsigned long long* ctr, int lane,
                                             unsigned long long* row, unsigned long long* item) {
  const unsigned long long m = __ballot(want);
  uint32_t incl = n;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  const uint32_t tot = __shfl(incl, 63, 64);
  unsigned long long old = 0;
  if (lane == 0 && m) old = atomicAdd(ctr, ((unsigned long long)__popcll(m) << kPackShift) + tot);
  old = __shfl(old, 0, 64);
  *row = (old >> kPackShift) + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
  *item = (old & kPackMask) + incl - n;
}

// Thread per row of a rank CSR (txrec, fit): the ranks r with keep[r], order kept; rows with >=
// min_keep of them compacted through the packed counter (counts past the capacities as above)
__global__ __launch_bounds__(256) void k_csr_refilter(
    const uint2* __restrict__ in_rec, int64_t n, const uint16_t* __restrict__ in_fit,
    const uint8_t* __restrict__ keep, uint32_t min_keep, uint2* __restrict__ txrec,
    uint16_t* __restrict__ fit, unsigned long long* ctr, unsigned long long tx_cap,
    unsigned long long nnz_cap) {
  const int lane = threadIdx.x & 63;
  for (int64_t t0 = (int64_t)blockIdx.x * blockDim.x; t0 < n; t0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = t0 + threadIdx.x;
    uint2 rec = make_uint2(0u, 0u);
    if (t < n) rec = in_rec[t];
    const uint16_t* it = in_fit + rec.x;
    uint32_t kept = 0;
    for (uint32_t j = 0; j < rec.y; ++j) kept += keep[it[j]] ? 1u : 0u;
    const bool want = kept >= min_keep;
    unsigned long long ti, off;
    packed_alloc(want, want ? kept : 0u, ctr, lane, &ti, &off);
    if (want && ti < tx_cap && off + kept <= nnz_cap) {
      txrec[ti] = make_uint2((uint32_t)off, kept);
      uint32_t q = 0;
      for (uint32_t j = 0; j < rec.y; ++j) {
        const uint16_t r = it[j];
        if (keep[r]) fit[off + q++] = r;
      }
    }
  }
}

constexpr int kSortRegs = 16;  // mapped items a thread sorts in registers (longer: in place)
constexpr int kFU = 4;         // items read per step, their gathers in flight together

// Thread per transaction: its mapped items (pr[item] >= 0) as ranks, ascending — a 16-entry
// register insertion network; longer rows are sorted in place in their output slot.
// Transactions with >= min_keep of them get a slot (off, len) and their ranks, through the packed
// counter ctr[0] (transactions << 36 | items), which counts past the capacities, so the caller can
// re-run with the exact sizes.  err |= 1: a row kept > 65535 items; |= 2: a row holds an item twice.
__global__ __launch_bounds__(256) void k_map_filter(
    const int64_t* __restrict__ tx_ptr, const int32_t* __restrict__ items, int64_t n_tx,
    const int16_t* __restrict__ pr, uint32_t min_keep, uint2* __restrict__ txrec,
    uint16_t* __restrict__ fit, unsigned long long* ctr, unsigned long long tx_cap,
    unsigned long long nnz_cap, unsigned* err) {
  const int lane = threadIdx.x & 63;
  for (int64_t t0 = (int64_t)blockIdx.x * blockDim.x; t0 < n_tx; t0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = t0 + threadIdx.x;
    uint32_t v[kSortRegs];
#pragma unroll
    for (int q = 0; q < kSortRegs; ++q) v[q] = 0xFFFFFFFFu;
    uint32_t kept = 0;
    int64_t s = 0, e = 0;
    if (t < n_tx) {
      s = tx_ptr[t];
      e = tx_ptr[t + 1];
      for (int64_t p0 = s; p0 < e; p0 += kFU) {
        int32_t it[kFU];
#pragma unroll
        for (int u = 0; u < kFU; ++u) it[u] = p0 + u < e ? items[p0 + u] : -1;
        int32_t r[kFU];
#pragma unroll
        for (int u = 0; u < kFU; ++u) r[u] = it[u] >= 0 ? (int32_t)pr[it[u]] : -1;
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
          if (r[u] < 0) continue;
          uint32_t x = (uint32_t)r[u];
#pragma unroll
          for (int q = 0; q < kSortRegs; ++q) {
            const uint32_t lo = min(v[q], x), hi = max(v[q], x);
            v[q] = lo;
            x = hi;
          }
          ++kept;
        }
      }
    }
    if (kept > 65535u) atomicOr(err, 1u);
    bool dup = false;
#pragma unroll
    for (int q = 0; q + 1 < kSortRegs; ++q) dup |= (uint32_t)(q + 1) < kept && v[q] == v[q + 1];
    if (dup) atomicOr(err, 2u);
    const bool want = kept >= min_keep && kept <= 65535u;
    unsigned long long ti, off;
    packed_alloc(want, want ? kept : 0u, ctr, lane, &ti, &off);
    if (want) {
      if (ti < tx_cap && off + kept <= nnz_cap) {
        txrec[ti] = make_uint2((uint32_t)off, kept);
        uint16_t* dst = fit + off;
        if (kept <= (uint32_t)kSortRegs) {
#pragma unroll
          for (int q = 0; q < kSortRegs; ++q)
            if ((uint32_t)q < kept) dst[q] = (uint16_t)v[q];
        } else {  // long row: write, then insertion-sort in place (rare)
          uint32_t n = 0;
          for (int64_t p = s; p < e; ++p) {
            const int32_t r = pr[items[p]];
            if (r < 0) continue;
            const uint16_t x = (uint16_t)r;
            uint32_t j = n++;
            while (j > 0 && dst[j - 1] > x) {
              dst[j] = dst[j - 1];
              --j;
            }
            if (j > 0 && dst[j - 1] == x) atomicOr(err, 2u);
            dst[j] = x;
          }
        }
      }
    }
  }
}

}  // namespace
}  // namespace devbuf
}  // namespace kern
}  // namespace kmls
