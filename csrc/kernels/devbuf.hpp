// Device-side building blocks shared by the sparse (CSR-driven) level kernels: grow-only device
// buffers, a hipCUB exclusive scan, wave-aggregated slot allocation, and the frequent-rank CSR
// filter (pairrows.hip builds it for the level-2 row count, hlevels.hip re-filters it).
#pragma once

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <kmls/wave.hpp>

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
  // grow keeping the first `used` elements (stream-ordered copy)
  void need_keep(size_t n, size_t used, hipStream_t s) {
    if (n <= cap) return;
    T* old = p;
    const size_t c = std::max<size_t>(n + (n >> 2), 1024);
    hip_ok(hipMalloc((void**)&p, c * sizeof(T)), "Buf alloc");
    if (old && used) hip_ok(hipMemcpyAsync(p, old, used * sizeof(T), hipMemcpyDeviceToDevice, s), "Buf copy");
    if (old) {
      hip_ok(hipStreamSynchronize(s), "Buf sync");
      hip_ok(hipFree(old), "Buf free");
    }
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

// item id -> rank (unsigned 16-bit, F <= kMaxRank16 + 1) for the ranks with keep[r] != 0
// (keep == nullptr: all); the map starts at kNoRank16 (memset 0xFF)
constexpr uint32_t kNoRank16 = 0xFFFFu;
constexpr int64_t kMaxF16 = 65535;  // ranks 0 .. 65534; 0xFFFF marks an item without one
__device__ __forceinline__ int rank16(uint16_t v) { return v == kNoRank16 ? -1 : (int)v; }
__global__ void k_rank_map(const int32_t* __restrict__ ids, int64_t F, const uint8_t* __restrict__ keep,
                           uint16_t* __restrict__ pr) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < F && (keep == nullptr || keep[r])) pr[ids[r]] = (uint16_t)r;
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

// The same slots from a PER-WAVE pool: a wave reserves rows_res rows and items_res items of the
// packed counter at a time and hands them out chunk by chunk.  One atomic per 64-transaction chunk
// on the single counter serialised the 100M-transaction filter: one address takes ~88 atomics per
// microsecond, 1.56M chunks ~18 ms of its 20.  A chunk that does not fit the rest of the wave's
// range abandons that tail (rows left zero: the caller zeroes txrec, so they read as empty
// (0, 0) rows; items never referenced) and reserves a new range; the counter therefore ends past
// the rows/items actually written, and consumers size by it.
struct WavePool {
  unsigned long long r0, r1, i0, i1;
};
// reservation sizes: ~16 chunks' rows per atomic, fewer when a wave gets few chunks (so the
// abandoned tails stay a few % of the output); items from the mean kept per transaction
struct PoolRes {
  uint32_t rows, items;
};
inline PoolRes pool_res(int64_t n_tx, double kept_per_tx, int64_t waves) {
  const int64_t chunks = (n_tx + 63) / 64;
  const int64_t per_wave = std::max<int64_t>(1, chunks / std::max<int64_t>(waves, 1));
  const int64_t k = std::max<int64_t>(1, std::min<int64_t>(16, per_wave / 4));
  const double kept = std::max(kept_per_tx, 2.0);
  PoolRes r;
  r.rows = (uint32_t)(64 * k);
  r.items = (uint32_t)std::min<double>(1u << 30, 64.0 * (double)k * kept * 1.25 + 64.0);
  return r;
}
__device__ __forceinline__ void pool_alloc(bool want, uint32_t n, unsigned long long* ctr, int lane,
                                           WavePool& P, uint32_t rows_res, uint32_t items_res,
                                           unsigned long long* row, unsigned long long* item) {
  const unsigned long long m = __ballot(want);
  uint32_t incl = n;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  const uint32_t tot = __shfl(incl, 63, 64);
  const uint32_t nr = (uint32_t)__popcll(m);
  if (m && (P.r0 + nr > P.r1 || P.i0 + tot > P.i1)) {  // wave-uniform
    const unsigned long long rr = nr > rows_res ? nr : rows_res;
    const unsigned long long ii = tot > items_res ? tot : items_res;
    unsigned long long old = 0;
    if (lane == 0) old = atomicAdd(ctr, (rr << kPackShift) + ii);
    old = __shfl(old, 0, 64);
    P.r0 = old >> kPackShift;
    P.r1 = P.r0 + rr;
    P.i0 = old & kPackMask;
    P.i1 = P.i0 + ii;
  }
  *row = P.r0 + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
  *item = P.i0 + incl - n;
  P.r0 += nr;
  P.i0 += tot;
}

// Thread per row of a rank CSR (txrec, fit): the ranks r with keep[r], order kept; rows with >=
// min_keep of them compacted through the packed counter (counts past the capacities as above).
// A wave takes kRG blocks of 64 rows per reservation (count pass, one atomic, write pass): one
// atomic per 64 rows on the single counter serialised the pass (~1.9 ms for 9.2M rows).
constexpr int kRG = 16;
__global__ __launch_bounds__(256) void k_csr_refilter(
    const uint2* __restrict__ in_rec, int64_t n, const uint16_t* __restrict__ in_fit,
    const uint8_t* __restrict__ keep, uint32_t min_keep, uint2* __restrict__ txrec,
    uint16_t* __restrict__ fit, unsigned long long* ctr, unsigned long long tx_cap,
    unsigned long long nnz_cap) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t nblk = (n + 63) / 64;
  for (int64_t g0 = wave * kRG; g0 < nblk; g0 += nwaves * kRG) {
    const int64_t g1 = g0 + kRG < nblk ? g0 + kRG : nblk;
    uint32_t R = 0, I = 0;
    for (int64_t blk = g0; blk < g1; ++blk) {
      const int64_t t = blk * 64 + lane;
      uint2 rec = make_uint2(0u, 0u);
      if (t < n) rec = in_rec[t];
      const uint16_t* it = in_fit + rec.x;
      uint32_t kept = 0;
      for (uint32_t j = 0; j < rec.y; ++j) kept += keep[it[j]] ? 1u : 0u;
      if (kept >= min_keep) {
        ++R;
        I += kept;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      R += __shfl_xor(R, o, 64);
      I += __shfl_xor(I, o, 64);
    }
    unsigned long long old = 0;
    if (lane == 0 && R) old = atomicAdd(ctr, ((unsigned long long)R << kPackShift) + I);
    old = __shfl(old, 0, 64);
    unsigned long long row_base = old >> kPackShift, item_base = old & kPackMask;
    for (int64_t blk = g0; blk < g1; ++blk) {
      const int64_t t = blk * 64 + lane;
      uint2 rec = make_uint2(0u, 0u);
      if (t < n) rec = in_rec[t];
      const uint16_t* it = in_fit + rec.x;
      uint32_t kept = 0;
      for (uint32_t j = 0; j < rec.y; ++j) kept += keep[it[j]] ? 1u : 0u;
      const bool want = kept >= min_keep;
      const unsigned long long m = __ballot(want);
      uint32_t win = want ? kept : 0u;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(win, o, 64);
        if (lane >= o) win += u;
      }
      const unsigned long long ti = row_base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
      const unsigned long long off = item_base + win - (want ? kept : 0u);
      if (want && ti < tx_cap && off + kept <= nnz_cap) {
        txrec[ti] = make_uint2((uint32_t)off, kept);
        uint32_t q = 0;
        for (uint32_t j = 0; j < rec.y; ++j) {
          const uint16_t r = it[j];
          if (keep[r]) fit[off + q++] = r;
        }
      }
      row_base += (unsigned long long)__popcll(m);
      item_base += __shfl(win, 63, 64);
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
    const uint16_t* __restrict__ pr, uint32_t min_keep, uint2* __restrict__ txrec,
    uint16_t* __restrict__ fit, unsigned long long* ctr, unsigned long long tx_cap,
    unsigned long long nnz_cap, unsigned* err, uint32_t rows_res, uint32_t items_res) {
  const int lane = threadIdx.x & 63;
  WavePool pool{0, 0, 0, 0};
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
        for (int u = 0; u < kFU; ++u) r[u] = it[u] >= 0 ? rank16(pr[it[u]]) : -1;
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
    pool_alloc(want, want ? kept : 0u, ctr, lane, pool, rows_res, items_res, &ti, &off);
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
            const int32_t r = rank16(pr[items[p]]);
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

// The same filter for large vocabularies with a frequent-item bit mask: the mask (<= 128 KB)
// lives in LDS, so only frequent items (a quarter of the nonzeros at configs 3/5) gather their
// rank from L2, and each wave reads a 64-transaction chunk's CSR span with coalesced loads
// (kMU rows of 64 items in flight).  The chunk's ranks are compacted into a per-wave LDS buffer
// in CSR order; each lane then sorts its own transaction's run.  Chunks with more frequent
// entries than the buffer holds take the per-lane path of k_map_filter.
constexpr int kMW = 8;       // waves per workgroup (mask in L2)
constexpr int kMW16 = 16;    // waves per workgroup (mask in LDS: one workgroup per CU, 4 waves/SIMD)
constexpr int kMEnt = 1024;  // per-wave entry buffer
constexpr int kMEnt16 = 768; // (16 waves: the buffers fit next to a 125 KB mask)
constexpr int kMU = 4;       // 64-item rows of the span scan in flight (8: no faster at config 5)
template <int ENT>
struct MapLdsT {
  uint16_t ent[ENT];
  uint32_t pt[65];
  uint32_t kc[64];
};
// next chunk's CSR bounds, loaded before the current chunk is scanned (a dependent round trip
// less per chunk): lane l holds tx_ptr[t0 + l] (l < n), every lane tx_ptr[t0 + n]
struct ChunkPtr {
  int64_t p, e;
  unsigned n;
};
__device__ __forceinline__ ChunkPtr load_chunk_ptr(const int64_t* __restrict__ tx_ptr, int64_t c,
                                                   int64_t nchunks, int64_t n_tx, int lane) {
  ChunkPtr r{0, 0, 0u};
  if (c < nchunks) {
    const int64_t t0 = c * 64;
    r.n = (unsigned)(n_tx - t0 < 64 ? n_tx - t0 : 64);
    r.p = tx_ptr[t0 + ((unsigned)lane < r.n ? lane : 0)];
    r.e = tx_ptr[t0 + r.n];
  }
  return r;
}
template <bool LDS_MASK, int NW, int ENT>
__global__ __launch_bounds__(64 * NW) void k_map_filter_lds(
    const int64_t* __restrict__ tx_ptr, const int32_t* __restrict__ items, int64_t n_tx,
    const uint32_t* __restrict__ fmask, int64_t mask_words, const uint16_t* __restrict__ pr,
    uint32_t min_keep, uint2* __restrict__ txrec, uint16_t* __restrict__ fit,
    unsigned long long* ctr, unsigned long long tx_cap, unsigned long long nnz_cap,
    unsigned* err, uint32_t rows_res, uint32_t items_res) {
  // LDS_MASK: the mask copied into LDS (one workgroup per CU); else read from L2 (more waves)
  WavePool pool{0, 0, 0, 0};
  KMLS_DYN_LDS(uint32_t, smask_lds);
  __shared__ MapLdsT<ENT> lds[NW];
  if constexpr (LDS_MASK) {
    for (int64_t i = threadIdx.x; i < mask_words; i += 64 * NW) smask_lds[i] = fmask[i];
    __syncthreads();
  }
  const uint32_t* smask = LDS_MASK ? smask_lds : fmask;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  MapLdsT<ENT>& L = lds[w];
  const unsigned long long lanelt = (1ull << lane) - 1ull;
  const int64_t nchunks = (n_tx + 63) / 64;
  const int64_t stride = (int64_t)gridDim.x * NW;
  ChunkPtr nx = load_chunk_ptr(tx_ptr, (int64_t)blockIdx.x * NW + w, nchunks, n_tx, lane);
  for (int64_t c = (int64_t)blockIdx.x * NW + w; c < nchunks; c += stride) {
    const ChunkPtr cp = nx;
    nx = load_chunk_ptr(tx_ptr, c + stride, nchunks, n_tx, lane);
    const unsigned n = cp.n;
    const int64_t b0 = (int64_t)__shfl((long long)cp.p, 0, 64);
    const unsigned span = (unsigned)(cp.e - b0);
    L.pt[lane] = (unsigned)lane < n ? (unsigned)(cp.p - b0) : span;
    if (lane == 0) L.pt[64] = span;
    L.kc[lane] = 0u;
    __builtin_amdgcn_wave_barrier();
    unsigned ne = 0;
    // 16-byte loads: lane l reads items [a0 + 4 l, a0 + 4 l + 4) of each 256-item row, a0 = the
    // span start rounded down to 4 (the item array carries 16 items of padding), so a wave
    // instruction moves 1 KB and kMU of them are in flight
    const int64_t a0 = b0 & ~(int64_t)3;
    const unsigned lead = (unsigned)(b0 - a0), end = lead + span;
    for (unsigned p0 = 0; p0 < end; p0 += 256u * kMU) {
      int4 v4[kMU];
#pragma unroll
      for (int u = 0; u < kMU; ++u) {
        const unsigned q = p0 + 256u * (unsigned)u + 4u * (unsigned)lane;
        v4[u] = q < end ? *reinterpret_cast<const int4*>(items + a0 + q) : make_int4(-1, -1, -1, -1);
      }
#pragma unroll
      for (int u = 0; u < kMU; ++u) {
        const unsigned qb = p0 + 256u * (unsigned)u + 4u * (unsigned)lane;
        const int iv[4] = {v4[u].x, v4[u].y, v4[u].z, v4[u].w};
        int r[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned q = qb + (unsigned)e;
          const int x = iv[e];
          r[e] = (q >= lead && q < end && x >= 0 && ((smask[x >> 5] >> (x & 31)) & 1u)) ? rank16(pr[x]) : -1;
        }
        // the 4 items of a lane are consecutive: ranks in CSR order = lane-major, item-minor
        const unsigned cnt = (r[0] >= 0) + (r[1] >= 0) + (r[2] >= 0) + (r[3] >= 0);
        unsigned incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
          const unsigned t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        unsigned e0 = ne + incl - cnt;
        if (cnt) {
          // transaction of the lane's first kept item by ONE binary search (the last x with
          // pt[x] <= q), the later ones by stepping forward: 4 consecutive items rarely cross
          // a boundary (a search per kept item was 6 dependent LDS reads each)
          int ef = 0;
          while (r[ef] < 0) ++ef;
          const unsigned qf = qb + (unsigned)ef - lead;
          unsigned x = 0;
          for (unsigned step = 32; step; step >>= 1)
            if (L.pt[x + step] <= qf) x += step;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (r[e] < 0) continue;
            const unsigned q = qb + (unsigned)e - lead;  // position in the span
            while (x < 63u && L.pt[x + 1] <= q) ++x;
            atomicAdd(&L.kc[x], 1u);
            if (e0 < (unsigned)ENT) L.ent[e0] = (uint16_t)r[e];
            ++e0;
          }
        }
        ne += __shfl(incl, 63, 64);
      }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t kept = (unsigned)lane < n ? L.kc[lane] : 0u;
    uint32_t incl = kept;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    const uint32_t toff = incl - kept;
    const bool buffered = ne <= (unsigned)ENT;
    uint32_t v[kSortRegs];
#pragma unroll
    for (int q = 0; q < kSortRegs; ++q) v[q] = 0xFFFFFFFFu;
    const int64_t ts = (unsigned)lane < n ? b0 + L.pt[lane] : 0;
    const int64_t te = (unsigned)lane < n ? b0 + L.pt[lane + 1] : 0;
    if (kept <= (uint32_t)kSortRegs) {
      if (buffered) {
        for (uint32_t j = 0; j < kept; ++j) {
          uint32_t x = L.ent[toff + j];
#pragma unroll
          for (int q = 0; q < kSortRegs; ++q) {
            const uint32_t lo = min(v[q], x), hi = max(v[q], x);
            v[q] = lo;
            x = hi;
          }
        }
      } else {
        for (int64_t p = ts; p < te; ++p) {
          const int32_t iv = items[p];
          if (!((smask[iv >> 5] >> (iv & 31)) & 1u)) continue;
          uint32_t x = (uint32_t)pr[iv];
#pragma unroll
          for (int q = 0; q < kSortRegs; ++q) {
            const uint32_t lo = min(v[q], x), hi = max(v[q], x);
            v[q] = lo;
            x = hi;
          }
        }
      }
    }
    if (kept > 65535u) atomicOr(err, 1u);
    bool dup = false;  // (rows longer than the registers check while sorting in place)
#pragma unroll
    for (int q = 0; q + 1 < kSortRegs; ++q)
      dup |= kept <= (uint32_t)kSortRegs && (uint32_t)(q + 1) < kept && v[q] == v[q + 1];
    if (dup) atomicOr(err, 2u);
    const bool want = kept >= min_keep && kept <= 65535u;
    unsigned long long ti, off;
    pool_alloc(want, want ? kept : 0u, ctr, lane, pool, rows_res, items_res, &ti, &off);
    if (want && ti < tx_cap && off + kept <= nnz_cap) {
      txrec[ti] = make_uint2((uint32_t)off, kept);
      uint16_t* dst = fit + off;
      if (kept <= (uint32_t)kSortRegs) {
#pragma unroll
        for (int q = 0; q < kSortRegs; ++q)
          if ((uint32_t)q < kept) dst[q] = (uint16_t)v[q];
      } else {  // long row: insertion-sort in place (rare)
        uint32_t nn = 0;
        for (int64_t p = ts; p < te; ++p) {
          const int32_t iv = items[p];
          if (!((smask[iv >> 5] >> (iv & 31)) & 1u)) continue;
          const uint16_t x = (uint16_t)pr[iv];
          uint32_t j = nn++;
          while (j > 0 && dst[j - 1] > x) {
            dst[j] = dst[j - 1];
            --j;
          }
          if (j > 0 && dst[j - 1] == x) atomicOr(err, 2u);
          dst[j] = x;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace
}  // namespace devbuf
}  // namespace kern
}  // namespace kmls
