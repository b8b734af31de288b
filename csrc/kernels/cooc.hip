// Horizontal co-occurrence counting: level-2 supports (the pair gram) of SPARSE
// transaction data straight from the transaction CSR, without tid-bitmaps.
//
// The dense bit-GEMM (gram_mfma.hip) does F^2/2 * T bit-ANDs whatever the data.  At the large
// BASELINE shapes (configs 3/5: 10M-100M transactions, 14.8k frequent items at 2e-4) more than
// 99.98 % of its outputs are below minsup: each transaction holds only ~7 frequent items, so the
// pairs that actually co-occur number sum_t k_t(k_t-1)/2 ~ 2.6e8 per 10M transactions, six
// orders of magnitude fewer than the GEMM's bit operations.  Here every such pair is counted
// once, where it occurs (the reference's own rule map is this pair-support matrix,
// machine-learning/main.py:282-304).
//
// Layout of the work (one 64-lane wave = a chunk of 64 consecutive transactions):
//   1. the wave streams the chunk's contiguous CSR span with coalesced loads (frequent-mask bit,
//      then the rank gather), compacts the frequent ranks in order into its LDS entry buffer and
//      counts them per transaction (LDS atomics; a binary search of the chunk's offsets gives an
//      item's transaction);
//   2. chunks with more frequent entries than the buffer holds (long transactions) fall back to
//      sub-chunks of lanes whose entries fit, each lane reading its own transaction;
//   3. the pairs of all those transactions are enumerated FLAT over the wave (pair p -> its
//      transaction by a binary search of the pair prefix, (i, j) by inverting the row-major
//      triangle), so a wave64 instruction carries 64 pairs whatever the transaction lengths;
//   4. each pair adds 1 to gram[lo][hi] (rank order, upper triangle, as the GEMM writes it):
//      pairs of two HEAD items (the kHead most frequent ranks, where the hot pairs concentrate)
//      go to an LDS table flushed once per workgroup, every other pair is one no-return global
//      atomic (spread over ~1e8 addresses, no hot spot).
// Counts are exact (u32: T < 2^32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "kernels.hpp"
#include <kmls/wave.hpp>

namespace kmls {
namespace kern {

namespace {

constexpr int kW = 4;       // waves per workgroup
constexpr int kTx = 64;     // transactions per wave chunk (lane = transaction)
constexpr int kEnt = 2048;  // frequent entries of one sub-chunk (LDS, per wave)
constexpr int kHead = 64;   // most frequent ranks whose pairs are counted in LDS
constexpr int kScanU = 4;   // 64-item rows of the CSR scan in flight per wave

__device__ __forceinline__ int frequent_rank(int it, const int32_t* __restrict__ rank_of,
                                             const uint32_t* __restrict__ fmask) {
  if (fmask != nullptr && !((fmask[it >> 5] >> (it & 31)) & 1u)) return -1;
  return rank_of[it];
}

// Per-wave LDS of one 64-transaction chunk.
struct ChunkLds {
  int32_t ent[kEnt];          // frequent ranks of the chunk, in CSR (transaction) order
  uint32_t pt[kTx + 1];       // CSR offsets of the chunk's transactions, relative to pt[0]
  uint32_t kc[kTx];           // frequent items per transaction
  uint32_t toff[kTx + 1];     // entry offset of transaction x
  uint32_t poff[kTx + 1];     // pair offset of transaction x
};

// the stats pass only counts: offsets and per-transaction counts (0.5 KB per wave, so its
// occupancy is set by registers, not by an unused entry buffer)
struct ScanLds {
  uint32_t pt[kTx + 1];
  uint32_t kc[kTx];
};

// Coalesced scan of the chunk's items (the contiguous CSR span of its transactions): frequent
// ranks compacted in order into L.ent (while they fit: WRITE), per-transaction counts in L.kc.
// Returns the chunk's frequent entries (may exceed kEnt; then L.ent holds only the first kEnt).
template <bool WRITE, typename Lds>
__device__ __forceinline__ unsigned chunk_scan(Lds& L, const int64_t* __restrict__ ptr,
                                               const int32_t* __restrict__ items,
                                               const int32_t* __restrict__ rank_of,
                                               const uint32_t* __restrict__ fmask, int64_t t0,
                                               unsigned n, int lane) {
  const int64_t b0 = ptr[t0];
  const unsigned span = (unsigned)(ptr[t0 + n] - b0);  // (n may be 64: no lane holds it)
  if ((unsigned)lane < n) L.pt[lane] = (unsigned)(ptr[t0 + lane] - b0);
  if (lane < kTx) L.kc[lane] = 0u;
  __builtin_amdgcn_wave_barrier();
  const unsigned long long lanelt = (1ull << lane) - 1ull;
  unsigned ne = 0;
  // kScanU rows of 64 items per iteration: their item loads, then their mask-word and rank
  // gathers, are all in flight before the first is used (one row at a time left the scan
  // latency-bound: ~280 GB/s of items at 100M x 1M)
  for (unsigned p0 = 0; p0 < span; p0 += 64u * kScanU) {
    int it[kScanU], r[kScanU];
#pragma unroll
    for (int u = 0; u < kScanU; ++u) {
      const unsigned p = p0 + 64u * (unsigned)u + (unsigned)lane;
      it[u] = p < span ? items[b0 + p] : -1;
    }
    uint32_t fw[kScanU];
#pragma unroll
    for (int u = 0; u < kScanU; ++u)
      fw[u] = (fmask != nullptr && it[u] >= 0) ? fmask[it[u] >> 5] : ~0u;
#pragma unroll
    for (int u = 0; u < kScanU; ++u)
      r[u] = (it[u] >= 0 && ((fw[u] >> (it[u] & 31)) & 1u)) ? rank_of[it[u]] : -1;
#pragma unroll
    for (int u = 0; u < kScanU; ++u) {
      const unsigned p = p0 + 64u * (unsigned)u + (unsigned)lane;
      const unsigned long long m = __ballot(r[u] >= 0);
      if (r[u] >= 0) {
        // transaction: the last x with pt[x] <= p
        unsigned x = 0;
        for (unsigned step = 32; step; step >>= 1)
          if (x + step < n && L.pt[x + step] <= p) x += step;
        atomicAdd(&L.kc[x], 1u);
        if constexpr (WRITE) {
          const unsigned e = ne + (unsigned)__popcll(m & lanelt);
          if (e < (unsigned)kEnt) L.ent[e] = r[u];
        }
      }
      ne += (unsigned)__popcll(m);
    }
  }
  __builtin_amdgcn_wave_barrier();
  return ne;
}

// per transaction k = its frequent items: sum of k(k-1)/2 and max k (the host's cost model and
// the entry-buffer bound)
__global__ __launch_bounds__(256) void k_cooc_stats(const int64_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ items, int64_t n_tx,
                                                    const int32_t* __restrict__ rank_of,
                                                    const uint32_t* __restrict__ fmask,
                                                    unsigned long long* __restrict__ out) {
  __shared__ ScanLds lds[kW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  ScanLds& L = lds[wid];
  unsigned long long pairs = 0;
  unsigned kmax = 0;
  const int64_t nchunks = (n_tx + kTx - 1) / kTx;
  for (int64_t c = (int64_t)blockIdx.x * kW + wid; c < nchunks; c += (int64_t)gridDim.x * kW) {
    const int64_t t0 = c * kTx;
    const unsigned n = (unsigned)(n_tx - t0 < kTx ? n_tx - t0 : kTx);
    chunk_scan<false>(L, ptr, items, rank_of, fmask, t0, n, lane);
    const unsigned k = (unsigned)lane < n ? L.kc[lane] : 0u;
    pairs += (unsigned long long)k * (k - (k > 0)) / 2;
    kmax = k > kmax ? k : kmax;
    __builtin_amdgcn_wave_barrier();
  }
  for (int off = 32; off; off >>= 1) {
    pairs += shfl_xor64(pairs, off);
    const unsigned o = __shfl_xor(kmax, off, 64);
    kmax = o > kmax ? o : kmax;
  }
  if (lane == 0) {
    atomicAdd(out, pairs);
    atomicMax(out + 1, (unsigned long long)kmax);
  }
}

// the pairs of sub-chunk lanes [x0, x0 + nx) whose entries sit at L.ent[L.toff[x]..]: flat over
// the wave (pair -> transaction by a binary search of L.poff, (i, j) by inverting the triangle)
__device__ __forceinline__ void chunk_pairs(ChunkLds& L, unsigned nx, unsigned P, int head0,
                                            uint32_t* head, uint32_t* __restrict__ gram,
                                            int64_t ld, unsigned* __restrict__ err, int lane) {
  for (unsigned p0 = 0; p0 < P; p0 += 64) {
    const unsigned p = p0 + lane;
    if (p < P) {
      unsigned x = 0;
      for (unsigned step = 32; step; step >>= 1)
        if (x + step < nx && L.poff[x + step] <= p) x += step;
      const unsigned qq = p - L.poff[x];
      const unsigned e0 = L.toff[x];
      const unsigned kk = L.toff[x + 1] - e0;
      // row-major triangle: row i holds (kk-1-i) pairs, S(i) = i(2kk-1-i)/2 before it
      const float m2 = (float)(2 * kk - 1);
      int i = (int)((m2 - sqrtf(m2 * m2 - 8.0f * (float)qq)) * 0.5f);
      if (i < 0) i = 0;
      while (i > 0 && (unsigned)(i * (2 * (int)kk - 1 - i) / 2) > qq) --i;
      while ((unsigned)((i + 1) * (2 * (int)kk - 2 - i) / 2) <= qq) ++i;
      const unsigned j = (unsigned)i + 1u + (qq - (unsigned)(i * (2 * (int)kk - 1 - i) / 2));
      const int ra = L.ent[e0 + (unsigned)i], rb = L.ent[e0 + j];
      const int lo = ra < rb ? ra : rb, hi = ra < rb ? rb : ra;
      if (lo == hi)  // a duplicated item (rows must be duplicate-free): flag, count nothing
        atomicOr(err, 2u);
      else if (lo >= head0)
        atomicAdd(&head[(lo - head0) * kHead + (hi - head0)], 1u);
      else
        atomicAdd(&gram[(int64_t)lo * ld + hi], 1u);
    }
  }
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(256) void k_cooc_count(const int64_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ items, int64_t n_tx,
                                                    const int32_t* __restrict__ rank_of,
                                                    const uint32_t* __restrict__ fmask, int F,
                                                    uint32_t* __restrict__ gram, int64_t ld,
                                                    unsigned* __restrict__ err) {
  __shared__ uint32_t head[kHead * kHead];  // [a - head0][b - head0], a < b
  __shared__ ChunkLds lds[kW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  ChunkLds& L = lds[wid];
  const int head0 = F > kHead ? F - kHead : 0;
  for (int e = threadIdx.x; e < kHead * kHead; e += blockDim.x) head[e] = 0u;
  __syncthreads();
  const int64_t nchunks = (n_tx + kTx - 1) / kTx;
  for (int64_t c = (int64_t)blockIdx.x * kW + wid; c < nchunks; c += (int64_t)gridDim.x * kW) {
    const int64_t t0 = c * kTx;
    const unsigned n = (unsigned)(n_tx - t0 < kTx ? n_tx - t0 : kTx);
    const unsigned ne = chunk_scan<true>(L, ptr, items, rank_of, fmask, t0, n, lane);
    unsigned k = (unsigned)lane < n ? L.kc[lane] : 0u;
    if (k > (unsigned)kEnt) {  // the host checks max k first; never write past the buffer
      atomicOr(err, 1u);
      k = 0;
    }
    // inclusive scan of k over the lanes
    unsigned incl = k;
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    if (ne <= (unsigned)kEnt) {
      // the whole chunk's entries are in LDS, in transaction order: one pass of its pairs
      const unsigned q = k * (k - (k > 0)) / 2;
      unsigned pin = q;
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(pin, o, 64);
        if (lane >= o) pin += v;
      }
      if ((unsigned)lane < n) {
        L.toff[lane] = incl - k;
        L.poff[lane] = pin - q;
      }
      const unsigned P = uni(__shfl(pin, 63, 64));
      if (lane == 0) {
        L.toff[n] = ne;
        L.poff[n] = P;
      }
      __builtin_amdgcn_wave_barrier();
      chunk_pairs(L, n, P, head0, head, gram, ld, err, lane);
      continue;
    }
    // more entries than fit (long transactions): sub-chunks of lanes whose entries fit, each
    // lane re-reading its own transaction's items
    const int64_t t = t0 + lane;
    const bool act = (unsigned)lane < n;
    const int64_t b = act ? ptr[t] : 0, e = act ? ptr[t + 1] : 0;
    unsigned l0 = 0, base = 0;
    while (l0 < 64u) {
      const unsigned long long fit = __ballot((unsigned)lane >= l0 && incl - base <= (unsigned)kEnt);
      const unsigned long long run = fit >> l0;
      const unsigned len = ~run == 0ull ? 64u - l0 : (unsigned)__builtin_ctzll(~run);
      const unsigned l1 = l0 + (len ? len : 1u);
      const bool in_sub = (unsigned)lane >= l0 && (unsigned)lane < l1;
      const unsigned off = incl - k - base;
      if (in_sub) {
        unsigned j = 0;
        for (int64_t p = b; p < e && j < k; ++p) {
          const int r = frequent_rank(items[p], rank_of, fmask);
          if (r >= 0) L.ent[off + j++] = r;
        }
        L.toff[lane - l0] = off;
      }
      const unsigned q = in_sub ? k * (k - (k > 0)) / 2 : 0u;
      unsigned pin = q;
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(pin, o, 64);
        if (lane >= o) pin += v;
      }
      const unsigned n_sub = l1 - l0;
      if (in_sub) L.poff[lane - l0] = pin - q;
      const unsigned P = uni(__shfl(pin, 63, 64));
      const unsigned last = uni(__shfl(incl, (int)l1 - 1, 64));  // entries up to lane l1-1
      if (lane == 0) {
        L.poff[n_sub] = P;
        L.toff[n_sub] = last - base;
      }
      __builtin_amdgcn_wave_barrier();
      chunk_pairs(L, n_sub, P, head0, head, gram, ld, err, lane);
      base = last;
      l0 = l1;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kHead * kHead; e += blockDim.x) {
    const int a = e / kHead, bb = e - a * kHead;
    const uint32_t v = head[e];
    if (a < bb && v) atomicAdd(&gram[(int64_t)(head0 + a) * ld + head0 + bb], v);
  }
}

// ---- tx-DP combine of shard grams: frequent entries of a reduce-scattered row block ----
// rows [nrows][ld] = global rows r0.. of the summed gram (upper triangle valid): entries (r, c)
// with c > r and count >= minsup.  emit == nullptr: count them into cnt[0]; else write
// (row, col, count) triples at slots taken from cnt[0].
__global__ __launch_bounds__(256) void k_gram_frequent(const uint32_t* __restrict__ rows,
                                                       int64_t ld, int64_t r0, int64_t nrows,
                                                       int64_t F, uint32_t minsup,
                                                       unsigned long long* __restrict__ cnt,
                                                       uint32_t* __restrict__ emit) {
  const int64_t n = nrows * F;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63;
  for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x; e0 < n; e0 += stride) {
    const int64_t e = e0 + threadIdx.x;
    bool hit = false;
    int64_t r = 0, c = 0;
    uint32_t v = 0;
    if (e < n) {
      r = e / F;
      c = e - r * F;
      v = rows[r * ld + c];
      hit = c > r0 + r && v >= minsup && v > 0;
    }
    const unsigned long long m = __ballot(hit);
    if (!m) continue;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(cnt, (unsigned long long)__popcll(m));
    base = bcast64(base, 0);
    if (hit && emit != nullptr) {
      const unsigned long long slot = base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
      emit[3 * slot + 0] = (uint32_t)(r0 + r);
      emit[3 * slot + 1] = (uint32_t)c;
      emit[3 * slot + 2] = v;
    }
  }
}

// gram[row * ld + col] = count for every triple with count > 0 (padding triples are zero)
__global__ void k_gram_scatter(const uint32_t* __restrict__ t, int64_t n, uint32_t* __restrict__ gram,
                               int64_t ld) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t v = t[3 * i + 2];
    if (v) gram[(int64_t)t[3 * i] * ld + t[3 * i + 1]] = v;
  }
}

}  // namespace

void gram_frequent(const uint32_t* rows, int64_t ld, int64_t r0, int64_t nrows, int64_t F,
                   uint32_t minsup, unsigned long long* cnt, uint32_t* emit, hipStream_t s) {
  const int64_t n = nrows * F;
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_gram_frequent, dim3((unsigned)blocks), dim3(256), 0, s, rows, ld, r0, nrows,
                     F, minsup, cnt, emit);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e));
}

void gram_scatter(const uint32_t* triples, int64_t n, uint32_t* gram, int64_t ld, hipStream_t s) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_gram_scatter, dim3((unsigned)blocks), dim3(256), 0, s, triples, n, gram, ld);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e));
}

int cooc_max_k() { return kEnt; }

void cooc_stats(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, const int32_t* rank_of,
                const uint32_t* fmask, unsigned long long* out, int n_cus, hipStream_t s) {
  if (n_tx <= 0) return;
  const int64_t blocks = std::min<int64_t>((n_tx + 255) / 256, (int64_t)std::max(n_cus, 1) * 8);
  hipLaunchKernelGGL(k_cooc_stats, dim3((unsigned)blocks), dim3(256), 0, s, tx_ptr, items, n_tx,
                     rank_of, fmask, out);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e));
}

void cooc_count(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, const int32_t* rank_of,
                const uint32_t* fmask, int64_t F, uint32_t* gram, int64_t ld, unsigned* err,
                int n_cus, hipStream_t s) {
  if (n_tx <= 0 || F < 2) return;
  const int64_t chunks = (n_tx + kTx - 1) / kTx;
  // ~2 workgroups per CU stay resident (LDS 52 KB each); a few rounds of them so each flushes
  // its head table once over many chunks
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((chunks + kW - 1) / kW,
                                                                (int64_t)std::max(n_cus, 1) * 4));
  hipLaunchKernelGGL(k_cooc_count, dim3((unsigned)blocks), dim3(64 * kW), 0, s, tx_ptr, items,
                     n_tx, rank_of, fmask, (int)F, gram, ld, err);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace kmls
