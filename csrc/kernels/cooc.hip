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
// Layout of the work (one 64-lane wave = 64 consecutive transactions, lane = transaction):
//   1. each lane counts the frequent items of its transaction (frequent-mask bit, then the rank
//      gather), a wave scan turns the counts into LDS offsets;
//   2. the lanes write their transactions' frequent ranks into the wave's LDS entry buffer
//      (sub-chunks of <= kEnt entries when 64 transactions hold more);
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

__device__ __forceinline__ int frequent_rank(int it, const int32_t* __restrict__ rank_of,
                                             const uint32_t* __restrict__ fmask) {
  if (fmask != nullptr && !((fmask[it >> 5] >> (it & 31)) & 1u)) return -1;
  return rank_of[it];
}

// per transaction k = its frequent items: sum of k(k-1)/2 and max k (the host's cost model and
// the entry-buffer bound)
__global__ __launch_bounds__(256) void k_cooc_stats(const int64_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ items, int64_t n_tx,
                                                    const int32_t* __restrict__ rank_of,
                                                    const uint32_t* __restrict__ fmask,
                                                    unsigned long long* __restrict__ out) {
  unsigned long long pairs = 0;
  unsigned kmax = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_tx; t += stride) {
    unsigned k = 0;
    for (int64_t p = ptr[t], e = ptr[t + 1]; p < e; ++p) k += frequent_rank(items[p], rank_of, fmask) >= 0;
    pairs += (unsigned long long)k * (k - (k > 0)) / 2;
    kmax = k > kmax ? k : kmax;
  }
  for (int off = 32; off; off >>= 1) {
    pairs += shfl_xor64(pairs, off);
    const unsigned o = __shfl_xor(kmax, off, 64);
    kmax = o > kmax ? o : kmax;
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out, pairs);
    atomicMax(out + 1, (unsigned long long)kmax);
  }
}

__global__ __launch_bounds__(256) void k_cooc_count(const int64_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ items, int64_t n_tx,
                                                    const int32_t* __restrict__ rank_of,
                                                    const uint32_t* __restrict__ fmask, int F,
                                                    uint32_t* __restrict__ gram, int64_t ld,
                                                    unsigned* __restrict__ err) {
  __shared__ uint32_t head[kHead * kHead];  // [a - head0][b - head0], a < b
  __shared__ int32_t ent[kW][kEnt];
  __shared__ uint32_t toff[kW][kTx + 1];    // entry offset of sub-chunk transaction x
  __shared__ uint32_t poff[kW][kTx + 1];    // pair offset of sub-chunk transaction x
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int head0 = F > kHead ? F - kHead : 0;
  for (int e = threadIdx.x; e < kHead * kHead; e += blockDim.x) head[e] = 0u;
  __syncthreads();
  int32_t* E = ent[wid];
  uint32_t* TO = toff[wid];
  uint32_t* PO = poff[wid];
  const int64_t nchunks = (n_tx + kTx - 1) / kTx;
  for (int64_t c = (int64_t)blockIdx.x * kW + wid; c < nchunks; c += (int64_t)gridDim.x * kW) {
    const int64_t t = c * kTx + lane;
    const bool act = t < n_tx;
    const int64_t b = act ? ptr[t] : 0, e = act ? ptr[t + 1] : 0;
    unsigned k = 0;
    for (int64_t p = b; p < e; ++p) k += frequent_rank(items[p], rank_of, fmask) >= 0;
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
    unsigned l0 = 0, base = 0;
    while (l0 < 64u) {
      // the sub-chunk: lanes l0 .. l1-1 whose entries fit (every single lane fits: k <= kEnt)
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
          if (r >= 0) E[off + j++] = r;
        }
        TO[lane - l0] = off;
      }
      // pairs per transaction, inclusive scan over the sub-chunk's lanes
      const unsigned q = in_sub ? k * (k - (k > 0)) / 2 : 0u;
      unsigned pin = q;
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(pin, o, 64);
        if (lane >= o) pin += v;
      }
      const unsigned n_sub = l1 - l0;
      if (in_sub) PO[lane - l0] = pin - q;
      const unsigned P = uni(__shfl(pin, 63, 64));
      const unsigned last = uni(__shfl(incl, (int)l1 - 1, 64));  // entries up to lane l1-1
      if (lane == 0) {
        PO[n_sub] = P;
        TO[n_sub] = last - base;
      }
      __builtin_amdgcn_wave_barrier();
      for (unsigned p0 = 0; p0 < P; p0 += 64) {
        const unsigned p = p0 + lane;
        if (p < P) {
          // transaction x: the last with PO[x] <= p
          unsigned x = 0;
          for (unsigned step = 32; step; step >>= 1)
            if (x + step < n_sub && PO[x + step] <= p) x += step;
          const unsigned qq = p - PO[x];
          const unsigned e0 = TO[x];
          const unsigned kk = TO[x + 1] - e0;
          // row-major triangle: row i holds (kk-1-i) pairs, S(i) = i(2kk-1-i)/2 before it
          const float m2 = (float)(2 * kk - 1);
          int i = (int)((m2 - sqrtf(m2 * m2 - 8.0f * (float)qq)) * 0.5f);
          if (i < 0) i = 0;
          while (i > 0 && (unsigned)(i * (2 * (int)kk - 1 - i) / 2) > qq) --i;
          while ((unsigned)((i + 1) * (2 * (int)kk - 2 - i) / 2) <= qq) ++i;
          const unsigned j = (unsigned)i + 1u + (qq - (unsigned)(i * (2 * (int)kk - 1 - i) / 2));
          const int ra = E[e0 + (unsigned)i], rb = E[e0 + j];
          const int lo = ra < rb ? ra : rb, hi = ra < rb ? rb : ra;
          if (lo >= head0)
            atomicAdd(&head[(lo - head0) * kHead + (hi - head0)], 1u);
          else
            atomicAdd(&gram[(int64_t)lo * ld + hi], 1u);
        }
      }
      __builtin_amdgcn_wave_barrier();
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
