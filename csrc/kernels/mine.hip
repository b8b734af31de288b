// CDNA4 (gfx950) kernels of the GPU FP-Growth miner.
//
// Replaces the reference's mining hot path (mlxtend TransactionEncoder + fpgrowth + the rule
// loop, machine-learning/main.py:262-296) with vertical tid-bitmaps:
//   item_support      O5  per-item supports (LDS-privatised histogram)
//   encode_bitmap     O4  CSR → item-major bit-packed tid bitmaps (uint64 words, HBM resident)
//   pair_gram_*       O8  level-2 co-occurrence "GEMM" over the transaction axis
//   extend_count      O8  |S|>=3 candidate supports: wave64 teams AND + popcount
//   extend_materialize    survivors' bitmaps + itemset-trie append (ordered compaction)
//
// All kernels are wave64-native: teams are power-of-two lane groups inside a 64-lane wave,
// reductions use __shfl_xor within the team, block sizes are multiples of 64.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "kernels.hpp"
#include "kmls/hooks.hpp"

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

constexpr int kBlock = 256;

inline int grid_for(int64_t work, int per_block, int cap = 4096) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// ----------------------------------------------------------------------------------------
// O5 item supports
// ----------------------------------------------------------------------------------------
template <bool kLds>
__global__ __launch_bounds__(kBlock) void k_item_support(const int32_t* __restrict__ items,
                                                         int64_t nnz, int32_t n_items,
                                                         uint32_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  if constexpr (kLds) {
    for (int i = threadIdx.x; i < n_items; i += blockDim.x) hist[i] = 0;
    __syncthreads();
  }
  uint32_t* dst = kLds ? hist : counts;
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  // 16-byte vector loads over the aligned body (items comes from hipMalloc)
  const int64_t n4 = nnz >> 2;
  const int4* v = reinterpret_cast<const int4*>(items);
  for (int64_t i = gtid; i < n4; i += nthr) {
    const int4 q = v[i];
    atomicAdd(&dst[q.x], 1u);
    atomicAdd(&dst[q.y], 1u);
    atomicAdd(&dst[q.z], 1u);
    atomicAdd(&dst[q.w], 1u);
  }
  for (int64_t i = (n4 << 2) + gtid; i < nnz; i += nthr) atomicAdd(&dst[items[i]], 1u);
  if constexpr (kLds) {
    __syncthreads();
    for (int i = threadIdx.x; i < n_items; i += blockDim.x) {
      const uint32_t h = hist[i];
      if (h) atomicAdd(&counts[i], h);
    }
  }
}

// Large vocabularies (1M items, Zipf popularity): a dense LDS histogram does not fit, and plain
// global atomics serialise on the hottest items (the top item alone is ~2% of all occurrences).
// Each block privatises whatever items it sees in an LDS open-addressing table (4096 slots, 8
// probes); misses fall through to a global atomic; the table is flushed once per block.
constexpr int kHashSlots = 4096;

__device__ __forceinline__ void hash_count(int32_t x, int32_t* hk, uint32_t* hv,
                                           uint32_t* __restrict__ counts) {
  const uint32_t h = ((uint32_t)x * 2654435761u) >> 20;  // 12 bits
#pragma unroll 1
  for (int p = 0; p < 8; ++p) {
    const uint32_t slot = (h + p) & (kHashSlots - 1);
    int32_t k = hk[slot];
    if (k == -1) {
      k = atomicCAS(&hk[slot], -1, x);
      if (k == -1) k = x;
    }
    if (k == x) {
      atomicAdd(&hv[slot], 1u);
      return;
    }
  }
  atomicAdd(&counts[x], 1u);
}

__global__ __launch_bounds__(kBlock) void k_item_support_hash(const int32_t* __restrict__ items,
                                                              int64_t nnz,
                                                              uint32_t* __restrict__ counts) {
  __shared__ int32_t hk[kHashSlots];
  __shared__ uint32_t hv[kHashSlots];
  for (int i = threadIdx.x; i < kHashSlots; i += blockDim.x) {
    hk[i] = -1;
    hv[i] = 0;
  }
  __syncthreads();
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = nnz >> 2;
  const int4* v = reinterpret_cast<const int4*>(items);
  for (int64_t i = gtid; i < n4; i += nthr) {
    const int4 q = v[i];
    hash_count(q.x, hk, hv, counts);
    hash_count(q.y, hk, hv, counts);
    hash_count(q.z, hk, hv, counts);
    hash_count(q.w, hk, hv, counts);
  }
  for (int64_t i = (n4 << 2) + gtid; i < nnz; i += nthr) hash_count(items[i], hk, hv, counts);
  __syncthreads();
  for (int i = threadIdx.x; i < kHashSlots; i += blockDim.x)
    if (hk[i] >= 0 && hv[i]) atomicAdd(&counts[hk[i]], hv[i]);
}

// ----------------------------------------------------------------------------------------
// Large vocabularies, large inputs: partitioned histogram.  PMC counters showed the hash kernel
// atomic-bound (2.6e8 fabric write requests for 2.7e8 items on 10M x 1M: the long tail misses the
// LDS table).  Three passes, no global atomics per item:
//   1. k_part_hist:    per block, counts of its chunk's items per vocabulary partition
//                      (partition = id >> 15, 32768 ids);
//   2. (device scan of the partition-major [P][G] counts → every (partition, block) run's offset)
//      k_part_scatter: per 4096-item tile, an LDS counting sort by partition, then each
//                      partition's run is written contiguously (coalesced) as uint16 local ids;
//   3. k_part_count:   per partition, blocks with a dense 32768-bin LDS histogram (128 KB) over a
//                      slice of the partition's ids; one global atomic per nonzero bin per block.
// ~2.5 passes over the int32 items instead of one fabric atomic per item.
// ----------------------------------------------------------------------------------------
// 32768-id partitions (a 1M vocabulary splits 31 ways).  16384-id partitions (62 ways, fewer
// counter collisions in the scatter's LDS counting sort) measured slower: scatter 1.12 -> 1.25
// ms and count 0.38 -> 0.42 ms per 686M-item tile (profiles/r2_s8_support_partitions.md)
constexpr int kPartBits = 15;
constexpr int kPartBins = 1 << kPartBits;
constexpr int kPartMax = 64;     // partitions: n_items <= 2M
constexpr int kPartGrid = 1024;  // blocks of passes 1 and 2
constexpr int kPartGridMax = 2048;
constexpr int kPartTile = 4096;  // items per LDS counting-sort tile (16 per thread)

__device__ __forceinline__ void part_chunk(int64_t nnz, int64_t* b0, int64_t* b1) {
  const int64_t chunk = (nnz + gridDim.x - 1) / gridDim.x;
  *b0 = min(nnz, (int64_t)blockIdx.x * chunk);
  *b1 = min(nnz, *b0 + chunk);
}

__global__ __launch_bounds__(kBlock) void k_part_hist(const int32_t* __restrict__ items,
                                                      int64_t nnz, int P,
                                                      int64_t* __restrict__ blk_cnt) {
  // per-wave bins (no cross-wave LDS contention), 16-byte loads, two in flight per thread
  __shared__ uint32_t h[kBlock / 64][kPartMax];
  const int w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < (kBlock / 64) * kPartMax; i += kBlock) (&h[0][0])[i] = 0;
  __syncthreads();
  int64_t b0, b1;
  part_chunk(nnz, &b0, &b1);
  uint32_t* hw = h[w];
  const int64_t head = ((4 - (int64_t)(((uintptr_t)(items + b0) >> 2) & 3)) & 3);
  const int64_t a0 = min(b1, b0 + head);
  for (int64_t i = b0 + threadIdx.x; i < a0; i += blockDim.x) atomicAdd(&hw[items[i] >> kPartBits], 1u);
  const int4* __restrict__ v = reinterpret_cast<const int4*>(items + a0);
  const int64_t n4 = (b1 - a0) >> 2;
  for (int64_t j = threadIdx.x; j < n4; j += 2 * (int64_t)blockDim.x) {
    const int4 x = v[j];
    const bool two = j + blockDim.x < n4;
    const int4 y = two ? v[j + blockDim.x] : make_int4(0, 0, 0, 0);
    atomicAdd(&hw[x.x >> kPartBits], 1u);
    atomicAdd(&hw[x.y >> kPartBits], 1u);
    atomicAdd(&hw[x.z >> kPartBits], 1u);
    atomicAdd(&hw[x.w >> kPartBits], 1u);
    if (two) {
      atomicAdd(&hw[y.x >> kPartBits], 1u);
      atomicAdd(&hw[y.y >> kPartBits], 1u);
      atomicAdd(&hw[y.z >> kPartBits], 1u);
      atomicAdd(&hw[y.w >> kPartBits], 1u);
    }
  }
  for (int64_t i = a0 + (n4 << 2) + threadIdx.x; i < b1; i += blockDim.x)
    atomicAdd(&hw[items[i] >> kPartBits], 1u);
  __syncthreads();
  if ((int)threadIdx.x < P) {
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) t += h[k][threadIdx.x];
    blk_cnt[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = t;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) blk_cnt[(int64_t)P * gridDim.x] = 0;  // scan sentinel
}

__global__ __launch_bounds__(kBlock) void k_part_scatter(const int32_t* __restrict__ items,
                                                         int64_t nnz, int P,
                                                         const int64_t* __restrict__ off,
                                                         uint16_t* __restrict__ out) {
  __shared__ uint32_t cnt[kPartMax];
  __shared__ uint32_t scn[kPartMax];
  __shared__ int64_t base[kPartMax];
  __shared__ uint16_t stage[kPartTile];
  __shared__ uint8_t stage_p[kPartTile];
  constexpr int kPer = kPartTile / kBlock;
  int64_t b0, b1;
  part_chunk(nnz, &b0, &b1);
  if ((int)threadIdx.x < P) base[threadIdx.x] = off[(int64_t)threadIdx.x * gridDim.x + blockIdx.x];
  // the next tile's ids are loaded while this tile is sorted and written (register double
  // buffer), so each block keeps a tile of loads in flight through its LDS phases
  int32_t xn[kPer];
  {
    const int n_t = (int)min((int64_t)kPartTile, b1 - b0);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int li = j * kBlock + (int)threadIdx.x;
      xn[j] = li < n_t ? items[b0 + li] : -1;
    }
  }
  for (int64_t t0 = b0; t0 < b1; t0 += kPartTile) {
    const int n_t = (int)min((int64_t)kPartTile, b1 - t0);
    if (threadIdx.x < kPartMax) cnt[threadIdx.x] = 0;
    __syncthreads();
    int32_t x[kPer];
    uint32_t loc[kPer];
    const int64_t t1 = t0 + kPartTile;
    const int n_n = (int)max((int64_t)0, min((int64_t)kPartTile, b1 - t1));
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int li = j * kBlock + (int)threadIdx.x;
      x[j] = xn[j];
      xn[j] = li < n_n ? items[t1 + li] : -1;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (x[j] >= 0) loc[j] = atomicAdd(&cnt[x[j] >> kPartBits], 1u);
    __syncthreads();
    // exclusive scan of <= 128 partition counts: waves 0 and 1 scan 64 each, then wave 1's
    // half adds wave 0's total
    uint32_t v = 0, incl = 0;
    if (threadIdx.x < kPartMax) {
      v = cnt[threadIdx.x];
      incl = v;
      const int ln = threadIdx.x & 63;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (ln >= o) incl += y;
      }
      scn[threadIdx.x] = incl;
    }
    __syncthreads();
    const uint32_t lo_total = scn[63];
    __syncthreads();
    if (threadIdx.x < kPartMax) scn[threadIdx.x] = incl - v + (threadIdx.x >= 64 ? lo_total : 0u);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (x[j] >= 0) {
        const int pp = x[j] >> kPartBits;
        const uint32_t pos = scn[pp] + loc[j];
        stage[pos] = (uint16_t)(x[j] & (kPartBins - 1));
        stage_p[pos] = (uint8_t)pp;
      }
    __syncthreads();
    for (int pos = threadIdx.x; pos < n_t; pos += kBlock) {  // runs per partition: coalesced
      const int pp = stage_p[pos];
      out[base[pp] + (pos - (int)scn[pp])] = stage[pos];
    }
    __syncthreads();
    if ((int)threadIdx.x < P) base[threadIdx.x] += cnt[threadIdx.x];
    __syncthreads();
  }
}

// Pass 3, balanced: every block takes an equal slice of the whole partition-major id array, so
// a partition holding a Zipf head item (its partition is ~1.6x the mean length) gets
// proportionally more blocks; a slice that straddles a boundary histograms each partition in
// turn.  (A per-thread sort + run-length dedup of the 8 ids, against same-address LDS atomics
// on head items, measured no faster at 100M x 1M: 8.97 vs 8.70 ms support; removed.)
__global__ __launch_bounds__(1024) void k_part_count_bal(const uint16_t* __restrict__ part,
                                                         const int64_t* __restrict__ off, int G,
                                                         int P, int64_t n_items,
                                                         uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[kPartBins];
  __shared__ int64_t bnd[kPartMax + 1];
  if ((int)threadIdx.x <= P) bnd[threadIdx.x] = off[(int64_t)threadIdx.x * G];
  __syncthreads();
  const int64_t total = bnd[P];
  const int64_t sl = (total + gridDim.x - 1) / gridDim.x;
  const int64_t lo = min(total, (int64_t)blockIdx.x * sl), hi = min(total, lo + sl);
  int p = 0;
  while (p < P - 1 && bnd[p + 1] <= lo) ++p;
  for (; p < P && bnd[p] < hi; ++p) {
    const int64_t a = max(lo, bnd[p]), b = min(hi, bnd[p + 1]);
    if (a >= b) continue;
    for (int i = threadIdx.x; i < kPartBins; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const int64_t head = ((8 - (int64_t)(((uintptr_t)(part + a) >> 1) & 7)) & 7);
    const int64_t a0 = min(b, a + head);
    for (int64_t i = a + threadIdx.x; i < a0; i += blockDim.x) atomicAdd(&h[part[i]], 1u);
    const uint4* __restrict__ v = reinterpret_cast<const uint4*>(part + a0);
    const int64_t n8 = (b - a0) >> 3;
    for (int64_t j = threadIdx.x; j < n8; j += blockDim.x) {
      const uint4 x = v[j];
      atomicAdd(&h[x.x & 0xFFFFu], 1u);
      atomicAdd(&h[x.x >> 16], 1u);
      atomicAdd(&h[x.y & 0xFFFFu], 1u);
      atomicAdd(&h[x.y >> 16], 1u);
      atomicAdd(&h[x.z & 0xFFFFu], 1u);
      atomicAdd(&h[x.z >> 16], 1u);
      atomicAdd(&h[x.w & 0xFFFFu], 1u);
      atomicAdd(&h[x.w >> 16], 1u);
    }
    for (int64_t i = a0 + (n8 << 3) + threadIdx.x; i < b; i += blockDim.x) atomicAdd(&h[part[i]], 1u);
    __syncthreads();
    const int64_t id0 = (int64_t)p << kPartBits;
    for (int i = threadIdx.x; i < kPartBins; i += blockDim.x) {
      const uint32_t val = h[i];
      if (val && id0 + i < n_items) atomicAdd(&counts[id0 + i], val);
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------------------
// O4 bitmap encode: bit t of row rank_of[item] for every (t, item) of the CSR shard.
// One wave64 per transaction (lanes stride its items), so a 2k-transaction shard already
// spreads over ~560 workgroups; 64 transactions share a word column, hence atomicOr.
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_encode_bitmap(const int64_t* __restrict__ tx_ptr,
                                                          const int32_t* __restrict__ items,
                                                          int64_t n_tx,
                                                          const int32_t* __restrict__ rank_of,
                                                          unsigned long long* __restrict__ bm,
                                                          int64_t Wp, int64_t word_off,
                                                          const uint32_t* __restrict__ fmask) {
  const int lane = threadIdx.x & 63;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t t = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < n_tx; t += nwaves) {
    const unsigned long long bit = 1ull << (t & 63);
    const int64_t w = word_off + (t >> 6);
    const int64_t p1 = tx_ptr[t + 1];
    for (int64_t p = tx_ptr[t] + lane; p < p1; p += 64) {
      const int32_t it = items[p];
      if (fmask && !((fmask[it >> 5] >> (it & 31)) & 1u)) continue;
      const int32_t r = rank_of[it];
      if (r >= 0) atomicOr(&bm[(int64_t)r * Wp + w], bit);
    }
  }
}

// Tiled encode for long shards (large T, F <= kEncodeTileMaxF): block b owns the 64*TW
// transactions of word columns [b*TW, b*TW + TW) and builds that F x TW slab of the bitmap in LDS
// (ds_or_b64), then writes it out as whole 8*TW-byte row segments.  The atomic kernel above does
// one fabric atomic per (transaction, frequent item) with 64 waves contending for each word
// column; here the only global traffic is the CSR read and one coalesced write of every word.
// Items are taken kEncodeU per thread per round (loads issued together), each item's
// transaction found by binary search over the tile's LDS copy of tx_ptr.  More frequent rows than
// one slab holds (config 5: ~15k) split into row bands, one block per (tile, band) with the band
// index fastest, so a tile's bands run together and re-read its items from L2, not HBM.
constexpr int kEncodeU = 8;  // items per thread per round (16 measured no faster)
__global__ __launch_bounds__(1024) void k_encode_tile(const int64_t* __restrict__ tx_ptr,
                                                        const int32_t* __restrict__ items,
                                                        int64_t n_tx,
                                                        const int32_t* __restrict__ rank_of,
                                                        unsigned long long* __restrict__ bm,
                                                        int64_t Wp, int64_t word_off, int64_t F,
                                                        int tw_log2, int band_rows,
                                                        const uint32_t* __restrict__ fmask,
                                                        bool xcd_order,
                                                        const unsigned long long* __restrict__ fgroup,
                                                        const int32_t* __restrict__ c2r,
                                                        int txmap_cap) {
  // [band rows][TW], then tx_ptr[64*TW + 1], then (fgroup path) c2r[F], then (txmap_cap > 0)
  // the tile's item-position -> local-transaction map, one byte per item
  extern __shared__ unsigned long long s_bm[];
  const int TW = 1 << tw_log2;
  const int64_t tile_tx = 64ll << tw_log2;
  const int64_t n_bands = (F + band_rows - 1) / band_rows;
  // XCD-aware order: the hardware deals consecutive workgroups round-robin over the 8 XCDs, so
  // neighbouring tiles (which write the two halves of the same 128-byte lines of every row)
  // would meet in different L2s and reach HBM as partial lines.  Logical block L runs on XCD
  // L / ceil(nb / 8): each XCD walks a contiguous run of tiles.
  int64_t lb = blockIdx.x;
  if (xcd_order) {
    const int64_t nb = gridDim.x, q = nb / 8, rr = nb % 8, x = lb % 8;
    lb = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + lb / 8;
  }
  const int64_t tile = lb / n_bands;
  const int32_t r0 = (int32_t)((lb - tile * n_bands) * band_rows);
  const int32_t nr = (int32_t)min((int64_t)band_rows, F - r0);
  const int64_t t0 = tile * tile_tx;
  const int nt = (int)min(tile_tx, n_tx - t0);
  int64_t* s_ptr = (int64_t*)(s_bm + (int64_t)band_rows * TW);
  for (int64_t i = threadIdx.x; i < (int64_t)nr * TW; i += blockDim.x) s_bm[i] = 0ull;
  for (int i = threadIdx.x; i <= nt; i += blockDim.x) s_ptr[i] = tx_ptr[t0 + i];
  int32_t* s_c2r = (int32_t*)(s_ptr + 64 * TW + 1);
  if (fgroup)
    for (int i = threadIdx.x; i < (int)F; i += blockDim.x) s_c2r[i] = c2r[i];
  uint8_t* s_tx = (uint8_t*)(s_c2r + (fgroup ? F : 0));
  __syncthreads();
  const int64_t p0 = s_ptr[0], p1 = s_ptr[nt];
  // item -> transaction without a per-item binary search (8 dependent LDS reads for 256
  // transactions): each wave stamps its transactions' local index over their item ranges
  // (TW <= 4, so a local index fits one byte); tiles with more items than the map fall back
  const bool use_map = txmap_cap > 0 && (p1 - p0) <= txmap_cap && nt <= 256;
  if (use_map) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int lt = wv; lt < nt; lt += (int)(blockDim.x >> 6)) {
      const int a = (int)(s_ptr[lt] - p0), b = (int)(s_ptr[lt + 1] - p0);
      for (int q = a + lane; q < b; q += 64) s_tx[q] = (uint8_t)lt;
    }
    __syncthreads();
  }
  const int64_t step = (int64_t)blockDim.x * kEncodeU;
  // the next round's item loads are issued before this round's gathers and LDS work, so their
  // HBM latency overlaps the dependent chain of the current round
  int32_t nx[kEncodeU];
#pragma unroll
  for (int u = 0; u < kEncodeU; ++u) {
    const int64_t p = p0 + (int64_t)u * blockDim.x + threadIdx.x;
    nx[u] = p < p1 ? items[p] : -1;
  }
  for (int64_t pb = p0; pb < p1; pb += step) {
    int32_t it[kEncodeU];
#pragma unroll
    for (int u = 0; u < kEncodeU; ++u) {
      it[u] = nx[u];
      const int64_t p = pb + step + (int64_t)u * blockDim.x + threadIdx.x;
      nx[u] = p < p1 ? items[p] : -1;
    }
    int32_t rk[kEncodeU];
    if (fgroup) {
      // one 8-byte gather per item: the frequent bits of its 32-id group and the number of
      // frequent ids before the group; the rank comes from the LDS compact-index → rank table
#pragma unroll
      for (int u = 0; u < kEncodeU; ++u) {
        rk[u] = -1;
        if (it[u] < 0) continue;
        const unsigned long long g = fgroup[it[u] >> 5];
        const uint32_t m = (uint32_t)g, b = (uint32_t)it[u] & 31u;
        if ((m >> b) & 1u)
          rk[u] = s_c2r[(uint32_t)(g >> 32) + (uint32_t)__popc(m & ((1u << b) - 1u))] - r0;
      }
    } else {
#pragma unroll
      for (int u = 0; u < kEncodeU; ++u)
        if (fmask && it[u] >= 0 && !((fmask[it[u] >> 5] >> (it[u] & 31)) & 1u)) it[u] = -1;
#pragma unroll
      for (int u = 0; u < kEncodeU; ++u) rk[u] = it[u] >= 0 ? rank_of[it[u]] - r0 : -1;
    }
#pragma unroll
    for (int u = 0; u < kEncodeU; ++u) {
      if (rk[u] < 0 || rk[u] >= nr) continue;
      const int64_t p = pb + (int64_t)u * blockDim.x + threadIdx.x;
      int lo = 0, hi = nt;  // largest lt with s_ptr[lt] <= p
      if (use_map) {
        lo = s_tx[p - p0];
      } else {
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (s_ptr[mid] <= p) lo = mid; else hi = mid;
        }
      }
      atomicOr(&s_bm[(int64_t)rk[u] * TW + (lo >> 6)], 1ull << (lo & 63));
    }
  }
  __syncthreads();
  // only this shard's words (ceil(n_tx/64) of them): a neighbouring shard may own the next ones
  const int64_t wbase = word_off + (t0 >> 6);
  const int64_t wn = min((int64_t)TW, min(Wp - wbase, ((n_tx + 63) >> 6) - (t0 >> 6)));
  for (int64_t i = threadIdx.x; i < (int64_t)nr * TW; i += blockDim.x) {
    const int64_t row = i >> tw_log2, w = i & (TW - 1);
    if (w < wn) bm[(r0 + row) * Wp + wbase + w] = s_bm[i];
  }
}

// Multi-band encode for wide frequent sets (config 5: ~15k rows, more than one LDS slab).  The
// band-per-block kernel above re-reads every tile's items and redoes both lookup gathers for
// each of its row bands (10 bands at config 5).  Here one block owns a tile and all its bands:
// pass A looks every item up once and appends (rank, local transaction) pairs of the frequent
// ones to LDS (wave-aggregated append); pass B builds each band's slab from the pairs and writes
// it out.  A tile with more than kMbCap items is done in item chunks; chunks after the first
// OR their nonzero words into the words the first chunk stored.
constexpr int kMbCap = 8192;
constexpr int kMbBand = 1024;
__global__ __launch_bounds__(1024) void k_encode_multiband(const int64_t* __restrict__ tx_ptr,
                                                             const int32_t* __restrict__ items,
                                                             int64_t n_tx,
                                                             const int32_t* __restrict__ rank_of,
                                                             unsigned long long* __restrict__ bm,
                                                             int64_t Wp, int64_t word_off,
                                                             int64_t F,
                                                             const uint32_t* __restrict__ fmask) {
  constexpr int TW = 4;
  __shared__ unsigned long long s_bm[kMbBand * TW];
  __shared__ int64_t s_ptr[64 * TW + 1];
  __shared__ uint32_t s_pair[kMbCap];
  __shared__ uint32_t s_n;
  int64_t lb = blockIdx.x;  // XCD-aware tile order, as in k_encode_tile
  {
    const int64_t nb = gridDim.x, q = nb / 8, rr = nb % 8, x = lb % 8;
    lb = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + lb / 8;
  }
  const int64_t t0 = lb * 64 * TW;
  const int nt = (int)min((int64_t)(64 * TW), n_tx - t0);
  for (int i = threadIdx.x; i <= nt; i += blockDim.x) s_ptr[i] = tx_ptr[t0 + i];
  __syncthreads();
  const int64_t p0 = s_ptr[0], p1 = s_ptr[nt];
  const int64_t wbase = word_off + (t0 >> 6);
  const int64_t wn = min((int64_t)TW, min(Wp - wbase, ((n_tx + 63) >> 6) - (t0 >> 6)));
  const int lane = threadIdx.x & 63;
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  bool first = true;
  for (int64_t pc = p0; pc < p1 || first; pc += kMbCap) {
    const int64_t pe = min(p1, pc + kMbCap);
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    // pass A: lookups (mask gather, then rank gather for the frequent ids) and the append
    for (int64_t pb = pc; pb < pe; pb += (int64_t)blockDim.x * 4) {
      int32_t it[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t p = pb + (int64_t)u * blockDim.x + threadIdx.x;
        it[u] = p < pe ? items[p] : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (it[u] >= 0 && fmask && !((fmask[it[u] >> 5] >> (it[u] & 31)) & 1u)) it[u] = -1;
      int32_t rk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) rk[u] = it[u] >= 0 ? rank_of[it[u]] : -1;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool v = rk[u] >= 0;
        uint32_t e = 0;
        if (v) {
          const int64_t p = pb + (int64_t)u * blockDim.x + threadIdx.x;
          int lo = 0, hi = nt;  // largest lt with s_ptr[lt] <= p
          while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (s_ptr[mid] <= p) lo = mid; else hi = mid;
          }
          e = ((uint32_t)rk[u] << 8) | (uint32_t)lo;
        }
        const unsigned long long bal = __ballot(v);
        uint32_t base = 0;
        if (lane == 0 && bal) base = atomicAdd(&s_n, (uint32_t)__popcll(bal));
        base = __shfl(base, 0, 64);
        if (v) s_pair[base + (uint32_t)__popcll(bal & lt_mask)] = e;
      }
    }
    __syncthreads();
    const int np = (int)s_n;
    // pass B: one slab per band from the pairs
    for (int64_t r0 = 0; r0 < F; r0 += kMbBand) {
      const int nr = (int)min((int64_t)kMbBand, F - r0);
      for (int i = threadIdx.x; i < nr * TW; i += blockDim.x) s_bm[i] = 0ull;
      __syncthreads();
      for (int i = threadIdx.x; i < np; i += blockDim.x) {
        const uint32_t e = s_pair[i];
        const int64_t rr = (int64_t)(e >> 8) - r0;
        if (rr >= 0 && rr < nr) {
          const uint32_t lt = e & 255u;
          atomicOr(&s_bm[rr * TW + (lt >> 6)], 1ull << (lt & 63));
        }
      }
      __syncthreads();
      for (int i = threadIdx.x; i < nr * TW; i += blockDim.x) {
        const int row = i >> 2, w = i & 3;
        if (w >= wn) continue;
        unsigned long long* dst = &bm[(r0 + row) * Wp + wbase + w];
        if (first) *dst = s_bm[i];
        else if (s_bm[i]) atomicOr(dst, s_bm[i]);
      }
      __threadfence_block();
      __syncthreads();
    }
    first = false;
    if (pe >= p1) break;
  }
}

// flag(i) = (i < n && cnt[i] >= minsup); scanning n+1 flags gives pos[n] = #survivors directly
struct FlagOp {
  const uint32_t* cnt;
  int64_t n;
  uint32_t minsup;
  __host__ __device__ int64_t operator()(int64_t i) const {
    return (i < n && cnt[i] >= minsup) ? 1 : 0;
  }
};

// ----------------------------------------------------------------------------------------
// candidate → (row a, sibling b) decode: largest a with cand_off[a] <= c
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t find_row(const int64_t* __restrict__ cand_off, int64_t n_rows,
                                            int64_t c) {
  int64_t lo = 0, hi = n_rows;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (cand_off[mid] <= c) lo = mid; else hi = mid;
  }
  return lo;
}

// ----------------------------------------------------------------------------------------
// O8 |S|>=3: team-per-candidate AND + popcount (TS lanes of a wave64 per candidate)
// ----------------------------------------------------------------------------------------
// Long rows with few candidates (the 10M-100M shapes: a few hundred candidates of 1.5M words)
// split each candidate's row into `split` contiguous slices, one team each, so the grid still
// fills the chip; partial counts are combined with integer atomics (cnt zeroed by the host).
template <int TS>
__global__ __launch_bounds__(kBlock) void k_extend_count(const unsigned long long* __restrict__ bm,
                                                         int64_t Wp,
                                                         const int64_t* __restrict__ cand_off,
                                                         int64_t n_rows, int64_t c0, int64_t c1,
                                                         int64_t split,
                                                         uint32_t* __restrict__ cnt) {
  const int tl = threadIdx.x & (TS - 1);
  const int64_t team = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / TS;
  const int64_t nteams = ((int64_t)gridDim.x * blockDim.x) / TS;
  const int64_t n2 = Wp >> 1;
  for (int64_t wi = team; wi < (c1 - c0) * split; wi += nteams) {
    const int64_t c = c0 + wi / split, part = wi % split;
    const int64_t a = find_row(cand_off, n_rows, c);
    const int64_t b = a + 1 + (c - cand_off[a]);
    const ulonglong2* x = reinterpret_cast<const ulonglong2*>(bm + a * Wp);
    const ulonglong2* y = reinterpret_cast<const ulonglong2*>(bm + b * Wp);
    const int64_t lo = n2 * part / split, hi = n2 * (part + 1) / split;
    uint32_t s = 0;
    for (int64_t w = lo + tl; w < hi; w += TS) {
      const ulonglong2 u = x[w], v = y[w];
      s += (uint32_t)__popcll(u.x & v.x) + (uint32_t)__popcll(u.y & v.y);
    }
#pragma unroll
    for (int off = TS >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, TS);
    if (tl == 0) {
      if (split == 1) cnt[c - c0] = s;
      else if (s) atomicAdd(&cnt[c - c0], s);
    }
  }
}

template <int TS>
__global__ __launch_bounds__(kBlock) void k_extend_materialize(
    const unsigned long long* __restrict__ bm, int64_t Wp, const int64_t* __restrict__ cand_off,
    int64_t n_rows, const int32_t* __restrict__ rank, const int64_t* __restrict__ gid,
    const int32_t* __restrict__ ids, int64_t c0, int64_t c1, const uint32_t* __restrict__ cnt,
    uint32_t minsup, const int64_t* __restrict__ pos, int64_t split, LevelOut o) {
  const int tl = threadIdx.x & (TS - 1);
  const int64_t team = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / TS;
  const int64_t nteams = ((int64_t)gridDim.x * blockDim.x) / TS;
  const int64_t n2 = Wp >> 1;
  for (int64_t wi = team; wi < (c1 - c0) * split; wi += nteams) {
    const int64_t c = c0 + wi / split, part = wi % split;
    const uint32_t k = cnt[c - c0];
    if (k < minsup) continue;  // team-uniform
    const int64_t a = find_row(cand_off, n_rows, c);
    const int64_t b = a + 1 + (c - cand_off[a]);
    const int64_t s = pos[c - c0];
    if (o.bm) {  // leaf level (max_len reached): no child bitmaps, rows or classes
      const ulonglong2* x = reinterpret_cast<const ulonglong2*>(bm + a * Wp);
      const ulonglong2* y = reinterpret_cast<const ulonglong2*>(bm + b * Wp);
      ulonglong2* z = reinterpret_cast<ulonglong2*>(o.bm + s * Wp);
      const int64_t lo = n2 * part / split, hi = n2 * (part + 1) / split;
      for (int64_t w = lo + tl; w < hi; w += TS) {
        const ulonglong2 u = x[w], v = y[w];
        z[w] = make_ulonglong2(u.x & v.x, u.y & v.y);
      }
    }
    if (tl == 0 && part == 0) {
      const int32_t rb = rank[b];
      if (o.bm) {
        o.rank[s] = rb;
        o.gid[s] = o.out_base + s;
        const int64_t re = pos[cand_off[a + 1] - c0];
        o.row_end[s] = (int32_t)re;
        o.len[s] = re - s - 1;
      }
      o.out_parent[o.out_base + s] = gid[a];
      o.out_item[o.out_base + s] = ids[rb];
      o.out_count[o.out_base + s] = k;
      o.out_depth[o.out_base + s] = o.depth;
    }
  }
}

// Survivor-driven materialize for long rows.  The candidate-driven kernel above gives each
// candidate one team, so at level 2 of a 100M-transaction shard (284k candidates, ~160
// survivors of 1.56M words each) a handful of wave64 teams copy 12.5 MB rows alone.  Here the
// survivors are listed first (k_surv_index: surv[pos[c]] = c) and the grid runs over
// (survivor, slice) pairs, so every survivor's AND row is streamed by many teams at once.
__global__ __launch_bounds__(kBlock) void k_surv_index(const uint32_t* __restrict__ cnt,
                                                       uint32_t minsup,
                                                       const int64_t* __restrict__ pos,
                                                       int64_t c0, int64_t nc,
                                                       int64_t* __restrict__ surv) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nc;
       i += (int64_t)gridDim.x * blockDim.x)
    if (cnt[i] >= minsup) surv[pos[i]] = c0 + i;
}

__global__ __launch_bounds__(kBlock) void k_materialize_surv(
    const unsigned long long* __restrict__ bm, int64_t Wp, const int64_t* __restrict__ cand_off,
    int64_t n_rows, const int32_t* __restrict__ rank, const int64_t* __restrict__ gid,
    const int32_t* __restrict__ ids, int64_t c0, const uint32_t* __restrict__ cnt,
    const int64_t* __restrict__ pos, const int64_t* __restrict__ surv, int64_t n_surv,
    int64_t split, LevelOut o) {
  constexpr int TS = 64;
  const int tl = threadIdx.x & (TS - 1);
  const int64_t team = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / TS;
  const int64_t nteams = ((int64_t)gridDim.x * blockDim.x) / TS;
  const int64_t n2 = Wp >> 1;
  for (int64_t wi = team; wi < n_surv * split; wi += nteams) {
    const int64_t s = wi / split, part = wi % split;
    const int64_t c = surv[s];
    const int64_t a = find_row(cand_off, n_rows, c);
    const int64_t b = a + 1 + (c - cand_off[a]);
    const ulonglong2* x = reinterpret_cast<const ulonglong2*>(bm + a * Wp);
    const ulonglong2* y = reinterpret_cast<const ulonglong2*>(bm + b * Wp);
    ulonglong2* z = reinterpret_cast<ulonglong2*>(o.bm + s * Wp);
    const int64_t lo = n2 * part / split, hi = n2 * (part + 1) / split;
    for (int64_t w = lo + tl; w < hi; w += TS) {
      const ulonglong2 u = x[w], v = y[w];
      z[w] = make_ulonglong2(u.x & v.x, u.y & v.y);
    }
    if (tl == 0 && part == 0) {
      const int32_t rb = rank[b];
      o.rank[s] = rb;
      o.gid[s] = o.out_base + s;
      const int64_t re = pos[cand_off[a + 1] - c0];
      o.row_end[s] = (int32_t)re;
      o.len[s] = re - s - 1;
      o.out_parent[o.out_base + s] = gid[a];
      o.out_item[o.out_base + s] = ids[rb];
      o.out_count[o.out_base + s] = cnt[c - c0];
      o.out_depth[o.out_base + s] = o.depth;
    }
  }
}

// ----------------------------------------------------------------------------------------
// O8 level 2: tiled bit-GEMM  G[i][j] = popcount(row_i & row_j), 64x64 output tile / block,
// K staged through LDS in transposed [k][row] layout (16 words per stage).
// ----------------------------------------------------------------------------------------
constexpr int kGT = 64;   // tile rows/cols
constexpr int kGK = 16;   // words per K stage

// KGK words per K stage: 16 for long rows; short rows (the playlist datasets, Wp <= 48) take
// the whole row in ONE stage, so the block's latency chain is one load round trip, not three
template <int KGK>
__global__ __launch_bounds__(kBlock) void k_pair_gram_popcount(
    const unsigned long long* __restrict__ bm, int64_t Wp, int64_t F_host, int64_t n_tiles,
    uint32_t* __restrict__ out, int64_t ld, const int64_t* __restrict__ dF) {
  constexpr int kGK = KGK;
  __shared__ unsigned long long As[kGK][kGT + 2];
  __shared__ unsigned long long Bs[kGK][kGT + 2];
  // F from the device when the selection ran there (grid sized for an upper bound)
  const int64_t F = dF ? *dF : F_host;
  // upper-triangular tile decode: blockIdx.x → (ti <= tj)
  int64_t idx = blockIdx.x, ti = 0;
  while (idx >= n_tiles - ti) { idx -= n_tiles - ti; ++ti; }
  const int64_t tj = ti + idx;
  const int64_t r0 = ti * kGT, q0 = tj * kGT;
  if (q0 >= F) return;  // block-uniform
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  uint32_t acc[4][4] = {};
  // staging map: thread → (row = tid>>2, words (tid&3)*(kGK/4) .. +kGK/4-1)
  constexpr int kPerT = kGK / 4;
  const int lr = threadIdx.x >> 2, lk = (threadIdx.x & 3) * kPerT;
  // split-K over blockIdx.y (word slices, multiples of kGK); partials combine with atomics
  const int64_t slice = (((Wp + gridDim.y - 1) / gridDim.y) + kGK - 1) / kGK * kGK;
  const int64_t kb = (int64_t)blockIdx.y * slice, ke = min(Wp, kb + slice);
  for (int64_t k0 = kb; k0 < ke; k0 += kGK) {
#pragma unroll
    for (int i = 0; i < kPerT; ++i) {
      const int64_t kk = k0 + lk + i;
      const int64_t ra = r0 + lr, rb = q0 + lr;
      As[lk + i][lr] = (ra < F && kk < ke) ? bm[ra * Wp + kk] : 0ull;
      Bs[lk + i][lr] = (rb < F && kk < ke) ? bm[rb * Wp + kk] : 0ull;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < kGK; ++k) {
      unsigned long long a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[k][ty * 4 + i]; b[i] = Bs[k][tx * 4 + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += (uint32_t)__popcll(a[i] & b[j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t r = r0 + ty * 4 + i;
    if (r >= F) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t q = q0 + tx * 4 + j;
      if (q < F && q > r) {
        if (gridDim.y == 1) out[r * ld + q] = acc[i][j];
        else if (acc[i][j]) atomicAdd(&out[r * ld + q], acc[i][j]);
      }
    }
  }
}

// Rectangular bit-GEMM C[i][j] += popcount(A_i & B_j) over Wp words (the ring-pass pair
// counter's per-step product of the owned rows against a rotating transaction block).  Same
// LDS tiling as the square kernel; split-K over blockIdx.y with integer atomics.
__global__ __launch_bounds__(kBlock) void k_bitgemm_rect(const unsigned long long* __restrict__ A,
                                                         int64_t Fa, const unsigned long long* __restrict__ B,
                                                         int64_t Fb, int64_t Wp, int64_t ntb,
                                                         uint32_t* __restrict__ C, int64_t ldc) {
  __shared__ unsigned long long As[kGK][kGT + 2];
  __shared__ unsigned long long Bs[kGK][kGT + 2];
  const int64_t ti = blockIdx.x / ntb, tj = blockIdx.x % ntb;
  const int64_t r0 = ti * kGT, q0 = tj * kGT;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  uint32_t acc[4][4] = {};
  const int lr = threadIdx.x >> 2, lk = (threadIdx.x & 3) * 4;
  const int64_t slice = (((Wp + gridDim.y - 1) / gridDim.y) + kGK - 1) / kGK * kGK;
  const int64_t kb = (int64_t)blockIdx.y * slice, ke = min(Wp, kb + slice);
  for (int64_t k0 = kb; k0 < ke; k0 += kGK) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t kk = k0 + lk + i;
      const int64_t ra = r0 + lr, rb = q0 + lr;
      As[lk + i][lr] = (ra < Fa && kk < ke) ? A[ra * Wp + kk] : 0ull;
      Bs[lk + i][lr] = (rb < Fb && kk < ke) ? B[rb * Wp + kk] : 0ull;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < kGK; ++k) {
      unsigned long long a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[k][ty * 4 + i]; b[i] = Bs[k][tx * 4 + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += (uint32_t)__popcll(a[i] & b[j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t r = r0 + ty * 4 + i;
    if (r >= Fa) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t q = q0 + tx * 4 + j;
      if (q < Fb && acc[i][j]) atomicAdd(&C[r * ldc + q], acc[i][j]);
    }
  }
}

// gram (dense F x F, i<j valid) → per-candidate counts in (a, b) row-major candidate order
__global__ void k_gram_to_cand(const uint32_t* __restrict__ gram, int64_t F,
                               const int64_t* __restrict__ cand_off, int64_t c0, int64_t c1,
                               uint32_t* __restrict__ cnt) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t c = c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < c1; c += nthr) {
    const int64_t a = find_row(cand_off, F, c);
    const int64_t b = a + 1 + (c - cand_off[a]);
    cnt[c - c0] = gram[a * F + b];
  }
}

int team_size(int64_t Wp) {
  const int64_t chunks = Wp >> 1;  // 16-byte chunks per row
  if (chunks >= 128) return 64;
  if (chunks >= 64) return 32;
  if (chunks >= 32) return 16;
  if (chunks >= 12) return 8;
  return 4;
}

}  // namespace

void item_support(const int32_t* items, int64_t nnz, int32_t n_items, uint32_t* counts,
                  hipStream_t s) {
  if (nnz <= 0) return;
  // the kernels read int4 vectors: peel a misaligned head (tile sub-ranges start anywhere)
  const int64_t mis = ((uintptr_t)items & 15) / 4;
  const int64_t head = mis ? std::min<int64_t>(nnz, 4 - mis) : 0;
  if (head) {
    hipLaunchKernelGGL(k_item_support<false>, dim3(1), dim3(64), 0, s, items, head, n_items, counts);
    items += head;
    nnz -= head;
    if (nnz <= 0) {
      KMLS_HIP(hipGetLastError());
      return;
    }
  }
  const size_t lds = (size_t)n_items * sizeof(uint32_t);
  if (lds <= 64 * 1024) {
    // 16 items per thread: a 240k-item playlist dataset spreads over ~60 blocks (64 per thread
    // left 15 blocks latency-bound); the per-block flush is n_items atomics at most
    const int g = grid_for(nnz, kBlock * 16, 1024);
    hipLaunchKernelGGL(k_item_support<true>, dim3(g), dim3(kBlock), lds, s, items, nnz, n_items,
                       counts);
  } else {
    const int g = grid_for(nnz, kBlock * 64, 1024);
    hipLaunchKernelGGL(k_item_support_hash, dim3(g), dim3(kBlock), 0, s, items, nnz, counts);
  }
  KMLS_HIP(hipGetLastError());
}

bool encode_bitmap_tiled(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                         const int32_t* rank_of, uint64_t* bm, int64_t Wp, int64_t word_off,
                         int64_t F, hipStream_t s, const uint32_t* fmask,
                         const unsigned long long* fgroup, const int32_t* c2r) {
  if (n_tx <= 0 || F <= 0 || F > kEncodeTileMaxF) return false;
  // frequent sets wider than one slab: the multi-band kernel (one block per tile, every band;
  // 22.2 -> 11.7 ms at config-5 10M against one block per (tile, band)), 256 threads (12.4 ms
  // vs 13.2 at 1024)
  if (F > 1536 && F < (1 << 24)) {
    const int64_t tiles = (n_tx + 255) / 256;
    if (tiles > INT32_MAX) return false;
    hipLaunchKernelGGL(k_encode_multiband, dim3((unsigned)tiles), dim3(256), 0, s,
                       tx_ptr, items, n_tx, rank_of, (unsigned long long*)bm, Wp, word_off, F, fmask);
    KMLS_HIP(hipGetLastError());
    return true;
  }
  if (F > kEncodeGroupMaxF) fgroup = nullptr, c2r = nullptr;  // c2r must fit LDS beside the slab
  // words per tile: the slab within 48 KB of LDS.  TW = 4 words (32-byte row segments: measured
  // ahead of 8 and 2 at 100M x 754, 19.5 / 18.3 / 23.2 ms); XCD-aware tile order; the item ->
  // transaction byte map sized for a tile of 256 transactions of up to 32 items on average
  constexpr int64_t kSlab = 48 * 1024;
  const int tw_log2 = 2;
  const int64_t TW = 1ll << tw_log2;
  const int64_t band = std::min<int64_t>(F, kSlab / (8 * TW));
  const int64_t n_bands = (F + band - 1) / band;
  const int txmap_cap = (int)(64 * TW * 32);
  const size_t lds = (size_t)band * TW * 8 + (size_t)(64 * TW + 1) * 8 +
                     (fgroup ? (size_t)F * 4 : 0) + (size_t)txmap_cap;
  const int64_t blocks = (n_tx + 64 * TW - 1) / (64 * TW) * n_bands;
  if (blocks > INT32_MAX) return false;
  // 512 threads: LDS-bound to 4 blocks per CU at 40 VGPRs, so more waves per block are more waves
  // per CU on the same LDS (12.3 ms at 100M against 13.1 at 256 and 15.9 at 1024)
  hipLaunchKernelGGL(k_encode_tile, dim3((unsigned)blocks), dim3(512), lds, s, tx_ptr, items,
                     n_tx, rank_of, (unsigned long long*)bm, Wp, word_off, F, tw_log2, (int)band,
                     fmask, true, fgroup, c2r, txmap_cap);
  KMLS_HIP(hipGetLastError());
  return true;
}

void encode_bitmap(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                   const int32_t* rank_of, uint64_t* bm, int64_t Wp, int64_t word_off,
                   hipStream_t s, const uint32_t* fmask) {
  if (n_tx <= 0) return;
  hipLaunchKernelGGL(k_encode_bitmap, dim3(grid_for(n_tx, kBlock / 64, 8192)), dim3(kBlock), 0, s,
                     tx_ptr, items, n_tx, rank_of, (unsigned long long*)bm, Wp, word_off, fmask);
  KMLS_HIP(hipGetLastError());
}

__global__ void k_add_u32(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, int64_t n) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr) dst[i] += src[i];
}

void add_u32(uint32_t* dst, const uint32_t* src, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_add_u32, dim3(grid_for(n, kBlock, 2048)), dim3(kBlock), 0, s, dst, src, n);
  KMLS_HIP(hipGetLastError());
}

size_t support_scratch_bytes(int64_t nnz, int64_t n_items) {
  const int64_t P = (n_items + kPartBins - 1) / kPartBins;
  if (P > kPartMax || n_items <= 16384) return 0;
  const int64_t n = P * kPartGridMax;
  return ((size_t)nnz * 2 + 255) / 256 * 256 + (size_t)(n + 1) * 8 * 2 + scan_temp_bytes(n) + 256;
}

bool item_support_partitioned(const int32_t* items, int64_t nnz, int32_t n_items, uint32_t* counts,
                              void* scratch, size_t scratch_bytes, hipStream_t s) {
  const int64_t P = ((int64_t)n_items + kPartBins - 1) / kPartBins;
  if (nnz <= 0 || P > kPartMax || scratch_bytes < support_scratch_bytes(nnz, n_items)) return false;
  // blocks of passes 1-2: 1024 = 4 resident blocks per CU (the scatter's 93 VGPRs allow 5);
  // 1280 / 2048 measured no faster (support 8.73 / 8.62 vs 8.37 ms at 100M)
  const int64_t G = kPartGrid;
  const int64_t n = P * G;
  char* q = (char*)scratch;
  uint16_t* part = (uint16_t*)q;
  q += ((size_t)nnz * 2 + 255) / 256 * 256;
  int64_t* blk = (int64_t*)q;
  q += (size_t)(n + 1) * 8;
  int64_t* off = (int64_t*)q;
  q += (size_t)(n + 1) * 8;
  const size_t tb = scan_temp_bytes(n);
  hipLaunchKernelGGL(k_part_hist, dim3((unsigned)G), dim3(kBlock), 0, s, items, nnz, (int)P, blk);
  exclusive_scan_i64(blk, off, n, q, tb, s);
  hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)G), dim3(kBlock), 0, s, items, nnz, (int)P, off,
                     part);
  // pass 3: equal global slices, one 128 KB-LDS block per CU: 512 slices = 2 rounds over the
  // 256 CUs (per-partition blocks measured 8.79 vs 8.70 ms support at 100M x 1M)
  {
    const unsigned B = (unsigned)std::min<int64_t>(512, std::max<int64_t>(1, nnz / 65536));
    hipLaunchKernelGGL(k_part_count_bal, dim3(B), dim3(1024), 0, s, part, off, (int)G, (int)P,
                       (int64_t)n_items, counts);
  }
  KMLS_HIP(hipGetLastError());
  return true;
}

// ----------------------------------------------------------------------------------------
// Device selection for large vocabularies (the tx-DP call): frequent items ranked by (count asc,
// id asc) = select_frequent, without copying the support vector to the host.  One 64-bit key per
// item (count << 32 | id; ~0 for infrequent items, which sort last), a radix sort, and a scatter
// of the first F keys into ids / counts / rank_of / the frequent-item mask.
__global__ void k_sel_keys(const uint32_t* __restrict__ cnt, int64_t n_items, uint32_t c1,
                           unsigned long long* __restrict__ keys, int32_t* __restrict__ rank_of,
                           uint32_t* __restrict__ fmask, unsigned long long* __restrict__ dF) {
  __shared__ unsigned int s_n;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_items) {
    const uint32_t c = cnt[i];
    const bool f = c >= c1;
    keys[i] = f ? (((unsigned long long)c << 32) | (unsigned long long)i) : ~0ull;
    rank_of[i] = -1;
    if (f) atomicAdd(&s_n, 1u);
  }
  if (fmask && i < (n_items + 31) / 32) fmask[i] = 0u;
  __syncthreads();
  if (threadIdx.x == 0 && s_n) atomicAdd(dF, (unsigned long long)s_n);
}

__global__ void k_sel_scatter(const unsigned long long* __restrict__ keys, int64_t n_items,
                              const unsigned long long* __restrict__ dF, int32_t* __restrict__ ids,
                              uint32_t* __restrict__ fcounts, int32_t* __restrict__ rank_of,
                              uint32_t* __restrict__ fmask) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= (int64_t)*dF || r >= n_items) return;
  const unsigned long long k = keys[r];
  const int32_t id = (int32_t)(k & 0xFFFFFFFFull);
  ids[r] = id;
  fcounts[r] = (uint32_t)(k >> 32);
  rank_of[id] = (int32_t)r;
  if (fmask) atomicOr(&fmask[id >> 5], 1u << (id & 31));
}

size_t select_large_temp_bytes(int64_t n_items) {
  size_t b = 0;
  KMLS_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, b, (const unsigned long long*)nullptr,
                                             (unsigned long long*)nullptr, (int)n_items));
  return 2 * (((size_t)n_items * 8 + 255) & ~(size_t)255) + 256 + b;
}

void select_large(const uint32_t* cnt, int64_t n_items, uint32_t c1, void* tmp, size_t tmp_bytes,
                  int32_t* ids, uint32_t* fcounts, int32_t* rank_of, uint32_t* fmask,
                  unsigned long long* dF, hipStream_t s) {
  if (tmp_bytes < select_large_temp_bytes(n_items))
    throw std::runtime_error("select_large: scratch too small");
  const size_t kb = ((size_t)n_items * 8 + 255) & ~(size_t)255;
  unsigned long long* keys = (unsigned long long*)tmp;
  unsigned long long* sorted = (unsigned long long*)((char*)tmp + kb);
  void* cub = (char*)tmp + 2 * kb + 256;
  size_t cb = tmp_bytes - 2 * kb - 256;
  KMLS_HIP(hipMemsetAsync(dF, 0, 8, s));
  const unsigned nb = (unsigned)((n_items + 255) / 256);
  hipLaunchKernelGGL(k_sel_keys, dim3(nb), dim3(256), 0, s, cnt, n_items, c1, keys, rank_of, fmask,
                     dF);
  KMLS_HIP(hipcub::DeviceRadixSort::SortKeys(cub, cb, keys, sorted, (int)n_items, 0, 64, s));
  hipLaunchKernelGGL(k_sel_scatter, dim3(nb), dim3(256), 0, s, sorted, n_items, dF, ids, fcounts,
                     rank_of, fmask);
  KMLS_HIP(hipGetLastError());
}

// Encode lookup tables from the frequent-item mask (any selection path): per 32-id group its mask
// bits and the number of frequent ids before it (one 8-byte gather per item in the encode), and
// compact index (frequent ids in id order) → Eclat rank.
__global__ void k_grp_pop(const uint32_t* __restrict__ fmask, int64_t G, int64_t* __restrict__ pop) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < G) pop[g] = __popc(fmask[g]);
  if (g == G) pop[G] = 0;
}
__global__ void k_grp_fill(const uint32_t* __restrict__ fmask, int64_t G,
                           const int64_t* __restrict__ pre, const int32_t* __restrict__ rank_of,
                           unsigned long long* __restrict__ fgroup, int32_t* __restrict__ c2r) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  const uint32_t m = fmask[g];
  const int64_t base = pre[g];
  fgroup[g] = (unsigned long long)m | ((unsigned long long)base << 32);
  uint32_t x = m;
  for (int j = 0; x; ++j, x &= x - 1u)
    c2r[base + j] = rank_of[g * 32 + __builtin_ctz(x)];
}

size_t frequent_groups_temp_bytes(int64_t n_items) {
  const int64_t G = (n_items + 31) / 32;
  return 2 * (((size_t)(G + 1) * 8 + 255) & ~(size_t)255) + scan_temp_bytes(G);
}

void frequent_groups(const uint32_t* fmask, int64_t n_items, const int32_t* rank_of,
                     unsigned long long* fgroup, int32_t* c2r, void* tmp, size_t tmp_bytes,
                     hipStream_t s) {
  const int64_t G = (n_items + 31) / 32;
  if (tmp_bytes < frequent_groups_temp_bytes(n_items))
    throw std::runtime_error("frequent_groups: scratch too small");
  const size_t ab = ((size_t)(G + 1) * 8 + 255) & ~(size_t)255;
  int64_t* pop = (int64_t*)tmp;
  int64_t* pre = (int64_t*)((char*)tmp + ab);
  void* cub = (char*)tmp + 2 * ab;
  const unsigned nb = (unsigned)((G + 1 + 255) / 256);
  hipLaunchKernelGGL(k_grp_pop, dim3(nb), dim3(256), 0, s, fmask, G, pop);
  exclusive_scan_i64(pop, pre, G, cub, scan_temp_bytes(G), s);
  hipLaunchKernelGGL(k_grp_fill, dim3(nb), dim3(256), 0, s, fmask, G, pre, rank_of, fgroup, c2r);
  KMLS_HIP(hipGetLastError());
}

size_t scan_temp_bytes(int64_t n) {
  size_t bytes = 0;
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int64_t*)nullptr,
                                            (int64_t*)nullptr, (int)(n + 1)));
  return bytes;
}

// in has n+1 entries with in[n] == 0, so out[n] is the total
void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, void* temp, size_t temp_bytes,
                        hipStream_t s) {
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)(n + 1), s));
}

using FlagIt = hipcub::TransformInputIterator<int64_t, FlagOp, hipcub::CountingInputIterator<int64_t>>;

size_t flag_scan_temp_bytes(int64_t n) {
  size_t bytes = 0;
  FlagIt it(hipcub::CountingInputIterator<int64_t>(0), FlagOp{nullptr, n, 0});
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, it, (int64_t*)nullptr, (int)(n + 1)));
  return bytes;
}

void flag_scan(const uint32_t* cnt, uint32_t minsup, int64_t n, int64_t* pos, void* temp,
               size_t temp_bytes, hipStream_t s) {
  FlagIt it(hipcub::CountingInputIterator<int64_t>(0), FlagOp{cnt, n, minsup});
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, it, pos, (int)(n + 1), s));
}

// After the flag scan of chunk [c0, c1) over rows [a0, a1): child class of row a has
// size k_a = pos[cand_off[a+1]-c0] - pos[cand_off[a]-c0]; the next level's candidate total is
// Σ k_a (k_a - 1) / 2.  Written to out[1] (out[0] = #survivors) so ONE readback serves both.
__global__ __launch_bounds__(kBlock) void k_child_totals(const int64_t* __restrict__ cand_off,
                                                        int64_t a0, int64_t a1, int64_t c0,
                                                        const int64_t* __restrict__ pos, int64_t nc,
                                                        unsigned long long* __restrict__ out) {
  __shared__ unsigned long long part[kBlock / 64];
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  unsigned long long acc = 0;
  for (int64_t a = a0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; a < a1; a += nthr) {
    const int64_t k = pos[cand_off[a + 1] - c0] - pos[cand_off[a] - c0];
    acc += (unsigned long long)(k * (k - 1) / 2);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  // one same-address atomic per block, not per wave: they serialise in L2
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) t += part[w];
    if (t) atomicAdd(&out[1], t);
    if (blockIdx.x == 0) atomicAdd(&out[0], (unsigned long long)pos[nc]);
  }
}

void child_totals(const int64_t* cand_off, int64_t a0, int64_t a1, int64_t c0, const int64_t* pos,
                  int64_t nc, uint64_t* out2, hipStream_t s) {
  KMLS_HIP(hipMemsetAsync(out2, 0, 2 * sizeof(uint64_t), s));
  hipLaunchKernelGGL(k_child_totals, dim3(grid_for(std::max<int64_t>(a1 - a0, 1), kBlock, 256)),
                     dim3(kBlock), 0, s, cand_off, a0, a1, c0, pos, nc,
                     (unsigned long long*)out2);
  KMLS_HIP(hipGetLastError());
}

#define KMLS_TEAM_DISPATCH(TS_VAR, KERNEL, ...)                                              \
  switch (TS_VAR) {                                                                          \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                               \
    case 8: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;                               \
    case 16: hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__); break;                             \
    case 32: hipLaunchKernelGGL(KERNEL<32>, __VA_ARGS__); break;                             \
    default: hipLaunchKernelGGL(KERNEL<64>, __VA_ARGS__); break;                             \
  }

// row slices per candidate: enough (candidate, slice) teams for ~8 wave64 teams per CU, each
// slice >= 2048 16-byte units (32 KB per row)
std::atomic<long long> g_split_launches{0};  // extend_count launches that split rows (tests)

static int64_t extend_split(int64_t Wp, int64_t n_cand, int ts) {
  if (ts != 64 || n_cand <= 0) return 1;
  const int64_t forced = test_hook("extend_split", 0);  // slices per row
  if (forced > 0) return std::max<int64_t>(1, std::min<int64_t>(forced, (Wp >> 1) / 64));
  const int64_t want = (256 * 8 + n_cand - 1) / n_cand;
  return std::max<int64_t>(1, std::min<int64_t>(want, (Wp >> 1) / 2048));
}

long long extend_split_launches() { return g_split_launches.load(); }

void extend_count(const uint64_t* bm, int64_t Wp, const int64_t* cand_off, int64_t n_rows,
                  int64_t c0, int64_t c1, uint32_t* cnt, hipStream_t s) {
  if (c1 <= c0) return;
  const int ts = team_size(Wp);
  const int64_t teams_per_block = kBlock / ts;
  const int64_t split = extend_split(Wp, c1 - c0, ts);
  if (split > 1) {
    KMLS_HIP(hipMemsetAsync(cnt, 0, (size_t)(c1 - c0) * sizeof(uint32_t), s));
    g_split_launches.fetch_add(1);
  }
  const int g = grid_for((c1 - c0) * split, (int)teams_per_block, 256 * 32);
  KMLS_TEAM_DISPATCH(ts, k_extend_count, dim3(g), dim3(kBlock), 0, s,
                     (const unsigned long long*)bm, Wp, cand_off, n_rows, c0, c1, split, cnt);
  KMLS_HIP(hipGetLastError());
}

void extend_materialize(const uint64_t* bm, int64_t Wp, const int64_t* cand_off, int64_t n_rows,
                        const int32_t* rank, const int64_t* gid, const int32_t* ids, int64_t c0,
                        int64_t c1, const uint32_t* cnt, uint32_t minsup, const int64_t* pos,
                        const LevelOut& o, hipStream_t s, int64_t n_surv, int64_t* surv) {
  if (c1 <= c0) return;
  const int ts = team_size(Wp);
  const int64_t teams_per_block = kBlock / ts;
  // long rows with a known survivor count: survivor-driven grid
  if (o.bm && ts == 64 && n_surv > 0 && surv) {
    hipLaunchKernelGGL(k_surv_index, dim3(grid_for(c1 - c0, kBlock, 2048)), dim3(kBlock), 0, s,
                       cnt, minsup, pos, c0, c1 - c0, surv);
    // >= 8192 teams over the survivors' rows, slices of >= 1024 16-byte chunks
    const int64_t sp = std::max<int64_t>(
        1, std::min<int64_t>((8192 + n_surv - 1) / n_surv, (Wp >> 1) / 1024));
    const int g = grid_for(n_surv * sp, kBlock / 64, 256 * 32);
    hipLaunchKernelGGL(k_materialize_surv, dim3(g), dim3(kBlock), 0, s,
                       (const unsigned long long*)bm, Wp, cand_off, n_rows, rank, gid, ids, c0, cnt,
                       pos, surv, n_surv, sp, o);
    KMLS_HIP(hipGetLastError());
    return;
  }
  const int64_t split = o.bm ? extend_split(Wp, c1 - c0, ts) : 1;  // leaves copy no words
  const int g = grid_for((c1 - c0) * split, (int)teams_per_block, 256 * 32);
  KMLS_TEAM_DISPATCH(ts, k_extend_materialize, dim3(g), dim3(kBlock), 0, s,
                     (const unsigned long long*)bm, Wp, cand_off, n_rows, rank, gid, ids, c0, c1,
                     cnt, minsup, pos, split, o);
  KMLS_HIP(hipGetLastError());
}

void pair_gram_popcount(const uint64_t* bm, int64_t Wp, int64_t F, uint32_t* out, hipStream_t s) {
  if (F < 2) return;
  const int64_t nt = (F + kGT - 1) / kGT;
  const int64_t blocks = nt * (nt + 1) / 2;
  const int64_t ks = std::max<int64_t>(1, std::min<int64_t>((1024 + blocks - 1) / blocks, Wp / 1024));
  if (Wp <= 48 && ks == 1)
    hipLaunchKernelGGL(k_pair_gram_popcount<48>, dim3((unsigned)blocks, 1), dim3(kBlock), 0, s,
                       (const unsigned long long*)bm, Wp, F, nt, out, F, (const int64_t*)nullptr);
  else
    hipLaunchKernelGGL(k_pair_gram_popcount<16>, dim3((unsigned)blocks, (unsigned)ks), dim3(kBlock), 0, s,
                       (const unsigned long long*)bm, Wp, F, nt, out, F, (const int64_t*)nullptr);
  KMLS_HIP(hipGetLastError());
}

namespace {
int64_t gram_split_k(int64_t Wp, int64_t F_max) {
  const int64_t nt = (F_max + kGT - 1) / kGT;
  const int64_t blocks = nt * (nt + 1) / 2;
  return std::max<int64_t>(1, std::min<int64_t>((1024 + blocks - 1) / blocks, Wp / 1024));
}
}  // namespace

bool pair_gram_dev_needs_zero(int64_t Wp, int64_t F_max) { return gram_split_k(Wp, F_max) > 1; }

void pair_gram_popcount_dev(const uint64_t* bm, int64_t Wp, const int64_t* dF, int64_t F_max,
                            uint32_t* out, hipStream_t s) {
  if (F_max < 2) return;
  const int64_t nt = (F_max + kGT - 1) / kGT;
  const int64_t blocks = nt * (nt + 1) / 2;
  const int64_t ks = gram_split_k(Wp, F_max);
  if (Wp <= 48 && ks == 1)
    hipLaunchKernelGGL(k_pair_gram_popcount<48>, dim3((unsigned)blocks, 1), dim3(kBlock), 0, s,
                       (const unsigned long long*)bm, Wp, F_max, nt, out, F_max, dF);
  else
    hipLaunchKernelGGL(k_pair_gram_popcount<16>, dim3((unsigned)blocks, (unsigned)ks), dim3(kBlock), 0, s,
                       (const unsigned long long*)bm, Wp, F_max, nt, out, F_max, dF);
  KMLS_HIP(hipGetLastError());
}

void bitgemm_rect(const uint64_t* A, int64_t Fa, const uint64_t* B, int64_t Fb, int64_t Wp,
                  uint32_t* C, int64_t ldc, hipStream_t s) {
  if (Fa <= 0 || Fb <= 0 || Wp <= 0) return;
  const int64_t nta = (Fa + kGT - 1) / kGT, ntb = (Fb + kGT - 1) / kGT;
  const int64_t blocks = nta * ntb;
  const int64_t ks = std::max<int64_t>(1, std::min<int64_t>((1024 + blocks - 1) / blocks, Wp / 1024));
  hipLaunchKernelGGL(k_bitgemm_rect, dim3((unsigned)blocks, (unsigned)ks), dim3(kBlock), 0, s,
                     (const unsigned long long*)A, Fa, (const unsigned long long*)B, Fb, Wp, ntb, C,
                     ldc);
  KMLS_HIP(hipGetLastError());
}

void gram_to_cand(const uint32_t* gram, int64_t F, const int64_t* cand_off, int64_t c0, int64_t c1,
                  uint32_t* cnt, hipStream_t s) {
  if (c1 <= c0) return;
  hipLaunchKernelGGL(k_gram_to_cand, dim3(grid_for(c1 - c0, kBlock, 8192)), dim3(kBlock), 0, s,
                     gram, F, cand_off, c0, c1, cnt);
  KMLS_HIP(hipGetLastError());
}

}  // namespace kern
}  // namespace kmls
