// Level-2 pair counts of sparse transaction data, row by row in LDS (the Gustavson form of the
// co-occurrence product A^T A).  Replaces the scattered-atomic horizontal count (cooc.hip) on
// long shards: there every co-occurring pair was one no-return atomic into an F x F gram in HBM
// (870 MB at 14.8k frequent items), ~25 G atomics/s and ~32 B of HBM write per atomic
// (profiles/r4z_pmc_cooc_c3_write.md); the row form makes every increment an LDS atomic.
//
//   1. frequent-rank CSR: each transaction's frequent items as ranks, ascending, 16-bit
//      (devbuf::k_map_filter; rows with < 2 of them dropped — they hold no pair);
//   2. the PAIR LISTS: row a's list holds, for every transaction containing a, the items after
//      a — i.e. every co-occurring pair (a, b > a) once, 16 bits each.  Per-workgroup LDS
//      histograms of a contiguous block of transactions (pairs each rank heads), written
//      rank-major; one exclusive scan gives every (rank, block) segment; the fill pass appends
//      each transaction's runs at LDS cursors (no global atomics, deterministic layout);
//   3. row a = one or more 1024-thread workgroups (slices of kSlice list entries), each streaming
//      its slice with coalesced loads into an F-counter LDS accumulator; a one-slice row stores
//      its counters straight into gram row a, slices of a split row add their non-zero counters
//      (the gram is zeroed first).  (A first version walked a transposed CSR instead, re-reading
//      every transaction's record and items at random for each of its items: 40 ms of the 100 ms
//      config-5 step, HBM-latency bound.)
// The CSR built in step 1 is kept for the horizontal levels (hlevels.hip re-filters it to the
// pair items instead of re-reading the 32-bit item CSR).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "devbuf.hpp"
#include "kernels.hpp"
#include "kmls/common.hpp"
#include "kmls/hooks.hpp"

namespace kmls {
namespace kern {

namespace {

using devbuf::Buf;

constexpr int kRowThreads = 1024;
constexpr uint64_t kSlice = 65536;  // pair-list entries per row workgroup
constexpr int64_t kBlockTx = 32768;  // CSR rows per histogram workgroup
constexpr int64_t kPartTx = 1024;    // CSR rows per partition workgroup (one per thread)
constexpr int kNGMax = 256;          // coarse row groups of the first partition pass (max; 64 default)
constexpr uint32_t kChunkDflt = 65536;  // group-list entries per split workgroup (default)

void ok(hipError_t e, const char* what) { devbuf::hip_ok(e, what); }

__device__ __forceinline__ void block_rows(int64_t n_tx, int64_t& t0, int64_t& t1) {
  t0 = (int64_t)blockIdx.x * kBlockTx;
  t1 = t0 + kBlockTx < n_tx ? t0 + kBlockTx : n_tx;
}

// pairs each rank heads (the later items of its rows) in this block of rows, rank-major
__global__ __launch_bounds__(kRowThreads) void k_pl_hist(const uint2* __restrict__ txrec,
                                                         int64_t n_tx,
                                                         const uint16_t* __restrict__ fit, int64_t F,
                                                         int64_t n_wg,
                                                         unsigned long long* __restrict__ hist,
                                                         int own_rank, int own_world,
                                                         uint32_t r_lo, uint32_t r_hi) {
  // ranks [r_lo, r_hi) only: the LDS counters of a window (past ~40k ranks a full table no
  // longer fits the 160 KB of LDS; the caller launches one window after another)
  KMLS_DYN_LDS(uint32_t, h);
  for (uint32_t i = threadIdx.x; i < r_hi - r_lo; i += kRowThreads) h[i] = 0u;
  __syncthreads();
  int64_t t0, t1;
  block_rows(n_tx, t0, t1);
  for (int64_t t = t0 + threadIdx.x; t < t1; t += kRowThreads) {
    const uint2 rec = txrec[t];
    const uint16_t* it = fit + rec.x;
    for (uint32_t i = 0; i + 1 < rec.y; ++i) {
      const uint32_t a = it[i];
      if (a >= r_lo && a < r_hi && (int)(a % (uint32_t)own_world) == own_rank)
        atomicAdd(&h[a - r_lo], rec.y - 1u - i);
    }
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < r_hi - r_lo; r += kRowThreads)
    hist[(int64_t)(r_lo + r) * n_wg + blockIdx.x] = h[r];
  (void)F;
}

// Group table and split chunks from the scanned row bases (one block): row r's group =
// floor(base[r] * kNG / total) (groups of ~equal pair mass, rows contiguous); gcur[g] = the
// first list position of group g; per group its row range and chunks of kChunk entries;
// meta[0] = total chunks.
__global__ __launch_bounds__(1024) void k_pl_groups(const unsigned long long* __restrict__ base,
                                                   int64_t F, uint8_t* __restrict__ grp,
                                                   unsigned long long* __restrict__ gcur,
                                                   uint32_t* __restrict__ grow,  // [ng][2]
                                                   uint32_t* __restrict__ gch,   // [ng + 1]
                                                   uint32_t* __restrict__ meta, int ng,
                                                   uint32_t chunk) {
  __shared__ uint32_t lo[kNGMax], hi[kNGMax];
  const unsigned long long total = base[F];
  if ((int)threadIdx.x < ng) {
    lo[threadIdx.x] = 0xFFFFFFFFu;
    hi[threadIdx.x] = 0u;
  }
  __syncthreads();
  for (int64_t r = threadIdx.x; r < F; r += blockDim.x) {
    const unsigned g = total ? (unsigned)(base[r] * (unsigned long long)ng / total) : 0u;
    const unsigned gg = g < (unsigned)ng ? g : (unsigned)ng - 1u;
    grp[r] = (uint8_t)gg;
    atomicMin(&lo[gg], (uint32_t)r);
    atomicMax(&hi[gg], (uint32_t)r + 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (int g = 0; g < ng; ++g) {
      gch[g] = c;
      if (lo[g] < hi[g]) {
        const unsigned long long b0 = base[lo[g]], b1 = base[hi[g]];
        gcur[g] = b0;
        grow[2 * g] = lo[g];
        grow[2 * g + 1] = hi[g];
        c += (uint32_t)((b1 - b0 + chunk - 1) / chunk);
      } else {
        gcur[g] = 0;
        grow[2 * g] = grow[2 * g + 1] = 0;
      }
    }
    gch[ng] = c;
    meta[0] = c;
  }
}

// Pass A: every pair (a, b) of a block of rows appended to a's GROUP list as (a << 16 | b):
// per-group LDS counts, one global reservation per (block, group), then LDS cursors.  A block's
// 64 segments stay in L2 while they fill (the per-row version wrote 7-byte runs to 14.8k places).
__global__ __launch_bounds__(kPartTx) void k_pl_part(const uint2* __restrict__ txrec, int64_t n_tx,
                                                     const uint16_t* __restrict__ fit, int64_t F,
                                                     const uint8_t* __restrict__ grp_g,
                                                     unsigned long long* __restrict__ gcur,
                                                     uint32_t* __restrict__ gl, int own_rank,
                                                     int own_world, int ng) {
  KMLS_DYN_LDS(uint8_t, grp);  // [F]
  __shared__ uint32_t cnt[kNGMax];
  __shared__ unsigned long long gb[kNGMax];
  for (int64_t r = threadIdx.x; r < F; r += kPartTx) grp[r] = grp_g[r];
  if ((int)threadIdx.x < ng) cnt[threadIdx.x] = 0u;
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * kPartTx + threadIdx.x;
  uint2 rec = make_uint2(0u, 0u);
  if (t < n_tx) rec = txrec[t];
  const uint16_t* it = fit + rec.x;
  for (uint32_t i = 0; i + 1 < rec.y; ++i)
    if ((int)(it[i] % (uint32_t)own_world) == own_rank) atomicAdd(&cnt[grp[it[i]]], rec.y - 1u - i);
  __syncthreads();
  if ((int)threadIdx.x < ng) {
    const uint32_t c = cnt[threadIdx.x];
    gb[threadIdx.x] = c ? atomicAdd(&gcur[threadIdx.x], (unsigned long long)c) : 0ull;
    cnt[threadIdx.x] = 0u;
  }
  __syncthreads();
  for (uint32_t i = 0; i + 1 < rec.y; ++i) {
    const uint32_t a = it[i], n = rec.y - 1u - i;
    if ((int)(a % (uint32_t)own_world) != own_rank) continue;
    const uint32_t g = grp[a];
    uint32_t* dst = gl + gb[g] + atomicAdd(&cnt[g], n);
    for (uint32_t j = 0; j < n; ++j) dst[j] = (a << 16) | (uint32_t)it[i + 1u + j];
  }
}

// Pass B: a chunk of one group's list split into its rows' lists (the b halves): per-row LDS
// counts over the group's row range, one global reservation per (chunk, row) through a relative
// row cursor, then LDS cursors.
__global__ __launch_bounds__(kRowThreads) void k_pl_split(
    const uint32_t* __restrict__ gl, const unsigned long long* __restrict__ gbeg_all,
    const unsigned long long* __restrict__ base, const uint32_t* __restrict__ grow,
    const uint32_t* __restrict__ gch, uint32_t* __restrict__ rcur, uint16_t* __restrict__ pl,
    int ng, uint32_t chunk) {
  KMLS_DYN_LDS(uint32_t, rc);  // [rows of the group]
  __shared__ int32_t s_g;
  if (threadIdx.x == 0) {
    int g = 0;
    while (g + 1 < ng && gch[g + 1] <= blockIdx.x) ++g;
    s_g = g;
  }
  __syncthreads();
  const int g = s_g;
  const uint32_t r0 = grow[2 * g], r1 = grow[2 * g + 1];
  const unsigned long long g0 = base[r0], g1 = base[r1];
  const unsigned long long c0 = g0 + (unsigned long long)(blockIdx.x - gch[g]) * chunk;
  const unsigned long long c1 = c0 + chunk < g1 ? c0 + chunk : g1;
  for (uint32_t r = threadIdx.x; r < r1 - r0; r += kRowThreads) rc[r] = 0u;
  __syncthreads();
  for (unsigned long long i = c0 + threadIdx.x; i < c1; i += kRowThreads)
    atomicAdd(&rc[(gl[i] >> 16) - r0], 1u);
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < r1 - r0; r += kRowThreads) {
    const uint32_t c = rc[r];
    rc[r] = c ? atomicAdd(&rcur[r0 + r], c) : 0u;  // relative position in the row's list
  }
  __syncthreads();
  for (unsigned long long i = c0 + threadIdx.x; i < c1; i += kRowThreads) {
    const uint32_t v = gl[i];
    const uint32_t a = v >> 16;
    pl[base[a] + atomicAdd(&rc[a - r0], 1u)] = (uint16_t)(v & 0xFFFFu);
  }
  (void)gbeg_all;
}

// ---- staged forms of passes A and B: the same lists, written as contiguous runs ----
// Pass A and pass B above write every entry to its own scattered address (a thread's pairs one
// by one; a chunk's entries to the cursors of ~230 rows), ~0.9-1.4 TB/s of partial-line writes
// at config 5.  The staged forms collect a tile's entries in LDS grouped by destination first,
// then copy each destination's run out with consecutive threads on consecutive addresses.
constexpr int kStA = 256;        // pass A: rows (= threads) per tile
constexpr int kStAEnt = 12288;   // pass A: staged pairs per tile (u32), 48 KB (~37 pairs a row
                                 // at config 5: two blocks per CU)
constexpr int kStBThreads = 1024;
constexpr int64_t kRankWindow = 32768;  // LDS counters of one hist / row window (128 KB)
constexpr int64_t kMaxDynLds = 160 * 1024;  // a workgroup's LDS on gfx950
constexpr int kStBEnt = 16384;   // pass B: entries per chunk (u32 staged), 64 KB
constexpr int kStBRows = 4096;   // pass B: group rows the staged form takes (else the direct form)

__global__ __launch_bounds__(kStA) void k_pl_part_staged(const uint2* __restrict__ txrec,
                                                          int64_t n_tx,
                                                          const uint16_t* __restrict__ fit,
                                                          int64_t F,
                                                          const uint8_t* __restrict__ grp_g,
                                                          unsigned long long* __restrict__ gcur,
                                                          uint32_t* __restrict__ gl, int own_rank,
                                                          int own_world, int ng) {
  KMLS_DYN_LDS(uint8_t, grp);  // [F]
  __shared__ uint32_t cnt[kNGMax], loff[kNGMax + 1], cur[kNGMax];
  __shared__ unsigned long long gb[kNGMax];
  __shared__ uint32_t stage[kStAEnt];
  for (int64_t r = threadIdx.x; r < F; r += kStA) grp[r] = grp_g[r];
  const int64_t ntiles = (n_tx + kStA - 1) / kStA;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    if ((int)threadIdx.x < ng) cnt[threadIdx.x] = 0u;
    __syncthreads();
    const int64_t t = tile * kStA + threadIdx.x;
    uint2 rec = make_uint2(0u, 0u);
    if (t < n_tx) rec = txrec[t];
    const uint16_t* it = fit + rec.x;
    for (uint32_t i = 0; i + 1 < rec.y; ++i)
      if ((int)(it[i] % (uint32_t)own_world) == own_rank)
        atomicAdd(&cnt[grp[it[i]]], rec.y - 1u - i);
    __syncthreads();
    if (threadIdx.x < 64) {  // one wave: the group reservations and the exclusive scan
      uint32_t run = 0;
      for (int g0 = 0; g0 < ng; g0 += 64) {
        const int g = g0 + (int)threadIdx.x;
        const uint32_t c = g < ng ? cnt[g] : 0u;
        if (g < ng) gb[g] = c ? atomicAdd(&gcur[g], (unsigned long long)c) : 0ull;
        uint32_t incl = c;
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t u = __shfl_up(incl, o, 64);
          if ((int)threadIdx.x >= o) incl += u;
        }
        if (g < ng) {
          loff[g] = run + incl - c;
          cur[g] = run + incl - c;
        }
        run += __shfl(incl, 63, 64);
      }
      if (threadIdx.x == 0) loff[ng] = run;
    }
    __syncthreads();
    const uint32_t total = loff[ng];
    const bool staged = total <= (uint32_t)kStAEnt;
    for (uint32_t i = 0; i + 1 < rec.y; ++i) {
      const uint32_t a = it[i], n = rec.y - 1u - i;
      if ((int)(a % (uint32_t)own_world) != own_rank) continue;
      const uint32_t g = grp[a];
      const uint32_t p = atomicAdd(&cur[g], n);
      if (staged) {
        for (uint32_t j = 0; j < n; ++j) stage[p + j] = (a << 16) | (uint32_t)it[i + 1u + j];
      } else {  // a tile of very long rows: the direct form for this tile
        uint32_t* dst = gl + gb[g] + (p - loff[g]);
        for (uint32_t j = 0; j < n; ++j) dst[j] = (a << 16) | (uint32_t)it[i + 1u + j];
      }
    }
    __syncthreads();
    if (staged)
      for (uint32_t k = threadIdx.x; k < total; k += kStA) {
        const uint32_t v = stage[k];
        const uint32_t g = grp[v >> 16];
        gl[gb[g] + (k - loff[g])] = v;
      }
    __syncthreads();
  }
}

// pass B staged: one chunk of kStBEnt entries of one group's list; the group's rows (<= kStBRows)
// get LDS counts, an exclusive scan, one global reservation each, and the chunk is staged in row
// order, then copied out row run by row run.  Dynamic LDS: 3 x rows u32.
__global__ __launch_bounds__(kStBThreads) void k_pl_split_staged(
    const uint32_t* __restrict__ gl, const unsigned long long* __restrict__ base,
    const uint32_t* __restrict__ grow, const uint32_t* __restrict__ gch,
    uint32_t* __restrict__ rcur, uint16_t* __restrict__ pl, int ng) {
  KMLS_DYN_LDS(uint32_t, rw);  // loff [rows + 1] | cur [rows] | gpos [rows]
  __shared__ uint32_t stage[kStBEnt];
  __shared__ uint32_t wsum[kStBThreads / 64];
  __shared__ int32_t s_g;
  if (threadIdx.x == 0) {
    int g = 0;
    while (g + 1 < ng && gch[g + 1] <= blockIdx.x) ++g;
    s_g = g;
  }
  __syncthreads();
  const int g = s_g;
  const uint32_t r0 = grow[2 * g], r1 = grow[2 * g + 1], nr = r1 - r0;
  uint32_t* loff = rw;
  uint32_t* cur = rw + nr + 1;
  uint32_t* gpos = rw + 2 * nr + 1;
  const unsigned long long g0 = base[r0], g1 = base[r1];
  const unsigned long long c0 = g0 + (unsigned long long)(blockIdx.x - gch[g]) * kStBEnt;
  const unsigned long long c1 = c0 + kStBEnt < g1 ? c0 + kStBEnt : g1;
  const uint32_t n = (uint32_t)(c1 - c0);
  for (uint32_t r = threadIdx.x; r < nr; r += kStBThreads) cur[r] = 0u;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += kStBThreads) atomicAdd(&cur[(gl[c0 + i] >> 16) - r0], 1u);
  __syncthreads();
  // exclusive scan of the row counts: thread t takes rows [t*per, (t+1)*per)
  const uint32_t per = (nr + kStBThreads - 1) / kStBThreads;
  const uint32_t lo = threadIdx.x * per, hi = lo + per < nr ? lo + per : nr;
  uint32_t sum = 0;
  for (uint32_t r = lo; r < hi; ++r) sum += cur[r];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t wb = 0;
  for (int q = 0; q < w; ++q) wb += wsum[q];
  uint32_t run = wb + incl - sum;
  for (uint32_t r = lo; r < hi; ++r) {
    const uint32_t c = cur[r];
    loff[r] = run;
    gpos[r] = c ? atomicAdd(&rcur[r0 + r], c) : 0u;  // the row's relative position
    cur[r] = run;
    run += c;
  }
  if (threadIdx.x == 0) loff[nr] = n;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += kStBThreads) {
    const uint32_t v = gl[c0 + i];
    stage[atomicAdd(&cur[(v >> 16) - r0], 1u)] = v;
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < n; k += kStBThreads) {
    const uint32_t v = stage[k];
    const uint32_t a = v >> 16, r = a - r0;
    pl[base[a] + gpos[r] + (k - loff[r])] = (uint16_t)(v & 0xFFFFu);
  }
}

// all-gathered CSRs (world blocks of cap_tx records / cap_nnz items) -> one CSR: rank q's rows
// at tbase[q], its items at nbase[q] (record offsets rebased)
__global__ void k_pr_gather_rows(const uint2* __restrict__ rec_all, int64_t cap_tx,
                                 const unsigned long long* __restrict__ sz, int world,
                                 uint2* __restrict__ out) {
  const int q = blockIdx.y;
  unsigned long long tb = 0, nb = 0;
  for (int i = 0; i < q; ++i) {
    tb += sz[2 * i];
    nb += sz[2 * i + 1];
  }
  const unsigned long long n = sz[2 * q];
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x) {
    const uint2 r = rec_all[(unsigned long long)q * cap_tx + i];
    out[tb + i] = make_uint2((uint32_t)(r.x + nb), r.y);
  }
}
__global__ void k_pr_gather_items(const uint16_t* __restrict__ fit_all, int64_t cap_nnz,
                                  const unsigned long long* __restrict__ sz, int world,
                                  uint16_t* __restrict__ out) {
  const int q = blockIdx.y;
  unsigned long long nb = 0;
  for (int i = 0; i < q; ++i) nb += sz[2 * i + 1];
  const unsigned long long n = sz[2 * q + 1];
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x)
    out[nb + i] = fit_all[(unsigned long long)q * cap_nnz + i];
}

// row bases / slices per rank (0 slices for a rank heading no pair); nsl[F] = 0 for the total
__global__ void k_pl_slices(const unsigned long long* __restrict__ off, int64_t F, int64_t n_wg,
                            unsigned long long* __restrict__ base, uint32_t* __restrict__ nsl) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < F) {
    const unsigned long long a = off[r * n_wg], b = off[(r + 1) * n_wg];
    base[r] = a;
    nsl[r] = (uint32_t)((b - a + kSlice - 1) / kSlice);
  } else if (r == F) {
    base[F] = off[F * n_wg];
    nsl[F] = 0u;
  }
}

__global__ __launch_bounds__(kRowThreads) void k_pl_rows(
    const uint32_t* __restrict__ slice_off, int64_t F, const unsigned long long* __restrict__ base,
    const uint16_t* __restrict__ pl, uint32_t* __restrict__ gram, int64_t ld, uint32_t c_lo,
    uint32_t c_hi) {
  // columns [c_lo, c_hi) of every row (one LDS window per launch when F x 4 bytes pass the LDS)
  KMLS_DYN_LDS(uint32_t, acc);
  __shared__ int32_t s_r;
  if (threadIdx.x == 0) {  // the rank whose slices hold this block: last r with slice_off[r] <= b
    const uint32_t b = blockIdx.x;
    int64_t lo = 0, hi = F;  // slice_off[0] = 0 <= b < slice_off[F]
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (slice_off[mid] <= b) lo = mid; else hi = mid;
    }
    s_r = (int32_t)lo;
  }
  __syncthreads();
  const uint32_t r = (uint32_t)s_r;
  const uint32_t y0 = r + 1 > c_lo ? r + 1 : c_lo;  // this row's columns in the window
  if (y0 >= c_hi) return;                             // (uniform: the whole block leaves)
  for (uint32_t i = threadIdx.x; i < c_hi - c_lo; i += kRowThreads) acc[i] = 0u;
  __syncthreads();
  const uint32_t k = blockIdx.x - slice_off[r];
  const uint32_t nsl = slice_off[r + 1] - slice_off[r];
  const unsigned long long b0 = base[r] + (unsigned long long)k * kSlice;
  const unsigned long long b1 = min(b0 + kSlice, base[r + 1]);
  if (c_lo == 0 && c_hi >= (uint32_t)F) {
    for (unsigned long long i = b0 + threadIdx.x; i < b1; i += kRowThreads) atomicAdd(&acc[pl[i]], 1u);
  } else {
    for (unsigned long long i = b0 + threadIdx.x; i < b1; i += kRowThreads) {
      const uint32_t b = pl[i];
      if (b >= c_lo && b < c_hi) atomicAdd(&acc[b - c_lo], 1u);
    }
  }
  __syncthreads();
  uint32_t* row = gram + (int64_t)r * ld;
  if (nsl == 1) {
    for (uint32_t y = y0 + threadIdx.x; y < c_hi; y += kRowThreads) row[y] = acc[y - c_lo];
  } else {
    for (uint32_t y = y0 + threadIdx.x; y < c_hi; y += kRowThreads)
      if (acc[y - c_lo]) atomicAdd(&row[y], acc[y - c_lo]);
  }
}

}  // namespace

struct PairRows::Impl {
  Buf<uint16_t> pr;
  Buf<uint2> txrec;
  Buf<uint16_t> fit;
  Buf<unsigned long long> hist, hoff, base;
  Buf<uint32_t> nsl, soff;
  Buf<uint16_t> pl;  // the pair lists, row after row
  Buf<uint32_t> gl;  // the group lists (a << 16 | b)
  Buf<uint8_t> grp;
  Buf<unsigned long long> gcur;
  Buf<uint32_t> grow, gch, meta, rcur;
  Buf<uint2> gtxrec, txrec_all;     // item-sharded: the all-gathered CSR (and the raw blocks)
  Buf<uint16_t> gfit, fit_all;
  Buf<unsigned long long> gsz;
  bool gathered = false;
  int64_t pairs = 0;
  Buf<unsigned long long> ctr;
  Buf<unsigned> err;
  Buf<uint8_t> tmp;
  unsigned long long* h = nullptr;  // pinned readbacks
  int64_t n_tx = 0, nnz = 0;
  Impl() { ok(hipHostMalloc((void**)&h, 4 * sizeof(unsigned long long), hipHostMallocDefault), "pin"); }
  ~Impl() {
    if (h) (void)hipHostFree(h);
  }
};

PairRows::PairRows() : p_(new Impl) {}
PairRows::~PairRows() { delete p_; }
const uint2* PairRows::txrec() const { return p_->gathered ? p_->gtxrec.p : p_->txrec.p; }
const uint16_t* PairRows::fit() const { return p_->gathered ? p_->gfit.p : p_->fit.p; }
int64_t PairRows::n_rows() const { return p_->n_tx; }
int64_t PairRows::nnz() const { return p_->nnz; }
int64_t PairRows::pairs() const { return p_->pairs; }

size_t PairRows::lds_bytes(int64_t F) {
  return (size_t)std::min<int64_t>(std::max<int64_t>(F, 1), kRankWindow) * 4;
}

bool PairRows::count(const PrInput& in, uint32_t* gram, int64_t ld, hipStream_t s,
                     const std::function<void()>& wait, const PrShard* shard) {
  Impl& I = *p_;
  const int64_t F = in.F;
  KMLS_CHECK(F >= 0 && F <= kSparseMaxF && ld >= F, "pair rows: F <= 65535 ranks, ld >= F");
  I.n_tx = I.nnz = I.pairs = 0;
  I.gathered = false;
  const int own_rank = shard ? shard->rank : 0, own_world = shard ? std::max(shard->world, 1) : 1;
  if (F > 0) ok(hipMemsetAsync(gram, 0, (size_t)F * ld * 4, s), "gram zero");
  if (F < 2 || in.n_tx <= 0) return true;
  // 1. frequent-rank CSR
  const int64_t NI = std::max<int64_t>(in.n_items, 1);
  I.pr.need((size_t)NI);
  ok(hipMemsetAsync(I.pr.p, 0xFF, (size_t)NI * 2, s), "pr");
  hipLaunchKernelGGL(devbuf::k_rank_map, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, s, in.ids,
                     F, (const uint8_t*)nullptr, I.pr.p);
  ok(hipGetLastError(), "rank map");
  I.ctr.need(2);
  I.err.need(1);
  unsigned long long tx_cap = std::max<unsigned long long>(I.txrec.cap, 1ull << 16);
  unsigned long long nnz_cap = std::max<unsigned long long>(I.fit.cap, 1ull << 20);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((in.n_tx + 255) / 256,
                                                                      (int64_t)in.n_cus * 32));
  // the LDS-mask filter when the frequent-item mask fits next to the wave buffers
  const int64_t mask_words = (in.n_items + 31) / 32;
  const bool lds_mask = in.fmask != nullptr && mask_words * 4 <= (128 << 10);
  // (test hook filter_lds=0: the L2-mask instance of the same kernel, at full occupancy)
  const bool mask_in_lds = lds_mask && test_hook("filter_lds", 1) != 0;
  // (the mask-in-LDS instance: one 16-wave workgroup per CU)
  auto* const k_lds = devbuf::k_map_filter_lds<true, devbuf::kMW16, devbuf::kMEnt16>;
  auto* const k_l2 = devbuf::k_map_filter_lds<false, devbuf::kMW, devbuf::kMEnt>;
  if (mask_in_lds && mask_words * 4 > 65536)
    ok(hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)(mask_words * 4)), "attr");
  const int64_t chunks = (in.n_tx + 63) / 64;
  const unsigned gm = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((chunks + devbuf::kMW - 1) / devbuf::kMW, (int64_t)in.n_cus * 2));
  const unsigned gm16 = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>((chunks + devbuf::kMW16 - 1) / devbuf::kMW16, (int64_t)in.n_cus));
  const int64_t waves = lds_mask ? (mask_in_lds ? (int64_t)gm16 * devbuf::kMW16
                                                : (int64_t)gm * 4 * devbuf::kMW)
                                 : (int64_t)g * 4;
  const devbuf::PoolRes pres = devbuf::pool_res(in.n_tx, in.kept_per_tx, waves);
  for (int attempt = 0;; ++attempt) {
    I.txrec.need(tx_cap);
    I.fit.need(nnz_cap);
    tx_cap = I.txrec.cap;
    nnz_cap = I.fit.cap;
    ok(hipMemsetAsync(I.ctr.p, 0, sizeof(unsigned long long), s), "ctr");
    ok(hipMemsetAsync(I.err.p, 0, sizeof(unsigned), s), "err");
    // (the pools' abandoned rows must read as empty)
    ok(hipMemsetAsync(I.txrec.p, 0, (size_t)tx_cap * sizeof(uint2), s), "txrec zero");
    if (lds_mask) {
      if (mask_in_lds)
        hipLaunchKernelGGL(k_lds, dim3(gm16), dim3(64 * devbuf::kMW16), (size_t)mask_words * 4,
                           s, in.tx_ptr, in.items, in.n_tx, in.fmask, mask_words, I.pr.p, 2u,
                           I.txrec.p, I.fit.p, I.ctr.p, tx_cap, nnz_cap, I.err.p, pres.rows,
                           pres.items);
      else
        hipLaunchKernelGGL(k_l2, dim3(gm * 4), dim3(64 * devbuf::kMW), 0, s, in.tx_ptr,
                           in.items, in.n_tx, in.fmask, mask_words, I.pr.p, 2u, I.txrec.p,
                           I.fit.p, I.ctr.p, tx_cap, nnz_cap, I.err.p, pres.rows, pres.items);
    } else {
      hipLaunchKernelGGL(devbuf::k_map_filter, dim3(g), dim3(256), 0, s, in.tx_ptr, in.items,
                         in.n_tx, I.pr.p, 2u, I.txrec.p, I.fit.p, I.ctr.p, tx_cap, nnz_cap, I.err.p,
                         pres.rows, pres.items);
    }
    ok(hipGetLastError(), "filter");
    ok(hipMemcpyAsync(I.h, I.ctr.p, 8, hipMemcpyDeviceToHost, s), "rb");
    ok(hipMemcpyAsync(I.h + 1, I.err.p, 4, hipMemcpyDeviceToHost, s), "rb");
    wait();
    const unsigned e = (unsigned)(I.h[1] & 0xFFFFFFFFull);
    KMLS_CHECK(!(e & 2u), "pair rows: a transaction holds the same frequent item twice (load_csr "
                          "requires duplicate-free rows)");
    if (e & 1u) return false;
    const unsigned long long nt = I.h[0] >> devbuf::kPackShift, nn = I.h[0] & devbuf::kPackMask;
    if (nt <= tx_cap && nn <= nnz_cap) {
      I.n_tx = (int64_t)nt;
      I.nnz = (int64_t)nn;
      break;
    }
    // (the pools' tails differ from run to run: leave room for every wave to abandon more)
    KMLS_CHECK(attempt < 3, "pair rows: CSR sizes grew between passes");
    tx_cap = nt + (unsigned long long)waves * pres.rows;
    nnz_cap = nn + (unsigned long long)waves * pres.items;
  }
  if (own_world > 1) {  // item-sharded: every rank's CSR on every rank
    I.gsz.need((size_t)2 * own_world + 2);
    unsigned long long mine[2] = {(unsigned long long)I.n_tx, (unsigned long long)I.nnz};
    ok(hipMemcpyAsync(I.gsz.p + 2 * own_world, mine, 16, hipMemcpyHostToDevice, s), "sz");
    shard->all_gather(I.gsz.p + 2 * own_world, I.gsz.p, 4);
    std::vector<unsigned long long> sz((size_t)2 * own_world);
    ok(hipMemcpyAsync(sz.data(), I.gsz.p, sz.size() * 8, hipMemcpyDeviceToHost, s), "sz");
    wait();
    unsigned long long cap_tx = 1, cap_nnz = 2, tot_tx = 0, tot_nnz = 0;
    for (int q = 0; q < own_world; ++q) {
      cap_tx = std::max(cap_tx, sz[2 * q]);
      cap_nnz = std::max(cap_nnz, sz[2 * q + 1]);
      tot_tx += sz[2 * q];
      tot_nnz += sz[2 * q + 1];
    }
    cap_nnz = (cap_nnz + 1) & ~1ull;  // whole u32 words
    KMLS_CHECK(tot_nnz < (1ull << 32) && tot_tx < (1ull << 32), "pair rows: gathered CSR too large");
    I.txrec.need_keep(cap_tx, (size_t)I.n_tx, s);  // send blocks are read up to the cap
    I.fit.need_keep(cap_nnz, (size_t)I.nnz, s);
    I.txrec_all.need(cap_tx * own_world);
    I.fit_all.need(cap_nnz * own_world);
    shard->all_gather(I.txrec.p, I.txrec_all.p, cap_tx * 2);
    shard->all_gather(I.fit.p, I.fit_all.p, cap_nnz / 2);
    I.gtxrec.need(std::max<unsigned long long>(tot_tx, 1));
    I.gfit.need(std::max<unsigned long long>(tot_nnz, 1));
    hipLaunchKernelGGL(k_pr_gather_rows, dim3(1024, own_world), dim3(256), 0, s, I.txrec_all.p,
                       (int64_t)cap_tx, I.gsz.p, own_world, I.gtxrec.p);
    hipLaunchKernelGGL(k_pr_gather_items, dim3(1024, own_world), dim3(256), 0, s, I.fit_all.p,
                       (int64_t)cap_nnz, I.gsz.p, own_world, I.gfit.p);
    ok(hipGetLastError(), "gather");
    I.gathered = true;
    I.n_tx = (int64_t)tot_tx;
    I.nnz = (int64_t)tot_nnz;
  }
  KMLS_CHECK(I.nnz < (1ll << 32), "pair rows: the rank CSR passed 2^32 entries");
  if (I.n_tx == 0) return true;
  const uint2* txrec = I.gathered ? I.gtxrec.p : I.txrec.p;
  const uint16_t* fit = I.gathered ? I.gfit.p : I.fit.p;
  // 2. pair lists by per-block histograms, a rank-major scan, LDS-cursor fill
  const int64_t n_wg = (I.n_tx + kBlockTx - 1) / kBlockTx;
  const int64_t H = F * n_wg;
  KMLS_CHECK(H + 1 < (1ll << 31), "pair rows: histogram too large");
  I.hist.need((size_t)H + 1);
  I.hoff.need((size_t)H + 1);
  ok(hipMemsetAsync(I.hist.p + H, 0, 8, s), "hist tail");
  // rank windows of kRankWindow LDS counters (one window up to F = 32768)
  const size_t lds = lds_bytes(F);
  if (lds > 65536) {  // past the default dynamic-LDS limit (F > 16384): up to 128 KB per block
    ok(hipFuncSetAttribute((const void*)k_pl_hist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "attr");
    ok(hipFuncSetAttribute((const void*)k_pl_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "attr");
  }
  for (int64_t lo = 0; lo < F; lo += kRankWindow)
    hipLaunchKernelGGL(k_pl_hist, dim3((unsigned)n_wg), dim3(kRowThreads), lds, s, txrec, I.n_tx,
                       fit, F, n_wg, I.hist.p, own_rank, own_world, (uint32_t)lo,
                       (uint32_t)std::min<int64_t>(F, lo + kRankWindow));
  ok(hipGetLastError(), "hist");
  devbuf::scan_u64(I.hist.p, I.hoff.p, H + 1, I.tmp, s);
  I.base.need((size_t)F + 1);
  I.nsl.need((size_t)F + 1);
  I.soff.need((size_t)F + 1);
  hipLaunchKernelGGL(k_pl_slices, dim3((unsigned)((F + 1 + 255) / 256)), dim3(256), 0, s, I.hoff.p,
                     F, n_wg, I.base.p, I.nsl.p);
  ok(hipGetLastError(), "slices");
  devbuf::scan_u32(I.nsl.p, I.soff.p, F + 1, I.tmp, s);
  I.grp.need((size_t)F);
  // (test hooks pl_groups / pl_chunk: the partition's group count and split chunk)
  const int ng = (int)std::max<long long>(1, std::min<long long>(kNGMax, test_hook("pl_groups", 64)));
  const uint32_t chunk = (uint32_t)std::max<long long>(1024, test_hook("pl_chunk", kChunkDflt));
  // (test hook pl_staged=0: the direct (unstaged) passes A and B)
  const bool staged = test_hook("pl_staged", 1) != 0;
  const uint32_t chunk_b = staged ? (uint32_t)kStBEnt : chunk;
  I.gcur.need(ng);
  I.grow.need(2 * ng);
  I.gch.need(ng + 1);
  I.meta.need(4);
  hipLaunchKernelGGL(k_pl_groups, dim3(1), dim3(1024), 0, s, I.base.p, F, I.grp.p, I.gcur.p,
                     I.grow.p, I.gch.p, I.meta.p, ng, chunk_b);
  ok(hipGetLastError(), "groups");
  std::vector<uint32_t> grow_h((size_t)2 * ng);
  ok(hipMemcpyAsync(I.h, I.base.p + F, 8, hipMemcpyDeviceToHost, s), "rb");
  ok(hipMemcpyAsync(I.h + 1, I.soff.p + F, 4, hipMemcpyDeviceToHost, s), "rb");
  ok(hipMemcpyAsync(I.h + 2, I.meta.p, 4, hipMemcpyDeviceToHost, s), "rb");
  ok(hipMemcpyAsync(grow_h.data(), I.grow.p, grow_h.size() * 4, hipMemcpyDeviceToHost, s), "rb");
  wait();
  I.pairs = (int64_t)I.h[0];
  const uint32_t n_sl = (uint32_t)(I.h[1] & 0xFFFFFFFFull);
  const uint32_t n_ch = (uint32_t)(I.h[2] & 0xFFFFFFFFull);
  if (I.pairs == 0) return true;
  uint32_t max_rows = 0;
  for (int q = 0; q < ng; ++q) max_rows = std::max(max_rows, grow_h[2 * q + 1] - grow_h[2 * q]);
  // pass A: group lists; pass B: row lists
  I.gl.need((size_t)I.pairs);
  I.pl.need((size_t)I.pairs);
  I.rcur.need((size_t)F);
  ok(hipMemsetAsync(I.rcur.p, 0, (size_t)F * 4, s), "rcur");
  if (staged && test_hook("pl_staged_a", 0) != 0) {  // (measured slower than the direct pass A
                                                      // at config 5: 14.8 vs 11.3 ms)
    const int64_t ntiles = (I.n_tx + kStA - 1) / kStA;
    const unsigned gA = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ntiles, (int64_t)in.n_cus * 2));
    hipLaunchKernelGGL(k_pl_part_staged, dim3(gA), dim3(kStA), (size_t)F, s, txrec, I.n_tx, fit,
                       F, I.grp.p, I.gcur.p, I.gl.p, own_rank, own_world, ng);
  } else {
    const int64_t n_pb = (I.n_tx + kPartTx - 1) / kPartTx;
    hipLaunchKernelGGL(k_pl_part, dim3((unsigned)n_pb), dim3(kPartTx), (size_t)F, s, txrec,
                       I.n_tx, fit, F, I.grp.p, I.gcur.p, I.gl.p, own_rank, own_world, ng);
  }
  ok(hipGetLastError(), "part");
  // the direct split keeps a counter per row of the group in LDS
  const size_t lds_split = (size_t)std::max<uint32_t>(max_rows, 1u) * 4;
  if (!(staged && max_rows <= (uint32_t)kStBRows) && n_ch > 0) {
    if (lds_split > (size_t)kMaxDynLds) return false;  // (a group of > 40k rows: the caller's
                                                       // scattered-atomic count takes it)
    if (lds_split > 65536)
      ok(hipFuncSetAttribute((const void*)k_pl_split, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds_split), "attr");
  }
  if (n_ch > 0) {
    if (staged && max_rows <= (uint32_t)kStBRows)
      hipLaunchKernelGGL(k_pl_split_staged, dim3(n_ch), dim3(kStBThreads),
                         (size_t)(3 * max_rows + 1) * 4, s, I.gl.p, I.base.p, I.grow.p, I.gch.p,
                         I.rcur.p, I.pl.p, ng);
    else if (staged)  // a group of more rows than the staged form holds: direct, same chunks
      hipLaunchKernelGGL(k_pl_split, dim3(n_ch), dim3(kRowThreads), lds_split, s, I.gl.p,
                         (const unsigned long long*)nullptr, I.base.p, I.grow.p, I.gch.p,
                         I.rcur.p, I.pl.p, ng, chunk_b);
    else
      hipLaunchKernelGGL(k_pl_split, dim3(n_ch), dim3(kRowThreads), lds_split, s, I.gl.p,
                         (const unsigned long long*)nullptr, I.base.p, I.grow.p, I.gch.p,
                         I.rcur.p, I.pl.p, ng, chunk);
  }
  ok(hipGetLastError(), "split");
  // 3. the rows
  if (n_sl > 0)
    for (int64_t lo = 0; lo < F; lo += kRankWindow)
      hipLaunchKernelGGL(k_pl_rows, dim3(n_sl), dim3(kRowThreads), lds, s, I.soff.p, F, I.base.p,
                         I.pl.p, gram, ld, (uint32_t)lo,
                         (uint32_t)std::min<int64_t>(F, lo + kRankWindow));
  ok(hipGetLastError(), "rows");
  return true;
}

}  // namespace kern
}  // namespace kmls
