// O10 pairs_to_csr: the reference's rule-map build (machine-learning/main.py:
// 282-304 -- for every itemset S and song a in S, rec[a][b] = max(rec[a][b], support(S))) is
// exactly the pair-support matrix (support is anti-monotone, so the max over all
// itemsets containing {a, b} is support({a, b})).  The level-2 gram already sits in HBM after the
// mining prologue, so the whole rule map is built there:
//
//   count  : 64x64 upper-triangle tiles of the gram; survivors (count >= minsup) are counted per
//            row AND per column in LDS, one global atomic per touched row per tile
//   scan   : per-item row lengths (item-id order, non-frequent items 0) → row_ptr (hipCUB)
//   fill   : the same tiles again; each tile reserves its slice of every touched row with one
//            atomic, then places entries with LDS atomics.  An entry is one 64-bit key
//            (count << 32 | ~tie(consequent)), so a descending sort gives the reference's row
//            order: score desc, then the deterministic tie key asc (consequent name order)
//   sort   : one block per row, bitonic sort of the row's keys in LDS (rows <= 2048 in a 16 KB
//            kernel, rows <= 16384 in a 128 KB one-block-per-CU kernel), writes cons/count
//   copyout: the finished CSR to pinned host memory, sized by the device nnz (no host round
//            trip, graph-capturable)
//
// F (the number of frequent items) may live on the device (resident path): every kernel reads
// it there and the grids are sized for F_max.
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

constexpr int kPT = 64;          // gram tile edge
constexpr int kSortSmall = 2048; // rows sorted by the 256-thread kernel
constexpr int kSortBig = kPairsSortMax;

__device__ __forceinline__ uint32_t tie_of(const int32_t* tie, int32_t id) {
  return tie ? (uint32_t)tie[id] : (uint32_t)id;
}

// Survivor pass over one upper tile: calls f(i, j, v) for i < j < F, v >= minsup.  Thread t
// owns row t/4 of the tile and 16 consecutive columns.
template <typename Fn>
__device__ __forceinline__ void tile_scan(const uint32_t* __restrict__ gram, int64_t ld, int64_t F,
                                          uint32_t minsup, int64_t i0, int64_t j0, Fn&& f) {
  const int r = threadIdx.x >> 2;
  const int c0 = (threadIdx.x & 3) * 16;
  const int64_t i = i0 + r;
  if (i >= F) return;
  const uint32_t* row = gram + i * ld;
#pragma unroll 4
  for (int k = 0; k < 16; ++k) {
    const int64_t j = j0 + c0 + k;
    if (j > i && j < F) {
      const uint32_t v = row[j];
      if (v >= minsup) f(r, c0 + k, v);
    }
  }
}

__global__ __launch_bounds__(256) void k_pairs_count(const uint32_t* __restrict__ gram, int64_t ld,
                                                     const int64_t* __restrict__ dF, int64_t F_host,
                                                     uint32_t minsup, uint32_t* __restrict__ len_r) {
  const int64_t F = dF ? *dF : F_host;
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  if (bi > bj) return;
  const int64_t i0 = bi * kPT, j0 = bj * kPT;
  if (i0 >= F || j0 >= F) return;
  __shared__ uint32_t s_r[kPT], s_c[kPT];
  if (threadIdx.x < kPT) s_r[threadIdx.x] = 0;
  else if (threadIdx.x < 2 * kPT) s_c[threadIdx.x - kPT] = 0;
  __syncthreads();
  uint32_t mine = 0;
  tile_scan(gram, ld, F, minsup, i0, j0, [&](int, int c, uint32_t) {
    ++mine;
    atomicAdd(&s_c[c], 1u);
  });
  if (mine) atomicAdd(&s_r[threadIdx.x >> 2], mine);
  __syncthreads();
  if (threadIdx.x < kPT) {
    if (s_r[threadIdx.x]) atomicAdd(&len_r[i0 + threadIdx.x], s_r[threadIdx.x]);
  } else if (threadIdx.x < 2 * kPT) {
    const int c = threadIdx.x - kPT;
    if (s_c[c]) atomicAdd(&len_r[j0 + c], s_c[c]);
  }
}

// per item id: its row length (frequent items) or 0; slot n_items is the scan's total slot.
// Rows longer than the small sort's capacity are listed for the big-row sort.
__device__ __forceinline__ int64_t len_of_item(const int32_t* __restrict__ rank_of, int64_t i,
                                               int64_t n_items, int64_t F,
                                               const uint32_t* __restrict__ len_r,
                                               unsigned int* __restrict__ n_long,
                                               int32_t* __restrict__ long_rows) {
  if (i >= n_items) return 0;
  const int32_t r = rank_of[i];
  if (r < 0 || r >= F) return 0;
  const uint32_t v = len_r[r];
  if (v > (uint32_t)kSortSmall) long_rows[atomicAdd(n_long, 1u)] = r;
  return v;
}

__global__ void k_pairs_len_by_id(const int32_t* __restrict__ rank_of, int64_t n_items,
                                  const int64_t* __restrict__ dF, int64_t F_host,
                                  const uint32_t* __restrict__ len_r, int64_t* __restrict__ len_id,
                                  unsigned int* __restrict__ n_long, int32_t* __restrict__ long_rows) {
  const int64_t F = dF ? *dF : F_host;
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n_items; i += nthr)
    len_id[i] = len_of_item(rank_of, i, n_items, F, len_r, n_long, long_rows);
}

// Small vocabularies (the resident path): lengths by item id + exclusive scan → row_ptr in ONE
// block (1024 threads, a contiguous run of items each), instead of a lengths pass and a
// multi-launch device scan.
constexpr int kScanThreads = 1024;
constexpr int64_t kScanSmallMax = 64 * kScanThreads;
__global__ __launch_bounds__(kScanThreads) void k_pairs_scan_small(
    const int32_t* __restrict__ rank_of, int64_t n_items, const int64_t* __restrict__ dF,
    int64_t F_host, const uint32_t* __restrict__ len_r, int64_t* __restrict__ row_ptr,
    unsigned int* __restrict__ n_long, int32_t* __restrict__ long_rows) {
  __shared__ int64_t s_w[kScanThreads / 64];
  const int64_t F = dF ? *dF : F_host;
  const int64_t n = n_items + 1;
  const int64_t per = (n + kScanThreads - 1) / kScanThreads;
  const int64_t i0 = (int64_t)threadIdx.x * per;
  int64_t sum = 0;
  for (int64_t k = 0; k < per; ++k) {
    const int64_t i = i0 + k;
    if (i < n) sum += len_of_item(rank_of, i, n_items, F, len_r, n_long, long_rows);
  }
  // block exclusive scan of the per-thread sums: wave64 inclusive scan, then wave totals
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t inc = sum;
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int k = 0; k < kScanThreads / 64; ++k) {
      const int64_t t = s_w[k];
      s_w[k] = run;
      run += t;
    }
  }
  __syncthreads();
  int64_t pre = s_w[w] + inc - sum;
  for (int64_t k = 0; k < per; ++k) {  // second pass re-reads the (cached) lengths
    const int64_t i = i0 + k;
    if (i >= n) break;
    row_ptr[i] = pre;
    if (i < n_items) {
      const int32_t r = rank_of[i];
      if (r >= 0 && r < F) pre += len_r[r];
    }
  }
}

__global__ __launch_bounds__(256) void k_pairs_fill(const uint32_t* __restrict__ gram, int64_t ld,
                                                    const int64_t* __restrict__ dF, int64_t F_host,
                                                    uint32_t minsup, const int32_t* __restrict__ ids,
                                                    const int32_t* __restrict__ tie,
                                                    const int64_t* __restrict__ row_ptr,
                                                    uint32_t* __restrict__ cursor,
                                                    unsigned long long* __restrict__ ent,
                                                    int64_t ent_cap, unsigned int* __restrict__ status) {
  const int64_t F = dF ? *dF : F_host;
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  if (bi > bj) return;
  const int64_t i0 = bi * kPT, j0 = bj * kPT;
  if (i0 >= F || j0 >= F) return;
  __shared__ uint32_t s_r[kPT], s_c[kPT];
  __shared__ int64_t s_rb[kPT], s_cb[kPT];
  __shared__ uint32_t s_tie_i[kPT], s_tie_j[kPT];
  if (threadIdx.x < kPT) {
    s_r[threadIdx.x] = 0;
    const int64_t i = i0 + threadIdx.x;
    s_tie_i[threadIdx.x] = i < F ? ~tie_of(tie, ids[i]) : 0u;
  } else if (threadIdx.x < 2 * kPT) {
    const int c = threadIdx.x - kPT;
    s_c[c] = 0;
    const int64_t j = j0 + c;
    s_tie_j[c] = j < F ? ~tie_of(tie, ids[j]) : 0u;
  }
  __syncthreads();
  uint32_t mine = 0;
  tile_scan(gram, ld, F, minsup, i0, j0, [&](int, int c, uint32_t) {
    ++mine;
    atomicAdd(&s_c[c], 1u);
  });
  if (mine) atomicAdd(&s_r[threadIdx.x >> 2], mine);
  __syncthreads();
  // reserve this tile's slice of every touched row (row i: its consequents j; row j: its i)
  if (threadIdx.x < kPT) {
    const uint32_t n = s_r[threadIdx.x];
    const int64_t i = i0 + threadIdx.x;
    s_rb[threadIdx.x] = n ? row_ptr[ids[i]] + atomicAdd(&cursor[i], n) : 0;
    s_r[threadIdx.x] = 0;
  } else if (threadIdx.x < 2 * kPT) {
    const int c = threadIdx.x - kPT;
    const uint32_t n = s_c[c];
    const int64_t j = j0 + c;
    s_cb[c] = n ? row_ptr[ids[j]] + atomicAdd(&cursor[j], n) : 0;
    s_c[c] = 0;
  }
  __syncthreads();
  bool over = false;
  tile_scan(gram, ld, F, minsup, i0, j0, [&](int r, int c, uint32_t v) {
    const int64_t p = s_rb[r] + atomicAdd(&s_r[r], 1u);
    const int64_t q = s_cb[c] + atomicAdd(&s_c[c], 1u);
    if (p < ent_cap && q < ent_cap) {
      ent[p] = ((unsigned long long)v << 32) | s_tie_j[c];
      ent[q] = ((unsigned long long)v << 32) | s_tie_i[r];
    } else {
      over = true;
    }
  });
  if (over) atomicOr(status, 1u);
}

// bitonic sort (descending) of P = pow2 keys in LDS by the whole block
__device__ __forceinline__ void block_bitonic_desc(unsigned long long* s, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < P; t += blockDim.x) {
        const int o = t ^ j;
        if (o > t) {
          const unsigned long long a = s[t], b = s[o];
          const bool desc = (t & k) == 0;
          if (desc ? (a < b) : (a > b)) {
            s[t] = b;
            s[o] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}

template <int CAP>
__device__ __forceinline__ void sort_row(unsigned long long* s, int64_t r, int64_t F,
                                         const uint32_t* __restrict__ len_r,
                                         const int32_t* __restrict__ ids,
                                         const int32_t* __restrict__ inv_tie,
                                         const int64_t* __restrict__ row_ptr,
                                         const unsigned long long* __restrict__ ent, int64_t ent_cap,
                                         int32_t* __restrict__ cons, uint32_t* __restrict__ cnt,
                                         int lo_exclusive) {
  if (r >= F) return;
  const int64_t n = len_r[r];
  if (n <= lo_exclusive || n > CAP) return;
  const int64_t base = ids ? row_ptr[ids[r]] : row_ptr[r];  // (row blocks: local row index)
  if (base + n > ent_cap) return;  // fill overflowed (status set): host redoes the call
  int P = 1;
  while (P < n) P <<= 1;
  for (int t = threadIdx.x; t < P; t += blockDim.x) s[t] = t < n ? ent[base + t] : 0ull;
  __syncthreads();
  if (n > 1) block_bitonic_desc(s, P);
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const unsigned long long k = s[t];
    const uint32_t tie = ~(uint32_t)(k & 0xFFFFFFFFull);
    cons[base + t] = inv_tie ? inv_tie[tie] : (int32_t)tie;
    cnt[base + t] = (uint32_t)(k >> 32);
  }
}

__global__ __launch_bounds__(256) void k_pairs_sort_small(
    const int64_t* __restrict__ dF, int64_t F_host, const uint32_t* __restrict__ len_r,
    const int32_t* __restrict__ ids, const int32_t* __restrict__ inv_tie,
    const int64_t* __restrict__ row_ptr, const unsigned long long* __restrict__ ent, int64_t ent_cap,
    int32_t* __restrict__ cons, uint32_t* __restrict__ cnt) {
  __shared__ unsigned long long s[kSortSmall];
  const int64_t F = dF ? *dF : F_host;
  sort_row<kSortSmall>(s, blockIdx.x, F, len_r, ids, inv_tie, row_ptr, ent, ent_cap, cons, cnt, 0);
}

__global__ __launch_bounds__(1024) void k_pairs_sort_big(
    const int64_t* __restrict__ dF, int64_t F_host, const uint32_t* __restrict__ len_r,
    const int32_t* __restrict__ ids, const int32_t* __restrict__ inv_tie,
    const int64_t* __restrict__ row_ptr, const unsigned long long* __restrict__ ent, int64_t ent_cap,
    int32_t* __restrict__ cons, uint32_t* __restrict__ cnt, unsigned int* __restrict__ status,
    const unsigned int* __restrict__ n_long, const int32_t* __restrict__ long_rows) {
  extern __shared__ unsigned long long s_dyn[];
  const int64_t F = dF ? *dF : F_host;
  const unsigned int nl = *n_long;
  for (unsigned int i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t r = long_rows[i];
    if (threadIdx.x == 0 && len_r[r] > (uint32_t)kSortBig) atomicOr(status, 2u);
    sort_row<kSortBig>(s_dyn, r, F, len_r, ids, inv_tie, row_ptr, ent, ent_cap, cons, cnt,
                       kSortSmall);
    __syncthreads();
  }
}

__global__ void k_pairs_copyout(const int64_t* __restrict__ row_ptr, int64_t n_items,
                                const int32_t* __restrict__ cons, const uint32_t* __restrict__ cnt,
                                const unsigned int* __restrict__ status,
                                const PairsHost* __restrict__ hp) {
  const PairsHost h = *hp;
  if (!h.meta) return;
  const int64_t nnz = row_ptr[n_items];
  const bool fits = nnz <= h.cap && status[0] == 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    h.meta[0] = nnz;
    h.meta[1] = (int64_t)status[0] | (fits ? 0 : 4);
  }
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = t0; i <= n_items; i += nthr) h.row_ptr[i] = row_ptr[i];
  if (!fits) return;
  for (int64_t i = t0; i < nnz; i += nthr) {
    h.cons[i] = cons[i];
    h.cnt[i] = cnt[i];
  }
}

// ---- row blocks of the FULL symmetric gram (the multi-GPU rule map) ----
// After the reduce-scatter, rank g holds rows [r0, r0 + nrows) of the summed gram, every column
// (both triangles), so its rows of the rule map need no other rank's data.

// lower triangle from the upper: 64x64 tiles through LDS (coalesced reads and writes)
__global__ __launch_bounds__(256) void k_gram_mirror(uint32_t* __restrict__ gram, int64_t ld,
                                                     int64_t F) {
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  if (bi > bj) return;
  const int64_t i0 = bi * kPT, j0 = bj * kPT;
  __shared__ uint32_t t[kPT][kPT + 1];
  for (int e = threadIdx.x; e < kPT * kPT; e += blockDim.x) {
    const int r = e / kPT, c = e % kPT;
    const int64_t i = i0 + r, j = j0 + c;
    t[r][c] = (i < F && j < F && j > i) ? gram[i * ld + j] : 0u;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kPT * kPT; e += blockDim.x) {
    const int r = e / kPT, c = e % kPT;  // element (j0 + r, i0 + c) of the lower triangle
    const int64_t j = j0 + r, i = i0 + c;
    if (i < F && j < F && j > i) gram[j * ld + i] = t[c][r];
  }
}

// row lengths: one block per row, survivors j != own row
__global__ __launch_bounds__(256) void k_rows_count(const uint32_t* __restrict__ rows, int64_t ld,
                                                    int64_t nrows, int64_t F, int64_t r0,
                                                    uint32_t minsup, uint32_t* __restrict__ len_r,
                                                    unsigned int* __restrict__ n_long,
                                                    int32_t* __restrict__ long_rows) {
  const int64_t r = blockIdx.x;
  if (r >= nrows) return;
  const uint32_t* row = rows + r * ld;
  uint32_t n = 0;
  for (int64_t j = threadIdx.x; j < F; j += blockDim.x) n += (row[j] >= minsup && j != r0 + r);
  for (int off = 32; off; off >>= 1) n += __shfl_xor(n, off, 64);
  __shared__ uint32_t s_w[4];
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    len_r[r] = tot;
    if (tot > (uint32_t)kSortSmall) long_rows[atomicAdd(n_long, 1u)] = (int32_t)r;
  }
}

// entries of one row in column order (block-wide compaction), keyed for the descending sort
__global__ __launch_bounds__(256) void k_rows_fill(const uint32_t* __restrict__ rows, int64_t ld,
                                                   int64_t nrows, int64_t F, int64_t r0,
                                                   uint32_t minsup, const int32_t* __restrict__ ids,
                                                   const int32_t* __restrict__ tie,
                                                   const int64_t* __restrict__ row_ptr,
                                                   unsigned long long* __restrict__ ent) {
  const int64_t r = blockIdx.x;
  if (r >= nrows) return;
  const uint32_t* row = rows + r * ld;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ uint32_t s_w[4];
  int64_t base = row_ptr[r];
  for (int64_t c0 = 0; c0 < F; c0 += blockDim.x) {
    const int64_t j = c0 + threadIdx.x;
    const uint32_t v = j < F ? row[j] : 0u;
    const bool keep = j < F && v >= minsup && j != r0 + r;
    const unsigned long long m = __ballot(keep);
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = 0;
    for (int k = 0; k < w; ++k) pre += s_w[k];
    const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    if (keep) {
      const uint32_t pos = pre + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      ent[base + pos] = ((unsigned long long)v << 32) | ~tie_of(tie, ids[j]);
    }
    base += tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_rows_sort_small(
    int64_t nrows, const uint32_t* __restrict__ len_r, const int32_t* __restrict__ inv_tie,
    const int64_t* __restrict__ row_ptr, const unsigned long long* __restrict__ ent, int64_t ent_cap,
    int32_t* __restrict__ cons, uint32_t* __restrict__ cnt) {
  __shared__ unsigned long long s[kSortSmall];
  sort_row<kSortSmall>(s, blockIdx.x, nrows, len_r, nullptr, inv_tie, row_ptr, ent, ent_cap, cons,
                       cnt, 0);
}

__global__ __launch_bounds__(1024) void k_rows_sort_big(
    int64_t nrows, const uint32_t* __restrict__ len_r, const int32_t* __restrict__ inv_tie,
    const int64_t* __restrict__ row_ptr, const unsigned long long* __restrict__ ent, int64_t ent_cap,
    int32_t* __restrict__ cons, uint32_t* __restrict__ cnt, unsigned int* __restrict__ status,
    const unsigned int* __restrict__ n_long, const int32_t* __restrict__ long_rows) {
  extern __shared__ unsigned long long s_dyn[];
  const unsigned int nl = *n_long;
  for (unsigned int i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t r = long_rows[i];
    if (threadIdx.x == 0 && len_r[r] > (uint32_t)kSortBig) atomicOr(status, 2u);
    sort_row<kSortBig>(s_dyn, r, nrows, len_r, nullptr, inv_tie, row_ptr, ent, ent_cap, cons, cnt,
                       kSortSmall);
    __syncthreads();
  }
}

}  // namespace

void gram_mirror(uint32_t* gram, int64_t ld, int64_t F, hipStream_t s) {
  if (F <= 1) return;
  const unsigned nt = (unsigned)((F + kPT - 1) / kPT);
  hipLaunchKernelGGL(k_gram_mirror, dim3(nt, nt), dim3(256), 0, s, gram, ld, F);
  KMLS_HIP(hipGetLastError());
}

void rows_count(const uint32_t* rows, int64_t ld, int64_t nrows, int64_t F, int64_t r0,
                uint32_t minsup, uint32_t* len_r, unsigned int* n_long, int32_t* long_rows,
                hipStream_t s) {
  if (nrows <= 0) return;
  hipLaunchKernelGGL(k_rows_count, dim3((unsigned)nrows), dim3(256), 0, s, rows, ld, nrows, F, r0,
                     minsup, len_r, n_long, long_rows);
  KMLS_HIP(hipGetLastError());
}

void rows_fill_sort(const uint32_t* rows, int64_t ld, int64_t nrows, int64_t F, int64_t r0,
                    uint32_t minsup, const int32_t* ids, const int32_t* tie, const int32_t* inv_tie,
                    const uint32_t* len_r, const int64_t* row_ptr, unsigned long long* ent,
                    int64_t ent_cap, int32_t* cons, uint32_t* cnt, unsigned int* status,
                    const unsigned int* n_long, const int32_t* long_rows, bool any_long,
                    hipStream_t s) {
  if (nrows <= 0) return;
  hipLaunchKernelGGL(k_rows_fill, dim3((unsigned)nrows), dim3(256), 0, s, rows, ld, nrows, F, r0,
                     minsup, ids, tie, row_ptr, ent);
  KMLS_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_rows_sort_small, dim3((unsigned)nrows), dim3(256), 0, s, nrows, len_r,
                     inv_tie, row_ptr, ent, ent_cap, cons, cnt);
  KMLS_HIP(hipGetLastError());
  if (any_long) {
    hipLaunchKernelGGL(k_rows_sort_big, dim3(64), dim3(1024),
                       (size_t)kSortBig * sizeof(unsigned long long), s, nrows, len_r, inv_tie,
                       row_ptr, ent, ent_cap, cons, cnt, status, n_long, long_rows);
    KMLS_HIP(hipGetLastError());
  }
}

namespace {
size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
size_t cub_scan_bytes(int64_t n_items) {
  if (n_items + 1 <= kScanSmallMax) return 0;
  size_t b = 0;
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int64_t*)nullptr,
                                            (int64_t*)nullptr, (int)(n_items + 1)));
  return b;
}
}  // namespace

// scratch: [status | n_long | len_r | cursor] (zeroed by ONE memset) | long_rows | len_id | cub
size_t pairs_scratch_bytes(int64_t F_max, int64_t n_items) {
  return 256 + align256((size_t)F_max * 8) + align256((size_t)F_max * 4) +
         align256((size_t)(n_items + 1) * 8) + align256(cub_scan_bytes(n_items)) + 256;
}

void pairs_to_csr(const PairsArgs& a, hipStream_t s) {
  if (a.F_max <= 0) throw std::runtime_error("pairs_to_csr: F_max must be > 0");
  if (a.scratch_bytes < pairs_scratch_bytes(a.F_max, a.n_items))
    throw std::runtime_error("pairs_to_csr: scratch too small");
  char* p = (char*)a.scratch;
  unsigned int* status = (unsigned int*)p;
  unsigned int* n_long = status + 1;
  uint32_t* len_r = (uint32_t*)(p + 256);
  uint32_t* cursor = len_r + a.F_max;
  const size_t zero_bytes = 256 + (size_t)a.F_max * 8;
  p += 256 + align256((size_t)a.F_max * 8);
  int32_t* long_rows = (int32_t*)p;
  p += align256((size_t)a.F_max * 4);
  int64_t* len_id = (int64_t*)p;
  p += align256((size_t)(a.n_items + 1) * 8);
  void* cub_tmp = p;
  const unsigned nt = (unsigned)((a.F_max + kPT - 1) / kPT);
  KMLS_HIP(hipMemsetAsync(a.scratch, 0, zero_bytes, s));
  hipLaunchKernelGGL(k_pairs_count, dim3(nt, nt), dim3(256), 0, s, a.gram, a.ld, a.dF, a.F_host,
                     a.minsup, len_r);
  KMLS_HIP(hipGetLastError());
  if (a.n_items + 1 <= kScanSmallMax) {
    hipLaunchKernelGGL(k_pairs_scan_small, dim3(1), dim3(kScanThreads), 0, s, a.rank_of, a.n_items,
                       a.dF, a.F_host, len_r, a.row_ptr, n_long, long_rows);
    KMLS_HIP(hipGetLastError());
  } else {
    const unsigned nb = (unsigned)std::min<int64_t>((a.n_items + 256) / 256, 4096);
    hipLaunchKernelGGL(k_pairs_len_by_id, dim3(nb), dim3(256), 0, s, a.rank_of, a.n_items, a.dF,
                       a.F_host, len_r, len_id, n_long, long_rows);
    KMLS_HIP(hipGetLastError());
    size_t tb = cub_scan_bytes(a.n_items);
    KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(cub_tmp, tb, len_id, a.row_ptr,
                                              (int)(a.n_items + 1), s));
  }
  hipLaunchKernelGGL(k_pairs_fill, dim3(nt, nt), dim3(256), 0, s, a.gram, a.ld, a.dF, a.F_host,
                     a.minsup, a.ids, a.tie, a.row_ptr, cursor, a.ent, a.ent_cap, status);
  KMLS_HIP(hipGetLastError());
  const unsigned rows = (unsigned)a.F_max;
  hipLaunchKernelGGL(k_pairs_sort_small, dim3(rows), dim3(256), 0, s, a.dF, a.F_host, len_r,
                     a.ids, a.inv_tie, a.row_ptr, a.ent, a.ent_cap, a.cons, a.cnt);
  KMLS_HIP(hipGetLastError());
  if (a.F_max > kSortSmall + 1) {  // a row can only exceed 2048 entries if F > 2049
    hipLaunchKernelGGL(k_pairs_sort_big, dim3(64), dim3(1024),
                       (size_t)kSortBig * sizeof(unsigned long long), s, a.dF, a.F_host, len_r,
                       a.ids, a.inv_tie, a.row_ptr, a.ent, a.ent_cap, a.cons, a.cnt, status,
                       n_long, long_rows);
    KMLS_HIP(hipGetLastError());
  }
  if (a.host) {
    hipLaunchKernelGGL(k_pairs_copyout, dim3(64), dim3(256), 0, s, a.row_ptr, a.n_items, a.cons,
                       a.cnt, status, a.host);
    KMLS_HIP(hipGetLastError());
  }
}

void pairs_enable_big_lds() {
  for (const void* f : {(const void*)k_pairs_sort_big, (const void*)k_rows_sort_big})
    KMLS_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)(kSortBig * sizeof(unsigned long long))));
}

}  // namespace kern
}  // namespace kmls
