// Level-2 pair counts of sparse transaction data, row by row in LDS (the Gustavson form of the
// co-occurrence product A^T A).  Replaces the scattered-atomic horizontal count (cooc.hip) on
// long shards: there every co-occurring pair was one no-return atomic into an F x F gram in HBM
// (870 MB at 14.8k frequent items), ~25 G atomics/s and ~32 B of HBM write per atomic
// (profiles/r4z_pmc_cooc_c3_write.md); the row form makes every increment an LDS atomic.
//
//   1. frequent-rank CSR: each transaction's frequent items as ranks, ascending, 16-bit
//      (devbuf::k_map_filter; rows with < 2 of them dropped — they hold no pair);
//   2. its transpose (CSC: for each rank a, the rows containing a): per-workgroup LDS histograms
//      of a contiguous row block, written rank-major, one exclusive scan = every (rank,
//      workgroup) output base; the fill pass scatters with LDS cursors (no global atomics,
//      deterministic);
//   3. row a = one or more 1024-thread workgroups (slices of kSlice rows of its column), each
//      with an F-counter LDS accumulator: for every transaction containing a, +1 at each later
//      (higher-ranked) item; a one-slice row stores its counters straight into gram row a
//      (coalesced, no zero fill needed), slices of a split row add their non-zero counters.
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

namespace kmls {
namespace kern {

namespace {

using devbuf::Buf;

constexpr int kRowThreads = 1024;
constexpr uint32_t kSlice = 8192;   // column entries per row workgroup
constexpr int64_t kBlockTx = 4096;  // CSR rows per histogram / fill workgroup

void ok(hipError_t e, const char* what) { devbuf::hip_ok(e, what); }

// rows [t0, t1) of the workgroup's block; their items are fit[e0, e1) (row order = item order)
__device__ __forceinline__ void block_rows(const uint2* __restrict__ txrec, int64_t n_tx,
                                           int64_t& t0, int64_t& t1) {
  t0 = (int64_t)blockIdx.x * kBlockTx;
  t1 = t0 + kBlockTx < n_tx ? t0 + kBlockTx : n_tx;
}

__global__ __launch_bounds__(kRowThreads) void k_pr_hist(const uint2* __restrict__ txrec,
                                                         int64_t n_tx,
                                                         const uint16_t* __restrict__ fit, int64_t F,
                                                         int64_t n_wg, uint32_t* __restrict__ hist) {
  extern __shared__ uint32_t h[];
  for (int64_t i = threadIdx.x; i < F; i += kRowThreads) h[i] = 0u;
  __syncthreads();
  int64_t t0, t1;
  block_rows(txrec, n_tx, t0, t1);
  if (t0 < t1) {
    const uint2 last = txrec[t1 - 1];
    const uint32_t e0 = txrec[t0].x, e1 = last.x + last.y;
    for (uint32_t p = e0 + threadIdx.x; p < e1; p += kRowThreads) atomicAdd(&h[fit[p]], 1u);
  }
  __syncthreads();
  for (int64_t r = threadIdx.x; r < F; r += kRowThreads) hist[r * n_wg + blockIdx.x] = h[r];
}

// the CSC: csc[base(r, wg) ...] = the rows of this block containing rank r
__global__ __launch_bounds__(kRowThreads) void k_pr_fill(const uint2* __restrict__ txrec,
                                                         int64_t n_tx,
                                                         const uint16_t* __restrict__ fit, int64_t F,
                                                         int64_t n_wg, const uint32_t* __restrict__ off,
                                                         uint32_t* __restrict__ csc) {
  extern __shared__ uint32_t cur[];
  for (int64_t r = threadIdx.x; r < F; r += kRowThreads) cur[r] = off[r * n_wg + blockIdx.x];
  __syncthreads();
  int64_t t0, t1;
  block_rows(txrec, n_tx, t0, t1);
  for (int64_t t = t0 + threadIdx.x; t < t1; t += kRowThreads) {
    const uint2 rec = txrec[t];
    for (uint32_t j = 0; j < rec.y; ++j) {
      const uint32_t slot = atomicAdd(&cur[fit[rec.x + j]], 1u);
      csc[slot] = (uint32_t)t;
    }
  }
}

// slices per rank (0 for a rank that occurs in no kept row); cnt[F] = 0 for the scan's total
__global__ void k_pr_slices(const uint32_t* __restrict__ off, int64_t F, int64_t n_wg,
                            uint32_t* __restrict__ col, uint32_t* __restrict__ nsl) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < F) {
    const uint32_t a = off[r * n_wg], b = off[(r + 1) * n_wg];
    col[r] = a;
    nsl[r] = (b - a + kSlice - 1) / kSlice;
  } else if (r == F) {
    col[F] = off[F * n_wg];
    nsl[F] = 0u;
  }
}

__global__ __launch_bounds__(kRowThreads) void k_pr_rows(
    const uint32_t* __restrict__ slice_off, int64_t F, const uint32_t* __restrict__ col,
    const uint32_t* __restrict__ csc, const uint2* __restrict__ txrec,
    const uint16_t* __restrict__ fit, uint32_t* __restrict__ gram, int64_t ld) {
  extern __shared__ uint32_t acc[];
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
  for (int64_t i = threadIdx.x; i < F; i += kRowThreads) acc[i] = 0u;
  __syncthreads();
  const uint32_t r = (uint32_t)s_r;
  const uint32_t k = blockIdx.x - slice_off[r];
  const uint32_t nsl = slice_off[r + 1] - slice_off[r];
  const uint32_t b0 = col[r] + k * kSlice;
  const uint32_t b1 = min(b0 + kSlice, col[r + 1]);
  for (uint32_t i = b0 + threadIdx.x; i < b1; i += kRowThreads) {
    const uint2 rec = txrec[csc[i]];
    const uint16_t* it = fit + rec.x;
    for (int j = (int)rec.y - 1; j >= 0; --j) {
      const uint32_t y = it[j];
      if (y <= r) break;
      atomicAdd(&acc[y], 1u);
    }
  }
  __syncthreads();
  uint32_t* row = gram + (int64_t)r * ld;
  if (nsl == 1) {
    for (int64_t y = r + 1 + threadIdx.x; y < F; y += kRowThreads) row[y] = acc[y];
  } else {
    for (int64_t y = r + 1 + threadIdx.x; y < F; y += kRowThreads)
      if (acc[y]) atomicAdd(&row[y], acc[y]);
  }
}

}  // namespace

struct PairRows::Impl {
  Buf<int16_t> pr;
  Buf<uint2> txrec;
  Buf<uint16_t> fit;
  Buf<uint32_t> hist, hoff, col, nsl, soff, csc;
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
const uint2* PairRows::txrec() const { return p_->txrec.p; }
const uint16_t* PairRows::fit() const { return p_->fit.p; }
int64_t PairRows::n_rows() const { return p_->n_tx; }
int64_t PairRows::nnz() const { return p_->nnz; }

size_t PairRows::lds_bytes(int64_t F) { return (size_t)std::max<int64_t>(F, 1) * 4; }

bool PairRows::count(const PrInput& in, uint32_t* gram, int64_t ld, hipStream_t s,
                     const std::function<void()>& wait) {
  Impl& I = *p_;
  const int64_t F = in.F;
  KMLS_CHECK(F >= 0 && F <= 32768 && ld >= F, "pair rows: F <= 32768 ranks, ld >= F");
  I.n_tx = I.nnz = 0;
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
  for (int attempt = 0;; ++attempt) {
    I.txrec.need(tx_cap);
    I.fit.need(nnz_cap);
    tx_cap = I.txrec.cap;
    nnz_cap = I.fit.cap;
    ok(hipMemsetAsync(I.ctr.p, 0, sizeof(unsigned long long), s), "ctr");
    ok(hipMemsetAsync(I.err.p, 0, sizeof(unsigned), s), "err");
    hipLaunchKernelGGL(devbuf::k_map_filter, dim3(g), dim3(256), 0, s, in.tx_ptr, in.items, in.n_tx,
                       I.pr.p, 2u, I.txrec.p, I.fit.p, I.ctr.p, tx_cap, nnz_cap, I.err.p);
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
    KMLS_CHECK(attempt == 0, "pair rows: CSR sizes grew between passes");
    tx_cap = nt;
    nnz_cap = nn;
  }
  KMLS_CHECK(I.nnz < (1ll << 32), "pair rows: the rank CSR passed 2^32 entries");
  if (I.n_tx == 0) return true;
  // 2. CSC by per-block histograms, rank-major scan, LDS-cursor fill
  const int64_t n_wg = (I.n_tx + kBlockTx - 1) / kBlockTx;
  const int64_t H = F * n_wg;
  KMLS_CHECK(H + 1 < (1ll << 31), "pair rows: histogram too large");
  I.hist.need((size_t)H + 1);
  I.hoff.need((size_t)H + 1);
  ok(hipMemsetAsync(I.hist.p + H, 0, 4, s), "hist tail");
  const size_t lds = lds_bytes(F);
  if (lds > 65536) {  // past the default dynamic-LDS limit (F > 16384): up to 160 KB per block
    ok(hipFuncSetAttribute((const void*)k_pr_hist, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "attr");
    ok(hipFuncSetAttribute((const void*)k_pr_fill, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "attr");
    ok(hipFuncSetAttribute((const void*)k_pr_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), "attr");
  }
  hipLaunchKernelGGL(k_pr_hist, dim3((unsigned)n_wg), dim3(kRowThreads), lds, s, I.txrec.p, I.n_tx,
                     I.fit.p, F, n_wg, I.hist.p);
  ok(hipGetLastError(), "hist");
  devbuf::scan_u32(I.hist.p, I.hoff.p, H + 1, I.tmp, s);
  I.csc.need((size_t)I.nnz);
  hipLaunchKernelGGL(k_pr_fill, dim3((unsigned)n_wg), dim3(kRowThreads), lds, s, I.txrec.p, I.n_tx,
                     I.fit.p, F, n_wg, I.hoff.p, I.csc.p);
  ok(hipGetLastError(), "fill");
  // 3. row slices, then the rows
  I.col.need((size_t)F + 1);
  I.nsl.need((size_t)F + 1);
  I.soff.need((size_t)F + 1);
  hipLaunchKernelGGL(k_pr_slices, dim3((unsigned)((F + 1 + 255) / 256)), dim3(256), 0, s, I.hoff.p,
                     F, n_wg, I.col.p, I.nsl.p);
  ok(hipGetLastError(), "slices");
  devbuf::scan_u32(I.nsl.p, I.soff.p, F + 1, I.tmp, s);
  ok(hipMemcpyAsync(I.h, I.soff.p + F, 4, hipMemcpyDeviceToHost, s), "rb");
  wait();
  const uint32_t n_sl = (uint32_t)(I.h[0] & 0xFFFFFFFFull);
  if (n_sl > 0)
    hipLaunchKernelGGL(k_pr_rows, dim3(n_sl), dim3(kRowThreads), lds, s, I.soff.p, F, I.col.p,
                       I.csc.p, I.txrec.p, I.fit.p, gram, ld);
  ok(hipGetLastError(), "rows");
  return true;
}

}  // namespace kern
}  // namespace kmls
