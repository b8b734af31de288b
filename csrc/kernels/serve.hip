// serve_match_topk: batched antecedent matching over an HBM-resident CSR rule index.
//
// Exact semantics of recommend_tracks_for_track (rest_api/app/main.py:235-254):
//   merged[r] = max over present seeds' rows of score(r)          (max-merge)
//   order     = score desc, ties by first insertion position      (stable sort over dict order)
// The insertion position of r is the first position where r occurs in the concatenation of
// the present seeds' rows (request order, row order), so both reductions are commutative:
// (max score-rank, min position).
//
// One WAVE64 per query (4 queries per 256-thread block; a query merges a few rows of tens to
// hundreds of entries, so a whole workgroup per query left 3/4 of it idle at the reductions):
//   * seeds: 64 per pass, one per lane — is_key / row length loads in parallel, request-order
//     compaction of the present seeds by ballot + popcount, row offsets by a wave prefix scan;
//   * merge: entries strided over the lanes into a per-wave LDS open-address table
//     (1024 slots: key, score rank via atomicMax, first position via atomicMin);
//   * top-k: every lane keeps the best key of its 16 slots; k rounds of a wave max, the winning
//     lane retires its slot and rescans only its own 16 (no block barriers anywhere).
// Queries with > kMaxSeeds seeds report -2 and are answered on the host.  Queries whose merged
// set could overflow the wave's table (long rows: the HBM-scale indexes of config 5, rows of
// thousands of entries) are answered by k_serve_topk_big, a workgroup per query:
//   * threshold: rows are sorted by score, so with tau = the largest k-th score over the seeds'
//     rows, the top-k lies among the entries scoring >= tau — a short prefix of every row (a
//     consequent scoring < tau everywhere is beaten by the k distinct consequents of the row
//     that defines tau);
//   * those prefixes are max-merged in a 4096-slot LDS table;
//   * first positions are completed against the rows' suffixes (a candidate may first occur
//     at a low score in an EARLIER row): a binary search per (candidate, earlier row) in a
//     per-row by-consequent copy of the index (built once, hipcub segmented sort);
//   * block-wide top-k over the table.
// Queries are read from, and results written to, mapped pinned host memory: no staging copies.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/kmls/gpu.hpp"
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

constexpr int kWaves = 4;                 // queries per block
constexpr int kSlots = 1024;              // hash slots per wave
constexpr int kPerLane = kSlots / 64;     // slots each lane owns in the top-k scan
constexpr int kMaxSeeds = 256;

// ---- large merges: one 256-thread workgroup per query ----
constexpr int kBigThreads = 256;
constexpr int kBigSlots = 4096;
constexpr int kBigMaxCand = kBigSlots / 2;
constexpr int kBigPer = kBigSlots / kBigThreads;

__device__ __forceinline__ int64_t blk_scan_excl(int64_t v, int64_t* s_w, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  __syncthreads();  // s_w reuse across calls
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  int64_t wbase = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kBigThreads / 64; ++i) {
    if (i < w) wbase += s_w[i];
    tot += s_w[i];
  }
  *total = tot;
  return wbase + x - v;
}

__global__ __launch_bounds__(kBigThreads) void k_serve_topk_big(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ cons,
    const uint32_t* __restrict__ srank, const uint8_t* __restrict__ is_key, int64_t n_items,
    const int32_t* __restrict__ id_cons, const int32_t* __restrict__ id_pos,
    const int64_t* __restrict__ q_ptr, const int32_t* __restrict__ seeds,
    const int32_t* __restrict__ qlist, int k, int32_t* __restrict__ out) {
  __shared__ int32_t s_key[kBigSlots];
  __shared__ uint32_t s_val[kBigSlots];
  __shared__ uint32_t s_pos[kBigSlots];
  __shared__ int64_t s_row[kMaxSeeds];
  __shared__ int64_t s_seg[kMaxSeeds + 1];   // concatenation offsets (full rows)
  __shared__ int64_t s_cseg[kMaxSeeds + 1];  // candidate-prefix offsets
  __shared__ int32_t s_len[kMaxSeeds];
  __shared__ int32_t s_pl[kMaxSeeds];
  __shared__ int64_t s_w[kBigThreads / 64];
  __shared__ uint32_t s_tau;
  __shared__ unsigned long long s_best[kBigThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t b = qlist[blockIdx.x];
  const int64_t q0 = q_ptr[b], q1 = q_ptr[b + 1];
  int32_t* o = out + b * (int64_t)(k + 1);
  for (int i = tid; i < kBigSlots; i += kBigThreads) {
    s_key[i] = -1;
    s_val[i] = 0;
    s_pos[i] = 0xFFFFFFFFu;
  }
  if (tid == 0) s_tau = 0;
  // present seeds in request order (the host sends only queries with <= kMaxSeeds seeds)
  bool present = false;
  int64_t rs = 0, len = 0;
  if (tid < q1 - q0) {
    const int32_t sd = seeds[q0 + tid];
    if (sd >= 0 && sd < n_items && is_key[sd]) {
      present = true;
      rs = row_ptr[sd];
      len = row_ptr[sd + 1] - rs;
    }
  }
  int64_t np64;
  const int64_t rk = blk_scan_excl(present ? 1 : 0, s_w, &np64);
  const int np = (int)np64;
  int64_t acc;
  const int64_t seg = blk_scan_excl(len, s_w, &acc);
  if (present) {
    s_row[rk] = rs;
    s_len[rk] = (int32_t)len;
    s_seg[rk] = seg;
  }
  if (tid == 0) s_seg[np] = acc;
  __syncthreads();
  if (np == 0) {
    if (tid == 0) o[0] = -1;
    return;
  }
  // tau = max over rows of the k-th best score rank (0: no row has k entries → all candidates)
  if (tid < np && s_len[tid] >= k) atomicMax(&s_tau, srank[s_row[tid] + k - 1]);
  __syncthreads();
  const uint32_t tau = s_tau;
  int64_t pl = 0;
  if (tid < np) {
    const int64_t r0 = s_row[tid];
    int64_t lo = 0, hi = s_len[tid];  // first index with srank < tau (ranks are non-increasing)
    if (tau > 0) {
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (srank[r0 + mid] >= tau) lo = mid + 1; else hi = mid;
      }
      pl = lo;
    } else {
      pl = s_len[tid];
    }
    s_pl[tid] = (int32_t)pl;
  }
  int64_t M;
  const int64_t cs = blk_scan_excl(pl, s_w, &M);
  if (tid < np) s_cseg[tid] = cs;
  if (tid == 0) s_cseg[np] = M;
  __syncthreads();
  if (M > kBigMaxCand) {  // pathological ties at tau: host path
    if (tid == 0) o[0] = -2;
    return;
  }
  // max-merge of the candidate prefixes
  for (int64_t e = tid; e < M; e += kBigThreads) {
    int lo = 0, hi = np;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s_cseg[mid] <= e) lo = mid; else hi = mid;
    }
    const int64_t idx = e - s_cseg[lo];
    const int64_t p = s_row[lo] + idx;
    const int32_t c = cons[p];
    const uint32_t v = srank[p];
    uint32_t h = ((uint32_t)c * 2654435761u) & (kBigSlots - 1);
    while (true) {
      const int32_t prev = atomicCAS(&s_key[h], -1, c);
      if (prev == -1 || prev == c) break;
      h = (h + 1) & (kBigSlots - 1);
    }
    atomicMax(&s_val[h], v + 1);
    atomicMin(&s_pos[h], (uint32_t)(s_seg[lo] + idx));
  }
  __syncthreads();
  // first positions: an earlier row may hold the consequent past its prefix
  for (int i = tid; i < kBigSlots; i += kBigThreads) {
    const int32_t c = s_key[i];
    if (c < 0) continue;
    uint32_t p = s_pos[i];
    for (int j = 0; j < np && (uint32_t)s_seg[j] < p; ++j) {
      const int32_t n = s_len[j];
      if (n <= s_pl[j]) continue;
      const int64_t r0 = s_row[j];
      int lo = 0, hi = n;  // consequents of row j sorted by id
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (id_cons[r0 + mid] < c) lo = mid + 1; else hi = mid;
      }
      if (lo < n && id_cons[r0 + lo] == c) {
        const int32_t ix = id_pos[r0 + lo];
        if (ix >= s_pl[j]) p = min(p, (uint32_t)(s_seg[j] + ix));
      }
    }
    s_pos[i] = p;
  }
  __syncthreads();
  // top-k: thread-local best over its slots, k rounds of a block max
  auto best_of = [&](int& slot) {
    unsigned long long best = 0;
    slot = -1;
    for (int j = 0; j < kBigPer; ++j) {
      const int i = j * kBigThreads + tid;
      if (s_key[i] >= 0) {
        const unsigned long long kk =
            ((unsigned long long)s_val[i] << 32) | (unsigned long long)(0xFFFFFFFFu - s_pos[i]);
        if (kk > best) {
          best = kk;
          slot = i;
        }
      }
    }
    return best;
  };
  int my_slot;
  unsigned long long mine = best_of(my_slot);
  int n_out = 0;
  for (; n_out < k; ++n_out) {
    unsigned long long bb = mine;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long t = __shfl_xor(bb, off, 64);
      bb = t > bb ? t : bb;
    }
    if (lane == 0) s_best[w] = bb;
    __syncthreads();
    unsigned long long g = 0;
#pragma unroll
    for (int i = 0; i < kBigThreads / 64; ++i) g = s_best[i] > g ? s_best[i] : g;
    __syncthreads();  // s_best reused next round
    if (g == 0) break;
    if (mine == g) {  // unique: positions are distinct per consequent
      o[1 + n_out] = s_key[my_slot];
      s_key[my_slot] = -1;
      mine = best_of(my_slot);
    }
  }
  if (tid == 0) o[0] = n_out;
}

__global__ __launch_bounds__(64 * kWaves) void k_serve_match_topk(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ cons,
    const uint32_t* __restrict__ srank, const uint8_t* __restrict__ is_key, int64_t n_items,
    const int64_t* __restrict__ q_ptr, const int32_t* __restrict__ seeds, int64_t B, int k,
    int32_t* __restrict__ out) {
  __shared__ int32_t s_key[kWaves][kSlots];
  __shared__ uint32_t s_val[kWaves][kSlots];
  __shared__ uint32_t s_pos[kWaves][kSlots];
  __shared__ int64_t s_seg[kWaves][kMaxSeeds + 1];  // concatenation offsets of present seeds
  __shared__ int64_t s_row[kWaves][kMaxSeeds];      // row start of each present seed
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * kWaves + w;
  if (b >= B) return;  // wave-uniform: no block barrier below
  int32_t* key = s_key[w];
  uint32_t* val = s_val[w];
  uint32_t* pos = s_pos[w];
  int64_t* seg = s_seg[w];
  int64_t* rowp = s_row[w];
  const int64_t q0 = q_ptr[b], q1 = q_ptr[b + 1];
  int32_t* o = out + b * (int64_t)(k + 1);
  for (int i = lane; i < kSlots; i += 64) {
    key[i] = -1;
    val[i] = 0;
    pos[i] = 0xFFFFFFFFu;
  }
  if (q1 - q0 > kMaxSeeds) {
    if (lane == 0) o[0] = -2;  // too many seeds for the LDS tables: host path
    return;
  }
  // ---- present seeds, request order, 64 per pass ----
  int np = 0;
  int64_t acc = 0;
  for (int64_t c0 = q0; c0 < q1; c0 += 64) {
    const int64_t i = c0 + lane;
    int64_t len = 0;
    bool present = false;
    int64_t rs = 0;
    if (i < q1) {
      const int32_t sd = seeds[i];
      if (sd >= 0 && sd < n_items && is_key[sd]) {
        present = true;
        rs = row_ptr[sd];
        len = row_ptr[sd + 1] - rs;
      }
    }
    const unsigned long long bal = __ballot(present);
    const int rank = __popcll(bal & ((1ull << lane) - 1ull));
    int64_t inc = len;  // inclusive scan of the row lengths (0 for absent seeds)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t t = __shfl_up(inc, d, 64);
      if (lane >= d) inc += t;
    }
    if (present) {
      seg[np + rank] = acc + inc - len;
      rowp[np + rank] = rs;
    }
    np += __popcll(bal);
    acc += __shfl(inc, 63, 64);
  }
  if (np == 0) {
    if (lane == 0) o[0] = -1;  // no seed is a key: static fallback on the host
    return;
  }
  if (acc > kSlots / 2) {
    if (lane == 0) o[0] = -2;  // merged set could overflow the table: host path
    return;
  }
  if (lane == 0) seg[np] = acc;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  // ---- max-merge into the wave's table ----
  for (int64_t e = lane; e < acc; e += 64) {
    int lo = 0, hi = np;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (seg[mid] <= e) lo = mid; else hi = mid;
    }
    const int64_t p = rowp[lo] + (e - seg[lo]);
    const int32_t c = cons[p];
    const uint32_t v = srank[p];
    uint32_t h = ((uint32_t)c * 2654435761u) & (kSlots - 1);
    while (true) {
      const int32_t prev = atomicCAS(&key[h], -1, c);
      if (prev == -1 || prev == c) break;
      h = (h + 1) & (kSlots - 1);
    }
    atomicMax(&val[h], v + 1);  // +1: a touched slot is never 0
    atomicMin(&pos[h], (uint32_t)e);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
  // ---- top-k: per-lane best over its own slots, k rounds of a wave max ----
  auto lane_best = [&](int& slot) {
    unsigned long long best = 0;
    slot = -1;
#pragma unroll 4
    for (int j = 0; j < kPerLane; ++j) {
      const int i = j * 64 + lane;
      if (key[i] >= 0) {
        const unsigned long long kk =
            ((unsigned long long)val[i] << 32) | (unsigned long long)(0xFFFFFFFFu - pos[i]);
        if (kk > best) {
          best = kk;
          slot = i;
        }
      }
    }
    return best;
  };
  int my_slot;
  unsigned long long mine = lane_best(my_slot);
  int n_out = 0;
  for (; n_out < k; ++n_out) {
    unsigned long long bb = mine;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long t = __shfl_xor(bb, off, 64);
      bb = t > bb ? t : bb;
    }
    if (bb == 0) break;
    if (mine == bb) {  // unique: positions are distinct per consequent
      o[1 + n_out] = key[my_slot];
      key[my_slot] = -1;
      mine = lane_best(my_slot);
    }
  }
  if (lane == 0) o[0] = n_out;
}

}  // namespace

void serve_topk_big(const int64_t* row_ptr, const int32_t* cons, const uint32_t* srank,
                    const uint8_t* is_key, int64_t n_items, const int32_t* id_cons,
                    const int32_t* id_pos, const int64_t* q_ptr, const int32_t* seeds,
                    const int32_t* qlist, int64_t nq, int k, int32_t* out, hipStream_t s) {
  if (nq <= 0) return;
  hipLaunchKernelGGL(k_serve_topk_big, dim3((unsigned)nq), dim3(kBigThreads), 0, s, row_ptr, cons,
                     srank, is_key, n_items, id_cons, id_pos, q_ptr, seeds, qlist, k, out);
  KMLS_HIP(hipGetLastError());
}

void serve_match_topk(const int64_t* row_ptr, const int32_t* cons, const uint32_t* srank,
                      const uint8_t* is_key, int64_t n_items, const int64_t* q_ptr,
                      const int32_t* seeds, int64_t B, int k, int32_t* out, hipStream_t s) {
  if (B <= 0) return;
  const unsigned blocks = (unsigned)((B + kWaves - 1) / kWaves);
  hipLaunchKernelGGL(k_serve_match_topk, dim3(blocks), dim3(64 * kWaves), 0, s, row_ptr, cons,
                     srank, is_key, n_items, q_ptr, seeds, B, k, out);
  KMLS_HIP(hipGetLastError());
}

}  // namespace kern

namespace gpu {

GpuRuleIndex::GpuRuleIndex(int device, const RuleIndex& host, uintptr_t stream)
    : device_(device), n_items_(host.n_items()), nnz_(host.nnz()) {
  KMLS_HIP(hipSetDevice(device));
  if (stream) {
    stream_ = (void*)stream;
  } else {
    hipStream_t st;
    KMLS_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    stream_ = (void*)st;
    own_stream_ = true;
  }
  // exact order key: dense rank of each distinct score (ascending) → uint32
  const auto& sc = host.score();
  std::vector<double> uniq(sc.begin(), sc.end());
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  std::vector<uint32_t> sr(sc.size());
  for (size_t i = 0; i < sc.size(); ++i)
    sr[i] = (uint32_t)(std::lower_bound(uniq.begin(), uniq.end(), sc[i]) - uniq.begin()) + 1;
  const auto& rp = host.row_ptr();
  for (int64_t i = 0; i < n_items_; ++i) max_row_ = std::max<int>(max_row_, (int)(rp[i + 1] - rp[i]));
  h_row_ptr_.assign(rp.begin(), rp.end());
  h_is_key_.assign(host.is_key().begin(), host.is_key().end());
  hipStream_t s = (hipStream_t)stream_;
  KMLS_HIP(hipMalloc((void**)&d_row_ptr_, rp.size() * sizeof(int64_t)));
  KMLS_HIP(hipMalloc((void**)&d_cons_, std::max<size_t>(nnz_, 1) * sizeof(int32_t)));
  KMLS_HIP(hipMalloc((void**)&d_score_, std::max<size_t>(nnz_, 1) * sizeof(uint32_t)));
  KMLS_HIP(hipMalloc((void**)&d_is_key_, std::max<size_t>(n_items_, 1)));
  KMLS_HIP(hipMemcpyAsync(d_row_ptr_, rp.data(), rp.size() * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (nnz_) {
    KMLS_HIP(hipMemcpyAsync(d_cons_, host.cons().data(), nnz_ * sizeof(int32_t), hipMemcpyHostToDevice, s));
    KMLS_HIP(hipMemcpyAsync(d_score_, sr.data(), nnz_ * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  }
  if (n_items_)
    KMLS_HIP(hipMemcpyAsync(d_is_key_, host.is_key().data(), n_items_, hipMemcpyHostToDevice, s));
  // by-consequent copy of every row (the long-merge kernel's position lookups): a segmented
  // radix sort of (consequent, index in row) over the rows
  // the threshold pruning needs every row in non-increasing score order (our builders write
  // them so; a reference-format pickle may not): otherwise long merges stay on the host
  bool rows_sorted = true;
  for (int64_t i = 0; i < n_items_ && rows_sorted; ++i)
    for (int64_t e = rp[i] + 1; e < rp[i + 1]; ++e)
      if (sr[(size_t)e] > sr[(size_t)e - 1]) {
        rows_sorted = false;
        break;
      }
  if (nnz_ && max_row_ > 1 && rows_sorted) {
    std::vector<int32_t> ix((size_t)nnz_);
    for (int64_t i = 0; i < n_items_; ++i)
      for (int64_t e = rp[i]; e < rp[i + 1]; ++e) ix[(size_t)e] = (int32_t)(e - rp[i]);
    int32_t* d_ix_in = nullptr;
    void* tmp = nullptr;
    size_t tb = 0;
    KMLS_HIP(hipMalloc((void**)&d_id_cons_, nnz_ * sizeof(int32_t)));
    KMLS_HIP(hipMalloc((void**)&d_id_pos_, nnz_ * sizeof(int32_t)));
    KMLS_HIP(hipMalloc((void**)&d_ix_in, nnz_ * sizeof(int32_t)));
    KMLS_HIP(hipMemcpyAsync(d_ix_in, ix.data(), nnz_ * sizeof(int32_t), hipMemcpyHostToDevice, s));
    int end_bit = 1;
    while ((1ll << end_bit) < n_items_) ++end_bit;
    KMLS_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(
        nullptr, tb, d_cons_, d_id_cons_, d_ix_in, d_id_pos_, (int)nnz_, (int)n_items_,
        d_row_ptr_, d_row_ptr_ + 1, 0, end_bit, s));
    KMLS_HIP(hipMalloc(&tmp, std::max<size_t>(tb, 1)));
    KMLS_HIP(hipcub::DeviceSegmentedRadixSort::SortPairs(
        tmp, tb, d_cons_, d_id_cons_, d_ix_in, d_id_pos_, (int)nnz_, (int)n_items_,
        d_row_ptr_, d_row_ptr_ + 1, 0, end_bit, s));
    KMLS_HIP(hipStreamSynchronize(s));
    (void)hipFree(tmp);
    (void)hipFree(d_ix_in);
  }
  KMLS_HIP(hipStreamSynchronize(s));
}

GpuRuleIndex::~GpuRuleIndex() {
  (void)hipSetDevice(device_);
  for (void* p : {(void*)d_row_ptr_, (void*)d_cons_, (void*)d_score_, (void*)d_is_key_,
                  (void*)d_id_cons_, (void*)d_id_pos_})
    if (p) (void)hipFree(p);
  if (h_pinned_) (void)hipHostFree(h_pinned_);
  if (own_stream_) (void)hipStreamDestroy((hipStream_t)stream_);
}

void GpuRuleIndex::query_batch(const int64_t* q_ptr, int64_t B, const int32_t* seeds, int k,
                               int32_t* out_ids, int32_t* out_n) {
  KMLS_HIP(hipSetDevice(device_));
  hipStream_t s = (hipStream_t)stream_;
  const int64_t ns = q_ptr[B] - q_ptr[0];
  const int64_t no = B * (int64_t)(k + 1);
  // mapped pinned staging [q_ptr (rebased) | seeds | out]: the kernel reads the queries and
  // writes the results over PCIe directly (one launch per batch, no copy commands)
  // long merges (more entries than the wave kernel's table) go to the workgroup kernel
  std::vector<int32_t> big;
  if (d_id_cons_) {
    for (int64_t b = 0; b < B; ++b) {
      if (q_ptr[b + 1] - q_ptr[b] > kern::kServeMaxSeeds) continue;  // host path (-2)
      int64_t acc = 0;
      for (int64_t i = q_ptr[b]; i < q_ptr[b + 1]; ++i) {
        const int32_t sd = seeds[i];
        if (sd >= 0 && sd < n_items_ && h_is_key_[(size_t)sd])
          acc += h_row_ptr_[(size_t)sd + 1] - h_row_ptr_[(size_t)sd];
      }
      if (acc > kern::kServeWaveMerge) big.push_back((int32_t)b);
    }
  }
  const int64_t nb = (int64_t)big.size();
  const int64_t words = 2 * (B + 1) + ns + no + nb;
  if (words > cap_pinned_) {
    if (h_pinned_) KMLS_HIP(hipHostFree(h_pinned_));
    h_pinned_ = nullptr;
    cap_pinned_ = std::max<int64_t>(words, cap_pinned_ * 2);
    KMLS_HIP(hipHostMalloc((void**)&h_pinned_, (size_t)cap_pinned_ * sizeof(int32_t),
                           hipHostMallocMapped));
  }
  int64_t* hq = reinterpret_cast<int64_t*>(h_pinned_);
  int32_t* hs = h_pinned_ + 2 * (B + 1);
  int32_t* ho = hs + ns;
  int32_t* hb = ho + no;
  for (int64_t i = 0; i <= B; ++i) hq[i] = q_ptr[i] - q_ptr[0];
  std::copy(seeds + q_ptr[0], seeds + q_ptr[B], hs);
  std::copy(big.begin(), big.end(), hb);
  int32_t* dev = nullptr;
  KMLS_HIP(hipHostGetDevicePointer((void**)&dev, h_pinned_, 0));
  const int64_t* dq = reinterpret_cast<const int64_t*>(dev);
  int32_t* dout = dev + 2 * (B + 1) + ns;
  kern::serve_match_topk(d_row_ptr_, d_cons_, d_score_, d_is_key_, n_items_, dq,
                         dev + 2 * (B + 1), B, k, dout, s);
  // same stream: overwrites the wave kernel's -2 for the long merges
  kern::serve_topk_big(d_row_ptr_, d_cons_, d_score_, d_is_key_, n_items_, d_id_cons_,
                       d_id_pos_, dq, dev + 2 * (B + 1), dout + no, nb, k, dout, s);
  KMLS_HIP(hipStreamSynchronize(s));
  for (int64_t b = 0; b < B; ++b) {
    const int32_t n = ho[b * (k + 1)];
    out_n[b] = n;
    for (int j = 0; j < k; ++j) out_ids[b * k + j] = (j < n) ? ho[b * (k + 1) + 1 + j] : -1;
  }
}

}  // namespace gpu
}  // namespace kmls
