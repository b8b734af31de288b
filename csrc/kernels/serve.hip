// serve_match_topk: batched antecedent matching over an HBM-resident CSR rule index.
//
// Exact semantics of recommend_tracks_for_track (rest_api/app/main.py:235-254):
//   merged[r] = max over present seeds' rows of score(r)          (max-merge)
//   order     = score desc, ties by first insertion position      (stable sort over dict order)
// The insertion position of r is the first position where r occurs in the concatenation of
// the present seeds' rows (request order, row order), so both reductions are commutative:
// (max score-rank, min position).  One 256-thread workgroup per query; an LDS open-address
// hash table (4096 slots) accumulates both with LDS atomics; top-k = k rounds of a wave64
// shuffle + LDS block argmax over the 64-bit key (score_rank << 32 | ~position).
// Queries whose merged set would not fit the table report -2 and are answered on the host.
#include <hip/hip_runtime.h>

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

constexpr int kSlots = 4096;
constexpr int kMaxSeeds = 256;
constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void k_serve_match_topk(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ cons,
    const uint32_t* __restrict__ srank, const uint8_t* __restrict__ is_key, int64_t n_items,
    const int64_t* __restrict__ q_ptr, const int32_t* __restrict__ seeds, int k,
    int32_t* __restrict__ out) {
  __shared__ int32_t s_key[kSlots];
  __shared__ uint32_t s_val[kSlots];
  __shared__ uint32_t s_pos[kSlots];
  __shared__ int64_t s_seg[kMaxSeeds + 1];  // concatenation offsets of present seeds
  __shared__ int64_t s_row[kMaxSeeds];      // row start of each present seed
  __shared__ int s_np;
  __shared__ unsigned long long s_red[kThreads / 64];

  const int64_t b = blockIdx.x;
  const int64_t q0 = q_ptr[b], q1 = q_ptr[b + 1];
  int32_t* o = out + b * (int64_t)(k + 1);
  const int tid = threadIdx.x;
  for (int i = tid; i < kSlots; i += kThreads) {
    s_key[i] = -1;
    s_val[i] = 0;
    s_pos[i] = 0xFFFFFFFFu;
  }
  if (tid == 0) {
    // present seeds in request order (serial: #seeds is small)
    int np = 0;
    int64_t acc = 0;
    for (int64_t i = q0; i < q1 && np < kMaxSeeds; ++i) {
      const int32_t sd = seeds[i];
      if (sd < 0 || sd >= n_items || !is_key[sd]) continue;
      s_seg[np] = acc;
      s_row[np] = row_ptr[sd];
      acc += row_ptr[sd + 1] - row_ptr[sd];
      ++np;
    }
    s_seg[np] = acc;
    int flag = np;
    if (q1 - q0 > kMaxSeeds) flag = -2;          // too many seeds: host path
    if (np > 0 && acc > kSlots / 2) flag = -2;   // table would overflow: host path
    s_np = flag;
  }
  __syncthreads();
  const int np = s_np;
  if (np <= 0) {
    if (tid == 0) o[0] = (np == 0) ? -1 : -2;
    return;
  }
  const int64_t L = s_seg[np];
  // insert all entries
  for (int64_t e = tid; e < L; e += kThreads) {
    int lo = 0, hi = np;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (s_seg[mid] <= e) lo = mid; else hi = mid;
    }
    const int64_t p = s_row[lo] + (e - s_seg[lo]);
    const int32_t c = cons[p];
    const uint32_t v = srank[p];
    uint32_t hsh = ((uint32_t)c * 2654435761u) & (kSlots - 1);
    while (true) {
      const int32_t prev = atomicCAS(&s_key[hsh], -1, c);
      if (prev == -1 || prev == c) break;
      hsh = (hsh + 1) & (kSlots - 1);
    }
    // first touch initialises (val 0 / pos max) lazily via atomics on zero-initialised slots
    atomicMax(&s_val[hsh], v + 1);  // +1: distinguish "touched" from untouched 0
    atomicMin(&s_pos[hsh], (uint32_t)e);
  }
  __syncthreads();
  // top-k rounds
  int n_out = 0;
  for (int round = 0; round < k; ++round) {
    unsigned long long best = 0;
    for (int i = tid; i < kSlots; i += kThreads) {
      if (s_key[i] >= 0) {
        const unsigned long long key =
            ((unsigned long long)s_val[i] << 32) | (unsigned long long)(0xFFFFFFFFu - s_pos[i]);
        best = key > best ? key : best;
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned long long other = __shfl_xor(best, off, 64);
      best = other > best ? other : best;
    }
    if ((tid & 63) == 0) s_red[tid >> 6] = best;
    __syncthreads();
    unsigned long long bb = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) bb = s_red[w] > bb ? s_red[w] : bb;
    __syncthreads();
    if (bb == 0) break;
    // the winner slot: unique (positions are unique per distinct consequent)
    const uint32_t wpos = 0xFFFFFFFFu - (uint32_t)(bb & 0xFFFFFFFFu);
    for (int i = tid; i < kSlots; i += kThreads) {
      if (s_key[i] >= 0 && s_pos[i] == wpos) {
        o[1 + round] = s_key[i];
        s_key[i] = -1;  // remove
      }
    }
    ++n_out;
    __syncthreads();
  }
  if (tid == 0) o[0] = n_out;
}

}  // namespace

void serve_match_topk(const int64_t* row_ptr, const int32_t* cons, const uint32_t* srank,
                      const uint8_t* is_key, int64_t n_items, const int64_t* q_ptr,
                      const int32_t* seeds, int64_t B, int k, int32_t* out, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(k_serve_match_topk, dim3((unsigned)B), dim3(kThreads), 0, s, row_ptr, cons,
                     srank, is_key, n_items, q_ptr, seeds, k, out);
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
  KMLS_HIP(hipStreamSynchronize(s));
}

GpuRuleIndex::~GpuRuleIndex() {
  (void)hipSetDevice(device_);
  for (void* p : {(void*)d_row_ptr_, (void*)d_cons_, (void*)d_score_, (void*)d_is_key_,
                  (void*)d_q_ptr_, (void*)d_seeds_, (void*)d_out_})
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
  auto grow = [&](auto*& p, int64_t& cap, int64_t need, size_t el) {
    if (need <= cap) return;
    if (p) KMLS_HIP(hipFree(p));
    cap = std::max<int64_t>(need, cap * 2);
    KMLS_HIP(hipMalloc((void**)&p, (size_t)cap * el));
  };
  grow(d_q_ptr_, cap_q_, B + 1, sizeof(int64_t));
  grow(d_seeds_, cap_s_, std::max<int64_t>(ns, 1), sizeof(int32_t));
  grow(d_out_, cap_o_, no, sizeof(int32_t));
  // pinned staging: [q_ptr (rebased) | seeds | out]
  const int64_t words = 2 * (B + 1) + ns + no;
  if (words > cap_pinned_) {
    if (h_pinned_) KMLS_HIP(hipHostFree(h_pinned_));
    cap_pinned_ = std::max<int64_t>(words, cap_pinned_ * 2);
    KMLS_HIP(hipHostMalloc((void**)&h_pinned_, (size_t)cap_pinned_ * sizeof(int32_t)));
  }
  int64_t* hq = reinterpret_cast<int64_t*>(h_pinned_);
  int32_t* hs = h_pinned_ + 2 * (B + 1);
  int32_t* ho = hs + ns;
  for (int64_t i = 0; i <= B; ++i) hq[i] = q_ptr[i] - q_ptr[0];
  std::copy(seeds + q_ptr[0], seeds + q_ptr[B], hs);
  KMLS_HIP(hipMemcpyAsync(d_q_ptr_, hq, (B + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
  if (ns) KMLS_HIP(hipMemcpyAsync(d_seeds_, hs, ns * sizeof(int32_t), hipMemcpyHostToDevice, s));
  kern::serve_match_topk(d_row_ptr_, d_cons_, d_score_, d_is_key_, n_items_,
                         d_q_ptr_, d_seeds_, B, k, d_out_, s);
  KMLS_HIP(hipMemcpyAsync(ho, d_out_, no * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  KMLS_HIP(hipStreamSynchronize(s));
  for (int64_t b = 0; b < B; ++b) {
    const int32_t n = ho[b * (k + 1)];
    out_n[b] = n;
    for (int j = 0; j < k; ++j) out_ids[b * k + j] = (j < n) ? ho[b * (k + 1) + 1 + j] : -1;
  }
}

}  // namespace gpu
}  // namespace kmls
