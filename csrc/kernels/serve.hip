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
// Queries whose merged set would overflow the table (or with > kMaxSeeds seeds) report -2 and
// are answered on the host.  Queries are read from, and results written to, mapped pinned host
// memory: one kernel launch per batch, no staging copies.
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

constexpr int kWaves = 4;                 // queries per block
constexpr int kSlots = 1024;              // hash slots per wave
constexpr int kPerLane = kSlots / 64;     // slots each lane owns in the top-k scan
constexpr int kMaxSeeds = 256;

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
  for (void* p : {(void*)d_row_ptr_, (void*)d_cons_, (void*)d_score_, (void*)d_is_key_})
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
  const int64_t words = 2 * (B + 1) + ns + no;
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
  for (int64_t i = 0; i <= B; ++i) hq[i] = q_ptr[i] - q_ptr[0];
  std::copy(seeds + q_ptr[0], seeds + q_ptr[B], hs);
  int32_t* dev = nullptr;
  KMLS_HIP(hipHostGetDevicePointer((void**)&dev, h_pinned_, 0));
  kern::serve_match_topk(d_row_ptr_, d_cons_, d_score_, d_is_key_, n_items_,
                         reinterpret_cast<const int64_t*>(dev), dev + 2 * (B + 1), B, k,
                         dev + 2 * (B + 1) + ns, s);
  KMLS_HIP(hipStreamSynchronize(s));
  for (int64_t b = 0; b < B; ++b) {
    const int32_t n = ho[b * (k + 1)];
    out_n[b] = n;
    for (int j = 0; j < k; ++j) out_ids[b * k + j] = (j < n) ? ho[b * (k + 1) + 1 + j] : -1;
  }
}

}  // namespace gpu
}  // namespace kmls
