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
#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../include/kmls/gpu.hpp"
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

// Wave-wide max of a u32 through DPP row shifts and row broadcasts (an inclusive max-scan
// whose lane 63 holds the total), then a lane-63 read: ~8 short-latency DPP steps instead of
// six 64-lane permutes through the LDS crossbar.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x113, 0xf, 0xf, false));  // row_shr:3
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xf, 0xe, false));  // row_shr:4
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xf, 0xc, false));  // row_shr:8
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// 64-bit wave max as two u32 passes (high words, then the low words of the lanes that hold it)
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
  const uint32_t hi = wave_max_u32((uint32_t)(v >> 32));
  const uint32_t lo = wave_max_u32((uint32_t)(v >> 32) == hi ? (uint32_t)v : 0u);
  return ((unsigned long long)hi << 32) | lo;
}

// one query (seeds[q0, q1), request order) answered by the calling wave into o[0 .. k]: o[0] =
// the number of ids (-1 no seed is a key, -2 host path), o[1 ..] = ids; per-wave LDS tables
__device__ __forceinline__ void serve_query_wave(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ cons,
    const uint32_t* __restrict__ srank, const uint8_t* __restrict__ is_key, int64_t n_items,
    const int32_t* __restrict__ seeds, int64_t q0, int64_t q1, int k, int32_t* __restrict__ o,
    int32_t* key, uint32_t* val, uint32_t* pos, int64_t* seg, int64_t* rowp, int lane,
    unsigned long long* stamps = nullptr, bool narrow = false) {
  // (stamps: instrumentation, the serving loop's first query; lane 0 writes wall clock ticks)
  auto stamp = [&](int i) {
    if (stamps && lane == 0) stamps[i] = wall_clock64();
  };
  stamp(0);
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
      if (sd >= 0 && sd < n_items) {
        // the three loads in flight together (is_key gated a dependent second round trip)
        const uint8_t kk = is_key[sd];
        const int64_t r0 = row_ptr[sd], r1 = row_ptr[sd + 1];
        if (kk) {
          present = true;
          rs = r0;
          len = r1 - r0;
        }
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
  stamp(1);
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
  // every entry of this lane (<= kSlots / 2 / 64) is loaded first, all loads in flight at once;
  // then inserted (the LDS atomics kept each iteration's HBM loads from overlapping the next:
  // ~1 us of latency per 64 entries)
  constexpr int kPer = kSlots / 2 / 64;
  int32_t ec[kPer];
  uint32_t ev[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t e = lane + 64 * u;
    ec[u] = -1;
    ev[u] = 0;
    if (e < acc) {
      int lo = 0, hi = np;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (seg[mid] <= e) lo = mid; else hi = mid;
      }
      const int64_t p = rowp[lo] + (e - seg[lo]);
      ec[u] = cons[p];
      ev[u] = srank[p];
    }
  }
  stamp(2);
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t e = lane + 64 * u;
    if (e >= acc) continue;
    const int32_t c = ec[u];
    const uint32_t v = ev[u];
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
  stamp(3);
  // ---- top-k: each lane's own slots held in registers (one pipelined round of LDS loads),
  // k rounds of a wave max; the winning lane clears its entry and re-takes its register max.
  // (Rescanning the winner's slots from LDS every round cost ~1 us per round: 12 of the 14 us
  // of a one-query request in the serving loop.)
  int n_out = 0;
  bool done_small = false;
  if (narrow) {
    // small merges (<= 128 distinct consequents, the common request): compact the occupied
    // slots into LDS, then every lane ranks its (one or two) entries against all of them
    // (broadcast reads) and writes each at its rank if it is in the top k — no serial rounds
    uint32_t* cv = reinterpret_cast<uint32_t*>(seg);  // (free after the merge)
    int32_t* ck = reinterpret_cast<int32_t*>(rowp);
    uint32_t nocc = 0;
    const unsigned long long lanelt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) {
      const int i = j * 64 + lane;
      const int32_t c = key[i];
      const bool occ = c >= 0;
      const unsigned long long m = __ballot(occ);
      if (occ) {
        const uint32_t q = nocc + (uint32_t)__popcll(m & lanelt);
        if (q < 128u) {
          cv[q] = (val[i] << 9) | (511u - pos[i]);
          ck[q] = c;
        }
      }
      nocc += (uint32_t)__popcll(m);
    }
    if (nocc <= 128u) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      __builtin_amdgcn_wave_barrier();
      const uint32_t a_idx = (uint32_t)lane, b_idx = (uint32_t)lane + 64u;
      const uint32_t va = a_idx < nocc ? cv[a_idx] : 0u;
      const uint32_t vb = b_idx < nocc ? cv[b_idx] : 0u;
      uint32_t ra = 0, rb = 0;
      // 8 broadcast reads in flight per step: one dependent LDS round trip per 8 entries
      // instead of per entry (~64 cycles each: 128 entries took ~3 us of a one-query request)
      uint32_t t = 0;
      for (; t + 8 <= nocc; t += 8) {
        uint32_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = cv[t + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          ra += x[u] > va ? 1u : 0u;
          rb += x[u] > vb ? 1u : 0u;
        }
      }
      for (; t < nocc; ++t) {
        const uint32_t x = cv[t];
        ra += x > va ? 1u : 0u;
        rb += x > vb ? 1u : 0u;
      }
      if (a_idx < nocc && ra < (uint32_t)k) o[1 + ra] = ck[a_idx];
      if (b_idx < nocc && rb < (uint32_t)k) o[1 + rb] = ck[b_idx];
      n_out = (int)min(nocc, (uint32_t)k);
      done_small = true;
    }
  }
  if (narrow && !done_small) {
    // score ranks < 2^23 (checked at index load) and first positions < 512: the order key fits
    // 32 bits, so a round is one 32-bit DPP max
    uint32_t kk[kPerLane];
    int32_t kc[kPerLane];
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) {
      const int i = j * 64 + lane;
      const int32_t c = key[i];
      const uint32_t v = val[i], ps = pos[i];
      kc[j] = c;
      kk[j] = c >= 0 ? ((v << 9) | (511u - ps)) : 0u;
    }
    auto reg_best = [&]() {
      uint32_t b = 0;
#pragma unroll
      for (int j = 0; j < kPerLane; ++j) b = max(b, kk[j]);
      return b;
    };
    uint32_t mine = reg_best();
    for (; n_out < k; ++n_out) {
      const uint32_t bb = wave_max_u32(mine);
      if (bb == 0) break;
      if (mine == bb) {
        int32_t id = -1;
#pragma unroll
        for (int j = 0; j < kPerLane; ++j)
          if (kk[j] == bb) {
            id = kc[j];
            kk[j] = 0u;
          }
        o[1 + n_out] = id;
        mine = reg_best();
      }
    }
  } else if (!narrow) {
    unsigned long long kk[kPerLane];
    int32_t kc[kPerLane];
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) {
      const int i = j * 64 + lane;
      const int32_t c = key[i];
      const uint32_t v = val[i], ps = pos[i];
      kc[j] = c;
      kk[j] = c >= 0 ? (((unsigned long long)v << 32) | (unsigned long long)(0xFFFFFFFFu - ps)) : 0ull;
    }
    auto reg_best = [&]() {
      unsigned long long b = 0;
#pragma unroll
      for (int j = 0; j < kPerLane; ++j) b = kk[j] > b ? kk[j] : b;
      return b;
    };
    unsigned long long mine = reg_best();
    for (; n_out < k; ++n_out) {
      const unsigned long long bb = wave_max_u64(mine);
      if (bb == 0) break;
      if (mine == bb) {  // unique: positions are distinct per consequent
        int32_t id = -1;
#pragma unroll
        for (int j = 0; j < kPerLane; ++j)
          if (kk[j] == bb) {
            id = kc[j];
            kk[j] = 0ull;
          }
        o[1 + n_out] = id;
        mine = reg_best();
      }
    }
  }
  if (lane == 0) o[0] = n_out;
  stamp(4);
}

__global__ __launch_bounds__(64 * kWaves) void k_serve_match_topk(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ cons,
    const uint32_t* __restrict__ srank, const uint8_t* __restrict__ is_key, int64_t n_items,
    const int64_t* __restrict__ q_ptr, const int32_t* __restrict__ seeds, int64_t B, int k,
    int32_t* __restrict__ out, int narrow) {
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
  serve_query_wave(row_ptr, cons, srank, is_key, n_items, seeds, q0, q1, k,
                   out + b * (int64_t)(k + 1), key, val, pos, seg, rowp, lane, nullptr,
                   narrow != 0);
}

// ---- the persistent serving loop (gpu::GpuServeLoop) ----
// The mailbox and the payload live in fine-grained (coherent, uncached) host memory: relaxed
// system-scope accesses go to the host every time, so no acquire/release fences are used — a
// system-scope acquire invalidates, and a release writes back, the XCD's whole L2 on every poll
// and every answer (measured: ~33 us per round trip with them).  Ordering instead: the host
// writes payload and descriptor before the request word (x86 store order); the kernel's result
// stores drain (vmcnt 0) before the done word is written, and PCIe keeps posted writes in order.
__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kLoopStage = kServeLoopStage;
constexpr int kLoopOut = kServeLoopOut;

// One workgroup per request slot (blockIdx.x = slot): lane 0 of wave 0 polls the slot's request
// word (a short sleep between polls); a new sequence number is broadcast through LDS, the request
// is staged into LDS by every thread in one round of loads, every wave answers queries w, w + 4,
// ... with the wave matcher (results written straight to mapped host memory), and after the
// barrier lane 0 publishes the slot's done word.  The slots are independent: host threads with
// requests in different slots are answered concurrently by different workgroups (one mailbox
// serialised every front thread behind one request in flight).
// Exit: the stop word, or (decided by workgroup 0 for the whole launch, from the newest request
// clock any workgroup recorded) no request for idle_ticks or life_ticks since the launch: it
// sets ctl->quit = gen, which every workgroup sees within one poll round.  A leaving workgroup
// writes its slot's exited_gen = gen: the host tells "this launch exited" from "not started
// yet" by that word alone (an alive flag set by the kernel once it ran could not).
__global__ __launch_bounds__(64 * kWaves) void k_serve_loop(ServeMail* mail, ServeLoopCtl* ctl,
                                                            unsigned gen,
                                                            unsigned long long idle_ticks,
                                                            unsigned long long life_ticks) {
  __shared__ int32_t s_key[kWaves][kSlots];
  __shared__ uint32_t s_val[kWaves][kSlots];
  __shared__ uint32_t s_pos[kWaves][kSlots];
  __shared__ int64_t s_seg[kWaves][kMaxSeeds + 1];
  __shared__ int64_t s_row[kWaves][kMaxSeeds];
  __shared__ long long s_stage64[kLoopStage / 2];  // (8-byte aligned: q_ptr is int64)
  __shared__ int32_t s_out[kLoopOut];
  int32_t* s_stage = (int32_t*)s_stage64;
  __shared__ unsigned s_cmd, s_seq, s_words;
  __shared__ unsigned long long s_stamps[6];
  __shared__ ServeReq s_req;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  ServeSlot* slot = &mail->slot[blockIdx.x];
  unsigned last = 0;
  const unsigned long long t0 = wall_clock64();
  if (tid == 0) {
    // a request the host gave up on was marked consumed (done_seq = its seq) before this
    // launch, so only requests still pending are served
    last = ld_sys(&slot->done_seq);
    if (blockIdx.x == 0) atomicMax(&ctl->last_activity, t0);
  }
  while (true) {
    if (tid == 0) {
      unsigned cmd = 0;
      for (unsigned n = 0;; ++n) {
        const unsigned long long r =
            __hip_atomic_load(&slot->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((unsigned)r != last) {
          cmd = 1;
          s_seq = (unsigned)r;
          s_words = (unsigned)(r >> 32);
          break;
        }
        if ((n & 15u) == 15u) {
          if (ld_sys(&mail->stop) != 0u) break;
          if (__hip_atomic_load(&ctl->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen)
            break;
          if (blockIdx.x == 0) {
            const unsigned long long now = wall_clock64();
            const unsigned long long la =
                __hip_atomic_load(&ctl->last_activity, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((now > la && now - la > idle_ticks) || now - t0 > life_ticks) {
              __hip_atomic_store(&ctl->quit, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (cmd)
        __hip_atomic_store(&slot->t_seen, wall_clock64(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);  // (instrumentation: device clock)
      s_cmd = cmd;
    }
    __syncthreads();
    if (s_cmd == 0u) break;
    // stage [descriptor | q_ptr | seeds] in ONE round of parallel system-scope loads, which
    // bypass the caches (the mailbox is rewritten by the host for every request)
    {
      constexpr int kDesc = (int)(sizeof(ServeReq) / 4);
      const int total = kDesc + (int)min(s_words, (unsigned)kLoopStage);
      const unsigned* src = (const unsigned*)&slot->req_desc;
      unsigned* dreq = (unsigned*)&s_req;
      unsigned* dst = (unsigned*)s_stage;
      for (int i = tid; i < total; i += 64 * kWaves) {
        const unsigned v = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (i < kDesc) dreq[i] = v;
        else dst[i - kDesc] = v;
      }
    }
    __syncthreads();
    const ServeReq rq = s_req;
    if (tid == 0)
      __hip_atomic_store(&slot->t_staged, wall_clock64(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    const long long* qp = (const long long*)s_stage;
    const int32_t* sd = s_stage + 2 * (rq.B + 1);
    const long long ow = rq.B * (rq.k + 1);
    for (long long b = w; b < rq.B; b += kWaves) {
      const long long q0 = qp[b], q1 = qp[b + 1];
      serve_query_wave(rq.row_ptr, rq.cons, rq.srank, rq.is_key, rq.n_items, sd, q0, q1, rq.k,
                       s_out + b * (long long)(rq.k + 1), s_key[w], s_val[w], s_pos[w],
                       s_seg[w], s_row[w], lane, b == 0 ? s_stamps : nullptr,
                       rq.narrow != 0);
    }
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_store(&slot->t_computed, wall_clock64(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      for (int i = 0; i < 5; ++i)
        __hip_atomic_store(&slot->t_phase[i], s_stamps[i], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // results out with system-scope (write-through) stores, drained before the done word
    for (long long i = tid; i < ow && i < kLoopOut; i += 64 * kWaves)
      __hip_atomic_store(rq.out + i, s_out[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      last = s_seq;
      const unsigned long long now = wall_clock64();
      atomicMax(&ctl->last_activity, now);
      __hip_atomic_store(&slot->t_done, now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      st_sys(&slot->done_seq, last);
    }
  }
  if (tid == 0) st_sys(&slot->exited_gen, gen);
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

void serve_loop_launch(ServeMail* mail, ServeLoopCtl* ctl, unsigned gen, int nslots,
                       unsigned long long idle_ticks, unsigned long long life_ticks,
                       hipStream_t s) {
  if (nslots < 1 || nslots > kServeLoopSlots)
    throw std::runtime_error("serve_loop_launch: 1 <= nslots <= kServeLoopSlots");
  hipLaunchKernelGGL(k_serve_loop, dim3((unsigned)nslots), dim3(64 * kWaves), 0, s, mail, ctl,
                     gen, idle_ticks, life_ticks);
  KMLS_HIP(hipGetLastError());
}

void serve_match_topk(const int64_t* row_ptr, const int32_t* cons, const uint32_t* srank,
                      const uint8_t* is_key, int64_t n_items, const int64_t* q_ptr,
                      const int32_t* seeds, int64_t B, int k, int32_t* out, hipStream_t s,
                      bool narrow) {
  if (B <= 0) return;
  const unsigned blocks = (unsigned)((B + kWaves - 1) / kWaves);
  hipLaunchKernelGGL(k_serve_match_topk, dim3(blocks), dim3(64 * kWaves), 0, s, row_ptr, cons,
                     srank, is_key, n_items, q_ptr, seeds, B, k, out, narrow ? 1 : 0);
  KMLS_HIP(hipGetLastError());
}

}  // namespace kern

namespace gpu {

// ---- the persistent serving loop ----
namespace {
std::mutex g_loops_mu;
std::vector<std::unique_ptr<GpuServeLoop>> g_loops;  // by device (never destroyed before exit)
std::vector<int> g_pending_pause;                     // pauses requested before a loop existed
}  // namespace

GpuServeLoop& GpuServeLoop::for_device(int device) {
  std::lock_guard<std::mutex> lk(g_loops_mu);
  if ((int)g_loops.size() <= device) g_loops.resize((size_t)device + 1);
  if (!g_loops[(size_t)device]) {
    g_loops[(size_t)device].reset(new GpuServeLoop(device));
    if ((int)g_pending_pause.size() > device) g_loops[(size_t)device]->paused_ = g_pending_pause[(size_t)device];
  }
  return *g_loops[(size_t)device];
}

ServeLoopPause::ServeLoopPause(int dev) : device(dev) {
  GpuServeLoop* l = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_loops_mu);
    if ((int)g_loops.size() > dev && g_loops[(size_t)dev]) l = g_loops[(size_t)dev].get();
    else {
      if ((int)g_pending_pause.size() <= dev) g_pending_pause.resize((size_t)dev + 1, 0);
      ++g_pending_pause[(size_t)dev];
    }
  }
  if (l) l->pause();
}

ServeLoopPause::~ServeLoopPause() {
  GpuServeLoop* l = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_loops_mu);
    if ((int)g_loops.size() > device && g_loops[(size_t)device]) l = g_loops[(size_t)device].get();
    else if ((int)g_pending_pause.size() > device) --g_pending_pause[(size_t)device];
  }
  if (l) l->resume();
}

GpuServeLoop::GpuServeLoop(int device) : device_(device) {
  KMLS_HIP(hipSetDevice(device));
  hipStream_t st;
  KMLS_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  stream_ = (void*)st;
  KMLS_HIP(hipHostMalloc(&mail_, sizeof(kern::ServeMail), hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(mail_, 0, sizeof(kern::ServeMail));
  KMLS_HIP(hipMalloc(&ctl_, sizeof(kern::ServeLoopCtl)));
  KMLS_HIP(hipMemset(ctl_, 0, sizeof(kern::ServeLoopCtl)));
  // slots (polling workgroups): KMLS_SERVE_SLOTS, default 4 = the native front's I/O threads
  nslots_ = (int)std::max<long long>(1, std::min<long long>(kern::kServeLoopSlots,
                                                            test_hook("serve_slots", [] {
    const char* e = std::getenv("KMLS_SERVE_SLOTS");
    return e ? std::atoll(e) : 4ll;
  }())));
  free_mask_.store((uint32_t)((1ull << nslots_) - 1ull));
  KMLS_HIP(hipHostMalloc((void**)&buf_, (size_t)nslots_ * kern::kServeLoopOut * sizeof(int32_t),
                         hipHostMallocMapped | hipHostMallocCoherent));
  int khz = 0;
  KMLS_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
  const unsigned long long per_ms = (unsigned long long)std::max(khz, 1);
  ticks_per_us_ = (double)per_ms / 1000.0;
  idle_ticks_ = per_ms * 20;     // 20 ms without a request: exit (relaunched on demand)
  life_ticks_ = per_ms * 2000;   // and at most 2 s per launch
}

GpuServeLoop::~GpuServeLoop() {
  try {
    std::lock_guard<std::mutex> lk(launch_mu_);
    stop_and_wait_locked();
  } catch (...) {
  }
  if (buf_) (void)hipHostFree(buf_);
  if (mail_) (void)hipHostFree(mail_);
  if (ctl_) (void)hipFree(ctl_);
  if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
}

bool GpuServeLoop::exited_locked(unsigned gen) const {
  volatile kern::ServeMail* m = (volatile kern::ServeMail*)mail_;
  for (int s = 0; s < nslots_; ++s)
    if (m->slot[s].exited_gen != gen) return false;
  return true;
}

void GpuServeLoop::stop_and_wait_locked() {
  if (!launched_) return;
  volatile kern::ServeMail* m = (volatile kern::ServeMail*)mail_;
  m->stop = 1u;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  KMLS_HIP(hipStreamSynchronize((hipStream_t)stream_));  // the kernel exits within one poll
  launched_ = false;
}

void GpuServeLoop::consume_locked(int slot, unsigned seq) {
  // only while no kernel runs: the next launch starts from done_seq and never serves it
  volatile kern::ServeMail* m = (volatile kern::ServeMail*)mail_;
  m->slot[slot].done_seq = seq;
  std::atomic_thread_fence(std::memory_order_seq_cst);
}

unsigned GpuServeLoop::ensure_running_locked() {
  if (paused_ > 0) return 0;
  if (launched_ && !exited_locked(gen_)) return gen_;
  if (launched_) {  // every workgroup of it has left (idle / lifetime): it is finishing
    KMLS_HIP(hipStreamSynchronize((hipStream_t)stream_));
    launched_ = false;
  }
  volatile kern::ServeMail* m = (volatile kern::ServeMail*)mail_;
  m->stop = 0u;
  const unsigned gen = ++gen_;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  kmls::kern::ServeMail* dm = nullptr;
  KMLS_HIP(hipHostGetDevicePointer((void**)&dm, mail_, 0));
  kern::serve_loop_launch(dm, (kern::ServeLoopCtl*)ctl_, gen, nslots_, idle_ticks_, life_ticks_,
                          (hipStream_t)stream_);
  launched_ = true;
  {
    std::lock_guard<std::mutex> sl(stats_mu_);
    ++st_.launches;
  }
  return gen;
}

void GpuServeLoop::pause() {
  std::lock_guard<std::mutex> lk(launch_mu_);
  ++paused_;
  stop_and_wait_locked();
}

void GpuServeLoop::resume() {
  std::lock_guard<std::mutex> lk(launch_mu_);
  if (paused_ > 0) --paused_;
}

ServeLoopStats GpuServeLoop::stats() {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return st_;
}

int GpuServeLoop::claim_slot() {
  uint32_t m = free_mask_.load(std::memory_order_acquire);
  while (m) {
    const int s = __builtin_ctz(m);
    if (free_mask_.compare_exchange_weak(m, m & ~(1u << s), std::memory_order_acq_rel))
      return s;
  }
  return -1;
}

void GpuServeLoop::release_slot(int slot) {
  free_mask_.fetch_or(1u << slot, std::memory_order_acq_rel);
}

bool GpuServeLoop::run(const int64_t* d_row_ptr, const int32_t* d_cons, const uint32_t* d_score,
                       const uint8_t* d_is_key, int64_t n_items, const int64_t* q_ptr, int64_t B,
                       const int32_t* seeds, int k, int32_t* out_ids, int32_t* out_n,
                       bool narrow) {
  const int slot = claim_slot();
  if (slot < 0) {  // every slot holds a request in flight: the caller answers on the host
    std::lock_guard<std::mutex> sl(stats_mu_);
    ++st_.refused;
    return false;
  }
  struct Release {
    GpuServeLoop* l;
    int s;
    ~Release() { l->release_slot(s); }
  } rel{this, slot};
  // one round trip holds what the kernel stages in LDS: split longer batches
  int64_t b0 = 0;
  while (b0 < B) {
    int64_t b1 = b0;
    while (b1 < B) {
      const int64_t nb = b1 + 1 - b0;
      if (2 * (nb + 1) + (q_ptr[b1 + 1] - q_ptr[b0]) > kern::kServeLoopStage ||
          nb * (k + 1) > kern::kServeLoopOut)
        break;
      ++b1;
    }
    if (b1 == b0) {  // one query past the stage (hundreds of seeds): not the loop's
      out_n[b0] = -2;
      for (int j = 0; j < k; ++j) out_ids[b0 * k + j] = -1;
      ++b0;
      continue;
    }
    if (!run_one(slot, d_row_ptr, d_cons, d_score, d_is_key, n_items, q_ptr + b0, b1 - b0,
                 seeds, k, out_ids + b0 * k, out_n + b0, narrow))
      return false;
    b0 = b1;
  }
  return true;
}

bool GpuServeLoop::run_one(int slot, const int64_t* d_row_ptr, const int32_t* d_cons,
                           const uint32_t* d_score, const uint8_t* d_is_key, int64_t n_items,
                           const int64_t* q_ptr, int64_t B, const int32_t* seeds, int k,
                           int32_t* out_ids, int32_t* out_n, bool narrow) {
  if (B <= 0) return false;
  const auto t0 = std::chrono::steady_clock::now();
  const int64_t ns = q_ptr[B] - q_ptr[0];
  KMLS_CHECK(2 * (B + 1) + ns <= kern::kServeLoopStage, "serve loop: request past the stage");
  KMLS_CHECK(B * (int64_t)(k + 1) <= kern::kServeLoopOut, "serve loop: answers past the slot");
  volatile kern::ServeSlot* m = &((volatile kern::ServeMail*)mail_)->slot[slot];
  kern::ServeSlot* mw = &((kern::ServeMail*)mail_)->slot[slot];
  int64_t* hq = reinterpret_cast<int64_t*>(mw->payload);
  int32_t* hs = mw->payload + 2 * (B + 1);
  int32_t* ho = buf_ + (size_t)slot * kern::kServeLoopOut;
  for (int64_t i = 0; i <= B; ++i) hq[i] = q_ptr[i] - q_ptr[0];
  std::copy(seeds + q_ptr[0], seeds + q_ptr[B], hs);
  int32_t* dev = nullptr;
  KMLS_HIP(hipHostGetDevicePointer((void**)&dev, buf_, 0));
  kern::ServeReq rq;
  rq.row_ptr = d_row_ptr;
  rq.cons = d_cons;
  rq.srank = d_score;
  rq.is_key = d_is_key;
  rq.n_items = n_items;
  rq.q_ptr = nullptr;  // inline: staged from the mailbox
  rq.seeds = nullptr;
  rq.out = dev + (size_t)slot * kern::kServeLoopOut;
  rq.B = B;
  rq.k = k;
  rq.n_seeds = ns;
  rq.narrow = narrow ? 1 : 0;
  std::memcpy((void*)&m->req_desc, &rq, sizeof rq);
  for (int64_t i = 0; i < B; ++i) ho[i * (k + 1)] = -3;  // (never a real answer)
  unsigned gen;
  {
    std::lock_guard<std::mutex> lk(launch_mu_);
    gen = ensure_running_locked();
  }
  if (gen == 0) {  // paused
    std::lock_guard<std::mutex> sl(stats_mu_);
    ++st_.refused;
    return false;
  }
  const unsigned seq = ++seq_[slot];
  std::atomic_thread_fence(std::memory_order_seq_cst);  // descriptor and payload before the word
  m->req = ((unsigned long long)(2 * (B + 1) + ns) << 32) | (unsigned long long)seq;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  // wait for the done word.  The launch can leave without serving it (its idle exit raced the
  // request, or a pause stopped it): then relaunch (the new launch serves the pending word) or,
  // paused, mark it consumed and refuse.
  const auto t_start = std::chrono::steady_clock::now();
  for (unsigned n = 0;; ++n) {
    if (m->done_seq == seq) break;
    if ((n & 255u) == 255u) {
      if (m->exited_gen == gen) {
        std::lock_guard<std::mutex> lk(launch_mu_);
        if (m->done_seq != seq) {
          if (gen_ == gen) {
            gen = ensure_running_locked();  // 0: paused (the kernel is stopped)
          } else {
            gen = (launched_ && paused_ == 0) ? gen_ : 0u;
          }
          if (gen == 0) {
            if (launched_) stop_and_wait_locked();
            consume_locked(slot, seq);
            std::lock_guard<std::mutex> sl(stats_mu_);
            ++st_.refused;
            return false;
          }
        }
      }
      if (std::chrono::steady_clock::now() - t_start > std::chrono::milliseconds(500)) {
        std::lock_guard<std::mutex> lk(launch_mu_);
        if (m->done_seq != seq) {
          stop_and_wait_locked();  // lost: no kernel runs now; the next request relaunches
          if (m->done_seq != seq) consume_locked(slot, seq);
          std::lock_guard<std::mutex> sl(stats_mu_);
          ++st_.refused;
          return false;
        }
      }
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_seq_cst);
  for (int64_t b = 0; b < B; ++b) {
    const int32_t n = ho[b * (k + 1)];
    out_n[b] = n;
    for (int j = 0; j < k; ++j) out_ids[b * k + j] = (j < n) ? ho[b * (k + 1) + 1 + j] : -1;
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  std::lock_guard<std::mutex> sl(stats_mu_);
  st_.kernel_us += (double)(m->t_done - m->t_seen) / ticks_per_us_;
  st_.stage_us += (double)(m->t_staged - m->t_seen) / ticks_per_us_;
  st_.compute_us += (double)(m->t_computed - m->t_staged) / ticks_per_us_;
  for (int i = 0; i < 4; ++i)
    st_.phase_us[i] += (double)(m->t_phase[i + 1] - m->t_phase[i]) / ticks_per_us_;
  ++st_.requests;
  st_.queries += (uint64_t)B;
  st_.last_us = us;
  st_.sum_us += us;
  return true;
}

int64_t GpuRuleIndex::merged_size(const int32_t* seeds, int64_t n) const {
  int64_t acc = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t sd = seeds[i];
    if (sd >= 0 && sd < n_items_ && h_is_key_[(size_t)sd])
      acc += h_row_ptr_[(size_t)sd + 1] - h_row_ptr_[(size_t)sd];
  }
  return acc;
}

bool GpuRuleIndex::query_loop(const int64_t* q_ptr, int64_t B, const int32_t* seeds, int k,
                              int32_t* out_ids, int32_t* out_n) {
  KMLS_CHECK(k >= 0 && k <= 256, "query_loop: 0 <= k <= 256");
  return GpuServeLoop::for_device(device_).run(d_row_ptr_, d_cons_, d_score_, d_is_key_, n_items_,
                                               q_ptr, B, seeds, k, out_ids, out_n, narrow_);
}

GpuRuleIndex::GpuRuleIndex(int device, const RuleIndex& host, uintptr_t stream)
    : device_(device), n_items_(host.n_items()), nnz_(host.nnz()) {
  KMLS_HIP(hipSetDevice(device));
  ServeLoopPause pause(device);  // allocation calls must not wait behind the serving kernel
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
  // merged order keys fit 32 bits (serve_query_wave); test hook serve_wide=1 keeps 64-bit keys
  narrow_ = uniq.size() + 2 < (1u << 23) && test_hook("serve_wide", 0) == 0;
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
  ServeLoopPause pause(device_);  // (frees must not wait behind the serving kernel)
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
                         dev + 2 * (B + 1), B, k, dout, s, narrow_);
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
