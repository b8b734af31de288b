// Persistent device-driven DFS over equivalence classes (levels >= 3 in ONE launch).
//
// The level-wise driver (miner_gpu.hip) pays a host readback + ~7 launches per level chunk; on
// the reference's ds2-shaped data the tree is 14 levels deep with ~1M tiny classes, so that
// path is latency-bound (SURVEY §7.7 hard part 3).  Here every wave64 of a resident grid runs
// a loop: pop a task from a device work queue, expand it, push the child classes.
//
//   task      = (class members' bitmaps/ranks/gids, class size n, itemset size, row range
//               [a0,a1) of members to expand); big classes are split into row ranges so that a
//               task holds <= kTaskCands candidates.
//   expand a  = for b in (a, n): cnt = popcount(bits(a) & bits(b)) by TS-lane teams;
//               pass 1 counts survivors (ballot), one atomicAdd reserves S rows (= S trie
//               nodes), pass 2 recomputes and writes child bitmaps + node records, the child
//               class of a (S >= 2) is pushed as new task(s).
//   publish   = producer wave: plain stores of payload → s_waitcnt vmcnt(0) → agent-scope
//               release fence → vmcnt(0) → relaxed agent atomic store of the slot's ready flag
//               (cdna_hip_programming.md §6 Guideline 16, recipe R1).
//   consume   = lane 0 polls the flag relaxed (s_sleep back-off); whole wave executes an
//               agent-scope acquire fence; then plain loads.
//   terminate = `pending` counts published-but-unfinished tasks (children are added before the
//               parent is retired), so pending == 0 ⇔ no task can ever appear again.  Every spin
//               is bounded by a wall-clock timeout that sets an error flag.
//   overflow  = row or task capacity exceeded → flag; the host re-runs with 4x capacity (the
//               result is recomputed from scratch, so it stays exact).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "kernels.hpp"

namespace kmls {
namespace kern {

namespace {

constexpr int kWaves = 4;             // waves per workgroup
constexpr int kTaskCands = 4096;      // max candidates per task (row-range split)

__device__ __forceinline__ unsigned long long ld_relaxed(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned int ld_relaxed(const unsigned int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Ctx {
  DfsTask* tasks;
  unsigned int* ready;
  DfsCtl* ctl;
  unsigned long long* pool_bm;
  int32_t* pool_rank;
  int64_t* pool_gid;
  int64_t* out_parent;
  int32_t* out_item;
  uint32_t* out_count;
  uint8_t* out_depth;
  const int32_t* ids;
  int64_t out_base;
  int64_t Wp;
  int64_t row_cap;
  int64_t task_cap;
  uint32_t minsup;
  int max_len;
  unsigned long long timeout_ticks;
  const unsigned int* abort_flag;
  unsigned int* wave_state;
};

__device__ __forceinline__ bool host_abort(const Ctx& cx) {
  return __hip_atomic_load(cx.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
}

__device__ __forceinline__ void crumb(const Ctx& cx, int gw, int lane, unsigned st, unsigned a,
                                      unsigned b, unsigned c) {
  if (lane == 0 && cx.wave_state) {
    __hip_atomic_store(&cx.wave_state[4 * gw + 0], st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cx.wave_state[4 * gw + 1], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cx.wave_state[4 * gw + 2], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cx.wave_state[4 * gw + 3], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Split a class into row-range tasks and publish them.  Called by ONE wave; lane 0 does the
// bookkeeping (classes larger than a task are rare).  Payload (child bitmaps, ranks, gids) was
// written by this same wave before the call.
__device__ void push_class(const Ctx& cx, const unsigned long long* bm, const int32_t* rank,
                           const int64_t* gid, int n, int depth, int lane) {
  if (lane != 0) return;
  // count tasks
  int n_tasks = 0;
  {
    long long acc = 0;
    for (int a = 0; a < n - 1; ++a) {
      const long long m = n - a - 1;
      if (acc > 0 && acc + m > kTaskCands) { ++n_tasks; acc = 0; }
      acc += m;
    }
    if (acc > 0) ++n_tasks;
  }
  if (n_tasks == 0) return;
  atomicAdd(&cx.ctl->pending, (unsigned long long)n_tasks);
  const unsigned long long base = atomicAdd(&cx.ctl->q_tail, (unsigned long long)n_tasks);
  if (base + n_tasks > (unsigned long long)cx.task_cap) {
    atomicOr(&cx.ctl->overflow, 2u);
    atomicAdd(&cx.ctl->pending, (unsigned long long)(-(long long)n_tasks));
    // slots beyond capacity are never published; waiters exit through pending == 0
    return;
  }
  int t = 0, a0 = 0;
  long long acc = 0;
  for (int a = 0; a < n - 1; ++a) {
    const long long m = n - a - 1;
    if (acc > 0 && acc + m > kTaskCands) {
      cx.tasks[base + t] = DfsTask{bm, rank, gid, n, depth, a0, a};
      ++t; a0 = a; acc = 0;
    }
    acc += m;
  }
  cx.tasks[base + t] = DfsTask{bm, rank, gid, n, depth, a0, n - 1};
  // publish: drain this wave's stores (payload + records), release at agent scope, then flags
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int i = 0; i < n_tasks; ++i)
    __hip_atomic_store(&cx.ready[base + i], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int TS>
__device__ __forceinline__ uint32_t team_and_popcount(const ulonglong2* x, const ulonglong2* y,
                                                      int64_t n2, int tl) {
  uint32_t s = 0;
  for (int64_t w = tl; w < n2; w += TS) {
    const ulonglong2 u = x[w], v = y[w];
    s += (uint32_t)__popcll(u.x & v.x) + (uint32_t)__popcll(u.y & v.y);
  }
#pragma unroll
  for (int off = TS >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, TS);
  return s;
}

template <int TS>
__device__ void expand_task(const Ctx& cx, const DfsTask& tk, int lane) {
  constexpr int TPW = 64 / TS;  // teams per wave
  const int tl = lane & (TS - 1);
  const int team = lane / TS;
  const unsigned long long leader_mask = [] {
    unsigned long long m = 0;
    for (int i = 0; i < 64; i += TS) m |= 1ull << i;
    return m;
  }();
  const int64_t Wp = cx.Wp, n2 = Wp >> 1;
  const int n = tk.n;
  unsigned long long cands = 0;
  for (int a = tk.a0; a < tk.a1; ++a) {
    int ab = 0;
    if (lane == 0) ab = host_abort(cx) ? 1 : 0;
    if (__shfl(ab, 0)) break;
    const ulonglong2* xa = reinterpret_cast<const ulonglong2*>(tk.bm + (int64_t)a * Wp);
    // pass 1: survivor count
    uint32_t S = 0;
    for (int g = a + 1; g < n; g += TPW) {
      const int b = g + team;
      uint32_t c = 0;
      if (b < n) c = team_and_popcount<TS>(xa, reinterpret_cast<const ulonglong2*>(tk.bm + (int64_t)b * Wp), n2, tl);
      const bool pass = (b < n) && c >= cx.minsup;
      S += (uint32_t)__popcll(__ballot(pass) & leader_mask);
    }
    cands += (unsigned long long)(n - a - 1);
    if (S == 0) continue;
    unsigned long long row0 = 0;
    if (lane == 0) row0 = atomicAdd(&cx.ctl->row_top, (unsigned long long)S);
    row0 = __shfl(row0, 0);
    if (row0 + S > (unsigned long long)cx.row_cap) {
      if (lane == 0) atomicOr(&cx.ctl->overflow, 1u);
      continue;
    }
    // pass 2: recompute, compact by ballot prefix, write child rows + trie nodes
    uint32_t j0 = 0;
    const int64_t gid_a = tk.gid[a];
    for (int g = a + 1; g < n; g += TPW) {
      const int b = g + team;
      uint32_t c = 0;
      if (b < n) c = team_and_popcount<TS>(xa, reinterpret_cast<const ulonglong2*>(tk.bm + (int64_t)b * Wp), n2, tl);
      const bool pass = (b < n) && c >= cx.minsup;
      const unsigned long long bal = __ballot(pass) & leader_mask;
      const int leader = lane - tl;
      const uint32_t j = j0 + (uint32_t)__popcll(bal & ((1ull << leader) - 1ull));
      if (pass) {
        const int64_t row = (int64_t)row0 + j;
        const ulonglong2* yb = reinterpret_cast<const ulonglong2*>(tk.bm + (int64_t)b * Wp);
        ulonglong2* z = reinterpret_cast<ulonglong2*>(cx.pool_bm + row * Wp);
        for (int64_t w = tl; w < n2; w += TS) {
          const ulonglong2 u = xa[w], v = yb[w];
          z[w] = make_ulonglong2(u.x & v.x, u.y & v.y);
        }
        if (tl == 0) {
          const int32_t rb = tk.rank[b];
          cx.pool_rank[row] = rb;
          cx.pool_gid[row] = cx.out_base + row;
          cx.out_parent[cx.out_base + row] = gid_a;
          cx.out_item[cx.out_base + row] = cx.ids[rb];
          cx.out_count[cx.out_base + row] = c;
          cx.out_depth[cx.out_base + row] = (uint8_t)(tk.depth + 1);
        }
      }
      j0 += (uint32_t)__popcll(bal);
    }
    if (lane == 0) atomicMax(&cx.ctl->max_depth, (unsigned int)(tk.depth + 1));
    if (S >= 2 && (cx.max_len == 0 || tk.depth + 1 < cx.max_len))
      push_class(cx, cx.pool_bm + (int64_t)row0 * Wp, cx.pool_rank + row0, cx.pool_gid + row0,
                 (int)S, tk.depth + 1, lane);
  }
  if (lane == 0) atomicAdd(&cx.ctl->candidates, cands);
}

template <int TS>
__global__ __launch_bounds__(64 * kWaves) void k_dfs_persistent(Ctx cx) {
  const int lane = threadIdx.x & 63;
  const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const unsigned long long t_start = wall_clock64();
  unsigned long long polls = 0;
  while (true) {
    unsigned long long idx = 0;
    if (lane == 0) idx = atomicAdd(&cx.ctl->q_head, 1ull);
    idx = __shfl(idx, 0);
    crumb(cx, gw, lane, 1u, (unsigned)idx, 0u, 0u);
    // wait until slot idx is published, or until no task can ever be published again
    // Back-off polling: 2k waves re-reading the hot `ready`/`pending` lines (which producers
    // update with atomics) at full rate starve the producers' atomics; the first version of
    // this loop made no progress at all.  Poll the slot every iteration with a growing sleep,
    // check termination every 8th and the host abort flag / clock every 256th poll.
    bool got = false;
    unsigned it = 0;
    while (true) {
      int st = 0;  // 1 = ready, 2 = terminate
      if (lane == 0) {
        ++polls;
        if (idx < (unsigned long long)cx.task_cap && ld_relaxed(&cx.ready[idx]) != 0u) {
          st = 1;
        } else if ((it & 7u) == 7u && ld_relaxed(&cx.ctl->pending) == 0ull) {
          st = (idx < (unsigned long long)cx.task_cap && ld_relaxed(&cx.ready[idx]) != 0u) ? 1 : 2;
        } else if ((it & 255u) == 255u) {
          if (host_abort(cx)) {
            atomicOr(&cx.ctl->aborted, 1u);
            st = 2;
          } else if (wall_clock64() - t_start > cx.timeout_ticks || polls > (1ull << 26)) {
            atomicOr(&cx.ctl->timeout, 1u);
            st = 2;
          }
        }
      }
      st = __shfl(st, 0);
      if (st == 1) { got = true; break; }
      if (st == 2) break;
      if (it < 16) __builtin_amdgcn_s_sleep(1);
      else if (it < 256) __builtin_amdgcn_s_sleep(8);
      else __builtin_amdgcn_s_sleep(32);
      ++it;
    }
    if (!got) {
      crumb(cx, gw, lane, 9u, (unsigned)idx, 0u, 0u);
      if (lane == 0) atomicAdd(&cx.ctl->exited, 1u);
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const DfsTask tk = cx.tasks[idx];
    crumb(cx, gw, lane, 2u, (unsigned)idx, (unsigned)tk.n, (unsigned)tk.a1);
    if (tk.n < 2 || tk.n > (1 << 24) || tk.a0 < 0 || tk.a1 > tk.n - 1 || tk.a0 > tk.a1 ||
        tk.bm == nullptr) {
      if (lane == 0) atomicOr(&cx.ctl->bad_task, 1u);
    } else {
      expand_task<TS>(cx, tk, lane);
    }
    crumb(cx, gw, lane, 3u, (unsigned)idx, 0u, 0u);
    // retire: children (if any) were added to pending inside expand_task
    if (lane == 0) atomicAdd(&cx.ctl->pending, (unsigned long long)(-1ll));
  }
}

// Seed: every class of the input level (rows [s, row_end[s]) starting where row_end[s-1] == s)
// with >= 2 members becomes task(s).  Runs before the persistent launch (kernel boundary =
// visibility), so it publishes with plain stores.
__global__ void k_dfs_seed(const unsigned long long* __restrict__ bm, const int32_t* __restrict__ rank,
                           const int64_t* __restrict__ gid, const int32_t* __restrict__ row_end,
                           int64_t n_rows, int64_t Wp, int depth, DfsTask* tasks,
                           unsigned int* ready, DfsCtl* ctl, int64_t task_cap) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_rows; s += nthr) {
    if (s > 0 && row_end[s - 1] != s) continue;  // not a class start
    const int n = (int)(row_end[s] - s);
    if (n < 2) continue;
    int n_tasks = 0;
    long long acc = 0;
    for (int a = 0; a < n - 1; ++a) {
      const long long m = n - a - 1;
      if (acc > 0 && acc + m > kTaskCands) { ++n_tasks; acc = 0; }
      acc += m;
    }
    if (acc > 0) ++n_tasks;
    atomicAdd(&ctl->pending, (unsigned long long)n_tasks);
    const unsigned long long base = atomicAdd(&ctl->q_tail, (unsigned long long)n_tasks);
    if (base + n_tasks > (unsigned long long)task_cap) {
      atomicOr(&ctl->overflow, 2u);
      atomicAdd(&ctl->pending, (unsigned long long)(-(long long)n_tasks));
      continue;
    }
    const unsigned long long* cbm = bm + s * Wp;
    int t = 0, a0 = 0;
    acc = 0;
    for (int a = 0; a < n - 1; ++a) {
      const long long m = n - a - 1;
      if (acc > 0 && acc + m > kTaskCands) {
        tasks[base + t] = DfsTask{cbm, rank + s, gid + s, n, depth, a0, a};
        ready[base + t] = 1u;
        ++t; a0 = a; acc = 0;
      }
      acc += m;
    }
    tasks[base + t] = DfsTask{cbm, rank + s, gid + s, n, depth, a0, n - 1};
    ready[base + t] = 1u;
  }
}

int team_size_for(int64_t Wp) {
  const int64_t chunks = Wp >> 1;
  if (chunks >= 128) return 64;
  if (chunks >= 64) return 32;
  if (chunks >= 32) return 16;
  if (chunks >= 12) return 8;
  return 4;
}

}  // namespace

void dfs_persistent(const DfsArgs& a, hipStream_t s) {
  Ctx cx{a.tasks, a.ready, a.ctl, (unsigned long long*)a.pool_bm, a.pool_rank, a.pool_gid,
         a.out_parent, a.out_item, a.out_count, a.out_depth, a.ids, a.out_base, a.Wp, a.row_cap,
         a.task_cap, a.minsup, a.max_len, a.timeout_ticks, a.abort_flag, a.wave_state};
  // seed
  const int64_t nr = a.seed_rows;
  const int sg = (int)std::min<int64_t>(std::max<int64_t>((nr + 255) / 256, 1), 4096);
  hipLaunchKernelGGL(k_dfs_seed, dim3(sg), dim3(256), 0, s, (const unsigned long long*)a.seed_bm,
                     a.seed_rank, a.seed_gid, a.seed_row_end, nr, a.Wp, a.seed_depth, a.tasks,
                     a.ready, a.ctl, a.task_cap);
  // persistent grid: 2 workgroups of 4 waves per CU (resident; no grid barrier is needed)
  const dim3 grid(a.n_cus * 2), block(64 * kWaves);
  switch (team_size_for(a.Wp)) {
    case 4: hipLaunchKernelGGL(k_dfs_persistent<4>, grid, block, 0, s, cx); break;
    case 8: hipLaunchKernelGGL(k_dfs_persistent<8>, grid, block, 0, s, cx); break;
    case 16: hipLaunchKernelGGL(k_dfs_persistent<16>, grid, block, 0, s, cx); break;
    case 32: hipLaunchKernelGGL(k_dfs_persistent<32>, grid, block, 0, s, cx); break;
    default: hipLaunchKernelGGL(k_dfs_persistent<64>, grid, block, 0, s, cx); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace kmls
