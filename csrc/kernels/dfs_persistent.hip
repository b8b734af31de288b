// Persistent device-driven DFS over equivalence classes (all levels >= 3 in ONE launch).
//
// The level-wise driver (miner_gpu.hip) pays a host readback + ~7 launches per level chunk; on
// the reference's ds2-shaped data the class tree is 14 levels deep with ~10^5-10^6 tiny
// classes, so that path is latency-bound (SURVEY §7.7 hard part 3).  Here each wave64 of a
// resident grid runs its own depth-first search:
//
//   frame     = class members' bitmaps/ranks/gids + class size n + itemset size + next row a
//               (+ row limit a1), kept on a per-wave LDS stack (kStack frames).
//   expand a  = for b in (a, n): popcount(bits(a) & bits(b)) by TS-lane teams; pass 1 counts
//               survivors (ballot), S rows are carved from the wave's private row chunk, pass 2
//               recomputes and writes child bitmaps + trie-node records.  The child class of a
//               (S >= 2) is pushed on the LOCAL stack (depth-first, no global traffic) ...
//   share     = ... unless another wave is idle (`idle` counter, sampled every 16 rows) or the
//               local stack is full: then it is published to the global queue, split into row
//               ranges of <= kTaskCands candidates.
//   coherence = FENCE-FREE (cdna_hip_programming.md §6 G16, the sc1 form of recipe R1): every
//               pool write (child bitmaps, ranks, gids, task records) is a write-through sc1
//               store; a wave drains them (s_waitcnt vmcnt(0)) before raising a slot flag (sc1
//               store); a consumer polls the flag with sc1 loads and reads a POPPED class with
//               sc1 loads only.  Classes a wave produced itself are read with plain 16-B loads
//               (same wave, same XCD L2).  Agent-scope fences would write back / invalidate the
//               whole XCD L2 per task — the first version of this kernel spent 97% of its time
//               there.  Row chunks are 16-row aligned so no 128-B line holds rows of two
//               writers.
//   rows      = each wave reserves 256-row chunks from one counter (1 atomic per chunk, not per
//               class); unused chunk tails leave holes (depth 0) that a scan + scatter pass
//               removes afterwards, remapping parent ids (dfs_compact).
//   terminate = `pending` counts published-but-unretired tasks; a task is retired only when the
//               wave's local stack for it is empty, and shared children are counted before they
//               are published, so pending == 0 ⇔ no work can ever appear again.  Every spin is
//               bounded (clock + poll count) and a host watchdog can raise a mapped abort flag.
//   overflow  = row/task capacity exhausted → flag; the host falls back to the level-wise path
//               (exact), so capacity only affects speed.
// Hot counters live on separate 128-byte lines; per-wave statistics are reduced in registers.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>
#include <stdexcept>
#include <string>

#include "kernels.hpp"

namespace kmls {
namespace kern {

namespace {

constexpr int kWaves = 4;          // waves per workgroup
constexpr int kStack = 24;         // local DFS frames per wave
constexpr int kTaskCands = 4096;   // max candidates per shared task (row-range split)
constexpr unsigned kRowChunk = 256;

__device__ __forceinline__ unsigned long long ld_relaxed(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned int ld_relaxed(const unsigned int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned int* p, unsigned int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Task records as 5 x 8-byte words (sc1 stores / loads).
__device__ __forceinline__ void store_task(DfsTask* t, const DfsTask& v) {
  unsigned long long* w = reinterpret_cast<unsigned long long*>(t);
  st_sc1(w + 0, (unsigned long long)v.bm);
  st_sc1(w + 1, (unsigned long long)v.rank);
  st_sc1(w + 2, (unsigned long long)v.gid);
  st_sc1(w + 3, (unsigned long long)(unsigned)v.n | ((unsigned long long)(unsigned)v.depth << 32));
  st_sc1(w + 4, (unsigned long long)(unsigned)v.a0 | ((unsigned long long)(unsigned)v.a1 << 32));
}
__device__ __forceinline__ DfsTask load_task(const DfsTask* t) {
  const unsigned long long* w = reinterpret_cast<const unsigned long long*>(t);
  DfsTask v;
  v.bm = (const unsigned long long*)ld_sc1(w + 0);
  v.rank = (const int32_t*)ld_sc1(w + 1);
  v.gid = (const int64_t*)ld_sc1(w + 2);
  const unsigned long long nd = ld_sc1(w + 3), aa = ld_sc1(w + 4);
  v.n = (int32_t)(unsigned)(nd & 0xFFFFFFFFu);
  v.depth = (int32_t)(unsigned)(nd >> 32);
  v.a0 = (int32_t)(unsigned)(aa & 0xFFFFFFFFu);
  v.a1 = (int32_t)(unsigned)(aa >> 32);
  return v;
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
  if (cx.wave_state != nullptr && lane == 0) {
    __hip_atomic_store(&cx.wave_state[4 * gw + 0], st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cx.wave_state[4 * gw + 1], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cx.wave_state[4 * gw + 2], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cx.wave_state[4 * gw + 3], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ int count_tasks(int n) {
  int n_tasks = 0;
  long long acc = 0;
  for (int a = 0; a < n - 1; ++a) {
    const long long m = n - a - 1;
    if (acc > 0 && acc + m > kTaskCands) { ++n_tasks; acc = 0; }
    acc += m;
  }
  return n_tasks + (acc > 0 ? 1 : 0);
}

// Publish a class to the global queue as row-range tasks.  Lane 0 only; the payload (child
// bitmaps, ranks, gids) was written by this wave before the call.  Returns false on overflow.
__device__ bool share_class(const Ctx& cx, const unsigned long long* bm, const int32_t* rank,
                            const int64_t* gid, int n, int depth) {
  const int n_tasks = count_tasks(n);
  if (n_tasks == 0) return true;
  atomicAdd(&cx.ctl->pending, (unsigned long long)n_tasks);
  const unsigned long long base = atomicAdd(&cx.ctl->q_tail, (unsigned long long)n_tasks);
  if (base + n_tasks > (unsigned long long)cx.task_cap) {
    atomicOr(&cx.ctl->overflow, 2u);
    atomicAdd(&cx.ctl->pending, (unsigned long long)(-(long long)n_tasks));
    return false;
  }
  int t = 0, a0 = 0;
  long long acc = 0;
  for (int a = 0; a < n - 1; ++a) {
    const long long m = n - a - 1;
    if (acc > 0 && acc + m > kTaskCands) {
      store_task(&cx.tasks[base + t], DfsTask{bm, rank, gid, n, depth, a0, a});
      ++t; a0 = a; acc = 0;
    }
    acc += m;
  }
  store_task(&cx.tasks[base + t], DfsTask{bm, rank, gid, n, depth, a0, n - 1});
  // payload (written through by the whole wave before this call) + records are performed
  // once this wave's vmcnt drains; then the flags
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int i = 0; i < n_tasks; ++i) st_sc1(&cx.ready[base + i], 1u);
  return true;
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
__device__ __forceinline__ uint32_t team_and_popcount_sc1(const unsigned long long* x,
                                                          const unsigned long long* y,
                                                          int64_t Wp, int tl) {
  uint32_t s = 0;
  for (int64_t w = tl; w < Wp; w += TS) s += (uint32_t)__popcll(ld_sc1(x + w) & ld_sc1(y + w));
#pragma unroll
  for (int off = TS >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, TS);
  return s;
}

struct WaveState {  // per-wave registers (uniform)
  unsigned long long row_next, row_end;  // private row chunk [row_next, row_end)
  unsigned long long cands;
  unsigned max_depth;
  unsigned rows_since_probe;
  bool share_hint;
  bool dead;                             // overflow: stop producing
};

// Expand row a of frame f.  Returns (row0, S) of the child class (S = 0: none).  REMOTE frames
// (popped from the queue) read their class through sc1 loads; local frames with plain loads.
template <int TS, bool REMOTE>
__device__ void expand_row(const Ctx& cx, const DfsTask& f, int a, int lane, WaveState& ws,
                           unsigned long long& row0_out, unsigned& S_out) {
  constexpr int TPW = 64 / TS;
  constexpr unsigned long long kLeaders = [] {
    unsigned long long m = 0;
    for (int i = 0; i < 64; i += TS) m |= 1ull << i;
    return m;
  }();
  const int tl = lane & (TS - 1);
  const int team = lane / TS;
  const int64_t Wp = cx.Wp, n2 = Wp >> 1;
  const int n = f.n;
  const unsigned long long* xa8 = f.bm + (int64_t)a * Wp;
  const ulonglong2* xa = reinterpret_cast<const ulonglong2*>(xa8);
  auto pc = [&](int b) -> uint32_t {
    const unsigned long long* y8 = f.bm + (int64_t)b * Wp;
    if constexpr (REMOTE) return team_and_popcount_sc1<TS>(xa8, y8, Wp, tl);
    else return team_and_popcount<TS>(xa, reinterpret_cast<const ulonglong2*>(y8), n2, tl);
  };
  unsigned S = 0;
  for (int g = a + 1; g < n; g += TPW) {  // pass 1
    const int b = g + team;
    uint32_t c = 0;
    if (b < n) c = pc(b);
    S += (unsigned)__popcll(__ballot((b < n) && c >= cx.minsup) & kLeaders);
  }
  ws.cands += (unsigned long long)(n - a - 1);
  S_out = 0;
  if (S == 0 || ws.dead) return;
  // carve S contiguous rows from the private chunk (refill: 1 atomic per chunk; chunks are
  // multiples of 16 rows so chunk boundaries are 128-byte aligned in every pool array)
  if (ws.row_next + S > ws.row_end) {
    unsigned take = S > kRowChunk ? S : kRowChunk;
    take = (take + 31u) & ~31u;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&cx.ctl->row_top, (unsigned long long)take);
    base = __shfl(base, 0);
    if (base + take > (unsigned long long)cx.row_cap) {
      if (lane == 0) atomicOr(&cx.ctl->overflow, 1u);
      ws.dead = true;
      return;
    }
    ws.row_next = base;
    ws.row_end = base + take;
  }
  const unsigned long long row0 = ws.row_next;
  ws.row_next += S;
  unsigned j0 = 0;
  int64_t gid_a;
  if constexpr (REMOTE) gid_a = (int64_t)ld_sc1(reinterpret_cast<const unsigned long long*>(f.gid + a));
  else gid_a = f.gid[a];
  const uint8_t dchild = (uint8_t)(f.depth + 1);
  for (int g = a + 1; g < n; g += TPW) {  // pass 2
    const int b = g + team;
    uint32_t c = 0;
    if (b < n) c = pc(b);
    const bool pass = (b < n) && c >= cx.minsup;
    const unsigned long long bal = __ballot(pass) & kLeaders;
    if (pass) {
      const int leader = lane - tl;
      const int64_t row = (int64_t)row0 + j0 + (unsigned)__popcll(bal & ((1ull << leader) - 1ull));
      const unsigned long long* y8 = f.bm + (int64_t)b * Wp;
      unsigned long long* z = cx.pool_bm + row * Wp;
      for (int64_t w = tl; w < Wp; w += TS) {  // write-through child bitmap
        unsigned long long u, v;
        if constexpr (REMOTE) { u = ld_sc1(xa8 + w); v = ld_sc1(y8 + w); }
        else { u = xa8[w]; v = y8[w]; }
        st_sc1(z + w, u & v);
      }
      if (tl == 0) {
        // frames carry ORIGINAL item ids (seeds are converted once by k_seed_items)
        int32_t ib;
        if constexpr (REMOTE)
          ib = (int32_t)__hip_atomic_load(f.rank + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else ib = f.rank[b];
        st_sc1(reinterpret_cast<unsigned int*>(cx.pool_rank + row), (unsigned)ib);
        st_sc1(reinterpret_cast<unsigned long long*>(cx.pool_gid + row),
               (unsigned long long)(cx.out_base + row));
        cx.out_parent[cx.out_base + row] = gid_a;
        cx.out_item[cx.out_base + row] = ib;
        cx.out_count[cx.out_base + row] = c;
        cx.out_depth[cx.out_base + row] = dchild;
      }
    }
    j0 += (unsigned)__popcll(bal);
  }
  if (dchild > ws.max_depth) ws.max_depth = dchild;
  row0_out = row0;
  S_out = S;
}

template <int TS>
__global__ __launch_bounds__(64 * kWaves) void k_dfs_persistent(Ctx cx) {
  __shared__ DfsTask stack_all[kWaves][kStack];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  DfsTask* stack = stack_all[wid];
  const unsigned long long t_start = wall_clock64();
  unsigned long long polls = 0;
  WaveState ws{0, 0, 0, 0, 0, false, false};
  while (true) {
    // ---- get a task from the global queue -------------------------------------------------
    unsigned long long idx = 0;
    if (lane == 0) {
      idx = atomicAdd(&cx.ctl->q_head, 1ull);
      atomicAdd(&cx.ctl->idle, 1u);
    }
    idx = __shfl(idx, 0);
    crumb(cx, gw, lane, 1u, (unsigned)idx, 0u, 0u);
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
    if (lane == 0) atomicSub(&cx.ctl->idle, 1u);
    if (!got) break;
    const DfsTask root = load_task(&cx.tasks[idx]);
    crumb(cx, gw, lane, 2u, (unsigned)idx, (unsigned)root.n, (unsigned)root.a1);
    if (root.n < 2 || root.n > (1 << 24) || root.a0 < 0 || root.a1 > root.n - 1 ||
        root.a0 > root.a1 || root.bm == nullptr) {
      if (lane == 0) atomicOr(&cx.ctl->bad_task, 1u);
    } else {
      // ---- local depth-first search rooted at the task ----------------------------------
      // The stack is wave-private LDS: lane 0 writes a frame, every lane reads it after the
      // wave barrier (LDS ops of one wave complete in order, the barrier orders the compiler).
      if (lane == 0) stack[0] = root;
      int top = 1;  // stack[0] is the popped (remote) class, deeper frames are local
      bool aborted = false;
      while (top > 0 && !aborted) {
        __builtin_amdgcn_wave_barrier();
        const DfsTask f = stack[top - 1];
        __builtin_amdgcn_wave_barrier();
        if (f.a0 >= f.a1) { --top; continue; }
        const int a = f.a0;
        if (lane == 0) stack[top - 1].a0 = a + 1;
        if (++ws.rows_since_probe >= 4) {
          ws.rows_since_probe = 0;
          int probe = 0;
          if (lane == 0) {
            probe = ld_relaxed(&cx.ctl->idle) > 0u ? 1 : 0;
            if (host_abort(cx)) probe = 2;
          }
          probe = __shfl(probe, 0);
          if (probe == 2) {
            aborted = true;
            if (lane == 0) atomicOr(&cx.ctl->aborted, 1u);
            break;
          }
          if (probe == 1 && lane == 0) {
            // work splitting: give away the upper half (by candidates) of the remaining rows of
            // the OLDEST frame that still has >= 2 rows — the largest pending subtrees.  Its
            // class data is already performed in memory (written through + drained before the
            // frame was pushed, or published by another wave).
            for (int i = 0; i < top; ++i) {
              const DfsTask& bf = stack[i];
              const int lo = (i == top - 1) ? a + 1 : bf.a0;
              if (bf.a1 - lo < 2) continue;
              long long total = 0;
              for (int r = lo; r < bf.a1; ++r) total += bf.n - 1 - r;
              long long acc = 0;
              int mid = lo;
              while (mid < bf.a1 - 1 && 2 * (acc + (bf.n - 1 - mid)) <= total) {
                acc += bf.n - 1 - mid;
                ++mid;
              }
              if (mid <= lo) mid = lo + 1;
              const unsigned long long slot = [&] {
                atomicAdd(&cx.ctl->pending, 1ull);
                return atomicAdd(&cx.ctl->q_tail, 1ull);
              }();
              if (slot >= (unsigned long long)cx.task_cap) {
                atomicOr(&cx.ctl->overflow, 2u);
                atomicAdd(&cx.ctl->pending, (unsigned long long)(-1ll));
                break;
              }
              store_task(&cx.tasks[slot], DfsTask{bf.bm, bf.rank, bf.gid, bf.n, bf.depth, mid, bf.a1});
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              st_sc1(&cx.ready[slot], 1u);
              stack[i].a1 = mid;
              break;
            }
          }
        }
        unsigned long long row0 = 0;
        unsigned S = 0;
        if (top == 1) expand_row<TS, true>(cx, f, a, lane, ws, row0, S);
        else expand_row<TS, false>(cx, f, a, lane, ws, row0, S);
        if (S >= 2 && (cx.max_len == 0 || f.depth + 1 < cx.max_len)) {
          const unsigned long long* cbm = cx.pool_bm + row0 * cx.Wp;
          const int32_t* crk = cx.pool_rank + row0;
          const int64_t* cgd = cx.pool_gid + row0;
          // child rows were written through by this wave (cross-lane): drain before they are
          // read back locally or handed to another wave
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (top >= kStack) {
            int ok = 1;
            if (lane == 0) ok = share_class(cx, cbm, crk, cgd, (int)S, f.depth + 1) ? 1 : 0;
            ok = __shfl(ok, 0);
            if (!ok) ws.dead = true;
          } else {
            if (lane == 0) stack[top] = DfsTask{cbm, crk, cgd, (int)S, f.depth + 1, 0, (int)S - 1};
            ++top;
          }
        }
      }
    }
    crumb(cx, gw, lane, 3u, (unsigned)idx, 0u, 0u);
    if (lane == 0) atomicAdd(&cx.ctl->pending, (unsigned long long)(-1ll));
  }
  crumb(cx, gw, lane, 9u, 0u, 0u, 0u);
  if (lane == 0) {
    atomicAdd(&cx.ctl->candidates, ws.cands);
    atomicMax(&cx.ctl->max_depth, ws.max_depth);
    atomicAdd(&cx.ctl->exited, 1u);
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
    const int n_tasks = count_tasks(n);
    atomicAdd(&ctl->pending, (unsigned long long)n_tasks);
    const unsigned long long base = atomicAdd(&ctl->q_tail, (unsigned long long)n_tasks);
    if (base + n_tasks > (unsigned long long)task_cap) {
      atomicOr(&ctl->overflow, 2u);
      atomicAdd(&ctl->pending, (unsigned long long)(-(long long)n_tasks));
      continue;
    }
    const unsigned long long* cbm = bm + s * Wp;
    int t = 0, a0 = 0;
    long long acc = 0;
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

// frames carry original item ids: convert the seed level's Eclat ranks once
__global__ void k_seed_items(const int32_t* __restrict__ rank, const int32_t* __restrict__ ids,
                             int64_t n, int32_t* __restrict__ out) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr) out[i] = ids[rank[i]];
}

// ---- hole compaction + topological order ---------------------------------------------------
// Rows come from per-wave chunks, so a child row may precede its parent row.  Sorting the DFS
// region stably by depth (holes = depth 0 sort first) restores "parents before children" (the
// trie invariant every consumer relies on); rows are then scattered with parents remapped.
__global__ void k_iota(int64_t* __restrict__ v, int64_t n) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr) v[i] = i;
}

__global__ void k_count_zero(const uint8_t* __restrict__ keys, int64_t n,
                             unsigned long long* __restrict__ out) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr)
    c += keys[i] == 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

__global__ void k_inverse(const int64_t* __restrict__ sorted_rows, int64_t n,
                          const unsigned long long* __restrict__ holes, int64_t* __restrict__ inv) {
  const int64_t H = (int64_t)*holes;
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = H + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr)
    inv[sorted_rows[i]] = i - H;
}

__global__ void k_dfs_scatter(const int64_t* __restrict__ sorted_rows, int64_t n,
                              const unsigned long long* __restrict__ holes,
                              const int64_t* __restrict__ inv, int64_t out_base,
                              const int64_t* __restrict__ par, const int32_t* __restrict__ item,
                              const uint32_t* __restrict__ cnt, const uint8_t* __restrict__ dep,
                              int64_t* __restrict__ par2, int32_t* __restrict__ item2,
                              uint32_t* __restrict__ cnt2, uint8_t* __restrict__ dep2) {
  const int64_t H = (int64_t)*holes;
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = H + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr) {
    const int64_t r = sorted_rows[i], k = i - H;
    int64_t p = par[r];
    if (p >= out_base) p = out_base + inv[p - out_base];  // parent inside the DFS region
    par2[k] = p;
    item2[k] = item[r];
    cnt2[k] = cnt[r];
    dep2[k] = dep[r];
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

void check(hipError_t e) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e));
}

}  // namespace

void dfs_persistent(const DfsArgs& a, hipStream_t s) {
  Ctx cx{a.tasks, a.ready, a.ctl, (unsigned long long*)a.pool_bm, a.pool_rank, a.pool_gid,
         a.out_parent, a.out_item, a.out_count, a.out_depth, a.ids, a.out_base, a.Wp, a.row_cap,
         a.task_cap, a.minsup, a.max_len, a.timeout_ticks, a.abort_flag, a.wave_state};
  const int64_t nr = a.seed_rows;
  const int sg = (int)std::min<int64_t>(std::max<int64_t>((nr + 255) / 256, 1), 4096);
  hipLaunchKernelGGL(k_seed_items, dim3(sg), dim3(256), 0, s, a.seed_rank, a.ids, nr, a.seed_items);
  hipLaunchKernelGGL(k_dfs_seed, dim3(sg), dim3(256), 0, s, (const unsigned long long*)a.seed_bm,
                     a.seed_items, a.seed_gid, a.seed_row_end, nr, a.Wp, a.seed_depth, a.tasks,
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
  check(hipGetLastError());
}

size_t dfs_compact_temp_bytes(int64_t rows) {
  size_t bytes = 0;
  check(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint8_t*)nullptr,
                                           (uint8_t*)nullptr, (const int64_t*)nullptr,
                                           (int64_t*)nullptr, (int)std::max<int64_t>(rows, 1), 0, 8));
  // + keys_out (rows) + vals_in/vals_out/inv (3 * rows * 8) + holes counter, 256-B aligned parts
  return bytes + 256 + ((size_t)rows + 256) + 3 * ((size_t)rows * 8 + 256) + 256;
}

int64_t dfs_compact(int64_t rows, int64_t out_base, int64_t* par, int32_t* item, uint32_t* cnt,
                    uint8_t* dep, void* temp, size_t temp_bytes, int64_t* par2, int32_t* item2,
                    uint32_t* cnt2, uint8_t* dep2, unsigned long long* h_holes, hipStream_t s) {
  size_t sort_bytes = 0;
  check(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint8_t*)nullptr,
                                           (uint8_t*)nullptr, (const int64_t*)nullptr,
                                           (int64_t*)nullptr, (int)rows, 0, 8));
  char* p = (char*)temp;
  auto carve = [&](size_t n) { char* q = p; p += (n + 255) & ~(size_t)255; return q; };
  void* sort_tmp = carve(sort_bytes);
  uint8_t* keys_out = (uint8_t*)carve((size_t)rows);
  int64_t* vals_in = (int64_t*)carve((size_t)rows * 8);
  int64_t* vals_out = (int64_t*)carve((size_t)rows * 8);
  int64_t* inv = (int64_t*)carve((size_t)rows * 8);
  unsigned long long* holes = (unsigned long long*)carve(8);
  if ((size_t)(p - (char*)temp) > temp_bytes) throw std::runtime_error("kmls: dfs_compact temp");
  const int g = (int)std::min<int64_t>(std::max<int64_t>((rows + 255) / 256, 1), 8192);
  hipLaunchKernelGGL(k_iota, dim3(g), dim3(256), 0, s, vals_in, rows);
  check(hipcub::DeviceRadixSort::SortPairs(sort_tmp, sort_bytes, dep + out_base, keys_out, vals_in,
                                           vals_out, (int)rows, 0, 8, s));
  check(hipMemsetAsync(holes, 0, 8, s));
  hipLaunchKernelGGL(k_count_zero, dim3(std::min(g, 1024)), dim3(256), 0, s, keys_out, rows, holes);
  hipLaunchKernelGGL(k_inverse, dim3(g), dim3(256), 0, s, vals_out, rows, holes, inv);
  hipLaunchKernelGGL(k_dfs_scatter, dim3(g), dim3(256), 0, s, vals_out, rows, holes, inv,
                     out_base, par + out_base, item + out_base, cnt + out_base, dep + out_base,
                     par2, item2, cnt2, dep2);
  check(hipGetLastError());
  check(hipMemcpyAsync(h_holes, holes, 8, hipMemcpyDeviceToHost, s));
  check(hipStreamSynchronize(s));
  return rows - (int64_t)*h_holes;
}

}  // namespace kern
}  // namespace kmls
