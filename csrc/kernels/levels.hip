// Fused, host-sync-free level expansion for the GPU FP-Growth miner (levels >= 2).
//
// The chunked driver (mine.hip + miner_gpu.hip "process") needs the host between every step of a
// level: survivor counts size the child buffers, candidate totals size the next launch.  Here
// every size lives in a device-resident descriptor (FLevel) and every launch is a fixed grid of
// persistent blocks that pull tiles from a ticket counter, so the host enqueues all levels back
// to back and synchronises ONCE per mining call.  ONE kernel per level:
//
//   k_level_count: per 256-candidate tile — decode (a, b) against an LDS window of cand_off,
//     AND+popcount (or a gram lookup at the root), block scan of the survivor flags + decoupled
//     look-back → global survivor index, then materialise survivors (child bitmap, rank, gid,
//     trie append) AND lay out the next level: every survivor's candidate offset, the next
//     level's tile → first-row map, and (last tile) the next level's buffers.
//
// Candidate order ("owner-major"): rows of a class are ordered by DESCENDING frequency rank and
// row b owns the candidates (a, b) with every EARLIER sibling a.  The child (a, b) extends b's
// itemset by a's last item (trie parent = b), so a row's candidate count is its number of earlier
// siblings — known as soon as the survivors before it are: the previous round's separate scan
// kernel (candidates = LATER siblings, known only when the class is complete) folds into the
// count's look-back.  Paths still run from the least to the most frequent item, so the classes
// and candidate totals are those of ascending-frequency Eclat.  The look-back carries a
// segmented-scan state per tile (survivors, next-level candidates, survivors of the open owner,
// see SegAgg), published as three 64-bit words that each carry the epoch and the flag.
//
// Streamed download: the materialise phase also writes each survivor's trie node straight into
// pinned host memory (coalesced PCIe writes), so finished levels reach the host while deeper
// levels run, with no copy kernel or cross-stream event.
//
// Status words pack (epoch:12 | flag:2 | value:50), so publishing needs no fence, and the per-call
// epoch makes re-zeroing the status array unnecessary.  Every spin is bounded: a bug sets
// FCtl::overflow and the host falls back to the chunked path instead of hanging the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
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

constexpr int kBlock = 256;
constexpr int kTile = 256;              // candidates per count tile
constexpr int kWin = 1024;              // LDS cand_off window (rows) per count tile
constexpr unsigned long long kValMask = (1ull << 50) - 1;  // status word payload
constexpr unsigned kEpochMask = 0xFFFu;                     // 12-bit look-back tags
constexpr long long kRowLimit = 1ll << 31;                  // level rows are int32-indexed
constexpr long long kSpinLimit = 1ll << 26;

__device__ __forceinline__ unsigned long long ld_relaxed(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// status word: epoch:12 | flag:2 (1 aggregate, 2 inclusive prefix) | payload:50
__device__ __forceinline__ unsigned long long pack(unsigned epoch, unsigned flag,
                                                   unsigned long long v) {
  return ((unsigned long long)(epoch & kEpochMask) << 52) | ((unsigned long long)flag << 50) |
         (v & kValMask);
}
__device__ __forceinline__ unsigned w_epoch(unsigned long long w) { return (unsigned)(w >> 52); }
__device__ __forceinline__ unsigned w_flag(unsigned long long w) { return (unsigned)(w >> 50) & 3u; }

// Tile aggregate of the segmented scan that lays out the next level (a segment = the survivors
// of one owner row b; segments start at the owner's first candidate, a "head"):
//   S  survivors, C  next-level candidates = sum over survivors of their earlier siblings
//   counted inside this tile's span (a continuing first segment counted from 0), O  survivors
//   since the last head (all S when the tile has no head), F  survivors before the first head
//   (the part of the first segment that continues the previous tile), H  a head is present.
// x ⊕ y (x first) is associative with identity 0; an inclusive prefix needs only (S, C, O).
struct SegAgg {  // S, O, F count rows (< 2^31: level rows are int32-indexed), C candidates
  int32_t S, O, F;
  bool H;
  int64_t C;
};
__device__ __forceinline__ SegAgg seg_cat(const SegAgg& x, const SegAgg& y) {
  SegAgg r;
  r.S = x.S + y.S;
  r.C = x.C + y.C + (int64_t)x.O * y.F;  // y's continuing survivors: x.O more earlier siblings each
  r.O = y.H ? y.O : x.O + y.S;
  r.F = x.H ? x.F : x.S + y.F;
  r.H = x.H || y.H;
  return r;
}
__device__ __forceinline__ SegAgg seg_shfl_xor(const SegAgg& v, int off) {
  SegAgg p;
  p.S = __shfl_xor(v.S, off, 64);
  p.C = __shfl_xor(v.C, off, 64);
  p.O = __shfl_xor(v.O, off, 64);
  p.F = __shfl_xor(v.F, off, 64);
  p.H = __shfl_xor((int)v.H, off, 64) != 0;
  return p;
}
// Two words per tile.  An aggregate fits ONE word (S, O, F <= 256 and C <= 256*255/2: 9+9+9+1+15
// bits), so the common case of the look-back reads one word per predecessor; an inclusive prefix
// spans both, w1 written before w0 and accepted only when both carry the flag.  S and O count
// this level's rows (< 2^31: rows are int32-indexed; 31 bits each) but C, the NEXT level's
// candidate total, is quadratic in the survivors per class: it gets 38 bits and saturates
// there, so a prefix past the limit reads as >= 2^31 and the last tile's capacity guard
// (Ct >= 2^31 -> overflow 4 -> chunked path) fires instead of accepting wrapped offsets.
// (Round 3 packed S / O in 28 bits with 16-bit tags: config 2 at max_len 4 overflowed.)
__device__ __forceinline__ void seg_publish(unsigned long long* my, unsigned e, unsigned flag,
                                            const SegAgg& v) {
  if (flag == 1) {
    st_relaxed(my, pack(e, 1, (unsigned long long)v.S | ((unsigned long long)v.O << 9) |
                                  ((unsigned long long)v.F << 18) | ((unsigned long long)v.H << 27) |
                                  ((unsigned long long)v.C << 28)));
  } else {
    const unsigned long long o = (unsigned long long)v.O;
    const unsigned long long c = v.C >= (1ll << 38) ? (1ull << 38) - 1 : (unsigned long long)v.C;
    st_relaxed(my + 1, pack(e, 2, c | ((o >> 19) << 38)));
    st_relaxed(my, pack(e, 2, (unsigned long long)v.S | ((o & 0x7FFFFull) << 31)));
  }
}
__device__ __forceinline__ bool seg_valid(unsigned long long w0, unsigned long long w1, unsigned e) {
  const unsigned f = w_flag(w0);
  return w_epoch(w0) == e && f != 0 && (f == 1 || (w_epoch(w1) == e && w_flag(w1) == 2));
}
__device__ __forceinline__ SegAgg seg_decode(unsigned long long w0, unsigned long long w1) {
  SegAgg v;
  const unsigned long long x = w0 & kValMask;
  if (w_flag(w0) == 1) {
    v.S = (int32_t)(x & 0x1FFull);
    v.O = (int32_t)((x >> 9) & 0x1FFull);
    v.F = (int32_t)((x >> 18) & 0x1FFull);
    v.H = (x >> 27) & 1ull;
    v.C = (int64_t)(x >> 28);
  } else {
    const unsigned long long y = w1 & kValMask;
    v.S = (int32_t)(x & 0x7FFFFFFFull);
    v.O = (int32_t)((x >> 31) | ((y >> 38) << 19));
    v.F = 0;
    v.H = true;
    v.C = (int64_t)(y & 0x3FFFFFFFFFull);
  }
  return v;
}
// fold of the 64 lanes' values, the higher lane (older tile) always the left operand (an xor
// butterfly: every lane ends with the whole fold)
__device__ __forceinline__ SegAgg wave_fold(SegAgg v) {
  const int lane = threadIdx.x & 63;
#pragma unroll 1
  for (int off = 1; off < 64; off <<= 1) {
    const SegAgg p = seg_shfl_xor(v, off);
    v = (lane & off) ? seg_cat(v, p) : seg_cat(p, v);
  }
  return v;
}

// Wave-parallel decoupled look-back for tile t (called by all 64 lanes of wave 0): each round
// inspects 64 predecessors at once (lane 0 = nearest), folds them up to the nearest inclusive
// prefix, and only spins while one of those is unpublished or half-written.  Returns the tile's
// exclusive prefix (every lane).
__device__ SegAgg lookback_seg(unsigned long long* st, int64_t t, unsigned epoch, const SegAgg& agg,
                               FCtl* ctl) {
  const unsigned e = epoch & kEpochMask;
  const int lane = threadIdx.x & 63;
  unsigned long long* my = st + 2 * t;
  const SegAgg zero{0, 0, 0, false, 0};
  if (t == 0) {
    if (lane == 0) seg_publish(my, e, 2, agg);
    return zero;
  }
  if (lane == 0) seg_publish(my, e, 1, agg);
  SegAgg acc = zero;
  int64_t end = t;  // window = predecessors [end-64, end)
  long long spins = 0;
  while (true) {
    const int64_t j = end - 1 - lane;
    unsigned long long w0 = pack(e, 2, 0), w1 = w0;  // virtual P(0) before tile 0
    if (j >= 0) {
      w0 = ld_relaxed(st + 2 * j);
      w1 = ld_relaxed(st + 2 * j + 1);
    }
    const bool valid = seg_valid(w0, w1, e);
    const unsigned long long pmask = __ballot(valid && w_flag(w0) == 2);
    const unsigned long long imask = __ballot(!valid);
    const int first_p = pmask ? __builtin_ctzll(pmask) : 64;
    const unsigned long long need = first_p >= 63 ? ~0ull : ((1ull << (first_p + 1)) - 1ull);
    if (imask & need) {
      if (++spins > kSpinLimit) {  // never expected: predecessors always make progress
        if (lane == 0) atomicExch(&ctl->overflow, 2u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    acc = seg_cat(wave_fold(lane <= first_p ? seg_decode(w0, w1) : zero), acc);
    if (first_p < 64) break;
    end -= 64;
  }
  if (lane == 0) seg_publish(my, e, 2, seg_cat(acc, agg));
  return acc;
}

// One trie node into the pinned host arrays (widths per HostTrie); false if past the capacity.
__device__ __forceinline__ void host_store(const HostTrie& h, FCtl* ctl, int64_t node, int64_t par,
                                           int32_t it, uint32_t cnt, uint8_t dep) {
  if (node >= h.cap) {
    ctl->dl_overflow = 1u;
    return;
  }
  if (h.par_w == 4) ((int32_t*)h.parent)[node] = (int32_t)par;
  else ((int64_t*)h.parent)[node] = par;
  if (h.item_w == 2) ((uint16_t*)h.item)[node] = (uint16_t)it;
  else ((int32_t*)h.item)[node] = it;
  if (h.cnt_w == 2) ((uint16_t*)h.count)[node] = (uint16_t)cnt;
  else ((uint32_t*)h.count)[node] = cnt;
  h.depth[node] = dep;
}

// Trie nodes [base, base + n) from the device trie arrays to the host trie; this thread copies
// relative nodes first, first + step, ... in rounds of kCopyBatch whose loads are all issued
// before its stores: CDNA's vmcnt counts stores too, so a load/store-interleaved loop waited for
// every PCIe write of one node before the loads of the next could be consumed.  Widths are
// uniform per call, so each width combination gets its own straight-line loop (32-bit indices
// from uniform bases keep the batch within the count kernels' register budget).
constexpr int kCopyBatch = 8;
template <typename PT, typename IT, typename CT>
__device__ __forceinline__ void copy_nodes_t(const HostTrie& h, const int64_t* __restrict__ par,
                                             const int32_t* __restrict__ item,
                                             const uint32_t* __restrict__ cnt,
                                             const uint8_t* __restrict__ dep, int64_t base,
                                             uint32_t n, uint32_t first, uint32_t step) {
  par += base;
  item += base;
  cnt += base;
  dep += base;
  PT* __restrict__ hp = (PT*)h.parent + base;
  IT* __restrict__ hi = (IT*)h.item + base;
  CT* __restrict__ hc = (CT*)h.count + base;
  uint8_t* __restrict__ hd = h.depth + base;
  for (uint32_t r0 = first; r0 < n; r0 += step * kCopyBatch) {
    int64_t p[kCopyBatch];
    int32_t it[kCopyBatch];
    uint32_t c[kCopyBatch];
    uint8_t d[kCopyBatch];
#pragma unroll
    for (int u = 0; u < kCopyBatch; ++u) {
      const uint32_t r = r0 + u * step;
      if (r < n) {
        p[u] = par[r];
        it[u] = item[r];
        c[u] = cnt[r];
        d[u] = dep[r];
      }
    }
#pragma unroll
    for (int u = 0; u < kCopyBatch; ++u) {
      const uint32_t r = r0 + u * step;
      if (r < n) {
        hp[r] = (PT)p[u];
        hi[r] = (IT)it[u];
        hc[r] = (CT)c[u];
        hd[r] = d[u];
      }
    }
  }
}
__device__ void copy_nodes(const HostTrie& h, FCtl* ctl, const int64_t* __restrict__ par,
                           const int32_t* __restrict__ item, const uint32_t* __restrict__ cnt,
                           const uint8_t* __restrict__ dep, int64_t base, int64_t n,
                           int64_t first, int64_t step) {
  if (base + n > h.cap) {  // past the host capacity: flag it (the host retries bigger)
    if (first == 0) ctl->dl_overflow = 1u;
    n = max((int64_t)0, h.cap - base);
  }
  if (first >= n) return;
  const uint32_t un = (uint32_t)n, uf = (uint32_t)first, us = (uint32_t)step;
  const int sel = (h.par_w == 4 ? 4 : 0) | (h.item_w == 2 ? 2 : 0) | (h.cnt_w == 2 ? 1 : 0);
  switch (sel) {
    case 7: copy_nodes_t<int32_t, uint16_t, uint16_t>(h, par, item, cnt, dep, base, un, uf, us); break;
    case 6: copy_nodes_t<int32_t, uint16_t, uint32_t>(h, par, item, cnt, dep, base, un, uf, us); break;
    case 5: copy_nodes_t<int32_t, int32_t, uint16_t>(h, par, item, cnt, dep, base, un, uf, us); break;
    case 4: copy_nodes_t<int32_t, int32_t, uint32_t>(h, par, item, cnt, dep, base, un, uf, us); break;
    case 3: copy_nodes_t<int64_t, uint16_t, uint16_t>(h, par, item, cnt, dep, base, un, uf, us); break;
    case 2: copy_nodes_t<int64_t, uint16_t, uint32_t>(h, par, item, cnt, dep, base, un, uf, us); break;
    case 1: copy_nodes_t<int64_t, int32_t, uint16_t>(h, par, item, cnt, dep, base, un, uf, us); break;
    default: copy_nodes_t<int64_t, int32_t, uint32_t>(h, par, item, cnt, dep, base, un, uf, us); break;
  }
}

// Copy role of the deferred download (LevelCountArgs::deferred_dl): trie nodes
// [desc[L-1].child_base, + desc[L].n_rows) — level L's rows, finished by the previous launch —
// from the device trie arrays to the host trie.  Runs in the first kCopyBlocks blocks of the
// launch (dispatched before any tile block, so the PCIe writes start at once and drain while the
// tiles compute instead of waiting for tile blocks to retire).
__device__ void copy_prev_level(const FLevel* lv, FCtl* ctl, const LevelCountArgs& A, int cb) {
  const FLevel* pv = lv - 1;
  const int64_t base = pv->child_base, n = lv->n_rows;
  // the destination in registers: host_store's flat stores may alias *ctl as far as the compiler
  // knows, so reading ctl->h in the loop reloaded it (a dependent round trip) for every node
  const HostTrie h = ctl->h;
  copy_nodes(h, ctl, A.out_parent, A.out_item, A.out_count, A.out_depth, base, n,
             (int64_t)cb * blockDim.x + threadIdx.x, (int64_t)A.copy_blocks * blockDim.x);
}

// Bump allocation from the device region (256-byte aligned); nullptr + overflow flag if full.
__device__ void* bump(FCtl* ctl, unsigned long long bytes) {
  bytes = (bytes + 255ull) & ~255ull;
  const unsigned long long off = atomicAdd(&ctl->bump_top, bytes);
  if (off + bytes > ctl->bump_cap) {
    atomicExch(&ctl->overflow, 1u);
    return nullptr;
  }
  return ctl->bump_base + off;
}

// Several bump allocations with ONE device atomic (each a serial ~1-2 µs round trip on the
// critical path of a level's last tile); out[i] = nullptr + overflow flag if the region is full.
template <int N>
__device__ void bump_n(FCtl* ctl, const unsigned long long (&bytes)[N], void* (&out)[N]) {
  unsigned long long off[N], tot = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    off[i] = tot;
    tot += (bytes[i] + 255ull) & ~255ull;
  }
  const unsigned long long base = atomicAdd(&ctl->bump_top, tot);
  const bool ok = base + tot <= ctl->bump_cap;
  if (!ok) atomicExch(&ctl->overflow, 1u);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = ok ? (void*)(ctl->bump_base + base + off[i]) : nullptr;
}

// Tile of a persistent level kernel.  When the grid covers every tile, tile = blockIdx.x (no
// atomic): a look-back only waits on lower block indices, which in-order dispatch has already
// placed even when fewer blocks than the grid are resident (sgpr-limited occupancy).  Otherwise
// every tile comes from the ticket counter — never a mix: a resident block holding a ticket
// tile could then spin on a block-index tile whose block cannot be dispatched.
__device__ __forceinline__ int64_t next_tile(unsigned int* ticket, bool first, int64_t n_tiles,
                                             int64_t* s_ticket, int64_t grid, int64_t bid) {
  if (n_tiles <= grid) return first ? bid : n_tiles;
  if (threadIdx.x == 0) *s_ticket = (int64_t)atomicAdd(ticket, 1u);
  __syncthreads();
  return *s_ticket;
}

// Block-wide exclusive scan of one int64 per thread (256 threads = 4 waves); returns the
// thread's exclusive prefix, *total = block sum.
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* s_w, int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  int64_t wbase = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kBlock / 64; ++i) {
    if (i < w) wbase += s_w[i];
    tot += s_w[i];
  }
  *total = tot;
  return wbase + x - v;
}

__device__ __forceinline__ int64_t find_row_g(const int64_t* __restrict__ off, int64_t lo,
                                              int64_t hi, int64_t c) {
  // largest a in [lo, hi) with off[a] <= c
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (off[mid] <= c) lo = mid; else hi = mid;
  }
  return lo;
}

// Buffers for the rows that counting T candidates can produce (the next level): child bitmaps at
// candidate slots (64-interleaved, see k_level_count_small), last-item rank, trie id, bitmap
// slot, and the children's own cand_off — one device atomic for all five.
__device__ void alloc_level(FCtl* ctl, FLevel* nx, int64_t T, int64_t Wp) {
  const unsigned long long t = (unsigned long long)T;
  const unsigned long long T64 = (t + 63ull) & ~63ull;
  const unsigned long long sz[5] = {T64 * (unsigned long long)Wp * 8ull, t * 4ull, t * 8ull,
                                    t * 4ull, (t + 1ull) * 8ull};
  void* p[5];
  bump_n<5>(ctl, sz, p);
  nx->bm = (const uint64_t*)p[0];
  nx->rank = (const int32_t*)p[1];
  nx->gid = (const int64_t*)p[2];
  nx->slot = (const int32_t*)p[3];
  nx->cand_off = (int64_t*)p[4];
}

struct EpiSmem {
  uint8_t fl[kBlock];     // per candidate: bit 0 survivor, bit 1 its owner's first candidate
  int64_t srow[kBlock];   // per candidate: survivor's next-level row (-1: failed)
};

// Wave-inclusive scan helpers (64 lanes)
__device__ __forceinline__ int32_t wave_incl_sum(int32_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}
__device__ __forceinline__ int64_t wave_incl_sum64(int64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  return x;
}

// Survivor layout of one count tile and the next level's candidate layout.  Every thread of the
// block calls this with its candidate's flags (thread i = candidate i of the tile); WAVE 0 alone
// does the tile's scans with shuffles (4 candidates per lane: survivors before each candidate,
// the segmented count of earlier siblings, their prefix), publishes the aggregate, runs the
// look-back and writes the next level's candidate offsets and tile→row entries, so the block
// meets only twice.  Returns the survivor's row index in the next level (-1: failed); the last
// tile sets the next level's sizes and allocates its children's buffers (not at a leaf level).
// capacity guard (overflow 4): when the trie arrays are what ran out, record the node count the
// level needs (MiB units) so the host sizes the next call's arrays for it
__device__ inline void fail_capacity(FCtl* ctl, int64_t need, int64_t out_cap) {
  if (need > out_cap) atomicMax(&ctl->need_out_m, (unsigned)((need + (1ll << 20) - 1) >> 20));
  atomicExch(&ctl->overflow, 4u);
}

__device__ int64_t tile_epilogue(EpiSmem& sm, int64_t t, int64_t n_tiles, bool live, int flag,
                                 bool head, unsigned long long* status, unsigned epoch, FCtl* ctl,
                                 FLevel* nx, int64_t* co_nx, int32_t* tile_row_nx, int64_t scap,
                                 int64_t child_base, int64_t n_cand, int64_t Wp, int64_t out_cap,
                                 bool leaf) {
  const int tid = threadIdx.x;
  sm.fl[tid] = (uint8_t)((flag ? 1 : 0) | ((live && head) ? 2 : 0));
  __syncthreads();
  if (tid < 64) {
    const int lane = tid;
    const uint32_t packed = *reinterpret_cast<const uint32_t*>(&sm.fl[4 * lane]);
    int f[4], h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] = (packed >> (8 * j)) & 1;
      h[j] = (packed >> (8 * j + 1)) & 1;
    }
    const int nf = f[0] + f[1] + f[2] + f[3];
    const bool lh_any = (h[0] | h[1] | h[2] | h[3]) != 0;
    // survivors in this lane after its last head (all of them without a head)
    int tail = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) tail = h[j] ? f[j] : tail + f[j];
    const int32_t incl = wave_incl_sum(nf);
    const int32_t lx0 = incl - nf;               // survivors before this lane
    const int32_t S = __shfl(incl, 63, 64);
    const unsigned long long hmask = __ballot(lh_any);
    // open-segment survivors entering this lane: from the nearest earlier lane with a head
    // (its tail, plus every survivor of the lanes in between), or from the tile start
    const unsigned long long before = hmask & ((1ull << lane) - 1ull);
    const int src = before ? 63 - __builtin_clzll(before) : -1;
    const int32_t tail_src = __shfl(tail, src < 0 ? 0 : src, 64);
    const int32_t incl_src = __shfl(incl, src < 0 ? 0 : src, 64);
    const int32_t run0 = src < 0 ? lx0 : tail_src + (lx0 - incl_src);
    // this lane's items: earlier siblings inside the tile's span (len0) and their sum
    int32_t lsum = 0, before_first = lx0;
    {
      int32_t run = run0, l = lx0;
      bool seen = false;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (h[j]) {
          run = 0;
          if (!seen) before_first = l;
          seen = true;
        }
        if (f[j]) lsum += run;
        run += f[j];
        l += f[j];
      }
    }
    const int64_t cincl = wave_incl_sum64(lsum);
    const int64_t C0 = __shfl(cincl, 63, 64);
    // tile aggregate: F = survivors before the first head, O = survivors since the last head
    const bool H = hmask != 0;
    int32_t Fh = S, O = S;
    if (H) {
      Fh = __shfl(before_first, __builtin_ctzll(hmask), 64);
      O = __shfl(tail + (S - incl), 63 - __builtin_clzll(hmask), 64);  // last head lane on
    }
    const SegAgg p = lookback_seg(status, t, epoch, SegAgg{S, O, Fh, H, C0}, ctl);
    const int64_t base = p.S, cex = p.C, carry = p.O;
    // second pass over the lane's items (recomputed: little stays live across the look-back)
    {
      int32_t run = run0, l = lx0;
      bool cont = src < 0;  // no head yet: the segment continuing from the previous tile
      int64_t cl = cincl - lsum;  // candidates of this lane's earlier survivors (carry 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int fj = (packed >> (8 * j)) & 1, hj = (packed >> (8 * j + 1)) & 1;
        if (hj) {
          run = 0;
          cont = false;
        }
        int64_t srow = -1;
        if (fj) {
          srow = base + l;
          if (!leaf) {
            const int64_t len = run + (cont ? carry : 0);  // earlier siblings
            const int64_t co = cex + cl + carry * (cont ? (int64_t)l : (int64_t)Fh);
            co_nx[srow] = co;
            for (int64_t c = (co + kTile - 1) / kTile; c * kTile < co + len; ++c)
              if (c < scap) tile_row_nx[c] = (int32_t)srow;
          }
          cl += run;
        }
        sm.srow[4 * lane + j] = srow;
        run += fj;
        l += fj;
      }
    }
    if (t == n_tiles - 1 && lane == 0) {
      const int64_t St = base + S;
      const int64_t Ct = cex + C0 + carry * Fh;
      nx->n_rows = St;
      nx->child_base = child_base + St;
      nx->n_cand = leaf ? 0 : Ct;
      atomicAdd(&ctl->candidates, (unsigned long long)n_cand);
      if (!leaf) {
        co_nx[St] = Ct;
        if (child_base + St + Ct > out_cap || (Ct + kTile - 1) / kTile > scap ||
            Ct >= kRowLimit)
          fail_capacity(ctl, child_base + St + Ct, out_cap);
        else
          alloc_level(ctl, nx + 1, Ct, Wp);
      }
    }
  }
  __syncthreads();
  return sm.srow[tid];
}

// A level without candidates: empty next level, and a one-entry cand_off for the level after
__device__ void empty_level(FCtl* ctl, FLevel* nx, int64_t child_base) {
  nx->n_rows = 0;
  nx->n_cand = 0;
  nx->child_base = child_base;
  if (nx->cand_off) nx->cand_off[0] = 0;
  alloc_level(ctl, nx + 1, 0, 0);
}

// ---------------------------------------------------------------------------------------------
// Long rows (T > 4096 transactions): a team of TS lanes per candidate; survivors' rows are written
// compactly at their next-level row index (the next level reads rows row-major).
template <int TS>
__global__ __launch_bounds__(kBlock) void k_level_count(FLevel* __restrict__ lv,
                                                        FLevel* __restrict__ nx, FCtl* ctl,
                                                        unsigned long long* __restrict__ status,
                                                        unsigned epoch, LevelCountArgs A,
                                                        const int32_t* __restrict__ tile_row,
                                                        int32_t* __restrict__ tile_row_nx) {
  __shared__ int64_t s_off[kWin];
  __shared__ uint32_t s_cnt[kTile];
  __shared__ int64_t s_a[kTile];   // candidate → earlier sibling a
  __shared__ int64_t s_b[kTile];   // candidate → owner row b
  __shared__ int64_t s_row[kTile];  // candidate → survivor's next-level row (-1: failed)
  __shared__ int64_t s_r0;
  __shared__ int64_t s_ticket;
  __shared__ EpiSmem epi;
  if (ctl->overflow) return;
  epoch = (ctl->epoch_base + epoch) & kEpochMask;  // per-call base (FCtl) + launch index
  const int cbk = A.deferred_dl ? A.copy_blocks : 0;  // copy blocks (lead the grid by default)
  const int64_t tgrid = (int64_t)gridDim.x - cbk;     // tile blocks
  const int64_t cb0 = A.copy_last ? tgrid : 0;
  if ((int64_t)blockIdx.x >= cb0 && (int64_t)blockIdx.x < cb0 + cbk) {
    copy_prev_level(lv, ctl, A, (int)(blockIdx.x - cb0));
    return;
  }
  const int64_t bid = A.copy_last ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - cbk;
  const int64_t n_cand = lv->n_cand;
  const int64_t n_rows = lv->n_rows;
  const int64_t n_tiles = (n_cand + kTile - 1) / kTile;
  const int64_t child_base = lv->child_base;
  if (n_tiles == 0) {
    if (bid == 0 && threadIdx.x == 0) empty_level(ctl, nx, child_base);
    return;
  }
  if (bid >= n_tiles) return;  // idle blocks: no ticket atomic
  const int64_t* __restrict__ co = lv->cand_off;
  const unsigned long long* __restrict__ bm = (const unsigned long long*)lv->bm;
  const int32_t* __restrict__ rank = lv->rank;
  const int64_t* __restrict__ gid = lv->gid;
  unsigned long long* __restrict__ cbm = (unsigned long long*)nx->bm;
  int32_t* __restrict__ crank = (int32_t*)nx->rank;
  int64_t* __restrict__ cgid = (int64_t*)nx->gid;
  int64_t* __restrict__ co_nx = nx->cand_off;
  const int64_t scap = (int64_t)ctl->status_cap;
  const int64_t Wp = A.Wp;
  const int64_t n2 = Wp >> 1;
  const int tl = threadIdx.x & (TS - 1);
  const int team = threadIdx.x / TS;
  constexpr int kTeams = kBlock / TS;
  constexpr int kPer = kTile / kTeams;
  // bitmap row of a level row: the root's rows are the frequent items in descending rank order
  // over a bitmap stored by rank; deeper levels are compact
  auto brow = [&](int64_t r) { return A.root ? (int64_t)rank[r] : r; };
  for (bool first = true;; first = false) {
    const int64_t t = next_tile(&lv->count_ticket, first, n_tiles, &s_ticket, tgrid, bid);
    if (t >= n_tiles) return;
    const int64_t c0 = t * kTile;
    const int cn = (int)min((int64_t)kTile, n_cand - c0);
    if (tile_row) {  // first row of the tile, recorded by the previous level's count
      if (threadIdx.x == 0) s_r0 = tile_row[t];
    } else if (threadIdx.x < 64) {  // root level: 64-ary search by wave 0
      const int64_t c = c0;
      int64_t lo = 0, hi = n_rows;  // invariant: co[lo] <= c < co[hi]
      while (hi - lo > 64) {
        const int64_t step = (hi - lo + 63) / 64;
        const int64_t p = lo + (int64_t)threadIdx.x * step;
        const unsigned long long bal = __ballot(p < hi && co[p] <= c);
        const int last = 63 - __builtin_clzll(bal);  // lane 0 always true (p = lo)
        const int64_t nlo = lo + (int64_t)last * step;
        hi = min(hi, nlo + step);
        lo = nlo;
      }
      const int64_t p = lo + threadIdx.x;
      const unsigned long long bal = __ballot(p < hi && co[p] <= c);
      if (threadIdx.x == 0) s_r0 = lo + (63 - __builtin_clzll(bal));
    }
    __syncthreads();
    // window co[r0 .. r0 + nw) in LDS; a candidate past the window searches HBM (rare: only
    // when the tile spans more than kWin rows)
    const int64_t r0 = s_r0;
    const int64_t nw = min((int64_t)kWin, n_rows + 1 - r0);
    for (int64_t i = threadIdx.x; i < nw; i += kBlock) s_off[i] = co[r0 + i];
    __syncthreads();
    // one decode per candidate: owner b = the row whose range holds c, a = an earlier sibling
    bool head = false;
    const bool live = (int)threadIdx.x < cn;
    if (live) {
      const int64_t c = c0 + threadIdx.x;
      int64_t b, oa, ob;
      if (nw >= 2 && s_off[nw - 1] > c) {  // row in window: largest k < nw-1 with s_off[k] <= c
        int64_t lo = 0, hi = nw - 1;
        while (hi - lo > 1) {
          const int64_t mid = (lo + hi) >> 1;
          if (s_off[mid] <= c) lo = mid; else hi = mid;
        }
        b = r0 + lo;
        oa = s_off[lo];
        ob = s_off[lo + 1];
      } else {
        b = find_row_g(co, r0, n_rows, c);
        oa = co[b];
        ob = co[b + 1];
      }
      head = c == oa;
      s_a[threadIdx.x] = b - (ob - c);
      s_b[threadIdx.x] = b;
    }
    __syncthreads();
    // ---- phase 1: supports (team per candidate, 2 candidates in flight) ----
    for (int j = 0; j < kPer; j += 2) {
      const int i0 = team * kPer + j, i1 = i0 + 1;
      if (i0 >= cn) break;  // team-uniform
      const bool two = i1 < cn;
      if (A.gram) {
        if (tl == 0) {
          for (int q = 0; q < (two ? 2 : 1); ++q) {
            const int64_t ra = rank[s_a[i0 + q]], rb = rank[s_b[i0 + q]];
            s_cnt[i0 + q] = A.gram[min(ra, rb) * A.F + max(ra, rb)];
          }
        }
        continue;
      }
      const ulonglong2* x0 = reinterpret_cast<const ulonglong2*>(bm + brow(s_a[i0]) * Wp);
      const ulonglong2* y0 = reinterpret_cast<const ulonglong2*>(bm + brow(s_b[i0]) * Wp);
      const ulonglong2* x1 = reinterpret_cast<const ulonglong2*>(bm + brow(s_a[two ? i1 : i0]) * Wp);
      const ulonglong2* y1 = reinterpret_cast<const ulonglong2*>(bm + brow(s_b[two ? i1 : i0]) * Wp);
      uint32_t k0 = 0, k1 = 0;
      for (int64_t w = tl; w < n2; w += TS) {
        const ulonglong2 u0 = x0[w], v0 = y0[w], u1 = x1[w], v1 = y1[w];
        k0 += (uint32_t)__popcll(u0.x & v0.x) + (uint32_t)__popcll(u0.y & v0.y);
        k1 += (uint32_t)__popcll(u1.x & v1.x) + (uint32_t)__popcll(u1.y & v1.y);
      }
#pragma unroll
      for (int off = TS >> 1; off > 0; off >>= 1) {
        k0 += __shfl_xor(k0, off, TS);
        k1 += __shfl_xor(k1, off, TS);
      }
      if (tl == 0) {
        s_cnt[i0] = k0;
        if (two) s_cnt[i1] = k1;
      }
    }
    __syncthreads();
    // ---- phase 2: survivor rows + next-level layout (block scans + segmented look-back) ----
    const int flag = (live && s_cnt[threadIdx.x] >= A.minsup) ? 1 : 0;
    const int64_t s = tile_epilogue(epi, t, n_tiles, live, flag, head, status, epoch, ctl, nx,
                                    co_nx, tile_row_nx, scap, child_base, n_cand, Wp, A.out_cap,
                                    A.leaf);
    s_row[threadIdx.x] = s;
    if (flag) {  // per-survivor scalars: one thread each
      const int64_t a = s_a[threadIdx.x], b = s_b[threadIdx.x];
      const int32_t ra = rank[a];
      const int64_t node = child_base + s;
      crank[s] = ra;
      cgid[s] = node;
      const int64_t par = gid[b];
      const int32_t it = A.ids[ra];
      const uint32_t cnt = s_cnt[threadIdx.x];
      A.out_parent[node] = par;
      A.out_item[node] = it;
      A.out_count[node] = cnt;
      A.out_depth[node] = A.child_depth;
      // streamed download: consecutive survivors → coalesced PCIe writes
      if (A.download && !A.deferred_dl) host_store(ctl->h, ctl, node, par, it, cnt, A.child_depth);
    }
    __syncthreads();
    // ---- phase 3: survivors' bitmaps (team per survivor), compact at their row ----
    for (int j = 0; j < kPer; ++j) {
      const int i = team * kPer + j;
      if (i >= cn) break;
      const int64_t srow = s_row[i];
      if (srow < 0 || A.leaf) continue;  // team-uniform
      const ulonglong2* x = reinterpret_cast<const ulonglong2*>(bm + brow(s_a[i]) * Wp);
      const ulonglong2* y = reinterpret_cast<const ulonglong2*>(bm + brow(s_b[i]) * Wp);
      ulonglong2* z = reinterpret_cast<ulonglong2*>(cbm + srow * Wp);
      for (int64_t w = tl; w < n2; w += TS) {
        const ulonglong2 u = x[w], v = y[w];
        z[w] = make_ulonglong2(u.x & v.x, u.y & v.y);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// Short-row variant (n2 = Wp/2 <= kSmallChunks 16-byte chunks, i.e. T <= 4096 transactions —
// the reference's playlist datasets).  Per-tile phase traces (KMLS_LEVEL_TRACE, see
// profiles/r1_s3_level_traces.md) showed the team kernel latency-bound: about one tile per
// resident block on the big levels, each a chain of dependent memory round trips, and the
// survivor-materialise phase (re-reading both parent rows after the look-back) the longest
// link.  Here
//   * phase 1: ONE thread per candidate ANDs its row pair with independent 16-byte loads,
//     popcounts in registers (no cross-lane reduction) and writes the AND row straight to the
//     child bitmap array at the CANDIDATE index (fire-and-forget stores; a row that fits one
//     load batch is held until its count is known, so only survivors' rows are written).
//     Child rows then reach their bitmap through FLevel::slot, so there is no compaction pass at
//     all.  Candidate rows are stored 64-interleaved (chunk w of slot c at ((c/64)*n2 + w)*64 +
//     c%64): the 64 lanes of a wave write 64 consecutive slots, and the next level's lanes read
//     siblings with consecutive slots, so both directions are coalesced 1 KB accesses;
//   * the root level (pair counts from the gram) computes AND rows only for survivors.
// Decode, look-back, trie/host writes and the next level's layout are shared with k_level_count.
constexpr int kSmallChunks = 32;

template <int KB>
__global__ __launch_bounds__(kBlock, KB <= 6 ? 4 : 1) void k_level_count_small(FLevel* __restrict__ lv,
                                                              FLevel* __restrict__ nx, FCtl* ctl,
                                                              unsigned long long* __restrict__ status,
                                                              unsigned epoch, LevelCountArgs A,
                                                              const int32_t* __restrict__ tile_row,
                                                              int32_t* __restrict__ tile_row_nx) {
  __shared__ int64_t s_off[kWin];
  __shared__ int64_t s_r0;
  __shared__ int64_t s_ticket;
  __shared__ EpiSmem epi;
  // Every descriptor field the first tile needs, loaded as one batch before the first branch
  // (an early-return on ctl->overflow first made these a chain of dependent round trips — about
  // a microsecond each, on every launch), plus the tile→row entry of this block's tile in
  // block-index mode (bid < grid <= status_cap, so the speculative load stays in bounds).
  const unsigned ovf = ctl->overflow;
  const unsigned ebase = ctl->epoch_base;
  const int64_t scap = (int64_t)ctl->status_cap;
  const int64_t n_cand = lv->n_cand;
  const int64_t n_rows = lv->n_rows;
  const int64_t child_base = lv->child_base;
  const int64_t* __restrict__ co = lv->cand_off;
  const ulonglong2* __restrict__ bm2 = (const ulonglong2*)lv->bm;
  const int32_t* __restrict__ slot = lv->slot;
  const int32_t* __restrict__ rank = lv->rank;
  const int64_t* __restrict__ gid = lv->gid;
  ulonglong2* __restrict__ cbm2 = (ulonglong2*)nx->bm;
  int32_t* __restrict__ crank = (int32_t*)nx->rank;
  int64_t* __restrict__ cgid = (int64_t*)nx->gid;
  int32_t* __restrict__ cslot = (int32_t*)nx->slot;
  int64_t* __restrict__ co_nx = nx->cand_off;
  const int cbk = A.deferred_dl ? A.copy_blocks : 0;  // copy blocks (lead the grid by default)
  const int64_t tgrid = (int64_t)gridDim.x - cbk;     // tile blocks
  const int64_t cb0 = A.copy_last ? tgrid : 0;
  const bool copy_role = (int64_t)blockIdx.x >= cb0 && (int64_t)blockIdx.x < cb0 + cbk;
  const int64_t bid = A.copy_last ? (int64_t)blockIdx.x : (int64_t)blockIdx.x - cbk;
  const int32_t r0_spec = (tile_row && !copy_role) ? tile_row[bid] : 0;
  // keep the batch above the branch (the compiler otherwise sinks each load to its first use)
  asm volatile("" ::"s"(n_cand), "s"(n_rows), "s"(child_base), "s"(co), "s"(bm2), "s"(slot),
               "s"(rank), "s"(gid));
  asm volatile("" ::"s"(cbm2), "s"(crank), "s"(cgid), "s"(cslot), "s"(r0_spec), "s"(ebase));
  if (ovf) return;
  epoch = (ebase + epoch) & kEpochMask;  // per-call base (FCtl) + launch index
  if (copy_role) {
    copy_prev_level(lv, ctl, A, (int)(blockIdx.x - cb0));
    return;
  }
  const int64_t n_tiles = (n_cand + kTile - 1) / kTile;
  if (n_tiles == 0) {
    if (bid == 0 && threadIdx.x == 0) empty_level(ctl, nx, child_base);
    return;
  }
  if (bid >= n_tiles) return;
  const int n2 = (int)(A.Wp >> 1);
  for (bool first = true;; first = false) {
    const int64_t t = next_tile(&lv->count_ticket, first, n_tiles, &s_ticket, tgrid, bid);
    if (t >= n_tiles) return;
    unsigned long long* tr = (A.trace && threadIdx.x == 0) ? A.trace + t * 8 : nullptr;
    if (tr) tr[0] = wall_clock64();
    const int64_t c0 = t * kTile;
    const int cn = (int)min((int64_t)kTile, n_cand - c0);
    if (tile_row) {  // first row of the tile, recorded by the previous level's count
      if (threadIdx.x == 0) s_r0 = (first && n_tiles <= tgrid) ? (int64_t)r0_spec : tile_row[t];
    } else if (threadIdx.x < 64) {  // root level: 64-ary search by wave 0
      const int64_t c = c0;
      int64_t lo = 0, hi = n_rows;
      while (hi - lo > 64) {
        const int64_t step = (hi - lo + 63) / 64;
        const int64_t p = lo + (int64_t)threadIdx.x * step;
        const unsigned long long bal = __ballot(p < hi && co[p] <= c);
        const int last = 63 - __builtin_clzll(bal);
        const int64_t nlo = lo + (int64_t)last * step;
        hi = min(hi, nlo + step);
        lo = nlo;
      }
      const int64_t p = lo + threadIdx.x;
      const unsigned long long bal = __ballot(p < hi && co[p] <= c);
      if (threadIdx.x == 0) s_r0 = lo + (63 - __builtin_clzll(bal));
    }
    __syncthreads();
    const int64_t r0 = s_r0;
    const int64_t nw = min((int64_t)kWin, n_rows + 1 - r0);
    for (int64_t i = threadIdx.x; i < nw; i += kBlock) s_off[i] = co[r0 + i];
    __syncthreads();
    if (tr) tr[1] = wall_clock64();
    // ---- decode + phase 1: one thread per candidate, AND row written in place ----
    uint32_t k = 0;
    int32_t a = 0, b = 0;  // level rows are int32-indexed (the count kernels check the sizes)
    bool head = false;  // this candidate is its owner's first
    const bool live = (int)threadIdx.x < cn;
    const int64_t c = c0 + threadIdx.x;
    if (live) {
      int64_t oa, ob;
      if (nw >= 2 && s_off[nw - 1] > c) {
        int64_t lo = 0, hi = nw - 1;
        while (hi - lo > 1) {
          const int64_t mid = (lo + hi) >> 1;
          if (s_off[mid] <= c) lo = mid; else hi = mid;
        }
        b = (int32_t)(r0 + lo);
        oa = s_off[lo];
        ob = s_off[lo + 1];
      } else {
        b = (int32_t)find_row_g(co, r0, n_rows, c);
        oa = co[b];
        ob = co[b + 1];
      }
      head = c == oa;
      a = (int32_t)(b - (ob - c));
      bool need_row = true;
      if (A.gram) {  // root: pair counts by rank (rows are in descending rank order)
        const int64_t ra = rank[a], rb = rank[b];
        k = A.gram[min(ra, rb) * A.F + max(ra, rb)];
        need_row = k >= A.minsup && !A.leaf;
      }
      if (need_row) {
        // parent rows: by rank at the root (row-major), 64-interleaved candidate slots below it
        const ulonglong2* __restrict__ x;
        const ulonglong2* __restrict__ y;
        int sxy;
        if (slot) {
          const int64_t sa = slot[a], sb = slot[b];
          x = bm2 + ((sa >> 6) * n2 << 6) + (sa & 63);
          y = bm2 + ((sb >> 6) * n2 << 6) + (sb & 63);
          sxy = 64;
        } else {
          x = bm2 + (A.root ? (int64_t)rank[a] : a) * n2;
          y = bm2 + (A.root ? (int64_t)rank[b] : b) * n2;
          sxy = 1;
        }
        ulonglong2* __restrict__ z = cbm2 + ((c >> 6) * n2 << 6) + (c & 63);
        // batches of kB chunk pairs: all loads of a batch are issued before its stores (a
        // load/store-interleaved loop compiles to one full memory round trip per chunk).  KB
        // trades registers (occupancy, for the big levels) against round trips per candidate
        // (the latency of the small ones)
        constexpr int kB = KB;
        uint32_t kk = 0;
        // a row that fits one batch stays in registers until its count is known, so only
        // survivors' rows are written (a multi-batch row streams out unconditionally)
        const bool one_batch = n2 <= kB;
        for (int w0 = 0; w0 < n2; w0 += kB) {
          ulonglong2 u[kB], v[kB];
#pragma unroll
          for (int q = 0; q < kB; ++q)
            if (w0 + q < n2) {
              u[q] = x[(w0 + q) * sxy];
              v[q] = y[(w0 + q) * sxy];
            }
#pragma unroll
          for (int q = 0; q < kB; ++q)
            if (w0 + q < n2) {
              u[q] = make_ulonglong2(u[q].x & v[q].x, u[q].y & v[q].y);
              kk += (uint32_t)__popcll(u[q].x) + (uint32_t)__popcll(u[q].y);
            }
          const bool keep = !A.leaf && (!one_batch || A.gram || kk >= A.minsup);
          if (keep) {
#pragma unroll
            for (int q = 0; q < kB; ++q)
              if (w0 + q < n2) z[(w0 + q) << 6] = u[q];
          }
        }
        if (!A.gram) k = kk;
      }
    }
    // ---- phase 2: survivor rows + next-level layout, trie + host writes ----
    const int flag = (live && k >= A.minsup) ? 1 : 0;
    if (tr) tr[2] = wall_clock64();
    const int64_t s = tile_epilogue(epi, t, n_tiles, live, flag, head, status, epoch, ctl, nx,
                                    co_nx, tile_row_nx, scap, child_base, n_cand, A.Wp, A.out_cap,
                                    A.leaf);
    if (tr) tr[3] = wall_clock64();
    if (flag) {
      const int32_t ra = rank[a];
      const int64_t node = child_base + s;
      crank[s] = ra;
      cgid[s] = node;
      cslot[s] = (int32_t)c;
      const int64_t par = gid[b];
      const int32_t it = A.ids[ra];
      A.out_parent[node] = par;
      A.out_item[node] = it;
      A.out_count[node] = k;
      A.out_depth[node] = A.child_depth;
      if (A.download && !A.deferred_dl) host_store(ctl->h, ctl, node, par, it, k, A.child_depth);
    }
    if (tr) tr[4] = wall_clock64();
    if (tr) tr[5] = wall_clock64();
    __syncthreads();
    if (tr) {
      tr[6] = wall_clock64();
      tr[7] = (unsigned long long)cn;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Deferred-download tail: the last launched level's children have no following count launch to
// carry them, so this copies trie nodes [lv->child_base, + nx->n_rows) after the level loop.
// The last block also copies the level descriptors + control block (`rb_words` 16-byte words
// from rb_src) to pinned host memory: the host's one readback per call, without a
// hipMemcpyAsync (whose host-side cost dominated the step's idle gap).
__global__ __launch_bounds__(kBlock) void k_level_copyout(const FLevel* __restrict__ lv,
                                                          const FLevel* __restrict__ nx, FCtl* ctl,
                                                          const int64_t* __restrict__ d_parent,
                                                          const int32_t* __restrict__ d_item,
                                                          const uint32_t* __restrict__ d_count,
                                                          const uint8_t* __restrict__ d_depth,
                                                          bool download, const uint4* __restrict__ rb_src,
                                                          int rb_words) {
  if (rb_words && blockIdx.x == gridDim.x - 1) {
    // The copy blocks of this same launch flag a host-capacity overflow, possibly after this
    // block has read the control block: decide it here too (it depends only on sizes), or the
    // host would trust a truncated download.
    if (threadIdx.x == 0 && download && !ctl->overflow &&
        lv->child_base + nx->n_rows > ctl->h.cap)
      ctl->dl_overflow = 1u;
    __threadfence();
    __syncthreads();
    uint4* __restrict__ rb_dst = (uint4*)ctl->rb_dst;
    for (int i = threadIdx.x; i < rb_words; i += blockDim.x) rb_dst[i] = rb_src[i];
    return;
  }
  if (!download || ctl->overflow) return;
  const HostTrie h = ctl->h;
  const int64_t base = lv->child_base;
  const int64_t S = nx->n_rows;
  if (S <= 0) return;
  // the readback block (last, when present) copies no nodes: stride over the copy blocks only
  const int64_t nthr = (int64_t)(gridDim.x - (rb_words ? 1 : 0)) * blockDim.x;
  copy_nodes(h, ctl, d_parent, d_item, d_count, d_depth, base, S,
             (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nthr);
}

// ---------------------------------------------------------------------------------------------
// device-resident prologue
// Frequent-item ranking by (count asc, id asc) as select_frequent: a 2-D grid compares item
// tiles against j-tiles (256 x 256 per block, j-tile in LDS) and accumulates how many frequent
// items precede each item; a 1-D pass scatters ids/counts by rank.  O(n^2) work but n <= 16k and
// fully parallel (a one-block version took 300 µs at n = 2171).
__global__ __launch_bounds__(256) void k_select_rank(const uint32_t* __restrict__ cnt,
                                                     int64_t n_items, uint32_t c1,
                                                     int32_t* __restrict__ rank_acc) {
  __shared__ uint32_t s_c[256];
  const int64_t j0 = (int64_t)blockIdx.y * 256;
  const int64_t jn = min((int64_t)256, n_items - j0);
  if ((int64_t)threadIdx.x < jn) s_c[threadIdx.x] = cnt[j0 + threadIdx.x];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_items) return;
  const uint32_t ci = cnt[i];
  if (ci < c1) return;
  int32_t r = 0;
  for (int64_t jj = 0; jj < jn; ++jj) {
    const uint32_t cj = s_c[jj];
    const int64_t j = j0 + jj;
    r += (cj >= c1 && (cj < ci || (cj == ci && j < i))) ? 1 : 0;
  }
  if (r) atomicAdd(&rank_acc[i], r);
}

__global__ __launch_bounds__(256) void k_prologue_init(uint32_t* __restrict__ cnt, int64_t n_items,
                                                       uint64_t* __restrict__ bm, int64_t bm_words,
                                                       FLevel* __restrict__ desc, int n_desc,
                                                       FCtl* __restrict__ ctl,
                                                       const FCtl* __restrict__ params,
                                                       unsigned int* __restrict__ seq) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = tid; i < n_items; i += nthr) cnt[i] = 0u;
  for (int64_t i = tid; i < bm_words; i += nthr) bm[i] = 0ull;
  const int64_t dwords = (int64_t)n_desc * (int64_t)(sizeof(FLevel) / 8);
  for (int64_t i = tid; i < dwords; i += nthr) ((unsigned long long*)desc)[i] = 0ull;
  // two parameter slots, alternating per call (the host fills slot (call index & 1)), so the
  // host can prepare and launch call n+1 while call n is still running
  if (tid == 0) {
    const unsigned int k = *seq;
    *ctl = params[k & 1u];
    *seq = k + 1u;
  }
}

// 16 lanes per item, each comparing against every 16th item (a one-thread-per-item loop ran
// one wave per SIMD on 9 CUs: 113 µs at 2171 items); partial ranks meet in a 16-lane shuffle.
__global__ __launch_bounds__(256) void k_select_fused(const uint32_t* __restrict__ cnt,
                                                      int64_t n_items, uint32_t c1,
                                                      int32_t* __restrict__ ids,
                                                      uint32_t* __restrict__ fcounts,
                                                      int32_t* __restrict__ rank_of, FLevel* desc,
                                                      const FCtl* __restrict__ ctl) {
  int32_t* __restrict__ host_tab = ctl->host_tab;
  const int64_t tab_stride = ctl->tab_stride;
  __shared__ unsigned int s_F;
  __shared__ uint32_t s_c[kSelectFusedMax];  // the whole histogram (a global load per compare
                                             // made the loop one memory latency per step)
  if (threadIdx.x == 0) s_F = 0;
  for (int64_t j = threadIdx.x; j < n_items; j += blockDim.x) s_c[j] = cnt[j];
  __syncthreads();
  const int p = threadIdx.x & 15;
  const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const uint32_t ci = i < n_items ? s_c[i] : 0u;
  int32_t r = 0;
  if (i < n_items && ci >= c1) {
    const int ii = (int)i;
    for (int j = p; j < (int)n_items; j += 16) {
      const uint32_t cj = s_c[j];
      r += (cj >= c1 && (cj < ci || (cj == ci && j < ii))) ? 1 : 0;
    }
  }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) r += __shfl_xor(r, off, 16);
  if (p == 0 && i < n_items) {
    const bool f = ci >= c1;
    rank_of[i] = f ? r : -1;
    if (host_tab) host_tab[2 * tab_stride + i] = f ? r : -1;
    if (f) {  // (ids/counts reach host_tab from the root setup, in rank order: coalesced)
      ids[r] = (int32_t)i;
      fcounts[r] = ci;
      atomicAdd(&s_F, 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_F) atomicAdd((unsigned long long*)&desc[1].n_rows, (unsigned long long)s_F);
}

__global__ __launch_bounds__(256) void k_select_scatter(const uint32_t* __restrict__ cnt,
                                                        int64_t n_items, uint32_t c1,
                                                        const int32_t* __restrict__ rank_acc,
                                                        int32_t* __restrict__ ids,
                                                        uint32_t* __restrict__ fcounts,
                                                        int32_t* __restrict__ rank_of,
                                                        FLevel* desc) {
  __shared__ unsigned int s_F;
  if (threadIdx.x == 0) s_F = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n_items) {
    const uint32_t ci = cnt[i];
    if (ci < c1) {
      rank_of[i] = -1;
    } else {
      const int32_t r = rank_acc[i];
      rank_of[i] = r;
      ids[r] = (int32_t)i;
      fcounts[r] = ci;
      atomicAdd(&s_F, 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_F) atomicAdd((unsigned long long*)&desc[1].n_rows, (unsigned long long)s_F);
}

// Root-class partition for replicated-data multi-GPU mining (identical on every rank, so no
// collective): cost(a) = n_a^2 + 1 with n_a = frequent extensions of item a (gram row), ranked
// by (cost desc, a asc) and dealt in snake order — the device twin of dist_miner.lpt_partition.
__global__ __launch_bounds__(256) void k_root_costs(const uint32_t* __restrict__ gram, int64_t ld,
                                                    const FLevel* desc, uint32_t minsup,
                                                    int64_t* __restrict__ cost) {
  __shared__ int64_t s_w[4];
  const int64_t F = desc[1].n_rows;
  const int64_t a = blockIdx.x;
  if (a >= F) return;
  int64_t n = 0;
  for (int64_t b = a + 1 + threadIdx.x; b < F; b += blockDim.x) n += gram[a * ld + b] >= minsup;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int64_t t = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    cost[a] = t * t + 1;
  }
}

// rank(i) = #{j : cost_j > cost_i or (cost_j == cost_i and j < i)} — (cost desc, item asc).
// Block b ranks items [64b, 64b + 64): wave w compares them against the w-th quarter of all
// costs (32-bit, staged through LDS and read 8 at a time so the loop is not bound by one LDS
// round trip per compare), the partial ranks are summed in LDS and written directly.  (A 2-D
// grid accumulating partial ranks needed a zeroed accumulator: two fill kernels plus the
// ranking launch on every multi-GPU step.  Ranking inside the one-block root setup cost 30 µs:
// a CU retires only 64 lane-ops per cycle.)
constexpr int kRankChunk = 8192;
__global__ __launch_bounds__(256) void k_rank_desc(const int64_t* __restrict__ cost,
                                                   const FLevel* desc, int32_t* __restrict__ rank) {
  __shared__ __attribute__((aligned(16))) int32_t s_c[kRankChunk];
  __shared__ int32_t s_r[4][64];
  const int64_t F = desc[1].n_rows;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  if ((int64_t)blockIdx.x * 64 >= F) return;
  const int32_t ci = i < F ? (int32_t)cost[i] : 0;  // n^2 + 1 <= F^2 + 1 fits 32 bits
  int32_t r = 0;
  for (int64_t j0 = 0; j0 < F; j0 += kRankChunk) {
    const int32_t jn = (int32_t)min((int64_t)kRankChunk, F - j0);
    __syncthreads();
    for (int32_t j = threadIdx.x; j < jn; j += blockDim.x) s_c[j] = (int32_t)cost[j0 + j];
    __syncthreads();
    const int32_t q = ((jn + 31) / 32) * 8, jb = w * q, je = min(jn, jb + q);  // 8-aligned quarters
    const int32_t il = (int32_t)(i - j0);  // this item's index relative to the chunk
    int32_t j = jb;
    for (; j + 8 <= je; j += 8) {
      const int4 c0 = *(const int4*)&s_c[j];
      const int4 c1 = *(const int4*)&s_c[j + 4];
      const int32_t cj[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
      for (int u = 0; u < 8; ++u) r += (cj[u] > ci || (cj[u] == ci && j + u < il)) ? 1 : 0;
    }
    for (; j < je; ++j) r += (s_c[j] > ci || (s_c[j] == ci && j < il)) ? 1 : 0;
  }
  s_r[w][lane] = r;
  __syncthreads();
  if (w == 0 && i < F) rank[i] = s_r[0][lane] + s_r[1][lane] + s_r[2][lane] + s_r[3][lane];
}

__global__ __launch_bounds__(1024) void k_level_root_setup(FLevel* desc, FCtl* ctl,
                                                           RootSetupArgs a) {
  __shared__ int ok;
  __shared__ int64_t s_scan[1024];
  __shared__ int64_t s_carry;
  const int64_t F = desc[1].n_rows;
  // root rows in descending rank (row r = frequent item of rank F-1-r); row r owns its pairs
  // with the r rows before it (owner-major order, see the header).  Every class owned → closed
  // form; else a block scan of the owned rows' lengths (row r ↔ root class of rank F-1-r)
  int64_t n_cand;
  if (a.world <= 1) {
    n_cand = F * (F - 1) / 2;
    for (int64_t i = threadIdx.x; i <= F; i += blockDim.x) a.cand_off[i] = i * (i - 1) / 2;
  } else {
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int64_t base = 0; base <= F; base += blockDim.x) {
      const int64_t i = base + threadIdx.x;
      int64_t v = 0;
      if (i < F) {
        const int64_t k = a.prank[F - 1 - i];  // cost rank from level_partition (k_rank_desc)
        const int64_t rnd = k / a.world, p = k % a.world;
        const int64_t owner = (rnd % 2 == 0) ? p : a.world - 1 - p;
        v = owner == a.my_rank ? i : 0;
      }
      s_scan[threadIdx.x] = v;
      __syncthreads();
      for (int off = 1; off < (int)blockDim.x; off <<= 1) {  // Hillis-Steele inclusive
        const int64_t add = (int)threadIdx.x >= off ? s_scan[threadIdx.x - off] : 0;
        __syncthreads();
        s_scan[threadIdx.x] += add;
        __syncthreads();
      }
      if (i <= F) a.cand_off[i] = s_carry + s_scan[threadIdx.x] - v;
      __syncthreads();
      if (threadIdx.x == blockDim.x - 1) s_carry += s_scan[threadIdx.x];
      __syncthreads();
    }
    n_cand = s_carry;
  }
  // gram-driven root: survivor and next-level candidate offsets of the root rows (row r's m
  // frequent pairs become m level-2 rows with 0..m-1 earlier siblings: m(m-1)/2 candidates)
  int64_t S2 = 0, C2 = 0;
  if (a.m) {
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int pass = 0; pass < 2; ++pass) {
      int64_t* outp = pass == 0 ? a.soff : a.coff;
      for (int64_t base = 0; base <= F; base += blockDim.x) {
        const int64_t i = base + threadIdx.x;
        const int64_t mi = i < F ? (int64_t)a.m[i] : 0;
        const int64_t v = pass == 0 ? mi : mi * (mi - 1) / 2;
        s_scan[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < (int)blockDim.x; off <<= 1) {
          const int64_t add = (int)threadIdx.x >= off ? s_scan[threadIdx.x - off] : 0;
          __syncthreads();
          s_scan[threadIdx.x] += add;
          __syncthreads();
        }
        if (i <= F) outp[i] = s_carry + s_scan[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == blockDim.x - 1) s_carry += s_scan[threadIdx.x];
        __syncthreads();
      }
      if (pass == 0) S2 = s_carry; else C2 = s_carry;
      __syncthreads();
      if (threadIdx.x == 0) s_carry = 0;
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    FLevel& r = desc[1];
    r.bm = a.bm;
    r.rank = a.rank;
    r.gid = a.gid;
    r.cand_off = a.cand_off;
    r.n_cand = n_cand;
    r.child_base = F;
    desc[0].child_base = 0;  // level-1 trie nodes [0, F) for the copy-out of "level 0"
    ok = 1;
    if (!a.m) {
      if (F + n_cand > a.out_cap || (n_cand + kTile - 1) / kTile > (int64_t)ctl->status_cap ||
          n_cand >= kRowLimit) {
        fail_capacity(ctl, F + n_cand, a.out_cap);
        ok = 0;
      } else {
        alloc_level(ctl, &desc[2], n_cand, a.Wp);
        if (ctl->overflow) ok = 0;
      }
    } else {
      // level 2 exists now: its rows, and the buffers of its children (unless it is the last)
      FLevel& l2 = desc[2];
      atomicAdd(&ctl->candidates, (unsigned long long)n_cand);
      if (a.leaf) C2 = 0;  // level 2 is the last: no candidates below it
      if (F + S2 + C2 > a.out_cap || (C2 + kTile - 1) / kTile > (int64_t)ctl->status_cap ||
          C2 >= kRowLimit || S2 >= kRowLimit) {
        fail_capacity(ctl, F + S2 + C2, a.out_cap);
        ok = 0;
      } else {
        alloc_level(ctl, &l2, S2, a.Wp);
        l2.n_rows = S2;
        l2.child_base = F + S2;
        l2.n_cand = a.leaf ? 0 : C2;
        if (!a.leaf) alloc_level(ctl, &desc[3], C2, a.Wp);
        if (ctl->overflow) ok = 0;
        else if (!a.leaf) l2.cand_off[S2] = C2;
      }
    }
  }
  __syncthreads();
  if (!ok) return;
  for (int64_t i = threadIdx.x; i < F; i += blockDim.x) {
    // row i ↔ rank F-1-i; level-1 trie node ids stay the ranks
    a.rank[i] = (int32_t)(F - 1 - i);
    a.gid[i] = F - 1 - i;
    a.out_parent[i] = -1;
    a.out_item[i] = a.ids[i];
    a.out_count[i] = a.fcounts[i];
    a.out_depth[i] = 1;
    if (a.m ? a.dl_level1 : a.download) host_store(ctl->h, ctl, i, -1, a.ids[i], a.fcounts[i], 1);
    if (a.host_tab) {
      ctl->host_tab[i] = a.ids[i];
      ((uint32_t*)ctl->host_tab)[ctl->tab_stride + i] = a.fcounts[i];
    }
  }
}

// Frequent pairs per root row: block r scans gram row rank F-1-r beyond the diagonal (its
// pairs with the more frequent items = the root rows before r), contiguous and coalesced.
__global__ __launch_bounds__(256) void k_root_rows(const uint32_t* __restrict__ gram, int64_t ld,
                                                   const FLevel* desc, uint32_t minsup,
                                                   const int32_t* __restrict__ prank, int world,
                                                   int my_rank, int32_t* __restrict__ m) {
  __shared__ int32_t s_w[4];
  const int64_t F = desc[1].n_rows;
  const int64_t r = blockIdx.x;
  if (r >= F) return;
  const int64_t rb = F - 1 - r;
  bool own = true;
  if (world > 1) {
    const int64_t k = prank[rb];
    const int64_t rnd = k / world, p = k % world;
    own = ((rnd % 2 == 0) ? p : world - 1 - p) == my_rank;
  }
  int32_t n = 0;
  if (own)
    for (int64_t ra = rb + 1 + threadIdx.x; ra < F; ra += blockDim.x) n += gram[rb * ld + ra] >= minsup;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) m[r] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// Level 2 from the gram (one block per root row r = owner b): the row's pairs with the earlier
// rows a (a ascending) that are frequent become level-2 rows soff[r] + idx, each with idx earlier
// siblings, i.e. candidates coff[r] + idx(idx-1)/2 ...; their AND bitmaps go to their own slots.
__global__ __launch_bounds__(256) void k_root_fill(FLevel* desc, FCtl* ctl,
                                                   const uint32_t* __restrict__ gram, int64_t ld,
                                                   uint32_t minsup, RootSetupArgs A,
                                                   int32_t* __restrict__ tile_row_nx) {
  __shared__ int64_t s_w[kBlock / 64];
  __shared__ int64_t s_run;
  if (ctl->overflow) return;
  const int64_t F = desc[1].n_rows;
  const int64_t r = blockIdx.x;
  if (r >= F || A.m[r] == 0) return;
  const FLevel& l2 = desc[2];
  const int64_t rb = F - 1 - r;
  const int64_t s0 = A.soff[r], c0 = A.coff[r];
  const int64_t child_base = desc[1].child_base;
  const int64_t scap = (int64_t)ctl->status_cap;
  const int n2 = (int)(A.Wp >> 1);
  const ulonglong2* __restrict__ bm2 = (const ulonglong2*)A.bm;
  ulonglong2* __restrict__ cbm2 = (ulonglong2*)l2.bm;
  int32_t* __restrict__ crank = (int32_t*)l2.rank;
  int64_t* __restrict__ cgid = (int64_t*)l2.gid;
  int32_t* __restrict__ cslot = (int32_t*)l2.slot;
  int64_t* __restrict__ co_nx = l2.cand_off;
  const HostTrie h = ctl->h;
  if (threadIdx.x == 0) s_run = 0;
  for (int64_t a0 = 0; a0 < r; a0 += kBlock) {
    const int64_t a = a0 + threadIdx.x;
    const int64_t ra = F - 1 - a;  // a < r: rank ra > rb
    uint32_t k = 0;
    int flag = 0;
    if (a < r) {
      k = gram[rb * ld + ra];
      flag = k >= minsup ? 1 : 0;
    }
    int64_t tot;
    const int64_t lx = block_excl_scan(flag, s_w, &tot);
    const int64_t idx = s_run + lx;
    if (flag) {
      const int64_t s = s0 + idx;
      const int64_t node = child_base + s;
      crank[s] = (int32_t)ra;
      cgid[s] = node;
      cslot[s] = (int32_t)s;
      const int32_t it = A.ids[ra];
      A.out_parent[node] = rb;
      A.out_item[node] = it;
      A.out_count[node] = k;
      A.out_depth[node] = 2;
      if (A.download) host_store(h, ctl, node, rb, it, k, 2);
      if (!A.leaf) {
        const int64_t co = c0 + idx * (idx - 1) / 2;
        co_nx[s] = co;
        for (int64_t ct = (co + kTile - 1) / kTile; ct * kTile < co + idx; ++ct)
          if (ct < scap) tile_row_nx[ct] = (int32_t)s;
        const ulonglong2* __restrict__ x = bm2 + ra * n2;
        const ulonglong2* __restrict__ y = bm2 + rb * n2;
        // the short-row count kernel reads 64-interleaved slots, the team kernel compact rows
        ulonglong2* __restrict__ z = A.interleaved ? cbm2 + ((s >> 6) * n2 << 6) + (s & 63)
                                                  : cbm2 + s * n2;
        const int zs = A.interleaved ? 64 : 1;
        for (int w0 = 0; w0 < n2; w0 += 6) {
          ulonglong2 u[6], v[6];
#pragma unroll
          for (int q = 0; q < 6; ++q)
            if (w0 + q < n2) {
              u[q] = x[w0 + q];
              v[q] = y[w0 + q];
            }
#pragma unroll
          for (int q = 0; q < 6; ++q)
            if (w0 + q < n2) z[(w0 + q) * zs] = make_ulonglong2(u[q].x & v[q].x, u[q].y & v[q].y);
        }
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_run += tot;
    __syncthreads();
  }
}

int team_size_for(int64_t Wp) {  // lanes per candidate: ~4-8 16-byte chunks per lane
  const int64_t chunks = Wp >> 1;  // 16-byte chunks per row
  if (chunks >= 256) return 64;
  if (chunks >= 128) return 32;
  if (chunks >= 64) return 16;
  if (chunks >= 32) return 8;
  return 4;
}

}  // namespace

int level_grid(int n_cus) { return std::max(64, n_cus * 8); }  // 8 x 256-thread blocks per CU

bool level_rows_interleaved(int64_t Wp) {
  const int64_t n2 = Wp >> 1;
  return n2 >= 1 && n2 <= kSmallChunks;
}

void level_count(FLevel* lv, FLevel* nx, FCtl* ctl, unsigned long long* status, unsigned epoch,
                 const LevelCountArgs& a, const int32_t* tile_row, int32_t* tile_row_nx, int grid,
                 int64_t cand_hint, hipStream_t s) {
  if (a.deferred_dl) grid += a.copy_blocks;
  const int64_t n2 = a.Wp >> 1;
  if (level_rows_interleaved(a.Wp)) {
    // a level expected to be small (the previous call's size: steady-state re-mining) is
    // latency-bound: load each candidate's whole row pair in one batch
    constexpr int64_t kb18_tiles = 64;  // size bound of the one-batch variant
    if (cand_hint >= 0 && cand_hint <= kb18_tiles * kTile && n2 <= 18)
      hipLaunchKernelGGL(k_level_count_small<18>, dim3(grid), dim3(kBlock), 0, s, lv, nx, ctl,
                         status, epoch, a, tile_row, tile_row_nx);
    else
      hipLaunchKernelGGL(k_level_count_small<6>, dim3(grid), dim3(kBlock), 0, s, lv, nx, ctl,
                         status, epoch, a, tile_row, tile_row_nx);
    KMLS_HIP(hipGetLastError());
    return;
  }
  switch (team_size_for(a.Wp)) {
    case 4: hipLaunchKernelGGL(k_level_count<4>, dim3(grid), dim3(kBlock), 0, s, lv, nx, ctl, status, epoch, a, tile_row, tile_row_nx); break;
    case 8: hipLaunchKernelGGL(k_level_count<8>, dim3(grid), dim3(kBlock), 0, s, lv, nx, ctl, status, epoch, a, tile_row, tile_row_nx); break;
    case 16: hipLaunchKernelGGL(k_level_count<16>, dim3(grid), dim3(kBlock), 0, s, lv, nx, ctl, status, epoch, a, tile_row, tile_row_nx); break;
    case 32: hipLaunchKernelGGL(k_level_count<32>, dim3(grid), dim3(kBlock), 0, s, lv, nx, ctl, status, epoch, a, tile_row, tile_row_nx); break;
    default: hipLaunchKernelGGL(k_level_count<64>, dim3(grid), dim3(kBlock), 0, s, lv, nx, ctl, status, epoch, a, tile_row, tile_row_nx); break;
  }
  KMLS_HIP(hipGetLastError());
}

void level_copyout(const FLevel* lv, const FLevel* nx, FCtl* ctl, const int64_t* d_parent,
                   const int32_t* d_item, const uint32_t* d_count, const uint8_t* d_depth,
                   bool download, const void* rb_src, size_t rb_bytes, hipStream_t s) {
  if (rb_bytes % 16) throw std::runtime_error("level_copyout: readback size not a multiple of 16");
  hipLaunchKernelGGL(k_level_copyout, dim3(rb_bytes ? 129 : 128), dim3(kBlock), 0, s, lv, nx, ctl,
                     d_parent, d_item, d_count, d_depth, download, (const uint4*)rb_src,
                     (int)(rb_bytes / 16));
  KMLS_HIP(hipGetLastError());
}

void level_select(const uint32_t* cnt, int64_t n_items, uint32_t c1, int32_t* ids,
                  uint32_t* fcounts, int32_t* rank_of, int32_t* rank_acc, FLevel* desc,
                  hipStream_t s) {
  if (n_items > kSelectMaxItems) throw std::runtime_error("level_select: vocabulary too large");
  const unsigned nb = (unsigned)((n_items + 255) / 256);
  KMLS_HIP(hipMemsetAsync(rank_acc, 0, (size_t)n_items * 4, s));
  hipLaunchKernelGGL(k_select_rank, dim3(nb, nb), dim3(256), 0, s, cnt, n_items, c1, rank_acc);
  hipLaunchKernelGGL(k_select_scatter, dim3(nb), dim3(256), 0, s, cnt, n_items, c1, rank_acc, ids,
                     fcounts, rank_of, desc);
  KMLS_HIP(hipGetLastError());
}

void level_prologue_init(uint32_t* cnt, int64_t n_items, uint64_t* bm, int64_t bm_words,
                         FLevel* desc, int n_desc, FCtl* ctl, const FCtl* params,
                         unsigned int* seq, hipStream_t s) {
  const int64_t work = std::max<int64_t>(std::max<int64_t>(n_items, bm_words), 1);
  const unsigned blocks = (unsigned)std::min<int64_t>((work + 255) / 256, 2048);
  hipLaunchKernelGGL(k_prologue_init, dim3(blocks), dim3(256), 0, s, cnt, n_items, bm, bm_words,
                     desc, n_desc, ctl, params, seq);
  KMLS_HIP(hipGetLastError());
}

void level_select_fused(const uint32_t* cnt, int64_t n_items, uint32_t c1, int32_t* ids,
                        uint32_t* fcounts, int32_t* rank_of, FLevel* desc, const FCtl* ctl,
                        hipStream_t s) {
  if (n_items > kSelectFusedMax) throw std::runtime_error("level_select_fused: vocabulary too large");
  const unsigned nb = (unsigned)((n_items + 15) / 16);
  hipLaunchKernelGGL(k_select_fused, dim3(nb), dim3(256), 0, s, cnt, n_items, c1, ids, fcounts,
                     rank_of, desc, ctl);
  KMLS_HIP(hipGetLastError());
}

void level_partition(const uint32_t* gram, int64_t ld, FLevel* desc, uint32_t minsup,
                     int64_t F_max, int64_t* cost, int32_t* prank, hipStream_t s) {
  hipLaunchKernelGGL(k_root_costs, dim3((unsigned)std::max<int64_t>(F_max, 1)), dim3(256), 0, s,
                     gram, ld, desc, minsup, cost);
  const unsigned nb = (unsigned)std::max<int64_t>((F_max + 63) / 64, 1);
  if (prank) hipLaunchKernelGGL(k_rank_desc, dim3(nb), dim3(256), 0, s, cost, desc, prank);
  KMLS_HIP(hipGetLastError());
}

void level_root_setup(FLevel* desc, FCtl* ctl, const RootSetupArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_level_root_setup, dim3(1), dim3(1024), 0, s, desc, ctl, a);
  KMLS_HIP(hipGetLastError());
}

void level_root_rows(const uint32_t* gram, int64_t ld, const FLevel* desc, uint32_t minsup,
                     const int32_t* prank, int world, int my_rank, int64_t F_max, int32_t* m,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_root_rows, dim3((unsigned)std::max<int64_t>(F_max, 1)), dim3(256), 0, s,
                     gram, ld, desc, minsup, prank, world, my_rank, m);
  KMLS_HIP(hipGetLastError());
}

void level_root_fill(FLevel* desc, FCtl* ctl, const uint32_t* gram, int64_t ld, uint32_t minsup,
                     const RootSetupArgs& a, int32_t* tile_row_nx, int64_t F_max, hipStream_t s) {
  hipLaunchKernelGGL(k_root_fill, dim3((unsigned)std::max<int64_t>(F_max, 1)), dim3(kBlock), 0, s,
                     desc, ctl, gram, ld, minsup, a, tile_row_nx);
  KMLS_HIP(hipGetLastError());
}

int64_t level_tile() { return kTile; }

}  // namespace kern
}  // namespace kmls
