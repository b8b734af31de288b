// Horizontal levels >= 3 for sparse, long transaction sets (BASELINE config 3: 10M transactions
// x 1M items @2e-4, 14.8k frequent items, ~17k frequent pairs, ~14k itemsets of size >= 3).
//
// The bitmap miners AND two T-bit rows per candidate: at T = 1e7 that is 1.25 MB per candidate
// and an 11.7 ms bitmap encode before the first one, for itemsets whose supports are a few
// thousand.  Here nothing is vertical.  Level 2 comes from the co-occurrence gram (cooc.hip
// counts it from the CSR); every later level is counted from a FILTERED copy of the CSR, in which
// a transaction keeps only the items that occur in some frequent pair (rank order, ascending)
// and only transactions with >= 3 of them survive (k_hl_filter: ~1 % of the nonzeros at config 3).
//
// Counting level k+1 needs, per transaction, the frequent k-itemsets it contains.  Those are the
// previous level's HITS: (transaction, k-itemset node, position of its last item in the
// transaction).  One thread per hit probes (node, y) for every later item y of its transaction in
// a hash table of the level's candidates (siblings joined under a common parent, exactly the
// Apriori join), adds 1 to the candidate's count and appends a new hit.  A transaction contains
// X u {y} once for every containing (X, y) with y after X's last item, so the counts are exact
// supports — and they are sums, so tx-DP ranks all-reduce them (the candidate set is the same on
// every rank: it is built from the previous, all-reduced level).  The survivors (count >=
// minsup) are compacted in candidate order (grouped by parent, items ascending), which is what
// the next join needs, and written straight into the product trie (parents before children).
// The hits of non-surviving candidates are skipped by the next pass through a node map.
//
// Level 2's hits come from a bootstrap pass: every item pair (i < j) of a filtered transaction
// probed in the frequent-pair table.  Sizes cross to the host once per level (candidate total,
// survivor total, hit total); a hit list that outgrows its buffer is re-counted with the exact
// size the counter reached.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "devbuf.hpp"
#include "kernels.hpp"
#include "kmls/common.hpp"
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

constexpr unsigned long long kEmpty = ~0ull;
constexpr int kSortRegs = 16;  // filtered items a thread sorts in registers (longer: in place)

struct alignas(16) HSlot {
  unsigned long long key;  // (node << 16) | item rank; kEmpty = free
  int32_t val;
  int32_t pad;
};

__device__ __forceinline__ unsigned long long hkey(uint32_t node, uint32_t y) {
  return ((unsigned long long)node << 16) | (unsigned long long)y;
}
__device__ __forceinline__ uint32_t hslot(unsigned long long k, uint32_t mask) {
  k *= 0x9E3779B97F4A7C15ull;
  return (uint32_t)(k >> 29) & mask;
}
__device__ __forceinline__ void ht_insert(HSlot* t, uint32_t mask, unsigned long long k, int32_t v) {
  uint32_t h = hslot(k, mask);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long prev = atomicCAS(&t[h].key, kEmpty, k);
    if (prev == kEmpty || prev == k) {
      t[h].val = v;
      return;
    }
    h = (h + 1) & mask;
  }
}
// one 16-byte load per probe (key and value of a slot together)
__device__ __forceinline__ int32_t ht_find(const HSlot* __restrict__ t, uint32_t mask,
                                           unsigned long long k) {
  uint32_t h = hslot(k, mask);
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const ulonglong2 s = *reinterpret_cast<const ulonglong2*>(t + h);
    if (s.x == k) return (int32_t)(uint32_t)s.y;
    if (s.x == kEmpty) return -1;
    h = (h + 1) & mask;
  }
  return -1;
}

__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  uint32_t t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  __syncthreads();
  return t;
}

// ---- level 2 from the gram ----------------------------------------------------------------

__global__ __launch_bounds__(256) void k_hl_row_count(const uint32_t* __restrict__ gram, int64_t ld,
                                                      int64_t F, uint32_t minsup,
                                                      uint32_t* __restrict__ row_cnt) {
  __shared__ uint32_t red[4];
  const int64_t a = blockIdx.x;
  const uint32_t* row = gram + a * ld;
  uint32_t c = 0;
  for (int64_t b = a + 1 + threadIdx.x; b < F; b += 256) c += row[b] >= minsup ? 1u : 0u;
  c = block_sum_u32(c, red);
  if (threadIdx.x == 0) row_cnt[a] = c;
  if (a == 0 && threadIdx.x == 0) row_cnt[F] = 0u;
}

// Row a's frequent pairs (a, b > a), in b order, at [row_off[a], row_off[a+1]).  Level-2 node j:
// parent a, item b, sibling group end row_off[a+1]; (a, b) -> j in the pair table; the trie node
// F + j (parent a, the level-1 node of rank a); both items flagged as pair items.
__global__ __launch_bounds__(256) void k_hl_row_fill(
    const uint32_t* __restrict__ gram, int64_t ld, int64_t F, uint32_t minsup,
    const uint32_t* __restrict__ row_off, uint32_t* __restrict__ lv_par,
    uint32_t* __restrict__ lv_item, uint32_t* __restrict__ lv_end, HSlot* ht, uint32_t hmask,
    uint8_t* __restrict__ inpair, HlTrieOut o) {
  __shared__ uint32_t wsum[4];
  const int64_t a = blockIdx.x;
  const uint32_t* row = gram + a * ld;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t pos = row_off[a];
  const uint32_t end = row_off[a + 1];
  if (pos == end) return;  // (uniform per block: no barrier skipped by part of it)
  inpair[a] = 1;
  for (int64_t b0 = a + 1; b0 < F; b0 += 256) {
    const int64_t b = b0 + threadIdx.x;
    const uint32_t v = b < F ? row[b] : 0u;
    const bool f = b < F && v >= minsup;
    const unsigned long long m = __ballot(f);
    if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (int i = 0; i < 4; ++i) {
      before += i < w ? wsum[i] : 0u;
      total += wsum[i];
    }
    if (f) {
      const uint32_t j = pos + before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      lv_par[j] = (uint32_t)a;
      lv_item[j] = (uint32_t)b;
      lv_end[j] = end;
      ht_insert(ht, hmask, hkey((uint32_t)a, (uint32_t)b), (int32_t)j);
      inpair[b] = 1;
      const int64_t nd = o.base + (int64_t)j;
      o.parent[nd] = a;
      o.item[nd] = o.ids[b];
      o.count[nd] = v;
      o.depth[nd] = 2;
    }
    pos += total;
    __syncthreads();
  }
}

// ---- filtered CSR ------------------------------------------------------------------------

// Hit lists are appended through per-wave blocks of kHitBlk slots (one global atomic per block,
// not per hit: a single counter taking an atomic per wave iteration serialised the first version
// at ~1e8 atomics/s).  The probe loops are FLAT over the wave — 64 sources (transactions or hits)
// per group, their probes enumerated 64 at a time through a prefix of the per-source probe
// counts — so every lane runs every iteration and the block state is wave-uniform.  A wave's
// last block is closed with invalid hits (tx = kNoTx) that the next pass skips.
constexpr int kHitBlk = 256;
constexpr uint32_t kNoTx = 0xFFFFFFFFu;
constexpr int kHW = 4;  // waves per block of the hit kernels

struct HitCursor {
  unsigned long long base = 0;  // next free slot of the wave's block
  unsigned left = 0;            // free slots left in it
};

// slot of this lane's hit (all 64 lanes call it together)
__device__ __forceinline__ unsigned long long hit_slot(bool hit, HitCursor& hc,
                                                       unsigned long long* ctr, int lane) {
  const unsigned long long m = __ballot(hit);
  const unsigned need = (unsigned)__popcll(m);
  const unsigned r = (unsigned)__popcll(m & ((1ull << lane) - 1ull));
  if (need <= hc.left) {
    const unsigned long long slot = hc.base + r;
    hc.base += need;
    hc.left -= need;
    return slot;
  }
  const unsigned rest = need - hc.left;  // <= 64 < kHitBlk
  unsigned long long nb = 0;
  if (lane == 0) nb = atomicAdd(ctr, (unsigned long long)kHitBlk);
  nb = __shfl(nb, 0, 64);
  const unsigned long long slot = r < hc.left ? hc.base + r : nb + (r - hc.left);
  hc.base = nb + rest;
  hc.left = (unsigned)kHitBlk - rest;
  return slot;
}

__device__ __forceinline__ void hit_close(const HitCursor& hc, uint2* __restrict__ h_tn,
                                          unsigned long long hcap, int lane) {
  for (unsigned i = (unsigned)lane; i < hc.left; i += 64u) {
    const unsigned long long slot = hc.base + i;
    if (slot < hcap) h_tn[slot] = make_uint2(kNoTx, 0u);
  }
}

struct HitLds {          // per wave: the group's 64 sources
  uint32_t pst[65];      // probe prefix (exclusive), pst[64] = total
  uint32_t off[64];      // filtered items of the source's transaction
  uint32_t len[64];
  uint32_t tx[64];
  uint32_t node[64];     // count: the source itemset's node (boot: unused)
  uint32_t pos[64];      // count: position of its last item
};

// inclusive scan over the 64 lanes; the wave's total returned in *tot
__device__ __forceinline__ uint32_t wave_incl(uint32_t v, uint32_t* tot, int lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  *tot = __shfl(v, 63, 64);
  return v;
}

__device__ __forceinline__ uint32_t src_of(const HitLds& L, uint32_t p) {
  uint32_t x = 0;
  for (uint32_t step = 32; step; step >>= 1)
    if (L.pst[x + step] <= p) x += step;  // pst[64] = total > p: x stays < 64
  return x;
}

// Level 2's hits: every pair (i < j) of a filtered transaction that is a frequent pair.
__global__ __launch_bounds__(64 * kHW) void k_hl_boot(const uint2* __restrict__ txrec, int64_t n_ftx,
                                                      const uint16_t* __restrict__ fit,
                                                      const HSlot* __restrict__ ht, uint32_t hmask,
                                                      uint2* __restrict__ h_tn, uint16_t* __restrict__ h_pos,
                                                      unsigned long long* hctr, unsigned long long hcap) {
  __shared__ HitLds lds[kHW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  HitLds& L = lds[w];
  HitCursor hc;
  const int64_t groups = (n_ftx + 63) / 64;
  for (int64_t g = (int64_t)blockIdx.x * kHW + w; g < groups; g += (int64_t)gridDim.x * kHW) {
    const int64_t t = g * 64 + lane;
    uint2 rec = make_uint2(0u, 0u);
    if (t < n_ftx) rec = txrec[t];
    const uint32_t P = rec.y * (rec.y - (rec.y > 0u)) / 2u;
    uint32_t tot;
    const uint32_t incl = wave_incl(P, &tot, lane);
    L.pst[lane] = incl - P;
    if (lane == 63) L.pst[64] = incl;
    L.off[lane] = rec.x;
    L.len[lane] = rec.y;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t p0 = 0; p0 < tot; p0 += 64u) {
      const uint32_t p = p0 + (uint32_t)lane;
      int32_t c = -1;
      uint32_t j = 0, x = 0;
      if (p < tot) {
        x = src_of(L, p);
        const uint32_t q = p - L.pst[x];
        const int kk = (int)L.len[x];
        // row-major triangle over (i, j): row i holds kk-1-i pairs, i(2kk-1-i)/2 before it
        const float m2 = (float)(2 * kk - 1);
        int i = (int)((m2 - sqrtf(m2 * m2 - 8.0f * (float)q)) * 0.5f);
        if (i < 0) i = 0;
        while (i > 0 && (uint32_t)(i * (2 * kk - 1 - i) / 2) > q) --i;
        while ((uint32_t)((i + 1) * (2 * kk - 2 - i) / 2) <= q) ++i;
        j = (uint32_t)i + 1u + (q - (uint32_t)(i * (2 * kk - 1 - i) / 2));
        const uint16_t* it = fit + L.off[x];
        c = ht_find(ht, hmask, hkey(it[i], it[j]));
      }
      const bool hit = c >= 0;
      const unsigned long long slot = hit_slot(hit, hc, hctr, lane);
      if (hit && slot < hcap) {
        h_tn[slot] = make_uint2((uint32_t)(g * 64 + x), (uint32_t)c);
        h_pos[slot] = (uint16_t)j;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  hit_close(hc, h_tn, hcap, lane);
}

// Level k+1's counts: per level-k hit (transaction, node through `map` when given, position)
// every later item y of the transaction probes (node, y); flat over the wave's 64 hits.
__global__ __launch_bounds__(64 * kHW) void k_hl_count(
    const uint2* __restrict__ e_tn, const uint16_t* __restrict__ e_pos, int64_t n_e,
    const int32_t* __restrict__ map, const uint2* __restrict__ txrec,
    const uint16_t* __restrict__ fit, const HSlot* __restrict__ ht, uint32_t hmask,
    uint32_t* __restrict__ cnt, uint2* __restrict__ h_tn, uint16_t* __restrict__ h_pos,
    unsigned long long* hctr, unsigned long long hcap) {
  __shared__ HitLds lds[kHW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  HitLds& L = lds[w];
  HitCursor hc;
  const int64_t groups = (n_e + 63) / 64;
  for (int64_t g = (int64_t)blockIdx.x * kHW + w; g < groups; g += (int64_t)gridDim.x * kHW) {
    const int64_t e = g * 64 + lane;
    uint2 tn = make_uint2(kNoTx, 0u);
    uint32_t pos = 0;
    if (e < n_e) {
      tn = e_tn[e];
      pos = e_pos[e];
    }
    int32_t node = -1;
    if (tn.x != kNoTx) node = map ? map[tn.y] : (int32_t)tn.y;
    uint2 rec = make_uint2(0u, 0u);
    if (node >= 0) rec = txrec[tn.x];
    const uint32_t P = rec.y > pos + 1u ? rec.y - pos - 1u : 0u;
    uint32_t tot;
    const uint32_t incl = wave_incl(P, &tot, lane);
    L.pst[lane] = incl - P;
    if (lane == 63) L.pst[64] = incl;
    L.off[lane] = rec.x;
    L.tx[lane] = tn.x;
    L.node[lane] = (uint32_t)node;
    L.pos[lane] = pos;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t p0 = 0; p0 < tot; p0 += 64u) {
      const uint32_t p = p0 + (uint32_t)lane;
      int32_t c = -1;
      uint32_t j = 0, x = 0;
      if (p < tot) {
        x = src_of(L, p);
        j = L.pos[x] + 1u + (p - L.pst[x]);
        c = ht_find(ht, hmask, hkey(L.node[x], fit[L.off[x] + j]));
      }
      const bool hit = c >= 0;
      if (hit) atomicAdd(&cnt[c], 1u);
      const unsigned long long slot = hit_slot(hit, hc, hctr, lane);
      if (hit && slot < hcap) {
        h_tn[slot] = make_uint2(L.tx[x], (uint32_t)c);
        h_pos[slot] = (uint16_t)j;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  hit_close(hc, h_tn, hcap, lane);
}

// ---- candidates ----------------------------------------------------------------------------

__global__ void k_hl_cand_n(const uint32_t* __restrict__ lv_end, int64_t n, uint32_t* __restrict__ cn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) cn[i] = lv_end[i] - (uint32_t)i - 1u;
  if (i == n) cn[n] = 0u;
}

// node i joined with each later sibling j: candidate (parent i, item of j), grouped by i, items
// ascending (siblings are item-ascending)
__global__ void k_hl_cand_fill(const uint32_t* __restrict__ lv_item, const uint32_t* __restrict__ lv_end,
                               const uint32_t* __restrict__ coff, int64_t n,
                               uint32_t* __restrict__ c_par, uint32_t* __restrict__ c_item,
                               HSlot* ht, uint32_t hmask) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t c = coff[i];
  const uint32_t end = lv_end[i];
  for (uint32_t j = (uint32_t)i + 1; j < end; ++j, ++c) {
    const uint32_t y = lv_item[j];
    c_par[c] = (uint32_t)i;
    c_item[c] = y;
    ht_insert(ht, hmask, hkey((uint32_t)i, y), (int32_t)c);
  }
}

__global__ void k_hl_flag(const uint32_t* __restrict__ cnt, int64_t C, uint32_t minsup,
                          uint32_t* __restrict__ flag) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) flag[c] = cnt[c] >= minsup ? 1u : 0u;
  if (c == C) flag[C] = 0u;
}

// survivors -> the next level (compacted in candidate order) + trie nodes; map[c] = new index
// or -1.  A survivor's sibling group ends where its parent's candidates end.
__global__ void k_hl_select(const uint32_t* __restrict__ cnt, int64_t C, uint32_t minsup,
                            const uint32_t* __restrict__ sidx, const uint32_t* __restrict__ c_par,
                            const uint32_t* __restrict__ c_item, const uint32_t* __restrict__ coff,
                            uint32_t* __restrict__ lv_par, uint32_t* __restrict__ lv_item,
                            uint32_t* __restrict__ lv_end, int32_t* __restrict__ map,
                            int64_t parent_base, uint8_t depth, HlTrieOut o) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const uint32_t v = cnt[c];
  if (v < minsup) {
    map[c] = -1;
    return;
  }
  const uint32_t j = sidx[c];
  const uint32_t p = c_par[c];
  const uint32_t y = c_item[c];
  lv_par[j] = p;
  lv_item[j] = y;
  lv_end[j] = sidx[coff[p + 1]];
  map[c] = (int32_t)j;
  const int64_t nd = o.base + (int64_t)j;
  o.parent[nd] = parent_base + (int64_t)p;
  o.item[nd] = o.ids[y];
  o.count[nd] = v;
  o.depth[nd] = depth;
}

template <typename T>
struct Buf {
  T* p = nullptr;
  size_t cap = 0;
  void need(size_t n) {
    if (n <= cap) return;
    if (p) KMLS_HIP(hipFree(p));
    p = nullptr;
    const size_t c = std::max<size_t>(n + (n >> 2), 1024);
    KMLS_HIP(hipMalloc((void**)&p, c * sizeof(T)));
    cap = c;
  }
  ~Buf() {
    if (p) (void)hipFree(p);
  }
};

size_t scan_bytes(int64_t m) {
  size_t b = 0;
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const uint32_t*)nullptr,
                                            (uint32_t*)nullptr, (int)m));
  return b;
}

uint32_t table_mask(int64_t n) {
  uint64_t s = 1024;
  while (s < (uint64_t)n * 2) s <<= 1;
  KMLS_CHECK(s <= (1ull << 31), "hlevels: hash table past 2^31 slots");
  return (uint32_t)(s - 1);
}

// blocks of kHW waves, one 64-source group per wave and round; ~8 blocks per CU resident
unsigned grid_groups(int64_t n, int n_cus) {
  const int64_t groups = (n + 63) / 64;
  const int64_t b = (groups + kHW - 1) / kHW;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, (int64_t)n_cus * 8));
}

unsigned grid_for(int64_t n, int n_cus) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(b, (int64_t)n_cus * 32));
}

}  // namespace

struct HLevels::Impl {
  Buf<uint8_t> inpair;
  Buf<uint16_t> pr;  // item -> pair-item rank
  Buf<uint32_t> row_cnt, row_off;
  Buf<uint32_t> lv_par[2], lv_item[2], lv_end[2];
  Buf<uint32_t> c_par, c_item, c_cnt, c_n, c_off, flag, sidx;
  Buf<int32_t> map;
  Buf<HSlot> ht;
  Buf<uint2> txrec;
  Buf<uint16_t> fit;
  Buf<uint2> tn[2];
  Buf<uint16_t> pos[2];
  Buf<unsigned long long> ctr;
  Buf<unsigned> err;
  Buf<uint8_t> cub;
  unsigned long long* h = nullptr;  // pinned readbacks
  Impl() { KMLS_HIP(hipHostMalloc((void**)&h, 8 * sizeof(unsigned long long), hipHostMallocDefault)); }
  ~Impl() {
    if (h) (void)hipHostFree(h);
  }
  void scan(const uint32_t* in, uint32_t* out, int64_t m, hipStream_t s) {
    KMLS_CHECK(m < (1ll << 31), "hlevels: scan past 2^31 elements");
    size_t b = scan_bytes(m);
    cub.need(b + 256);
    KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(cub.p, b, in, out, (int)m, s));
  }
  // pinned readback of n u32/u64 values (the caller's wait orders it)
  void read_u32(const uint32_t* d, int n, hipStream_t s) {
    KMLS_HIP(hipMemcpyAsync(h, d, (size_t)n * 4, hipMemcpyDeviceToHost, s));
  }
};

HLevels::HLevels() : p_(new Impl) {}
HLevels::~HLevels() { delete p_; }

bool HLevels::run(const HlInput& in, const HlHooks& hk, hipStream_t s, HlStats& st) {
  Impl& I = *p_;
  const int64_t F = in.F;
  st = HlStats{};
  if (F < 2 || in.max_len == 1) return true;
  KMLS_CHECK(F <= kSparseMaxF, "hlevels: item ranks are 16-bit (0xFFFF: none)");
  // ---- level 2: frequent pairs from the gram ----
  I.row_cnt.need((size_t)F + 1);
  I.row_off.need((size_t)F + 1);
  hipLaunchKernelGGL(k_hl_row_count, dim3((unsigned)F), dim3(256), 0, s, in.gram, in.ld, F,
                     in.minsup, I.row_cnt.p);
  KMLS_HIP(hipGetLastError());
  I.scan(I.row_cnt.p, I.row_off.p, F + 1, s);
  I.read_u32(I.row_off.p + F, 1, s);
  hk.wait();
  const int64_t n2 = (int64_t)((uint32_t*)I.h)[0];
  st.per_level.push_back(n2);
  if (n2 == 0) return true;
  int cur = 0;
  I.lv_par[cur].need((size_t)n2);
  I.lv_item[cur].need((size_t)n2);
  I.lv_end[cur].need((size_t)n2 + 1);
  I.inpair.need((size_t)F);
  KMLS_HIP(hipMemsetAsync(I.inpair.p, 0, (size_t)F, s));
  uint32_t hmask = table_mask(n2);
  I.ht.need((size_t)hmask + 1);
  KMLS_HIP(hipMemsetAsync(I.ht.p, 0xFF, ((size_t)hmask + 1) * sizeof(HSlot), s));
  HlTrieOut o = hk.reserve(n2);
  const int64_t base2 = o.base;
  o.ids = in.ids;
  hipLaunchKernelGGL(k_hl_row_fill, dim3((unsigned)F), dim3(256), 0, s, in.gram, in.ld, F,
                     in.minsup, I.row_off.p, I.lv_par[cur].p, I.lv_item[cur].p, I.lv_end[cur].p,
                     I.ht.p, hmask, I.inpair.p, o);
  KMLS_HIP(hipGetLastError());
  hk.commit(n2);
  st.max_depth = 2;
  if (in.max_len == 2) return true;

  // ---- filtered CSR ----
  I.ctr.need(8);
  I.err.need(1);
  KMLS_HIP(hipMemsetAsync(I.err.p, 0, sizeof(unsigned), s));
  // initial capacities (KMLS_TEST_HOOKS hl_cap=<n> shrinks them: the re-count paths)
  const unsigned long long cap0 = (unsigned long long)test_hook("hl_cap", 1ll << 20);
  unsigned long long tx_cap = std::max<unsigned long long>(I.txrec.cap, cap0);
  unsigned long long nnz_cap = std::max<unsigned long long>(I.fit.cap, cap0);
  if (in.f_txrec == nullptr) {  // no rank CSR given: map the items straight to pair-item ranks
    I.pr.need((size_t)std::max<int64_t>(in.n_items, 1));
    KMLS_HIP(hipMemsetAsync(I.pr.p, 0xFF, (size_t)std::max<int64_t>(in.n_items, 1) * 2, s));
    hipLaunchKernelGGL(devbuf::k_rank_map, dim3((unsigned)((F + 255) / 256)), dim3(256), 0, s,
                       in.ids, F, (const uint8_t*)I.inpair.p, I.pr.p);
    KMLS_HIP(hipGetLastError());
  }
  const int64_t f_waves = (int64_t)grid_for(in.n_tx, in.n_cus) * 4;
  const devbuf::PoolRes pres = devbuf::pool_res(in.n_tx, 4.0, f_waves);
  for (int attempt = 0;; ++attempt) {
    I.txrec.need(tx_cap);
    I.fit.need(nnz_cap);
    tx_cap = I.txrec.cap;
    nnz_cap = I.fit.cap;
    KMLS_HIP(hipMemsetAsync(I.ctr.p, 0, sizeof(unsigned long long), s));
    KMLS_HIP(hipMemsetAsync(I.err.p, 0, sizeof(unsigned), s));
    if (in.f_txrec == nullptr)  // (the filter pools' abandoned rows must read as empty)
      KMLS_HIP(hipMemsetAsync(I.txrec.p, 0, (size_t)tx_cap * sizeof(uint2), s));
    if (in.f_txrec != nullptr) {
      if (in.f_rows > 0)
        hipLaunchKernelGGL(devbuf::k_csr_refilter, dim3(grid_for(in.f_rows, in.n_cus)), dim3(256),
                           0, s, in.f_txrec, in.f_rows, in.f_fit, (const uint8_t*)I.inpair.p, 3u,
                           I.txrec.p, I.fit.p, I.ctr.p, tx_cap, nnz_cap);
    } else if (in.n_tx > 0) {
      hipLaunchKernelGGL(devbuf::k_map_filter, dim3(grid_for(in.n_tx, in.n_cus)), dim3(256), 0, s,
                         in.tx_ptr, in.items, in.n_tx, I.pr.p, 3u, I.txrec.p, I.fit.p, I.ctr.p,
                         tx_cap, nnz_cap, I.err.p, pres.rows, pres.items);
    }
    KMLS_HIP(hipGetLastError());
    KMLS_HIP(hipMemcpyAsync(I.h, I.ctr.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    KMLS_HIP(hipMemcpyAsync(I.h + 2, I.err.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    hk.wait();
    const unsigned e = ((unsigned*)(I.h + 2))[0];
    KMLS_CHECK(!(e & 1u), "hlevels: a transaction kept > 65535 items");
    KMLS_CHECK(!(e & 2u), "hlevels: a transaction holds the same frequent item twice");
    const unsigned long long nt = I.h[0] >> devbuf::kPackShift, nn = I.h[0] & devbuf::kPackMask;
    if (nt <= tx_cap && nn <= nnz_cap) {
      I.h[0] = nt;
      I.h[1] = nn;
      break;
    }
    KMLS_CHECK(attempt < 3, "hlevels: filtered CSR sizes grew between passes");
    const bool pooled = in.f_txrec == nullptr;  // the map filter's tails vary run to run
    tx_cap = nt + (pooled ? (unsigned long long)f_waves * pres.rows : 0ull);
    nnz_cap = nn + (pooled ? (unsigned long long)f_waves * pres.items : 0ull);
  }
  const int64_t n_ftx = (int64_t)I.h[0];
  st.n_tx_kept = n_ftx;
  st.nnz_kept = (int64_t)I.h[1];
  KMLS_CHECK(st.nnz_kept < (1ll << 32), "hlevels: filtered CSR past 2^32 items");

  // ---- level 2's hits ----
  int hb = 0;  // hit buffer holding the current level's hits
  int64_t n_hits = 0;
  for (int attempt = 0;; ++attempt) {
    const unsigned long long cap = std::max<unsigned long long>(I.tn[hb].cap, cap0);
    I.tn[hb].need(cap);
    I.pos[hb].need(cap);
    KMLS_HIP(hipMemsetAsync(I.ctr.p + 2, 0, sizeof(unsigned long long), s));
    if (n_ftx > 0)
      hipLaunchKernelGGL(k_hl_boot, dim3(grid_groups(n_ftx, in.n_cus)), dim3(64 * kHW), 0, s, I.txrec.p,
                         n_ftx, I.fit.p, I.ht.p, hmask, I.tn[hb].p, I.pos[hb].p, I.ctr.p + 2,
                         (unsigned long long)std::min(I.tn[hb].cap, I.pos[hb].cap));
    KMLS_HIP(hipGetLastError());
    KMLS_HIP(hipMemcpyAsync(I.h, I.ctr.p + 2, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    hk.wait();
    n_hits = (int64_t)I.h[0];
    if ((size_t)n_hits <= std::min(I.tn[hb].cap, I.pos[hb].cap)) break;
    KMLS_CHECK(attempt == 0, "hlevels: hit count grew between passes");
    I.tn[hb].need((size_t)n_hits);
    I.pos[hb].need((size_t)n_hits);
  }
  st.hits.push_back(n_hits);

  // ---- levels 3, 4, ... ----
  int64_t n_cur = n2, base_cur = base2;
  bool mapped = false;  // the current hits name candidates of the previous count (map them)
  for (int k = 2; in.max_len <= 0 || k < in.max_len; ++k) {
    // candidates of size k+1: each node joined with its later siblings
    I.c_n.need((size_t)n_cur + 1);
    I.c_off.need((size_t)n_cur + 1);
    hipLaunchKernelGGL(k_hl_cand_n, dim3((unsigned)((n_cur + 1 + 255) / 256)), dim3(256), 0, s,
                       I.lv_end[cur].p, n_cur, I.c_n.p);
    KMLS_HIP(hipGetLastError());
    I.scan(I.c_n.p, I.c_off.p, n_cur + 1, s);
    I.read_u32(I.c_off.p + n_cur, 1, s);
    hk.wait();
    const int64_t C = (int64_t)((uint32_t*)I.h)[0];
    st.candidates += C;
    if (C == 0) break;
    // the previous level's map is still needed by this count; candidates go to fresh buffers
    I.c_par.need((size_t)C);
    I.c_item.need((size_t)C);
    I.c_cnt.need((size_t)C);
    hmask = table_mask(C);
    I.ht.need((size_t)hmask + 1);
    KMLS_HIP(hipMemsetAsync(I.ht.p, 0xFF, ((size_t)hmask + 1) * sizeof(HSlot), s));
    hipLaunchKernelGGL(k_hl_cand_fill, dim3((unsigned)((n_cur + 255) / 256)), dim3(256), 0, s,
                       I.lv_item[cur].p, I.lv_end[cur].p, I.c_off.p, n_cur, I.c_par.p,
                       I.c_item.p, I.ht.p, hmask);
    KMLS_HIP(hipGetLastError());
    // count: the current hits probe the candidates, the next level's hits appended
    const int nb = hb ^ 1;
    int64_t n_next_hits = 0;
    for (int attempt = 0;; ++attempt) {
      const unsigned long long cap = std::max<unsigned long long>(I.tn[nb].cap, cap0);
      I.tn[nb].need(cap);
      I.pos[nb].need(cap);
      KMLS_HIP(hipMemsetAsync(I.c_cnt.p, 0, (size_t)C * 4, s));
      KMLS_HIP(hipMemsetAsync(I.ctr.p + 2, 0, sizeof(unsigned long long), s));
      if (n_hits > 0)
        hipLaunchKernelGGL(k_hl_count, dim3(grid_groups(n_hits, in.n_cus)), dim3(64 * kHW), 0, s,
                           I.tn[hb].p, I.pos[hb].p, n_hits, mapped ? I.map.p : nullptr, I.txrec.p,
                           I.fit.p, I.ht.p, hmask, I.c_cnt.p, I.tn[nb].p, I.pos[nb].p,
                           I.ctr.p + 2, (unsigned long long)std::min(I.tn[nb].cap, I.pos[nb].cap));
      KMLS_HIP(hipGetLastError());
      KMLS_HIP(hipMemcpyAsync(I.h, I.ctr.p + 2, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
      hk.wait();
      n_next_hits = (int64_t)I.h[0];
      if ((size_t)n_next_hits <= std::min(I.tn[nb].cap, I.pos[nb].cap)) break;
      KMLS_CHECK(attempt == 0, "hlevels: hit count grew between passes");
      I.tn[nb].need((size_t)n_next_hits);
      I.pos[nb].need((size_t)n_next_hits);
    }
    if (hk.allreduce) hk.allreduce(I.c_cnt.p, C);
    // survivors
    I.flag.need((size_t)C + 1);
    I.sidx.need((size_t)C + 1);
    hipLaunchKernelGGL(k_hl_flag, dim3((unsigned)((C + 1 + 255) / 256)), dim3(256), 0, s, I.c_cnt.p,
                       C, in.minsup, I.flag.p);
    KMLS_HIP(hipGetLastError());
    I.scan(I.flag.p, I.sidx.p, C + 1, s);
    I.read_u32(I.sidx.p + C, 1, s);
    hk.wait();
    const int64_t n_next = (int64_t)((uint32_t*)I.h)[0];
    st.hits.push_back(n_next_hits);
    if (n_next == 0) break;
    st.per_level.push_back(n_next);
    const int nx = cur ^ 1;
    I.lv_par[nx].need((size_t)n_next);
    I.lv_item[nx].need((size_t)n_next);
    I.lv_end[nx].need((size_t)n_next + 1);
    I.map.need((size_t)C);
    HlTrieOut on = hk.reserve(n_next);
    on.ids = in.ids;
    KMLS_CHECK(k + 1 < 256, "hlevels: itemset size past 255");
    hipLaunchKernelGGL(k_hl_select, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, I.c_cnt.p,
                       C, in.minsup, I.sidx.p, I.c_par.p, I.c_item.p, I.c_off.p, I.lv_par[nx].p,
                       I.lv_item[nx].p, I.lv_end[nx].p, I.map.p, base_cur, (uint8_t)(k + 1), on);
    KMLS_HIP(hipGetLastError());
    hk.commit(n_next);
    st.max_depth = k + 1;
    cur = nx;
    n_cur = n_next;
    base_cur = on.base;
    hb = nb;
    n_hits = n_next_hits;
    mapped = true;
  }
  return true;
}

}  // namespace kern
}  // namespace kmls
