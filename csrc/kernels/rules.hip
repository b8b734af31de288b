// O11 rule_score on the GPU: association rules over the itemset trie.
//
// Reference semantics: fpgrowth_py's rule loop (machine-learning/main.py:224-260 — every proper
// non-empty antecedent A of every frequent S, conf = supp(S)/supp(A)) and mlxtend's
// association_rules metrics; CPU twin: csrc/host/rules_cpu.cpp (same output, same order).
//
// Layout: trie nodes are looked up through an open-addressing hash keyed (parent+1, item) → node
// built once per call (k_hash_build).  One wave64 per itemset S (tickets of 16 itemsets):
//   1. S's items: pointer chase to the root, skipped for siblings (consecutive nodes with the
//      same parent share the prefix — the miners emit classes contiguously);
//   2. node(m) for every subset mask m, by rounds over the highest bit b:
//      node(m) = child(node(m - 2^b), item_b) — ONE hash probe per subset, lanes parallel
//      within a round, the table in LDS (k <= 12) or a per-wave global scratch (k <= 18);
//      larger k walks popcount(m) probes per subset;
//   3. every mask 1..2^k-2 in 64-lane chunks: A = node(m), C = node(~m), conf = cnt(S)/cnt(A)
//      (exact count ratio), lift, leverage, conviction; wave ballot compaction.
// Pass 0 counts rules per itemset, an exclusive scan gives offsets, pass 1 writes — output
// order (itemset, then mask) equals the CPU engine's, so results are bit-identical.
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

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kLdsBits = 12;                 // LDS subset table: 4096 int32 per wave
constexpr unsigned long long kEmpty = ~0ull;

__device__ __forceinline__ unsigned long long hkey(int64_t parent, int32_t item) {
  return ((unsigned long long)(parent + 1) << 32) | (unsigned long long)(uint32_t)item;
}
__device__ __forceinline__ unsigned long long hmix(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xFF51AFD7ED558CCDull;
  k ^= k >> 33;
  return k;
}

__global__ void k_hash_build(const int64_t* __restrict__ parent, const int32_t* __restrict__ item,
                             int64_t n, unsigned long long* __restrict__ keys,
                             int32_t* __restrict__ vals, unsigned long long mask) {
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += nthr) {
    const unsigned long long k = hkey(parent[v], item[v]);
    unsigned long long h = hmix(k) & mask;
    while (true) {
      const unsigned long long prev = atomicCAS(&keys[h], kEmpty, k);
      if (prev == kEmpty || prev == k) {
        vals[h] = (int32_t)v;
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

__device__ __forceinline__ int32_t hlookup(const unsigned long long* __restrict__ keys,
                                           const int32_t* __restrict__ vals,
                                           unsigned long long mask, int32_t parent, int32_t item) {
  const unsigned long long k = hkey(parent, item);
  unsigned long long h = hmix(k) & mask;
  while (true) {
    const unsigned long long kk = keys[h];
    if (kk == k) return vals[h];
    if (kk == kEmpty) return -2;
    h = (h + 1) & mask;
  }
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(kBlock) void k_rules(RuleArgs a) {
  __shared__ int32_t s_tab[kWaves][1 << kLdsBits];
  __shared__ int32_t s_path[kWaves][32];
  __shared__ int64_t s_prev_parent[kWaves];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t gwave = (int64_t)blockIdx.x * kWaves + w;
  int32_t* tab_g = a.scratch ? a.scratch + gwave * ((int64_t)1 << a.scratch_bits) : nullptr;
  if (lane == 0) s_prev_parent[w] = -3;
  wave_sync();
  const double T = a.T;
  while (true) {
    int64_t base = 0;
    if (lane == 0) base = (int64_t)atomicAdd(a.ticket, 16ull);
    base = __shfl(base, 0, 64);
    if (base >= a.n) break;
    const int64_t end = min(a.n, base + 16);
    for (int64_t s = base; s < end; ++s) {
      const int k = a.depth[s];
      if (k < 2 || k > 30) {
        if (k > 30 && lane == 0) atomicExch(a.error, 2u);
        if (a.pass == 0 && lane == 0) a.nrules[s] = 0;
        continue;
      }
      // 1. items of S (root → leaf order)
      const int64_t par = a.parent[s];
      if (lane == 0) {
        if (par == s_prev_parent[w]) {
          s_path[w][k - 1] = a.item[s];
        } else {
          int64_t v = s;
          for (int i = k - 1; i >= 0; --i) {
            s_path[w][i] = a.item[v];
            v = a.parent[v];
          }
          s_prev_parent[w] = par;
        }
      }
      wave_sync();
      // 2. subset → node table
      const uint32_t full = (1u << k) - 1u;
      const bool in_lds = k <= kLdsBits;
      const bool in_glb = !in_lds && tab_g != nullptr && k <= a.scratch_bits;
      int32_t* tab = in_lds ? s_tab[w] : tab_g;
      if (in_lds || in_glb) {
        if (lane == 0) tab[0] = -1;
        wave_sync();
        for (int b = 0; b < k; ++b) {
          const uint32_t lo = 1u << b, hi = 2u << b;
          const int32_t it = s_path[w][b];
          for (uint32_t m = lo + lane; m < hi; m += 64) {
            const int32_t p = tab[m - lo];
            tab[m] = p < -1 ? -2 : hlookup(a.keys, a.vals, a.mask, p, it);
          }
          wave_sync();
        }
      }
      // 3. rules over masks 1 .. full-1
      const uint32_t cS = a.count[s];
      const double sS = (double)cS / T;
      int64_t run = a.pass == 1 ? a.off[s] : 0;
      int64_t cnt = 0;
      for (uint32_t m0 = 1; m0 < full; m0 += 64) {
        const uint32_t m = m0 + lane;
        bool keep = false;
        int32_t na = -1, nc = -1;
        double conf = 0.0, lift = 0.0;
        if (m < full && !(a.max_ante > 0 && __builtin_popcount(m) > a.max_ante)) {
          if (in_lds || in_glb) {
            na = tab[m];
            nc = tab[full ^ m];
          } else {  // walk: popcount probes per subset
            na = -1;
            nc = -1;
            for (int i = 0; i < k; ++i) {
              if ((m >> i) & 1u) na = na < -1 ? na : hlookup(a.keys, a.vals, a.mask, na, s_path[w][i]);
              else nc = nc < -1 ? nc : hlookup(a.keys, a.vals, a.mask, nc, s_path[w][i]);
            }
          }
          if (na < 0 || nc < 0) {
            atomicExch(a.error, 1u);
          } else {
            const double cA = (double)a.count[na], cC = (double)a.count[nc];
            conf = (double)cS / cA;
            lift = conf * T / cC;
            const double sA = cA / T, sC = cC / T;
            double val = conf;
            switch (a.metric) {
              case 1: val = lift; break;
              case 2: val = sS - sA * sC; break;
              case 3: val = sS; break;
              case 4: val = conf >= 1.0 ? __builtin_inf() : (1.0 - sC) / (1.0 - conf); break;
              default: break;
            }
            keep = a.metric == 5 ? val > a.thr : val >= a.thr;
          }
        }
        const unsigned long long bal = __ballot(keep);
        if (a.pass == 1 && keep) {
          const int64_t p = run + __builtin_popcountll(bal & ((1ull << lane) - 1ull));
          a.o_itemset[p] = s;
          a.o_ante[p] = na;
          a.o_cons[p] = nc;
          a.o_conf[p] = conf;
          a.o_lift[p] = lift;
        }
        run += __builtin_popcountll(bal);
        cnt += __builtin_popcountll(bal);
      }
      if (a.pass == 0 && lane == 0) a.nrules[s] = cnt;
      wave_sync();
    }
  }
}

}  // namespace

void rules_hash_build(const int64_t* parent, const int32_t* item, int64_t n,
                      unsigned long long* keys, int32_t* vals, unsigned long long mask,
                      hipStream_t s) {
  if (n <= 0) return;
  int g = (int)std::min<int64_t>(8192, (n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_hash_build, dim3(g), dim3(kBlock), 0, s, parent, item, n, keys, vals, mask);
  KMLS_HIP(hipGetLastError());
}

int rules_grid(int n_cus) { return n_cus * 4; }
int rules_waves_per_block() { return kWaves; }

void rules_pass(const RuleArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_rules, dim3(grid), dim3(kBlock), 0, s, a);
  KMLS_HIP(hipGetLastError());
}

size_t rules_scan_temp_bytes(int64_t n) {
  size_t b = 0;
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, (const int64_t*)nullptr, (int64_t*)nullptr,
                                            (int)(n + 1)));
  return b;
}

void rules_scan(const int64_t* in, int64_t* out, int64_t n, void* tmp, size_t tb, hipStream_t s) {
  KMLS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, (int)(n + 1), s));
}

}  // namespace kern
}  // namespace kmls
