// Order-independent content digest of an itemset trie: the bench's and tests' proof that two
// miners produced the SAME frequent itemsets with the SAME supports, not just the same number.
//
// Every node's itemset hash is built along its parent chain as a sum of per-item mixes (so it
// does not depend on the order in which a miner's trie lists the items of an itemset); the
// itemset's digest mixes that with its support count; the trie digest is (count, sum, xor) of
// the mixed itemset digests -- a multiset hash, independent of node order and additive over
// disjoint parts (sum mod 2^64, xor), so per-rank sub-tries combine without moving them.  The
// count-only miners (mine_cpu_count, the GPU deep miner) produce the same digest without a
// trie (kmls/digest.hpp).  Parents must come before children (every miner's trie is built
// that way).
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <stdexcept>
#include <vector>

#include "kmls/digest.hpp"
#include "kmls/host.hpp"

namespace kmls {

namespace {

inline int64_t load_int(const void* p, int w, int64_t i) {
  switch (w) {
    case 2: return ((const uint16_t*)p)[i];
    case 4: return ((const int32_t*)p)[i];
    case 8: return ((const int64_t*)p)[i];
  }
  throw std::runtime_error("trie_digest: unsupported element width " + std::to_string(w));
}

inline uint64_t load_uint(const void* p, int w, int64_t i) {
  switch (w) {
    case 2: return ((const uint16_t*)p)[i];
    case 4: return ((const uint32_t*)p)[i];
    case 8: return ((const uint64_t*)p)[i];
  }
  throw std::runtime_error("trie_digest: unsupported count width " + std::to_string(w));
}

}  // namespace

namespace {

// one size range [lo, hi) of a size-major trie, split over threads (parents are hashed already)
TrieDigest trie_digest_by_size(const void* parent, int pw, const void* item, int iw,
                               const void* count, int cw, const uint8_t* depth, int64_t n,
                               int min_depth, std::vector<uint64_t>& h) {
  const int nt = (int)std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
  TrieDigest d;
  std::string err;
  std::mutex mu;
  int64_t lo = 0;
  while (lo < n) {
    int64_t hi = lo;
    while (hi < n && depth[hi] == depth[lo]) ++hi;
    const int dep = depth[lo];
    std::vector<TrieDigest> part((size_t)nt);
    std::vector<std::thread> th;
    const int64_t per = (hi - lo + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
      th.emplace_back([&, t] {
        const int64_t a = lo + (int64_t)t * per, b = std::min(hi, a + per);
        TrieDigest& pd = part[(size_t)t];
        for (int64_t i = a; i < b; ++i) {
          const int64_t p = pw == 4 ? (int64_t)((const int32_t*)parent)[i] : ((const int64_t*)parent)[i];
          if (p >= lo || p < -1 || (p >= 0 && depth[p] + 1 != dep)) {
            std::lock_guard<std::mutex> lk(mu);
            err = "trie_digest: node " + std::to_string(i) + " has parent " + std::to_string(p) +
                  " (parents must precede children)";
            return;
          }
          const uint64_t set = (p >= 0 ? h[(size_t)p] : 0ull) + item_mix((uint64_t)load_int(item, iw, i));
          h[(size_t)i] = set;
          if (dep < min_depth) continue;
          const DigestTerms tt = digest_terms(set, load_uint(count, cw, i));
          pd.sum += tt.sum;
          pd.xr ^= tt.xr;
          ++pd.n;
        }
      });
    }
    for (auto& x : th) x.join();
    if (!err.empty()) throw std::runtime_error(err);
    if (dep >= min_depth) {
      uint64_t cnt = 0;
      for (auto& pd : part) {
        d.sum += pd.sum;
        d.xr ^= pd.xr;
        cnt += pd.n;
      }
      d.n += cnt;
      if ((int)d.per_depth.size() <= dep) d.per_depth.resize((size_t)dep + 1, 0);
      d.per_depth[(size_t)dep] += cnt;
    }
    lo = hi;
  }
  return d;
}

}  // namespace

TrieDigest trie_digest(const void* parent, int pw, const void* item, int iw, const void* count,
                       int cw, const uint8_t* depth, int64_t n, int min_depth) {
  if (pw != 4 && pw != 8)
    throw std::runtime_error("trie_digest: parent width must be 4 or 8 bytes, got " + std::to_string(pw));
  if (cw != 2 && cw != 4 && cw != 8)
    throw std::runtime_error("trie_digest: count width must be 2, 4 or 8 bytes, got " + std::to_string(cw));
  if (iw != 2 && iw != 4 && iw != 8)
    throw std::runtime_error("trie_digest: item width must be 2, 4 or 8 bytes, got " + std::to_string(iw));
  TrieDigest d;
  std::vector<uint64_t> h((size_t)n);
  if (depth && n >= (1 << 22)) {
    // size-major tries (the deep miner's product trie): every size's nodes depend only on the
    // previous size's hashes, so each size is hashed by all cores (1.4e9 nodes: ~10x faster)
    bool sorted = true;
    for (int64_t i = 1; i < n && sorted; ++i) sorted = depth[i] >= depth[i - 1];
    if (sorted) return trie_digest_by_size(parent, pw, item, iw, count, cw, depth, n, min_depth, h);
  }
  for (int64_t i = 0; i < n; ++i) {
    // parent: signed (-1 = root); 2-byte parents never occur
    int64_t p = pw == 4 ? (int64_t)((const int32_t*)parent)[i] : ((const int64_t*)parent)[i];
    const uint64_t it = (uint64_t)load_int(item, iw, i);
    const uint64_t c = load_uint(count, cw, i);
    if (p >= i || p < -1)
      throw std::runtime_error("trie_digest: node " + std::to_string(i) + " has parent " +
                               std::to_string(p) + " (parents must precede children)");
    const uint64_t set = (p >= 0 ? h[(size_t)p] : 0ull) + item_mix(it);
    h[(size_t)i] = set;
    const int dep = depth ? depth[i] : 0;
    if (depth && dep < min_depth) continue;  // parent-chain only (e.g. replicated level 1)
    const DigestTerms t = digest_terms(set, c);
    d.sum += t.sum;
    d.xr ^= t.xr;
    ++d.n;
    if ((int)d.per_depth.size() <= dep) d.per_depth.resize((size_t)dep + 1, 0);
    d.per_depth[(size_t)dep]++;
  }
  return d;
}

}  // namespace kmls
