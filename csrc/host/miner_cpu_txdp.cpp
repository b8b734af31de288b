// Transaction-data-parallel miner on the CPU: the protocol of GpuMiner::mine_txdp (tx-DP
// supports, shard-local bitmaps, every level's candidate counts all-reduced) with host kernels
// and the shared-memory communicator, so the multi-rank level loop runs as several processes on
// a machine without any GPU (the CPU test tier; SURVEY §5.8 "loopback / Gloo" test backend).
//
// Level-wise Eclat: level L's rows are itemsets of size L in class order (rows sharing a parent
// are consecutive); a candidate joins row a with a later row b of the same class.  Counts are
// local popcounts over this rank's transaction shard, summed over ranks in chunks, then
// thresholded identically everywhere, so every rank builds the same trie (parents first).
#include <algorithm>
#include <cstring>
#include <vector>

#include "kmls/comm_host.hpp"
#include "kmls/host.hpp"

namespace kmls {

namespace {
constexpr int64_t kChunk = 1 << 22;  // candidates per all-reduce
}

ItemsetTrie mine_cpu_txdp(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx_local,
                          int64_t n_items, int64_t n_tx_global, double min_support, int max_len,
                          ShmComm* comm, MineStats* stats) {
  // 1. global supports
  std::vector<uint32_t> cnt((size_t)n_items);
  count_items(tx_ptr, items, n_tx_local, n_items, cnt.data());
  if (comm) comm->all_reduce(cnt.data(), (size_t)n_items, 4, 0, false);
  FrequentItems fi = select_frequent(cnt.data(), n_items, (uint64_t)n_tx_global, min_support);
  const int64_t F = (int64_t)fi.ids.size();
  const int64_t W = (n_tx_local + 63) / 64;
  ItemsetTrie out;
  for (int64_t r = 0; r < F; ++r) out.push(-1, fi.ids[r], fi.counts[r], 1);
  int64_t cands = 0;
  int maxd = F > 0 ? 1 : 0;
  // level state: rows = (bitmap, last rank, trie id, class id)
  std::vector<uint64_t> bm((size_t)std::max<int64_t>(F * W, 1), 0);
  encode_bitmaps_cpu(tx_ptr, items, n_tx_local, fi.rank_of.data(), bm.data(), W);
  std::vector<int32_t> rank((size_t)F);
  std::vector<int64_t> gid((size_t)F), cls((size_t)F, 0);  // level 1: one class
  for (int64_t r = 0; r < F; ++r) {
    rank[(size_t)r] = (int32_t)r;
    gid[(size_t)r] = r;
  }
  int64_t n = F;
  for (int depth = 1; n >= 2 && (max_len == 0 || depth < max_len); ++depth) {
    // candidate list of this level: (a, b) with b a later row of a's class
    std::vector<int64_t> ca, cb;
    for (int64_t a = 0; a < n; ++a)
      for (int64_t b = a + 1; b < n && cls[(size_t)b] == cls[(size_t)a]; ++b) {
        ca.push_back(a);
        cb.push_back(b);
      }
    const int64_t nc = (int64_t)ca.size();
    if (nc == 0) break;
    cands += nc;
    std::vector<uint32_t> c((size_t)nc);
    for (int64_t k = 0; k < nc; ++k) {
      const uint64_t* x = bm.data() + (size_t)ca[(size_t)k] * W;
      const uint64_t* y = bm.data() + (size_t)cb[(size_t)k] * W;
      uint32_t v = 0;
      for (int64_t w = 0; w < W; ++w) v += (uint32_t)__builtin_popcountll(x[w] & y[w]);
      c[(size_t)k] = v;
    }
    if (comm)
      for (int64_t k0 = 0; k0 < nc; k0 += kChunk)
        comm->all_reduce(c.data() + k0, (size_t)std::min(kChunk, nc - k0), 4, 0, false);
    // survivors → next level (class = the parent row a)
    std::vector<uint64_t> nbm;
    std::vector<int32_t> nrank;
    std::vector<int64_t> ngid, ncls;
    for (int64_t k = 0; k < nc; ++k) {
      if (c[(size_t)k] < fi.minsup2) continue;
      const int64_t a = ca[(size_t)k], b = cb[(size_t)k];
      const int64_t id = out.size();
      out.push(gid[(size_t)a], fi.ids[(size_t)rank[(size_t)b]], c[(size_t)k], (uint8_t)(depth + 1));
      const size_t o = nbm.size();
      nbm.resize(o + (size_t)W);
      const uint64_t* x = bm.data() + (size_t)a * W;
      const uint64_t* y = bm.data() + (size_t)b * W;
      for (int64_t w = 0; w < W; ++w) nbm[o + (size_t)w] = x[w] & y[w];
      nrank.push_back(rank[(size_t)b]);
      ngid.push_back(id);
      ncls.push_back(a);
    }
    if (ngid.empty()) break;
    maxd = depth + 1;
    bm.swap(nbm);
    rank.swap(nrank);
    gid.swap(ngid);
    cls.swap(ncls);
    n = (int64_t)gid.size();
  }
  if (stats) {
    stats->n_frequent_items = F;
    stats->n_itemsets = out.size();
    stats->n_candidates = cands;
    stats->max_depth = maxd;
  }
  return out;
}

}  // namespace kmls
