// Common types and helpers for the kmls native runtime (host side).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace kmls {

// Compact itemset trie produced by every miner (CPU and HIP):
//   node n = itemset(parent[n]) ∪ {item[n]}, support count count[n]; parent -1 = root.
// Level-1 nodes come first.  This is the whole FP-Growth result: every frequent itemset
// with its support (mlxtend's DataFrame is a materialisation of it).
struct ItemsetTrie {
  std::vector<int64_t> parent;
  std::vector<int32_t> item;   // original item id
  std::vector<uint32_t> count;
  std::vector<uint8_t> depth;  // itemset size
  int64_t size() const { return (int64_t)item.size(); }
  void reserve(size_t n) {
    parent.reserve(n); item.reserve(n); count.reserve(n); depth.reserve(n);
  }
  void push(int64_t p, int32_t it, uint32_t c, uint8_t d) {
    parent.push_back(p); item.push_back(it); count.push_back(c); depth.push_back(d);
  }
};

// Thresholds with mlxtend's exact float semantics.
inline bool level1_frequent(uint64_t count, uint64_t n_tx, double min_support) {
  return ((double)count / (double)n_tx) >= min_support;
}
uint32_t level2_threshold(uint64_t n_tx, double min_support);  // ceil(ms * T) in double
uint32_t level1_threshold(uint64_t n_tx, double min_support);  // min c with c/T >= ms

struct MineConfig {
  double min_support = 0.05;
  int max_len = 0;          // 0 = unbounded
  int threads = 0;          // 0 = hardware_concurrency
  bool pairs_only = false;  // stop after 2-itemsets (rule-map fast path)
  bool level2_gram = true;  // GPU: level 2 through the tiled bit-GEMM
  bool level2_mfma = false; // GPU: ... on the i8 matrix cores instead of VALU popcount
  bool rule_index = false;  // GPU resident path: also build the rule map (pair-support CSR,
                            // machine-learning/main.py:282-304) on the device and download it
};

// Frequent-item selection shared by all miners: ids ordered by ascending support
// (ties by id), as the Eclat class order.
struct FrequentItems {
  std::vector<int32_t> ids;       // frequent item ids, ascending support
  std::vector<uint32_t> counts;   // their supports
  std::vector<int32_t> rank_of;   // item id -> position in ids, or -1
  uint32_t minsup2 = 0;           // count threshold for |S| >= 2
};
FrequentItems select_frequent(const uint32_t* item_counts, int64_t n_items, uint64_t n_tx,
                              double min_support);

#define KMLS_CHECK(cond, msg)                                              \
  do {                                                                     \
    if (!(cond)) throw std::runtime_error(std::string("kmls: ") + (msg)); \
  } while (0)

// Worker threads when a caller passes 0: OMP_NUM_THREADS if set (the GPU pool exports the
// process's CPU share there; hardware_concurrency() reports the whole host), else all cores.
int default_threads();

}  // namespace kmls
