// Host-side (CPU) native runtime API: CSV ingest, CSR build, CPU miner, CPU matcher.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "kmls/common.hpp"

namespace kmls {

// ---- ingest -------------------------------------------------------------------------------
struct EncodedTable {
  int64_t n_rows = 0;
  std::vector<std::string> header;
  std::vector<std::string> columns;                  // requested columns
  std::vector<std::vector<int32_t>> codes;           // per column, per row: dictionary code
  std::vector<std::vector<std::string>> uniques;     // per column: code -> string
};
EncodedTable read_csv_encoded(const std::string& path, const std::vector<std::string>& wanted);

struct CSR {
  std::vector<int64_t> ptr;
  std::vector<int32_t> idx;
};
// Group `vals` by `keys` (codes in [0, n_keys)), preserving row order inside a group unless
// sort_rows/dedup are requested.
CSR group_to_csr(const int32_t* keys, const int32_t* vals, int64_t n, int32_t n_keys, bool dedup,
                 bool sort_rows);

// ---- CPU miner (bitmap Eclat, std::thread) -------------------------------------------------
// CSR rows must be duplicate-free.  Produces the complete FP-Growth itemset set.
struct MineStats {
  int64_t n_frequent_items = 0;
  int64_t n_itemsets = 0;
  int64_t n_candidates = 0;
  int max_depth = 0;
  double seconds = 0.0;
};
ItemsetTrie mine_cpu(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, int64_t n_items,
                     const MineConfig& cfg, MineStats* stats);

// Same search from prebuilt item-major bitmaps [F][W] (the multi-rank protocol's replicated
// bitmaps); `owned` (size F, optional) restricts the root classes expanded by this rank.
ItemsetTrie mine_cpu_bitmaps(const uint64_t* bm, int64_t F, int64_t W, const FrequentItems& fi,
                             int max_len, int threads, const uint8_t* owned, MineStats* stats);
void encode_bitmaps_cpu(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                        const int32_t* rank_of, uint64_t* bm, int64_t W);

class ShmComm;
// Transaction-data-parallel CPU miner (miner_cpu_txdp.cpp): this rank holds a transaction shard;
// supports and every level's candidate counts are all-reduced through `comm` (nullptr: world
// size 1), so every rank returns the identical global trie (level order, parents first).
ItemsetTrie mine_cpu_txdp(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx_local,
                          int64_t n_items, int64_t n_tx_global, double min_support, int max_len,
                          ShmComm* comm, MineStats* stats);

// Count-only search: per-level itemset totals and the content digest (the one trie_digest gives
// for the full trie) without a trie; stops once the running total exceeds `cap` (capped = true,
// counts are then a lower bound).  The CPU reference of the GPU count-only (deep) miner.
// rank/world: this rank's share of a split problem (levels 1-2 on rank 0, level-3 task q on
// rank q % world); summing per_level / digest_sum and xoring digest_xor over the ranks gives
// the whole problem.
struct CountResult {
  std::vector<int64_t> per_level;  // [d] = #frequent itemsets of size d (index 0 unused)
  int64_t n_frequent_items = 0, n_itemsets = 0;
  int max_depth = 0;
  bool capped = false;
  double seconds = 0.0;
  uint64_t digest_sum = 0, digest_xor = 0;  // content digest (kmls/digest.hpp); partial if capped
};
CountResult mine_cpu_count(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                           int64_t n_items, double min_support, int max_len, int64_t cap,
                           int threads, int rank = 0, int world = 1);

// Order-independent content digest of an itemset trie (digest.cpp): equal digests <=> (with
// overwhelming probability) the same multiset of (itemset, support).  Element widths in bytes:
// parent 4|8, item 2|4|8, count 2|4.
struct TrieDigest {
  int64_t n = 0;
  uint64_t sum = 0, xr = 0;
  std::vector<int64_t> per_depth;
};
TrieDigest trie_digest(const void* parent, int pw, const void* item, int iw, const void* count,
                       int cw, const uint8_t* depth, int64_t n, int min_depth = 0);

// Pair supports among frequent items (rule-map fast path).
struct PairTable {
  std::vector<int32_t> a, b;     // item ids, a has lower Eclat rank than b
  std::vector<uint32_t> count;
};
void count_items(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, int64_t n_items,
                 uint32_t* out_counts);

// ---- association rules (rules_cpu.cpp) ------------------------------------------------------
enum class RuleMetric { Confidence = 0, Lift = 1, Leverage = 2, Support = 3, Conviction = 4,
                        ConfidenceStrict = 5 /* fpgrowth_py: conf > minConf */ };
struct RuleSet {  // rule r: antecedent node -> consequent node (trie ids), from itemset node
  std::vector<int64_t> itemset, antecedent, consequent;
  std::vector<double> confidence, lift;
  void reserve(size_t n) {
    itemset.reserve(n); antecedent.reserve(n); consequent.reserve(n);
    confidence.reserve(n); lift.reserve(n);
  }
  size_t size() const { return itemset.size(); }
};
RuleSet association_rules_cpu(const int64_t* parent, const int32_t* item, const uint32_t* count,
                              const uint8_t* depth, int64_t n_nodes, int64_t n_tx,
                              RuleMetric metric, double min_threshold, int max_antecedent,
                              int threads);

// ---- CPU matcher ---------------------------------------------------------------------------
// Rule index: for each key item, an ordered row of (consequent, score).  Rows may be empty
// (frequent songs without pairs are keys with `{}`; rest_api/app/main.py:235 distinguishes
// "key with empty row" from "not a key").
class RuleIndex {
 public:
  RuleIndex(int64_t n_items, std::vector<int64_t> row_ptr, std::vector<int32_t> cons,
            std::vector<double> score, std::vector<uint8_t> is_key);
  int64_t n_items() const { return n_items_; }
  int64_t nnz() const { return (int64_t)cons_.size(); }
  // Reference matcher semantics (rest_api/app/main.py:235-254): present seeds in request
  // order; max-merge; stable sort by score desc (ties: first-insertion order); top-k.
  // Returns -1 when no seed is a key (caller falls back), else the number of results.
  int query(const int32_t* seeds, int n_seeds, int k, int32_t* out_ids, double* out_scores) const;
  const std::vector<int64_t>& row_ptr() const { return row_ptr_; }
  const std::vector<int32_t>& cons() const { return cons_; }
  const std::vector<double>& score() const { return score_; }
  const std::vector<uint8_t>& is_key() const { return is_key_; }

 private:
  int64_t n_items_;
  std::vector<int64_t> row_ptr_;
  std::vector<int32_t> cons_;
  std::vector<double> score_;
  std::vector<uint8_t> is_key_;
};

// Multi-threaded synthetic transactions (csrc/host/synth.cpp): CSR with sorted, unique items.
void synth_transactions(int64_t n_tx, int64_t n_items, double mean_len, int n_genres,
                        double affinity, double zipf_s, uint64_t seed, int threads,
                        std::vector<int64_t>& tx_ptr, std::vector<int32_t>& items,
                        int64_t tx_begin = 0, int64_t tx_end = -1);

}  // namespace kmls
