// Association-rule generation over the itemset trie (SURVEY §2.C O11 "rule_score", J15).
//
// The reference computes confidence rules only in its dead fpgrowth_py path
// (machine-learning/main.py:224-260: every proper non-empty antecedent A of every frequent S,
// conf = supp(S)/supp(A)); mlxtend's association_rules adds lift/leverage/conviction/... .
// Every subset of a frequent itemset is frequent, so supp(A) is always in the trie: A's node is
// reached by walking its items in trie order (the miners extend classes in one global item
// order) through a (parent node, item) → child hash map.  Work is split over threads by itemset;
// output order is deterministic (itemset order, then antecedent bitmask order).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <thread>
#include <unordered_map>
#include <vector>

#include "kmls/host.hpp"

namespace kmls {

namespace {

struct KeyHash {
  size_t operator()(const std::pair<int64_t, int32_t>& k) const {
    uint64_t h = (uint64_t)k.first * 0x9E3779B97F4A7C15ull ^ ((uint64_t)(uint32_t)k.second + 0x632BE59BD9B4E019ull);
    h ^= h >> 31;
    return (size_t)(h * 0xBF58476D1CE4E5B9ull);
  }
};

}  // namespace

RuleSet association_rules_cpu(const int64_t* parent, const int32_t* item, const uint32_t* count,
                              const uint8_t* depth, int64_t n_nodes, int64_t n_tx,
                              RuleMetric metric, double min_threshold, int max_antecedent,
                              int threads) {
  RuleSet out;
  if (n_nodes == 0 || n_tx == 0) return out;
  // child map and root map
  std::unordered_map<std::pair<int64_t, int32_t>, int64_t, KeyHash> child;
  child.reserve((size_t)n_nodes * 2);
  for (int64_t v = 0; v < n_nodes; ++v) child.emplace(std::make_pair(parent[v], item[v]), v);
  auto lookup = [&](const int32_t* items, int k) -> int64_t {
    int64_t node = -1;
    for (int i = 0; i < k; ++i) {
      auto it = child.find(std::make_pair(node, items[i]));
      if (it == child.end()) return -2;
      node = it->second;
    }
    return node;
  };
  const double T = (double)n_tx;
  const int nth = std::max(1, threads > 0 ? threads : default_threads());
  std::vector<RuleSet> parts((size_t)nth);
  std::atomic<int64_t> next{0};
  std::atomic<bool> bad{false};
  constexpr int64_t kBlock = 256;
  auto worker = [&](int tid) {
    RuleSet& rs = parts[(size_t)tid];
    std::vector<int32_t> path, ante, cons;
    while (true) {
      const int64_t b0 = next.fetch_add(kBlock);
      if (b0 >= n_nodes) break;
      const int64_t b1 = std::min(n_nodes, b0 + kBlock);
      for (int64_t s = b0; s < b1; ++s) {
        const int k = depth[s];
        if (k < 2) continue;
        if (k > 30) { bad = true; continue; }
        path.assign((size_t)k, 0);
        int64_t v = s;
        for (int i = k - 1; i >= 0; --i) { path[(size_t)i] = item[v]; v = parent[v]; }
        const double sS = count[s] / T;
        const uint32_t full = (1u << k) - 1u;
        for (uint32_t m = 1; m < full; ++m) {
          const int ka = __builtin_popcount(m);
          if (max_antecedent > 0 && ka > max_antecedent) continue;
          ante.clear();
          cons.clear();
          for (int i = 0; i < k; ++i) ((m >> i) & 1u ? ante : cons).push_back(path[(size_t)i]);
          const int64_t na = lookup(ante.data(), (int)ante.size());
          const int64_t nc = lookup(cons.data(), (int)cons.size());
          if (na < 0 || nc < 0) { bad = true; continue; }
          const double sA = count[na] / T, sC = count[nc] / T;
          // exact count ratios (fpgrowth_py: getSupport(S) / getSupport(A)); a ratio of float
          // supports can land 1 ulp above an exactly-representable threshold
          const double conf = (double)count[s] / (double)count[na];
          const double lift = conf * T / (double)count[nc];
          const double lev = sS - sA * sC;
          double val = 0;
          switch (metric) {
            case RuleMetric::Confidence: val = conf; break;
            case RuleMetric::Lift: val = lift; break;
            case RuleMetric::Leverage: val = lev; break;
            case RuleMetric::Support: val = sS; break;
            case RuleMetric::Conviction: val = conf >= 1.0 ? INFINITY : (1.0 - sC) / (1.0 - conf); break;
            case RuleMetric::ConfidenceStrict: val = conf; break;
          }
          const bool keep = metric == RuleMetric::ConfidenceStrict ? val > min_threshold
                                                                   : val >= min_threshold;
          if (!keep) continue;
          rs.itemset.push_back(s);
          rs.antecedent.push_back(na);
          rs.consequent.push_back(nc);
          rs.confidence.push_back(conf);
          rs.lift.push_back(lift);
        }
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 0; t < nth; ++t) pool.emplace_back(worker, t);
  for (auto& th : pool) th.join();
  KMLS_CHECK(!bad, "association rules: a subset of a frequent itemset is missing from the trie "
                   "(trie not closed under subsets, or itemset longer than 30)");
  // deterministic merge: parts hold disjoint block sets; order by itemset then insertion
  std::vector<std::pair<int64_t, std::pair<int, size_t>>> order;
  for (int t = 0; t < nth; ++t)
    for (size_t i = 0; i < parts[(size_t)t].itemset.size(); ++i)
      order.push_back({parts[(size_t)t].itemset[i], {t, i}});
  std::stable_sort(order.begin(), order.end(),
                   [](const auto& a, const auto& b) { return a.first < b.first; });
  out.reserve(order.size());
  for (auto& o : order) {
    const RuleSet& p = parts[(size_t)o.second.first];
    const size_t i = o.second.second;
    out.itemset.push_back(p.itemset[i]);
    out.antecedent.push_back(p.antecedent[i]);
    out.consequent.push_back(p.consequent[i]);
    out.confidence.push_back(p.confidence[i]);
    out.lift.push_back(p.lift[i]);
  }
  return out;
}

}  // namespace kmls
