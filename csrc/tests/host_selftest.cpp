// Host-runtime self-test for sanitizer builds ("build with -fsanitize on host code
// for CI").  Drives every host component on synthetic data — CSV ingest + group-by, the threaded
// CPU miner (checked against a brute-force count), the threaded rule engine, the matcher — so
// ASan/UBSan (scripts/sanitize_host.sh asan) and TSan (… tsan) see real multi-threaded traffic.
// Exit code 0 = all checks passed.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "kmls/host.hpp"

using namespace kmls;

#define CHECK(c)                                                             \
  do {                                                                       \
    if (!(c)) {                                                              \
      std::fprintf(stderr, "selftest FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

static std::map<std::vector<int32_t>, uint32_t> trie_sets(const ItemsetTrie& t) {
  std::map<std::vector<int32_t>, uint32_t> out;
  std::vector<std::vector<int32_t>> memo(t.item.size());
  for (size_t n = 0; n < t.item.size(); ++n) {
    std::vector<int32_t> s = t.parent[n] >= 0 ? memo[(size_t)t.parent[n]] : std::vector<int32_t>{};
    s.push_back(t.item[n]);
    memo[n] = s;
    std::sort(s.begin(), s.end());
    out[s] = t.count[n];
  }
  return out;
}

int main() {
  // 1. synthetic CSR (multi-threaded generator) + CPU miner vs brute force on a small shape
  std::vector<int64_t> ptr;
  std::vector<int32_t> items;
  synth_transactions(400, 24, 6.0, 4, 0.8, 0.85, 3, 4, ptr, items);
  const int64_t T = (int64_t)ptr.size() - 1;
  MineConfig cfg;
  cfg.min_support = 0.05;
  cfg.threads = 4;
  MineStats st;
  ItemsetTrie t = mine_cpu(ptr.data(), items.data(), T, 24, cfg, &st);
  auto got = trie_sets(t);
  // brute force over every itemset up to size 4 with support >= ceil(ms*T) (level 1: float rule)
  std::vector<std::set<int32_t>> rows((size_t)T);
  for (int64_t r = 0; r < T; ++r) rows[(size_t)r] = std::set<int32_t>(items.begin() + ptr[r], items.begin() + ptr[r + 1]);
  const uint32_t minc = level2_threshold((uint64_t)T, cfg.min_support);
  int checked = 0;
  for (uint32_t m = 1; m < (1u << 24); ++m) {
    if (__builtin_popcount(m) > 3) continue;
    std::vector<int32_t> s;
    for (int i = 0; i < 24; ++i) if (m >> i & 1u) s.push_back(i);
    uint32_t c = 0;
    for (auto& row : rows) {
      bool all = true;
      for (int32_t x : s) if (!row.count(x)) { all = false; break; }
      c += all;
    }
    const bool freq = s.size() == 1 ? level1_frequent(c, (uint64_t)T, cfg.min_support) : c >= minc;
    auto it = got.find(s);
    CHECK(freq == (it != got.end()));
    if (freq) CHECK(it->second == c);
    ++checked;
  }
  std::printf("miner: %zu itemsets, %d subsets brute-forced\n", got.size(), checked);
  // 2. threaded rules engine: confidence of every rule equals count ratio
  RuleSet rs = association_rules_cpu(t.parent.data(), t.item.data(), t.count.data(), t.depth.data(),
                                     (int64_t)t.item.size(), T, RuleMetric::Confidence, 0.3, 0, 4);
  for (size_t i = 0; i < rs.size(); ++i) {
    const double conf = (double)t.count[(size_t)rs.itemset[i]] / (double)t.count[(size_t)rs.antecedent[i]];
    CHECK(conf == rs.confidence[i] && conf >= 0.3);
  }
  std::printf("rules: %zu\n", rs.size());
  // 3. matcher: pair rows from the trie, queries with duplicates / unknown seeds
  const int64_t I = 24;
  std::vector<std::vector<std::pair<int32_t, double>>> adj((size_t)I);
  std::vector<uint8_t> is_key((size_t)I, 0);
  for (size_t n = 0; n < t.item.size(); ++n) {
    if (t.depth[n] == 1) is_key[(size_t)t.item[n]] = 1;
    if (t.depth[n] == 2) {
      const int32_t a = t.item[(size_t)t.parent[n]], b = t.item[n];
      const double sup = (double)t.count[n] / (double)T;
      adj[(size_t)a].push_back({b, sup});
      adj[(size_t)b].push_back({a, sup});
    }
  }
  std::vector<int64_t> rp(1, 0);
  std::vector<int32_t> cons;
  std::vector<double> score;
  for (auto& row : adj) {
    for (auto& e : row) { cons.push_back(e.first); score.push_back(e.second); }
    rp.push_back((int64_t)cons.size());
  }
  RuleIndex ix(I, rp, cons, score, is_key);
  int32_t out[10];
  double sc[10];
  const int32_t q1[] = {0, 1, 1, 23};
  const int n1 = ix.query(q1, 4, 10, out, sc);
  CHECK(n1 >= -1 && n1 <= 10);
  for (int i = 1; i < n1; ++i) CHECK(sc[i - 1] >= sc[i]);
  // 4. CSV ingest + group-by (quotes, embedded commas, escaped quotes)
  const char* path = "/tmp/kmls_selftest.csv";
  {
    std::ofstream f(path);
    f << "pid,track_name,artist_name\n";
    f << "1,\"A, b\",x\n2,\"say \"\"hi\"\"\",y\n1,plain,z\n3,\"A, b\",x\n";
  }
  EncodedTable tb = read_csv_encoded(path, {"pid", "track_name"});
  CHECK(tb.n_rows == 4);
  CHECK(tb.uniques[1].size() == 3);
  CSR g = group_to_csr(tb.codes[0].data(), tb.codes[1].data(), tb.n_rows, (int32_t)tb.uniques[0].size(), true, true);
  CHECK(g.ptr.size() == tb.uniques[0].size() + 1 && g.ptr.back() == 4);
  std::remove(path);
  std::printf("host selftest OK\n");
  return 0;
}
