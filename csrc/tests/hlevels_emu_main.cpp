// The horizontal levels (csrc/kernels/hlevels.hip: level 2 from the gram, the filtered CSR, the
// hit lists, the Apriori sibling join into the open-addressing candidate table and its CAS
// insert, the flat wave probes with per-wave slot blocks, the compaction into the trie) run on
// the CPU wave emulator under AddressSanitizer/UBSan (tests/test_emu_pairrows.py): every frequent
// itemset of size >= 2 and its support must equal a host depth-first tid-list miner's.
//
//   hlevels_emu <n_tx> <n_items> <max_len> <seed> <min_count> <hooks>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "../kernels/kernels.hpp"

using namespace kmls;
using Set = std::vector<int32_t>;

static void dfs(const std::vector<std::vector<int32_t>>& tids, const std::vector<int32_t>& ids,
                Set& cur, const std::vector<int32_t>& tl, int32_t from, uint32_t minc,
                std::map<Set, uint32_t>& out) {
  for (int32_t r = from; r < (int32_t)ids.size(); ++r) {
    std::vector<int32_t> nt;
    std::set_intersection(tl.begin(), tl.end(), tids[(size_t)r].begin(), tids[(size_t)r].end(),
                          std::back_inserter(nt));
    if (nt.size() < minc) continue;
    cur.push_back(ids[(size_t)r]);
    if (cur.size() >= 2) {
      Set k = cur;
      std::sort(k.begin(), k.end());
      out[k] = (uint32_t)nt.size();
    }
    dfs(tids, ids, cur, nt, r + 1, minc, out);
    cur.pop_back();
  }
}

int main(int argc, char** argv) {
  if (argc < 7) {
    std::fprintf(stderr, "usage: hlevels_emu n_tx n_items max_len seed min_count hooks\n");
    return 2;
  }
  const int64_t T = std::atoll(argv[1]), I = std::atoll(argv[2]);
  const int max_len = std::atoi(argv[3]);
  const unsigned seed = (unsigned)std::atoi(argv[4]);
  const uint32_t minc = (uint32_t)std::atoi(argv[5]);
  if (std::string(argv[6]) != "-") setenv("KMLS_TEST_HOOKS", argv[6], 1);
  std::mt19937_64 rng(seed);
  std::vector<int64_t> ptr(1, 0);
  std::vector<int32_t> items;
  std::geometric_distribution<int> pick(4.0 / (double)I);
  for (int64_t t = 0; t < T; ++t) {
    const int len = (int)(rng() % (uint64_t)(max_len + 1));
    std::vector<int32_t> row;
    while ((int)row.size() < len) {
      const int32_t x = (int32_t)(pick(rng) % I);
      if (std::find(row.begin(), row.end(), x) == row.end()) row.push_back(x);
    }
    items.insert(items.end(), row.begin(), row.end());
    ptr.push_back((int64_t)items.size());
  }
  std::vector<std::vector<int32_t>> tid_of((size_t)I);
  for (int64_t t = 0; t < T; ++t)
    for (int64_t p = ptr[(size_t)t]; p < ptr[(size_t)t + 1]; ++p)
      tid_of[(size_t)items[(size_t)p]].push_back((int32_t)t);
  std::vector<int32_t> ids, rank_of((size_t)I, -1);
  for (int64_t x = 0; x < I; ++x)
    if (tid_of[(size_t)x].size() >= minc) {
      rank_of[(size_t)x] = (int32_t)ids.size();
      ids.push_back((int32_t)x);
    }
  const int64_t F = (int64_t)ids.size();
  std::vector<std::vector<int32_t>> tids((size_t)F);
  for (int64_t r = 0; r < F; ++r) tids[(size_t)r] = tid_of[(size_t)ids[(size_t)r]];
  std::vector<uint32_t> gram((size_t)(F * F), 0u);
  for (int64_t a = 0; a < F; ++a)
    for (int64_t b = a + 1; b < F; ++b) {
      std::vector<int32_t> nt;
      std::set_intersection(tids[(size_t)a].begin(), tids[(size_t)a].end(), tids[(size_t)b].begin(),
                            tids[(size_t)b].end(), std::back_inserter(nt));
      gram[(size_t)(a * F + b)] = (uint32_t)nt.size();
    }
  std::map<Set, uint32_t> want;
  {
    std::vector<int32_t> all((size_t)T);
    for (int64_t t = 0; t < T; ++t) all[(size_t)t] = (int32_t)t;
    Set cur;
    dfs(tids, ids, cur, all, 0, minc, want);
  }
  // the trie: level 1 = ids [0, F) (the ranks), then what HLevels reserves
  std::vector<int64_t> parent((size_t)F, -1);
  std::vector<int32_t> item(ids.begin(), ids.end());
  std::vector<uint32_t> count((size_t)F);
  std::vector<uint8_t> depth((size_t)F, 1);
  for (int64_t r = 0; r < F; ++r) count[(size_t)r] = (uint32_t)tids[(size_t)r].size();
  int64_t used = F;
  kern::HlHooks hk;
  hk.reserve = [&](int64_t n) {
    parent.resize((size_t)(used + n));
    item.resize((size_t)(used + n));
    count.resize((size_t)(used + n));
    depth.resize((size_t)(used + n), 0);
    return kern::HlTrieOut{parent.data(), item.data(), count.data(), depth.data(), used, nullptr};
  };
  hk.commit = [&](int64_t n) { used += n; };
  hk.wait = [] {};
  items.resize(items.size() + 16, -1);
  kern::HlInput in{ptr.data(), items.data(), T, I, rank_of.data(), nullptr, ids.data(),
                   gram.data(), F, F, minc, 0, 2};
  kern::HLevels H;
  kern::HlStats st;
  if (!H.run(in, hk, nullptr, st)) {
    std::fprintf(stderr, "hlevels declined\n");
    return 1;
  }
  std::map<Set, uint32_t> got;
  int64_t bad = 0;
  for (int64_t v = F; v < used; ++v) {
    Set k;
    for (int64_t u = v; u >= 0; u = parent[(size_t)u]) {
      if (u >= (int64_t)item.size()) {
        ++bad;
        break;
      }
      k.push_back(item[(size_t)u]);
      if (u < F) break;
    }
    std::sort(k.begin(), k.end());
    if (k.size() != (size_t)depth[(size_t)v]) ++bad;
    if (!got.emplace(k, count[(size_t)v]).second) ++bad;  // no itemset twice
  }
  if (got != want) {
    int shown = 0;
    for (auto& kv : want) {
      auto it = got.find(kv.first);
      if ((it == got.end() || it->second != kv.second) && shown++ < 5)
        std::fprintf(stderr, "itemset of %zu: want %u, got %d\n", kv.first.size(), kv.second,
                     it == got.end() ? -1 : (int)it->second);
    }
    bad += 1 + (int64_t)std::max(got.size(), want.size()) - (int64_t)std::min(got.size(), want.size());
  }
  std::printf("{\"n_tx\": %lld, \"F\": %lld, \"itemsets\": %zu, \"max_depth\": %d, \"bad\": %lld}\n",
              (long long)T, (long long)F, want.size(), st.max_depth, (long long)bad);
  return bad ? 1 : 0;
}
