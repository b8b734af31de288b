// CPU bitmap-Eclat miner: the native CPU path (MINER=cpu) and the fast oracle for the HIP miner.
//
// Produces exactly the itemset set of mlxtend.fpgrowth (machine-learning/main.py:272; semantics
// in SURVEY Appendix A): level 1 uses `count/T >= ms`, deeper levels `count >= ceil(ms*T)`.
// The reference's pure-Python FP-tree recursion is replaced by vertical tid-bitmaps:
// support(P ∪ {b}) = popcount(bits(P) & bits(b)).  Work is split over threads by top-level
// equivalence class (dynamic scheduling); output order is deterministic (class order).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include <cstdlib>
#include <functional>
#include <stdexcept>

#include "kmls/common.hpp"
#include "kmls/digest.hpp"
#include "kmls/host.hpp"

namespace kmls {

int default_threads() {
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int n = std::atoi(e);
    if (n > 0) return n;
  }
  return std::max(1, (int)std::thread::hardware_concurrency());
}

uint32_t level2_threshold(uint64_t n_tx, double min_support) {
  return (uint32_t)std::ceil(min_support * (double)n_tx);
}

uint32_t level1_threshold(uint64_t n_tx, double min_support) {
  double guess = std::floor(min_support * (double)n_tx);
  int64_t c = std::max<int64_t>(0, (int64_t)guess - 2);
  while (!level1_frequent((uint64_t)c, n_tx, min_support)) ++c;
  while (c > 0 && level1_frequent((uint64_t)(c - 1), n_tx, min_support)) --c;
  return (uint32_t)c;
}

FrequentItems select_frequent(const uint32_t* cnt, int64_t n_items, uint64_t n_tx,
                              double min_support) {
  FrequentItems f;
  f.rank_of.assign((size_t)n_items, -1);
  for (int64_t i = 0; i < n_items; ++i)
    if (n_tx > 0 && level1_frequent(cnt[i], n_tx, min_support)) f.ids.push_back((int32_t)i);
  std::stable_sort(f.ids.begin(), f.ids.end(),
                   [&](int32_t a, int32_t b) { return cnt[a] < cnt[b]; });
  f.counts.resize(f.ids.size());
  for (size_t r = 0; r < f.ids.size(); ++r) {
    f.rank_of[f.ids[r]] = (int32_t)r;
    f.counts[r] = cnt[f.ids[r]];
  }
  f.minsup2 = level2_threshold(n_tx, min_support);
  return f;
}

void count_items(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, int64_t n_items,
                 uint32_t* out) {
  std::fill(out, out + n_items, 0u);
  for (int64_t i = tx_ptr[0]; i < tx_ptr[n_tx]; ++i) out[items[i]]++;
}

namespace {

// A class member: `off` >= 0 is an offset into the thread's arena, < 0 encodes the
// top-level bitmap of Eclat rank (-1 - off).  Offsets (not pointers) because the arena grows.
struct Member {
  int32_t rank;
  uint32_t cnt;
  int64_t off;
  int64_t node;  // task-local node id (>=0) or -1-global for level-1 nodes
};

struct Task {
  std::vector<int64_t> parent;  // >=0 local, <0 : -1-global
  std::vector<int32_t> item;
  std::vector<uint32_t> count;
  std::vector<uint8_t> depth;
  int64_t candidates = 0;
  int max_depth = 0;
};

struct Ctx {
  const FrequentItems* fi;
  const uint64_t* top_bm;  // [F][W]
  int64_t W;
  uint32_t minsup;
  int max_len;
};

inline const uint64_t* resolve(const Ctx& cx, const std::vector<uint64_t>& arena, int64_t off) {
  return off >= 0 ? arena.data() + off : cx.top_bm + (-1 - off) * cx.W;
}

// Expand member i of class `cls` (itemset size `depth`): intersect it with every later member,
// emit the frequent ones, then recurse into the child class.  Child bitmaps are bump-allocated
// at `top` in the per-thread arena.
void expand_member(const Ctx& cx, const std::vector<Member>& cls, size_t i, int depth,
                   std::vector<uint64_t>& arena, size_t top, Task& task) {
  const int64_t W = cx.W;
  const size_t need = top + (cls.size() - i - 1) * (size_t)W;
  if (arena.size() < need) arena.resize(need + (need >> 1) + 1024);
  const Member a = cls[i];
  const uint64_t* x = resolve(cx, arena, a.off);
  std::vector<Member> child;
  size_t cur = top;
  for (size_t j = i + 1; j < cls.size(); ++j) {
    const uint64_t* y = resolve(cx, arena, cls[j].off);
    uint64_t* o = arena.data() + cur;
    uint32_t c = 0;
    for (int64_t w = 0; w < W; ++w) {
      uint64_t v = x[w] & y[w];
      o[w] = v;
      c += (uint32_t)__builtin_popcountll(v);
    }
    ++task.candidates;
    if (c >= cx.minsup) {
      int64_t id = (int64_t)task.item.size();
      task.parent.push_back(a.node);
      task.item.push_back(cx.fi->ids[cls[j].rank]);
      task.count.push_back(c);
      task.depth.push_back((uint8_t)(depth + 1));
      child.push_back(Member{cls[j].rank, c, (int64_t)cur, id});
      cur += (size_t)W;
    }
  }
  if (!child.empty() && depth + 1 > task.max_depth) task.max_depth = depth + 1;
  if (child.size() >= 2 && (cx.max_len == 0 || depth + 1 < cx.max_len)) {
    for (size_t k = 0; k + 1 < child.size(); ++k) expand_member(cx, child, k, depth + 1, arena, cur, task);
  }
}

// Count-only search: no trie; per-level totals plus the content digest of every frequent itemset
// (kmls/digest.hpp: the same digest trie_digest computes from a miner's trie), so a count-only
// GPU result is checked by content, not just by number.  Stops once the shared counter passes
// `cap` (calibration / feasibility probes of outputs too big to hold).
struct CMember {
  int32_t rank;
  int64_t off;  // >= 0: offset into the thread arena; < 0: level-2 row (-1 - off) of the shared store
  uint64_t h;   // set hash of the member's itemset
};

struct CountCtx {
  const uint64_t* l2_bm;  // [#pairs][W] level-2 bitmaps (shared, read-only)
  const int32_t* ids;     // rank -> original item id
  int64_t W;
  uint32_t minsup;
  int max_len;
  int64_t cap;
  std::atomic<int64_t>* total;
};

struct CountAcc {
  std::vector<int64_t> per_level;
  uint64_t sum = 0, xr = 0;
  void add(int depth, uint64_t h, uint32_t c) {
    if ((int)per_level.size() <= depth) per_level.resize((size_t)depth + 1, 0);
    per_level[(size_t)depth]++;
    const DigestTerms t = digest_terms(h, c);
    sum += t.sum;
    xr ^= t.xr;
  }
};

// expand member i of class `cls` (itemsets of size `depth`): every later member j gives the
// candidate cls[i] ∪ cls[j]
void count_member(const CountCtx& cx, const std::vector<CMember>& cls, size_t i, int depth,
                  std::vector<uint64_t>& arena, size_t top, CountAcc& acc) {
  if (cx.total->load(std::memory_order_relaxed) > cx.cap) return;
  const int64_t W = cx.W;
  const size_t need = top + (cls.size() - i - 1) * (size_t)W;
  if (arena.size() < need) arena.resize(need + (need >> 1) + 1024);
  auto res = [&](int64_t off) {
    return off >= 0 ? arena.data() + off : cx.l2_bm + (-1 - off) * W;
  };
  const CMember a = cls[i];
  std::vector<CMember> child;
  size_t cur = top;
  const uint64_t* x = res(a.off);  // the arena does not move inside this loop (reserved above)
  for (size_t j = i + 1; j < cls.size(); ++j) {
    const uint64_t* y = res(cls[j].off);
    uint64_t* o = arena.data() + cur;
    uint32_t c = 0;
    for (int64_t w = 0; w < W; ++w) {
      const uint64_t v = x[w] & y[w];
      o[w] = v;
      c += (uint32_t)__builtin_popcountll(v);
    }
    if (c >= cx.minsup) {
      const uint64_t h = a.h + item_mix((uint64_t)cx.ids[cls[j].rank]);
      acc.add(depth + 1, h, c);
      child.push_back(CMember{cls[j].rank, (int64_t)cur, h});
      cur += (size_t)W;
    }
  }
  if (!child.empty()) cx.total->fetch_add((int64_t)child.size(), std::memory_order_relaxed);
  if (child.size() >= 2 && (cx.max_len == 0 || depth + 1 < cx.max_len)) {
    for (size_t k = 0; k + 1 < child.size(); ++k)
      count_member(cx, child, k, depth + 1, arena, cur, acc);
  }
}

}  // namespace

CountResult mine_cpu_count(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                           int64_t n_items, double min_support, int max_len, int64_t cap,
                           int threads, int rank, int world) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("mine_cpu_count: bad rank/world");
  auto t0 = std::chrono::steady_clock::now();
  std::vector<uint32_t> cnt((size_t)n_items);
  count_items(tx_ptr, items, n_tx, n_items, cnt.data());
  FrequentItems fi = select_frequent(cnt.data(), n_items, (uint64_t)n_tx, min_support);
  const int64_t F = (int64_t)fi.ids.size();
  const int64_t W = (n_tx + 63) / 64;
  std::vector<uint64_t> bm((size_t)(F * W), 0);
  encode_bitmaps_cpu(tx_ptr, items, n_tx, fi.rank_of.data(), bm.data(), W);
  CountResult r;
  CountAcc all;
  if (rank == 0)
    for (int64_t j = 0; j < F; ++j) all.add(1, item_mix((uint64_t)fi.ids[j]), fi.counts[j]);
  std::atomic<int64_t> total{F};
  int nth = threads > 0 ? threads : default_threads();
  nth = std::max(1, std::min<int>(nth, (int)std::max<int64_t>(F, 1)));
  auto run_pool = [&](const std::function<void(int)>& fn) {
    std::vector<std::thread> pool;
    for (int t = 0; t < nth; ++t) pool.emplace_back(fn, t);
    for (auto& th : pool) th.join();
  };
  if (F >= 2 && max_len != 1) {
    // level 2 (parallel over root classes): every root item's class of frequent pairs, stored
    // once and shared, so level-3 classes become the unit of dynamic scheduling (a dense root
    // class no longer lands on one thread)
    std::vector<std::vector<uint64_t>> l2b((size_t)F);
    std::vector<std::vector<int32_t>> l2r((size_t)F);
    std::vector<std::vector<uint32_t>> l2c((size_t)F);
    std::atomic<int64_t> next{0};
    run_pool([&](int) {
      std::vector<uint64_t> row((size_t)W);
      while (true) {
        const int64_t i = next.fetch_add(1);
        if (i >= F - 1) break;
        const uint64_t* x = bm.data() + i * W;
        for (int64_t j = i + 1; j < F; ++j) {
          const uint64_t* y = bm.data() + j * W;
          uint32_t c = 0;
          for (int64_t w = 0; w < W; ++w) {
            row[(size_t)w] = x[w] & y[w];
            c += (uint32_t)__builtin_popcountll(row[(size_t)w]);
          }
          if (c >= fi.minsup2) {
            l2b[(size_t)i].insert(l2b[(size_t)i].end(), row.begin(), row.end());
            l2r[(size_t)i].push_back((int32_t)j);
            l2c[(size_t)i].push_back(c);
          }
        }
      }
    });
    std::vector<int64_t> base((size_t)F + 1, 0);
    for (int64_t i = 0; i < F; ++i) base[(size_t)i + 1] = base[(size_t)i] + (int64_t)l2r[(size_t)i].size();
    std::vector<uint64_t> l2((size_t)(base[(size_t)F] * W));
    std::vector<std::vector<CMember>> cls((size_t)F);
    for (int64_t i = 0; i < F; ++i) {
      std::copy(l2b[(size_t)i].begin(), l2b[(size_t)i].end(), l2.begin() + base[(size_t)i] * W);
      std::vector<uint64_t>().swap(l2b[(size_t)i]);
      const uint64_t hi = item_mix((uint64_t)fi.ids[(size_t)i]);
      for (size_t k = 0; k < l2r[(size_t)i].size(); ++k) {
        const uint64_t h = hi + item_mix((uint64_t)fi.ids[(size_t)l2r[(size_t)i][k]]);
        if (rank == 0) all.add(2, h, l2c[(size_t)i][k]);
        cls[(size_t)i].push_back(CMember{l2r[(size_t)i][k], -1 - (base[(size_t)i] + (int64_t)k), h});
      }
    }
    total.fetch_add(base[(size_t)F]);
    // levels >= 3: tasks (root class i, member k)
    if (max_len == 0 || max_len > 2) {
      std::vector<std::pair<int32_t, int32_t>> tasks;
      uint64_t tasks_seen = 0;
      for (int64_t i = 0; i < F; ++i)
        for (size_t k = 0; k + 1 < cls[(size_t)i].size(); ++k) {
          if ((int64_t)(tasks_seen++ % (uint64_t)world) == rank) tasks.push_back({(int32_t)i, (int32_t)k});
        }
      CountCtx cx{l2.data(), fi.ids.data(), W, fi.minsup2, max_len, cap, &total};
      std::vector<CountAcc> acc((size_t)nth);
      std::atomic<int64_t> nt{0};
      run_pool([&](int t) {
        std::vector<uint64_t> arena;
        while (true) {
          const int64_t q = nt.fetch_add(1);
          if (q >= (int64_t)tasks.size() || total.load(std::memory_order_relaxed) > cap) break;
          count_member(cx, cls[(size_t)tasks[(size_t)q].first], (size_t)tasks[(size_t)q].second, 2,
                       arena, 0, acc[(size_t)t]);
        }
      });
      for (auto& a : acc) {
        if (a.per_level.size() > all.per_level.size()) all.per_level.resize(a.per_level.size(), 0);
        for (size_t d = 0; d < a.per_level.size(); ++d) all.per_level[d] += a.per_level[d];
        all.sum += a.sum;
        all.xr ^= a.xr;
      }
    }
  }
  r.per_level = all.per_level;
  if (r.per_level.size() < 2) r.per_level.resize(2, 0);
  r.per_level[0] = 0;
  r.digest_sum = all.sum;
  r.digest_xor = all.xr;
  r.n_frequent_items = F;
  r.n_itemsets = 0;
  for (size_t d = 1; d < r.per_level.size(); ++d) r.n_itemsets += r.per_level[d];
  r.capped = total.load() > cap;
  r.max_depth = 0;
  for (size_t d = 1; d < r.per_level.size(); ++d)
    if (r.per_level[d] > 0) r.max_depth = (int)d;
  r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

ItemsetTrie mine_cpu_bitmaps(const uint64_t* bm, int64_t F, int64_t W, const FrequentItems& fi,
                             int max_len, int threads, const uint8_t* owned, MineStats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  ItemsetTrie out;
  for (int64_t r = 0; r < F; ++r) out.push(-1, fi.ids[r], fi.counts[r], 1);
  std::vector<Task> tasks((size_t)std::max<int64_t>(F, 0));
  if (F >= 2 && max_len != 1) {
    Ctx cx{&fi, bm, W, fi.minsup2, max_len};
    int nth = threads > 0 ? threads : default_threads();
    nth = std::max(1, std::min<int>(nth, (int)F));
    std::atomic<int64_t> next{0};
    std::vector<Member> root((size_t)F);
    for (int64_t j = 0; j < F; ++j) root[(size_t)j] = Member{(int32_t)j, fi.counts[j], -1 - j, -1 - j};
    auto worker = [&]() {
      std::vector<uint64_t> arena;
      while (true) {
        int64_t i = next.fetch_add(1);
        if (i >= F - 1) break;
        if (owned && !owned[i]) continue;  // item-sharded: another rank expands this class
        expand_member(cx, root, (size_t)i, 1, arena, 0, tasks[(size_t)i]);
      }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < nth; ++t) pool.emplace_back(worker);
    for (auto& th : pool) th.join();
  }
  int64_t total = F, cands = 0;
  int maxd = F > 0 ? 1 : 0;
  for (auto& t : tasks) {
    total += (int64_t)t.item.size();
    cands += t.candidates;
    maxd = std::max(maxd, t.max_depth);
  }
  out.reserve((size_t)total);
  for (auto& t : tasks) {
    const int64_t off = out.size();
    for (size_t k = 0; k < t.item.size(); ++k) {
      int64_t p = t.parent[k];
      out.push(p >= 0 ? off + p : (-1 - p), t.item[k], t.count[k], t.depth[k]);
    }
    std::vector<int64_t>().swap(t.parent);
  }
  if (stats) {
    stats->n_frequent_items = F;
    stats->n_itemsets = out.size();
    stats->n_candidates = cands;
    stats->max_depth = maxd;
    stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return out;
}

void encode_bitmaps_cpu(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx,
                        const int32_t* rank_of, uint64_t* bm, int64_t W) {
  for (int64_t t = 0; t < n_tx; ++t)
    for (int64_t p = tx_ptr[t]; p < tx_ptr[t + 1]; ++p) {
      const int32_t r = rank_of[items[p]];
      if (r >= 0) bm[(size_t)r * W + (t >> 6)] |= (1ull << (t & 63));
    }
}

ItemsetTrie mine_cpu(const int64_t* tx_ptr, const int32_t* items, int64_t n_tx, int64_t n_items,
                     const MineConfig& cfg, MineStats* stats) {
  auto t0 = std::chrono::steady_clock::now();
  std::vector<uint32_t> cnt((size_t)n_items);
  count_items(tx_ptr, items, n_tx, n_items, cnt.data());
  FrequentItems fi = select_frequent(cnt.data(), n_items, (uint64_t)n_tx, cfg.min_support);
  const int64_t F = (int64_t)fi.ids.size();
  const int64_t W = (n_tx + 63) / 64;
  std::vector<uint64_t> bm((size_t)(F * W), 0);
  encode_bitmaps_cpu(tx_ptr, items, n_tx, fi.rank_of.data(), bm.data(), W);
  const int max_len = cfg.pairs_only ? 2 : cfg.max_len;
  ItemsetTrie out = mine_cpu_bitmaps(bm.data(), F, W, fi, max_len, cfg.threads, nullptr, stats);
  if (stats)
    stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return out;
}

}  // namespace kmls
