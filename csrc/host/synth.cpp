// Multi-threaded synthetic transaction generator for the large BASELINE shapes
// (10M x 1M "item-sharded" config, 100M-transaction HBM-sizing config).
//
// Same model as data/synthetic.py::generate_large (Zipf-like item popularity over a permuted
// vocabulary, genre clusters, Poisson playlist lengths, a genre-affinity mixture, duplicates
// collapsed) but generated per 64k-transaction chunk from a counter-based seed, so the output is
// identical for any thread count.  Sampling is O(1) per item through Walker alias tables (one
// global, one per genre).  numpy needs ~4 minutes for 10M transactions; this needs seconds.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <numeric>
#include <random>
#include <thread>
#include <vector>

#include "kmls/host.hpp"

namespace kmls {

namespace {

struct Alias {
  std::vector<double> prob;
  std::vector<int32_t> alias;
  std::vector<int32_t> items;  // local index → item id
  void build(const std::vector<double>& w, const std::vector<int32_t>& ids) {
    const size_t n = w.size();
    items = ids;
    prob.assign(n, 0.0);
    alias.assign(n, 0);
    if (n == 0) return;
    const double sum = std::accumulate(w.begin(), w.end(), 0.0);
    std::vector<double> p(n);
    std::vector<int32_t> small, large;
    for (size_t i = 0; i < n; ++i) {
      p[i] = w[i] * (double)n / sum;
      (p[i] < 1.0 ? small : large).push_back((int32_t)i);
    }
    while (!small.empty() && !large.empty()) {
      const int32_t s = small.back(), l = large.back();
      small.pop_back();
      prob[s] = p[s];
      alias[s] = l;
      p[l] = (p[l] + p[s]) - 1.0;
      if (p[l] < 1.0) {
        large.pop_back();
        small.push_back(l);
      }
    }
    for (int32_t i : large) prob[i] = 1.0;
    for (int32_t i : small) prob[i] = 1.0;
  }
  template <class R>
  int32_t sample(R& rng) const {
    std::uniform_real_distribution<double> u(0.0, 1.0);
    const size_t n = prob.size();
    const double x = u(rng) * (double)n;
    size_t i = (size_t)x;
    if (i >= n) i = n - 1;
    const double f = x - (double)i;
    return items[f < prob[i] ? i : (size_t)alias[i]];
  }
};

inline uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

}  // namespace

void synth_transactions(int64_t n_tx, int64_t n_items, double mean_len, int n_genres,
                        double affinity, double zipf_s, uint64_t seed, int threads,
                        std::vector<int64_t>& tx_ptr, std::vector<int32_t>& items,
                        int64_t tx_begin, int64_t tx_end) {
  KMLS_CHECK(n_tx >= 0 && n_items > 0 && n_genres > 0, "synth: bad shape");
  if (tx_end < 0 || tx_end > n_tx) tx_end = n_tx;
  tx_begin = std::max<int64_t>(0, std::min(tx_begin, tx_end));
  std::mt19937_64 g0(splitmix(seed));
  // popularity over a permuted vocabulary
  std::vector<int32_t> perm((size_t)n_items);
  std::iota(perm.begin(), perm.end(), 0);
  std::shuffle(perm.begin(), perm.end(), g0);
  std::vector<double> pop((size_t)n_items);
  for (int64_t r = 0; r < n_items; ++r) pop[(size_t)perm[(size_t)r]] = 1.0 / std::pow((double)(r + 1), zipf_s);
  std::vector<int32_t> genre((size_t)n_items);
  {
    std::uniform_int_distribution<int> ug(0, n_genres - 1);
    for (auto& g : genre) g = ug(g0);
  }
  Alias global;
  {
    std::vector<int32_t> ids((size_t)n_items);
    std::iota(ids.begin(), ids.end(), 0);
    global.build(pop, ids);
  }
  std::vector<Alias> per_genre((size_t)n_genres);
  std::vector<double> genre_mass((size_t)n_genres, 0.0);
  {
    std::vector<std::vector<int32_t>> members((size_t)n_genres);
    for (int64_t i = 0; i < n_items; ++i) {
      members[(size_t)genre[(size_t)i]].push_back((int32_t)i);
      genre_mass[(size_t)genre[(size_t)i]] += pop[(size_t)i];
    }
    for (int g = 0; g < n_genres; ++g) {
      std::vector<double> w;
      w.reserve(members[(size_t)g].size());
      for (int32_t i : members[(size_t)g]) w.push_back(pop[(size_t)i]);
      per_genre[(size_t)g].build(w, members[(size_t)g]);
    }
  }
  std::vector<int32_t> gids((size_t)n_genres);
  std::iota(gids.begin(), gids.end(), 0);
  Alias genre_pick;
  genre_pick.build(genre_mass, gids);

  // chunks are seeded by their global index, so a [tx_begin, tx_end) slice (one rank's shard)
  // is bit-identical to the same rows of the full dataset
  constexpr int64_t kChunk = 1 << 16;
  const int64_t ch0 = tx_begin / kChunk;
  const int64_t n_chunks = tx_end > tx_begin ? (tx_end - 1) / kChunk + 1 - ch0 : 0;
  std::vector<std::vector<int32_t>> c_items((size_t)n_chunks);
  std::vector<std::vector<int32_t>> c_lens((size_t)n_chunks);
  const int nth = std::max(1, threads > 0 ? threads : default_threads());
  std::atomic<int64_t> next{0};
  auto worker = [&]() {
    std::vector<int32_t> buf;
    while (true) {
      const int64_t c = next.fetch_add(1);
      if (c >= n_chunks) break;
      const int64_t gc = ch0 + c;
      std::mt19937_64 rng(splitmix(seed ^ splitmix((uint64_t)gc + 1)));
      std::poisson_distribution<int> plen(mean_len);
      std::uniform_real_distribution<double> u(0.0, 1.0);
      const int64_t t0 = gc * kChunk, t1 = std::min(n_tx, t0 + kChunk);
      auto& out = c_items[(size_t)c];
      auto& lens = c_lens[(size_t)c];
      out.reserve((size_t)((t1 - t0) * (mean_len + 1)));
      lens.reserve((size_t)(t1 - t0));
      for (int64_t t = t0; t < t1; ++t) {
        const bool keep = t >= tx_begin && t < tx_end;  // the stream advances either way
        const int len = std::max(1, plen(rng));
        const int g = genre_pick.sample(rng);
        const Alias& ga = per_genre[(size_t)g].prob.empty() ? global : per_genre[(size_t)g];
        buf.clear();
        for (int k = 0; k < len; ++k) buf.push_back(u(rng) < affinity ? ga.sample(rng) : global.sample(rng));
        std::sort(buf.begin(), buf.end());
        buf.erase(std::unique(buf.begin(), buf.end()), buf.end());
        if (!keep) continue;
        out.insert(out.end(), buf.begin(), buf.end());
        lens.push_back((int32_t)buf.size());
      }
    }
  };
  {
    std::vector<std::thread> pool;
    for (int i = 0; i < nth; ++i) pool.emplace_back(worker);
    for (auto& th : pool) th.join();
  }
  std::vector<int64_t> c_off((size_t)n_chunks + 1, 0);
  for (int64_t c = 0; c < n_chunks; ++c) c_off[(size_t)c + 1] = c_off[(size_t)c] + (int64_t)c_items[(size_t)c].size();
  tx_ptr.assign((size_t)(tx_end - tx_begin) + 1, 0);
  items.resize((size_t)c_off[(size_t)n_chunks]);
  next = 0;
  auto copier = [&]() {
    while (true) {
      const int64_t c = next.fetch_add(1);
      if (c >= n_chunks) break;
      int64_t p = c_off[(size_t)c];
      std::copy(c_items[(size_t)c].begin(), c_items[(size_t)c].end(), items.begin() + p);
      const int64_t t0 = std::max(tx_begin, (ch0 + c) * kChunk) - tx_begin;  // local row
      const auto& lens = c_lens[(size_t)c];
      for (size_t i = 0; i < lens.size(); ++i) {
        p += lens[i];
        tx_ptr[(size_t)(t0 + (int64_t)i) + 1] = p;
      }
      std::vector<int32_t>().swap(c_items[(size_t)c]);
    }
  };
  {
    std::vector<std::thread> pool;
    for (int i = 0; i < nth; ++i) pool.emplace_back(copier);
    for (auto& th : pool) th.join();
  }
}

}  // namespace kmls
