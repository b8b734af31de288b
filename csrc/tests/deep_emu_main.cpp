// Deep-miner check on the CPU wave emulator (tests/test_emu.py builds and runs this): the exact
// kernel source of csrc/kernels/deep.hip and the orchestration of csrc/host/deep_run.hip run over
// host memory (csrc/emu), optionally under AddressSanitizer/UBSan, and the per-size counts and
// content digest must equal mine_cpu_count's.
//
//   deep_emu n_tx n_items mean_len genres affinity min_support [budget0 budget split_min stack_mb
//            world max_len steal steal_idle presplit_cost emit]
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../host/deep_run.hpp"
#include "kmls/digest.hpp"
#include "kmls/host.hpp"

using namespace kmls;

int main(int argc, char** argv) {
  std::setvbuf(stdout, nullptr, _IONBF, 0);
  if (argc < 7) {
    std::fprintf(stderr, "usage: deep_emu n_tx n_items mean_len genres affinity min_support [...]\n");
    return 2;
  }
  const int64_t n_tx = std::atoll(argv[1]);
  int64_t n_items = std::atoll(argv[2]);
  const double mean_len = std::atof(argv[3]);
  const int genres = std::atoi(argv[4]);
  const double aff = std::atof(argv[5]), ms = std::atof(argv[6]);
  gpu::DeepOpts opt;
  if (argc > 7) opt.budget0 = std::strtoull(argv[7], nullptr, 10);
  if (argc > 8) opt.budget = std::strtoull(argv[8], nullptr, 10);
  if (argc > 9) opt.split_min = (unsigned)std::atoi(argv[9]);
  if (argc > 10) opt.stack_mb = std::atoi(argv[10]);
  const int world = argc > 11 ? std::atoi(argv[11]) : 1;
  const int max_len = argc > 12 ? std::atoi(argv[12]) : 0;
  opt.steal = argc > 13 ? std::atoi(argv[13]) != 0 : true;
  if (argc > 14) opt.steal_idle = (unsigned)std::atoi(argv[14]);
  if (argc > 15) opt.presplit_cost = (unsigned)std::atoi(argv[15]);
  opt.emit = argc > 16 && std::atoi(argv[16]) != 0;
  opt.blocks_per_cu = 1;

  std::vector<int64_t> ptr;
  std::vector<int32_t> items;
  if (n_items < 0) {
    // clique: every transaction holds items 0..|n_items|-1 (plus, in odd transactions, item
    // |n_items|): one dense class whose subtree dominates, so waves run dry while one is deep
    const int64_t k = -n_items;
    n_items = k + 1;
    ptr.push_back(0);
    for (int64_t t = 0; t < n_tx; ++t) {
      for (int64_t i = 0; i < k; ++i) items.push_back((int32_t)i);
      if (t & 1) items.push_back((int32_t)k);
      ptr.push_back((int64_t)items.size());
    }
  } else {
    synth_transactions(n_tx, n_items, mean_len, genres, aff, 0.85, 7, 1, ptr, items);
  }
  std::vector<uint32_t> cnt((size_t)n_items);
  count_items(ptr.data(), items.data(), n_tx, n_items, cnt.data());
  FrequentItems fi = select_frequent(cnt.data(), n_items, (uint64_t)n_tx, ms);
  const int64_t F = (int64_t)fi.ids.size();
  const int64_t W = (n_tx + 63) / 64, Wp = (W + 3) / 4 * 4;
  std::vector<uint64_t> bm((size_t)std::max<int64_t>(F, 1) * Wp, 0), tmp((size_t)std::max<int64_t>(F, 1) * W, 0);
  encode_bitmaps_cpu(ptr.data(), items.data(), n_tx, fi.rank_of.data(), tmp.data(), W);
  for (int64_t r = 0; r < F; ++r)
    for (int64_t w = 0; w < W; ++w) bm[(size_t)(r * Wp + w)] = tmp[(size_t)(r * W + w)];

  std::vector<uint64_t> per(64, 0);
  uint64_t dsum = 0, dxor = 0;
  per[1] = (uint64_t)F;
  for (int64_t r = 0; r < F; ++r) {
    const DigestTerms t = digest_terms(item_mix((uint64_t)fi.ids[(size_t)r]), fi.counts[(size_t)r]);
    dsum += t.sum;
    dxor ^= t.xr;
  }
  int rounds = 0;
  long long spilled = 0, handoffs = 0;
  // emit mode: the arenas' own digest (set hashes rebuilt along parent ids, size by size)
  std::vector<uint64_t> eper(64, 0);
  uint64_t esum = 0, exor = 0;
  for (int rank = 0; rank < world; ++rank) {
    gpu::DeepBufs b;
    gpu::DeepInput in;
    in.bm = bm.data();
    in.Wp = Wp;
    in.F = F;
    in.W_real = (int)W;
    in.d_ids = fi.ids.data();
    in.counts = fi.counts.data();
    in.minsup = fi.minsup2;
    in.max_len = max_len;
    in.n_cus = 2;
    gpu::DeepLocal loc;
    for (int attempt = 0;; ++attempt) {
      try {
        loc = gpu::deep_run(b, in, rank, world, opt);
        break;
      } catch (const gpu::ArenaOverflow&) {  // emit: regrown from the count, rerun (as mine_deep)
        if (attempt >= 2) throw;
      }
    }
    for (int d = 2; d < 64; ++d) per[(size_t)d] += loc.per_depth[(size_t)d];
    dsum += loc.dsum;
    dxor ^= loc.dxor;
    rounds += (int)loc.round_tasks.size();
    if (opt.emit) {
      const int64_t n = std::min(b.arena_used, b.arena_cap);
      std::vector<uint64_t> h((size_t)n, 0);
      for (int d = 1; d < 64; ++d)
        for (int64_t v = 0; v < n; ++v) {
          if (b.n_depth[v] != d) continue;
          if (d > 1 && (b.n_parent[v] >= (uint64_t)n || b.n_depth[b.n_parent[v]] != d - 1)) {
            std::printf("{\"ok\": false, \"error\": \"node %lld: bad parent\"}\n", (long long)v);
            return 1;
          }
          h[(size_t)v] = (d == 1 ? 0 : h[b.n_parent[v]]) + item_mix((uint64_t)fi.ids[b.n_item[v]]);
          if (rank > 0 && d < 3) continue;  // levels 1-2: rank 0's share
          const DigestTerms t = digest_terms(h[(size_t)v], b.n_count[v]);
          esum += t.sum;
          exor ^= t.xr;
          eper[(size_t)d] += 1;
        }
    }
    spilled += (long long)loc.spilled_tasks;
    handoffs += (long long)loc.handoffs;
  }
  CountResult c = mine_cpu_count(ptr.data(), items.data(), n_tx, n_items, ms, max_len, (int64_t)1 << 62, 2);
  bool ok = c.digest_sum == dsum && c.digest_xor == dxor;
  if (opt.emit) ok = ok && c.digest_sum == esum && c.digest_xor == exor && eper == per;
  for (size_t d = 1; d < 64; ++d) {
    const uint64_t want = d < c.per_level.size() ? (uint64_t)c.per_level[d] : 0;
    if (want != per[d]) ok = false;
  }
  std::printf("{\"F\": %lld, \"n_cpu\": %lld, \"rounds\": %d, \"spilled\": %lld, "
              "\"handoffs\": %lld, \"ok\": %s, \"per_level\": [", (long long)F,
              (long long)c.n_itemsets, rounds, spilled, handoffs, ok ? "true" : "false");
  for (size_t d = 1; d < 20; ++d) std::printf("%s%llu", d > 1 ? ", " : "", (unsigned long long)per[d]);
  std::printf("], \"cpu\": [");
  for (size_t d = 1; d < c.per_level.size(); ++d) std::printf("%s%lld", d > 1 ? ", " : "", (long long)c.per_level[d]);
  std::printf("]}\n");
  return ok ? 0 : 1;
}
