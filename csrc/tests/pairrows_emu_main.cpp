// The level-2 pair-row count (csrc/kernels/pairrows.hip) run on the CPU wave emulator under
// AddressSanitizer/UBSan (tests/test_emu_pairrows.py): every path of kern::PairRows::count —
// the LDS-mask and L2-mask frequent-rank filters with their per-wave pooled reservations (empty
// abandoned rows), the per-lane filter, the direct and staged pair-list passes, item-sharded
// owned rows — must give the co-occurrence counts a plain host loop gives.
//
//   pairrows_emu <n_tx> <n_items> <max_len> <seed> <hooks> [fmask 0|1] [world]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../kernels/kernels.hpp"

using namespace kmls;

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: pairrows_emu n_tx n_items max_len seed hooks [fmask] [world]\n");
    return 2;
  }
  const int64_t T = std::atoll(argv[1]), I = std::atoll(argv[2]);
  const int max_len = std::atoi(argv[3]);
  const unsigned seed = (unsigned)std::atoi(argv[4]);
  if (std::string(argv[5]) != "-") setenv("KMLS_TEST_HOOKS", argv[5], 1);
  const bool use_mask = argc > 6 && std::atoi(argv[6]) != 0;
  const int world = argc > 7 ? std::max(1, std::atoi(argv[7])) : 1;
  // skewed item popularity; distinct items per transaction; some empty rows
  std::mt19937_64 rng(seed);
  std::vector<int64_t> ptr(1, 0);
  std::vector<int32_t> items;
  std::geometric_distribution<int> pick(3.0 / (double)I);
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
  // frequent items: support >= 2; ranks in id order
  std::vector<int64_t> sup((size_t)I, 0);
  for (int32_t x : items) ++sup[(size_t)x];
  std::vector<int32_t> ids, rank_of((size_t)I, -1);
  for (int64_t x = 0; x < I; ++x)
    if (sup[(size_t)x] >= 2) {
      rank_of[(size_t)x] = (int32_t)ids.size();
      ids.push_back((int32_t)x);
    }
  const int64_t F = (int64_t)ids.size();
  double kept = 0;
  for (int32_t x : ids) kept += (double)sup[(size_t)x];
  kept /= (double)std::max<int64_t>(T, 1);
  std::vector<uint32_t> mask((size_t)(I + 31) / 32, 0u);
  for (int32_t x : ids) mask[(size_t)x >> 5] |= 1u << (x & 31);
  // reference counts (upper triangle)
  std::vector<uint32_t> want((size_t)(F * F), 0u);
  for (int64_t t = 0; t < T; ++t) {
    std::vector<int32_t> r;
    for (int64_t p = ptr[(size_t)t]; p < ptr[(size_t)t + 1]; ++p)
      if (rank_of[(size_t)items[(size_t)p]] >= 0) r.push_back(rank_of[(size_t)items[(size_t)p]]);
    std::sort(r.begin(), r.end());
    for (size_t a = 0; a < r.size(); ++a)
      for (size_t b = a + 1; b < r.size(); ++b) {
        const int32_t ra = r[a], rb = r[b];
        if (ra % world == 0 || world == 1) ++want[(size_t)(ra * F + rb)];
      }
  }
  // "device" buffers (the item array carries 16 items of padding for the 16-byte span loads)
  items.resize(items.size() + 16, -1);
  kern::PrInput in{ptr.data(), items.data(), T, I, ids.data(), F, 2,
                   use_mask ? mask.data() : nullptr, kept};
  std::vector<uint32_t> gram((size_t)(F * F), 0xDEADBEEFu);
  kern::PairRows P;
  kern::PrShard sh{0, world, [&](const void* send, void* recv, size_t words) {
                     // every simulated rank holds the same CSR: the gather repeats rank 0's block
                     for (int q = 0; q < world; ++q)
                       std::memcpy((uint32_t*)recv + (size_t)q * words, send, words * 4);
                   }};
  const bool ok = P.count(in, gram.data(), F, nullptr, [] {}, world > 1 ? &sh : nullptr);
  if (!ok) {
    std::fprintf(stderr, "count declined\n");
    return 1;
  }
  // (item-sharded, every simulated rank's CSR is this one: owned rows count world x)
  int64_t bad = 0;
  for (int64_t a = 0; a < F; ++a)
    for (int64_t b = 0; b < F; ++b) {
      const uint32_t w = b > a ? want[(size_t)(a * F + b)] * (uint32_t)world : 0u;
      if (gram[(size_t)(a * F + b)] != w) {
        if (bad < 5)
          std::fprintf(stderr, "gram[%lld][%lld] = %u, want %u\n", (long long)a, (long long)b,
                       gram[(size_t)(a * F + b)], w);
        ++bad;
      }
    }
  std::printf("{\"n_tx\": %lld, \"F\": %lld, \"pairs\": %lld, \"rows\": %lld, \"bad\": %lld}\n",
              (long long)T, (long long)F, (long long)P.pairs(), (long long)P.n_rows(),
              (long long)bad);
  return bad ? 1 : 0;
}
