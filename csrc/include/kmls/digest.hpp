// Itemset content digest primitives shared by the host miners, the trie digest (digest.cpp) and
// the GPU count-only miner (kernels/deep.hip).  constexpr functions are callable from device code
// under hip-clang, so one definition serves both sides.
//
// An itemset's hash is the SUM of per-item mixes (independent of the order in which a miner
// lists its items); its digest mixes that with the support count; a result's digest is the
// multiset hash (n, sum mod 2^64, xor) of its itemset digests, additive over disjoint parts.
#pragma once

#include <cstdint>

namespace kmls {

constexpr uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// hash contribution of one item (original item id, not the frequency rank)
constexpr uint64_t item_mix(uint64_t id) { return mix64(id * 0x100000001B3ull + 7); }

struct DigestTerms {
  uint64_t sum, xr;
};

constexpr uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// the two multiset-hash terms of one itemset (set hash `h`, support count `c`): one mix of the
// pair, then two different bijections of it for the sum and the xor aggregations.  (Round 3:
// was four mix64 per itemset; the GPU miner evaluates this once per surviving candidate, so
// it was ~a quarter of the deep kernel's VALU instructions.)
constexpr DigestTerms digest_terms(uint64_t h, uint64_t c) {
  const uint64_t dg = mix64(h + c * 0x9E3779B97F4A7C15ull);
  return DigestTerms{dg, rotl64(dg, 29) * 0xD6E8FEB86659FD93ull};
}

}  // namespace kmls
