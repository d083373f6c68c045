// Pair -> rank table shared by the host builder and the device lookups.
//
// Replaces the `merges` dict (shredword/base.py:101, filled at :145-148): key (a, b), value
// merges[(a, b)], which is both the pair's rank and the id of the merged token.
//
// Layout: two-choice cuckoo hash with 16-byte buckets, so a lookup is exactly two independent
// 16-byte loads (one per candidate bucket) issued back to back -- one memory round trip, no
// probe loop, no lane of a wave waiting on a longer probe chain than its neighbours.
//   narrow (every pair member <= 0xFFFF): bucket = 2 slots {key = a << 16 | b, value}
//   wide   (any member > 0xFFFF):         bucket = 1 slot  {a, b, value, 0}
// Empty slots hold key / a = 0xFFFFFFFF (never a valid key: ids are non-negative int32 and the
// narrow key (0xFFFF, 0xFFFF) forces the wide layout).
//
// Round 6, tables whose every id is <= 0xFFFD (SW_INFO_IDS16: the 32k / 50k vocabularies): a
// QUOTIENT table, one 16-byte bucket per lookup instead of two.  The 32-bit key a << 16 | b goes
// through a bijective mix x (two odd multiplies and xor-shifts, constants drawn per build); the
// bucket is x's top bits (at least 16 of them) and each of its four 4-byte entries holds x's low
// 16 bits as the tag and the value: bucket and tag together are x, hence the key -- the lookup is
// exact with no key stored.  The builder redraws the constants (and doubles the buckets) until no
// bucket holds more than four keys, so every lookup is one load and no lane ever needs a second
// probe.  Empty entries are 0xFFFFFFFF (value 0xFFFF: no pair, as values are <= 0xFFFD).  At 32k
// merges: 2^17 buckets, 2 MB (L2-resident), half the L2 requests of the two-bucket lookup.
#pragma once
#include <cstdint>

namespace sw {

constexpr uint32_t kInf = 0xFFFFFFFFu;     // "pair not in merges" (rank +inf)
constexpr uint32_t kEmptyKey = 0xFFFFFFFFu;

struct DevTable {
  const void* buckets;  // uint4[n_buckets]
  uint32_t shift;       // 32 - log2(n_buckets)
  uint32_t m1, m2;      // odd multipliers of the two hash functions
  uint32_t wide;
  uint32_t q16;         // the quotient layout (16-bit ids; m1, m2: the mix constants)
};

// the quotient table's bijective 32-bit mix (m1, m2 odd): invertible, so bucket + tag identify the key
__host__ __device__ inline uint32_t q16_mix(uint32_t k, uint32_t m1, uint32_t m2) {
  uint32_t x = k * m1;
  x ^= x >> 16;
  x *= m2;
  x ^= x >> 15;
  return x;
}

__host__ __device__ inline uint32_t mix_key(uint32_t a, uint32_t b) {
  // 32-bit fingerprint of the pair used by both bucket choices
  uint32_t x = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
  x ^= x >> 15;
  return x;
}
__host__ __device__ inline uint32_t bucket1(uint32_t f, const DevTable& t) { return (f * t.m1) >> t.shift; }
__host__ __device__ inline uint32_t bucket2(uint32_t f, const DevTable& t) { return ((f ^ 0xA5A5A5A5u) * t.m2) >> t.shift; }

}  // namespace sw
