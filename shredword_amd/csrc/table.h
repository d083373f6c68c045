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
};

__host__ __device__ inline uint32_t mix_key(uint32_t a, uint32_t b) {
  // 32-bit fingerprint of the pair used by both bucket choices
  uint32_t x = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
  x ^= x >> 15;
  return x;
}
__host__ __device__ inline uint32_t bucket1(uint32_t f, const DevTable& t) { return (f * t.m1) >> t.shift; }
__host__ __device__ inline uint32_t bucket2(uint32_t f, const DevTable& t) { return ((f ^ 0xA5A5A5A5u) * t.m2) >> t.shift; }

}  // namespace sw
