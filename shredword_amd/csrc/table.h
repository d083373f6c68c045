// Pair -> rank table shared by the host builder and the device lookups.
//
// Replaces the `merges` dict (shredword/base.py:101, filled at :145-148): key (a, b), value
// merges[(a, b)], which is both the pair's rank and the id of the merged token.
//
// Two layouts, picked per table at build time:
//   narrow: every pair element <= 0xFFFF -> 32-bit key (a << 16 | b), 8-byte slots {key, val}
//   wide:   any element > 0xFFFF         -> 16-byte slots {a, b, val, 0}
// Open addressing, linear probing, capacity = pow2 >= 2 n (load <= 0.5), Fibonacci hash.
#pragma once
#include <cstdint>

namespace sw {

constexpr uint32_t kInf = 0xFFFFFFFFu;     // "pair not in merges" (rank +inf)
constexpr uint32_t kRecomp = 0xFFFFFFFEu;  // rank not yet looked up
constexpr uint32_t kEmptyKey = 0xFFFFFFFFu;

struct DevTable {
  const void* slots;
  uint32_t mask;   // capacity - 1
  uint32_t shift;  // 32 - log2(capacity) (narrow) / 64 - log2(capacity) (wide)
  uint32_t wide;
};

__host__ __device__ inline uint32_t hash_narrow(uint32_t key, uint32_t shift) {
  return (uint32_t)((key * 0x9E3779B1u) >> shift);
}
__host__ __device__ inline uint32_t hash_wide(uint32_t a, uint32_t b, uint32_t shift) {
  uint64_t k = ((uint64_t)a << 32) | b;
  return (uint32_t)((k * 0x9E3779B97F4A7C15ULL) >> shift);
}

}  // namespace sw
