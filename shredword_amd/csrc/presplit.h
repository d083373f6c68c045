// Host pre-split: the cl100k / GPT-2 patterns of apply_regex (shredword/base.py:38-58), using
// the matchers shared with the device kernel (presplit_match.h).
#pragma once
#include <cstdint>

#include "presplit_match.h"
#include "ucd_tables.h"

namespace sw {

inline int ucd_class(uint32_t cp) {
  if (cp > 0x10FFFF) return kOther;
  const uint32_t blk = SW_UCD_STAGE1[cp >> 8];
  const uint32_t byte = SW_UCD_STAGE2[blk * 64 + ((cp & 255) >> 2)];
  return (int)((byte >> ((cp & 3) * 2)) & 3);
}

// a string in host memory
struct HostStr {
  const uint8_t* s;
  int64_t n;
  uint8_t byte(int64_t i) const { return s[i]; }
  int cls(uint32_t cp) const { return ucd_class(cp); }
};

// End (exclusive byte offset) of the chunk that starts at byte i of s[0..n).
inline int64_t match_cl100k(const uint8_t* s, int64_t n, int64_t i) { return match_cl100k_t(HostStr{s, n}, i); }
inline int64_t match_gpt2(const uint8_t* s, int64_t n, int64_t i) { return match_gpt2_t(HostStr{s, n}, i); }

// Marks the chunk starts of one string s[0..n) as bits (base + start) in `bits`, via
// fetch-or on whole words (safe when neighbouring strings share a word). Returns #chunks.
int64_t presplit_string(const uint8_t* s, int64_t n, int pattern, uint64_t* bits, int64_t base);

}  // namespace sw
