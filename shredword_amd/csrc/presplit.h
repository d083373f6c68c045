// Host pre-split: the cl100k / GPT-2 patterns of apply_regex (shredword/base.py:38-58)
// restated as hand-written matchers over UTF-8 bytes.  Shared by the host path and (as the
// same logic, re-expressed per lane) the device pre-split kernel.
#pragma once
#include <cstdint>

#include "ucd_tables.h"

namespace sw {

enum : int { kOther = 0, kL = 1, kN = 2, kS = 3 };
constexpr uint32_t kInvalidCp = 0xFFFFFFFFu;  // undecodable byte: class other, 1 byte

// Strict UTF-8 decode at s[i] (i < n).  Returns the code point (kInvalidCp for an invalid
// sequence) and its byte length in *len (1 for an invalid byte).
inline uint32_t utf8_decode(const uint8_t* s, int64_t n, int64_t i, int* len) {
  uint8_t c = s[i];
  if (c < 0x80) { *len = 1; return c; }
  int L; uint32_t v; uint8_t lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) { L = 2; v = c & 0x1F; }
  else if (c >= 0xE0 && c <= 0xEF) { L = 3; v = c & 0x0F; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
  else if (c >= 0xF0 && c <= 0xF4) { L = 4; v = c & 0x07; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
  else { *len = 1; return kInvalidCp; }
  if (i + L > n) { *len = 1; return kInvalidCp; }
  uint8_t d = s[i + 1];
  if (d < lo || d > hi) { *len = 1; return kInvalidCp; }
  v = (v << 6) | (d & 0x3F);
  for (int k = 2; k < L; ++k) {
    d = s[i + k];
    if ((d & 0xC0) != 0x80) { *len = 1; return kInvalidCp; }
    v = (v << 6) | (d & 0x3F);
  }
  *len = L;
  return v;
}

inline int ucd_class(uint32_t cp) {
  if (cp > 0x10FFFF) return kOther;
  uint32_t blk = SW_UCD_STAGE1[cp >> 8];
  uint32_t byte = SW_UCD_STAGE2[blk * 64 + ((cp & 255) >> 2)];
  return (int)((byte >> ((cp & 3) * 2)) & 3);
}

// End (exclusive byte offset) of the chunk that starts at byte i of s[0..n).
int64_t match_cl100k(const uint8_t* s, int64_t n, int64_t i);
int64_t match_gpt2(const uint8_t* s, int64_t n, int64_t i);

// Marks the chunk starts of one string s[0..n) as bits (base + start) in `bits`, via
// fetch-or on whole words (safe when neighbouring strings share a word). Returns #chunks.
int64_t presplit_string(const uint8_t* s, int64_t n, int pattern, uint64_t* bits, int64_t base);

}  // namespace sw
