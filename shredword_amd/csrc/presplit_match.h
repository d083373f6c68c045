// The pre-split matchers (apply_regex, shredword/base.py:38-58) written once for host and
// device: a chunk that starts at byte i of a string ends where these functions say.
//
// cl100k (base.py:56):
//   '(?i:[sdmt]|ll|ve|re) | [^\r\n\p{L}\p{N}]?+\p{L}+ | \p{N}{1,3} | ?[^\s\p{L}\p{N}]++[\r\n]*
//   | \s*[\r\n] | \s+(?!\S) | \s+
// GPT-2 (docstring, base.py:46):
//   '(?:[sdmt]|ll|ve|re) | ?\p{L}+ | ?\p{N}+ | ?[^\s\p{L}\p{N}]+ | \s+(?!\S) | \s+
//
// Leftmost-first alternation semantics of the `regex` module: at each position the first
// alternative that matches wins; every code point is covered by some alternative, so
// findall() never skips input and the chunks tile the string.
//
// `Src` supplies the string: n (its length), byte(i) and cls(cp) (the Unicode class of a
// decoded code point, ucd_tables.h).  The host reads a plain pointer; the device kernel reads
// an LDS window with a global fallback and the tables from constant memory.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define SW_HD __host__ __device__
#else
#define SW_HD
#endif

namespace sw {

enum : int { kOther = 0, kL = 1, kN = 2, kS = 3 };
constexpr uint32_t kInvalidCp = 0xFFFFFFFFu;  // undecodable byte: class other, 1 byte

struct Cp {
  uint32_t cp;
  int cls;
  int len;
};

// Strict UTF-8 decode at byte i (i < n): the code point (kInvalidCp for an invalid sequence)
// and its length (1 for an invalid byte).
template <class Src>
SW_HD inline uint32_t utf8_decode_t(const Src& s, int64_t i, int* len) {
  const uint8_t c = s.byte(i);
  if (c < 0x80) { *len = 1; return c; }
  int L; uint32_t v; uint8_t lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) { L = 2; v = c & 0x1F; }
  else if (c >= 0xE0 && c <= 0xEF) { L = 3; v = c & 0x0F; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
  else if (c >= 0xF0 && c <= 0xF4) { L = 4; v = c & 0x07; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
  else { *len = 1; return kInvalidCp; }
  if (i + L > s.n) { *len = 1; return kInvalidCp; }
  uint8_t d = s.byte(i + 1);
  if (d < lo || d > hi) { *len = 1; return kInvalidCp; }
  v = (v << 6) | (d & 0x3F);
  for (int k = 2; k < L; ++k) {
    d = s.byte(i + k);
    if ((d & 0xC0) != 0x80) { *len = 1; return kInvalidCp; }
    v = (v << 6) | (d & 0x3F);
  }
  *len = L;
  return v;
}

template <class Src>
SW_HD inline Cp cp_at(const Src& s, int64_t i) {
  Cp r;
  const uint8_t c = s.byte(i);
  if (c < 0x80) {
    r.cp = c; r.len = 1;
    // ASCII fast path of the class table
    r.cls = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') ? kL
          : (c >= '0' && c <= '9') ? kN
          : (c == ' ' || (c >= 9 && c <= 13)) ? kS : kOther;
    return r;
  }
  r.cp = utf8_decode_t(s, i, &r.len);
  r.cls = r.cp == kInvalidCp ? kOther : s.cls(r.cp);
  return r;
}

template <class Src>
SW_HD inline int64_t run_end_t(const Src& s, int64_t j, int cls) {
  while (j < s.n) {
    const Cp c = cp_at(s, j);
    if (c.cls != cls) break;
    j += c.len;
  }
  return j;
}

SW_HD inline bool ci_eq(uint32_t c, char lower) {  // (?i:x) per the regex module (see ucd_ranges.h)
  if (c == (uint32_t)lower || c == (uint32_t)(lower - 32)) return true;
  return lower == 's' && c == 0x17F;  // LATIN SMALL LETTER LONG S folds to s
}

SW_HD inline bool is_crlf(uint32_t c) { return c == '\r' || c == '\n'; }

// Whitespace-run alternatives shared by both patterns: \s+(?!\S) | \s+
SW_HD inline int64_t ws_tail(int64_t n, int64_t i, int64_t j, int64_t last_cp_start) {
  if (j == n) return j;                         // run reaches end of string: lookahead holds
  if (last_cp_start > i) return last_cp_start;  // give back the last \s so (?!\S) holds
  return j;                                     // single \s before \S: plain \s+
}

template <class Src>
SW_HD inline int64_t match_cl100k_t(const Src& s, int64_t i) {
  const int64_t n = s.n;
  const Cp c0 = cp_at(s, i);
  const int64_t i1 = i + c0.len;
  // '(?i:[sdmt]|ll|ve|re)
  if (c0.cp == '\'' && i1 < n) {
    const Cp c1 = cp_at(s, i1);
    if (ci_eq(c1.cp, 's') || ci_eq(c1.cp, 'd') || ci_eq(c1.cp, 'm') || ci_eq(c1.cp, 't')) return i1 + c1.len;
    const int64_t i2 = i1 + c1.len;
    if (i2 < n) {
      const Cp c2 = cp_at(s, i2);
      if ((ci_eq(c1.cp, 'l') && ci_eq(c2.cp, 'l')) || (ci_eq(c1.cp, 'v') && ci_eq(c2.cp, 'e')) ||
          (ci_eq(c1.cp, 'r') && ci_eq(c2.cp, 'e')))
        return i2 + c2.len;
    }
  }
  // [^\r\n\p{L}\p{N}]?+\p{L}+
  if (c0.cls == kL) return run_end_t(s, i1, kL);
  if (!is_crlf(c0.cp) && c0.cls != kN && i1 < n) {
    const Cp c1 = cp_at(s, i1);
    if (c1.cls == kL) return run_end_t(s, i1 + c1.len, kL);
  }
  // \p{N}{1,3}
  if (c0.cls == kN) {
    int64_t j = i1;
    for (int k = 1; k < 3 && j < n; ++k) {
      const Cp c = cp_at(s, j);
      if (c.cls != kN) break;
      j += c.len;
    }
    return j;
  }
  //  ?[^\s\p{L}\p{N}]++[\r\n]*
  int64_t p = -1;
  if (c0.cls == kOther) p = i;
  else if (c0.cp == ' ' && i1 < n && cp_at(s, i1).cls == kOther) p = i1;
  if (p >= 0) {
    int64_t k = run_end_t(s, p, kOther);
    while (k < n && (s.byte(k) == '\r' || s.byte(k) == '\n')) ++k;
    return k;
  }
  // c0 is \s here: \s*[\r\n] | \s+(?!\S) | \s+
  int64_t j = i, last_crlf_end = -1, last_start = i;
  while (j < n) {
    const Cp c = cp_at(s, j);
    if (c.cls != kS) break;
    last_start = j;
    j += c.len;
    if (is_crlf(c.cp)) last_crlf_end = j;
  }
  if (last_crlf_end > 0) return last_crlf_end;
  return ws_tail(n, i, j, last_start);
}

template <class Src>
SW_HD inline int64_t match_gpt2_t(const Src& s, int64_t i) {
  const int64_t n = s.n;
  const Cp c0 = cp_at(s, i);
  const int64_t i1 = i + c0.len;
  if (c0.cp == '\'' && i1 < n) {
    const uint8_t a = s.byte(i1);
    if (a == 's' || a == 'd' || a == 'm' || a == 't') return i1 + 1;
    if (i1 + 1 < n) {
      const uint8_t b = s.byte(i1 + 1);
      if ((a == 'l' && b == 'l') || (a == 'v' && b == 'e') || (a == 'r' && b == 'e')) return i1 + 2;
    }
  }
  //  ?\p{L}+ |  ?\p{N}+ |  ?[^\s\p{L}\p{N}]+   (the optional space backtracks)
  if (c0.cp == ' ' && i1 < n) {
    const Cp c1 = cp_at(s, i1);
    if (c1.cls != kS) return run_end_t(s, i1 + c1.len, c1.cls);
  }
  if (c0.cls != kS) return run_end_t(s, i1, c0.cls);
  int64_t j = i, last_start = i;
  while (j < n) {
    const Cp c = cp_at(s, j);
    if (c.cls != kS) break;
    last_start = j;
    j += c.len;
  }
  return ws_tail(n, i, j, last_start);
}

// A position that starts a chunk whatever precedes it in the string (both patterns), used
// by the device pre-split to start parsing mid-string: an ASCII letter after ' ' starts the
// chunk at the space (" ?\p{L}+" / "[^\r\n\p{L}\p{N}]?+\p{L}+"; a longer whitespace run gives
// its last space back through \s+(?!\S)), and an ASCII letter after '\n' starts a chunk
// itself (no alternative carries a letter run across a line feed).
SW_HD inline bool ascii_letter(uint8_t c) { return (c | 0x20) >= 'a' && (c | 0x20) <= 'z'; }

}  // namespace sw
