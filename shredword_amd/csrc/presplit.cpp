// Host pre-split: apply_regex (shredword/base.py:38-58) as hand-written matchers.
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
#include "presplit.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "shredword_hip.h"

namespace sw {
namespace {

struct Cp {
  uint32_t cp;
  int cls;
  int len;
};

inline Cp at(const uint8_t* s, int64_t n, int64_t i) {
  Cp r;
  uint8_t c = s[i];
  if (c < 0x80) {
    r.cp = c; r.len = 1;
    // ASCII fast path of the class table
    r.cls = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') ? kL
          : (c >= '0' && c <= '9') ? kN
          : (c == ' ' || (c >= 9 && c <= 13)) ? kS : kOther;
    return r;
  }
  r.cp = utf8_decode(s, n, i, &r.len);
  r.cls = r.cp == kInvalidCp ? kOther : ucd_class(r.cp);
  return r;
}

inline int64_t run_end(const uint8_t* s, int64_t n, int64_t j, int cls) {
  while (j < n) {
    Cp c = at(s, n, j);
    if (c.cls != cls) break;
    j += c.len;
  }
  return j;
}

inline bool ci(uint32_t c, char lower) {  // (?i:x) per the regex module (see ucd_ranges.h)
  if (c == (uint32_t)lower || c == (uint32_t)(lower - 32)) return true;
  return lower == 's' && c == 0x17F;  // LATIN SMALL LETTER LONG S folds to s
}

inline bool crlf(uint32_t c) { return c == '\r' || c == '\n'; }

// Whitespace-run alternatives shared by both patterns: \s+(?!\S) | \s+
inline int64_t ws_tail(const uint8_t* s, int64_t n, int64_t i, int64_t j, int64_t last_cp_start) {
  if (j == n) return j;                 // run reaches end of string: lookahead holds
  if (last_cp_start > i) return last_cp_start;  // give back the last \s so (?!\S) holds
  return j;                             // single \s before \S: plain \s+
}

}  // namespace

int64_t match_cl100k(const uint8_t* s, int64_t n, int64_t i) {
  Cp c0 = at(s, n, i);
  int64_t i1 = i + c0.len;
  // '(?i:[sdmt]|ll|ve|re)
  if (c0.cp == '\'' && i1 < n) {
    Cp c1 = at(s, n, i1);
    if (ci(c1.cp, 's') || ci(c1.cp, 'd') || ci(c1.cp, 'm') || ci(c1.cp, 't')) return i1 + c1.len;
    int64_t i2 = i1 + c1.len;
    if (i2 < n) {
      Cp c2 = at(s, n, i2);
      if ((ci(c1.cp, 'l') && ci(c2.cp, 'l')) || (ci(c1.cp, 'v') && ci(c2.cp, 'e')) ||
          (ci(c1.cp, 'r') && ci(c2.cp, 'e')))
        return i2 + c2.len;
    }
  }
  // [^\r\n\p{L}\p{N}]?+\p{L}+
  if (c0.cls == kL) return run_end(s, n, i1, kL);
  if (!crlf(c0.cp) && c0.cls != kN && i1 < n) {
    Cp c1 = at(s, n, i1);
    if (c1.cls == kL) return run_end(s, n, i1 + c1.len, kL);
  }
  // \p{N}{1,3}
  if (c0.cls == kN) {
    int64_t j = i1;
    for (int k = 1; k < 3 && j < n; ++k) {
      Cp c = at(s, n, j);
      if (c.cls != kN) break;
      j += c.len;
    }
    return j;
  }
  //  ?[^\s\p{L}\p{N}]++[\r\n]*
  int64_t p = -1;
  if (c0.cls == kOther) p = i;
  else if (c0.cp == ' ' && i1 < n && at(s, n, i1).cls == kOther) p = i1;
  if (p >= 0) {
    int64_t k = run_end(s, n, p, kOther);
    while (k < n && (s[k] == '\r' || s[k] == '\n')) ++k;
    return k;
  }
  // c0 is \s here: \s*[\r\n] | \s+(?!\S) | \s+
  int64_t j = i, last_crlf_end = -1, last_start = i;
  while (j < n) {
    Cp c = at(s, n, j);
    if (c.cls != kS) break;
    last_start = j;
    j += c.len;
    if (crlf(c.cp)) last_crlf_end = j;
  }
  if (last_crlf_end > 0) return last_crlf_end;
  return ws_tail(s, n, i, j, last_start);
}

int64_t match_gpt2(const uint8_t* s, int64_t n, int64_t i) {
  Cp c0 = at(s, n, i);
  int64_t i1 = i + c0.len;
  if (c0.cp == '\'' && i1 < n) {
    uint8_t a = s[i1];
    if (a == 's' || a == 'd' || a == 'm' || a == 't') return i1 + 1;
    if (i1 + 1 < n) {
      uint8_t b = s[i1 + 1];
      if ((a == 'l' && b == 'l') || (a == 'v' && b == 'e') || (a == 'r' && b == 'e')) return i1 + 2;
    }
  }
  //  ?\p{L}+ |  ?\p{N}+ |  ?[^\s\p{L}\p{N}]+   (the optional space backtracks)
  if (c0.cp == ' ' && i1 < n) {
    Cp c1 = at(s, n, i1);
    if (c1.cls != kS) return run_end(s, n, i1 + c1.len, c1.cls);
  }
  if (c0.cls != kS) return run_end(s, n, i1, c0.cls);
  int64_t j = i, last_start = i;
  while (j < n) {
    Cp c = at(s, n, j);
    if (c.cls != kS) break;
    last_start = j;
    j += c.len;
  }
  return ws_tail(s, n, i, j, last_start);
}

int64_t presplit_string(const uint8_t* s, int64_t n, int pattern, uint64_t* bits, int64_t base) {
  if (n <= 0) return 0;
  int64_t count = 0;
  uint64_t word = 0;
  int64_t widx = base >> 6;
  auto flush = [&]() {
    if (word) __atomic_fetch_or(&bits[widx], word, __ATOMIC_RELAXED);
    word = 0;
  };
  auto mark = [&](int64_t pos) {
    int64_t g = base + pos;
    if ((g >> 6) != widx) { flush(); widx = g >> 6; }
    word |= 1ULL << (g & 63);
    ++count;
  };
  if (pattern == SW_PAT_NONE) {
    mark(0);
  } else {
    for (int64_t i = 0; i < n;) {
      mark(i);
      int64_t e = pattern == SW_PAT_GPT2 ? match_gpt2(s, n, i) : match_cl100k(s, n, i);
      i = e > i ? e : i + 1;
    }
  }
  flush();
  return count;
}

}  // namespace sw

extern "C" int64_t sw_presplit_host(const uint8_t* bytes, const int64_t* str_off, int64_t n_str, int32_t pattern,
                                    uint64_t* chunk_bits, int32_t n_threads) {
  if (!str_off || n_str < 0 || (n_str > 0 && (!bytes || !chunk_bits))) return SW_ERR_ARG;
  if (pattern != SW_PAT_CL100K && pattern != SW_PAT_GPT2 && pattern != SW_PAT_NONE) return SW_ERR_ARG;
  if (n_str == 0) return 0;
  const int64_t b0 = str_off[0], nbytes = str_off[n_str] - b0;
  if (nbytes < 0) return SW_ERR_ARG;
  const int64_t nwords = (nbytes + 63) / 64;
  int nt = n_threads > 0 ? n_threads : (int)std::min(64u, std::max(1u, std::thread::hardware_concurrency()));
  if (nbytes < (1 << 20)) nt = 1;
  std::atomic<int64_t> total{0};
  std::atomic<bool> bad{false};
  auto work = [&](int t) {
    // zero this thread's share of the bitmap, then split its strings (byte-balanced ranges)
    int64_t w0 = nwords * t / nt, w1 = nwords * (t + 1) / nt;
    std::memset(chunk_bits + w0, 0, sizeof(uint64_t) * (size_t)(w1 - w0));
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  th.clear();
  auto split = [&](int t) {
    int64_t lo = nbytes * t / nt, hi = nbytes * (t + 1) / nt;
    // strings whose start offset falls in [lo, hi)
    int64_t s0 = std::lower_bound(str_off, str_off + n_str, b0 + lo) - str_off;
    int64_t s1 = std::lower_bound(str_off, str_off + n_str, b0 + hi) - str_off;
    if (t == nt - 1) s1 = n_str;
    int64_t c = 0;
    for (int64_t s = s0; s < s1; ++s) {
      int64_t a = str_off[s], e = str_off[s + 1];
      if (e < a) { bad = true; return; }
      c += sw::presplit_string(bytes + a, e - a, pattern, chunk_bits, a - b0);
    }
    total += c;
  };
  for (int t = 1; t < nt; ++t) th.emplace_back(split, t);
  split(0);
  for (auto& x : th) x.join();
  if (bad) return SW_ERR_ARG;
  return total.load();
}
