// Host pre-split: apply_regex (shredword/base.py:38-58) with the matchers of
// presplit_match.h, multithreaded over byte-balanced ranges of strings.
#include "presplit.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "shredword_hip.h"

namespace sw {

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
