// Test harness (CPU): the bit-parallel pre-split (presplit_bits.h) over a whole batch, chunk by
// chunk as the device lanes run it -- class masks of every 32-byte chunk, then each chunk's
// window rules, with the run carries walked over the neighbouring chunks when a rule asks for
// them.  Built by tests/test_presplit_bits.py and compared with the host pre-split.
#include <cstdint>
#include <cstring>
#include <vector>

#include "presplit_bits.h"
#include "ucd_tables.h"

namespace {

struct Ucd {
  int operator()(uint32_t cp) const {
    if (cp > 0x10FFFF) return sw::kOther;
    const uint32_t blk = SW_UCD_STAGE1[cp >> 8];
    const uint32_t v = SW_UCD_STAGE2[blk * 64 + ((cp & 255) >> 2)];
    return (int)((v >> ((cp & 3) * 2)) & 3);
  }
};

struct Src {
  const std::vector<sw::psb::Masks>* masks;
  const std::vector<uint8_t>* ssb;  // one flag per byte position 0..n
  int64_t n_chunks, n;
  sw::psb::Masks get(int64_t c) const {
    if (c < 0 || c >= n_chunks) return sw::psb::Masks{};
    return (*masks)[(size_t)c];
  }
  uint32_t ss(int64_t c) const {
    uint32_t v = 0;
    for (int k = 0; k < 32; ++k) {
      const int64_t p = 32 * c + k;
      if (p >= 0 && p <= n && (*ssb)[(size_t)p]) v |= 1u << k;
    }
    return v;
  }
};

}  // namespace

// bits: ceil(n / 64) words, cleared by the caller; returns the number of chunks that needed carries
extern "C" int64_t psb_emul(const uint8_t* bytes, const int64_t* off, int64_t n_str, int pattern, uint64_t* bits) {
  const int64_t n = off[n_str] - off[0];
  const uint8_t* g = bytes + off[0];
  const int64_t nc = (n + 31) / 32;
  std::vector<uint8_t> ssb((size_t)n + 1, 0);
  for (int64_t s = 0; s <= n_str; ++s) ssb[(size_t)(off[s] - off[0])] = 1;
  auto byte = [&](int64_t p) -> uint32_t { return (p >= 0 && p < n) ? g[p] : 0u; };
  auto ssat = [&](int64_t p) -> uint64_t { return (p >= 0 && p <= n && ssb[(size_t)p]) ? 1u : 0u; };
  const bool cl = pattern == 0;
  std::vector<sw::psb::Masks> masks((size_t)nc);
  for (int64_t c = 0; c < nc; ++c) {
    sw::psb::RegBytes by;
    uint64_t ss = 0;
    for (int i = 0; i < 10; ++i) {
      by.w[i] = 0;
      for (int k = 0; k < 4; ++k) by.w[i] |= byte(32 * c - 4 + 4 * i + k) << (8 * k);
    }
    for (int k = 0; k < 40; ++k) ss |= ssat(32 * c - 4 + k) << k;
    masks[(size_t)c] = sw::psb::classify(by, ss, Ucd{}, cl);
  }
  Src src{&masks, &ssb, nc, n};
  int64_t slow = 0;
  uint32_t* b32 = (uint32_t*)bits;
  for (int64_t c = 0; c < nc; ++c) {
    uint32_t r = 0;
    if (pattern == 2) {
      r = src.ss(c);
    } else {
      uint64_t ssw = 0;
      for (int k = 0; k < 64; ++k) ssw |= ssat(32 * c - 16 + k) << k;
      uint32_t need = 0;
      r = sw::psb::rules(src.get(c - 1), src.get(c), src.get(c + 1), ssw, cl, sw::psb::Carry{}, &need);
      if (need) {
        ++slow;
        const sw::psb::Carry cy = sw::psb::carries(src, c, need);
        uint32_t need2 = 0;
        r = sw::psb::rules(src.get(c - 1), src.get(c), src.get(c + 1), ssw, cl, cy, &need2);
        if (need2) return -1;
      }
    }
    if (32 * c + 32 > n) r &= (1u << (n - 32 * c)) - 1u;
    b32[c] = r;
  }
  return slow;
}

// fast_class (presplit_bits.h) against the UCD tables for every code point: the number of code
// points it answers differently (it may decline any: -1); *covered: how many it answers
extern "C" int64_t psb_fast_class_check(int64_t* covered) {
  const Ucd ucd;
  int64_t bad = 0, cov = 0;
  for (uint32_t cp = 0; cp <= 0x10FFFF; ++cp) {
    const int f = sw::psb::fast_class(cp);
    if (f < 0) continue;
    ++cov;
    if (f != ucd(cp)) ++bad;
  }
  *covered = cov;
  return bad;
}
