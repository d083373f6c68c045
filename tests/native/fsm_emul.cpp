// Test harness (CPU): runs presplit_fsm.h's per-segment parse serially over every 64-byte
// segment of a batch, exactly as the device lanes split it, so the transducer and its sync
// rules are checked against the host pre-split on the CPU.  Built by tests/test_presplit_fsm.py.
#include <cstdint>
#include <cstring>
#include <vector>

#include "presplit_fsm.h"
#include "ucd_tables.h"

namespace {
constexpr sw::fsm::Tables kCl = sw::fsm::make_tables(true);
constexpr sw::fsm::Tables kGpt2 = sw::fsm::make_tables(false);

struct Ctx {
  const uint8_t* g;
  const int64_t* off;
  int64_t n_str, si, a, b;
  const sw::fsm::Tables* tab;
  uint64_t* bits;
  uint8_t byte(int64_t p) const { return g[p]; }
  int cls(uint32_t cp) const {
    if (cp > 0x10FFFF) return sw::kOther;
    const uint32_t blk = SW_UCD_STAGE1[cp >> 8];
    const uint32_t v = SW_UCD_STAGE2[blk * 64 + ((cp & 255) >> 2)];
    return (int)((v >> ((cp & 3) * 2)) & 3);
  }
  bool next_string() {
    while (++si < n_str) {
      a = off[si];
      b = off[si + 1];
      if (b > a) return true;
    }
    return false;
  }
  void emit(int64_t q) { bits[q >> 6] |= 1ULL << (q & 63); }
};

struct ByteCtx {  // the byte-stepped form over precomputed info bytes
  const uint8_t* inf;
  const sw::fsm::Tables* tab;
  uint64_t* bits;
  uint32_t info(int64_t r) const { return inf[r]; }
  void emit(int64_t q) { bits[q >> 6] |= 1ULL << (q & 63); }
};

int cls_of(uint32_t cp) {
  if (cp > 0x10FFFF) return sw::kOther;
  const uint32_t blk = SW_UCD_STAGE1[cp >> 8];
  const uint32_t v = SW_UCD_STAGE2[blk * 64 + ((cp & 255) >> 2)];
  return (int)((v >> ((cp & 3) * 2)) & 3);
}

// byte-stepped: info bytes for the whole batch (4 at a time, as the device computes them),
// then every segment from its first sync position
void emul_bytes(const uint8_t* bytes, const int64_t* off, int64_t n_str, bool cl, int seg, uint64_t* bits) {
  const int64_t n = off[n_str];
  const sw::fsm::Tables* tab = cl ? &kCl : &kGpt2;
  std::vector<uint8_t> ss(n + 16, 0), inf(n + 8, 0);
  for (int64_t i = 0; i <= n_str; ++i) ss[off[i]] = 1;  // string starts and the batch end
  auto B = [&](int64_t i) -> uint32_t { return i >= 0 && i < n ? bytes[i] : 0; };
  auto S = [&](int64_t i) -> uint32_t { return i >= 0 && i <= n ? ss[i] : 0; };
  auto cls = [](uint32_t cp) { return cls_of(cp); };
  sw::fsm::LeadCarry carry{0, 0, 0};
  for (int64_t r0 = 0; r0 < n; r0 += 4) {
    uint32_t u[3] = {0, 0, 0}, sb = 0;
    for (int j = 0; j < 12; ++j) {
      u[j >> 2] |= B(r0 - 4 + j) << ((j & 3) * 8);
      sb |= S(r0 - 4 + j) << j;
    }
    if (r0 % 72 == 0) carry = sw::fsm::lead_carry(u, sb);  // (the device: a run of 18 groups per thread)
    const uint32_t w = sw::fsm::info4(u, sb, tab->asc, cls, cl, carry);
    for (int k = 0; k < 4; ++k) inf[r0 + k] = (uint8_t)(w >> (8 * k));
  }
  ByteCtx x{inf.data(), tab, bits};
  for (int64_t s0 = 0; s0 < n; s0 += seg) {
    const int64_t s1 = s0 + seg < n ? s0 + seg : n;
    int64_t r = s0;
    while (r < s1 && !(inf[r] >> 4)) ++r;
    if (r == s1) continue;
    int st = sw::fsm::sync_init_state(inf[r] >> 4);
    int64_t last_cr = -1, last_ws = 0;
    bool last_sp = false;
    sw::fsm::presplit_bytes<int64_t>(x, r, s1, n, true, cl, st, last_cr, last_ws, last_sp);
  }
}
}  // namespace

extern "C" int fsm_emul(const uint8_t* bytes, const int64_t* off, int64_t n_str, int pattern, int seg,
                        uint64_t* bits, int byte_stepped) {
  const int64_t n = off[n_str];
  std::memset(bits, 0, sizeof(uint64_t) * (size_t)((n + 63) / 64));
  if (byte_stepped && pattern != 2) {
    emul_bytes(bytes, off, n_str, pattern == 0, seg, bits);
    return 0;
  }
  for (int64_t s0 = 0; s0 < n; s0 += seg) {
    int64_t lo = 0, hi = n_str;  // last string with start <= s0
    while (lo < hi) {
      const int64_t m = (lo + hi + 1) >> 1;
      if (off[m] <= s0) lo = m; else hi = m - 1;
    }
    if (lo >= n_str) continue;
    Ctx x{bytes, off, n_str, lo, off[lo], off[lo + 1], pattern == 1 ? &kGpt2 : &kCl, bits};
    sw::fsm::presplit_segment<int64_t>(x, s0, s0 + seg < n ? s0 + seg : n, pattern == 0, pattern == 2);
  }
  return 0;
}
