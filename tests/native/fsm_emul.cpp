// Test harness (CPU): runs presplit_fsm.h's per-segment parse serially over every 64-byte
// segment of a batch, exactly as the device lanes split it, so the transducer and its sync
// rules are checked against the host pre-split on the CPU.  Built by tests/test_presplit_fsm.py.
#include <cstdint>
#include <cstring>
#include <vector>

#include "presplit_block.h"
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
  for (int64_t r0 = 0; r0 < n; r0 += 4) {
    uint32_t u[3] = {0, 0, 0}, sb = 0;
    for (int j = 0; j < 12; ++j) {
      u[j >> 2] |= B(r0 - 4 + j) << ((j & 3) * 8);
      sb |= S(r0 - 4 + j) << j;
    }
    const uint32_t w = sw::fsm::info4(u, sb, tab->asc, sw::PsUcdFull<decltype(cls)>{cls}, cl);
    for (int k = 0; k < 4; ++k) inf[r0 + k] = (uint8_t)(w >> (8 * k));
  }
  ByteCtx x{inf.data(), tab, bits};
  for (int64_t s0 = 0; s0 < n; s0 += seg) {
    const int64_t s1 = s0 + seg < n ? s0 + seg : n;
    int64_t r = s0;
    while (r < s1 && !(inf[r] >> 4)) ++r;
    if (r == s1) continue;
    int st = sw::fsm::sync_init_state(sw::fsm::info_sync(inf[r]));
    int64_t last_cr = -1, last_ws = 0;
    bool last_sp = false;
    sw::fsm::presplit_bytes<int64_t>(x, r, s1, n, true, cl, st, last_cr, last_ws, last_sp);
  }
}

// the device kernel (k_presplit) workgroup by workgroup: presplit_block.h's phases run for
// every thread in turn, with the kernel's window, halo and string-start bitmap
struct HostBits {
  uint64_t* bits;
  int64_t widx;
  uint64_t word;
  void flush() { if (word) bits[widx] |= word; }
  void set(int64_t pos) {
    const int64_t w = pos >> 6;
    const uint64_t bit = 1ULL << (pos & 63);
    if (w == widx) {
      word |= bit;
    } else if (w > widx) {
      flush();
      widx = w;
      word = bit;
    } else {
      bits[w] |= bit;
    }
  }
};

void emul_device(const uint8_t* bytes, const int64_t* off, int64_t n_str, int pattern, uint64_t* bits) {
  const int64_t n = off[n_str];
  const bool cl = pattern == 0, none = pattern == 2;
  const sw::fsm::Tables* tab = pattern == 1 ? &kGpt2 : &kCl;
  auto cls = [](uint32_t cp) { return cls_of(cp); };
  std::vector<uint32_t> w32(sw::kPsRaw / 4), ss(sw::kPsSsWords), wb(2 * sw::kPsOutWords);
  for (int64_t blk = 0; blk * sw::kPsBlock < n; ++blk) {
    const sw::PsGeom G = sw::ps_geom(blk, n);
    uint8_t* buf = (uint8_t*)w32.data();
    for (int i = 0; i < sw::kPsRaw; ++i) {
      const int64_t g = G.wb + i;
      buf[i] = (g >= 0 && g < G.wend) ? bytes[g] : 0;
    }
    std::fill(ss.begin(), ss.end(), 0u);
    std::fill(wb.begin(), wb.end(), 0u);
    for (int64_t i = 0; i <= n_str; ++i) {
      if (off[i] < G.wb || off[i] > G.wend) continue;
      const int r = (int)(off[i] - G.wb);
      ss[r >> 5] |= 1u << (r & 31);
    }
    if (none) {
      for (int i = 0; i < sw::kPsBlock / 64; ++i) {
        const int64_t gw = (G.b0 >> 6) + i;
        if (64 * gw >= n) break;
        uint64_t v = sw::ps_none_word((const uint32_t*)ss.data(), i);
        if (64 * gw + 64 > n) v &= (1ULL << (n - 64 * gw)) - 1;
        bits[gw] = v;
      }
      continue;
    }
    std::vector<sw::PsInfoRegs> regs(sw::kPsThreads);
    for (int t = 0; t < sw::kPsThreads; ++t) regs[t] = sw::ps_info_load(w32.data(), t);
    const sw::PsUcdFull<decltype(cls)> ucd{cls};
    std::vector<uint32_t> hi(sw::kPsHiWords, 0u);
    for (int t = 0; t < sw::kPsThreads; ++t)
      sw::ps_info_convert(w32.data(), (const uint32_t*)ss.data(), tab->asc, cl, G.info_hi, t, regs[t],
                          [&](int j) { hi[j >> 5] |= 1u << (j & 31); });
    std::vector<uint16_t> pre(sw::kPsHiWords + 1, 0);
    for (int j = 0; j < sw::kPsHiWords; ++j) pre[j + 1] = (uint16_t)(pre[j] + __builtin_popcount(hi[j]));
    for (int k = 0; k < pre[sw::kPsHiWords]; ++k)
      sw::ps_high_group(w32.data(), (const uint32_t*)ss.data(), ucd, cl, G, bytes,
                        sw::ps_high_select(pre.data(), hi.data(), k));
    uint32_t* wbp = wb.data();
    auto orw = [wbp](int w, uint32_t v) { wbp[w] |= v; };
    for (int t = 0; t < sw::kPsThreads; ++t) {
      sw::PsWinBits<decltype(orw)> lb{orw};
      HostBits gout{bits, -1, 0};
      sw::ps_lane(G, t, (const uint32_t*)w32.data(), tab, tab, bytes, n, off, n_str, cl, lb, gout, cls);
    }
    for (int i = 0; i < sw::kPsOutWords; ++i) {
      const int64_t gw = (G.b0 >> 6) + i;
      if (64 * gw >= n) break;
      bits[gw] |= (uint64_t)wb[2 * i] | ((uint64_t)wb[2 * i + 1] << 32);
    }
  }
}
}  // namespace

extern "C" int fsm_emul(const uint8_t* bytes, const int64_t* off, int64_t n_str, int pattern, int seg,
                        uint64_t* bits, int byte_stepped) {
  const int64_t n = off[n_str];
  std::memset(bits, 0, sizeof(uint64_t) * (size_t)((n + 63) / 64));
  if (byte_stepped == 2) {  // the device kernel's workgroups
    emul_device(bytes, off, n_str, pattern, bits);
    return 0;
  }
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
