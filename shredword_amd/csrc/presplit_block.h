// One workgroup of the device pre-split (k_presplit, presplit_kernel.h), written once for the
// device and for the CPU emulator (tests/native/fsm_emul.cpp, which runs every "thread" of
// every phase in turn).  The kernel supplies LDS pointers, the UCD lookup from constant
// memory and atomic bitmap words; the emulator plain arrays.
//
// A workgroup owns kPsBlock bytes of the batch (kPsSeg per lane), staged with a kPsPre pre-halo
// and a kPsHalo post-halo.  Phases (a barrier between each):
//   1. stage the window's bytes and mark its string starts (ps_geom, the kernel does this);
//   2. every thread turns kPsGroups words of staged bytes into INFO bytes in place
//      (ps_info_load before the barrier: the raw words it needs from its neighbours;
//      ps_info_convert after it);
//   3. every lane parses from the first sync position of its segment (ps_lane): byte-stepped
//      over the info bytes while they last, then code-point-stepped over global memory.
#pragma once
#include <cstdint>

#include "presplit_fsm.h"

namespace sw {

constexpr int kPsSeg = 64;                       // bytes per lane
constexpr int kPsThreads = 256;
constexpr int kPsBlock = kPsSeg * kPsThreads;    // 16 KiB per workgroup
constexpr int kPsHalo = 2048;                    // staged past the block for chunks that run on
constexpr int kPsPre = 16;                       // staged before it (context of the first bytes)
constexpr int kPsWin = kPsPre + kPsBlock + kPsHalo;
constexpr int kPsGroups = (kPsBlock + kPsHalo) / 4 / kPsThreads;  // info words per thread (18)
constexpr int kPsRaw = kPsWin + 32;              // (zero tail: the context of the last bytes)
constexpr int kPsSsWords = kPsWin / 32 + 2;      // string-start bitmap words of the window
static_assert(kPsGroups * 4 * kPsThreads == kPsBlock + kPsHalo, "window");

struct PsGeom {
  int64_t b0;      // first byte the workgroup owns
  int64_t wb;      // window start (b0 - kPsPre; may be negative)
  int64_t wend;    // staged bytes end here (exclusive)
  int wlen;        // wend - wb
  bool at_end;     // the window reaches the batch end
  int info_hi;     // info bytes exist for window positions [kPsPre, info_hi)
};

SW_HD inline PsGeom ps_geom(int64_t block, int64_t n_bytes) {
  PsGeom g;
  g.b0 = block * kPsBlock;
  g.wb = g.b0 - kPsPre;
  const int64_t e = g.b0 + (int64_t)(kPsBlock + kPsHalo);
  g.wend = e < n_bytes ? e : n_bytes;
  g.wlen = (int)(g.wend - g.wb);
  g.at_end = g.wend == n_bytes;
  // the info of a group needs the 4 bytes after it: the last 8 staged bytes have none unless
  // the window ends at the batch end (zeros past it are the real context there)
  g.info_hi = g.at_end ? g.wlen : kPsWin - 8;
  return g;
}

// ---- phase 2: info bytes in place of the staged bytes -------------------------------------
struct PsInfoRegs {
  uint32_t prev, first, edge;  // the words before, at and after this thread's run
};

template <class W32>
SW_HD inline PsInfoRegs ps_info_load(W32 w32, int tid) {
  const int wfirst = kPsPre / 4 + tid * kPsGroups;
  return PsInfoRegs{w32[wfirst - 1], w32[wfirst], w32[wfirst + kPsGroups]};
}

// converts this thread's kPsGroups words in order, holding the raw words it still needs in
// registers (its neighbours' edge words came from ps_info_load, before anyone wrote)
template <class W32, class SS, class Asc, class Cls>
SW_HD inline void ps_info_convert(W32 w32, SS s_ss, Asc asc, const Cls& cls, bool cl, int info_hi, int tid,
                                  const PsInfoRegs& regs) {
  const int wfirst = kPsPre / 4 + tid * kPsGroups;
  uint32_t u[3] = {regs.prev, regs.first, 0};
  fsm::LeadCarry carry{0, 0, 0};
  for (int i = 0; i < kPsGroups; ++i) {
    const int r0 = (wfirst + i) * 4;
    if (r0 >= info_hi) break;
    u[2] = i + 1 < kPsGroups ? w32[wfirst + i + 1] : regs.edge;
    const int q = r0 - 4;
    const uint64_t two = (uint64_t)s_ss[q >> 5] | ((uint64_t)s_ss[(q >> 5) + 1] << 32);
    const uint32_t ss = (uint32_t)(two >> (q & 31)) & 0xFFF;
    if (i == 0) carry = fsm::lead_carry(u, ss);
    w32[wfirst + i] = fsm::info4(u, ss, asc, cls, cl, carry);
    u[0] = u[1];
    u[1] = u[2];
  }
}

// ---- phase 3: one lane's segment -----------------------------------------------------------
template <class InfoP, class TabP, class Bits>
struct PsFast {  // presplit_bytes context: positions relative to the window start wb
  InfoP inf;
  TabP tab;
  Bits* out;
  int64_t wb;
  SW_HD uint32_t info(int r) const { return inf[r]; }
  SW_HD void emit(int r) { out->set(wb + r); }
};

template <class TabP, class Bits, class Cls>
struct PsSlow {  // presplit_run context over global memory, positions relative to wb
  const uint8_t* g;  // bytes + wb
  TabP tab;
  const int64_t* str_off;
  int64_t n_str, wb, si;
  int a, b;
  Bits* out;
  const Cls* cls_fn;
  SW_HD uint8_t byte(int p) const { return g[p]; }
  SW_HD int cls(uint32_t cp) const { return (*cls_fn)(cp); }
  SW_HD bool next_string() {
    while (++si < n_str) {
      a = (int)(str_off[si] - wb);
      b = (int)(str_off[si + 1] - wb);
      if (b > a) return true;
    }
    return false;
  }
  SW_HD void emit(int r) { out->set(wb + r); }
};

// Bits: set(pos) / flush(), word = the lane's own bitmap word to start with.  Returns with
// the lane's chunk starts passed to out (not flushed).
template <class InfoP, class SS, class TabP, class Bits, class Cls>
SW_HD inline void ps_lane(const PsGeom& G, int tid, InfoP info, SS s_ss, TabP tab, const uint8_t* bytes,
                          int64_t n_bytes, const int64_t* str_off, int64_t n_str, bool cl, bool none, Bits& out,
                          const Cls& cls) {
  const int s0 = kPsPre + tid * kPsSeg;
  const int n_rel = (int)(n_bytes - G.wb);
  if (s0 >= n_rel) return;
  const int s1 = s0 + kPsSeg < n_rel ? s0 + kPsSeg : n_rel;
  if (none) {  // the chunks are the strings: this word's string starts
    const int q = s0;
    const uint64_t lo = (uint64_t)s_ss[q >> 5] | ((uint64_t)s_ss[(q >> 5) + 1] << 32);
    const uint64_t hi = s_ss[(q >> 5) + 2];
    uint64_t w = (lo >> (q & 31)) | (hi << (64 - (q & 31)));  // (q & 31 == 16)
    if (s1 - s0 < 64) w &= (1ULL << (s1 - s0)) - 1;
    out.word |= w;
    return;
  }
  PsFast<InfoP, TabP, Bits> x{info, tab, &out, G.wb};
  int r = s0;
  while (r < s1 && !(x.info(r) >> 4)) ++r;
  if (r == s1) return;
  int st = fsm::sync_init_state(x.info(r) >> 4);
  int last_cr = -1, last_ws = 0;
  bool last_sp = false;
  if (fsm::presplit_bytes<int>(x, r, s1, G.info_hi, G.at_end, cl, st, last_cr, last_ws, last_sp)) return;
  // past the info bytes (r == info_hi): continue code point by code point over global memory.
  // The string: the one containing position r - 1 (the last byte stepped), so that a string
  // starting exactly at r is entered through next_string(), which settles the one before.
  int64_t lo = 0, hi = n_str - 1;  // last string with start < wb + r
  while (lo < hi) {
    const int64_t m = (lo + hi + 1) >> 1;
    if (str_off[m] < G.wb + r) lo = m; else hi = m - 1;
  }
  PsSlow<TabP, Bits, Cls> y{bytes + G.wb, tab, str_off, n_str, G.wb, lo, (int)(str_off[lo] - G.wb),
                            (int)(str_off[lo + 1] - G.wb), &out, &cls};
  if (r < y.b) {
    for (int k = 1; k <= 3; ++k) {  // r may be inside the code point the byte steps were in
      if (r - k < y.a) break;
      int len;
      fsm::cp_sym(y, r - k, cl, &len);
      if (len > k) {
        r += len - k;
        break;
      }
    }
  }
  fsm::presplit_run<int>(y, r, s1, cl, false, st, last_cr, last_ws, last_sp);
}

}  // namespace sw
