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
//      over the info bytes while they last (one word of info per 4 steps, one step-table
//      lookup per byte, chunk starts OR-ed into an LDS bitmap of the window), then, rarely,
//      code-point-stepped over global memory (chunk starts OR-ed into the global bitmap);
//   4. the window's LDS bitmap is OR-ed into the global one (the kernel does this).
#pragma once
#include <cstdint>

#include "presplit_fsm.h"

namespace sw {

// ---- Unicode classes ----------------------------------------------------------------------
// Cls interface of fsm::info4_high: near(cp) for the BMP, far(cp) past it, operator() for any.
// one full-table function (ucd_tables.h) behind that interface
template <class Fn>
struct PsUcdFull {
  Fn fn;
  SW_HD int near(uint32_t cp) const { return fn(cp); }
  SW_HD int far(uint32_t cp) const { return fn(cp); }
  SW_HD int operator()(uint32_t cp) const { return fn(cp); }
};

#ifndef SW_PS_SEG
#define SW_PS_SEG 68
#endif
constexpr int kPsSeg = SW_PS_SEG;                // bytes per lane (17 words: lanes' reads hit distinct LDS banks)
constexpr int kPsThreads = 256;
constexpr int kPsBlock = kPsSeg * kPsThreads;    // 17 KiB per workgroup (a multiple of 64)
constexpr int kPsHalo = 1024;                    // staged past the block for chunks that run on
constexpr int kPsPre = 16;                       // staged before it (context of the first bytes)
constexpr int kPsWin = kPsPre + kPsBlock + kPsHalo;
constexpr int kPsGroups = (kPsBlock + kPsHalo) / 4 / kPsThreads;  // info words per thread (18)
constexpr int kPsRaw = kPsWin + 32;              // (zero tail: the context of the last bytes)
constexpr int kPsSsWords = kPsWin / 32 + 2;      // string-start bitmap words of the window
constexpr int kPsOutWords = (kPsBlock + kPsHalo) / 64;  // chunk-start bitmap of [b0, b0 + block + halo)
static_assert(kPsGroups * 4 * kPsThreads == kPsBlock + kPsHalo, "window");
static_assert(kPsBlock % 64 == 0 && kPsPre % 4 == 0 && kPsSeg % 4 == 0, "alignment");

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

// the parts of fsm::Tables the converged phases read (kept in LDS)
struct PsStepTab {
  uint8_t asc[128];
  uint16_t lane[32 * 4 * 13];
};

// ---- phase 2: info bytes in place of the staged bytes -------------------------------------
// Pass 1 (every group, ps_info_convert) and pass 2 (groups holding a byte >= 0x80, spread
// densely over the threads: ps_high_select, ps_high_group); see presplit_fsm.h info4_ascii /
// info4_high.
struct PsInfoRegs {
  uint32_t prev, first, edge;  // the words before, at and after this thread's run
};

template <class W32>
SW_HD inline PsInfoRegs ps_info_load(W32 w32, int tid) {
  const int wfirst = kPsPre / 4 + tid * kPsGroups;
  return PsInfoRegs{w32[wfirst - 1], w32[wfirst], w32[wfirst + kPsGroups]};
}

constexpr int kPsHiWords = kPsGroups * kPsThreads / 32;  // bitmask of the groups with a byte >= 0x80

// string-start bits of window bytes r0 - 4 .. r0 + 7
template <class SS>
SW_HD inline uint32_t ps_ss_at(SS s_ss, int r0) {
  const int q = r0 - 4;
  const uint64_t two = (uint64_t)s_ss[q >> 5] | ((uint64_t)s_ss[(q >> 5) + 1] << 32);
  return (uint32_t)(two >> (q & 31)) & 0xFFF;
}

// pass 1: converts this thread's kPsGroups words in order (info4_ascii), holding the raw words
// it still needs in registers (its neighbours' edge words came from ps_info_load, before
// anyone wrote); marks the words with a byte >= 0x80 for pass 2 (mark(j), j = group index in
// the window's info)
template <class W32, class SS, class Asc, class Mark>
SW_HD inline void ps_info_convert(W32 w32, SS s_ss, Asc asc, bool cl, int info_hi, int tid, const PsInfoRegs& regs,
                                  const Mark& mark) {
  const int wfirst = kPsPre / 4 + tid * kPsGroups;
  uint32_t u[3] = {regs.prev, regs.first, 0};
  fsm::Ascii ap = fsm::ascii_classes(u[0]), ac = fsm::ascii_classes(u[1]), an;
  for (int i = 0; i < kPsGroups; ++i) {
    const int r0 = (wfirst + i) * 4;
    if (r0 >= info_hi) break;
    u[2] = i + 1 < kPsGroups ? w32[wfirst + i + 1] : regs.edge;
    an = fsm::ascii_classes(u[2]);
    w32[wfirst + i] = fsm::info4_ascii(u, ps_ss_at(s_ss, r0), ap, ac, an, asc, cl);
    if (u[1] & fsm::kLane7) mark(tid * kPsGroups + i);
    u[0] = u[1];
    u[1] = u[2];
    ap = ac;
    ac = an;
  }
}

// window word o / 4 of the staged bytes, re-read from global memory (zeros outside [0, wend),
// as staged)
SW_HD inline uint32_t ps_raw_word(const uint8_t* bytes, const PsGeom& G, int o) {
  const int64_t g = G.wb + o;
  if (g >= 0 && g + 4 <= G.wend && (((uintptr_t)bytes & 3) == 0)) return *(const uint32_t*)(bytes + g);
  uint32_t v = 0;
  for (int k = 0; k < 4; ++k) v |= (g + k >= 0 && g + k < G.wend) ? (uint32_t)bytes[g + k] << (8 * k) : 0u;
  return v;
}

// pass 2, for the j-th group of the window's info (one marked by pass 1): its high bytes'
// symbols, from the raw bytes around it (global memory: pass 1 overwrote the staged copy)
template <class W32, class SS, class Cls>
SW_HD inline void ps_high_group(W32 w32, SS s_ss, const Cls& cls, bool cl, const PsGeom& G, const uint8_t* bytes,
                                int j) {
  const int wi = kPsPre / 4 + j;
  const uint32_t u[3] = {ps_raw_word(bytes, G, 4 * wi - 4), ps_raw_word(bytes, G, 4 * wi),
                         ps_raw_word(bytes, G, 4 * wi + 4)};
  w32[wi] = fsm::info4_high(w32[wi], u, ps_ss_at(s_ss, 4 * wi), cls, cl);
}

// the k-th set bit of the marks (pre: exclusive prefix counts of the mark words, kPsHiWords + 1)
template <class HP, class HM>
SW_HD inline int ps_high_select(HP pre, HM marks, int k) {
  int lo = 0, hi = kPsHiWords - 1;  // last word with pre <= k
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if ((int)pre[m] <= k) lo = m; else hi = m - 1;
  }
  uint32_t x = marks[lo];
  int r = k - (int)pre[lo], pos = 0;
#pragma unroll
  for (int sh = 16; sh >= 1; sh >>= 1) {
    const int c = __builtin_popcount(x & ((1u << sh) - 1u));
    if (r >= c) {
      r -= c;
      x >>= sh;
      pos += sh;
    }
  }
  return 32 * lo + pos;
}

// ---- phase 3: one lane's segment -----------------------------------------------------------
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

// The settle of the open chunk at a sync position of code sc (presplit_bytes)
template <class Emit>
SW_HD inline void ps_settle(uint32_t sc, int pos, int st, int last_cr, int last_ws, bool cl, Emit& e) {
  const bool wsr = st == fsm::kWsRun, lcv = cl && last_cr >= 0;
  if (wsr && lcv) {
    if (sc <= 2) {
      if (last_cr < pos) e.set(last_cr);
    } else if (sc == 3 && last_cr != pos) {
      e.set(last_cr);
      e.set(last_ws);
    }
  } else if (wsr && sc == 3) {
    e.set(last_ws);
  }
  if (!cl && (st == fsm::kAL || st == fsm::kAVR)) e.set(pos - 1);
}

// The byte-stepped parse of presplit_fsm.h's presplit_bytes, restated for a converged wave:
// every step is the same straight-line code (one lane-table lookup: the string-start settle,
// the transition and its chunk starts), the info is read a word at a time (all lanes walk
// word-aligned, steps before the lane's start masked), and the chunk starts of a word's steps
// that fall at bytes 4w - 1 .. 4w + 3 gather in one mask, OR-ed into the LDS bitmap once per
// word; only a far one (the \r\n end or last code point of a long whitespace run) goes by
// itself.  The segment-end sync position (any sync at or past s1) is settled once, after the
// loop.  Positions are window-relative.  Returns true when the lane is done, false when it
// reached r_end (r == r_end) with the parse still open.
//   Info: info word w (bytes 4w..4w+3).  LB: set(pos) / set_near(pos, mask: bit j = pos + j)
//   on the window's bitmap (PsWinBits).
template <class InfoW, class TabP, class LB>
SW_HD inline bool ps_lane_steps(InfoW info, TabP tab, LB& lb, int& r, int s1, int r_end, bool at_end, bool cl,
                                int& st, int& last_cr, int& last_ws, bool& last_sp) {
  const int r0 = r;
  bool done = false;
  int fin_pos = 0;
  uint32_t fin_v = 0;
  for (int w = r0 >> 2; 4 * w < r_end; ++w) {
    const uint32_t cur = info[w];
    const int base = 4 * w - 1;
    uint32_t near = 0;  // chunk starts at base + j (bit j)
    int far_cr = -1, far_ws = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pos = 4 * w + k;
      const bool act = !done && pos >= r0 && pos < r_end;
      const uint32_t v = (cur >> (8 * k)) & 0xFFu;
      const bool fin = act && pos >= s1 && (v & 0xF0u);
      fin_pos = fin ? pos : fin_pos;
      fin_v = fin ? v : fin_v;
      const bool step = act && !fin;
      const uint32_t q = (last_sp ? 1u : 0u) | (last_cr == pos ? 2u : 0u);  // (last_cr is -1 for GPT-2)
#ifdef SW_PS_NOCHAIN  // (diagnostic timing builds only: wrong bitmaps)
      const uint32_t E = step ? (uint32_t)tab->lane[fsm::lane_index(v & 31u, q, k)] : 0u;
#else
      const uint32_t E = step ? (uint32_t)tab->lane[fsm::lane_index(v & 31u, q, st)] : 0u;
#endif
      near |= ((E & fsm::kLRetro) ? 1u : 0u) << k;
      near |= ((E & fsm::kLEnd) ? 2u : 0u) << k;
      const bool e_cr = (E & fsm::kLCr) && last_cr >= 0;
      const bool e_ws = E & fsm::kLWs;
      near |= (e_cr && last_cr >= base) ? 1u << (last_cr - base) : 0u;
      near |= (e_ws && last_ws >= base) ? 1u << (last_ws - base) : 0u;
      far_cr = (e_cr && last_cr < base) ? last_cr : far_cr;
      far_ws = (e_ws && last_ws < base) ? last_ws : far_ws;
      last_ws = (E & fsm::kLWsSet) ? pos : last_ws;
      last_sp = (E & fsm::kLWsSet) ? (E & fsm::kLSp) != 0 : last_sp;
      last_cr = (E & fsm::kLCrSet) ? pos + 1 : (E & fsm::kLCrClear) ? -1 : last_cr;
      st = step ? (int)(E & fsm::kStMask) : st;
      done = done || fin;
    }
    // (a far start of this word is of a run that ended here: at most one of each kind)
    if (far_cr >= 0) lb.set(far_cr);
    if (far_ws >= 0) lb.set(far_ws);
    if (near) lb.set_near(base, near);
    if (done) break;
  }
  if (done) {
    ps_settle(fsm::info_sync(fin_v), fin_pos, st, last_cr, last_ws, cl, lb);
    return true;
  }
  r = r_end;
  if (!at_end) return false;
  if (cl && st == fsm::kWsRun && last_cr >= 0 && last_cr < r) lb.set(last_cr);
  if (!cl && (st == fsm::kAL || st == fsm::kAVR)) lb.set(r - 1);
  return true;
}

// The window's chunk-start bitmap (bit p - kPsPre = window position p), over any word array
// with an OR: the kernel's is in LDS, the emulator's a plain array.
template <class OrFn>
struct PsWinBits {
  OrFn orw;  // orw(word index, bits)
  SW_HD void set(int p) {
    const int q = p - kPsPre;
    orw(q >> 5, 1u << (q & 31));
  }
  // bit 0 of m: position p, bits 1..4: the word-aligned group p + 1 .. p + 4 (one word)
  SW_HD void set_near(int p, uint32_t m) {
    if (m & 1u) set(p);
    const int q = p + 1 - kPsPre;
    if (m >> 1) orw(q >> 5, (m >> 1) << (q & 31));
  }
};

// One lane: from the first sync position of its segment [s0, s1) to the first one at or past
// s1.  LB: the window's LDS bitmap (ps_lane_steps); GB: the global bitmap, set(pos) / flush(),
// for the rare parse that runs past the info bytes.  tab: asc + step (PsStepTab or Tables);
// ftab: the full Tables (the fallback).
template <class InfoW, class TabP, class FTabP, class LB, class GB, class Cls>
SW_HD inline void ps_lane(const PsGeom& G, int tid, InfoW info, TabP tab, FTabP ftab, const uint8_t* bytes,
                          int64_t n_bytes, const int64_t* str_off, int64_t n_str, bool cl, LB& lb, GB& gout,
                          const Cls& cls) {
  const int s0 = kPsPre + tid * kPsSeg;
  const int n_rel = (int)(n_bytes - G.wb);
  if (s0 >= n_rel) return;
  const int s1 = s0 + kPsSeg < n_rel ? s0 + kPsSeg : n_rel;
  // the first sync position in [s0, s1): a set high nibble in the info bytes
  int r = s1;
  for (int w = s0 >> 2; 4 * w < s1; ++w) {
    const uint32_t m = info[w] & 0xF0F0F0F0u;
    if (m) {
      r = 4 * w + (__builtin_ctz(m) >> 3);
      break;
    }
  }
  if (r >= s1) return;
  int st = fsm::sync_init_state(fsm::info_sync((info[r >> 2] >> (8 * (r & 3))) & 0xFFu));
  int last_cr = -1, last_ws = 0;
  bool last_sp = false;
  if (ps_lane_steps(info, tab, lb, r, s1, G.info_hi, G.at_end, cl, st, last_cr, last_ws, last_sp)) return;
#ifdef SW_PS_NOFALLBACK  // (diagnostic timing builds only: wrong bitmaps)
  return;
#endif
  // past the info bytes (r == info_hi): chunk starts still inside the open whitespace run go
  // to the global bitmap like the rest.  Continue code point by code point over global memory
  // in the string containing r - 1 (the last byte stepped), so that a string starting
  // exactly at r is entered through next_string(), which settles the one before.
  int64_t lo = 0, hi = n_str - 1;  // last string with start < wb + r
  while (lo < hi) {
    const int64_t m = (lo + hi + 1) >> 1;
    if (str_off[m] < G.wb + r) lo = m; else hi = m - 1;
  }
  PsSlow<FTabP, GB, Cls> y{bytes + G.wb, ftab, str_off, n_str, G.wb, lo, (int)(str_off[lo] - G.wb),
                          (int)(str_off[lo + 1] - G.wb), &gout, &cls};
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
  gout.flush();
}

// pattern "none": the chunks are the (non-empty) strings; bitmap word i of the block from the
// window's string-start bits (s_ss, window-relative; the batch end is past n_bytes)
template <class SS>
SW_HD inline uint64_t ps_none_word(SS s_ss, int i) {
  const int q = kPsPre + 64 * i;  // (q & 31 == 16)
  const uint64_t lo = (uint64_t)s_ss[q >> 5] | ((uint64_t)s_ss[(q >> 5) + 1] << 32);
  const uint64_t hi = s_ss[(q >> 5) + 2];
  return (lo >> (q & 31)) | (hi << (64 - (q & 31)));
}

}  // namespace sw
