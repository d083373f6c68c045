// The pre-split (apply_regex, shredword/base.py:38-58) as a one-code-point-per-step
// transducer, for the device pre-split: every lane runs the same short step (read a byte,
// map it to a symbol, one table lookup) instead of the nested alternative matchers of
// presplit_match.h, so a wavefront stays converged.  The two formulations are checked
// against each other bit for bit (tests/test_presplit_fsm.py on the CPU,
// tests/test_gpu_presplit.py on the device).
//
// Symbols: the code-point classes of presplit_match.h refined by what the pattern looks at:
// the apostrophe, the letters a contraction can continue with ('(?i:[sdmt]|ll|ve|re) for
// cl100k, case-sensitive for GPT-2), ' ', \r\n and other whitespace.
//
// States: where the chunk being matched stands.  A table entry is the next state plus
//   kEnd   -- the chunk ended before this code point: it starts a chunk (bit set) and is
//             dispatched from kStart;
//   kRetro -- GPT-2 "'l" / "'v" / "'r" not completed: "'" was a chunk by itself, the letter
//             starts the next one (bit at the previous byte);
//   kWsx   -- a whitespace run ended: \s*[\r\n] (cl100k) ends the chunk after the run's last
//             \r or \n, \s+(?!\S) gives back the run's last code point, which then starts a
//             chunk that may take the following letters (or, after ' ', punctuation) as the
//             optional prefix of [^\r\n\p{L}\p{N}]?+\p{L}+ /  ?[^\s\p{L}\p{N}]++ -- decided
//             with the run's registers (last \r\n end, last code point, was it ' ').
//
// Resumption (the device splits the batch into 64-byte segments, one lane each): a lane
// starts at the first SYNC position of its segment, whose state is known whatever precedes
// it, and stops at the first sync position at or past its segment end, so the lanes
// together reproduce the sequential parse.  Sync positions (ASCII bytes, so always
// code-point starts):
//   string start                                          -> kStart (a chunk starts)
//   ' ' followed by an ASCII letter                       -> kStart (the chunk " word")
//   ASCII letter after '\n'                               -> kStart
//   ASCII letter after three ASCII letters                -> kLRun  (inside a letter chunk:
//       a chunk boundary inside a letter run only follows a contraction, whose letters are
//       at most two after an apostrophe)
//   ASCII punctuation after ASCII punctuation (both classes [^\s\p{L}\p{N}])
//                                                         -> kORun  (inside a possessive run)
//   GPT-2 only: ASCII digit after ASCII digit             -> kNRun  ( ?\p{N}+ runs whole)
#pragma once
#include <cstdint>

#include "presplit_match.h"

namespace sw {
namespace fsm {

enum : uint8_t { kSymO, kSymA, kSymLs, kSymLl, kSymLvr, kSymLe, kSymL, kSymN, kSymSp, kSymCr, kSymWs, kNumSym };
constexpr uint8_t kSymCont = kNumSym;  // (device, byte-stepped) continuation byte of a code point: no step
// states and flags of a table entry
constexpr uint8_t kStart = 0, kLRun = 1, kA0 = 2, kAL = 3, kAVR = 4, kDone = 5, kN1 = 6, kN2 = 7, kO0 = 8,
                  kORun = 9, kORunCr = 10, kWsRun = 11, kNRun = 12;
constexpr uint8_t kStMask = 15, kEnd = 16, kRetro = 32, kWsx = 64;

struct Tables {
  uint8_t asc[128];      // symbol of an ASCII byte
  uint8_t t[16][16];     // [state][symbol] -> next state | flags
  uint8_t pre[2][16];    // after a whitespace run, [its last code point is ' '][symbol]
  // the device lane's step over an info byte (presplit_block.h): lane[lane_index(low 5 bits of
  // the info byte = symbol | string start << 4, q, state)] -> next state | kLEnd (a chunk starts
  // here) | kLRetro (one starts at the previous byte) | kLCr (one starts at the open whitespace
  // run's \r\n end, if any) | kLWs (one starts at its last code point) | the whitespace-run
  // registers' update: kLWsSet (last_ws = here, last_sp = kLSp), kLCrSet / kLCrClear (last_cr =
  // here + 1 / none).  A string start first settles the open chunk.
  uint16_t lane[32 * 4 * 13];
};
constexpr uint16_t kLEnd = 16, kLRetro = 32, kLCr = 64, kLWs = 128, kLWsSet = 256, kLSp = 512, kLCrSet = 1024,
                   kLCrClear = 2048;
SW_HD constexpr int lane_index(uint32_t sym_ss, uint32_t q, int st) { return (int)(sym_ss * 52 + q * 13) + st; }

constexpr bool sym_letter(int s) { return s >= kSymLs && s <= kSymL; }
constexpr bool sym_space(int s) { return s == kSymSp || s == kSymCr || s == kSymWs; }
constexpr bool sym_other(int s) { return s == kSymO || s == kSymA; }

constexpr uint8_t ascii_sym(int c, bool cl) {
  if (c == '\'') return kSymA;
  if (c == ' ') return kSymSp;
  if (c == '\r' || c == '\n') return kSymCr;
  if (c == 9 || c == 11 || c == 12) return kSymWs;
  if (c >= '0' && c <= '9') return kSymN;
  const bool lower = c >= 'a' && c <= 'z', upper = c >= 'A' && c <= 'Z';
  if (!lower && !upper) return kSymO;
  if (!lower && !cl) return kSymL;  // GPT-2 contractions are case-sensitive
  const int l = c | 0x20;
  if (l == 's' || l == 'd' || l == 'm' || l == 't') return kSymLs;
  if (l == 'l') return kSymLl;
  if (l == 'v' || l == 'r') return kSymLvr;
  if (l == 'e') return kSymLe;
  return kSymL;
}

constexpr Tables make_tables(bool cl) {
  Tables T{};
  for (int c = 0; c < 128; ++c) T.asc[c] = ascii_sym(c, cl);
  for (int st = 0; st < 16; ++st)
    for (int s = 0; s < 16; ++s) T.t[st][s] = kEnd | kLRun;  // (unused cells)
  for (int st = 0; st < 16; ++st) T.t[st][kSymCont] = (uint8_t)st;
  for (int s = 0; s < kNumSym; ++s) {
    const bool L = sym_letter(s), O = sym_other(s), S = sym_space(s), N = s == kSymN, CR = s == kSymCr;
    // kStart: which alternative a code point at a chunk start begins
    const uint8_t start = s == kSymA ? kA0 : L ? kLRun : N ? (cl ? kN1 : kNRun) : S ? kWsRun : (cl ? kO0 : kORun);
    T.t[kStart][s] = kEnd | start;
    T.t[kLRun][s] = L ? kLRun : kEnd;
    T.t[kDone][s] = kEnd;
    T.t[kWsRun][s] = S ? kWsRun : kWsx;
    if (cl) {
      // '(?i:[sdmt]|ll|ve|re) first; else "'" is the prefix of letters or starts a punctuation run
      T.t[kA0][s] = s == kSymLs ? kDone : s == kSymLl ? kAL : s == kSymLvr ? kAVR : L ? kLRun
                  : O ? kORun : CR ? kORunCr : kEnd;
      T.t[kAL][s] = s == kSymLl ? kDone : L ? kLRun : kEnd;
      T.t[kAVR][s] = s == kSymLe ? kDone : L ? kLRun : kEnd;
      T.t[kN1][s] = N ? kN2 : kEnd;           // \p{N}{1,3}
      T.t[kN2][s] = N ? kDone : kEnd;
      T.t[kO0][s] = L ? kLRun : O ? kORun : CR ? kORunCr : kEnd;  // prefix, or ?[^\s\p{L}\p{N}]++[\r\n]*
      T.t[kORun][s] = O ? kORun : CR ? kORunCr : kEnd;
      T.t[kORunCr][s] = CR ? kORunCr : kEnd;
      T.pre[0][s] = L ? kLRun : kEnd;
      T.pre[1][s] = L ? kLRun : O ? kORun : kEnd;
    } else {
      T.t[kA0][s] = s == kSymLs ? kDone : s == kSymLl ? kAL : s == kSymLvr ? kAVR : O ? kORun : kEnd;
      T.t[kAL][s] = s == kSymLl ? kDone : (uint8_t)(kRetro | (L ? kLRun : kEnd));
      T.t[kAVR][s] = s == kSymLe ? kDone : (uint8_t)(kRetro | (L ? kLRun : kEnd));
      T.t[kNRun][s] = N ? kNRun : kEnd;
      T.t[kORun][s] = O ? kORun : kEnd;
      T.pre[0][s] = kEnd;
      T.pre[1][s] = L ? kLRun : N ? kNRun : O ? kORun : kEnd;
    }
  }
  for (int st = 0; st <= kNRun; ++st)
    for (int s = 0; s < 16; ++s)
      for (int q = 0; q < 4; ++q)
        for (int ss = 0; ss < 2; ++ss) {
          if (s > kSymCont) {  // (no such symbol: a byte past the info, never stepped)
            T.lane[lane_index((uint32_t)(s | ss << 4), (uint32_t)q, st)] = (uint16_t)st;
            continue;
          }
          const bool last_sp = q & 1, crx = cl && (q & 2);
          int cur = st, f = 0;
          if (ss) {  // a string start settles the open chunk (presplit_bytes, sync code 1)
            if (cur == kWsRun && cl && !crx) f |= kLCr;
            if (!cl && (cur == kAL || cur == kAVR)) f |= kLRetro;
            cur = kStart;
          }
          int t = T.t[cur][s];
          if (t & kWsx) {
            if (crx) {
              t = kEnd;
            } else {
              f |= kLWs | (cl ? kLCr : 0);
              t = T.pre[last_sp][s];
            }
          } else if (t & kRetro) {
            f |= kLRetro;
          }
          if (t & kEnd) {
            f |= kLEnd;
            t = T.t[kStart][s];
          }
          if (s == kSymSp || s == kSymCr || s == kSymWs) {  // the whitespace-run registers
            f |= kLWsSet | (s == kSymSp ? kLSp : 0);
            if (cl && s == kSymCr) f |= kLCrSet;
            else if (cur != kWsRun) f |= kLCrClear;
          }
          T.lane[lane_index((uint32_t)(s | ss << 4), (uint32_t)q, st)] = (uint16_t)((t & kStMask) | f);
        }
  return T;
}

// Symbol of a decoded non-ASCII code point (class from the UCD table; U+017F folds to 's')
SW_HD inline int nonascii_sym(uint32_t cp, int cls, bool cl) {
  static_assert(kSymO == 0 && kSymL == 6 && kSymN == 7 && kSymWs == 10, "symbol numbering");
  const int s = (int)((0x0A070600u >> (8 * cls)) & 0xFFu);  // class other, L, N, S -> symbol
  return (cl && cp == 0x17F) ? (int)kSymLs : s;              // (U+017F is a letter)
}

// The state a sync position starts in, or -1.  `Ctx`: byte(p), string bounds a, b (p in [a, b)).
template <class I, class Ctx>
SW_HD inline int sync_state(const Ctx& x, I p, bool cl) {
  if (p == x.a) return kStart;
  const uint8_t c = x.byte(p);
  if (c == ' ') return (p + 1 < x.b && ascii_letter(x.byte(p + 1))) ? (int)kStart : -1;
  const uint8_t c1 = x.byte(p - 1);
  if (ascii_letter(c)) {
    if (c1 == '\n') return kStart;
    if (p - 3 >= x.a && ascii_letter(c1) && ascii_letter(x.byte(p - 2)) && ascii_letter(x.byte(p - 3))) return kLRun;
    return -1;
  }
  if (c < 0x80 && c1 < 0x80) {
    const int s = x.tab->asc[c], s1 = x.tab->asc[c1];
    if (sym_other(s) && sym_other(s1)) return kORun;
    if (!cl && s == kSymN && s1 == kSymN) return kNRun;
  }
  return -1;
}

// The code point at p (p < b): its symbol and length.  Strict UTF-8 as utf8_decode_t.
template <class I, class Ctx>
SW_HD inline int cp_sym(const Ctx& x, I p, bool cl, int* len) {
  const uint8_t c = x.byte(p);
  if (c < 0x80) {
    *len = 1;
    return x.tab->asc[c];
  }
  *len = 1;
  int L;
  uint32_t v;
  uint8_t lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) { L = 2; v = c & 0x1F; }
  else if (c >= 0xE0 && c <= 0xEF) { L = 3; v = c & 0x0F; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
  else if (c >= 0xF0 && c <= 0xF4) { L = 4; v = c & 0x07; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
  else return kSymO;
  if (p + L > x.b) return kSymO;
  uint8_t d = x.byte(p + 1);
  if (d < lo || d > hi) return kSymO;
  v = (v << 6) | (d & 0x3F);
  for (int k = 2; k < L; ++k) {
    d = x.byte(p + k);
    if ((d & 0xC0) != 0x80) return kSymO;
    v = (v << 6) | (d & 0x3F);
  }
  *len = L;
  return nonascii_sym(v, x.cls(v), cl);
}

// The parse from position p in state st (with the whitespace-run registers) up to the first
// sync position at or past s1, or the end of the batch.  `Ctx` supplies byte(p), cls(cp), tab
// (Tables*), the current string [a, b) containing p with next_string() (false past the last
// string; skips empty strings) and emit(q) (q starts a chunk).
template <class I, class Ctx>
SW_HD inline void presplit_run(Ctx& x, I p, I s1, bool cl, bool none, int st, I last_cr, I last_ws, bool last_sp) {
  while (true) {
    if (p == x.b) {  // string end: settle what the string's last chunk left open
      if (cl && st == kWsRun && last_cr >= 0 && last_cr < p) x.emit(last_cr);
      if (!cl && (st == kAL || st == kAVR)) x.emit(p - 1);
      if (!x.next_string()) break;
      p = x.a;
      if (p >= s1) break;  // (a string start is a sync position)
      st = kStart;
      continue;
    }
    if (none) {
      x.emit(p);
      p = x.b;
      continue;
    }
    if (p >= s1 && sync_state(x, p, cl) >= 0) {  // the next lane takes over here
      if (st == kWsRun) {
        if (x.byte(p) == ' ') {  // the run goes on through p (then a letter): the next lane ends it
          if (cl && last_cr >= 0) x.emit(last_cr);
        } else if (!(cl && last_cr == p)) {  // the run ends at p (a letter after '\n')
          if (cl && last_cr >= 0) x.emit(last_cr);
          x.emit(last_ws);
        }
      }
      if (!cl && (st == kAL || st == kAVR)) x.emit(p - 1);
      break;
    }
    int len;
    const int sym = cp_sym(x, p, cl, &len);
    int t = x.tab->t[st][sym];
    if (t & kWsx) {
      if (cl && last_cr == p) {  // the run ended with \r or \n: \s*[\r\n] took all of it
        t = kEnd;
      } else {
        if (cl && last_cr >= 0) x.emit(last_cr);
        x.emit(last_ws);
        t = x.tab->pre[last_sp][sym];
      }
    }
    if (t & kRetro) x.emit(p - 1);
    if (t & kEnd) {
      x.emit(p);
      t = x.tab->t[kStart][sym];
    }
    const int ns = t & kStMask;
    if (ns == kWsRun) {
      if (st != kWsRun) last_cr = -1;
      last_ws = p;
      last_sp = sym == kSymSp;
      if (cl && sym == kSymCr) last_cr = p + 1;
    }
    st = ns;
    p += len;
  }
}

// One lane's share of the parse: from the first sync position in [s0, s1) to the first sync
// position at or past s1 (or the end of the batch).  x's string is the one containing s0.
template <class I, class Ctx>
SW_HD inline void presplit_segment(Ctx& x, I s0, I s1, bool cl, bool none) {
  I p = s0;
  int st = -1;
  for (; p < s1; ++p) {  // the first sync position
    if (p == x.b && !x.next_string()) return;
    if (none) {
      if (p == x.a) { st = kStart; break; }
      continue;
    }
    st = sync_state(x, p, cl);
    if (st >= 0) break;
  }
  if (st < 0) return;
  presplit_run<I>(x, p, s1, cl, none, st, (I)-1, (I)0, false);
}

// ---- byte-stepped form (the device's fast path) -------------------------------------------
// A workgroup first computes, for every byte of its window, one INFO byte: bits 0-3 the symbol
// of the code point starting there (kSymCont for a continuation byte), bit 4 "a string starts
// here", bits 5-7 the sync code less one (info_sync):
//   0 none, 1 string start, 2 ' ' + ASCII letter, 3 ASCII letter after '\n',
//   4 fourth ASCII letter in a row, 5 ASCII punctuation pair, 6 (GPT-2) ASCII digit pair;
// the lanes then step one byte at a time through the info bytes.  Any sync: info & 0xF0.

constexpr int sync_init_state(uint32_t sc) {
  return sc <= 3 ? kStart : sc == 4 ? kLRun : sc == 5 ? kORun : kNRun;
}
SW_HD constexpr uint32_t info_sync(uint32_t v) { return (v & 16u) ? 1u : (v >> 5) ? (v >> 5) + 1u : 0u; }

// Info bytes are computed four at a time with SWAR masks: a 32-bit word holds 4 bytes, and a
// mask has bit 7 of a byte lane set where that byte has the property.  A group's context is
// the words before (bytes -4..-1), at (0..3) and after (4..7) it, and the string-start bits
// of those 12 bytes (ss, bit 4 + k = byte k of the group).
constexpr uint32_t kLane7 = 0x80808080u, kLow7 = 0x7F7F7F7Fu, kLane0 = 0x01010101u;

// lanes with lo <= x <= hi, for x7 < 0x80 in every lane and 0 <= lo <= hi <= 0x7F
SW_HD inline uint32_t in7(uint32_t x7, uint32_t lo, uint32_t hi) {
  return (x7 + kLane0 * (0x80 - lo)) & ~(x7 + kLane0 * (0x7F - hi)) & kLane7;
}
// the neighbour d bytes after (d > 0) or before (d < 0) each lane of `cur`
SW_HD inline uint32_t after(uint32_t cur, uint32_t next, int d) {
  return (uint32_t)((((uint64_t)next << 32) | cur) >> (8 * d));
}
SW_HD inline uint32_t before(uint32_t prev, uint32_t cur, int d) {
  return (uint32_t)((((uint64_t)cur << 32) | prev) >> (32 - 8 * d));
}
// string-start lanes of 4 bits
SW_HD inline uint32_t spread4(uint32_t b) { return ((b & 15) * 0x00204081u & kLane0) << 7; }

struct Ascii {  // ASCII classes of a word's lanes
  uint32_t let, dig, spc, nl, oth;
};
SW_HD inline Ascii ascii_classes(uint32_t x) {
  const uint32_t asc = ~x & kLane7, x7 = x & kLow7;
  Ascii a;
  a.let = in7(x7 | 0x20202020u, 'a', 'z') & asc;
  a.dig = in7(x7, '0', '9') & asc;
  a.spc = in7(x7, ' ', ' ') & asc;
  a.nl = in7(x7, '\n', '\n') & asc;
  const uint32_t ws = (in7(x7, 9, 13) & asc) | a.spc;
  a.oth = asc & ~(a.let | a.dig | ws);
  return a;
}

// Lanes of `cur` that lead a valid UTF-8 sequence (strict: no overlongs, surrogates or code
// points past U+10FFFF, and not crossing a string start), by length.
struct Leads {
  uint32_t v2, v3, v4;
};
SW_HD inline Leads valid_leads(uint32_t cur, uint32_t next, uint32_t ss_cur, uint32_t ss_next) {
  const uint32_t hc = cur & kLane7, h7c = (cur ^ kLane7) & kLow7;   // (bytes >= 0x80, less 0x80)
  const uint32_t hn = next & kLane7, h7n = (next ^ kLane7) & kLow7;
  const uint32_t cont_c = in7(h7c, 0x00, 0x3F) & hc, cont_n = in7(h7n, 0x00, 0x3F) & hn;
  const uint32_t n1 = after(cont_c, cont_n, 1), n2 = after(cont_c, cont_n, 2), n3 = after(cont_c, cont_n, 3);
  const uint32_t s1 = after(ss_cur, ss_next, 1), s2 = after(ss_cur, ss_next, 2), s3 = after(ss_cur, ss_next, 3);
  // the second byte's narrower ranges after E0, ED, F0, F4
  const uint32_t b1 = after(cur, next, 1), hb = b1 & kLane7, h7b = (b1 ^ kLane7) & kLow7;
  const uint32_t bad = (in7(h7c, 0x60, 0x60) & hc & ~(in7(h7b, 0x20, 0x3F) & hb)) |   // E0: A0..BF
                       (in7(h7c, 0x6D, 0x6D) & hc & ~(in7(h7b, 0x00, 0x1F) & hb)) |   // ED: 80..9F
                       (in7(h7c, 0x70, 0x70) & hc & ~(in7(h7b, 0x10, 0x3F) & hb)) |   // F0: 90..BF
                       (in7(h7c, 0x74, 0x74) & hc & ~(in7(h7b, 0x00, 0x0F) & hb));    // F4: 80..8F
  Leads l;
  l.v2 = in7(h7c, 0x42, 0x5F) & hc & n1 & ~s1;
  l.v3 = in7(h7c, 0x60, 0x6F) & hc & n1 & n2 & ~(s1 | s2) & ~bad;
  l.v4 = in7(h7c, 0x70, 0x74) & hc & n1 & n2 & n3 & ~(s1 | s2 | s3) & ~bad;
  return l;
}
SW_HD inline uint32_t any_lead(const Leads& l) { return l.v2 | l.v3 | l.v4; }

// The valid-lead lanes of u[0] (u[1] after it; ss as for info)
struct LeadCarry {
  uint32_t v2, v3, v4;
};
SW_HD inline LeadCarry lead_carry(const uint32_t* u, uint32_t ss) {
  if (((u[0] | u[1]) & kLane7) == 0) return LeadCarry{0, 0, 0};
  const Leads l = valid_leads(u[0], u[1], spread4(ss), spread4(ss >> 4));
  return LeadCarry{l.v2, l.v3, l.v4};
}

// Info is computed in two passes over a group u[1] (u[0] before it, u[2] after it; ss as above):
//   info4_ascii  every group: sync codes, the symbols of ASCII bytes, kSymO (0) for the rest;
//   info4_high   only groups with a byte >= 0x80: the symbols of those bytes (a continuation of
//                a valid sequence kSymCont, a valid lead its code point's symbol, else kSymO),
//                OR-ed into the first pass's word.  Independent of every other group, so the
//                device runs it over the (few) such groups densely.
template <class Asc>
SW_HD inline uint32_t info4_ascii(const uint32_t* u, uint32_t ss, const Ascii& p, const Ascii& c, const Ascii& n,
                                  Asc asc, bool cl) {
  const uint32_t ssp = spread4(ss), ssc = spread4(ss >> 4), ssn = spread4(ss >> 8);
  // sync codes (ASCII lanes only)
  const uint32_t sc2 = c.spc & after(c.let, n.let, 1) & ~after(ssc, ssn, 1);
  const uint32_t sc3 = c.let & before(p.nl, c.nl, 1);
  const uint32_t sc4 = c.let & before(p.let, c.let, 1) & before(p.let, c.let, 2) & before(p.let, c.let, 3) &
                       ~before(ssp, ssc, 1) & ~before(ssp, ssc, 2) & ~sc3;
  const uint32_t sc5 = c.oth & before(p.oth, c.oth, 1);
  const uint32_t sc6 = cl ? 0u : c.dig & before(p.dig, c.dig, 1);
  // (bits 5-7: the code less one; bit 4: a string start, which takes precedence)
  const uint32_t code = (sc2 >> 7) * 2 + (sc3 >> 7) * 4 + (sc4 >> 7) * 6 + (sc5 >> 7) * 8 + (sc6 >> 7) * 10 +
                        (ssc >> 7);
  uint32_t sym = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t b = (u[1] >> (8 * k)) & 0xFF;
    sym |= (uint32_t)asc[b & 0x7F] << (8 * k);
  }
  sym &= ~(((u[1] & kLane7) >> 7) * 0xFF);  // high bytes: kSymO until info4_high
  return sym | (code << 4);
}

template <class Cls>
SW_HD inline uint32_t info4_high(uint32_t info, const uint32_t* u, uint32_t ss, const Cls& cls, bool cl) {
  const uint32_t ssc = spread4(ss >> 4), ssn = spread4(ss >> 8);
  const LeadCarry carry = lead_carry(u, ss);  // leads of u[0]
  const Leads l = valid_leads(u[1], u[2], ssc, ssn);
  const uint32_t contv = before(carry.v2, l.v2, 1) | before(carry.v3, l.v3, 1) | before(carry.v3, l.v3, 2) |
                         before(carry.v4, l.v4, 1) | before(carry.v4, l.v4, 2) | before(carry.v4, l.v4, 3);
  uint32_t sym = (contv >> 7) * kSymCont;
  // the leads, one at a time (a group holds one or two on non-ASCII text)
  const uint64_t w64 = ((uint64_t)u[2] << 32) | u[1];
  uint32_t leads = any_lead(l);
  while (leads) {
    const int k = __builtin_ctz(leads) >> 3;
    leads &= leads - 1;
    const int L = ((l.v2 >> (8 * k + 7)) & 1) ? 2 : ((l.v3 >> (8 * k + 7)) & 1) ? 3 : 4;
    const uint64_t w = w64 >> (8 * k);
    uint32_t v = (uint32_t)w & (L == 2 ? 0x1F : L == 3 ? 0x0F : 0x07);
    for (int q = 1; q < L; ++q) v = (v << 6) | (uint32_t)((w >> (8 * q)) & 0x3F);
    // Cls: near(cp) for the BMP (no branch), far(cp) past it
    int c = cls.near(v < 0x10000u ? v : 0x80u);
    if (v >= 0x10000u) c = cls.far(v);
    sym |= (uint32_t)nonascii_sym(v, c, cl) << (8 * k);
  }
  return info | sym;
}

// both passes for one group (the CPU emulator's byte-stepped form)
template <class Asc, class Cls>
SW_HD inline uint32_t info4(const uint32_t* u, uint32_t ss, Asc asc, const Cls& cls, bool cl) {
  const uint32_t a = info4_ascii(u, ss, ascii_classes(u[0]), ascii_classes(u[1]), ascii_classes(u[2]), asc, cl);
  return (u[1] & kLane7) ? info4_high(a, u, ss, cls, cl) : a;
}

// The byte-stepped parse from r (state and whitespace-run registers in/out) while r < r_end:
// returns true once the lane is done (a sync position at or past s1, or the end of the batch
// when at_end says r_end is it), false when it ran out of info bytes at r_end.  `Ctx`:
// info(r), tab, emit(q).
template <class I, class Ctx>
SW_HD inline bool presplit_bytes(Ctx& x, I& r, I s1, I r_end, bool at_end, bool cl, int& st, I& last_cr, I& last_ws,
                                 bool& last_sp) {
  for (; r < r_end; ++r) {
    const uint32_t v = x.info(r);
    const uint32_t sc = info_sync(v);
    if (sc != 0 && (sc == 1 || r >= s1)) {  // settle the open chunk
      if (st == kWsRun && cl && last_cr >= 0) {
        if (sc == 1 || sc == 2) {
          if (last_cr < r) x.emit(last_cr);
        } else if (sc == 3 && last_cr != r) {
          x.emit(last_cr);
          x.emit(last_ws);
        }
      } else if (st == kWsRun && sc == 3) {
        x.emit(last_ws);  // (a letter after '\n' ends the run: \s+(?!\S) gave its last code point back)
      }
      if (!cl && (st == kAL || st == kAVR)) x.emit(r - 1);
      if (r >= s1) return true;
      st = kStart;
    }
    const uint32_t sym = v & 15;
    uint32_t t = x.tab->t[st][sym];
    if (t & (kWsx | kRetro)) {
      if (t & kWsx) {
        if (cl && last_cr == r) {
          t = kEnd;
        } else {
          if (cl && last_cr >= 0) x.emit(last_cr);
          x.emit(last_ws);
          t = x.tab->pre[last_sp][sym];
        }
      } else {
        x.emit(r - 1);
      }
    }
    if (t & kEnd) {
      x.emit(r);
      t = x.tab->t[kStart][sym];
    }
    if ((0x700u >> sym) & 1) {  // a whitespace code point (kSymSp, kSymCr, kSymWs)
      if (st != kWsRun) last_cr = -1;
      last_ws = r;
      last_sp = sym == kSymSp;
      if (cl && sym == kSymCr) last_cr = r + 1;
    }
    st = t & kStMask;
  }
  if (!at_end) return false;
  if (cl && st == kWsRun && last_cr >= 0 && last_cr < r) x.emit(last_cr);
  if (!cl && (st == kAL || st == kAVR)) x.emit(r - 1);
  return true;
}

}  // namespace fsm
}  // namespace sw
