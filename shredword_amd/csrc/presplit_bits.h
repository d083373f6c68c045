// Bit-parallel pre-split (apply_regex, shredword/base.py:38-58): the chunk starts of the cl100k
// pattern (base.py:56) and the GPT-2 pattern (base.py:46) as a handful of 64-bit mask
// operations per 32 bytes, for k_presplit_bits (presplit_bits_kernel.h) and its CPU harness
// (tests/native/psb_emul.cpp).  Written once for the device and the host (SW_HD).
//
// The regex alternation, applied leftmost-first from every chunk start, reduces to LOCAL rules
// over the code-point classes L (\p{L}), N (\p{N}), C (\r \n), P (' '), H (other \s), O (the
// rest; invalid UTF-8 bytes are one-byte O code points) -- checked against the `regex` module on
// random strings before this was written, and against the host pre-split by the tests.  With
// prev(i) / next(i) the neighbouring code points in the same string, a string start is a chunk
// start, and so is code point i when:
//   cl100k  (ost(p): p is O, prev(p) neither O nor P -- an O that starts a chunk)
//     L: prev L and i is the first letter after a contraction chunk ('s 't 'd 'm, 'll 've 're,
//        case-insensitive, at an apostrophe with ost); prev O and not ost(prev); prev N or C
//        (a prev P / H, or an ost O, is the optional prefix of [^\r\n\p{L}\p{N}]?+\p{L}+)
//     N: the first of a digit run, then every third one (\p{N}{1,3})
//     O: ost(i)                                  ( ?[^\s\p{L}\p{N}]++[\r\n]*)
//     ws: prev not ws, unless i is C and prev O  (the O run's [\r\n]* took it);
//         i in P|H after C: the C run before it follows an O (its leading C's were taken), or no
//         C follows i in its whitespace run      (\s*[\r\n] ends at the run's last C);
//         i in P|H after P|H: next exists and is not ws   (\s+(?!\S) gives the last one back)
//   GPT-2  (contractions case-sensitive, at an apostrophe with prev neither O nor P)
//     non-ws after P: never (` ?` prefixes of the three alternatives); L: prev L and the first
//     letter after a contraction, or prev not L and not the first contraction letter; N: prev not
//     N; O: prev not O; ws: prev not ws, or prev ws and next exists and is not ws.
//
// Two things are not local: a digit run's phase (every third from its start), and whether a C
// run follows an O / a whitespace run holds a later C.  Inside the 64-bit window they are mask
// fills; a run that crosses the window edge is reported (`need`) and resolved by the caller's
// walk over the neighbouring chunks (Carry).
#pragma once
#include <cstdint>

#include "presplit_match.h"

namespace sw {
namespace psb {

#define SW_PSB_FI __attribute__((always_inline))  // (the walks take the source by reference: keep it in registers)

constexpr int kChunk = 32;  // payload bytes per lane

// SWAR byte classes: a 32-bit word holds 4 bytes, and a mask has bit 7 of a byte lane set where
// that byte has the property
constexpr uint32_t kLane7 = 0x80808080u, kLow7 = 0x7F7F7F7Fu, kLane0 = 0x01010101u;

// lanes with lo <= x <= hi, for x7 < 0x80 in every lane and 0 <= lo <= hi <= 0x7F
SW_HD inline uint32_t in7(uint32_t x7, uint32_t lo, uint32_t hi) {
  return (x7 + kLane0 * (0x80 - lo)) & ~(x7 + kLane0 * (0x7F - hi)) & kLane7;
}

// Class masks of a 32-byte chunk: bit k = byte pos + k.  Classes are set at code-point leads;
// X marks the continuation bytes of valid UTF-8 sequences.  K1 / K2: an apostrophe followed by a
// one- / two-letter contraction of the pattern (not crossing a string start).
struct Masks {
  uint32_t L, N, C, P, H, A, X, K1, K2;
};

// bit 7 of each byte lane of x -> 4 bits
SW_HD inline uint32_t mm4(uint32_t x) { return ((x & 0x80808080u) * 0x00204081u) >> 28; }

SW_HD inline uint64_t rev64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bitreverse64(x);
#else
  x = ((x >> 1) & 0x5555555555555555ULL) | ((x & 0x5555555555555555ULL) << 1);
  x = ((x >> 2) & 0x3333333333333333ULL) | ((x & 0x3333333333333333ULL) << 2);
  x = ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL) | ((x & 0x0F0F0F0F0F0F0F0FULL) << 4);
  x = ((x >> 8) & 0x00FF00FF00FF00FFULL) | ((x & 0x00FF00FF00FF00FFULL) << 8);
  x = ((x >> 16) & 0x0000FFFF0000FFFFULL) | ((x & 0x0000FFFF0000FFFFULL) << 16);
  return (x >> 32) | (x << 32);
#endif
}

// the run of R (contiguous set bits) from each bit of Y upwards (Y's bits outside R: nothing)
SW_HD inline uint64_t fill_up(uint64_t Y, uint64_t R) { return ((R + (Y & R)) ^ R) & R; }
SW_HD inline uint64_t fill_down(uint64_t Y, uint64_t R) { return rev64(fill_up(rev64(Y), rev64(R))); }

// The class masks of the chunk at pos.  w: the bytes [pos - 4, pos + 36) as little-endian words
// (zeros outside the batch); ss: string-start bits of those 40 bytes (bit k = byte pos - 4 + k;
// the batch end counts as one).  Cls: cls(cp) -> kOther / kL / kN / kS (ucd_tables.h).
// The 40 bytes held in registers (w[0..9]); at4 by selects (no dynamically indexed registers)
struct RegBytes {
  uint32_t w[10];
  SW_HD uint32_t word(int i) const { return w[i]; }
  SW_HD uint32_t at4(int k) const {
    uint32_t lo_w = w[0], hi_w = w[1];
#pragma unroll
    for (int q = 1; q < 10; ++q) {
      lo_w = (k >> 2) == q ? w[q] : lo_w;
      hi_w = (k >> 2) == q ? (q + 1 < 10 ? w[q + 1] : 0u) : hi_w;
    }
    return (uint32_t)((((uint64_t)hi_w << 32) | lo_w) >> (8 * (k & 3)));
  }
};

// v_perm_b32: byte k of the result = byte sel_k of the 8 bytes hi:lo (selectors 0..7 here; 12
// gives 0x00)
SW_HD inline uint32_t perm_b32(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int k = 0; k < 4; ++k) {
    const uint32_t q = (sel >> (8 * k)) & 0xFFu;
    const uint32_t byte = q < 8 ? (uint32_t)(v >> (8 * q)) & 0xFFu : q == 12 ? 0u : q >= 13 ? 0xFFu : 0u;
    r |= byte << (8 * k);
  }
  return r;
#endif
}

// ASCII classes of 4 bytes at once, one class byte per byte: T = Thi[high nibble] & Tlo[low nibble]
// (three v_perm_b32 table lookups: 8 entries each, the low nibble's 16 in two halves), with
//   bit 7 L (0x41..0x4F, 0x61..0x6F)  bit 3 L (0x50..0x5A, 0x70..0x7A)  bit 6 N (0-9)
//   bit 2 C (\n \r)                  bit 5 P (space)                     bit 1 H (\t \v \f)
//   bit 4 A (apostrophe)
// so that one multiply gathers two classes (bits 7 and 3 of each byte).  Bytes >= 0x80 get
// garbage here; the caller clears them with the non-ASCII bits at mask level.
SW_HD inline uint32_t ascii_class4(uint32_t x) {
  const uint32_t lo = x & 0x07070707u;
  const uint32_t pa = perm_b32(0xD8C8C8C8u, 0xC8C8C868u, lo);   // low nibble 0..7
  const uint32_t pb = perm_b32(0x80808482u, 0x828CCAC8u, lo);   // low nibble 8..15
  const uint32_t nm8 = perm_b32(0xFFFFFFFFu, 0u, (x & 0x08080808u) | 0x04040404u);  // 0xFF where nibble < 8
  const uint32_t tlo = (nm8 & pa) | (~nm8 & pb);
  const uint32_t thi = perm_b32(0x08800880u, 0x40300006u, (x >> 4) & 0x07070707u);
  return tlo & thi;
}
// bits 7 and 3 of each byte lane of x -> 8 bits: bits 4..7 (bit 7s), bits 0..3 (bit 3s)
SW_HD inline uint32_t mm8(uint32_t x) { return ((x & 0x88888888u) * 0x00204081u) >> 24; }

// The class of a code point in one of the big single-class ranges of the most common non-ASCII
// scripts, from registers; -1 when cp is outside them (the caller then reads the UCD tables: two
// dependent memory reads, which a wave waits for if any of its lanes needs them).  Latin-1
// letters + Latin Extended-A/B + IPA, Greek, Cyrillic, Kana, CJK (+ extension A, B), Hangul
// syllables: \p{L}; the emoji / pictograph planes 0x1F10D-0x1FBEF: other.  Every range is one
// class in ucd_tables.h (tests/test_presplit_bits.py checks all of 0..0x10FFFF).
SW_HD inline int fast_class(uint32_t cp) {
  auto in = [](uint32_t x, uint32_t lo, uint32_t hi) -> uint32_t { return x - lo <= hi - lo ? 1u : 0u; };
  const uint32_t L = (in(cp, 0xC0, 0x2C1) & (cp != 0xD7 ? 1u : 0u) & (cp != 0xF7 ? 1u : 0u)) | in(cp, 0x391, 0x3A1) |
                     in(cp, 0x3A3, 0x3F5) | in(cp, 0x3F7, 0x481) | in(cp, 0x48A, 0x52F) | in(cp, 0x3041, 0x3096) |
                     in(cp, 0x30A1, 0x30FA) | in(cp, 0x3400, 0x4DBF) | in(cp, 0x4E00, 0xA48C) | in(cp, 0xAC00, 0xD7A3) |
                     in(cp, 0x20000, 0x2A6DF);
  return L ? kL : in(cp, 0x1F10D, 0x1FBEF) ? kOther : -1;
}

// Bytes: word(i) = bytes [pos - 4 + 4i, pos + 4i) as a little-endian word (i < 10); at4(k) = the
// bytes k .. k + 3 of those 40 (k <= 36).
template <class Cls, class Bytes>
SW_HD inline Masks classify(const Bytes& by, uint64_t ss, const Cls& cls, bool cl) {
  // ASCII classes of the chunk's bytes (words 1..8): a class byte per byte (ascii_class4), two
  // classes gathered per multiply
  uint32_t L = 0, N = 0, C = 0, P = 0, H = 0, A = 0;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    const uint32_t t = ascii_class4(by.word(i));
    const int s = 4 * (i - 1);
    const uint32_t l = mm8(t), nc = mm8(t << 1), ph = mm8(t << 2);
    L |= ((l >> 4) | (l & 15u)) << s;
    N |= (nc >> 4) << s;
    C |= (nc & 15u) << s;
    P |= (ph >> 4) << s;
    H |= (ph & 15u) << s;
    A |= mm4(t << 3) << s;
  }
  // UTF-8: every lead byte of [pos - 4, pos + 32) checked on its own (strict: no overlongs,
  // surrogates or code points past U+10FFFF, not crossing a string start); the continuation
  // bytes of the valid ones make X, and the chunk's non-ASCII code points get their class
  uint64_t X = 0;
  uint64_t hi40 = 0, ct40 = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) hi40 |= (uint64_t)mm4(by.word(i)) << (4 * i);
  {  // (the ASCII classes of bytes >= 0x80 were garbage)
    const uint32_t asc = ~(uint32_t)(hi40 >> 4);
    L &= asc; N &= asc; C &= asc; P &= asc; H &= asc; A &= asc;
  }
  if (hi40) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const uint32_t x = by.word(i), h7 = (x ^ kLane7) & kLow7;  // (bytes >= 0x80, less 0x80)
      ct40 |= (uint64_t)mm4(in7(h7, 0x00, 0x3F) & x & kLane7) << (4 * i);
    }
    // one lead: its continuation bytes (0 if invalid), its code point (kInvalidCp if it needs
    // no class: invalid, or before the chunk)
    auto lead = [&](int k, uint64_t* tail_out) -> uint32_t {
      const uint32_t b4 = by.at4(k), c0 = b4 & 0xFFu, c1 = (b4 >> 8) & 0xFFu;
      const int n = c0 >= 0xF0 ? 4 : c0 >= 0xE0 ? 3 : 2;
      const uint64_t tail = ((1ULL << (n - 1)) - 1ULL) << (k + 1);
      bool ok = (ct40 & tail) == tail && (ss & tail) == 0 && c0 >= 0xC2 && c0 <= 0xF4;
      ok = ok && !(c0 == 0xE0 && c1 < 0xA0) && !(c0 == 0xED && c1 > 0x9F) && !(c0 == 0xF0 && c1 < 0x90) &&
           !(c0 == 0xF4 && c1 > 0x8F);
      *tail_out = ok ? tail : 0ULL;
      if (!ok || k < 4) return kInvalidCp;
      uint32_t v = c0 & (n == 2 ? 0x1Fu : n == 3 ? 0x0Fu : 0x07u);
      for (int q = 1; q < n; ++q) v = (v << 6) | ((b4 >> (8 * q)) & 0x3Fu);
      return v;
    };
    // (selects, not an if-chain: the compiler turned the chain into a scratch array of {L, N, H}
    // indexed by the class -- a scratch load + store, i.e. a memory round trip, per lead)
    auto apply = [&](int k, uint32_t v, int c) {
      const uint32_t bit = v == kInvalidCp ? 0u : 1u << (k - 4);
      L |= c == kL ? bit : 0u;
      N |= c == kN ? bit : 0u;
      H |= c == kS ? bit : 0u;
    };
    // (a lane loops over its own leads: spreading a tile's leads over the wave's lanes through LDS
    // made k_split_classify slower, 3.01 -> 3.12 ms; two leads per step 1-2% slower, r4 A/B)
    for (uint64_t m = hi40 & ~ct40 & 0xFFFFFFFFFULL; m; m &= m - 1) {
      const int k = __builtin_ctzll(m);
      uint64_t t;
      const uint32_t v = lead(k, &t);
      X |= t;
      if (v != kInvalidCp) {
        int c = fast_class(v);
#if defined(SW_DIAG_NO_UCD)  // (diagnostic builds only: timing without the table reads, wrong classes)
        if (c < 0) c = kOther;
#endif
        if (c < 0) c = cls(v);
        apply(k, v, c);
      }
    }
  }
  // contractions after each apostrophe of the chunk (the next one or two code points, ASCII or
  // U+017F LONG S = C5 BF for cl100k's case-insensitive 's')
  uint32_t K1 = 0, K2 = 0;
  for (uint32_t m = A; m; m &= m - 1) {
    const int a = __builtin_ctz(m), k = a + 5;  // (the byte after it, in the 40)
    if ((ss >> k) & 1) continue;
    const uint32_t b4 = by.at4(k), c1 = b4 & 0xFFu, c2 = (b4 >> 8) & 0xFFu;
    const uint32_t l1 = cl && c1 >= 'A' && c1 <= 'Z' ? c1 | 0x20u : c1, l2 = cl && c2 >= 'A' && c2 <= 'Z' ? c2 | 0x20u : c2;
    const bool two_ok = !((ss >> (k + 1)) & 1);
    if (l1 == 's' || l1 == 'd' || l1 == 'm' || l1 == 't' || (cl && c1 == 0xC5 && c2 == 0xBF && two_ok)) {
      K1 |= 1u << a;
    } else if (two_ok && ((l1 == 'l' && l2 == 'l') || (l1 == 'v' && l2 == 'e') || (l1 == 'r' && l2 == 'e'))) {
      K2 |= 1u << a;
    }
  }
  Masks r;
  r.L = L; r.N = N; r.C = C; r.P = P; r.H = H; r.A = A; r.X = (uint32_t)(X >> 4); r.K1 = K1; r.K2 = K2;
  return r;
}

// Facts about runs crossing the window's edges (-1: unknown), found by the caller's walk:
struct Carry {
  int digit = -1;  // the digit run holding the window's first code point: its members before the window, mod 3
  int cro = -1;    // the C run holding the window's first code point follows an O
  int hasc = -1;   // the whitespace run holding the window's last byte has a C past the window
};
enum : uint32_t { kNeedDigit = 1, kNeedCro = 2, kNeedHasc = 4 };

SW_HD inline uint64_t window(uint32_t before, uint32_t mine, uint32_t after) {
  return (uint64_t)(before >> 16) | ((uint64_t)mine << 16) | ((uint64_t)after << 48);
}

// The chunk starts of the 32 bytes of chunk m1 (m0 before it, m2 after it).  ssw: string-start
// bits of the window [pos - 16, pos + 48) (bit j = byte pos - 16 + j).  *need: the carries the
// result depends on but cy does not give (then the result is not final).
SW_HD inline uint32_t rules(const Masks& m0, const Masks& m1, const Masks& m2, uint64_t ssw, bool cl, const Carry& cy,
                            uint32_t* need) {
  const uint64_t X = window(m0.X, m1.X, m2.X);
  const uint64_t L = window(m0.L, m1.L, m2.L), N = window(m0.N, m1.N, m2.N), C = window(m0.C, m1.C, m2.C);
  const uint64_t P = window(m0.P, m1.P, m2.P), H = window(m0.H, m1.H, m2.H), A = window(m0.A, m1.A, m2.A);
  const uint64_t K1 = window(m0.K1, m1.K1, m2.K1), K2 = window(m0.K2, m1.K2, m2.K2);
  const uint64_t LEAD = ~X, WS = C | P | H, O = LEAD & ~(L | N | WS), PH_ = P | H;
  constexpr uint64_t kPay = 0x0000FFFFFFFF0000ULL;  // the payload bytes
  // prev(i) in M, at every lead i (nothing at a string start): M one code point up
  auto F = [&](uint64_t M) -> uint64_t { return ((X + (M << 1)) & ~X) & ~ssw; };
  // next(i) in M (M's string starts excluded: the next code point is in another string)
  auto B = [&](uint64_t M) -> uint64_t {
    const uint64_t y = rev64(((M & LEAD & ~ssw) >> 1)), rx = rev64(X);
    return rev64((rx + y) & ~rx);
  };
  const uint64_t PL = F(L), PN = F(N), PO = F(O), PP = F(P), PC = F(C), PWS = F(WS);
  const uint64_t first = LEAD & (~LEAD + 1);  // the window's first code point (its prev is unknown)
  *need = 0;
  uint64_t st;
  const uint64_t NNW = B(LEAD & ~WS);  // next exists and is not ws
  if (cl) {
    const uint64_t OST = O & ~PO & ~PP;
    const uint64_t SLc = PL & (F(F(OST & K1)) | F(F(F(OST & K2))));
    const uint64_t STL = L & (SLc | (PO & ~F(OST)) | PN | PC);
    // digit runs: the first, then every third member (the window-edge run from its carry)
    const uint64_t NB = N | fill_up((N << 1) & X, X);  // digits with their continuation bytes
    const uint64_t edge = (first & N) ? fill_up(first, NB & ~ssw) & N : 0;  // (a run ends at a string start)
    uint64_t seed = N & ~PN & ~edge;
    if (edge) {
      if (cy.digit < 0) {
        if (edge & kPay) *need |= kNeedDigit;
      } else {
        uint64_t s = first;
        for (int k = (3 - cy.digit) % 3; k > 0; --k) s = F(s) & N;
        seed |= s;
      }
    }
    uint64_t STN = seed;
    for (uint64_t t = seed; t;) {
      t = F(F(F(t) & N) & N) & N;
      STN |= t;
    }
    // whitespace: C runs that follow an O, whitespace runs with a later C
    const uint64_t Rc = C & ~ssw;
    const uint64_t cedge = (first & C) ? fill_up(first, Rc) : 0;
    uint64_t CRO = fill_up(C & PO, Rc);
    if (cedge) {
      if (cy.cro < 0) {
        if (F(cedge) & PH_ & kPay) *need |= kNeedCro;
      } else if (cy.cro) {
        CRO |= cedge;
      }
    }
    const uint64_t WSB = WS | fill_up((WS << 1) & X, X), Rw = WSB & ~ssw;
    uint64_t HASC = fill_down(C, Rw);
    const uint64_t wedge = fill_down((Rw >> 63) << 63, Rw);
    const uint64_t after_c = PH_ & PC;
    if (wedge) {
      if (cy.hasc < 0) {
        if (after_c & kPay & wedge & ~HASC) *need |= kNeedHasc;
      } else if (cy.hasc) {
        HASC |= wedge;
      }
    }
    const uint64_t STW = (WS & ~PWS & ~(C & PO)) | (after_c & (F(CRO) | ~HASC)) | (PH_ & (PP | F(H)) & NNW);
    st = STL | STN | OST | STW;
  } else {
    const uint64_t OSG = A & ~PO & ~PP;
    const uint64_t SLc = PL & (F(F(OSG & K1)) | F(F(F(OSG & K2))));
    const uint64_t STL = L & ~PP & (SLc | (~PL & ~F(OSG & (K1 | K2))));
    const uint64_t STN = N & ~PP & ~PN;
    const uint64_t STO = O & ~PP & ~PO;
    const uint64_t STW = (WS & ~PWS) | (WS & PWS & NNW);
    st = STL | STN | STO | STW;
  }
  return (uint32_t)(((st & LEAD) | ssw) >> 16);
}

// ---- carries: walks over the chunk masks on either side of the window ----------------------
// Src: get(chunk index) -> Masks (zero masks past the batch), ss(chunk index) -> its string-start
// bits (the batch end included), n_chunks.  Chunk c covers bytes [32c, 32c + 32).
enum Field { kFX, kFN, kFC };
template <Field F, class Src>
SW_HD SW_PSB_FI inline bool bit_at(const Src& src, int64_t pos) {
  const Masks m = src.get(pos >> 5);
  const uint32_t v = F == kFX ? m.X : F == kFN ? m.N : m.C;
  return (v >> (pos & 31)) & 1u;
}

// The carries of the window of chunk c (bytes [32c - 16, 32c + 48)) that `need` asks for.
template <class Src>
SW_HD SW_PSB_FI inline Carry carries(const Src& src, int64_t c, uint32_t need) {
  Carry cy;
  const int64_t w0 = 32 * c - 16, w1 = 32 * c + 48;
  if (need & (kNeedDigit | kNeedCro)) {
    // the window's first code point (the first lead at or after w0)
    int64_t f = w0;
    while (f < 32 * c + 16 && bit_at<kFX>(src, f)) ++f;
    auto is_ss = [&](int64_t p) -> bool { return p <= 0 || ((src.ss(p >> 5) >> (p & 31)) & 1u); };
    auto lead_before = [&](int64_t p) -> int64_t {  // the lead of the code point ending at p - 1
      int64_t q = p - 1;
      while (q > 0 && bit_at<kFX>(src, q)) --q;
      return q;
    };
    if (need & kNeedDigit) {  // members of its digit run before f, mod 3
      int cnt = 0;
      for (int64_t p = f; !is_ss(p);) {
        const int64_t q = lead_before(p);
        if (!bit_at<kFN>(src, q)) break;
        cnt = (cnt + 1) % 3;
        p = q;
      }
      cy.digit = cnt;
    }
    if (need & kNeedCro) {  // the start of f's C run follows an O
      int64_t p = f;
      while (!is_ss(p) && bit_at<kFC>(src, p - 1)) --p;
      if (is_ss(p)) {
        cy.cro = 0;
      } else {
        const int64_t q = lead_before(p);
        const Masks m = src.get(q >> 5);
        const uint32_t b = 1u << (q & 31);
        cy.cro = ((m.L | m.N | m.C | m.P | m.H) & b) ? 0 : 1;
      }
    }
  }
  if (need & kNeedHasc) {  // a C in the whitespace run that goes on past the window
    cy.hasc = 0;
    for (int64_t p = w1;; ++p) {
      const int64_t ch = p >> 5;
      if (ch >= src.n_chunks) break;
      const Masks m = src.get(ch);
      const uint32_t b = 1u << (p & 31);
      if ((src.ss(ch) & b)) break;
      if (m.C & b) { cy.hasc = 1; break; }
      if (!((m.P | m.H | m.X) & b)) break;  // (X: a multi-byte whitespace code point's tail)
    }
  }
  return cy;
}

}  // namespace psb
}  // namespace sw
