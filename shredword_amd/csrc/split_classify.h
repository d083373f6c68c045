// The device pre-split fused into the classification: k_split_classify, one wave per 2 KiB tile,
// computes the tile's chunk starts (apply_regex, shredword/base.py:38-58, the bit-parallel rules
// of presplit_bits.h) from the tile's bytes staged once in LDS, and goes straight on to the
// classification of its chunks (classify_chunks, kernels.h) -- the input is read once and the
// chunk-start bitmap never makes a round trip through HBM before it is used.  The bitmap is
// still written (one dword per lane, coalesced) for the later kernels that need a chunk's end
// past its tile (k_lp_prep) and for sw_presplit_device's callers.
//
// A lane's rules read its neighbours' class masks: inside the tile they come from LDS; the two
// the tile does not compute -- lane 0's left neighbour (the previous tile's last 32 bytes) and
// lane 63's right one (the next tile's first 32 bytes) -- come from k_edges, a small pass over
// the tile boundaries before it: per boundary b (byte 2048 b) the class masks of the 32 bytes
// after it and the final chunk-start word of those 32 bytes (which lane 0 of tile b takes as its
// own, and which tells tile b - 1 where its last chunk ends).  Included by encode.hip only.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"
#include "presplit_bits.h"
#include "presplit_kernel.h"

namespace sw {

constexpr int kEdgeWords = 10;  // per boundary: the 9 class masks of its first 32 bytes + their chunk starts

// string-start bits of [p, p + 32) (bit k = byte p + k; the batch end n_bytes counts as one),
// the search narrowed to the strings of p's tile by tile_slo (k_tile_strings)
__device__ __forceinline__ uint32_t ss32_hint(const int64_t* str_off, int64_t n_str, int64_t n_bytes,
                                              const int64_t* tile_slo, int64_t n_tiles, int64_t p) {
  if (p > n_bytes) return 0u;
  int64_t lo = 0, hi = 0;
  if (p > 0) {
    const int64_t t = p >> kTileBits;
    lo = t < n_tiles ? tile_slo[t] : n_str;
    hi = t + 1 < n_tiles ? tile_slo[t + 1] : n_str;
  }
  while (lo < hi) {  // first string starting at or after p (str_off[n_str] = n_bytes >= p)
    const int64_t m = (lo + hi) >> 1;
    if (str_off[m] < p) lo = m + 1; else hi = m;
  }
  uint32_t v = 0;
  for (int64_t i = lo; i <= n_str; ++i) {
    const int64_t o = str_off[i];
    if (o >= p + 32) break;
    v |= 1u << (o - p);
  }
  return v;
}

// Special-token occurrences (SpArgs) in the pre-split: both ends of an occurrence are string
// boundaries, and the bits strictly inside it are cleared (it is one chunk).  The first
// occurrence whose end (pos + len) is at or after p: ends ascend; the ones before tile_sp[t] - 1
// end before tile t's first byte, and tile_sp[t + 1]'s starts past p.
__device__ __forceinline__ int64_t sp_first_end(const SpArgs& sp, int64_t n_tiles, int64_t p) {
  const int64_t n = sp.tile_sp[n_tiles];  // (the live count: the host's, or the device finder's)
  int64_t lo = 0, hi = n;
  if (p > 0) {
    const int64_t t = p >> kTileBits;
    if (t < n_tiles) {
      lo = max(sp.tile_sp[t] - 1, (int64_t)0);
      hi = sp.tile_sp[t + 1];
    } else {
      lo = max(n - 1, (int64_t)0);
    }
  }
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (sp.pos[m] + sp.len[m] < p) lo = m + 1; else hi = m;
  }
  return lo;
}

// bits of [p, p + 32): the occurrences' starts and ends (*ss) and their inner bytes (*inner)
// (j0: an index known to be at or before the first occurrence ending at or after p, or -1)
__device__ __forceinline__ void sp_bits32(const SpArgs& sp, int64_t n_tiles, int64_t p, uint32_t* ss, uint32_t* inner,
                                          int64_t j0 = -1) {
  uint32_t s = 0, in = 0;
  const int64_t n = sp.tile_sp[n_tiles];
  for (int64_t j = j0 >= 0 ? j0 : sp_first_end(sp, n_tiles, p); j < n; ++j) {
    const int64_t a = sp.pos[j], e = a + sp.len[j];
    if (a >= p + 32) break;
    if (a >= p) s |= 1u << (a - p);
    if (e >= p && e < p + 32) s |= 1u << (e - p);
    const int64_t lo = max(a + 1, p) - p, hi = min(e, p + 32) - p;  // inner bytes, chunk-relative
    if (lo < hi) in |= (hi - lo >= 32 ? ~0u : ((1u << (hi - lo)) - 1u)) << lo;
  }
  *ss = s;
  *inner = in;
}

struct GSrc;
__device__ __forceinline__ psb::Masks gsrc_masks(const GSrc& s, int64_t c);

// psb::carries' view of the batch from global memory only (k_edges, and k_split_classify's walks
// past its tile): every chunk classified from its 40 bytes
struct GSrc {
  PbArgs g;
  int64_t n_tiles, n_chunks;
  bool cl;
  __device__ __forceinline__ uint32_t ss_at(int64_t q) const {
    uint32_t v = ss32_hint(g.str_off, g.n_str, g.n_bytes, g.tile_slo, n_tiles, q);
    if (g.sp.n > 0) {
      uint32_t s, in;
      sp_bits32(g.sp, n_tiles, q, &s, &in);
      v |= s;
    }
    return v;
  }
  __device__ __forceinline__ uint32_t ss(int64_t c) const { return ss_at(32 * c); }
  __device__ __forceinline__ psb::Masks get(int64_t c) const {
    if (c < 0 || c >= n_chunks) return psb::Masks{};
    return gsrc_masks(*this, c);
  }
};

__device__ __forceinline__ psb::Masks gsrc_masks(const GSrc& s, int64_t c) {
  psb::RegBytes by;
  pb_load40(s.g, 32 * c, by.w);
  const uint64_t ss = (uint64_t)s.ss_at(32 * c - 4) | ((uint64_t)(s.ss_at(32 * c + 28) & 0xFFu) << 32);
  return psb::classify(by, ss, UcdClass{}, s.cl);
}

// string starts (special-token ends included) of [base, base + 160) as five words, from ONE
// search of str_off (and of the occurrences) -- k_edges' three classifies and its rules window
// otherwise searched eight times, each a chain of dependent loads
struct SsWin5 {
  uint32_t w[5];
  int64_t base;
  __device__ __forceinline__ uint32_t at(int64_t q) const {  // bits of [q, q + 32), q in [base, base + 128]
    const int r = (int)(q - base), i = r >> 5, sh = r & 31;
    uint32_t lo = w[0], hi = w[1];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      lo = i == k ? w[k] : lo;
      hi = i == k ? w[k + 1] : hi;
    }
    return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
  }
};

__device__ __forceinline__ void ss_win5(const PbArgs& g, int64_t n_tiles, int64_t base, SsWin5* out, int64_t sp_j0 = -1) {
  out->base = base;
#pragma unroll
  for (int k = 0; k < 5; ++k) out->w[k] = 0u;
  const int64_t end = base + 160;
  auto set = [&](int64_t q) {
    if (q >= base && q < end) {
      const int r = (int)(q - base);
#pragma unroll
      for (int k = 0; k < 5; ++k) out->w[k] |= (r >> 5) == k ? 1u << (r & 31) : 0u;
    }
  };
  if (base <= g.n_bytes) {
    int64_t lo = 0, hi = 0;
    if (base > 0) {
      const int64_t t = base >> kTileBits;
      lo = t < n_tiles ? g.tile_slo[t] : g.n_str;
      hi = t + 1 < n_tiles ? g.tile_slo[t + 1] : g.n_str;
    }
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (g.str_off[m] < base) lo = m + 1; else hi = m;
    }
    for (int64_t i = lo; i <= g.n_str; ++i) {
      const int64_t o = g.str_off[i];
      if (o >= end) break;
      set(o);
    }
  }
  if (g.sp.n > 0) {
    const int64_t n = g.sp.tile_sp[n_tiles];
    for (int64_t j = sp_j0 >= 0 ? sp_j0 : sp_first_end(g.sp, n_tiles, base); j < n; ++j) {
      const int64_t a = g.sp.pos[j];
      if (a >= end) break;
      set(a);
      set(a + g.sp.len[j]);
    }
  }
}

// k_edges: per tile boundary b in [0, n_tiles] (byte 2048 b, chunk c = 64 b): the class masks of
// chunk c and its final chunk-start word (zeros past the batch).  edge[k * (n_tiles + 1) + b].
// With clr (SW_EDGE_CLEAR) its threads also clear the dedupe table (n16 16-byte words) in place of
// the memset before it (profiles/r5_ab.txt r8a-r8b).
__global__ void __launch_bounds__(256) k_edges(PbArgs g, int64_t n_tiles, int pattern, uint32_t* edge,
                                               unsigned int* redo_count, uint4* clr, int64_t n16) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b == 0) *redo_count = 0;  // (k_split_classify's redo list, empty)
  if (clr) {
    const int64_t nth = (int64_t)gridDim.x * 256;
    for (int64_t i = b; i < n16; i += nth) clr[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  if (b > n_tiles) return;
  const int64_t n_chunks = (g.n_bytes + psb::kChunk - 1) / psb::kChunk;
  const int64_t c = b << (kTileBits - 5);
  const int64_t stride = n_tiles + 1;
  const GSrc src{g, n_tiles, n_chunks, pattern == 0};
  psb::Masks m1{};
  uint32_t r = 0;
  if (c < n_chunks) {
    // (the occurrences from k_tile_specials' index for this window's start, t0 - 64)
    const int64_t spj = g.sp.n > 0 ? g.sp.tile_spw[b] : -1;
    SsWin5 sw;
    ss_win5(g, n_tiles, 32 * c - 64, &sw, spj);  // (chunks c - 1 .. c + 1 with their 4-byte margins)
    if (pattern == 2) {  // (the chunks are the strings)
      r = sw.at(32 * c);
    } else {
      // (the bytes loaded per chunk, after the search: all three loaded ahead of it held 30 more
      // registers through it and made the kernel slower, 0.077 -> 0.110 ms on C2, r8a)
      auto masks = [&](int64_t k) -> psb::Masks {
        if (k < 0 || k >= n_chunks) return psb::Masks{};
        psb::RegBytes by;
        pb_load40(g, 32 * k, by.w);
        const uint64_t s = (uint64_t)sw.at(32 * k - 4) | ((uint64_t)(sw.at(32 * k + 28) & 0xFFu) << 32);
        return psb::classify(by, s, UcdClass{}, pattern == 0);
      };
      const psb::Masks m0 = masks(c - 1), m2 = masks(c + 1);
      m1 = masks(c);
      const uint64_t ssw = (uint64_t)sw.at(32 * c - 16) | ((uint64_t)sw.at(32 * c + 16) << 32);
      uint32_t need = 0;
      r = psb::rules(m0, m1, m2, ssw, pattern == 0, psb::Carry{}, &need);
      if (need) {
        const psb::Carry cy = psb::carries(src, c, need);
        r = psb::rules(m0, m1, m2, ssw, pattern == 0, cy, &need);
      }
    }
    if (g.sp.n > 0) {  // (an occurrence's inner bytes start no chunk)
      uint32_t s, in;
      sp_bits32(g.sp, n_tiles, 32 * c, &s, &in, spj);
      r &= ~in;
    }
    if (32 * c + 32 > g.n_bytes) r &= (1u << (g.n_bytes - 32 * c)) - 1u;
  }
  edge[0 * stride + b] = m1.L; edge[1 * stride + b] = m1.N; edge[2 * stride + b] = m1.C;
  edge[3 * stride + b] = m1.P; edge[4 * stride + b] = m1.H; edge[5 * stride + b] = m1.A;
  edge[6 * stride + b] = m1.X; edge[7 * stride + b] = m1.K1; edge[8 * stride + b] = m1.K2;
  edge[9 * stride + b] = r;
}

// a lane's 40 bytes [pos - 4, pos + 36) for psb::classify: word(i) = bytes [pos - 4 + 4 i, pos + 4 i)
// from registers (the lane staged its own 32 bytes and took the words on either side from its
// neighbours: no LDS reads, whose stride of 8 dwords per lane made every one an 8-way bank
// conflict); at4(k) = bytes k .. k + 3 of the 40 (k <= 36, dynamic: the rare UTF-8 leads and
// apostrophes) from the LDS window, two reads instead of a select chain over ten registers
struct MixBytes {
  const uint32_t (&r)[10];
  const uint32_t* w;
  __device__ __forceinline__ uint32_t word(int i) const { return r[i]; }
  __device__ __forceinline__ uint32_t at4(int k) const {
    const int q = k >> 2;
    return __builtin_amdgcn_alignbyte(w[q + 1], w[q], (uint32_t)(k & 3));
  }
};

// per-wave LDS of k_split_classify
constexpr int kScPre = 32;                         // bytes staged before the tile
constexpr int kScWinWords = (kScPre + kWin) / 4 + 8;  // [t0 - 32, t0 + kWin) + a zero tail
constexpr int kScSsPre = 64;                       // string-start bits staged from t0 - 64 ...
constexpr int kScSsWords = (kScSsPre + kTile + 128) / 32;  // ... to t0 + kTile + 128
struct ScMasks {
  uint32_t m[9][66];       // class masks: chunk c0 + j at column j + 1; column 0 zeros (lane 0's left
                           // neighbour, unused: k_edges has its word), column 65 the next tile's first
  uint32_t ss[kScSsWords]; // string starts
  uint32_t in[64];         // bytes inside special-token occurrences (lane l: bits 32 l ..), if any
};
template <int kCs>
union ScSharedT {          // the masks are dead once the tile's chunk starts are known
  ScMasks pre;
  uint16_t cstart[kCs];
};
using ScShared = ScSharedT<kTile + 2>;
// The chunk starts k_split_classify's LDS holds: with fewer than a tile's 2048 (+ 2), the union is
// no larger than the masks and a block of 4 waves fits 7 blocks per CU instead of 6; a tile with
// more chunks is listed for k_split_redo, which holds them all.
constexpr int kScCsCap = 1456;  // (r7h A/B: C2 k_split_classify 2.97 -> 2.91 ms, ENTROPY 5.76 -> 5.43, 7 waves per SIMD)

// psb::carries' view inside k_split_classify: the tile's masks from LDS, the rest from global memory
struct FSrc {
  GSrc gs;
  const ScMasks* sm;
  int64_t c0, t0;
  __device__ __forceinline__ uint32_t ss_at(int64_t q) const {
    const int64_t r = q - (t0 - kScSsPre);
    if (r >= 0 && r + 32 <= (int64_t)kScSsWords * 32) {
      const int wi = (int)(r >> 5), sh = (int)(r & 31);
      const uint64_t two = (uint64_t)sm->ss[wi] | ((wi + 1 < kScSsWords ? (uint64_t)sm->ss[wi + 1] : 0ULL) << 32);
      return (uint32_t)(two >> sh);
    }
    return gs.ss_at(q);
  }
  __device__ __forceinline__ uint32_t ss(int64_t c) const { return ss_at(32 * c); }
  int64_t n_chunks;
  __device__ __forceinline__ psb::Masks get(int64_t c) const {
    const int64_t j = c - c0;
    if (j >= 0 && j < 64 && c < gs.n_chunks) {
      const int k = (int)j + 1;
      return psb::Masks{sm->m[0][k], sm->m[1][k], sm->m[2][k], sm->m[3][k], sm->m[4][k],
                        sm->m[5][k], sm->m[6][k], sm->m[7][k], sm->m[8][k]};
    }
    return gs.get(c);
  }
};

// psb::carries' view inside k_split_classify: the tile's masks (and the next tile's first chunk,
// from k_edges) and string starts in LDS, nothing else.  A walk that leaves them sets *edge: the
// tile is then redone by k_split_redo (FSrc, global memory), so that the common kernel carries no
// inlined global classify (which made it ~100 KB of code and cost spills)
struct LSrc {
  const ScMasks* sm;
  int64_t c0, t0, n_chunks;
  bool* edge;
  __device__ __forceinline__ uint32_t ss_at(int64_t q) const {
    const int64_t r = q - (t0 - kScSsPre);
    if (r >= 0 && r + 32 <= (int64_t)kScSsWords * 32) {
      const int wi = (int)(r >> 5), sh = (int)(r & 31);
      const uint64_t two = (uint64_t)sm->ss[wi] | ((wi + 1 < kScSsWords ? (uint64_t)sm->ss[wi + 1] : 0ULL) << 32);
      return (uint32_t)(two >> sh);
    }
    *edge = true;
    return 0u;
  }
  __device__ __forceinline__ uint32_t ss(int64_t c) const { return ss_at(32 * c); }
  __device__ __forceinline__ psb::Masks get(int64_t c) const {
    if (c < 0 || c >= n_chunks) return psb::Masks{};  // (past the batch: no code points)
    const int64_t j = c - c0;
    if (j >= 0 && j <= 64) {
      const int k = (int)j + 1;
      return psb::Masks{sm->m[0][k], sm->m[1][k], sm->m[2][k], sm->m[3][k], sm->m[4][k],
                        sm->m[5][k], sm->m[6][k], sm->m[7][k], sm->m[8][k]};
    }
    *edge = true;
    return psb::Masks{};
  }
};

// k_split_classify's tiles whose pre-split needs a walk past the tile (k_split_redo redoes them)
struct RedoList {
  unsigned int* count;
  int64_t* tiles;
};

// one tile: pre-split, then classify_chunks.  kRedo: the walks may read global memory (FSrc) --
// k_split_redo; else they stay in LDS (LSrc) and a tile that needs more is listed in `redo`
template <bool kSp, bool kRedo, class ShT>
__device__ __forceinline__ void split_classify_tile(const EncArgs& a, const PbArgs& g, int pattern, const uint32_t* edge,
                                                    uint32_t* bits32, int64_t tile, uint32_t* s_win, ShT* sh,
                                                    uint16_t* s_qbuf, const RedoList& redo) {
  SW_STAMP_INIT;
  const int lane = threadIdx.x & 63;
  const int64_t t0 = tile * kTile;
  const int64_t t1 = tile_end(t0, a.n_bytes);
  const int64_t n_chunks = (a.n_bytes + psb::kChunk - 1) / psb::kChunk;
  const int64_t c0 = tile << (kTileBits - 5), c = c0 + lane;
  const int64_t stride = a.n_tiles + 1;
  const bool cl = pattern == 0;
  // 1. loads: the bytes [t0 - 32, t0 + kWin) into LDS (16-byte blocks: 2 before the tile, 128 of
  //    it, 4 after), each lane its own chunk's two blocks, which it also keeps in registers for the
  //    class masks (rw), the edge words, the first strings
  const int64_t wb = t0 - kScPre;
  uint32_t rw[10];
  static_assert(kScPre == 32 && kWin == kTile + 64, "block layout of the window");
  const bool fast = ((uintptr_t)a.bytes & 15) == 0 && wb >= 0 && wb + kScPre + kWin <= a.n_bytes;
  if (fast) {
    const u32x4* src = (const u32x4*)(a.bytes + wb);
    const u32x4 x0 = SW_LDNT(src + 2 + 2 * lane), x1 = SW_LDNT(src + 3 + 2 * lane);
    // the other six blocks: lane 0 block 1 (its word before the chunk), lane 63 block 130 (its word
    // after it), lanes 1..4 blocks 0, 131..133
    const bool ex = lane < 5 || lane == 63;
    const int eb = lane == 0 ? 1 : lane == 1 ? 0 : lane == 63 ? 130 : 129 + lane;
    u32x4 xe = u32x4{0, 0, 0, 0};
    if (ex) xe = SW_LDNT(src + eb);
    *(uint4*)(s_win + 4 * (2 + 2 * lane)) = make_uint4(x0[0], x0[1], x0[2], x0[3]);
    *(uint4*)(s_win + 4 * (3 + 2 * lane)) = make_uint4(x1[0], x1[1], x1[2], x1[3]);
    if (ex) *(uint4*)(s_win + 4 * eb) = make_uint4(xe[0], xe[1], xe[2], xe[3]);
    rw[1] = x0[0]; rw[2] = x0[1]; rw[3] = x0[2]; rw[4] = x0[3];
    rw[5] = x1[0]; rw[6] = x1[1]; rw[7] = x1[2]; rw[8] = x1[3];
    // the word before the chunk: lane - 1's last; the word after it: lane + 1's first
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rw[8], 0x13C, 0xF, 0xF, false);  // wave_ror:1
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)rw[1], 0x134, 0xF, 0xF, false);  // wave_rol:1
    rw[0] = lane == 0 ? xe[3] : up;
    rw[9] = lane == 63 ? xe[0] : dn;
  } else {
    for (int i = lane; i < (kScPre + kWin) / 4; i += 64) {
      const int64_t p = wb + 4 * (int64_t)i;
      uint32_t v = 0;
      for (int k = 0; k < 4; ++k) v |= (p + k >= 0 && p + k < a.n_bytes ? (uint32_t)a.bytes[p + k] : 0u) << (8 * k);
      s_win[i] = v;
    }
  }
  if (lane < 8) s_win[(kScPre + kWin) / 4 + lane] = 0;
  if (!fast) {  // (the batch's first and last tiles, an unaligned input: the words from LDS; and
                //  the A/B build without register bytes)
    wave_sync_mem();
#pragma unroll
    for (int i = 0; i < 10; ++i) rw[i] = s_win[kScPre / 4 - 1 + 8 * lane + i];
  }
  const uint32_t r0 = edge[9 * stride + tile], r_next = edge[9 * stride + tile + 1];
  const int64_t s_first = a.tile_slo[tile];
  ScMasks& sm = sh->pre;
  if (lane < 9) sm.m[lane][65] = edge[lane * stride + tile + 1];  // (k_edges: the next tile's first chunk)
  else if (lane < 18) sm.m[lane - 9][0] = 0u;
  // 2. string starts of [t0 - kScSsPre, t0 + kTile + 128) (the batch end, str_off[n_str], included)
  for (int i = lane; i < kScSsWords; i += 64) sm.ss[i] = 0;
  wave_sync_mem();
  {
    const int64_t first = tile > 0 ? a.tile_slo[tile - 1] : 0;  // (<= the first string past t0 - kScSsPre)
    for (int64_t i0 = first; i0 <= a.n_str; i0 += 64) {
      const int64_t i = i0 + lane;
      int64_t r = (int64_t)kScSsWords * 32;
      if (i <= a.n_str) r = a.str_off[i] - (t0 - kScSsPre);
      if (r >= 0 && r < (int64_t)kScSsWords * 32) atomicOr(&sm.ss[r >> 5], 1u << (r & 31));
      if (__ballot(r < (int64_t)kScSsWords * 32) != ~0ULL) break;  // (offsets ascend: past the window)
    }
  }
  constexpr bool has_sp = kSp;
  if (has_sp) {  // special-token occurrences: their ends as string starts, their inner bytes
    sm.in[lane] = 0u;
    wave_sync_mem();
    const int64_t w0 = t0 - kScSsPre, w1 = w0 + (int64_t)kScSsWords * 32;
    // (the first occurrence ending at or after w0 = t0 - 64, from k_tile_specials: one load beside
    // the live count, where a 64-wide search of the tile's range took one to two more round trips;
    // loaded here, not at the start: held through the class masks the indices cost 0.27 ms with a
    // vector tile index, r6q, and gave nothing with the scalar one, r7x)
    const int64_t nsp = a.sp.tile_sp[a.n_tiles];
    const int64_t j_first = a.sp.tile_spw[tile];
    for (int64_t j0 = j_first; j0 < nsp; j0 += 64) {
      const int64_t j = j0 + lane;
      int64_t pa = w1, pe = w1;
      if (j < nsp) {
        pa = a.sp.pos[j];
        pe = pa + a.sp.len[j];
      }
      if (pa < w1) {
        if (pa >= w0) atomicOr(&sm.ss[(pa - w0) >> 5], 1u << ((pa - w0) & 31));
        if (pe >= w0 && pe < w1) atomicOr(&sm.ss[(pe - w0) >> 5], 1u << ((pe - w0) & 31));
        for (int64_t q = max(pa + 1, t0); q < min(pe, t0 + (int64_t)kTile);) {  // (inner bytes, word by word)
          const int64_t qe = min(min(pe, t0 + (int64_t)kTile), ((q - t0) | 31) + 1 + t0);
          const int sh = (int)((q - t0) & 31), nb = (int)(qe - q);
          atomicOr(&sm.in[(q - t0) >> 5], (nb >= 32 ? ~0u : ((1u << nb) - 1u)) << sh);
          q = qe;
        }
      }
      if (__ballot(pa < w1) != ~0ULL) break;  // (positions ascend: past the window)
    }
  }
  wave_sync_mem();
#ifdef SW_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  SW_STAMP(12);
#endif
  const FSrc src{GSrc{g, a.n_tiles, n_chunks, cl}, &sm, c0, t0, n_chunks};
  // 3. this lane's chunk: class masks (to LDS, where the rules read them: nothing is held in
  //    registers across the rare walk of psb::carries, which would otherwise cost ~60 VGPRs)
  uint32_t r = 0;
  bool unresolved = false;  // (a walk left the tile: the tile goes to k_split_redo)
  if (pattern == 2) {  // the chunks are the strings
    if (c < n_chunks) r = src.ss(c);
  } else {
    {
      psb::Masks m1{};
      if (c < n_chunks) {
        const MixBytes by{rw, s_win + (kScPre / 4 - 1) + 8 * lane};  // bytes [t0 + 32 lane - 4, +40)
        const int64_t p = 32 * c;
        const uint64_t s = (uint64_t)src.ss_at(p - 4) | ((uint64_t)(src.ss_at(p + 28) & 0xFFu) << 32);
        m1 = psb::classify(by, s, UcdClass{}, cl);
      }
      const int k = lane + 1;
      sm.m[0][k] = m1.L; sm.m[1][k] = m1.N; sm.m[2][k] = m1.C; sm.m[3][k] = m1.P; sm.m[4][k] = m1.H;
      sm.m[5][k] = m1.A; sm.m[6][k] = m1.X; sm.m[7][k] = m1.K1; sm.m[8][k] = m1.K2;
    }
    wave_sync_mem();
    SW_STAMP(13);
    auto col = [&](int k) {
      return psb::Masks{sm.m[0][k], sm.m[1][k], sm.m[2][k], sm.m[3][k], sm.m[4][k], sm.m[5][k], sm.m[6][k], sm.m[7][k], sm.m[8][k]};
    };
    if (c < n_chunks) {
      const int64_t p = 32 * c;
      const uint64_t ssw = (uint64_t)src.ss_at(p - 16) | ((uint64_t)src.ss_at(p + 16) << 32);
      uint32_t need = 0;
      r = psb::rules(col(lane), col(lane + 1), col(lane + 2), ssw, cl, psb::Carry{}, &need);
      if (lane == 0) {  // (k_edges has lane 0's word, from the previous tile's masks)
        r = r0;
        need = 0;
      }
      if (need) {
        if constexpr (kRedo) {
          const psb::Carry cy = psb::carries(src, c, need);
          asm volatile("" ::: "memory");  // (the masks re-read from LDS, not kept live across the walk)
          r = psb::rules(col(lane), col(lane + 1), col(lane + 2), ssw, cl, cy, &need);
        } else {
          bool hit = false;
          const LSrc ls{&sm, c0, t0, n_chunks, &hit};
          const psb::Carry cy = psb::carries(ls, c, need);
          asm volatile("" ::: "memory");
          if (hit) unresolved = true;
          else r = psb::rules(col(lane), col(lane + 1), col(lane + 2), ssw, cl, cy, &need);
        }
      }
    }
  }
  if (c < n_chunks) {
    if (has_sp && lane > 0) r &= ~sm.in[lane];  // (lane 0: k_edges cleared them)
    if (32 * c + 32 > a.n_bytes) r &= (1u << (a.n_bytes - 32 * c)) - 1u;
  }
  if constexpr (!kRedo) {
    constexpr int kCap = (int)(sizeof(sh->cstart) / sizeof(uint16_t)) - 2;
    bool over = false;  // (more chunk starts than the LDS list holds)
    if constexpr (kCap < kTile) over = wave_sum((uint32_t)__popc(c < n_chunks ? r : 0u), lane) > (uint32_t)kCap;
    if (__ballot(unresolved) || over) {  // (rare: nothing of the tile is written yet; k_split_redo does it all)
      if (lane == 0) redo.tiles[atomicAdd(redo.count, 1u)] = tile;
      return;
    }
  }
  if (c < n_chunks) {
    bits32[c] = r;
    if (c == n_chunks - 1 && (c & 1) == 0) bits32[c + 1] = 0;  // (the last word's upper half)
  }
  SW_STAMP(14);
  // 4. the end of the tile's last chunk: the first chunk start of the next tile (k_edges)
  int rel_end;
  if (t1 >= a.n_bytes) rel_end = (int)(a.n_bytes - t0);
  else if (r_next != 0) rel_end = kTile + __builtin_ctz(r_next);
  else if (a.n_bytes <= t1 + 32) rel_end = (int)(a.n_bytes - t0);
  else rel_end = kRelEndLong;
  wave_sync_mem();  // (the masks' LDS becomes the chunk-start list)
    classify_chunks<kSp>(a, tile, s_win + kScPre / 4, sh->cstart, s_qbuf, r, rel_end, s_first, -1, -1);
}

template <bool kSp>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(7, 7)))
k_split_classify(EncArgs a, PbArgs g, int pattern, const uint32_t* edge, uint32_t* bits32, RedoList redo) {
  __shared__ __attribute__((aligned(16))) uint32_t s_win_all[kWaves][kScWinWords];
  __shared__ ScSharedT<kScCsCap> s_sh_all[kWaves];
  __shared__ uint16_t s_qb_all[kWaves][kQBuf];
  const int wv = wave_in_block_s();
  const int64_t tile = (int64_t)blockIdx.x * kWaves + wv;
  if (tile < a.n_tiles)
    split_classify_tile<kSp, false>(a, g, pattern, edge, bits32, tile, s_win_all[wv], &s_sh_all[wv], s_qb_all[wv],
                                    redo);
}

// the tiles k_split_classify listed (a run crossing the tile: walks over global memory), one wave
// each, the waves of a fixed grid taking them in turn
constexpr int kRedoGrid = 256;
template <bool kSp>
__global__ void __launch_bounds__(kThreads) k_split_redo(EncArgs a, PbArgs g, int pattern, const uint32_t* edge,
                                                         uint32_t* bits32, RedoList redo) {
  __shared__ __attribute__((aligned(16))) uint32_t s_win_all[kWaves][kScWinWords];
  __shared__ ScShared s_sh_all[kWaves];
  __shared__ uint16_t s_qb_all[kWaves][kQBuf];
  const int wv = wave_in_block_s();
  // (the count and the list are this launch's, written by k_split_classify: read them coherently,
  // never through the scalar cache, which can hold an earlier launch's values)
  const int64_t n = (int64_t)__hip_atomic_load(redo.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int64_t i = (int64_t)blockIdx.x * kWaves + wv; i < n; i += (int64_t)gridDim.x * kWaves) {
    const int64_t tile = __hip_atomic_load(&redo.tiles[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    split_classify_tile<kSp, true>(a, g, pattern, edge, bits32, tile, s_win_all[wv], &s_sh_all[wv], s_qb_all[wv],
                                   redo);
    wave_sync_mem();  // (the next tile reuses the wave's LDS)
  }
}

}  // namespace sw
