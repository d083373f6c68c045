// The special-token finder on the device (sw_find_specials_device): the occurrences that
// sw_find_specials_host finds on host threads (specials.cpp), bit for bit.  The rule (build-defined:
// the reference stores special_tokens, shredword/base.py:103, but defines no split): scanning each
// string left to right, the first position where some special matches starts an occurrence; at one
// position the first special in dict order wins; the scan resumes after it.
//
// Leftmost-first with resumption is a sequential rule, but its chain is short: an occurrence only
// hides the candidates that start inside it.  A candidate (a position where some special matches
// inside its string) that no earlier candidate covers is an occurrence ("clean"); the candidates a
// clean one covers form its cluster, which the sequential scan walks left to right, and so does one
// lane here (rare: only specials that overlap themselves or each other make clusters).
//
// The common path is one pass over the input, one wave per 2 KiB tile (k_sp_find): the tile and 128
// bytes before it staged in LDS with their string starts, every candidate of that window found
// (the first byte against the specials' first bytes by SWAR compares, the rest only there) and
// recorded in LDS as its special's index, the clusters walked from every clean candidate of the
// last 64 bytes before the tile on, and the tile's occurrences listed per tile; then a scan of the
// per-tile counts and k_sp_emit writes them out, ascending.  A cluster that began more than 64
// bytes before its tile (a long run of overlapping candidates, e.g. "aaaa..." with "aa" and "aaa")
// cannot be walked inside one window: the tile raises a flag, and the launch is redone by the
// global-memory path (k_sp_detect / k_sp_resolve / k_sp_count / k_sp_write: one bit per byte,
// clusters walked across tiles), whose kernels return at once when the flag is clear.
// Included by encode.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace sw {

constexpr int kSpMaxLen = 64;     // the longest special the device finder takes (longer: host finder)
constexpr int kSpMaxFirstSwar = 4;  // distinct first bytes compared by SWAR (more: a bit set in LDS)

// the tokenizer's specials on the device (sw_encoder_set_specials)
struct SpTab {
  const uint8_t* bytes;  // every special's bytes, concatenated
  const int32_t* off;    // [n + 1]
  const int32_t* ids;    // [n]
  const int32_t* list;   // the non-empty specials grouped by first byte, dict order within a group
  const int32_t* first;  // [257]: first byte b's group is list[first[b] .. first[b + 1])
  uint32_t filt[8];      // the first-byte set
  uint32_t fb;           // the distinct first bytes, one per byte (n_first <= kSpMaxFirstSwar)
  int32_t n_first;
  int32_t max_len;
  int32_t n;
  const uint32_t* img;   // the table as k_sp_find stages it in LDS (layout above sft_len)
  int32_t img_words, o_first, o_rec, o_tag, o_words;
};

struct SpFind {
  const uint8_t* bytes;
  int64_t n_bytes;
  const int64_t* str_off;
  int64_t n_str;
  const int64_t* tile_slo;  // k_tile_strings
  int64_t n_tiles;
  uint32_t* cbits;   // [n_tiles * 64] candidate starts, one bit per byte
  uint32_t* chosen;  // [n_tiles * 64] occurrence starts
  uint32_t* tcand;   // [n_tiles] candidates per tile
  uint32_t* tcnt;    // [n_tiles] occurrences per tile
  uint32_t* list;    // [n_tiles * tcap] k_sp_find: per tile, its occurrences (offset | special << 11)
  int64_t tcap;
  unsigned int* flag;  // set by k_sp_find: the global-memory path redoes the launch
};

// the end of the string holding byte p: the first string start past p
__device__ __forceinline__ int64_t sp_str_end(const SpFind& f, int64_t p) {
  const int64_t t = p >> kTileBits;
  int64_t lo = f.tile_slo[t], hi = t + 1 < f.n_tiles ? f.tile_slo[t + 1] : f.n_str;
  while (lo < hi) {  // (str_off[hi] > p: the next tile's first string, or the batch end)
    const int64_t m = (lo + hi) >> 1;
    if (f.str_off[m] <= p) lo = m + 1; else hi = m;
  }
  return f.str_off[lo];
}

// the special matching at p inside [p, end): the first of its first byte's group, in dict order,
// or -1
__device__ __forceinline__ int32_t sp_match(const SpTab& T, const SpFind& f, int64_t p, int64_t end) {
  const uint32_t b = f.bytes[p];
  for (int32_t g = T.first[b]; g < T.first[b + 1]; ++g) {
    const int32_t k = T.list[g];
    const int32_t o = T.off[k], L = T.off[k + 1] - o;
    if (p + L > end) continue;
    bool same = true;
    for (int32_t q = 1; q < L && same; ++q) same = f.bytes[p + q] == T.bytes[o + q];
    if (same) return k;
  }
  return -1;
}
__device__ __forceinline__ int32_t sp_len_at(const SpTab& T, const SpFind& f, int64_t p) {
  const int32_t k = sp_match(T, f, p, sp_str_end(f, p));
  return k < 0 ? 0 : T.off[k + 1] - T.off[k];
}

// exact zero bytes of x: bit 7 of each zero byte lane
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
__device__ __forceinline__ uint32_t mm4_hi(uint32_t x) { return ((x & 0x80808080u) * 0x00204081u) >> 28; }

// k_sp_detect: lane l of tile t's wave owns bytes [t0 + 32 l, + 32)
template <bool kSwar>
__global__ void __launch_bounds__(kThreads) k_sp_detect(SpTab T, SpFind f) {
  if (__hip_atomic_load(f.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;  // (the common path did it)
  __shared__ uint32_t s_filt[8];
  if (!kSwar) {
    if (threadIdx.x < 8) s_filt[threadIdx.x] = T.filt[threadIdx.x];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave_in_block(); t < f.n_tiles; t += (int64_t)gridDim.x * kWaves) {
  const int64_t p0 = (t << kTileBits) + 32 * lane;
  uint32_t w[8];
  if (((uintptr_t)f.bytes & 15) == 0 && p0 + 32 <= f.n_bytes) {
    const u32x4 x0 = SW_LDNT((const u32x4*)(f.bytes + p0)), x1 = SW_LDNT((const u32x4*)(f.bytes + p0 + 16));
    w[0] = x0[0]; w[1] = x0[1]; w[2] = x0[2]; w[3] = x0[3];
    w[4] = x1[0]; w[5] = x1[1]; w[6] = x1[2]; w[7] = x1[3];
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t v = 0;
      for (int k = 0; k < 4; ++k) {
        const int64_t p = p0 + 4 * i + k;
        v |= (p < f.n_bytes ? (uint32_t)f.bytes[p] : 0u) << (8 * k);
      }
      w[i] = v;
    }
  }
  uint32_t m = 0;  // bytes whose value starts some special
  if (kSwar) {
    for (int j = 0; j < T.n_first; ++j) {
      const uint32_t fb = ((T.fb >> (8 * j)) & 0xFFu) * 0x01010101u;
#pragma unroll
      for (int i = 0; i < 8; ++i) m |= mm4_hi(zero_bytes(w[i] ^ fb)) << (4 * i);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      for (int k = 0; k < 4; ++k) {
        const uint32_t b = (w[i] >> (8 * k)) & 0xFFu;
        m |= ((s_filt[b >> 5] >> (b & 31)) & 1u) << (4 * i + k);
      }
  }
  if (p0 + 32 > f.n_bytes) m &= p0 >= f.n_bytes ? 0u : (1u << (f.n_bytes - p0)) - 1u;
  // full matches only (inside the string)
  uint32_t c = 0;
  int64_t end = -1;
  for (uint32_t x = m; x; x &= x - 1) {
    const int64_t p = p0 + __builtin_ctz(x);
    if (p >= end) end = sp_str_end(f, p);
    if (sp_match(T, f, p, end) >= 0) c |= 1u << __builtin_ctz(x);
  }
  f.cbits[t * 64 + lane] = c;
  f.chosen[t * 64 + lane] = 0u;
  const uint32_t n = wave_sum((uint32_t)__popc(c), lane);
  if (lane == 0) f.tcand[t] = n;
  }
}

// the next candidate at or after q, below lim (-1: none); one word of the candidate bits at a time
__device__ __forceinline__ int64_t sp_next_cand(const SpFind& f, int64_t q, int64_t lim) {
  lim = min(lim, f.n_bytes);
  while (q < lim) {
    const uint32_t word = f.cbits[q >> 5] >> (q & 31);
    if (word) {
      const int64_t r = q + __builtin_ctz(word);
      return r < lim ? r : -1;
    }
    q = (q | 31) + 1;
  }
  return -1;
}

__global__ void __launch_bounds__(kThreads) k_sp_count(SpFind f) {
  if (__hip_atomic_load(f.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  const int lane = threadIdx.x & 63;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave_in_block(); t < f.n_tiles; t += (int64_t)gridDim.x * kWaves) {
    const uint32_t n = wave_sum(f.tcand[t] ? (uint32_t)__popc(f.chosen[t * 64 + lane]) : 0u, lane);
    if (lane == 0) f.tcnt[t] = n;
  }
}

__global__ void __launch_bounds__(kThreads) k_sp_write(SpTab T, SpFind f, const int64_t* toff, int64_t* pos,
                                                       int32_t* len, int32_t* id) {
  if (__hip_atomic_load(f.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  const int lane = threadIdx.x & 63;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave_in_block(); t < f.n_tiles; t += (int64_t)gridDim.x * kWaves) {
  if (f.tcnt[t] == 0) continue;
  const uint32_t c = f.chosen[t * 64 + lane];
  const uint32_t cnt = (uint32_t)__popc(c);
  const uint32_t incl = wave_incl_scan(cnt, lane);
  int64_t o = toff[t] + (incl - cnt);
  const int64_t p0 = (t << kTileBits) + 32 * lane;
  for (uint32_t x = c; x; x &= x - 1) {
    const int64_t p = p0 + __builtin_ctz(x);
    const int32_t k = sp_match(T, f, p, sp_str_end(f, p));
    pos[o] = p;
    len[o] = T.off[k + 1] - T.off[k];
    id[o] = T.ids[k];
    ++o;
  }
  }
}

// ---- the one-pass path ---------------------------------------------------------------------
constexpr int kSfPre = 128;                          // bytes staged before the tile
constexpr int kSfBytes = kSfPre + kTile + kSpMaxLen;  // the byte window [t0 - 128, t0 + 2048 + 64)
constexpr int kSfCand = kSfPre + kTile;              // candidate positions [t0 - 128, t0 + 2048)
constexpr int kSfCandWords = kSfCand / 32;
static_assert(kSfCand == 64 * 34, "k_sp_find: 34 candidate positions a lane");
constexpr int kSfSsWords = (kSfBytes + 32) / 32 + 1; // string-start bits of the window (+ its end)

struct SfShared {
  uint32_t b[kSfBytes / 4 + 4];  // the window's bytes (zeros outside the batch)
  uint32_t ss[kSfSsWords];       // string starts (the batch end included)
  uint32_t cb[kSfCandWords];     // candidates: some special matches there, inside its string
  uint32_t chosen[kTile / 32];   // occurrences starting in the tile
  uint32_t seen[kTile / 32];     // tile candidates some cluster walk decided
  uint8_t ci[kSfCand];           // a candidate's special (valid where cb is set)
};

// The specials' table as k_sp_find stages it in LDS (SpTab.img, built by sw_encoder_set_specials),
// 32-bit words:
//   [0, n)                special k: its first word in the byte area | its length << 16
//   [o_first, + 129)      first byte b's group starts at list entry group[b] (16 bits each, 257)
//   [o_rec, + 8 x list)   per list entry (the specials grouped by first byte, dict order within a
//                         group): the special's first 16 bytes zero padded, then their byte masks
//                         (16-byte aligned: two ds_read_b128, no chain through an index)
//   [o_tag, + list)       per list entry: special k | length << 8 | its first word in the byte area << 16
//   [o_words, ...)        every special's bytes from a word boundary, zero padded
constexpr int kSfRecWords = 8;
__device__ __forceinline__ int sft_len(const uint32_t* s, int k) { return (int)(s[k] >> 16); }
__device__ __forceinline__ int sft_group(const uint32_t* s, int o_first, int b) {
  return (int)((s[o_first + (b >> 1)] >> (16 * (b & 1))) & 0xFFFFu);
}
// the window's bytes r .. r + 3 as one word
__device__ __forceinline__ uint32_t sf_word(const SfShared& m, int r) {
  const int w = r >> 2;
  return __builtin_amdgcn_alignbyte(m.b[w + 1], m.b[w], (uint32_t)(r & 3));
}

// the first string start in (r, r + 64], r + 65 when there is none (a special of <= 64 bytes at r
// fits its string when it ends at or before it): three independent LDS reads instead of a word by
// word walk to the string's end, a chain of dependent reads as long as the string
__device__ __forceinline__ int sf_end_after(const SfShared& m, int r) {
  static_assert(kSpMaxLen <= 64 && kSfCand + 64 < 32 * (kSfSsWords - 1), "sf_end_after's three words");
  const int q = r + 1, w = q >> 5, sh = q & 31;
  const uint64_t lo = ((uint64_t)m.ss[w + 1] << 32) | m.ss[w];
  const uint64_t bits = (lo >> sh) | (sh ? (uint64_t)m.ss[w + 2] << (64 - sh) : 0ULL);
  return bits ? q + __builtin_ctzll(bits) : q + 64;
}

// ---- the global path's cluster walks ----------------------------------------------------------
// k_sp_resolve: the clean candidates (no earlier candidate covers them) found lane by lane, then each
// one's cluster walked by the whole wave, left to right as the sequential scan goes, 64 positions a
// step: the step's candidate bits and its 128 bytes (every special starting in it fits) staged in
// the wave's LDS, each lane matching one position against the LDS records; the step's end of the
// cluster by a prefix max of the candidates' ends and its choices by successor pointers (sr_walk)
// -- where one lane walking one candidate a step of dependent table loads took ~1 us a position of
// a run of self-overlapping specials, this takes ~35 ns (tools/probe_long_cluster.py)
constexpr int kSrWinWords = 32;  // 128 bytes: 64 positions + the longest special (64)

// the special matching at window offset j (< 64) inside [j, end) (end: the string's end, window-relative)
__device__ __forceinline__ int sr_match(const uint32_t* s, const SpTab& T, const uint32_t* win, int j, int64_t end) {
  uint32_t x[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) x[q] = __builtin_amdgcn_alignbyte(win[(j >> 2) + q + 1], win[(j >> 2) + q], (uint32_t)(j & 3));
  const int b = (int)(x[0] & 0xFFu);
  const int g1 = sft_group(s, T.o_first, b + 1);
  const uint8_t* wb = (const uint8_t*)win;
  for (int gi = sft_group(s, T.o_first, b); gi < g1; ++gi) {
    const uint4 w = *(const uint4*)(s + T.o_rec + kSfRecWords * gi);
    const uint4 mk4 = *(const uint4*)(s + T.o_rec + kSfRecWords * gi + 4);
    const uint32_t tag = s[T.o_tag + gi];
    const int L = (int)((tag >> 8) & 0xFFu);
    if (j + L > end) continue;
    bool same = (((x[0] ^ w.x) & mk4.x) | ((x[1] ^ w.y) & mk4.y) | ((x[2] ^ w.z) & mk4.z) | ((x[3] ^ w.w) & mk4.w)) == 0;
    const uint8_t* sb = (const uint8_t*)(s + T.o_words + (int)(tag >> 16));
    for (int q = 16; q < L && same; ++q) same = wb[j + q] == sb[q];
    if (same) return (int)(tag & 0xFFu);
  }
  return -1;
}

// the cluster of clean candidate p (wave-uniform), walked by the whole wave
__device__ __forceinline__ void sr_walk(const uint32_t* s, const SpTab& T, const SpFind& f, uint32_t* win, int64_t p,
                                        int lane) {
  const int64_t E = sp_str_end(f, p);  // (the cluster lies in p's string: no match crosses its end)
  const int32_t L = sp_len_at(T, f, p);
  if (lane == 0) atomicOr(&f.chosen[p >> 5], 1u << (p & 31));
  int64_t span = p + L, taken = p + L;
  const bool al4 = ((uintptr_t)f.bytes & 3) == 0;
  for (int64_t w0 = (p + 1) & ~(int64_t)63; w0 < span && w0 < f.n_bytes; w0 += 64) {
    uint64_t cand = (uint64_t)f.cbits[w0 >> 5] | ((uint64_t)f.cbits[(w0 >> 5) + 1] << 32);
    uint32_t v = 0;  // (the window's bytes, loaded beside its candidate bits: one round trip a step)
    if (lane < kSrWinWords) {
      const int64_t q = w0 + 4 * lane;
      if (al4 && q + 4 <= f.n_bytes) {
        v = *(const uint32_t*)(f.bytes + q);
      } else {
        for (int k = 0; k < 4; ++k) v |= (q + k < f.n_bytes ? (uint32_t)f.bytes[q + k] : 0u) << (8 * k);
      }
    }
    if (w0 < p + 1) cand &= ~0ULL << (int)(p + 1 - w0);
    if (!cand) continue;
    if (lane < kSrWinWords) win[lane] = v;
    if (lane == 0) win[kSrWinWords] = 0u;  // (the word after the window: read by the alignbyte of the last, masked out)
    wave_sync_mem();
    int Li = 0;  // (this lane's position's match length, 0: none)
    if ((cand >> lane) & 1ULL) {
      const int k = sr_match(s, T, win, lane, E - w0);
      Li = k < 0 ? 0 : sft_len(s, k);
    }
    // the step's choices without a lane-serial pass: the cluster ends at the first candidate no earlier
    // one reaches (a prefix max of the candidates' ends), and the choices are the chain from the first
    // candidate at or after `taken`, each one's successor the first candidate at or after its end
    const bool c = ((cand >> lane) & 1ULL) != 0;
    const int64_t sp_rel = span - w0, tk_rel = taken - w0;  // (wave-uniform)
    int ext = c ? lane + Li : -1;  // (a candidate's end, window-relative)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {  // inclusive prefix max over the lanes
      const int o = __shfl_up(ext, d, 64);
      if (lane >= d) ext = max(ext, o);
    }
    const int before = __shfl_up(ext, 1, 64);  // (exclusive: the candidates before this lane)
    const int64_t reach = max(sp_rel, (int64_t)(lane == 0 ? -1 : before));
    const uint64_t ends = __ballot(c && (int64_t)lane >= reach);
    const int s_end = ends ? __builtin_ctzll(ends) : 64;  // (the first candidate past the cluster)
    const bool stop = ends != 0;
    const uint64_t live = cand & (s_end >= 64 ? ~0ULL : ((1ULL << s_end) - 1ULL));
    // successor of lane i: the first live candidate at or after i + L_i (64: none in this step)
    const int e = lane + max(Li, 1);  // (a live candidate always matches, L >= 1; the guard keeps the hops moving)
    const uint64_t after = e >= 64 ? 0ULL : (live & (~0ULL << e));
    const int nxt = after ? __builtin_ctzll(after) : 64;
    uint64_t ch = 0;
    int last = -1;
    {
      const uint64_t from = tk_rel <= 0 ? live : tk_rel >= 64 ? 0ULL : (live & (~0ULL << (int)tk_rel));
      for (int r = from ? __builtin_ctzll(from) : 64; r < 64; r = __builtin_amdgcn_readlane(nxt, r)) {
        ch |= 1ULL << r;
        last = r;
      }
    }
    if (last >= 0) taken = w0 + last + __builtin_amdgcn_readlane(Li, last);
    {
      const int lm = live ? 63 - __builtin_clzll(live) : -1;  // (the last live candidate: the running max there)
      if (lm >= 0) span = max(span, w0 + (int64_t)__builtin_amdgcn_readlane(ext, lm));
    }
    if (lane == 0 && (uint32_t)ch) atomicOr(&f.chosen[w0 >> 5], (uint32_t)ch);
    if (lane == 1 && (uint32_t)(ch >> 32)) atomicOr(&f.chosen[(w0 >> 5) + 1], (uint32_t)(ch >> 32));
    wave_sync_mem();  // (the window is rewritten by the next step)
    if (stop) break;
  }
}

__global__ void __launch_bounds__(kThreads) k_sp_resolve(SpTab T, SpFind f) {
  if (__hip_atomic_load(f.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  extern __shared__ __align__(16) uint32_t s_sft[];  // T.img (its records)
  __shared__ uint32_t s_win[kWaves][kSrWinWords + 4];
  for (int i = threadIdx.x; i < T.img_words; i += kThreads) s_sft[i] = T.img[i];
  __syncthreads();
  const uint32_t* s = s_sft;
  uint32_t* win = s_win[wave_in_block()];
  const int lane = threadIdx.x & 63;
  for (int64_t t = (int64_t)blockIdx.x * kWaves + wave_in_block(); t < f.n_tiles; t += (int64_t)gridDim.x * kWaves) {
    if (f.tcand[t] == 0) continue;
    const int64_t p0 = (t << kTileBits) + 32 * lane;
    uint32_t heads = 0;  // this lane's clean candidates
    for (uint32_t x = f.cbits[t * 64 + lane]; x; x &= x - 1) {
      const int64_t p = p0 + __builtin_ctz(x);
      // clean: no earlier candidate covers p (candidates never cross a string; one inside an earlier
      // tile is read from its bits too)
      bool clean = true;
      for (int64_t q = sp_next_cand(f, max(p - (T.max_len - 1), (int64_t)0), p); q >= 0 && clean;
           q = sp_next_cand(f, q + 1, p))
        clean = q + sp_len_at(T, f, q) <= p;
      if (clean) heads |= 1u << __builtin_ctz(x);
    }
    for (uint64_t hl = __ballot(heads != 0); hl; hl &= hl - 1) {  // (the walks, one head at a time)
      const int hlane = __builtin_ctzll(hl);
      for (uint32_t hb = (uint32_t)__shfl((int)heads, hlane, 64); hb; hb &= hb - 1)
        sr_walk(s, T, f, win, (t << kTileBits) + 32 * hlane + __builtin_ctz(hb), lane);
    }
  }
}

// the next candidate at or after q, below lim (lim when none)
__device__ __forceinline__ int sf_next_cand(const SfShared& m, int q, int lim) {
  lim = min(lim, kSfCand);
  while (q < lim) {
    const uint32_t w = m.cb[q >> 5] >> (q & 31);
    if (w) return min(q + __builtin_ctz(w), lim);
    q = (q | 31) + 1;
  }
  return lim;
}

// clean: no earlier candidate (within the longest special) covers r
__device__ __forceinline__ bool sf_clean(const SfShared& m, const uint32_t* s, int r, int max_len) {
  for (int q = sf_next_cand(m, max(r - (max_len - 1), 0), r); q < r; q = sf_next_cand(m, q + 1, r))
    if (q + sft_len(s, m.ci[q]) > r) return false;
  return true;
}

template <bool kSwar>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(7, 7)))
k_sp_find(SpTab T, SpFind f) {
  extern __shared__ __align__(16) uint32_t s_sft[];  // T.img (T.img_words words; its records 16-byte aligned)
  __shared__ SfShared s_all[kWaves];
  __shared__ uint32_t s_filt[8];
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * kWaves + wave_in_block();
  const int64_t tc = min(t, f.n_tiles - 1);
  // the loads whose latencies overlap: the window's first string, the window's bytes, then its
  // string offsets (waiting for the first only)
  const int64_t first = tc > 0 ? f.tile_slo[tc - 1] : 0;  // (<= the first string starting in the window)
  const int64_t t0 = tc << kTileBits, wb = t0 - kSfPre;
  const bool fast = ((uintptr_t)f.bytes & 15) == 0 && wb >= 0 && wb + kSfBytes <= f.n_bytes;
  constexpr int kSfVec = (kSfBytes / 16 + 63) / 64;  // 16-byte loads a lane
  u32x4 xs[kSfVec];
  if (fast) {
#pragma unroll
    for (int j = 0; j < kSfVec; ++j) {
      const int i = lane + 64 * j;
      if (i < kSfBytes / 16) xs[j] = SW_LDNT((const u32x4*)(f.bytes + wb) + i);
    }
  }
  const int64_t span = (int64_t)kSfSsWords * 32;
  int64_t r0 = span;
  if (first + lane <= f.n_str) r0 = f.str_off[first + lane] - wb;
  for (int i = threadIdx.x; i < T.img_words; i += kThreads) s_sft[i] = T.img[i];
  if (!kSwar && threadIdx.x < 8) s_filt[threadIdx.x] = T.filt[threadIdx.x];
  __syncthreads();
  const uint32_t* s = s_sft;
  if (t >= f.n_tiles) return;
  SfShared& m = s_all[wave_in_block()];
  // 1. the window's bytes and its string starts
  if (fast) {
#pragma unroll
    for (int j = 0; j < kSfVec; ++j) {
      const int i = lane + 64 * j;
      if (i < kSfBytes / 16) *(uint4*)(m.b + 4 * i) = make_uint4(xs[j][0], xs[j][1], xs[j][2], xs[j][3]);
    }
  } else {
    for (int i = lane; i < kSfBytes / 4; i += 64) {
      uint32_t v = 0;
      for (int k = 0; k < 4; ++k) {
        const int64_t p = wb + 4 * i + k;
        v |= (p >= 0 && p < f.n_bytes ? (uint32_t)f.bytes[p] : 0u) << (8 * k);
      }
      m.b[i] = v;
    }
  }
  if (lane < 4) m.b[kSfBytes / 4 + lane] = 0;
  for (int i = lane; i < kSfSsWords; i += 64) m.ss[i] = 0;
  for (int i = lane; i < kSfCandWords; i += 64) m.cb[i] = 0;
  m.chosen[lane] = 0;
  m.seen[lane] = 0;
  wave_sync_mem();
  for (int64_t i0 = first;;) {
    if (r0 >= 0 && r0 < span) atomicOr(&m.ss[r0 >> 5], 1u << (r0 & 31));
    if (__ballot(r0 < span) != ~0ULL) break;  // (offsets ascend: past the window)
    i0 += 64;
    if (i0 > f.n_str) break;
    r0 = i0 + lane <= f.n_str ? f.str_off[i0 + lane] - wb : span;
  }
  wave_sync_mem();
  // 2. candidates of [t0 - 128, t0 + 2048), 34 positions a lane (2176 = 64 x 34: one pass, where
  //    32 a lane took a second pass for the last four words), found by their first byte (SWAR
  //    compares, or the first-byte set) and matched word by word against the LDS table, the first
  //    match in dict order.  The first-byte hits are kept transposed (bit 8 j + k: byte j of word k)
  //    so that each word's four zero-byte flags go in by one shift; their order does not matter.
  {
    const int P = 34 * lane, w0 = P >> 2;
    const uint32_t sh = (uint32_t)(P & 3);
    uint32_t d[10], w[9];
#pragma unroll
    for (int k = 0; k < 10; ++k) d[k] = m.b[w0 + k];
#pragma unroll
    for (int k = 0; k < 9; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
    uint32_t mlo = 0, mhi = 0;  // positions P + 4 k + j (k < 8) at bit 8 j + k; P + 32, P + 33 at bits 0, 1
    if (kSwar) {
      for (int j = 0; j < T.n_first; ++j) {
        const uint32_t fb = ((T.fb >> (8 * j)) & 0xFFu) * 0x01010101u;
#pragma unroll
        for (int k = 0; k < 8; ++k) mlo |= zero_bytes(w[k] ^ fb) >> (7 - k);
        const uint32_t z = zero_bytes(w[8] ^ fb);
        mhi |= ((z >> 7) & 1u) | ((z >> 14) & 2u);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t b = (w[k] >> (8 * j)) & 0xFFu;
          mlo |= ((s_filt[b >> 5] >> (b & 31)) & 1u) << (8 * j + k);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t b = (w[8] >> (8 * j)) & 0xFFu;
        mhi |= ((s_filt[b >> 5] >> (b & 31)) & 1u) << j;
      }
    }
    uint64_t hit = 0;  // bit i: position P + i
    for (uint64_t mk = ((uint64_t)mhi << 32) | mlo; mk; mk &= mk - 1) {
      const int bt = __builtin_ctzll(mk), i = bt < 32 ? 4 * (bt & 7) + (bt >> 3) : bt;
      const int r = P + i;
      if (wb + r < 0 || wb + r >= f.n_bytes) continue;  // (positions outside the batch match nothing)
      const int end = sf_end_after(m, r);
      uint32_t x[4];  // (the first 16 bytes, once)
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = sf_word(m, r + 4 * q);
      const int b = (int)(x[0] & 0xFFu);
      const int g1 = sft_group(s, T.o_first, b + 1);
      for (int gi = sft_group(s, T.o_first, b); gi < g1; ++gi) {
        const uint4 w = *(const uint4*)(s + T.o_rec + kSfRecWords * gi);
        const uint4 mk4 = *(const uint4*)(s + T.o_rec + kSfRecWords * gi + 4);
        const uint32_t tag = s[T.o_tag + gi];
        const int L = (int)((tag >> 8) & 0xFFu);
        if (r + L > end) continue;
        bool same = (((x[0] ^ w.x) & mk4.x) | ((x[1] ^ w.y) & mk4.y) | ((x[2] ^ w.z) & mk4.z) | ((x[3] ^ w.w) & mk4.w)) == 0;
        const int wo = T.o_words + (int)(tag >> 16);
        for (int q = 16; q < L && same; q += 4) {  // (past 16 bytes: word by word)
          const uint32_t msk = L - q >= 4 ? ~0u : (1u << (8 * (L - q))) - 1u;
          same = ((sf_word(m, r + q) ^ s[wo + (q >> 2)]) & msk) == 0;
        }
        if (same) {
          m.ci[r] = (uint8_t)(tag & 0xFFu);
          hit |= 1ULL << i;
          break;
        }
      }
    }
    if (hit) {  // (34 bits from bit P & 31 of word P >> 5: two words, shared with the neighbours)
      const uint64_t h = hit << (P & 31);
      atomicOr(&m.cb[P >> 5], (uint32_t)h);
      if (h >> 32) atomicOr(&m.cb[(P >> 5) + 1], (uint32_t)(h >> 32));
    }
  }
  wave_sync_mem();
  // 3. clean candidates of [t0 - 64, t0 + 2048) and their clusters' walks (decisions inside the tile)
  for (int g = lane + 2; g < kSfCandWords; g += 64) {
    for (uint32_t x = m.cb[g]; x; x &= x - 1) {
      const int r = 32 * g + __builtin_ctz(x);
      if (!sf_clean(m, s, r, T.max_len)) continue;
      const int L = sft_len(s, m.ci[r]);
      if (r >= kSfPre) atomicOr(&m.chosen[(r - kSfPre) >> 5], 1u << ((r - kSfPre) & 31));
      int span = r + L, taken = r + L;
      for (int q = sf_next_cand(m, r + 1, span); q < span && q < kSfCand; q = sf_next_cand(m, q + 1, span)) {
        const int Lq = sft_len(s, m.ci[q]);
        if (q >= kSfPre) atomicOr(&m.seen[(q - kSfPre) >> 5], 1u << ((q - kSfPre) & 31));
        if (q >= taken) {
          if (q >= kSfPre) atomicOr(&m.chosen[(q - kSfPre) >> 5], 1u << ((q - kSfPre) & 31));
          taken = q + Lq;
        }
        span = max(span, q + Lq);
      }
    }
  }
  wave_sync_mem();
  // 4. a tile candidate no walk decided (neither clean nor reached: its cluster began before the
  //    window's decidable part) sends the launch to the global-memory path
  {
    uint32_t undecided = 0;
    for (uint32_t x = m.cb[kSfPre / 32 + lane] & ~m.chosen[lane] & ~m.seen[lane]; x; x &= x - 1) {
      const int k = __builtin_ctz(x);
      if (!sf_clean(m, s, kSfPre + 32 * lane + k, T.max_len)) undecided |= 1u << k;
    }
    if (__ballot(undecided != 0) && lane == 0) __hip_atomic_store(f.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // 5. the tile's occurrences, ascending: offset | special << 11
  const uint32_t c = m.chosen[lane];
  const uint32_t cnt = (uint32_t)__popc(c);
  const uint32_t incl = wave_incl_scan(cnt, lane);
  uint32_t o = incl - cnt;
  for (uint32_t x = c; x; x &= x - 1) {
    const int k = __builtin_ctz(x), r = kSfPre + 32 * lane + k;
    f.list[t * f.tcap + o++] = (uint32_t)(32 * lane + k) | ((uint32_t)m.ci[r] << 11);
  }
  if (lane == 63) f.tcnt[t] = incl;
}

constexpr int kSfEmitTiles = 8;  // k_sp_emit: tiles a wave
constexpr unsigned kSfGlobalBlocks = 2048;  // the global path's grid (its kernels loop over the tiles)
__global__ void __launch_bounds__(kThreads) k_sp_emit(SpTab T, SpFind f, const int64_t* toff, int64_t* pos,
                                                      int32_t* len, int32_t* id) {
  __shared__ int32_t s_len[256], s_id[256];  // (the specials' lengths and ids: <= 255 of them here)
  for (int i = threadIdx.x; i < T.n; i += kThreads) {
    s_len[i] = T.off[i + 1] - T.off[i];
    s_id[i] = T.ids[i];
  }
  __syncthreads();
  if (__hip_atomic_load(f.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;  // (the global path writes)
  const int lane = threadIdx.x & 63;
  // kSfEmitTiles tiles a wave, their lists as one: lane q < kSfEmitTiles loads tile t0 + q's count
  // and output offset, and entry j of the joined lists belongs to the tile whose prefix holds it
  const int64_t tw = ((int64_t)blockIdx.x * kWaves + wave_in_block()) * kSfEmitTiles;
  const bool mine = lane < kSfEmitTiles && tw + lane < f.n_tiles;
  const uint32_t cnt = mine ? f.tcnt[tw + lane] : 0u;
  const int64_t o_t = mine ? toff[tw + lane] : 0;
  const uint32_t incl = wave_incl_scan(cnt, lane);  // (lanes 0 .. kSfEmitTiles - 1: the tiles' prefixes)
  uint32_t pre[kSfEmitTiles];  // (every lane holds the prefixes and offsets: shuffles outside the loop)
  int64_t ob[kSfEmitTiles];
#pragma unroll
  for (int d = 0; d < kSfEmitTiles; ++d) {
    pre[d] = (uint32_t)__shfl((int)incl, d, 64);
    ob[d] = __shfl(o_t, d, 64);
  }
  const uint32_t total = pre[kSfEmitTiles - 1];
  for (uint32_t j = lane; j < total; j += 64) {
    int q = 0;  // (the tile: the first whose inclusive prefix exceeds j)
    uint32_t before = 0;
    int64_t o = ob[0];
#pragma unroll
    for (int d = 0; d < kSfEmitTiles - 1; ++d)
      if (pre[d] <= j) {
        q = d + 1;
        before = pre[d];
        o = ob[d + 1];
      }
    const int64_t t = tw + q;
    const uint32_t i = j - before;
    const uint32_t e = f.list[t * f.tcap + i];
    const int32_t k = (int32_t)(e >> 11);
    pos[o + i] = (t << kTileBits) + (int64_t)(e & 2047u);
    len[o + i] = s_len[k];
    id[o + i] = s_id[k];
  }
}

// the global path's count replaces the one-pass count when it ran
__global__ void k_sp_fix_count(const unsigned int* flag, const int64_t* total2, int64_t* count) {
  if (threadIdx.x == 0 && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) *count = *total2;
}

}  // namespace sw
