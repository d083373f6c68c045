// Device pre-split (apply_regex, shredword/base.py:38-58) into the chunk-boundary bitmap
// (bit i of word i/64 = byte i starts a chunk): k_presplit_bits, the bit-parallel form of
// presplit_bits.h.  Included by encode.hip only.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"
#include "presplit_bits.h"
#include "presplit_match.h"
#include "ucd_tables.h"

namespace sw {

__constant__ uint8_t c_ucd1[SW_UCD_STAGE1_SIZE] = SW_UCD_STAGE1_INIT;
__constant__ uint8_t c_ucd2[SW_UCD_STAGE2_SIZE] = SW_UCD_STAGE2_INIT;

__device__ inline int ucd_class(uint32_t cp) {
  if (cp > 0x10FFFF) return kOther;
  const uint32_t blk = c_ucd1[cp >> 8];
  const uint32_t v = c_ucd2[blk * 64 + ((cp & 255) >> 2)];
  return (int)((v >> ((cp & 3) * 2)) & 3);
}

struct UcdClass {
  __device__ int operator()(uint32_t cp) const { return ucd_class(cp); }
};

// ---------------------------------------------------------------------------------------------
// k_presplit_bits: the bit-parallel pre-split (presplit_bits.h).  A workgroup owns kPbBlock
// bytes, one 32-byte chunk per thread:
//   0. the string starts of [b0 - 64, b0 + kPbBlock + 64) into an LDS bitmap;
//   1. every chunk's class masks (classify) for chunks -1 .. 256 of the block, into LDS;
//   2. every thread's window rules over chunks t - 1, t, t + 1, with the run carries walked over
//      the LDS masks (and, for runs past the block, over chunks classified from global memory);
//      the 32 chunk-start bits are stored as one dword of the bitmap (no atomics, no clearing).
// ---------------------------------------------------------------------------------------------
constexpr int kPbThreads = 256;
constexpr int kPbBlock = kPbThreads * psb::kChunk;         // 8 KiB
constexpr int kPbPre = 64;                                 // string starts staged before b0 ...
constexpr int kPbSsWords = (kPbPre + kPbBlock + 128) / 32;  // ... and after the block
// LDS holds the block's own chunks 0 .. 255, one per thread; the two neighbours of the block
// (chunks -1 and 256) are classified where they are needed (threads 0 and 255)
constexpr int kPbChunks = kPbThreads;

struct PbArgs {
  const uint8_t* bytes;
  int64_t n_bytes;
  const int64_t* str_off;
  int64_t n_str;
  const int64_t* tile_slo;  // first string starting at or after each 2 KiB tile (k_tile_strings)
  SpArgs sp;                // special-token occurrences: their ends are string boundaries (fused path only)
};

// string-start bits of bytes [p, p + 32) from str_off (batch end included): global fallback
__device__ __forceinline__ uint32_t pb_ss_global(const PbArgs g, int64_t p) {
  int64_t lo = 0, hi = g.n_str;  // first string start >= p
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (g.str_off[m] < p) lo = m + 1; else hi = m;
  }
  uint32_t v = 0;
  for (int64_t i = lo; i <= g.n_str; ++i) {
    const int64_t o = g.str_off[i];
    if (o >= p + 32) break;
    v |= 1u << (o - p);
  }
  return v;
}

// the 40 bytes [p - 4, p + 36) as words (zeros outside the batch); vector loads when in range
__device__ __forceinline__ void pb_load40(const PbArgs g, int64_t p, uint32_t* w) {
  if (p - 4 >= 0 && p + 36 <= g.n_bytes && (((uintptr_t)(g.bytes + p) & 15) == 0)) {
    const uint4 a = *(const uint4*)(g.bytes + p), b = *(const uint4*)(g.bytes + p + 16);
    w[0] = *(const uint32_t*)(g.bytes + p - 4);
    w[1] = a.x; w[2] = a.y; w[3] = a.z; w[4] = a.w;
    w[5] = b.x; w[6] = b.y; w[7] = b.z; w[8] = b.w;
    w[9] = *(const uint32_t*)(g.bytes + p + 32);
    return;
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t q = p - 4 + 4 * i + k;
      v |= (q >= 0 && q < g.n_bytes) ? (uint32_t)g.bytes[q] << (8 * k) : 0u;
    }
    w[i] = v;
  }
}

struct PbSrc {  // psb::carries' view: the block's chunks from LDS, the others classified on the fly
  PbArgs g;                         // (by value: a pointer to the kernel argument puts it on the stack)
  const uint32_t (*m)[kPbChunks];   // [9][kPbChunks]: chunk c0 + j at column j
  const uint32_t* ssb;              // the block's string-start bitmap (from b0 - kPbPre)
  int64_t c0, b0, n_chunks;
  bool cl;
  __device__ __forceinline__ uint32_t ss_at(int64_t q) const {  // string-start bits of [q, q + 32), any q
    const int64_t r = q - (b0 - kPbPre);
    if (r >= 0 && r + 32 <= (int64_t)kPbSsWords * 32) {
      const int wi = (int)(r >> 5), sh = (int)(r & 31);
      const uint64_t two = (uint64_t)ssb[wi] | ((wi + 1 < kPbSsWords ? (uint64_t)ssb[wi + 1] : 0ULL) << 32);
      return (uint32_t)(two >> sh);
    }
    return pb_ss_global(g, q);
  }
  __device__ __forceinline__ uint32_t ss(int64_t c) const { return ss_at(32 * c); }
  __device__ __forceinline__ psb::Masks get(int64_t c) const {
    if (c < 0 || c >= n_chunks) return psb::Masks{};
    const int64_t j = c - c0;
    if (j >= 0 && j < kPbChunks) {
      const int k = (int)j;
      return psb::Masks{m[0][k], m[1][k], m[2][k], m[3][k], m[4][k], m[5][k], m[6][k], m[7][k], m[8][k]};
    }
    psb::RegBytes by;
    pb_load40(g, 32 * c, by.w);
    const uint64_t s = (uint64_t)ss_at(32 * c - 4) | ((uint64_t)(ss_at(32 * c + 28) & 0xFFu) << 32);
    return psb::classify(by, s, UcdClass{}, cl);
  }
};

__global__ void __launch_bounds__(kPbThreads, 4) k_presplit_bits(PbArgs g, int pattern, uint32_t* bits32) {
  __shared__ uint32_t s_m[9][kPbChunks];
  __shared__ uint32_t s_ss[kPbSsWords];
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kPbBlock, c0 = b0 / psb::kChunk;
  const int64_t n_chunks = (g.n_bytes + psb::kChunk - 1) / psb::kChunk;
  const bool cl = pattern == 0;
  // 0. string starts of [b0 - kPbPre, b0 + kPbBlock + 64) (the batch end is str_off[n_str])
  for (int i = tid; i < kPbSsWords; i += kPbThreads) s_ss[i] = 0;
  __syncthreads();
  {  // (from the first string of the tile holding b0 - kPbPre: no search)
    const int64_t first = b0 >= kPbPre ? g.tile_slo[(b0 - kPbPre) / kTile] : 0;
    for (int64_t i = first + tid; i <= g.n_str; i += kPbThreads) {
      const int64_t r = g.str_off[i] - (b0 - kPbPre);
      if (r >= (int64_t)kPbSsWords * 32) break;
      if (r >= 0) atomicOr(&s_ss[r >> 5], 1u << (r & 31));
    }
  }
  __syncthreads();
  PbSrc src{g, s_m, s_ss, c0, b0, n_chunks, cl};
  if (pattern == 2) {  // the chunks are the strings
    const int64_t c = c0 + tid;
    if (c < n_chunks) {
      uint32_t r = src.ss(c);
      if (32 * c + 32 > g.n_bytes) r &= (1u << (g.n_bytes - 32 * c)) - 1u;
      bits32[c] = r;
      if (c == n_chunks - 1 && (c & 1) == 0) bits32[c + 1] = 0;  // (the last word's upper half)
    }
    return;
  }
  // 1. class masks of the block's chunks c0 .. c0 + 255 (40 bytes each straight from global
  //    memory: staging the block through LDS measured slower)
  {
    const int64_t c = c0 + tid;
    psb::Masks m{};
    if (c < n_chunks) {
      psb::RegBytes by;
      pb_load40(g, 32 * c, by.w);
      const uint64_t s = (uint64_t)src.ss_at(32 * c - 4) | ((uint64_t)(src.ss_at(32 * c + 28) & 0xFFu) << 32);
      m = psb::classify(by, s, UcdClass{}, cl);
    }
    s_m[0][tid] = m.L; s_m[1][tid] = m.N; s_m[2][tid] = m.C; s_m[3][tid] = m.P; s_m[4][tid] = m.H;
    s_m[5][tid] = m.A; s_m[6][tid] = m.X; s_m[7][tid] = m.K1; s_m[8][tid] = m.K2;
  }
  __syncthreads();
  // 2. this thread's chunk
  const int64_t c = c0 + tid;
  if (c >= n_chunks) return;
  const psb::Masks m0 = src.get(c - 1), m1 = src.get(c), m2 = src.get(c + 1);
  const uint64_t ssw = (uint64_t)src.ss_at(32 * c - 16) | ((uint64_t)src.ss_at(32 * c + 16) << 32);
  uint32_t need = 0;
  uint32_t r = psb::rules(m0, m1, m2, ssw, cl, psb::Carry{}, &need);
  if (need) {
    const psb::Carry cy = psb::carries(src, c, need);
    r = psb::rules(m0, m1, m2, ssw, cl, cy, &need);
  }
  if (32 * c + 32 > g.n_bytes) r &= (1u << (g.n_bytes - 32 * c)) - 1u;
  bits32[c] = r;
  if (c == n_chunks - 1 && (c & 1) == 0) bits32[c + 1] = 0;  // (the last word's upper half)
}

// number of set bits (chunks) in the bitmap
__global__ void __launch_bounds__(256) k_popcount(const uint64_t* bits, int64_t n_words, unsigned long long* out) {
  uint64_t c = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_words; i += (int64_t)gridDim.x * 256)
    c += __popcll(bits[i]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)c);
}

}  // namespace sw
