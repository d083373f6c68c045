// Device pre-split (apply_regex, shredword/base.py:38-58) into the chunk-boundary bitmap
// (bit i of word i/64 = byte i starts a chunk).  Included by encode.hip only.
//
// The workgroup's work is presplit_block.h (shared with the CPU emulator of the tests): a
// workgroup owns 16 KiB of the batch (64 bytes per lane) and stages it with a 16-byte
// pre-halo and a 2 KiB post-halo in LDS.  It marks the string starts of that window in an
// LDS bitmap, then computes, converged, one INFO byte per window byte (presplit_fsm.h:
// info4 -- the code point's symbol, or "continuation", and the position's sync code), which
// replaces the staged bytes.  Each lane then steps byte by byte through the info bytes from
// the first sync position of its segment to the first sync position at or past its end
// (presplit_bytes); a lane whose parse runs past the staged window continues in the
// code-point-stepped form over global memory (presplit_run).  Chunk starts are OR-ed into
// the bitmap one 64-bit word at a time.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "presplit_bits.h"
#include "presplit_block.h"
#include "presplit_fsm.h"
#include "presplit_match.h"
#include "ucd_tables.h"

namespace sw {

__constant__ uint8_t c_ucd1[SW_UCD_STAGE1_SIZE] = SW_UCD_STAGE1_INIT;
__constant__ uint8_t c_ucd2[SW_UCD_STAGE2_SIZE] = SW_UCD_STAGE2_INIT;

__constant__ __attribute__((aligned(16))) fsm::Tables c_fsm[2] = {fsm::make_tables(true), fsm::make_tables(false)};

#define SW_LDS __attribute__((address_space(3)))  // (explicit, so reads are ds_read, not flat)

__device__ inline int ucd_class(uint32_t cp) {
#ifdef SW_PS_NOUCD  // (diagnostic timing builds only)
  return (int)(cp & 1);
#endif
  if (cp > 0x10FFFF) return kOther;
  const uint32_t blk = c_ucd1[cp >> 8];
  const uint32_t v = c_ucd2[blk * 64 + ((cp & 255) >> 2)];
  return (int)((v >> ((cp & 3) * 2)) & 3);
}

struct UcdClass {
  __device__ int operator()(uint32_t cp) const { return ucd_class(cp); }
};

#ifndef SW_PS_ABL
#define SW_PS_ABL 0  // diagnostic ablations (timing only, wrong bitmaps): 1 staging, 2 + info, 3 + lanes
#endif

struct PsBits {  // a lane's chunk starts past the info bytes, gathered one 64-bit word at a time
  uint64_t* bits;
  int64_t widx;
  uint64_t word;
  __device__ void flush() {
    if (word) atomicOr((unsigned long long*)&bits[widx], (unsigned long long)word);
  }
  __device__ void set(int64_t pos) {
    const int64_t w = pos >> 6;
    const uint64_t bit = 1ULL << (pos & 63);
    if (w == widx) {
      word |= bit;
    } else if (w > widx) {
      flush();
      widx = w;
      word = bit;
    } else {
      atomicOr((unsigned long long*)&bits[w], (unsigned long long)bit);
    }
  }
};

struct LdsOr {
  uint32_t* b;  // (a __shared__ array)
  __device__ void operator()(int w, uint32_t v) const {
    __hip_atomic_fetch_or(&b[w], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
};


__global__ void __launch_bounds__(kPsThreads) k_presplit(const uint8_t* bytes, int64_t n_bytes, const int64_t* str_off,
                                                         int64_t n_str, int pattern, uint64_t* bits) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[kPsRaw];  // bytes, then info bytes
  // string starts (and the batch end) in the window; after the info phase, the chunk starts
  // of [b0, b0 + block + halo)
  __shared__ __attribute__((aligned(8))) uint32_t s_ss[kPsSsWords];
  __shared__ __attribute__((aligned(16))) uint8_t s_step[sizeof(PsStepTab)];
  __shared__ uint32_t s_hi[kPsHiWords];         // groups with a byte >= 0x80 (info pass 2)
  __shared__ uint16_t s_hpre[kPsHiWords + 1];    // exclusive prefix counts of s_hi
  __shared__ int64_t s_first;
  static_assert(kPsSsWords >= 2 * kPsOutWords, "the chunk-start bitmap reuses s_ss");
  const int tid = threadIdx.x;
  const PsGeom G = ps_geom(blockIdx.x, n_bytes);
  const bool cl = pattern == 0, none = pattern == 2;
  const fsm::Tables* ftab = &c_fsm[pattern == 1 ? 1 : 0];

  // 1. stage [wb, wend) (zeros outside the batch and in the tail) and the tables
  {
    const bool aligned = ((uintptr_t)bytes & 15) == 0;
    for (int i = tid * 16; i < kPsRaw; i += kPsThreads * 16) {
      const int64_t g = G.wb + i;
      if (g >= 0 && g + 16 <= G.wend && aligned) {
        *(uint4*)(s_buf + i) = *(const uint4*)(bytes + g);
      } else {
        for (int k = 0; k < 16; ++k) s_buf[i + k] = (g + k >= 0 && g + k < G.wend) ? bytes[g + k] : 0;
      }
    }
    for (int i = tid; i < kPsSsWords; i += kPsThreads) s_ss[i] = 0;
    for (int i = tid; i < kPsHiWords; i += kPsThreads) s_hi[i] = 0;
    {  // asc and lane table of the pattern
      const uint32_t* a = (const uint32_t*)ftab->asc;
      const uint32_t* ln = (const uint32_t*)ftab->lane;
      static_assert(offsetof(PsStepTab, lane) == 128 && sizeof(ftab->lane) % 4 == 0, "PsStepTab layout");
      for (int i = tid; i < 32; i += kPsThreads) ((uint32_t*)s_step)[i] = a[i];
      for (int i = tid; i < (int)sizeof(ftab->lane) / 4; i += kPsThreads) ((uint32_t*)s_step)[32 + i] = ln[i];
    }
    if (tid == 0) {  // first string starting at or after wb
      int64_t lo = 0, hi = n_str;
      while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (str_off[m] < G.wb) lo = m + 1; else hi = m;
      }
      s_first = lo;
    }
  }
  __syncthreads();
  // string starts in [wb, wend] (str_off[n_str] = n_bytes marks the batch end)
  for (int64_t i = s_first + tid; i <= n_str; i += kPsThreads) {
    const int64_t o = str_off[i];
    if (o > G.wend) break;
    const int r = (int)(o - G.wb);
    atomicOr(&s_ss[r >> 5], 1u << (r & 31));
  }
  __syncthreads();

  if (none) {  // the chunks are the strings: the block's words straight from the string starts
    for (int i = tid; i < kPsBlock / 64; i += kPsThreads) {
      const int64_t gw = (G.b0 >> 6) + i;
      if (64 * gw >= n_bytes) break;
      uint64_t v = ps_none_word((const uint32_t*)s_ss, i);
      if (64 * gw + 64 > n_bytes) v &= (1ULL << (n_bytes - 64 * gw)) - 1;
      bits[gw] = v;
    }
    return;
  }
#if SW_PS_ABL == 1
  return;
#endif

  // 2. info bytes, in place of the staged bytes: pass 1 over every group
  SW_LDS uint32_t* w32 = (SW_LDS uint32_t*)s_buf;
  const PsInfoRegs regs = ps_info_load(w32, tid);
  __syncthreads();
  ps_info_convert(w32, (const SW_LDS uint32_t*)s_ss, (const SW_LDS uint8_t*)s_step, cl, G.info_hi, tid, regs,
                  [&](int j) { atomicOr(&s_hi[j >> 5], 1u << (j & 31)); });
  __syncthreads();
  if (tid < 64) {  // prefix counts of the marks (wave 0; 3 words per lane)
    static_assert(kPsHiWords <= 3 * 64, "marks");
    uint32_t c[3], t = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int j = 3 * tid + q;
      c[q] = j < kPsHiWords ? (uint32_t)__popc(s_hi[j]) : 0u;
      t += c[q];
    }
    uint32_t x = t;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off, 64);
      if (tid >= off) x += y;
    }
    uint32_t run = x - t;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int j = 3 * tid + q;
      if (j <= kPsHiWords) s_hpre[j] = (uint16_t)run;
      run += c[q];
    }
  }
  __syncthreads();
  {  // pass 2 over the marked groups, spread densely over the threads
    const PsUcdFull<UcdClass> cls{UcdClass{}};  // (the full table in constant memory: pass 2 is sparse)
    const int total = s_hpre[kPsHiWords];
    for (int k = tid; k < total; k += kPsThreads)
      ps_high_group(w32, (const SW_LDS uint32_t*)s_ss, cls, cl, G, bytes,
                    ps_high_select((const SW_LDS uint16_t*)s_hpre, (const SW_LDS uint32_t*)s_hi, k));
  }
  __syncthreads();
  for (int i = tid; i < 2 * kPsOutWords; i += kPsThreads) s_ss[i] = 0;  // (now the chunk-start bitmap)
  __syncthreads();
#if SW_PS_ABL == 2
  if (n_bytes == 12345) bits[tid] = w32[4 + tid * kPsGroups] + w32[5 + tid * kPsGroups];  // (keeps the info live)
  return;
#endif

  // 3. this lane's segment
  PsWinBits<LdsOr> lb{LdsOr{s_ss}};
  PsBits gout{bits, -1, 0};
  ps_lane(G, tid, (const SW_LDS uint32_t*)s_buf, (const SW_LDS PsStepTab*)s_step, ftab, bytes, n_bytes, str_off,
          n_str, cl, lb, gout, UcdClass{});
  __syncthreads();
#if SW_PS_ABL == 3
  return;
#endif

  // 4. the window's chunk starts into the global bitmap (OR: the previous workgroup's lanes
  //    may have run into this block, and this one's into the next)
  for (int i = tid; i < kPsOutWords; i += kPsThreads) {
    const int64_t gw = (G.b0 >> 6) + i;
    if (64 * gw >= n_bytes) break;
    const uint64_t v = (uint64_t)s_ss[2 * i] | ((uint64_t)s_ss[2 * i + 1] << 32);
    if (v) atomicOr((unsigned long long*)&bits[gw], (unsigned long long)v);
  }
}

// ---------------------------------------------------------------------------------------------
// k_presplit_bits: the bit-parallel pre-split (presplit_bits.h).  A workgroup owns kPbBlock
// bytes, one 32-byte chunk per thread:
//   0. the string starts of [b0 - 64, b0 + kPbBlock + 64) into an LDS bitmap;
//   1. every chunk's class masks (classify) for chunks -1 .. 256 of the block, into LDS;
//   2. every thread's window rules over chunks t - 1, t, t + 1, with the run carries walked over
//      the LDS masks (and, for runs past the block, over chunks classified from global memory);
//      the 32 chunk-start bits are stored as one dword of the bitmap (no atomics, no clearing).
// ---------------------------------------------------------------------------------------------
#ifndef SW_PB_THREADS
#define SW_PB_THREADS 256
#endif
constexpr int kPbThreads = SW_PB_THREADS;
constexpr int kPbBlock = kPbThreads * psb::kChunk;      // 8 KiB
constexpr int kPbPre = 64;                               // string starts staged before b0 ...
constexpr int kPbSsWords = (kPbPre + kPbBlock + 128) / 32;  // ... and after the block
// SW_PB_HALO 0 (default): LDS holds the block's own chunks 0 .. 255, one per thread, and the two
// neighbours of the block (chunks -1 and 256) are classified where they are needed (threads 0 and
// 255); 1: they are classified into LDS too, a second pass of step 1 for two lanes of wave 0
// that the workgroup barrier makes every wave wait for
#ifndef SW_PB_HALO
#define SW_PB_HALO 0
#endif
constexpr int kPbHalo = SW_PB_HALO;
constexpr int kPbChunks = kPbThreads + 2 * kPbHalo;      // chunks -halo .. 255 + halo
constexpr int kPbStage = kPbPre + kPbBlock + 64;           // bytes staged in LDS, from b0 - kPbPre

#ifndef SW_PB_STAGE
#define SW_PB_STAGE 0  // 1: classify reads the block's bytes from LDS (0: each chunk's 40 bytes from global memory)
#endif
struct LdsBytes {  // classify's view of a chunk's 40 bytes in the staged block (word-aligned)
  const uint32_t* s;  // (an LDS array) the word holding byte pos - 4
  __device__ uint32_t word(int i) const { return s[i]; }
  __device__ uint32_t at4(int k) const { return __builtin_amdgcn_alignbyte(s[(k >> 2) + 1], s[k >> 2], k & 3); }
};

struct PbArgs {
  const uint8_t* bytes;
  int64_t n_bytes;
  const int64_t* str_off;
  int64_t n_str;
  const int64_t* tile_slo;  // first string starting at or after each 2 KiB tile (k_tile_strings)
  int64_t blk0;             // first block of this launch (a segment of the batch, see sw_encode_device)
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
  const uint32_t (*m)[kPbChunks];   // [9][kPbChunks]: chunk c0 - kPbHalo + j at column j
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
    const int64_t j = c - (c0 - kPbHalo);
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

#ifndef SW_PB_WAVES
#define SW_PB_WAVES 4
#endif
__global__ void __launch_bounds__(kPbThreads, SW_PB_WAVES) k_presplit_bits(PbArgs g, int pattern, uint32_t* bits32) {
  __shared__ uint32_t s_m[9][kPbChunks];
  __shared__ uint32_t s_ss[kPbSsWords];
  __shared__ __attribute__((aligned(16))) uint32_t s_b[kPbStage / 4 + 4];  // bytes [b0 - kPbPre, ..)
  const int tid = threadIdx.x;
  const int64_t b0 = (g.blk0 + (int64_t)blockIdx.x) * kPbBlock, c0 = b0 / psb::kChunk;
  const int64_t n_chunks = (g.n_bytes + psb::kChunk - 1) / psb::kChunk;
  const bool cl = pattern == 0;
  if (SW_PB_STAGE && pattern != 2) {  // the block's bytes (zeros outside the batch), coalesced, before anything waits
    const bool aligned = ((uintptr_t)g.bytes & 15) == 0;
    for (int i = tid; i < kPbStage / 16; i += kPbThreads) {
      const int64_t q = b0 - kPbPre + 16 * i;
      uint4 v;
      if (aligned && q >= 0 && q + 16 <= g.n_bytes) {
        v = *(const uint4*)(g.bytes + q);
      } else {
        uint32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t x = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t p = q + 4 * k + e;
            x |= (p >= 0 && p < g.n_bytes) ? (uint32_t)g.bytes[p] << (8 * e) : 0u;
          }
          t[k] = x;
        }
        v = make_uint4(t[0], t[1], t[2], t[3]);
      }
      *(uint4*)&s_b[4 * i] = v;
    }
    if (tid < 4) s_b[kPbStage / 4 + tid] = 0;
  }
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
  // 1. class masks of chunks c0 - kPbHalo .. c0 + 255 + kPbHalo
  for (int j = tid; j < kPbChunks; j += kPbThreads) {
    const int64_t c = c0 - kPbHalo + j;
    psb::Masks m{};
    if (c >= 0 && c < n_chunks) {
#if SW_PB_STAGE
      const LdsBytes by{&s_b[(32 * j + kPbPre - 32 * kPbHalo - 4) / 4]};
#else
      psb::RegBytes by;
      pb_load40(g, 32 * c, by.w);
#endif
      const uint64_t s = (uint64_t)src.ss_at(32 * c - 4) | ((uint64_t)(src.ss_at(32 * c + 28) & 0xFFu) << 32);
#if defined(SW_PB_ABL) && (SW_PB_ABL == 2 || SW_PB_ABL == 3)  // (diagnostic timing builds only: wrong bitmaps)
      m.L = by.word(1) ^ by.word(3) ^ by.word(5) ^ by.word(7) ^ (uint32_t)s; m.N = by.word(2) ^ by.word(8);
      m.X = by.word(0) ^ by.word(9);
#else
      m = psb::classify(by, s, UcdClass{}, cl);
#endif
    }
    s_m[0][j] = m.L; s_m[1][j] = m.N; s_m[2][j] = m.C; s_m[3][j] = m.P; s_m[4][j] = m.H;
    s_m[5][j] = m.A; s_m[6][j] = m.X; s_m[7][j] = m.K1; s_m[8][j] = m.K2;
  }
  __syncthreads();
  // 2. this thread's chunk
  const int64_t c = c0 + tid;
  if (c >= n_chunks) return;
  const psb::Masks m0 = src.get(c - 1), m1 = src.get(c), m2 = src.get(c + 1);
  const uint64_t ssw = (uint64_t)src.ss_at(32 * c - 16) | ((uint64_t)src.ss_at(32 * c + 16) << 32);
  uint32_t need = 0;
#if defined(SW_PB_ABL) && (SW_PB_ABL == 1 || SW_PB_ABL == 3)  // (diagnostic timing builds only: wrong bitmaps)
  uint32_t r = m0.L ^ m1.N ^ m2.C ^ (uint32_t)ssw;
#else
  uint32_t r = psb::rules(m0, m1, m2, ssw, cl, psb::Carry{}, &need);
#endif
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
