// Device pre-split (apply_regex, shredword/base.py:38-58) into the chunk-boundary bitmap
// (bit i of word i/64 = byte i starts a chunk).  Included by encode.hip only.
//
// One thread per 64-byte segment of the batch.  A thread finds the first SYNC position in its
// segment -- a string start, an ASCII letter after ' ' (the chunk starts at the space) or an
// ASCII letter after '\n' -- which is a chunk start whatever precedes it (presplit_match.h),
// and runs the sequential matcher from there until it reaches a sync position at or past its
// segment end: exactly where the next thread that owns a sync position starts.  So the
// threads together reproduce the sequential parse of every string, and a segment without any
// sync position (inside a long letter, digit or punctuation run) is covered by the thread
// before it.  A workgroup stages its 16 KiB of input (+ halo) in LDS; reads past the window
// fall back to global memory.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "presplit_match.h"
#include "ucd_tables.h"

namespace sw {

__constant__ uint8_t c_ucd1[SW_UCD_STAGE1_SIZE] = SW_UCD_STAGE1_INIT;
__constant__ uint8_t c_ucd2[SW_UCD_STAGE2_SIZE] = SW_UCD_STAGE2_INIT;

constexpr int kPsSeg = 64;                       // bytes per thread
constexpr int kPsThreads = 256;
constexpr int kPsBlock = kPsSeg * kPsThreads;    // 16 KiB per workgroup
constexpr int kPsHalo = 2048;                    // staged past the block for chunks that run on
constexpr int kPsWin = kPsBlock + kPsHalo;
constexpr int kPsStrCap = 512;                   // string starts of a block kept in LDS

struct DevStr {  // one string: bytes [a, a + n) of the batch
  const uint8_t* lds;   // staged window [w_lo, w_hi) of the batch
  int64_t w_lo, w_hi;
  const uint8_t* g;     // the batch in global memory
  int64_t a, n;
  __device__ uint8_t byte(int64_t i) const {
    const int64_t p = a + i;
    return (p >= w_lo && p < w_hi) ? lds[p - w_lo] : g[p];
  }
  __device__ int cls(uint32_t cp) const {
    if (cp > 0x10FFFF) return kOther;
    const uint32_t blk = c_ucd1[cp >> 8];
    const uint32_t b = c_ucd2[blk * 64 + ((cp & 255) >> 2)];
    return (int)((b >> ((cp & 3) * 2)) & 3);
  }
};

__global__ void __launch_bounds__(kPsThreads) k_presplit(const uint8_t* bytes, int64_t n_bytes, const int64_t* str_off,
                                                         int64_t n_str, int pattern, uint64_t* bits) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[kPsWin];
  __shared__ int64_t s_str[kPsStrCap + 1];  // str_off[first ..] (INT64_MAX past the end)
  __shared__ int64_t s_first;               // index of the first of them
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kPsBlock;
  const int64_t w_hi = min(b0 + (int64_t)kPsWin, n_bytes);

  // stage the window (16-byte loads when aligned)
  if (((uintptr_t)bytes & 15) == 0) {
    for (int64_t i = (int64_t)tid * 16; b0 + i < w_hi; i += kPsThreads * 16) {
      if (b0 + i + 16 <= n_bytes) {
        *(uint4*)(s_win + i) = *(const uint4*)(bytes + b0 + i);
      } else {
        for (int k = 0; b0 + i + k < w_hi; ++k) s_win[i + k] = bytes[b0 + i + k];
      }
    }
  } else {
    for (int64_t i = tid; b0 + i < w_hi; i += kPsThreads) s_win[i] = bytes[b0 + i];
  }
  // the strings overlapping [b0, b0 + kPsBlock): the one containing b0 and those starting in it
  if (tid == 0) {
    int64_t lo = 0, hi = n_str;  // last string with start <= b0
    while (lo < hi) {
      const int64_t m = (lo + hi + 1) >> 1;
      if (str_off[m] <= b0) lo = m; else hi = m - 1;
    }
    s_first = lo;
  }
  __syncthreads();
  const int64_t first = s_first;
  for (int i = tid; i <= kPsStrCap; i += kPsThreads) {
    const int64_t si = first + i;
    s_str[i] = si <= n_str ? str_off[si] : INT64_MAX;
  }
  __syncthreads();

  const int64_t s0 = b0 + (int64_t)tid * kPsSeg;
  if (s0 >= n_bytes) return;
  const int64_t s1 = min(s0 + (int64_t)kPsSeg, n_bytes);
  // the string containing s0 (index relative to `first`): last k with s_str[k] <= s0; past the
  // LDS list, search global memory
  int64_t si;
  {
    int lo = 0, hi = kPsStrCap;  // (sorted; INT64_MAX past the end)
    while (lo < hi) {
      const int m = (lo + hi + 1) >> 1;
      if (s_str[m] <= s0) lo = m; else hi = m - 1;
    }
    si = first + lo;
    if (lo == kPsStrCap) {  // (the block holds more strings than the LDS list)
      int64_t glo = si, ghi = n_str;
      while (glo < ghi) {
        const int64_t m = (glo + ghi + 1) >> 1;
        if (str_off[m] <= s0) glo = m; else ghi = m - 1;
      }
      si = glo;
    }
  }
  if (si >= n_str) return;
  int64_t a = str_off[si], b = str_off[si + 1];  // (b > s0 >= a)
  DevStr st{s_win, b0, w_hi, bytes, a, b - a};

  auto is_sync = [&](int64_t p) -> bool {  // p inside the current string [a, b)
    if (p == a) return true;
    if (pattern == 2) return false;  // no pre-split: strings are single chunks
    const uint8_t c = st.byte(p - a);
    if (c == ' ') return p + 1 < b && ascii_letter(st.byte(p + 1 - a));
    return ascii_letter(c) && st.byte(p - 1 - a) == '\n';
  };
  auto next_string = [&]() -> bool {  // move to the next non-empty string; false past the last
    while (++si < n_str) {
      a = str_off[si];
      b = str_off[si + 1];
      if (b > a) {
        st.a = a;
        st.n = b - a;
        return true;
      }
    }
    return false;
  };

  // the first sync position in [s0, s1)
  int64_t p = -1;
  for (int64_t q = s0; q < s1; ++q) {
    if (q == b && !next_string()) return;
    if (is_sync(q)) {
      p = q;
      break;
    }
  }
  if (p < 0) return;

  // parse until a sync position at or past s1 (or the end of the batch)
  uint64_t word = 0;
  int64_t widx = p >> 6;
  while (true) {
    if (p == b) {
      if (!next_string()) break;
      if (p >= s1) break;  // (a string start is a sync position)
    } else if (p >= s1 && is_sync(p)) {
      break;
    }
    if ((p >> 6) != widx) {
      if (word) atomicOr((unsigned long long*)&bits[widx], (unsigned long long)word);
      word = 0;
      widx = p >> 6;
    }
    word |= 1ULL << (p & 63);
    int64_t e;
    if (pattern == 1) e = match_gpt2_t(st, p - a);
    else if (pattern == 0) e = match_cl100k_t(st, p - a);
    else e = st.n;  // no pre-split: the string is one chunk
    p = a + (e > p - a ? e : p - a + 1);
  }
  if (word) atomicOr((unsigned long long*)&bits[widx], (unsigned long long)word);
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
