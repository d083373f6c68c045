// Device pre-split (apply_regex, shredword/base.py:38-58) into the chunk-boundary bitmap
// (bit i of word i/64 = byte i starts a chunk).  Included by encode.hip only.
//
// A workgroup owns 16 KiB of the batch (64 bytes per lane) and stages it with a 16-byte
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

#include "presplit_fsm.h"
#include "presplit_match.h"
#include "ucd_tables.h"

namespace sw {

__constant__ uint8_t c_ucd1[SW_UCD_STAGE1_SIZE] = SW_UCD_STAGE1_INIT;
__constant__ uint8_t c_ucd2[SW_UCD_STAGE2_SIZE] = SW_UCD_STAGE2_INIT;

#ifndef SW_PS_ABL
#define SW_PS_ABL 0  // (diagnostic ablations: 1 staging only, 2 + info, 3 no bitmap writes, 4 first sync only)
#endif
constexpr int kPsSeg = 64;                       // bytes per lane
constexpr int kPsThreads = 256;
constexpr int kPsBlock = kPsSeg * kPsThreads;    // 16 KiB per workgroup
constexpr int kPsHalo = 2048;                    // staged past the block for chunks that run on
constexpr int kPsPre = 16;                       // staged before it (context of the first bytes)
constexpr int kPsWin = kPsPre + kPsBlock + kPsHalo;
constexpr int kPsGroups = (kPsBlock + kPsHalo) / 4 / kPsThreads;  // info words per thread (18)
constexpr int kPsRaw = kPsWin + 32;              // (zero tail: the context of the last bytes)
static_assert(kPsGroups * 4 * kPsThreads == kPsBlock + kPsHalo, "window");

__constant__ fsm::Tables c_fsm[2] = {fsm::make_tables(true), fsm::make_tables(false)};

#define SW_LDS __attribute__((address_space(3)))  // (explicit, so reads are ds_read, not flat)

__device__ inline int ucd_class(uint32_t cp) {
  if (cp > 0x10FFFF) return kOther;
  const uint32_t blk = c_ucd1[cp >> 8];
  const uint32_t v = c_ucd2[blk * 64 + ((cp & 255) >> 2)];
  return (int)((v >> ((cp & 3) * 2)) & 3);
}

struct PsBits {  // one lane's chunk starts, gathered one 64-bit word at a time
  uint64_t* bits;
  int64_t widx;
  uint64_t word;
  __device__ void flush() {
    if (word) atomicOr((unsigned long long*)&bits[widx], (unsigned long long)word);
  }
  __device__ void set(int64_t pos) {
#if SW_PS_ABL == 3
    word ^= pos; return;
#endif
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

struct PsFast {  // presplit_bytes context: positions relative to the window start wb
  const SW_LDS uint8_t* inf;
  const SW_LDS fsm::Tables* tab;
  PsBits* out;
  int64_t wb;
  __device__ uint32_t info_at(int r) const { return inf[r]; }
  __device__ uint32_t info(int r) const { return info_at(r); }
  __device__ void emit(int r) { out->set(wb + r); }
};

struct PsSlow {  // presplit_run context over global memory, positions relative to wb
  const uint8_t* g;  // bytes + wb
  const SW_LDS fsm::Tables* tab;
  const int64_t* str_off;
  int64_t n_str, wb, si;
  int a, b;
  PsBits* out;
  __device__ uint8_t byte(int p) const { return g[p]; }
  __device__ int cls(uint32_t cp) const { return ucd_class(cp); }
  __device__ bool next_string() {
    while (++si < n_str) {
      a = (int)(str_off[si] - wb);
      b = (int)(str_off[si + 1] - wb);
      if (b > a) return true;
    }
    return false;
  }
  __device__ void emit(int r) { out->set(wb + r); }
};

__global__ void __launch_bounds__(kPsThreads) k_presplit(const uint8_t* bytes, int64_t n_bytes, const int64_t* str_off,
                                                         int64_t n_str, int pattern, uint64_t* bits) {
  __shared__ __attribute__((aligned(16))) uint8_t s_buf[kPsRaw];  // bytes, then info bytes
  __shared__ uint32_t s_ss[kPsWin / 32 + 2];  // string starts (and the batch end) in the window
  __shared__ fsm::Tables s_tab;
  __shared__ int64_t s_first;
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kPsBlock;
  const int64_t wb = b0 - kPsPre;
  const int64_t wend = min(b0 + (int64_t)(kPsBlock + kPsHalo), n_bytes);
  const int wlen = (int)(wend - wb);
  const bool at_end = wend == n_bytes;
  const bool cl = pattern == 0, none = pattern == 2;

  // 1. stage [wb, wend) (zeros outside the batch and in the tail) and the pattern's tables
  {
    const bool aligned = ((uintptr_t)bytes & 15) == 0;
    for (int i = tid * 16; i < kPsRaw; i += kPsThreads * 16) {
      const int64_t g = wb + i;
      if (g >= 0 && g + 16 <= wend && aligned) {
        *(uint4*)(s_buf + i) = *(const uint4*)(bytes + g);
      } else {
        for (int k = 0; k < 16; ++k) s_buf[i + k] = (g + k >= 0 && g + k < wend) ? bytes[g + k] : 0;
      }
    }
    for (int i = tid; i < kPsWin / 32 + 2; i += kPsThreads) s_ss[i] = 0;
    const uint8_t* src = (const uint8_t*)&c_fsm[pattern == 1 ? 1 : 0];
    for (int i = tid; i < (int)sizeof(fsm::Tables); i += kPsThreads) ((uint8_t*)&s_tab)[i] = src[i];
    if (tid == 0) {  // first string starting at or after wb
      int64_t lo = 0, hi = n_str;
      while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (str_off[m] < wb) lo = m + 1; else hi = m;
      }
      s_first = lo;
    }
  }
  __syncthreads();
  // 2. string starts in [wb, wend] (str_off[n_str] = n_bytes marks the batch end)
  for (int64_t i = s_first + tid; i <= n_str; i += kPsThreads) {
    const int64_t o = str_off[i];
    if (o > wend) break;
    const int r = (int)(o - wb);
    atomicOr(&s_ss[r >> 5], 1u << (r & 31));
  }
  __syncthreads();

#if SW_PS_ABL == 1
  return;
#endif
  const int info_hi = at_end ? wlen : kPsWin - 8;  // info bytes exist for [kPsPre, info_hi)
  if (!none) {
    // 3. info bytes, in place of the staged bytes: each thread converts a run of kPsGroups
    // words in order, holding the raw words it still needs in registers (its neighbours'
    // edge words are read before anyone writes)
    SW_LDS uint32_t* w32 = (SW_LDS uint32_t*)s_buf;
    const SW_LDS uint8_t* asc = ((const SW_LDS fsm::Tables*)&s_tab)->asc;
    auto cls = [](uint32_t cp) { return ucd_class(cp); };
    const int wfirst = kPsPre / 4 + tid * kPsGroups;
    uint32_t u[3] = {w32[wfirst - 1], w32[wfirst], 0};
    const uint32_t edge = w32[wfirst + kPsGroups];
    __syncthreads();
    fsm::LeadCarry carry{0, 0, 0};
    for (int i = 0; i < kPsGroups; ++i) {
      const int r0 = (wfirst + i) * 4;
      if (r0 >= info_hi) break;
      u[2] = i + 1 < kPsGroups ? w32[wfirst + i + 1] : edge;
      const int q = r0 - 4;
      const uint64_t two = (uint64_t)s_ss[q >> 5] | ((uint64_t)s_ss[(q >> 5) + 1] << 32);
      const uint32_t ss = (uint32_t)(two >> (q & 31)) & 0xFFF;
      if (i == 0) carry = fsm::lead_carry(u, ss);
      w32[wfirst + i] = fsm::info4(u, ss, asc, cls, cl, carry);
      u[0] = u[1];
      u[1] = u[2];
    }
    __syncthreads();
  }

#if SW_PS_ABL == 2
  return;
#endif
  // 4. this lane's segment
  const int s0 = kPsPre + tid * kPsSeg;
  const int n_rel = (int)(n_bytes - wb);
  if (s0 >= n_rel) return;
  const int s1 = min(s0 + kPsSeg, n_rel);
  PsBits out{bits, (b0 >> 6) + tid, 0};
  if (none) {  // the chunks are the strings: this word's string starts
    const int q = s0;
    const uint64_t lo = (uint64_t)s_ss[q >> 5] | ((uint64_t)s_ss[(q >> 5) + 1] << 32);
    const uint64_t hi = s_ss[(q >> 5) + 2];
    uint64_t w = (lo >> (q & 31)) | (hi << (64 - (q & 31)));  // (q & 31 == 16)
    if (s1 - s0 < 64) w &= (1ULL << (s1 - s0)) - 1;
    out.word = w;
    out.flush();
    return;
  }
  const SW_LDS uint8_t* info = (const SW_LDS uint8_t*)s_buf;
  PsFast x{info, (const SW_LDS fsm::Tables*)&s_tab, &out, wb};
  int r = s0;
  while (r < s1 && !(x.info_at(r) >> 4)) ++r;
  if (r == s1) return;
#if SW_PS_ABL == 4
  return;
#endif
  int st = fsm::sync_init_state(x.info_at(r) >> 4);
  int last_cr = -1, last_ws = 0;
  bool last_sp = false;
  if (!fsm::presplit_bytes<int>(x, r, s1, info_hi, at_end, cl, st, last_cr, last_ws, last_sp)) {
    // past the staged window: the string containing r, then code points from the next one
    int64_t lo = 0, hi = n_str - 1;  // last string with start <= wb + r
    while (lo < hi) {
      const int64_t m = (lo + hi + 1) >> 1;
      if (str_off[m] <= wb + r) lo = m; else hi = m - 1;
    }
    PsSlow y{bytes + wb, (const SW_LDS fsm::Tables*)&s_tab, str_off, n_str, wb, lo,
             (int)(str_off[lo] - wb), (int)(str_off[lo + 1] - wb), &out};
    for (int k = 1; k <= 3; ++k) {  // r may be inside the code point the byte steps were in
      if (r - k < y.a) break;
      int len;
      fsm::cp_sym(y, r - k, cl, &len);
      if (len > k) {
        r += len - k;
        break;
      }
    }
    fsm::presplit_run<int>(y, r, s1, cl, false, st, last_cr, last_ws, last_sp);
  }
  out.flush();
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
