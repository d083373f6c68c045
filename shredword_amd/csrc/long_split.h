// Long chunks (> kShort bytes) by exact SPLIT + VERIFY over the whole GPU (well-formed tables).
// Included by encode.hip after kernels.h (whose junction_conflict comment has the theory; the
// proof is in DESIGN.md §4.2).  Reference loop: shredword/base.py:10-36.
//
// Every long chunk of the launch is cut into pieces of ~kPieceW bytes (cut where the byte pair
// ranks highest) and ALL pieces of ALL long chunks are then processed side by side, one lane
// per piece, by a handful of grid-wide passes -- no chunk is walked by one wave, so a 1 MiB
// letter run costs as many passes as a 40-byte one:
//   k_lp_prep       the long chunks (k_classify's long list): start, length, piece count
//   (scan)          piece offsets of the chunks
//   k_lp_fill       every piece's chunk (one wave per chunk)
//   k_lp_encode     every piece's cuts (where the byte pair ranks highest), the piece encoded
//                   on its own, in registers (the per-lane loop), its ids
//                   written over its bytes' positions (holes after them), and round 0's
//                   junction checks (left neighbour's last id from the next lane down); the
//                   pieces whose left junction conflicts are listed
//   rounds r = 0 .. kLpRounds - 1, over compact lists:
//     k_lp_heads      each listed piece's previous live piece, when that one has no conflict on
//                     its left, heads a window: the maximal run of pieces joined by conflicts
//     k_lp_windows    every window encoded again from its bytes, one lane each (<= 32 bytes, in
//                     registers; longer: listed for k_lp_bigwin) and merged into its head; the
//                     junctions on either side are listed for the next round
//     k_lp_bigwin     the listed windows, one wave each (<= 64 bytes: one position per lane;
//                     <= 4 KiB: the LDS wave loop; longer: the chunk falls back)
//     k_lp_junctions  the listed junctions (previous live piece, piece) in conflict?  (spine
//                     walk); the conflicting pieces are listed for round r + 1 (after the last
//                     round: a conflict left sends the chunk to the fallback)
//   k_lp_fallback   fallen-back chunks: the exact wave loop over the whole chunk (LDS)
//   k_lp_gather     every chunk's ids, its positions with the holes dropped, into res[2 start]
// The grids are persistent (grid-stride); the counts they loop over live in device memory, so
// nothing waits on the host and a launch without long chunks costs a few empty passes.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace sw {

constexpr uint32_t kLpNone = 0xFFFFFFFFu;  // no previous / next live piece in the chunk
constexpr uint32_t kLpAlive = 1u;          // pflag: a live piece (a window absorbs its followers)
constexpr uint32_t kLpConf = 2u;           // pflag: the junction with the previous live piece conflicts
constexpr uint32_t kLpHole = 0xFFFFFFFFu;  // pid: no id at this position (k_lp_gather drops it)
// window rounds before a chunk falls back.  On the C5 stress corpus round 0 settles 95% of the
// conflicts (105k); what is left are mostly (a, a) runs, whose windows grow by one piece a round
// (rounds 1..5: 5.8k, 5.6k, 5.1k, 4.6k, 4.2k windows) -- a wave loop over the whole chunk is
// cheaper: a chunk of <= kLpFallMax bytes with a conflict after round 0 falls back at once.
constexpr int kLpRounds = 3;
constexpr int kLpFallMax = 512;
constexpr int kLpGrid = 8192;              // persistent grids (256-thread blocks; up to 8 waves per SIMD)
constexpr int kLpPrepGrid = 512;           // k_lp_prep
// ctl words (int64): counts the passes loop over, written on the device; per round r (and the
// final check, r = kLpRounds): junctions to check, conflicts, window heads, big windows
constexpr int kLcLong = 0, kLcPieces = 1, kLcWave = 2, kLcFall = 3;
constexpr int kLcJun = 4, kLcConf = kLcJun + kLpRounds + 1, kLcHead = kLcConf + kLpRounds + 1;
constexpr int kLcBig = kLcHead + kLpRounds + 1;
constexpr int kLcWords = kLcBig + kLpRounds + 1;
constexpr int kLcDbg = kLcWords;               // SW_LP_DEBUG builds: per round, big-window bytes (sum, max)
constexpr int kLcAlloc = kLcWords + 2 * kLpRounds;

struct LongArgs {
  // the long chunks of the per-chunk wave loop (EncArgs::lstart / llen, count ctl[kLcWave];
  // SW_OPT_LONG_SPLIT 0 or an ill-formed table)
  uint32_t* wstart;
  uint32_t* wlen;
  // per long chunk of these passes (index i: k_lp_prep's order), lcap of each
  uint32_t* lstart;  // first byte
  uint32_t* llen;    // bytes
  uint32_t* lnp;     // pieces
  int64_t* lpo;      // exclusive scan of lnp: the chunk's first piece
  uint32_t* lfall;   // 1: the chunk takes the exact wave loop (k_lp_fallback)
  uint32_t* flist;   // ... those chunks (count ctl[kLcFall])
  // per piece (index j: pieces of chunk i are lpo[i] .. lpo[i] + lnp[i] - 1), pcap of each
  uint32_t* pbeg;    // first byte
  uint32_t* pcnt;    // ids (0 once absorbed by a window)
  uint32_t* pchunk;  // its chunk
  uint32_t* pflag;   // kLpAlive | kLpConf
  uint32_t* pprev;   // previous / next live piece of the chunk (kLpNone at the ends)
  uint32_t* pnext;
  uint32_t* pid;     // [n_bytes] a live piece's ids from its first byte's position on, then holes
                     // (kLpHole) up to the next live piece
  uint32_t* wlist;   // big windows of the current round: (head, last) piece pairs
  uint32_t* jlist[2];  // junctions (their right piece) to check in an even / odd round (r > 0)
  uint32_t* clist;   // pieces whose left junction conflicts (this round)
  uint32_t* hlist;   // window heads (this round)
  uint32_t* pseen;   // the last round r > 0 that checked the piece's left junction (a piece can be
                     // listed twice: after one window and as the head of another)
  int64_t* ctl;      // kLcWords counters
  int64_t lcap, pcap;
};

__device__ __forceinline__ int64_t lp_count(const int64_t* p, int64_t cap) {
  const int64_t v = *p;
  return v < cap ? (v < 0 ? 0 : v) : cap;
}

// the end of live piece j (the next live piece's first byte, or the chunk's end)
__device__ __forceinline__ uint32_t lp_end(const LongArgs& L, uint32_t j) {
  const uint32_t nx = L.pnext[j];
  if (nx != kLpNone) return L.pbeg[nx];
  const uint32_t i = L.pchunk[j];
  return L.lstart[i] + L.llen[i];
}

// chunk i falls back to the exact wave loop (listed once)
__device__ __forceinline__ void lp_fall(const LongArgs& L, uint32_t i) {
  if (atomicExch(&L.lfall[i], 1u) != 0u) return;
  const unsigned long long w = atomicAdd((unsigned long long*)&L.ctl[kLcFall], 1ULL);
  L.flist[w] = i;
}

// the queue's long bucket (chunks > kShort bytes) -> two lists, in any order (the counters are
// zeroed before): chunks over lp_min bytes for these passes (lstart / llen / lnp, count
// ctl[kLcLong]), the others for the per-chunk kernels (wstart / wlen, count ctl[kLcWave])
__global__ void __launch_bounds__(kThreads) k_lp_prep(EncArgs a, LongArgs L, int64_t lp_min) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  const int64_t n = (int64_t)*a.l_count, stride = (int64_t)gridDim.x * kThreads;
  for (int64_t t0 = (int64_t)blockIdx.x * kThreads + (threadIdx.x & ~63); t0 < n; t0 += stride) {  // (whole waves)
    const int64_t t = t0 + lane;
    int64_t start = 0, len = 0;
    if (t < n) {
      const uint64_t e = a.llist[t];
      start = (int64_t)(e >> 32);
      const uint32_t ql = (uint32_t)e;  // (the length, from k_classify)
      len = ql != kNoDid ? (int64_t)ql : next_set_bit(a.bits, a.n_words, start + 1, a.n_bytes) - start;
    }
    const uint64_t mw = __ballot(t < n && len <= lp_min), ml = __ballot(t < n && len > lp_min);
    unsigned long long bw = 0, bl = 0;
    if (lane == 0) {
      if (mw) bw = atomicAdd((unsigned long long*)&L.ctl[kLcWave], (unsigned long long)__popcll(mw));
      if (ml) bl = atomicAdd((unsigned long long*)&L.ctl[kLcLong], (unsigned long long)__popcll(ml));
    }
    bw = __shfl(bw, 0, 64);  // (broadcast before the lanes diverge)
    bl = __shfl(bl, 0, 64);
    if (t >= n) continue;
    if (len > lp_min) {
      const int64_t i = (int64_t)bl + __popcll(ml & lt_mask);
      if (i >= L.lcap) continue;  // (cannot happen: lcap >= n_bytes / (kShort + 1))
      L.lstart[i] = (uint32_t)start;
      L.llen[i] = (uint32_t)len;
      L.lnp[i] = (uint32_t)((len + kPieceW - 1) / kPieceW);
      L.lfall[i] = 0;
    } else {
      const int64_t i = (int64_t)bw + __popcll(mw & lt_mask);
      if (i >= L.lcap) continue;
      L.wstart[i] = (uint32_t)start;
      L.wlen[i] = (uint32_t)len;
    }
  }
}

// every piece's chunk (pchunk), one wave per chunk
__global__ void __launch_bounds__(kThreads) k_lp_fill(LongArgs L) {
  const int64_t n_long = lp_count(&L.ctl[kLcLong], L.lcap);
  const int lane = threadIdx.x & 63;
  const int64_t n_waves = (int64_t)gridDim.x * (kThreads / 64);
  for (int64_t i = ((int64_t)blockIdx.x * kWaves + wave_in_block()); i < n_long; i += n_waves) {
    const int P = (int)L.lnp[i];
    const int64_t j0 = L.lpo[i];
    if (j0 + P > L.pcap) continue;  // (cannot happen: pcap >= n_bytes / 8)
    for (int k = lane; k < P; k += 64) L.pchunk[j0 + k] = (uint32_t)i;
  }
}

// piece k of a chunk [start, start + len) of P pieces starts at the position in [W k - H, W k + H)
// whose byte pair ranks highest (piece 0 at the chunk's start, piece P at its end): the cuts at
// both ends of piece k, all eight lookups in flight together
template <bool kWide>
__device__ __forceinline__ void lp_cuts(const DevTable& t, const uint8_t* src, int len, int P, int k, int& beg,
                                        int& end) {
  uint32_t r[2][2 * kCutHalf];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c0 = (k + h) * kPieceW - kCutHalf;
#pragma unroll
    for (int u = 0; u < 2 * kCutHalf; ++u) {
      const int p = min(max(c0 + u, 1), len - 1);  // (clamped: every lane loads)
      r[h][u] = lookup<kWide>(t, src[p - 1], src[p]);
      r[h][u] = c0 + u < len ? r[h][u] : 0u;
    }
  }
  int cut[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c0 = (k + h) * kPieceW - kCutHalf;
    int best = c0;
    uint32_t br = r[h][0];
#pragma unroll
    for (int u = 1; u < 2 * kCutHalf; ++u)
      if (r[h][u] > br) { br = r[h][u]; best = c0 + u; }
    cut[h] = best;
  }
  beg = k == 0 ? 0 : cut[0];
  end = k + 1 >= P ? len : cut[1];
}

// a live piece's (or window's) result in pid over its bytes [beg, beg + n): the m ids, then holes
__device__ __forceinline__ void lp_holes(const LongArgs& L, uint32_t beg, int m, int n) {
  for (int k = m; k < n; ++k) L.pid[beg + k] = kLpHole;
}

// every piece on its own, one lane each, in registers (<= kPieceN bytes), and round 0's junction
// checks.  A lane finds its piece's two cuts, encodes it, writes its ids over its bytes'
// positions (holes after them) and its links.  A wave takes 64 consecutive pieces, 63 of them its
// own: lane 0 encodes the piece before them again, so every junction (piece - 1, piece) is
// checked by the lane of its right piece with its left neighbour's last id from the next lane
// down.  Conflicts are listed for round 0.
template <bool kWide, bool k16>
__global__ void __launch_bounds__(kThreads) k_lp_encode(EncArgs a, LongArgs L) {
  constexpr bool kLds = k16 && !kWide;
  __shared__ uint32_t s_ids[kLds ? kWaves * 64 * kPieceN : 1];  // (lane_merge_lds_wf: the waves' ids)
  const int64_t np = lp_count(&L.ctl[kLcPieces], L.pcap);
  const int lane = threadIdx.x & 63;
  uint32_t* s_id = s_ids + (kLds ? wave_in_block() * 64 * kPieceN : 0);
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  const int64_t mis = (int64_t)((uintptr_t)a.bytes & 3);
  const SW_AS_GLOBAL uint32_t* words = (const SW_AS_GLOBAL uint32_t*)((uintptr_t)a.bytes - mis);
  const int64_t last_word = (mis + a.n_bytes - 1) >> 2;
  const int64_t n_waves = (int64_t)gridDim.x * (kThreads / 64);
  for (int64_t g = ((int64_t)blockIdx.x * kWaves + wave_in_block()); 63 * g < np; g += n_waves) {
    const int64_t j = 63 * g - 1 + lane;
    const bool act = j >= 0 && j < np;
    const bool own = act && lane > 0;
    uint32_t c = kLpNone, start = 0;
    int len = 2, P = 1, k = 0;
    if (act) {
      c = L.pchunk[j];
      start = L.lstart[c];
      len = (int)L.llen[c];
      P = (int)L.lnp[c];
      k = (int)(j - L.lpo[c]);
    }
    int b0, b1;
    lp_cuts<kWide>(a.table, a.bytes + start, len, P, k, b0, b1);
    const uint32_t beg = start + (uint32_t)b0;
    const int n = act ? b1 - b0 : 0;
    uint32_t u[kPieceN / 4];
    chunk_words<kPieceN>(words, last_word, (int64_t)beg + mis, n, u);
    uint32_t first = 0, last = 0;
    int m = 0;
    if constexpr (kLds) {  // (16-bit ids: the loop with the ids in LDS)
      const uint32_t alive = lane_merge_lds_wf<kWide, kPieceN>(a.table, u, n, s_id, lane);
      for (uint32_t al = alive; al; al &= al - 1) {
        const uint32_t x = s_id[64 * (__ffs(al) - 1) + lane];
        if (own) L.pid[beg + m] = x;
        first = m == 0 ? x : first;
        last = x;
        ++m;
      }
    } else {
      uint32_t id[kPieceN];
#pragma unroll
      for (int q = 0; q < kPieceN / 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) id[4 * q + r] = (u[q] >> (8 * r)) & 0xFFu;
      const uint32_t alive = lane_merge_reg<kWide, k16, kPieceN, true>(a.table, id, n);
#pragma unroll
      for (int k = 0; k < kPieceN; ++k) {
        if ((alive >> k) & 1u) {
          if (own) L.pid[beg + m] = id[k];
          first = m == 0 ? id[k] : first;
          last = id[k];
          ++m;
        }
      }
    }
    const uint32_t x = (uint32_t)__shfl_up((int)last, 1, 64);
    const uint32_t cx = (uint32_t)__shfl_up((int)c, 1, 64);
    bool conf = false;
    if (own) {
      lp_holes(L, beg, m, n);
      L.pbeg[j] = beg;
      L.pprev[j] = k > 0 ? (uint32_t)(j - 1) : kLpNone;
      L.pnext[j] = k + 1 < P ? (uint32_t)(j + 1) : kLpNone;
      L.pseen[j] = 0;
      L.pcnt[j] = (uint32_t)m;
      conf = cx == c && junction_conflict<kWide>(a.table, a.inv, a.n_inv, x, first);
      L.pflag[j] = conf ? (kLpAlive | kLpConf) : kLpAlive;
    }
    const uint64_t cm = __ballot(conf);
    if (cm) {
      unsigned long long w = 0;
      if (lane == 0) w = atomicAdd((unsigned long long*)&L.ctl[kLcConf], (unsigned long long)__popcll(cm));
      w = __shfl(w, 0, 64);
      if (conf) L.clist[w + __popcll(cm & lt_mask)] = (uint32_t)j;
    }
  }
}

// junctions of round r >= 1, the ones listed by round r - 1's windows (round 0's are checked by
// k_lp_encode; r == kLpRounds: the final check -- a conflict left sends its chunk to the fallback)
template <bool kWide>
__global__ void __launch_bounds__(kThreads) k_lp_junctions(EncArgs a, LongArgs L, int r) {
  const int64_t n = lp_count(&L.ctl[kLcJun + r], L.pcap);
  const uint32_t* jl = L.jlist[r & 1];
  for (int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x; t < n; t += (int64_t)gridDim.x * kThreads) {
    const uint32_t j = jl[t];
    if (!(L.pflag[j] & kLpAlive)) continue;  // (absorbed since it was listed)
    if (L.lfall[L.pchunk[j]]) continue;      // (its chunk fell back)
    if (atomicMax(&L.pseen[j], (uint32_t)r) >= (uint32_t)r) continue;  // (checked by another lane)
    const uint32_t p = L.pprev[j];
    if (p == kLpNone) continue;
    const uint32_t x = L.pid[L.pbeg[p] + L.pcnt[p] - 1], y = L.pid[L.pbeg[j]];
    const bool c = junction_conflict<kWide>(a.table, a.inv, a.n_inv, x, y);
    L.pflag[j] = c ? (kLpAlive | kLpConf) : kLpAlive;
    if (!c) continue;
    const uint32_t i = L.pchunk[j];
    if (r == kLpRounds || L.llen[i] <= (uint32_t)kLpFallMax) {
      lp_fall(L, i);
    } else {
      const unsigned long long w = atomicAdd((unsigned long long*)&L.ctl[kLcConf + r], 1ULL);
      L.clist[w] = j;
    }
  }
}

// the window heads of round r: the previous live piece of a conflicting piece, when its own left
// junction does not conflict (every head is found once: from its next piece)
__global__ void __launch_bounds__(kThreads) k_lp_heads(LongArgs L, int r) {
  const int64_t n = lp_count(&L.ctl[kLcConf + r], L.pcap);
  for (int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x; t < n; t += (int64_t)gridDim.x * kThreads) {
    const uint32_t p = L.pprev[L.clist[t]];
    if (L.pflag[p] & kLpConf) continue;
    const unsigned long long w = atomicAdd((unsigned long long*)&L.ctl[kLcHead + r], 1ULL);
    L.hlist[w] = p;
  }
}

// (every walk is bounded by the piece count: a broken link ends it rather than the kernel hanging)
__device__ __forceinline__ uint32_t lp_window_last(const LongArgs& L, uint32_t j, int64_t np) {
  uint32_t last = L.pnext[j];
  for (int64_t guard = 0; guard < np; ++guard) {
    const uint32_t nx = L.pnext[last];
    if (nx == kLpNone || !(L.pflag[nx] & kLpConf)) break;
    last = nx;
  }
  return last;
}

// the window (head j .. last) merged into its head, whose m ids are at pid[pbeg[j]]; the head's
// and the next piece's left junctions are listed for round r + 1
__device__ __forceinline__ void lp_absorb(const LongArgs& L, uint32_t j, uint32_t last, uint32_t m, int r) {
  for (uint32_t q = L.pnext[j], guard = 0; q != kLpNone && guard < (uint32_t)L.pcap; q = L.pnext[q], ++guard) {
    L.pflag[q] = 0;
    L.pcnt[q] = 0;
    if (q == last) break;
  }
  const uint32_t nx = L.pnext[last];
  L.pnext[j] = nx;
  if (nx != kLpNone) L.pprev[nx] = j;
  L.pcnt[j] = m;
  L.pflag[j] = kLpAlive;
  uint32_t* jl = L.jlist[(r + 1) & 1];
  const unsigned long long w = atomicAdd((unsigned long long*)&L.ctl[kLcJun + r + 1], nx != kLpNone ? 2ULL : 1ULL);
  jl[w] = j;
  if (nx != kLpNone) jl[w + 1] = nx;
}

// the windows of round r, one lane each: <= kShort bytes encoded in registers, longer listed
template <bool kWide, bool k16>
__global__ void __launch_bounds__(kThreads) k_lp_windows(EncArgs a, LongArgs L, int r) {
  constexpr bool kLds = k16 && !kWide;
  __shared__ uint32_t s_ids[kLds ? kWaves * 64 * kShort : 1];  // (lane_merge_lds_wf: the waves' ids)
  const int lane = threadIdx.x & 63;
  uint32_t* s_id = s_ids + (kLds ? wave_in_block() * 64 * kShort : 0);
  const int64_t nh = lp_count(&L.ctl[kLcHead + r], L.pcap), np = lp_count(&L.ctl[kLcPieces], L.pcap);
  const int64_t mis = (int64_t)((uintptr_t)a.bytes & 3);
  const SW_AS_GLOBAL uint32_t* words = (const SW_AS_GLOBAL uint32_t*)((uintptr_t)a.bytes - mis);
  const int64_t last_word = (mis + a.n_bytes - 1) >> 2;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t t0 = (int64_t)blockIdx.x * kThreads; t0 < nh; t0 += stride) {  // (whole waves: the loop is per lane)
    const int64_t t = t0 + threadIdx.x;
    bool act = false;
    uint32_t j = 0, last = 0, beg = 0;
    int n = 0;
    if (t < nh) {
      j = L.hlist[t];
      last = lp_window_last(L, j, np);
      beg = L.pbeg[j];
      n = (int)(lp_end(L, last) - beg);
      act = n <= kShort;
      if (!act) {  // (a wave each, k_lp_bigwin)
        const unsigned long long w = atomicAdd((unsigned long long*)&L.ctl[kLcBig + r], 1ULL);
        L.wlist[2 * w] = j;
        L.wlist[2 * w + 1] = last;
      }
    }
    if (!__ballot(act)) continue;
    uint32_t u[kShort / 4];
    chunk_words<kShort>(words, last_word, (int64_t)beg + mis, act ? n : 0, u);
    uint32_t m = 0;
    if constexpr (kLds) {  // (16-bit ids: the loop with the ids in LDS)
      const uint32_t alive = lane_merge_lds_wf<kWide, kShort>(a.table, u, act ? n : 0, s_id, lane);
      if (!act) continue;
      for (uint32_t al = alive; al; al &= al - 1) L.pid[beg + m++] = s_id[64 * (__ffs(al) - 1) + lane];
    } else {
      uint32_t id[kShort];
#pragma unroll
      for (int q = 0; q < kShort / 4; ++q)
#pragma unroll
        for (int b = 0; b < 4; ++b) id[4 * q + b] = (u[q] >> (8 * b)) & 0xFFu;
      const uint32_t alive = lane_merge_reg<kWide, k16, kShort, true>(a.table, id, act ? n : 0);
      if (!act) continue;
#pragma unroll
      for (int k = 0; k < kShort; ++k)
        if ((alive >> k) & 1u) L.pid[beg + m++] = id[k];
    }
    lp_holes(L, beg, (int)m, n);
    lp_absorb(L, j, last, m, r);
  }
}

// the windows over kShort bytes of round r, one 64-thread workgroup (a wave) each
template <bool kWide, bool k16>
__global__ void __launch_bounds__(64) k_lp_bigwin(EncArgs a, LongArgs L, int r) {
  typedef typename std::conditional<k16, uint16_t, uint32_t>::type T;
  __shared__ T s_id[kLongLds];
  __shared__ T s_rk[kLongLds];
  __shared__ uint64_t s_kill[64], s_dirty[64];
  const int64_t nw = min(L.ctl[kLcBig + r], L.pcap / 2);
  const int lane = threadIdx.x;
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  for (int64_t w = blockIdx.x; w < nw; w += gridDim.x) {
    const uint32_t j = L.wlist[2 * w], last = L.wlist[2 * w + 1];
    const uint32_t beg = L.pbeg[j];
    const int n = (int)(lp_end(L, last) - beg);
    const uint8_t* src = a.bytes + beg;
    uint32_t m = 0;
#ifdef SW_LP_DEBUG
    if (lane == 0) {
      atomicAdd((unsigned long long*)&L.ctl[kLcDbg + r], (unsigned long long)n);
      atomicMax((unsigned long long*)&L.ctl[kLcDbg + kLpRounds + r], (unsigned long long)n);
    }
#endif
    if (n <= 64) {  // one position per lane
      uint32_t id = lane < n ? (uint32_t)src[lane] : 0u;
      uint32_t rk = lane + 1 < n ? lookup<kWide>(a.table, src[lane], src[lane + 1]) : kInf;
      const uint64_t al = wave_merge64<kWide>(a.table, id, rk, n, lane);
      m = (uint32_t)__popcll(al);
      if ((al >> lane) & 1ULL) L.pid[beg + __popcll(al & lt_mask)] = id;
      if (lane >= (int)m && lane < n) L.pid[beg + lane] = kLpHole;
    } else if (n <= kLongLds) {  // the LDS wave loop
      m = (uint32_t)seg_merge<kWide, T>(a.table, src, s_id, s_rk, s_kill, s_dirty, n, lane, L.pid + beg);
      for (int q = (int)m + lane; q < n; q += 64) L.pid[beg + q] = kLpHole;
      wave_sync_mem();
    } else {  // (a window over 4 KiB: the whole chunk takes the exact wave loop)
      if (lane == 0) lp_fall(L, L.pchunk[j]);
      continue;
    }
    if (lane == 0) lp_absorb(L, j, last, m, r);
  }
}

// the chunks that fell back, one 64-thread workgroup (a wave) each: the exact wave loop over the
// whole chunk, its result straight into res[2 start ..] -- in LDS up to kLongLds bytes, else in
// the global work area (ids then ranks, 2 len words)
template <bool kWide, bool k16>
__global__ void __launch_bounds__(64) k_lp_fallback(EncArgs a, LongArgs L) {
  typedef typename std::conditional<k16, uint16_t, uint32_t>::type T;
  __shared__ T s_id[kLongLds];
  __shared__ T s_rk[kLongLds];
  __shared__ uint64_t s_kill[64], s_dirty[64];
  const int64_t nf = lp_count(&L.ctl[kLcFall], L.lcap);
  const int lane = threadIdx.x;
  for (int64_t w = blockIdx.x; w < nf; w += gridDim.x) {
    const uint32_t i = L.flist[w];
    const int64_t start = L.lstart[i], len = L.llen[i];
    const uint8_t* src = a.bytes + start;
    uint32_t* gid = a.res + 2 * start + 1;
    int64_t m;
    if (len <= kLongLds) {
      m = seg_merge<kWide, T>(a.table, src, s_id, s_rk, s_kill, s_dirty, (int)len, lane, gid);
    } else {
      for (int64_t q = lane; q < len; q += 64) gid[q] = src[q];
      wave_sync_mem();
      m = coop_merge<kWide>(a.table, gid, gid + len, len, lane);
    }
    if (lane == 0) gid[-1] = (uint32_t)m;
    wave_sync_mem();
  }
}

// every chunk's result (res[2 start] = count, then the ids): its positions in pid with the holes
// dropped, one wave per chunk, 64 kGatherU positions at a time (all loads in flight together)
constexpr int kGatherU = 8;
__global__ void __launch_bounds__(kThreads) k_lp_gather(EncArgs a, LongArgs L) {
  const int64_t n_long = lp_count(&L.ctl[kLcLong], L.lcap);
  const int lane = threadIdx.x & 63;
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  const int64_t n_waves = (int64_t)gridDim.x * (kThreads / 64);
  for (int64_t i = ((int64_t)blockIdx.x * kWaves + wave_in_block()); i < n_long; i += n_waves) {
    if (L.lfall[i]) continue;
    const int64_t start = L.lstart[i], len = L.llen[i];
    uint32_t* dst = a.res + 2 * start + 1;
    const uint32_t* src = L.pid + start;
    int64_t m = 0;
    for (int64_t q0 = 0; q0 < len; q0 += 64 * kGatherU) {
      uint32_t v[kGatherU];
#pragma unroll
      for (int u = 0; u < kGatherU; ++u) {
        const int64_t q = q0 + 64 * u + lane;
        v[u] = q < len ? src[q] : kLpHole;
      }
#pragma unroll
      for (int u = 0; u < kGatherU; ++u) {
        const uint64_t keep = __ballot(v[u] != kLpHole);
        if (v[u] != kLpHole) dst[m + __popcll(keep & lt_mask)] = v[u];
        m += __popcll(keep);
      }
    }
    if (lane == 0) dst[-1] = (uint32_t)m;
  }
}

}  // namespace sw
