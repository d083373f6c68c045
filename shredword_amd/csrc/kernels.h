// Device side of the batched encode (included by encode.hip only).
//
// Semantics per chunk (exact for ANY merge table; shredword/base.py:10-36): ids = bytes; while
// >= 2 ids: take the adjacent pair with the smallest merges-value (first occurrence on ties);
// stop if no pair is in merges; else replace every non-overlapping occurrence of that pair,
// left to right, by the value.
//
// k_encode_tiles: one 256-thread workgroup per 2 KiB tile of input bytes.
//   LDS holds the tile (+ a 32-byte halo) as an id array in POSITION SPACE: the chunk that
//   starts at byte p keeps its ids in id[p .. p+n) and its pair ranks in rk[p .. p+n-1), so
//   every chunk works in place, no per-lane scratch, and the LDS footprint is ~4 B (16-bit ids)
//   per input byte -> 6 workgroups (24 waves) per CU.
//   Chunks <= kShort bytes: one lane each, lanes ordered by chunk length (counting sort) so a
//   wave's lanes run loops of similar trip count.  Per merge step a single in-place pass both
//   applies the merge and finds the next minimum; only the <= 2 pairs touching each new token
//   are looked up again.
//   Longer chunks: one wave each, exact wave-cooperative loop (64-bit argmin over the wave,
//   ballot/popcount compaction, run-parity for (a,a) pairs) in LDS when the chunk lies inside
//   the tile window, else in a position-indexed global work area.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "table.h"

namespace sw {

constexpr int kTile = 2048;                  // input bytes per workgroup
constexpr int kThreads = 256;                // 4 waves
constexpr int kShort = 32;                   // per-lane path for chunks up to this many bytes
constexpr int kWin = kTile + kShort;         // LDS window: tile + halo for chunks crossing the end
constexpr int kTileWords = kTile / 64 + 1;   // bitmap words staged (tile + 64-bit halo)
constexpr int kMaxLong = kTile / (kShort + 1) + 1;

template <typename Id>
struct IdT {
  static constexpr Id inf = (Id)~(Id)0;
  using Key = typename std::conditional<sizeof(Id) == 2, uint32_t, uint64_t>::type;
  static constexpr Key key_inf = (Key)~(Key)0;
  __device__ static Key key(Id rank, int idx) { return ((Key)rank << 8) | (Key)idx; }
  __device__ static Id rank_of(Key k) { return (Id)(k >> 8); }
  __device__ static int idx_of(Key k) { return (int)(k & 0xFF); }
};

// merges.get((a, b)): the value, or kInf.  Two independent 16-byte loads (both cuckoo
// candidate buckets), no loop: one memory round trip for every lane.
template <bool kWide>
__device__ __forceinline__ uint32_t lookup(const DevTable& t, uint32_t a, uint32_t b) {
  const uint32_t f = mix_key(a, b);
  const uint4* B = (const uint4*)t.buckets;
  const uint4 q1 = B[bucket1(f, t)];
  const uint4 q2 = B[bucket2(f, t)];
  if (!kWide) {
    const uint32_t key = (a << 16) | b;
    uint32_t v = kInf;
    v = (q1.x == key) ? q1.y : v;
    v = (q1.z == key) ? q1.w : v;
    v = (q2.x == key) ? q2.y : v;
    v = (q2.z == key) ? q2.w : v;
    return ((a | b) > 0xFFFFu) ? kInf : v;
  } else {
    uint32_t v = kInf;
    v = (q1.x == a && q1.y == b) ? q1.z : v;
    v = (q2.x == a && q2.y == b) ? q2.z : v;
    return v;
  }
}

template <typename Id, bool kWide>
__device__ __forceinline__ Id lookup_id(const DevTable& t, Id a, Id b) {
  const uint32_t v = lookup<kWide>(t, a, b);
  return v == kInf ? IdT<Id>::inf : (Id)v;  // narrow-16 tables hold values <= 0xFFFD
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

// First set bit at position >= pos, or n_bits if none.
__device__ inline int64_t next_set_bit(const uint64_t* bits, int64_t n_words, int64_t pos, int64_t n_bits) {
  int64_t w = pos >> 6;
  if (w >= n_words) return n_bits;
  uint64_t word = bits[w] & (~0ULL << (pos & 63));
  while (!word) {
    if (++w >= n_words) return n_bits;
    word = bits[w];
  }
  const int64_t q = (w << 6) + __ffsll((long long)word) - 1;
  return q < n_bits ? q : n_bits;
}

// ---------------------------------------------------------------------------------------
// per-lane merge loop, in place on id[0..n), rk[0..n-1)   (n <= kShort)
// ---------------------------------------------------------------------------------------
template <typename Id, bool kWide>
__device__ int lane_merge(const DevTable& t, Id* id, Id* rk, int n) {
  using K = IdT<Id>;
  typename K::Key best = K::key_inf;
  // initial ranks: independent lookups, four in flight per lane
  for (int j0 = 0; j0 + 1 < n; j0 += 4) {
    Id r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = min(j0 + u, n - 2);  // clamped duplicates keep the loads unconditional
      r[u] = lookup_id<Id, kWide>(t, id[j], id[j + 1]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u;
      if (j + 1 < n) {
        rk[j] = r[u];
        const typename K::Key k = K::key(r[u], j);
        best = k < best ? k : best;
      }
    }
  }
  while (n >= 2) {
    const Id nv = K::rank_of(best);
    if (nv == K::inf) break;
    const int bi = K::idx_of(best);
    const Id p0 = id[bi], p1 = id[bi + 1];
    // one pass: apply the merge (left to right, non-overlapping) and collect the minimum of the
    // ranks that survive; positions whose pair changed are marked in `need`
    best = K::key_inf;
    uint32_t need = 0;
    int w = bi;  // positions before the first occurrence are unchanged
    bool prev_carried = false;
    Id prev_rank = 0;
    for (int j = 0; j < bi; ++j) {  // their ranks still count (except bi-1, re-looked up)
      if (j + 1 < bi) {
        const typename K::Key k = K::key(rk[j], j);
        best = k < best ? k : best;
      }
    }
    if (bi > 0) { prev_carried = true; prev_rank = rk[bi - 1]; }
    Id x = id[bi];
    for (int j = bi; j < n;) {
      const Id y = (j + 1 < n) ? id[j + 1] : K::inf;
      if (j + 1 < n && x == p0 && y == p1) {
        id[w] = nv;
        need |= 1u << w;
        if (w > 0) need |= 1u << (w - 1);
        prev_carried = false;
        ++w;
        j += 2;
        x = (j < n) ? id[j] : K::inf;
      } else {
        if (prev_carried && !((need >> (w - 1)) & 1u)) {
          const typename K::Key k = K::key(prev_rank, w - 1);
          best = k < best ? k : best;
        }
        id[w] = x;
        prev_rank = rk[j];
        rk[w] = prev_rank;
        prev_carried = true;
        ++w;
        ++j;
        x = y;
      }
    }
    n = w;
    need &= (n >= 2) ? ((1u << (n - 1)) - 1u) : 0u;
    while (need) {  // two lookups in flight per round
      const int j1 = __ffs(need) - 1;
      need &= need - 1;
      const int j2 = need ? __ffs(need) - 1 : j1;
      need &= need - 1;
      const Id r1 = lookup_id<Id, kWide>(t, id[j1], id[j1 + 1]);
      const Id r2 = lookup_id<Id, kWide>(t, id[j2], id[j2 + 1]);
      rk[j1] = r1;
      rk[j2] = r2;
      const typename K::Key k1 = K::key(r1, j1), k2 = K::key(r2, j2);
      best = k1 < best ? k1 : best;
      best = k2 < best ? k2 : best;
    }
  }
  return n;
}

// ---------------------------------------------------------------------------------------
// wave-cooperative exact merge loop on id[0..n), rk[0..n-1) (any n; LDS or global memory)
// ---------------------------------------------------------------------------------------
template <typename Id>
__device__ __forceinline__ void wave_sync_mem() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

template <typename Id, bool kWide>
__device__ int64_t coop_merge(const DevTable& t, Id* id, Id* rk, int64_t n, int lane) {
  constexpr Id INF = IdT<Id>::inf;
  constexpr Id RECOMP = (Id)(INF - 1);
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  for (int64_t i = lane; i + 1 < n; i += 64) rk[i] = RECOMP;
  wave_sync_mem<Id>();
  while (n >= 2) {
    // pass 1: resolve pending ranks; argmin over (rank, index)
    uint64_t best = ~0ULL;
    for (int64_t i = lane; i + 1 < n; i += 64) {
      Id r = rk[i];
      if (r == RECOMP) {
        r = lookup_id<Id, kWide>(t, id[i], id[i + 1]);
        rk[i] = r;
      }
      const uint64_t key = ((uint64_t)r << 32) | (uint32_t)i;
      best = key < best ? key : best;
    }
    best = wave_min_u64(best);
    const Id nv = (Id)(best >> 32);
    if (nv == INF) break;
    const int64_t b = (int64_t)(uint32_t)best;
    wave_sync_mem<Id>();
    const Id p0 = id[b], p1 = id[b + 1];
    // pass 2: replace every non-overlapping occurrence of (p0, p1), left to right, in place
    int64_t w = 0;
    bool prev_taken = false;
    for (int64_t seg = 0; seg < n; seg += 64) {
      const int64_t i = seg + lane;
      const bool valid = i < n;
      const Id e = valid ? id[i] : INF;
      const Id er = (valid && i + 1 < n) ? rk[i] : INF;
      Id nid = (Id)__shfl_down((uint32_t)e, 1, 64);
      if (lane == 63) nid = (i + 1 < n) ? id[i + 1] : INF;
      const bool match = valid && (i + 1 < n) && e == p0 && nid == p1;
      uint64_t M = __ballot(match);
      if (prev_taken) M &= ~1ULL;  // position seg is the right half of the previous take
      uint64_t T = M;
      if (p0 == p1) {  // runs of (a,a): take even offsets from each run start
        const uint64_t E = 0x5555555555555555ULL;
        const uint64_t S = M & ~(M << 1);
        const uint64_t runs_even = M & ~(M + (S & E));
        T = (runs_even & E) | (M & ~runs_even & ~E);
      }
      const uint64_t consumed = (T << 1) | (prev_taken ? 1ULL : 0ULL);
      const uint64_t keep = __ballot(valid) & ~consumed;
      const bool take = (T >> lane) & 1ULL;
      const bool next_take = lane < 63 ? ((T >> (lane + 1)) & 1ULL) : true;
      const int64_t pos = w + __popcll(keep & lt_mask);
      wave_sync_mem<Id>();  // all loads of this segment precede the in-place stores
      if ((keep >> lane) & 1ULL) {
        id[pos] = take ? nv : e;
        rk[pos] = (take || next_take) ? RECOMP : er;
      }
      w += __popcll(keep);
      prev_taken = (T >> 63) & 1ULL;
    }
    n = w;
    wave_sync_mem<Id>();
  }
  return n;
}

// ---------------------------------------------------------------------------------------
struct TileArgs {
  const uint8_t* bytes;
  int64_t n_bytes;
  const uint64_t* bits;
  int64_t n_words;
  const int64_t* str_off;
  int64_t n_str;
  DevTable table;
  int32_t* scratch;      // [n_bytes] tile outputs, position space (tile t at its first chunk)
  void* lw_id;           // [n_bytes] Id: long-chunk work area, position space
  void* lw_rk;           // [n_bytes] Id
  uint32_t* tile_cnt;    // [n_tiles]
  int64_t* tile_first;   // [n_tiles] first chunk start in tile (or -1)
  int64_t* out_off;      // [n_str+1] tile-local offsets, rebased by k_string_offsets
  const int64_t* tile_slo;  // [n_tiles] first string starting at or after the tile start
  unsigned long long* stamps;  // diagnostic builds (SW_STAMPS): cycles per phase, summed
};

#ifdef SW_STAMPS
#define SW_STAMP(k)                                                                 \
  do {                                                                              \
    if (threadIdx.x == 0) {                                                         \
      const unsigned long long now_ = __builtin_readcyclecounter();                 \
      atomicAdd(&a.stamps[k], now_ - stamp_prev_);                                  \
      stamp_prev_ = now_;                                                           \
    }                                                                               \
  } while (0)
#else
#define SW_STAMP(k) do {} while (0)
#endif

// exclusive block scan over kThreads threads (sh: kThreads/64 words); *total = block sum
__device__ inline uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kThreads / 64; ++k) {
    const uint32_t s = sh[k];
    if (k < wid) base += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

template <typename Id, bool kWide>
__global__ void __launch_bounds__(kThreads) k_encode_tiles(TileArgs a) {
  __shared__ __attribute__((aligned(16))) Id s_id[kWin];
  __shared__ __attribute__((aligned(16))) Id s_rk[kWin];
  __shared__ uint64_t s_bits[kTileWords];
  __shared__ uint16_t s_cstart[kTile + 1];
  __shared__ uint32_t s_cnt[kTile + 1];       // chunk length, then token count, then offset
  __shared__ uint16_t s_order[kTile];
  __shared__ uint32_t s_bin[kShort + 2];
  __shared__ uint16_t s_long[kMaxLong];
  __shared__ uint32_t s_wsum[kThreads / 64];
  __shared__ uint32_t s_nlong, s_nglobal;
  __shared__ int64_t s_last_end, s_slo;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t tile = blockIdx.x;
  const int64_t t0 = tile * kTile;
#ifdef SW_STAMPS
  unsigned long long stamp_prev_ = __builtin_readcyclecounter();
#endif
  if (tid == 0) s_slo = a.tile_slo[tile];
  const int64_t t1 = min(t0 + (int64_t)kTile, a.n_bytes);
  const int64_t w0 = t0 >> 6;

  // 1. stage the window's bytes as ids (4 bytes per thread-load) and the bitmap words
  for (int i = tid * 4; i < kWin; i += kThreads * 4) {
    const int64_t g = t0 + i;
    uint32_t v = 0;
    if (g + 4 <= a.n_bytes && ((uintptr_t)a.bytes & 3) == 0) v = *(const uint32_t*)(a.bytes + g);
    else
      for (int k = 0; k < 4; ++k) v |= (g + k < a.n_bytes ? (uint32_t)a.bytes[g + k] : 0u) << (8 * k);
    if (sizeof(Id) == 2) {  // one 8-byte LDS store per thread
      const uint32_t lo = (v & 0xFFu) | ((v & 0xFF00u) << 8), hi = ((v >> 16) & 0xFFu) | ((v >> 8) & 0xFF0000u);
      *(uint2*)(s_id + i) = make_uint2(lo, hi);
    } else {
      *(uint4*)(s_id + i) = make_uint4(v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF, v >> 24);
    }
  }
  if (tid < kTileWords) s_bits[tid] = (w0 + tid < a.n_words) ? a.bits[w0 + tid] : 0ULL;
  if (tid < kShort + 2) s_bin[tid] = 0;
  if (tid == 0) { s_nlong = 0; s_nglobal = 0; }
  __syncthreads();

  // 2. chunk starts in [t0, t1): one thread per bitmap word
  constexpr int nw_tile = kTile / 64;
  uint64_t myword = 0;
  if (tid < nw_tile) {
    myword = s_bits[tid];
    const int64_t lim = t1 - (t0 + 64 * tid);  // bits at or beyond t1 belong to the next tile
    if (lim <= 0) myword = 0;
    else if (lim < 64) myword &= (1ULL << lim) - 1;
  }
  uint32_t nchunks;
  const uint32_t wbase = block_excl_scan((uint32_t)__popcll(myword), s_wsum, &nchunks);
  if (tid < nw_tile) {
    uint64_t x = myword;
    uint32_t k = wbase;
    while (x) {
      s_cstart[k++] = (uint16_t)(64 * tid + __ffsll((long long)x) - 1);
      x &= x - 1;
    }
  }
  if (tid == 0 && nchunks > 0) {
    // end of the last chunk: next chunk start at or after t1 (staged halo word first)
    int64_t q = -1;
    for (int w = (int)((t1 - t0) >> 6); w < kTileWords && q < 0; ++w) {
      uint64_t word = s_bits[w];
      const int64_t bit0 = t0 + 64 * w;
      if (bit0 < t1) word &= ~0ULL << (t1 - bit0);
      if (word) q = bit0 + __ffsll((long long)word) - 1;
    }
    if (q < 0) q = next_set_bit(a.bits, a.n_words, t0 + 64 * kTileWords, a.n_bytes);
    s_last_end = min(q, a.n_bytes);
  }
  __syncthreads();
  const int C = (int)nchunks;
  SW_STAMP(0);

  // 3. lengths; histogram by length (short) / long list
  for (int k = tid; k < C; k += kThreads) {
    const int64_t start = t0 + s_cstart[k];
    const int64_t end = (k + 1 < C) ? t0 + s_cstart[k + 1] : s_last_end;
    const int64_t len = end - start;
    if (len > kShort) {
      s_long[atomicAdd(&s_nlong, 1u)] = (uint16_t)k;
      s_cnt[k] = 0;
    } else {
      s_cnt[k] = (uint32_t)len;
      atomicAdd(&s_bin[len], 1u);
    }
  }
  __syncthreads();
  if (tid == 0) {  // bins in descending length: the longest chunks go to the first lanes
    uint32_t acc = 0;
    for (int L = kShort; L >= 1; --L) {
      const uint32_t c = s_bin[L];
      s_bin[L] = acc;
      acc += c;
    }
    s_bin[kShort + 1] = acc;  // number of short chunks
  }
  __syncthreads();
  for (int k = tid; k < C; k += kThreads) {
    const uint32_t len = s_cnt[k];
    if (len >= 1) s_order[atomicAdd(&s_bin[len], 1u)] = (uint16_t)k;
  }
  __syncthreads();
  const int n_short = (int)s_bin[kShort + 1];
  SW_STAMP(1);

  // 4. per-lane merge loop on short chunks, in place in the LDS window
  // rounds alternate direction (zig-zag) so a lane with a long chunk in one round gets a short
  // one in the next and the four waves finish together
  for (int r0 = 0; r0 < n_short; r0 += kThreads) {
    const int r = r0 + (((r0 / kThreads) & 1) ? (kThreads - 1 - tid) : tid);
    if (r >= n_short) continue;
    const int k = s_order[r];
    const int ls = s_cstart[k];
    s_cnt[k] = (uint32_t)lane_merge<Id, kWide>(a.table, s_id + ls, s_rk + ls, (int)s_cnt[k]);
  }

#ifdef SW_STAMPS
  __syncthreads();
  SW_STAMP(2);
#endif
  // 5. long chunks: one wave per chunk (LDS window if it fits, else the global work area)
  const int nl = (int)s_nlong;
  for (int q = wid; q < nl; q += kThreads / 64) {
    const int k = s_long[q];
    const int ls = s_cstart[k];
    const int64_t start = t0 + ls;
    const int64_t end = (k + 1 < C) ? t0 + s_cstart[k + 1] : s_last_end;
    const int64_t len = end - start;
    int64_t n;
    if (ls + len <= kWin) {
      n = coop_merge<Id, kWide>(a.table, s_id + ls, s_rk + ls, len, lane);
    } else {
      Id* gid = (Id*)a.lw_id + start;
      Id* grk = (Id*)a.lw_rk + start;
      for (int64_t i = lane; i < len; i += 64) gid[i] = (Id)a.bytes[start + i];
      wave_sync_mem<Id>();
      n = coop_merge<Id, kWide>(a.table, gid, grk, len, lane);
      if (lane == 0) atomicAdd(&s_nglobal, 1u);
    }
    if (lane == 0) s_cnt[k] = (uint32_t)n;
  }
  __syncthreads();

  SW_STAMP(3);
  // 6. tile-local exclusive offsets over chunk token counts
  const int per = (C + kThreads - 1) / kThreads;
  const int c0 = min(C, tid * per), c1 = min(C, c0 + per);
  uint32_t local_sum = 0;
  for (int k = c0; k < c1; ++k) local_sum += s_cnt[k];
  uint32_t tile_total;
  uint32_t off = block_excl_scan(local_sum, s_wsum, &tile_total);
  for (int k = c0; k < c1; ++k) {
    const uint32_t c = s_cnt[k];
    s_cnt[k] = off;
    off += c;
  }
  if (tid == 0) s_cnt[C] = tile_total;
  __syncthreads();
  const int64_t first = C > 0 ? t0 + s_cstart[0] : -1;
  if (tid == 0) {
    a.tile_cnt[tile] = tile_total;
    a.tile_first[tile] = first;
  }

  // 7. write the tile's ids contiguously (position space at `first`)
  int32_t* dst = a.scratch + first;
  if (s_nglobal == 0) {
    // every chunk's ids are in s_id: compact them into s_rk, then one coalesced store
    for (int k = tid; k < C; k += kThreads) {
      const uint32_t o = s_cnt[k], cnt = s_cnt[k + 1] - o;
      const int ls = s_cstart[k];
      for (uint32_t j = 0; j < cnt; ++j) s_rk[o + j] = s_id[ls + j];
    }
    __syncthreads();
    for (uint32_t j = tid; j < tile_total; j += kThreads) dst[j] = (int32_t)s_rk[j];
  } else {
    for (int k = tid; k < C; k += kThreads) {
      const uint32_t o = s_cnt[k], cnt = s_cnt[k + 1] - o;
      const int ls = s_cstart[k];
      const int64_t len = ((k + 1 < C) ? t0 + s_cstart[k + 1] : s_last_end) - (t0 + ls);
      if (ls + len > kWin) continue;  // global-work-area chunk: copied below
      for (uint32_t j = 0; j < cnt; ++j) dst[o + j] = (int32_t)s_id[ls + j];
    }
    for (int q = wid; q < nl; q += kThreads / 64) {
      const int k = s_long[q];
      const int ls = s_cstart[k];
      const int64_t len = ((k + 1 < C) ? t0 + s_cstart[k + 1] : s_last_end) - (t0 + ls);
      if (ls + len <= kWin) continue;
      const uint32_t o = s_cnt[k], cnt = s_cnt[k + 1] - o;
      const Id* gid = (const Id*)a.lw_id + t0 + ls;
      for (uint32_t j = lane; j < cnt; j += 64) dst[o + j] = (int32_t)gid[j];
    }
  }

  // 8. strings starting in this tile: tile-local output offset (rebased later)
#ifdef SW_STAMPS
  __syncthreads();
  SW_STAMP(4);
#endif
  for (int64_t s = s_slo + tid; s < a.n_str; s += kThreads) {
    const int64_t p = a.str_off[s];
    if (p >= t1) break;
    int lo = 0, hi = C;  // first chunk with start >= p
    const int lp = (int)(p - t0);
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (s_cstart[m] < lp) lo = m + 1; else hi = m;
    }
    a.out_off[s] = (int64_t)s_cnt[lo];
  }
#ifdef SW_STAMPS
  __syncthreads();
  SW_STAMP(5);
#endif
}

// first string starting at or after each tile's first byte (binary search per tile)
__global__ void k_tile_strings(const int64_t* str_off, int64_t n_str, int64_t n_tiles, int64_t* tile_slo) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  const int64_t t0 = t * kTile;
  int64_t lo = 0, hi = n_str;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (str_off[m] < t0) lo = m + 1; else hi = m;
  }
  tile_slo[t] = lo;
}

// ---------------------------------------------------------------------------------------
// tile-count scan (3 small kernels) + compaction + per-string offsets
// ---------------------------------------------------------------------------------------
constexpr int kScanPer = 16;                      // tiles per thread in the scan kernels
constexpr int kScanBlock = kThreads * kScanPer;   // tiles per scan block

__global__ void __launch_bounds__(kThreads) k_scan_reduce(const uint32_t* cnt, int64_t n, int64_t* part) {
  __shared__ uint32_t sh[kThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  uint64_t s = 0;
  for (int k = 0; k < kScanPer; ++k)
    if (base + k < n) s += cnt[base + k];
  // wave reduce then block reduce (64-bit)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  __shared__ uint64_t sw[kThreads / 64];
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int k = 0; k < kThreads / 64; ++k) t += sw[k];
    part[blockIdx.x] = (int64_t)t;
  }
  (void)sh;
}

__global__ void __launch_bounds__(1024) k_scan_parts(int64_t* part, int64_t n_parts, int64_t* total) {
  __shared__ int64_t sh[1024];
  int64_t carry = 0;
  for (int64_t base = 0; base < n_parts; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < n_parts ? part[i] : 0;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int64_t y = threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
      __syncthreads();
      sh[threadIdx.x] += y;
      __syncthreads();
    }
    if (i < n_parts) part[i] = carry + sh[threadIdx.x] - v;
    carry += sh[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ void __launch_bounds__(kThreads) k_scan_apply(const uint32_t* cnt, int64_t n, const int64_t* part,
                                                         int64_t* base_out) {
  __shared__ uint32_t sh[kThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  uint32_t v[kScanPer];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    v[k] = base + k < n ? cnt[base + k] : 0u;
    s += v[k];
  }
  // a tile holds < 2^32 ids and a block < 2^32 too only if tiles are small; scan in 64-bit
  uint64_t x = s;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  __shared__ uint64_t sw[kThreads / 64];
  if (lane == 63) sw[wid] = x;
  __syncthreads();
  uint64_t wb = 0;
  for (int k = 0; k < wid; ++k) wb += sw[k];
  int64_t run = part[blockIdx.x] + (int64_t)(wb + x - s);
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    if (base + k < n) base_out[base + k] = run;
    run += v[k];
  }
  (void)sh;
}

__global__ void __launch_bounds__(256) k_compact(const int32_t* scratch, const uint32_t* tile_cnt,
                                                 const int64_t* tile_first, const int64_t* tile_base,
                                                 int32_t* out) {
  const int64_t t = blockIdx.x;
  const uint32_t cnt = tile_cnt[t];
  if (!cnt) return;
  const int32_t* src = scratch + tile_first[t];
  int32_t* dst = out + tile_base[t];
  for (uint32_t j = threadIdx.x; j < cnt; j += 256) dst[j] = src[j];
}

__global__ void k_string_offsets(const int64_t* str_off, int64_t n_str, int64_t n_bytes, const int64_t* tile_base,
                                 const int64_t* total, int64_t* out_off) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n_str) return;
  if (s == n_str) { out_off[s] = *total; return; }
  const int64_t p = str_off[s];
  if (p >= n_bytes) out_off[s] = *total;
  else out_off[s] += tile_base[p / kTile];
}

}  // namespace sw
