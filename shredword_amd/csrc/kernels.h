// Device side of the batched encode (included by encode.hip only).
//
// Semantics per chunk (exact for ANY merge table; shredword/base.py:10-36): ids = bytes; while
// >= 2 ids: take the adjacent pair with the smallest merges-value (first occurrence on ties);
// stop if no pair is in merges; else replace every non-overlapping occurrence of that pair,
// left to right, by the value.
//
// Pipeline (one stream):
//   k_classify      one 256-thread workgroup per 2 KiB tile.  Stages the tile's bytes and its
//                   pre-split bitmap in LDS, enumerates the chunks, and settles every chunk that
//                   is a single byte or whose bytes are in the whole-chunk table (chunktable.h)
//                   with one lookup.  Every other chunk reserves `len` output slots (ids <=
//                   bytes) holding a sentinel and is queued by length bucket.  Writes the tile's
//                   slot region to a position-indexed scratch.
//   k_merge_bucket  the exact merge loop, one chunk per lane, chunk in REGISTERS (fixed
//                   positions + alive mask, compile-time size N); the 64 lanes of a wave come
//                   from one length bucket so their loops have similar trip counts; persistent
//                   grid-stride over the bucket's queue.  Writes ids into the reserved slots and
//                   adds the count to its tile.
//   k_merge_long    chunks > 32 bytes: one wave each, wave-cooperative loop in a position-
//                   indexed global work area.
//   k_scan_*        exclusive scan of per-tile id counts
//   k_compact       per tile: drop the sentinels (block stream compaction), write the ids
//                   contiguously, and turn each string's slot offset into its id offset.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "chunktable.h"
#include "table.h"

namespace sw {

constexpr int kTile = 2048;                  // input bytes per classify workgroup
constexpr int kThreads = 256;                // 4 waves
constexpr int kShort = 32;                   // per-lane merge loop up to this many bytes
constexpr int kWin = kTile + 64;             // LDS byte window (tile + halo for key reads)
constexpr int kTileWords = kTile / 64 + 1;   // bitmap words staged (tile + 64-bit halo)
constexpr int32_t kSentinel = -1;            // reserved output slot not holding an id
constexpr int kNumBuckets = 11;              // length buckets of the merge queue
constexpr int kLongBucket = kNumBuckets - 1;

// length -> bucket: groups of similar loop trip count
//   [2] [3] [4] [5,6] [7,8] [9,10] [11,12] [13,16] [17,24] [25,32] long(>32)
__host__ __device__ inline int bucket_of(int64_t len) {
  if (len <= 4) return (int)len - 2;
  if (len <= 12) return 3 + (int)((len - 5) >> 1);
  if (len <= 16) return 7;
  if (len <= 24) return 8;
  if (len <= 32) return 9;
  return kLongBucket;
}
__host__ __device__ inline int bucket_min_len(int b) {
  return b <= 2 ? b + 2 : b <= 6 ? 5 + 2 * (b - 3) : b == 7 ? 13 : b == 8 ? 17 : b == 9 ? 25 : 33;
}

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

// Whole-chunk table lookup (chunktable.h): the single token a 2..16-byte chunk encodes to, or
// kInf if the chunk does not encode to exactly one token.  k0/k1: the chunk's bytes, LE, zero
// padded.  Two (short) or four (long) independent 16-byte loads, one round trip.
__device__ __forceinline__ uint32_t chunk_lookup(const DevChunkTable& c, uint64_t k0, uint64_t k1, uint32_t len) {
  const uint32_t f = chunk_hash(k0, k1, len);
  if (len <= 8) {
    const uint4 q1 = c.sb[(f * c.s_m1) >> c.s_shift];
    const uint4 q2 = c.sb[((f ^ 0xA5A5A5A5u) * c.s_m2) >> c.s_shift];
    const uint32_t lo = (uint32_t)k0, hi = (uint32_t)(k0 >> 32);
    uint32_t v = kInf;
    v = (q1.x == lo && q1.y == hi && (q1.z >> 24) == len) ? (q1.z & 0xFFFFFFu) : v;
    v = (q2.x == lo && q2.y == hi && (q2.z >> 24) == len) ? (q2.z & 0xFFFFFFu) : v;
    return v;
  }
  const uint32_t b1 = (f * c.l_m1) >> c.l_shift, b2 = ((f ^ 0xA5A5A5A5u) * c.l_m2) >> c.l_shift;
  const uint4 a1 = c.lb[2 * b1], t1 = c.lb[2 * b1 + 1];
  const uint4 a2 = c.lb[2 * b2], t2 = c.lb[2 * b2 + 1];
  const uint4 k = make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
  uint32_t v = kInf;
  v = (a1.x == k.x && a1.y == k.y && a1.z == k.z && a1.w == k.w && (t1.x >> 24) == len) ? (t1.x & 0xFFFFFFu) : v;
  v = (a2.x == k.x && a2.y == k.y && a2.z == k.z && a2.w == k.w && (t2.x >> 24) == len) ? (t2.x & 0xFFFFFFu) : v;
  return v;
}

// bytes [ls, ls + len) of an LDS byte window as two zero-padded little-endian words (len <= 16)
__device__ __forceinline__ void window_key(const uint32_t* w32, int ls, int len, uint64_t* k0, uint64_t* k1) {
  const int q = ls >> 2, sh = ls & 3;
  const uint32_t w0 = w32[q], w1 = w32[q + 1], w2 = w32[q + 2], w3 = w32[q + 3], w4 = w32[q + 4];
  uint32_t b[4] = {__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                   __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int keep = len - 4 * i;
    b[i] = keep >= 4 ? b[i] : keep <= 0 ? 0u : (b[i] & ((1u << (8 * keep)) - 1u));
  }
  *k0 = ((uint64_t)b[1] << 32) | b[0];
  *k1 = ((uint64_t)b[3] << 32) | b[2];
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

// ---------------------------------------------------------------------------------------
// per-lane merge loop with the chunk held in REGISTERS (n <= N, N a compile-time bucket size)
//
// Fixed positions + an alive mask instead of compaction: a merge rewrites the left slot and
// kills the right one, so every array index is a compile-time constant after unrolling.  Per
// step: argmin over N keys, one left-to-right sweep applying the merge, one right-to-left sweep
// refreshing right-neighbour ids, then the changed pairs are re-ranked two lookups at a time.
// Returns the alive mask; the surviving ids are id[k] for the set bits, in order.
// ---------------------------------------------------------------------------------------
template <bool k16>
struct RegKey {  // (rank, slot) packed so that min() picks the lowest rank, then the first slot
  using T = typename std::conditional<k16, uint32_t, uint64_t>::type;
  static constexpr T inf = (T)~(T)0;
  __device__ static T make(uint32_t rank, int k) {
    if (k16) return ((T)(rank > 0xFFFFu ? 0xFFFFu : rank) << 5) | (T)k;
    return ((T)rank << 5) | (T)k;
  }
  __device__ static uint32_t rank(T key) {
    if (k16) {
      const uint32_t r = (uint32_t)(key >> 5);
      return r >= 0xFFFFu ? kInf : r;
    }
    return (uint32_t)(key >> 5);
  }
};

template <bool kWide, bool k16, int N>
__device__ __forceinline__ uint32_t lane_merge_reg(const DevTable& t, uint32_t (&id)[N], int n, int* iters = nullptr) {
  using RK = RegKey<k16>;
  constexpr uint32_t NONE = 0xFFFFFFFFu;  // no right neighbour
  uint32_t rid[N], rk[N];
#pragma unroll
  for (int k = 0; k < N; ++k) rid[k] = (k + 1 < n) ? id[(k + 1) % N] : NONE;
  uint32_t alive = (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
  // initial ranks: four lookups in flight at a time (sched barriers cap the live registers)
#pragma unroll
  for (int g = 0; g < N; g += 4) {
#pragma unroll
    for (int k = g; k < g + 4 && k < N; ++k) rk[k] = lookup<kWide>(t, id[k], rid[k]);
#pragma unroll
    for (int k = g; k < g + 4 && k < N; ++k) rk[k] = (rid[k] == NONE) ? kInf : rk[k];
    __builtin_amdgcn_sched_barrier(0);
  }
  int it = 0;
  while (true) {
    typename RK::T best = RK::inf;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const typename RK::T key = ((alive >> k) & 1u) ? RK::make(rk[k], k) : RK::inf;
      best = key < best ? key : best;
    }
    const uint32_t nv = RK::rank(best);
    if (nv == kInf) break;
    ++it;
    const int bi = (int)(best & 31);
    uint32_t p0 = 0, p1 = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      p0 = (k == bi) ? id[k] : p0;
      p1 = (k == bi) ? rid[k] : p1;
    }
    // left-to-right: take every non-overlapping occurrence of (p0, p1) (base.py:29-35).
    // Branch-free: every slot is a handful of v_cndmask, no exec-mask juggling.
    bool took = false;
    uint32_t changed = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const bool al = (alive >> k) & 1u;
      const bool consume = al && took;
      const bool match = al && !took && id[k] == p0 && rid[k] == p1;
      alive = consume ? (alive & ~(1u << k)) : alive;
      id[k] = match ? nv : id[k];
      changed |= match ? (1u << k) : 0u;
      took = al ? match : took;
    }
    // right-to-left: new right neighbours; pairs touching a new token need a new rank
    uint32_t carry = NONE, need = 0;
    bool carry_chg = false;
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
      const bool al = (alive >> k) & 1u;
      const bool chg = (changed >> k) & 1u;
      rid[k] = al ? carry : rid[k];
      need |= (al && carry != NONE && (chg || carry_chg)) ? (1u << k) : 0u;
      rk[k] = (al && carry == NONE) ? kInf : rk[k];
      carry = al ? id[k] : carry;
      carry_chg = al ? chg : carry_chg;
    }
    while (need) {  // two lookups in flight per round
      const int j1 = __ffs(need) - 1;
      need &= need - 1;
      const int j2 = need ? __ffs(need) - 1 : j1;
      need &= need - 1;
      uint32_t a1 = 0, b1 = 0, a2 = 0, b2 = 0;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        a1 = (k == j1) ? id[k] : a1;
        b1 = (k == j1) ? rid[k] : b1;
        a2 = (k == j2) ? id[k] : a2;
        b2 = (k == j2) ? rid[k] : b2;
      }
      const uint32_t r1 = lookup<kWide>(t, a1, b1), r2 = lookup<kWide>(t, a2, b2);
#pragma unroll
      for (int k = 0; k < N; ++k) {
        rk[k] = (k == j1) ? r1 : rk[k];
        rk[k] = (k == j2) ? r2 : rk[k];
      }
    }
  }
  if (iters) *iters = it;
  return alive;
}

// ---------------------------------------------------------------------------------------
// wave-cooperative exact merge loop on id[0..n), rk[0..n-1) (any n; global memory)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync_mem() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

template <bool kWide>
__device__ int64_t coop_merge(const DevTable& t, uint32_t* id, uint32_t* rk, int64_t n, int lane) {
  constexpr uint32_t INF = kInf, RECOMP = kInf - 1;
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  for (int64_t i = lane; i + 1 < n; i += 64) rk[i] = RECOMP;
  wave_sync_mem();
  while (n >= 2) {
    // pass 1: resolve pending ranks; argmin over (rank, index)
    uint64_t best = ~0ULL;
    for (int64_t i = lane; i + 1 < n; i += 64) {
      uint32_t r = rk[i];
      if (r == RECOMP) {
        r = lookup<kWide>(t, id[i], id[i + 1]);
        rk[i] = r;
      }
      const uint64_t key = ((uint64_t)r << 32) | (uint32_t)i;
      best = key < best ? key : best;
    }
    best = wave_min_u64(best);
    const uint32_t nv = (uint32_t)(best >> 32);
    if (nv == INF) break;
    const int64_t b = (int64_t)(uint32_t)best;
    wave_sync_mem();
    const uint32_t p0 = id[b], p1 = id[b + 1];
    // pass 2: replace every non-overlapping occurrence of (p0, p1), left to right, in place
    int64_t w = 0;
    bool prev_taken = false;
    for (int64_t seg = 0; seg < n; seg += 64) {
      const int64_t i = seg + lane;
      const bool valid = i < n;
      const uint32_t e = valid ? id[i] : INF;
      const uint32_t er = (valid && i + 1 < n) ? rk[i] : INF;
      uint32_t nid = __shfl_down(e, 1, 64);
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
      wave_sync_mem();  // all loads of this segment precede the in-place stores
      if ((keep >> lane) & 1ULL) {
        id[pos] = take ? nv : e;
        rk[pos] = (take || next_take) ? RECOMP : er;
      }
      w += __popcll(keep);
      prev_taken = (T >> 63) & 1ULL;
    }
    n = w;
    wave_sync_mem();
  }
  return n;
}

// ---------------------------------------------------------------------------------------
// arguments shared by the pipeline's kernels
// ---------------------------------------------------------------------------------------
struct EncArgs {
  const uint8_t* bytes;
  int64_t n_bytes;
  const uint64_t* bits;
  int64_t n_words;
  const int64_t* str_off;
  int64_t n_str;
  DevTable table;
  DevChunkTable chunks;
  int32_t* scratch;          // [n_bytes] slot regions, position space (tile t at tile_first[t])
  uint32_t* lw_id;           // [n_bytes] long-chunk work area, position space
  uint32_t* lw_rk;           // [n_bytes]
  uint32_t* tile_cnt;        // [n_tiles] ids per tile (classify writes, merges add)
  uint32_t* tile_slots;      // [n_tiles] slots per tile region
  int64_t* tile_first;       // [n_tiles] first chunk start in tile (or -1)
  int64_t* out_off;          // [n_str+1] string -> slot offset in its tile (k_compact converts)
  const int64_t* tile_slo;   // [n_tiles] first string starting at or after the tile start
  int64_t n_tiles;
  uint32_t* qtmp;            // [n_bytes] tile-local queue entries, position space (aliases lw_id)
  uint32_t* bcnt;            // [kNumBuckets * n_tiles] queued chunks per (bucket, tile)
  const int64_t* boff;       // [kNumBuckets * n_tiles] exclusive scan of bcnt (bucket-major)
  const int64_t* q_total;    // queued chunks in all
  uint64_t* queue;           // dense merge queue, bucket-major: start << 24 | len << 18 | slot
  unsigned long long* stamps;  // SW_STAMPS builds: cycles per phase, summed
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
#define SW_STAMP_INIT unsigned long long stamp_prev_ = __builtin_readcyclecounter()
#else
#define SW_STAMP(k) do {} while (0)
#define SW_STAMP_INIT do {} while (0)
#endif

// ---------------------------------------------------------------------------------------
// k_classify
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_classify(EncArgs a) {
  __shared__ uint32_t s_b32[kWin / 4 + 8];    // raw bytes of the window (+ zero tail)
  __shared__ uint64_t s_bits[kTileWords];
  __shared__ uint16_t s_cstart[kTile + 1];
  __shared__ uint32_t s_val[kTile];           // settled token, or kInf (queued)
  __shared__ uint32_t s_off[kTile + 1];       // slots per chunk, then exclusive slot offsets
  __shared__ uint32_t s_wsum[kThreads / 64];
  __shared__ uint32_t s_bcnt[kNumBuckets];
  __shared__ uint32_t s_bbase[kNumBuckets];
  __shared__ int64_t s_last_end;
  __shared__ uint32_t s_settled;

  SW_STAMP_INIT;
  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const int64_t t0 = tile * kTile;
  const int64_t t1 = min(t0 + (int64_t)kTile, a.n_bytes);
  const int64_t w0 = t0 >> 6;

  // 1. stage the window's bytes (4 per thread-load) and bitmap words
  for (int i = tid * 4; i < kWin; i += kThreads * 4) {
    const int64_t g = t0 + i;
    uint32_t v = 0;
    if (g + 4 <= a.n_bytes && ((uintptr_t)a.bytes & 3) == 0) v = *(const uint32_t*)(a.bytes + g);
    else
      for (int k = 0; k < 4; ++k) v |= (g + k < a.n_bytes ? (uint32_t)a.bytes[g + k] : 0u) << (8 * k);
    s_b32[i >> 2] = v;
  }
  if (tid < 8) s_b32[kWin / 4 + tid] = 0;
  if (tid < kTileWords) s_bits[tid] = (w0 + tid < a.n_words) ? a.bits[w0 + tid] : 0ULL;
  if (tid < kNumBuckets) s_bcnt[tid] = 0;
  if (tid == 0) s_settled = 0;
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

  // 3. settle single bytes and whole-chunk-table hits; the rest reserve len slots
  for (int k = tid; k < C; k += kThreads) {
    const int ls = s_cstart[k];
    const int64_t end = (k + 1 < C) ? t0 + s_cstart[k + 1] : s_last_end;
    const int64_t len = end - (t0 + ls);
    uint32_t tok = kInf;
    if (len == 1) {
      tok = (s_b32[ls >> 2] >> (8 * (ls & 3))) & 0xFFu;
    } else if (len <= 16 && a.chunks.enabled) {
      uint64_t k0, k1;
      window_key(s_b32, ls, (int)len, &k0, &k1);
      tok = chunk_lookup(a.chunks, k0, k1, (uint32_t)len);
    }
    s_val[k] = tok;
    s_off[k] = tok != kInf ? 1u : (uint32_t)min(len, (int64_t)0xFFFFFFFF);
    if (tok == kInf) atomicAdd(&s_bcnt[bucket_of(len)], 1u);
    const uint64_t settled = __ballot(tok != kInf);
    if ((tid & 63) == 0) atomicAdd(&s_settled, (uint32_t)__popcll(settled));
  }
  __syncthreads();
  SW_STAMP(1);

  // 4. slot offsets (exclusive scan over chunk slot counts); queue space per bucket
  const int per = (C + kThreads - 1) / kThreads;
  const int c0 = min(C, tid * per), c1 = min(C, c0 + per);
  uint32_t local = 0;
  for (int k = c0; k < c1; ++k) local += s_off[k];
  uint32_t n_slots;
  uint32_t off = block_excl_scan(local, s_wsum, &n_slots);
  for (int k = c0; k < c1; ++k) {
    const uint32_t c = s_off[k];
    s_off[k] = off;
    off += c;
  }
  if (tid == 0) s_off[C] = n_slots;
  if (tid == 0) {  // tile-local start of each bucket's entries
    uint32_t acc = 0;
    for (int b = 0; b < kNumBuckets; ++b) {
      s_bbase[b] = acc;
      acc += s_bcnt[b];
    }
  }
  __syncthreads();
  if (tid < kNumBuckets) {
    a.bcnt[(int64_t)tid * a.n_tiles + tile] = s_bcnt[tid];
    s_bcnt[tid] = 0;
  }
  __syncthreads();
  const int64_t first = C > 0 ? t0 + s_cstart[0] : -1;
  if (tid == 0) {
    a.tile_cnt[tile] = s_settled;
    a.tile_slots[tile] = n_slots;
    a.tile_first[tile] = first;
  }

  // 5. write the slot region; queue the unsettled chunks
  int32_t* dst = a.scratch + first;
  for (int k = tid; k < C; k += kThreads) {
    const uint32_t o = s_off[k], ns = s_off[k + 1] - o;
    const uint32_t tok = s_val[k];
    if (tok != kInf) {
      dst[o] = (int32_t)tok;
      continue;
    }
    const int b = bucket_of(ns);
    const uint32_t qi = s_bbase[b] + atomicAdd(&s_bcnt[b], 1u);
    // tile-local entry: chunk start in tile (11 bits) | slot offset (13) | length (6, 0 = long)
    a.qtmp[t0 + qi] = (uint32_t)s_cstart[k] | (o << 11) | ((b != kLongBucket ? ns : 0u) << 24);
    if (b != kLongBucket)
      for (uint32_t j = 0; j < ns; ++j) dst[o + j] = kSentinel;  // k_merge_long writes all its own
  }
  SW_STAMP(2);

  // 6. strings starting in this tile: slot offset within the tile (k_compact converts)
  for (int64_t s = a.tile_slo[tile] + tid; s < a.n_str; s += kThreads) {
    const int64_t p = a.str_off[s];
    if (p >= t1) break;
    int lo = 0, hi = C;  // first chunk with start >= p
    const int lp = (int)(p - t0);
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (s_cstart[m] < lp) lo = m + 1; else hi = m;
    }
    a.out_off[s] = (int64_t)s_off[lo];
  }
#ifdef SW_STAMPS
  __syncthreads();
  SW_STAMP(3);
#endif
}

// ---------------------------------------------------------------------------------------
// k_scatter: tile-local queue entries -> the dense bucket-major queue
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_scatter(EncArgs a) {
  // one wave per tile: lane b < kNumBuckets fetches (count, destination) of bucket b at once
  const int64_t t = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (t >= a.n_tiles) return;
  const int64_t t0 = t * kTile;
  uint32_t c = 0;
  int64_t dst = 0;
  if (lane < kNumBuckets) {
    c = a.bcnt[(int64_t)lane * a.n_tiles + t];
    dst = a.boff[(int64_t)lane * a.n_tiles + t];
  }
  uint32_t local = c;  // exclusive prefix of the counts over buckets = tile-local start
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) {
    const uint32_t y = __shfl_up(local, off, 64);
    if (lane >= off) local += y;
  }
  local -= c;
  for (int b = 0; b < kNumBuckets; ++b) {
    const uint32_t cb = __shfl(c, b, 64), lb = __shfl(local, b, 64);
    const int64_t db = __shfl(dst, b, 64);
    for (uint32_t j = lane; j < cb; j += 64) {
      const uint32_t e = a.qtmp[t0 + lb + j];
      const uint64_t start = (uint64_t)(t0 + (e & 0x7FFu));
      a.queue[db + j] = (start << 24) | ((uint64_t)(e >> 24) << 18) | ((e >> 11) & 0x1FFFu);
    }
  }
}

// [lo, hi) of the dense queue holding buckets b_lo..b_hi
__device__ __forceinline__ void bucket_range(const EncArgs& a, int b_lo, int b_hi, int64_t* lo, int64_t* hi) {
  *lo = a.boff[(int64_t)b_lo * a.n_tiles];
  *hi = (b_hi + 1 < kNumBuckets) ? a.boff[(int64_t)(b_hi + 1) * a.n_tiles] : *a.q_total;
}

// ---------------------------------------------------------------------------------------
// k_merge_bucket<N>: queued chunks of buckets [b_lo, b_hi] (length <= N), one per lane;
// persistent grid-stride over 64-entry batches, next batch's entry prefetched
// ---------------------------------------------------------------------------------------
template <bool kWide, bool k16, int N>
__global__ void __launch_bounds__(kThreads) k_merge_bucket(EncArgs a, int b_lo, int b_hi) {
  SW_STAMP_INIT;
  const int64_t gw = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;  // global wave id
  const int64_t n_waves = ((int64_t)gridDim.x * kThreads) >> 6;
  const int lane = threadIdx.x & 63;
  int64_t lo, hi;
  bucket_range(a, b_lo, b_hi, &lo, &hi);
  constexpr int W = N / 4 + 1;  // aligned words covering any N-byte span
  const int64_t mis = (int64_t)((uintptr_t)a.bytes & 3);
  const uint32_t* words = (const uint32_t*)((uintptr_t)a.bytes - mis);
  const int64_t last_word = (mis + a.n_bytes - 1) >> 2;  // last word holding input bytes
  int64_t i = lo + gw * 64 + lane;
  uint64_t e = i < hi ? a.queue[i] : 0;
#ifdef SW_STAMPS
  unsigned long long st_b = 0, st_loop = 0, st_batch = 0, st_it = 0;
#endif
  while (i < hi) {
#ifdef SW_STAMPS
    const unsigned long long batch_t0 = __builtin_readcyclecounter();
#endif
    const int64_t inext = i + n_waves * 64;
    const uint64_t enext = inext < hi ? a.queue[inext] : 0;  // prefetch
    const int64_t start = (int64_t)(e >> 24);
    const int n = (int)((e >> 18) & 63u);
    const uint32_t o = (uint32_t)(e & 0x3FFFFu);
    // the chunk's bytes: W aligned words, realigned with v_alignbyte
    const int64_t g = start + mis, w0 = g >> 2;
    uint32_t w[W];
#pragma unroll
    for (int k = 0; k < W; ++k) w[k] = words[min(w0 + k, last_word)];
    const uint32_t sh = (uint32_t)(g & 3);
    uint32_t id[N];
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      const uint32_t u = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh);
#pragma unroll
      for (int r = 0; r < 4; ++r) id[4 * q + r] = (4 * q + r < n) ? ((u >> (8 * r)) & 0xFFu) : 0u;
    }
#ifdef SW_STAMPS
    const unsigned long long c0 = __builtin_readcyclecounter();
#endif
#ifdef SW_ABL_NOLOOP  // ablation builds only: timing experiments, results are wrong
    const uint32_t alive = (n >= 32) ? ~0u : ((1u << n) - 1u);
#else
    int iters = 0;
    const uint32_t alive = lane_merge_reg<kWide, k16, N>(a.table, id, n, &iters);
#endif
#ifdef SW_STAMPS
    {
      const unsigned long long c1 = __builtin_readcyclecounter();
      int mx = iters;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) { const int o2 = __shfl_xor(mx, off, 64); mx = o2 > mx ? o2 : mx; }
      st_b += 1; st_loop += c1 - c0; st_batch += c1 - batch_t0; st_it += (unsigned long long)mx;
    }
#endif
    const int64_t tile = start / kTile;
    int32_t* dst = a.scratch + a.tile_first[tile] + o;
    int m = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if ((alive >> k) & 1u) {
#ifndef SW_ABL_NOWRITE
        dst[m] = (int32_t)id[k];
#endif
        ++m;
      }
    }
#ifndef SW_ABL_NOATOMIC
    atomicAdd(&a.tile_cnt[tile], (uint32_t)m);
#else
    if (m == 99999) a.tile_cnt[0] = 0;
#endif
    i = inext;
    e = enext;
  }
#ifdef SW_STAMPS
  if (lane == 0 && st_b) {
    const int gi = 8 + 4 * (N == 4 ? 0 : N == 8 ? 1 : N == 16 ? 2 : 3);
    atomicAdd(&a.stamps[gi + 0], st_b);
    atomicAdd(&a.stamps[gi + 1], st_loop);
    atomicAdd(&a.stamps[gi + 2], st_batch);
    atomicAdd(&a.stamps[gi + 3], st_it);
  }
  SW_STAMP(N >= 16 ? 5 : 4);
#endif
}

// long chunks (> kShort bytes): one wave each, wave-cooperative loop in the global work area
template <bool kWide>
__global__ void __launch_bounds__(kThreads) k_merge_long(EncArgs a) {
  SW_STAMP_INIT;
  const int64_t gw = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int64_t n_waves = ((int64_t)gridDim.x * kThreads) >> 6;
  const int lane = threadIdx.x & 63;
  int64_t lo, hi;
  bucket_range(a, kLongBucket, kLongBucket, &lo, &hi);
  for (int64_t i = lo + gw; i < hi; i += n_waves) {
    const uint64_t e = a.queue[i];
    const int64_t start = (int64_t)(e >> 24);
    const int64_t end = next_set_bit(a.bits, a.n_words, start + 1, a.n_bytes);
    const int64_t len = end - start;
    uint32_t* gid = a.lw_id + start;
    uint32_t* grk = a.lw_rk + start;
    for (int64_t j = lane; j < len; j += 64) gid[j] = a.bytes[start + j];
    wave_sync_mem();
    const int64_t m = coop_merge<kWide>(a.table, gid, grk, len, lane);
    const int64_t tile = start / kTile;
    int32_t* dst = a.scratch + a.tile_first[tile] + (int64_t)(e & 0x3FFFFu);
    for (int64_t j = lane; j < len; j += 64) dst[j] = j < m ? (int32_t)gid[j] : kSentinel;
    if (lane == 0) atomicAdd(&a.tile_cnt[tile], (uint32_t)m);
  }
#ifdef SW_STAMPS
  SW_STAMP(6);
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
// tile-count scan (3 small kernels)
// ---------------------------------------------------------------------------------------
constexpr int kScanPer = 16;                      // tiles per thread in the scan kernels
constexpr int kScanBlock = kThreads * kScanPer;   // tiles per scan block

__global__ void __launch_bounds__(kThreads) k_scan_reduce(const uint32_t* cnt, int64_t n, int64_t* part) {
  const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  uint64_t s = 0;
  for (int k = 0; k < kScanPer; ++k)
    if (base + k < n) s += cnt[base + k];
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
  const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanPer;
  uint32_t v[kScanPer];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    v[k] = base + k < n ? cnt[base + k] : 0u;
    s += v[k];
  }
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
}

// ---------------------------------------------------------------------------------------
// k_compact: per tile, drop sentinels from the slot region, write the ids at the tile's base,
// and convert the tile's string slot offsets into id offsets (stored complemented: k_string_
// offsets restores them).
// ---------------------------------------------------------------------------------------
constexpr int kCompactPer = 8;                          // slots per thread per pass
constexpr int kCompactPass = kThreads * kCompactPer;    // slots per pass

__global__ void __launch_bounds__(kThreads) k_compact(EncArgs a, const int64_t* tile_base, int32_t* out) {
  __shared__ __attribute__((aligned(16))) int32_t s_io[kCompactPass];  // slots in, ids out
  __shared__ uint32_t s_pref[kCompactPass + 1];  // ids before each slot of the pass
  __shared__ uint32_t s_wsum[kThreads / 64];
  const int64_t t = blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t n_slots = a.tile_slots[t];
  const int64_t base = tile_base[t];
  const int64_t t1 = min(t * kTile + (int64_t)kTile, a.n_bytes);
  const int32_t* src = a.scratch + a.tile_first[t];
  const int64_t s_lo = a.tile_slo[t];
  uint32_t done = 0;  // ids written by earlier passes
  for (uint32_t p0 = 0; p0 == 0 || p0 < n_slots; p0 += kCompactPass) {
    // coalesced load of the pass's slots into LDS
#pragma unroll
    for (int k = 0; k < kCompactPer; ++k) {
      const uint32_t j = p0 + k * kThreads + tid;
      s_io[k * kThreads + tid] = j < n_slots ? src[j] : kSentinel;
    }
    __syncthreads();
    int32_t v[kCompactPer];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < kCompactPer; ++k) {
      v[k] = s_io[tid * kCompactPer + k];
      c += v[k] != kSentinel;
    }
    uint32_t pass_total;
    uint32_t o = block_excl_scan(c, s_wsum, &pass_total);  // (its barriers also fence s_io reads)
#pragma unroll
    for (int k = 0; k < kCompactPer; ++k) {
      s_pref[tid * kCompactPer + k] = done + o;
      if (v[k] != kSentinel) s_io[o++] = v[k];
    }
    if (tid == 0) s_pref[kCompactPass] = done + pass_total;
    __syncthreads();
    // coalesced store of the pass's ids
#pragma unroll
    for (int k = 0; k < kCompactPer; ++k) {
      const uint32_t j = k * kThreads + tid;
      if (j < pass_total) out[base + done + j] = s_io[j];
    }
    // strings of this tile whose slot offset falls in this pass (or is the region's end)
    for (int64_t s = s_lo + tid; s < a.n_str; s += kThreads) {
      if (a.str_off[s] >= t1) break;
      const int64_t so = a.out_off[s];
      if (so < (int64_t)p0) continue;  // done in an earlier pass (complemented values are < 0)
      if (so < (int64_t)p0 + kCompactPass || so == (int64_t)n_slots) a.out_off[s] = ~(base + s_pref[so - p0]);
    }
    done += pass_total;
    __syncthreads();
  }
}

// every string offset: a complemented value is one k_compact finished; strings starting at or
// past n_bytes (trailing empty strings) and the end sentinel get the total
__global__ void k_string_offsets(const int64_t* str_off, int64_t n_str, int64_t n_bytes, const int64_t* total,
                                 int64_t* out_off) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n_str) return;
  if (s == n_str || str_off[s] >= n_bytes) {
    out_off[s] = *total;
    return;
  }
  out_off[s] = ~out_off[s];
}

}  // namespace sw
