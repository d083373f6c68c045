// Device side of the batched encode (included by encode.hip only).
//
// Semantics per chunk (exact for ANY merge table; shredword/base.py:10-36): ids = bytes; while
// >= 2 ids: take the adjacent pair with the smallest merges-value (first occurrence on ties);
// stop if no pair is in merges; else replace every non-overlapping occurrence of that pair,
// left to right, by the value.
//
// Pipeline (one stream):
//   k_classify      one wave per 2 KiB tile.  Stages the tile's bytes in LDS and its
//                   pre-split bitmap in registers, enumerates the chunks, and settles every chunk that
//                   is a single byte or whose bytes are in the whole-chunk table (chunktable.h)
//                   with one lookup.  Writes ONE slot per chunk (the token, or a reference to
//                   the chunk's merge result) and queues the rest by length bucket (tile-local).
//   k_scan_*, k_scatter  the tile-local queues -> one dense bucket-major queue
//   k_merge_bucket  the exact merge loop, one chunk per lane, chunk in REGISTERS (fixed
//                   positions + alive mask, compile-time size N); merge results go to res at
//                   twice the chunk's start position.  Only distinct chunks get here: k_classify
//                   dedupes repeats within the launch (dedupe_claim).
//   k_merge_long    chunks > 32 bytes: one wave each, wave-cooperative loop in a position-
//                   indexed global work area.
//   k_tile_count, k_scan_*  ids per tile (one wave per tile) and their exclusive scan
//   k_compact       one wave per tile: expand the slots into ids at the tile's base, turn each
//                   string's chunk index into its id offset.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "chunktable.h"
#include "table.h"

namespace sw {

constexpr int kTileBits = 11;
constexpr int kTile = 1 << kTileBits;        // input bytes per classify workgroup
constexpr int kThreads = 256;                // 4 waves
constexpr int kWaves = kThreads / 64;
// The wave's index in its block as a scalar (readfirstlane): the compiler then keeps the tile
// indices in SGPRs.  k_split_classify: 80 VGPRs + 36 B of scratch -> 80 VGPRs, no scratch, 3.20 ->
// 3.09 ms on C2, 6.14 -> 5.88 on ENTROPY (r6r A/B).  Rounds 4-5 measured it 180x slower with wrong
// string offsets: a miscompiled 64-bit min (tile_end below), not the index.
__device__ __forceinline__ int wave_in_block() {
  return (int)(threadIdx.x >> 6);
}
// A tile's end, min(t0 + kTile, n_bytes), in 32 bits (a launch is < 2^30 bytes).  With the tile
// index in SGPRs (wave_in_block_s), ROCm 7.2's compiler lowered the 64-bit signed min to a VALU
// compare (writing VCC) followed by s_cselect reading SCC -- the carry of the add before it: t1 was
// always n_bytes, every wave walked the strings to the batch's end (the 180x slower kernel of
// rounds 4-5) and wrote other tiles' string offsets (a diagnostic build printing them, r6q).  The 32-bit min
// is one s_min_i32.
__device__ __forceinline__ int64_t tile_end(int64_t t0, int64_t n_bytes) {
  return (int64_t)min((int32_t)t0 + (int32_t)kTile, (int32_t)n_bytes);
}
__device__ __forceinline__ int wave_in_block_s() {
  return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}
constexpr int kShort = 32;                   // per-lane merge loop up to this many bytes
constexpr int kWin = kTile + 64;             // LDS byte window (tile + halo for key reads)
constexpr int kTileWords = kTile / 64 + 1;   // bitmap words staged (tile + 64-bit halo)
constexpr int kNumBuckets = 11;              // length buckets of the merge queue
constexpr int kLongBucket = kNumBuckets - 1;
constexpr int64_t kRefSpace = 1LL << 30;              // position references below, dense ones above
constexpr int64_t kMaxLaunchBytes = kRefSpace - 64;   // slot references are int32

// A slot holds a settled token (>= 0) or refers to a merge result:
//  - slot_ref(p): the result of the chunk starting at position p, res[2p + 1 .. 2p + 1 + res[2p])
//    (count, then the ids: one contiguous run, and it fits, since a chunk of len bytes owns the
//    2 * len words from 2p);
//  - slot_dref(d): dense result d of the launch's dedupe (dres[d], below): the head of a result
//    shared by every occurrence of a chunk, in an array of ~16 B per DISTINCT chunk, so the
//    gathers of k_tile_count and k_compact stay in a few MB instead of spreading over res.
__host__ __device__ inline int32_t slot_ref(int64_t p) { return -(int32_t)(p + 2); }
__host__ __device__ inline int64_t slot_pos(int32_t v) { return -(int64_t)v - 2; }
__host__ __device__ inline int32_t slot_dref(uint32_t d) { return -(int32_t)((int64_t)d + 2 + kRefSpace); }
__host__ __device__ inline bool slot_is_dref(int32_t v) { return v <= -(int32_t)(2 + kRefSpace); }
__host__ __device__ inline uint32_t slot_did(int32_t v) { return (uint32_t)(-(int64_t)v - 2 - kRefSpace); }
// dense result heads, dres[d] (uint4, d: the chunk's dedupe table entry; count <= 32, p: the
// position of the occurrence that was merged, whose full result is at res[2p]):
//   16-bit ids:  count | id0 << 16, id1 | id2 << 16, id3 | id4 << 16, id5 | id6 << 16
//                (count > 7: count | id0 << 16, p, -, -)
//   32-bit ids:  count, id0, id1, id2 (count > 3: count, id0, id1, p)
// so 99.9% of the shared results (2-3 ids typical, 7 at most for a 32k vocabulary on prose)
// need no second read.  A reference list entry (rlist) is p or kRlDense | d.
constexpr uint32_t kRlDense = 0x80000000u;
// a tile's chunk-start list (uint16, tile-relative positions < kTile): bit 15 marks a chunk that is a
// special-token occurrence (its slot already holds the special's id), and lookups skip it
constexpr uint32_t kCsPos = 0x7FFFu, kCsSpecial = 0x8000u;
constexpr uint32_t kSpDone = 0xFFFFFFFEu;  // (table_lookups: the chunk's slot is written already)
constexpr uint32_t kNoDid = 0x7FFFFFFu;    // (27-bit dense result field of a queue entry: none)
constexpr int64_t kDdSlotsDefault = 1LL << 22;  // dedupe table entries at most to start with (32 MiB)
constexpr int64_t kDdSlotsMax = 1LL << 26;      // ... and after growing (a queue entry's dense field: 27 bits)
constexpr int kDdWords = 1;                     // 64-bit words per dedupe entry
constexpr uint32_t kDdGroup = 8;                // entries per 64-byte line (a chunk's candidates)
constexpr int kDdExactMax = 7;                  // dedupe keys of <= this many bytes are exact (no verification)
constexpr int kPairMaxN = 16;  // k_merge_bucket<N>: two chunks per lane up to this N
constexpr int kQuadMaxN = 4;   // ... and four up to this N

// streaming accesses (read or written once per launch) carry the non-temporal hint, so the
// caches keep the randomly gathered merge results instead
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Pointers with their address space spelled out.  A generic pointer the compiler cannot place --
// a select between an LDS and a global address, a pointer rebuilt from an integer, one read from
// a struct -- becomes a FLAT access, which waits on both the vector-memory and the LDS counters
// (k_compact's "ids to LDS staging or straight to memory" store was 144 flat stores).
#define SW_AS_GLOBAL __attribute__((address_space(1)))
#define SW_AS_LDS __attribute__((address_space(3)))
template <class T> __device__ __forceinline__ SW_AS_GLOBAL T* gptr(T* p) { return (SW_AS_GLOBAL T*)p; }
template <class T> __device__ __forceinline__ SW_AS_LDS T* lptr(T* p) { return (SW_AS_LDS T*)p; }
#define SW_LDNT(p) __builtin_nontemporal_load(p)
#define SW_STNT(p, v) __builtin_nontemporal_store((v), (p))
// the other streaming arrays -- bitmap words, reference lists, tile-local queues -- too
// (SW_MORE_NT=0: plain accesses; 6.333 -> 6.318 ms per launch, A/B kernel trace)
#define SW_LDNT2(p) __builtin_nontemporal_load(p)
#define SW_STNT2(p, v) __builtin_nontemporal_store((v), (p))

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
  if (!kWide && t.q16) {  // the quotient table (table.h): one 16-byte bucket, four tagged entries
    const uint32_t x = q16_mix((a << 16) | b, t.m1, t.m2), tag = x & 0xFFFFu;
    const uint4 q = ((const uint4*)t.buckets)[x >> t.shift];
    uint32_t v = 0xFFFFu;
    v = ((q.x & 0xFFFFu) == tag) ? (q.x >> 16) : v;
    v = ((q.y & 0xFFFFu) == tag) ? (q.y >> 16) : v;
    v = ((q.z & 0xFFFFu) == tag) ? (q.z >> 16) : v;
    v = ((q.w & 0xFFFFu) == tag) ? (q.w >> 16) : v;
    return (v == 0xFFFFu || (a | b) > 0xFFFFu) ? kInf : v;
  }
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

// Whole-chunk table (chunktable.h): the single token a 2..16-byte chunk encodes to, or kInf if the
// chunk does not encode to exactly one token -- table_lookups below.  The first candidate bucket,
// then the second only when the first neither matches nor carries the spill bit (chunktable.h).
// The compares are bitwise and every entry is loaded whole into registers before any use:
// otherwise the compiler narrows a 16-byte load to the words the first compare needs and fetches
// the rest in a branch, a second dependent round trip (5.97 -> 5.52 ms per C2 launch).

// bytes [ls, ls + len) of an LDS byte window as four zero-padded little-endian words (len <= 16)
__device__ __forceinline__ void window_words(const uint32_t* w32, int ls, int len, uint32_t (&b)[4]) {
  const int q = ls >> 2, sh = ls & 3;
  const uint32_t w0 = w32[q], w1 = w32[q + 1], w2 = w32[q + 2], w3 = w32[q + 3], w4 = w32[q + 4];
  b[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
  b[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
  b[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
  b[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int keep = len - 4 * i;  // bytes of word i inside the chunk
    const uint32_t m = keep >= 4 ? ~0u : keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u);
    b[i] &= m;
  }
}

// every loaded value in registers at this point (one wait for all the loads before it, none
// narrowed into a branch)
template <int R>
__device__ __forceinline__ void regs_barrier(u32x4 (&x)[R], u32x4 (&y)[R]) {
  static_assert(R >= 1 && R <= 4, "rounds");
  if constexpr (R == 1) asm volatile("" : "+v"(x[0]), "+v"(y[0]));
  if constexpr (R == 2) asm volatile("" : "+v"(x[0]), "+v"(y[0]), "+v"(x[1]), "+v"(y[1]));
  if constexpr (R == 3) asm volatile("" : "+v"(x[0]), "+v"(y[0]), "+v"(x[1]), "+v"(y[1]), "+v"(x[2]), "+v"(y[2]));
  if constexpr (R == 4)
    asm volatile("" : "+v"(x[0]), "+v"(y[0]), "+v"(x[1]), "+v"(y[1]), "+v"(x[2]), "+v"(y[2]), "+v"(x[3]), "+v"(y[3]));
}

// The whole-chunk-table answers (chunk_lookup) for R rounds of a tile's chunks (chunk 64 r + lane
// in round r), every round's probe in flight at once: the first candidate entry of every lane
// and round is loaded (16 bytes for 2..8-byte chunks, 32 for 9..16), one wait, the compares,
// then the (rare) second candidates the same way.  The chunk's bytes are read from the LDS
// window again after the wait rather than held in registers across it.
template <int R, bool kSp>
__device__ __forceinline__ void table_lookups(const DevChunkTable& c, const uint32_t* s_b32, const uint16_t* s_cstart,
                                              int C, int rel_end, int r0, int lane, uint32_t (&tok)[R]) {
  u32x4 qa[R], qb[R];
  uint32_t w[R][4];
  int len[R];
  uint32_t need2 = 0;  // rounds whose lane must probe the second candidate
#pragma unroll
  for (int u = 0; u < R; ++u) {  // first candidates: issue (the 32-byte entries' second half only
    const int k = ((r0 + u) << 6) + lane;  // for 9..16-byte chunks: no extra request for the rest)
    const bool valid = k < C;
    const uint32_t cs = valid ? s_cstart[k] : 0u;
    const int ls = (int)(cs & kCsPos);
    const int end = (k + 1 < C) ? (int)(s_cstart[k + 1] & kCsPos) : rel_end;
    const bool sp = kSp && (cs & kCsSpecial);  // (a special-token occurrence: its slot is written)
    len[u] = valid && !sp ? end - ls : 0;
    window_words(s_b32, ls, min(max(len[u], 1), 16), w[u]);
    tok[u] = sp ? kSpDone : len[u] == 1 ? (w[u][0] & 0xFFu) : kInf;
    const SW_AS_GLOBAL u32x4* pa = gptr((const u32x4*)c.sb);  // (a lane without a probe loads the first bucket, unused)
    if (len[u] >= 2 && len[u] <= 8)
      pa = gptr((const u32x4*)&c.sb[chunk_b1(chunk_hash(w[u][0], w[u][1], 0, 0, len[u], c.s_m1), c.s_shift)]);
    if (len[u] > 8 && len[u] <= 16)
      pa = gptr((const u32x4*)&c.lb[2 * chunk_b1(chunk_hash(w[u][0], w[u][1], w[u][2], w[u][3], len[u], c.l_m1), c.l_shift)]);
    qa[u] = *pa;
    qb[u] = u32x4{0u, 0u, 0u, 0u};
    if (len[u] > 8 && len[u] <= 16) qb[u] = pa[1];
  }
  regs_barrier<R>(qa, qb);
  auto compare = [&](int u) -> bool {  // the entry in qa/qb holds the chunk: tok[u] set
    bool hit;
    if (len[u] <= 8) {
      hit = (qa[u][0] == w[u][0]) & (qa[u][1] == w[u][1]) & ((qa[u][2] >> 24) == (uint32_t)len[u]);
      tok[u] = hit ? (qa[u][2] & 0xFFFFFFu) : tok[u];
    } else {
      hit = (qa[u][0] == w[u][0]) & (qa[u][1] == w[u][1]) & (qa[u][2] == w[u][2]) & (qa[u][3] == w[u][3]) &
            ((qb[u][0] >> 24) == (uint32_t)len[u]);
      tok[u] = hit ? (qb[u][0] & 0xFFFFFFu) : tok[u];
    }
    return hit;
  };
#pragma unroll
  for (int u = 0; u < R; ++u) {  // compares; second candidates: issue
    if (len[u] < 2 || len[u] > 16) continue;
    const bool hit = compare(u);
    const bool spill = ((len[u] <= 8 ? qa[u][3] : qb[u][1]) & 1u) != 0;
    if (!hit && spill) {
      need2 |= 1u << u;
      if (len[u] <= 8) {
        qa[u] = *gptr((const u32x4*)&c.sb[chunk_b2(chunk_hash(w[u][0], w[u][1], 0, 0, len[u], c.s_m1), c.s_m2, c.s_shift)]);
      } else {
        const SW_AS_GLOBAL u32x4* pa = gptr((const u32x4*)&c.lb[2 * chunk_b2(
            chunk_hash(w[u][0], w[u][1], w[u][2], w[u][3], len[u], c.l_m1), c.l_m2, c.l_shift)]);
        qa[u] = pa[0];
        qb[u] = pa[1];
      }
    }
  }
  if (!__ballot(need2 != 0)) return;
  regs_barrier<R>(qa, qb);
#pragma unroll
  for (int u = 0; u < R; ++u)  // second candidates: compares
    if ((need2 >> u) & 1u) compare(u);
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

// Inclusive scan over the wave's 64 lanes (every lane active), by DPP: row shifts 1, 2, 4, 8 within
// each 16-lane row, then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) -- six VALU
// operations instead of six shuffles through the LDS crossbar (ds_bpermute), each a round trip.
// r7x A/B: C2 234.8 -> 238.5 GB/s (k_compact 0.94 -> 0.89 ms), C3 GPT-2 + specials 251 -> 264
// (k_classify<true> 2.39 -> 2.24 ms).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
  (void)lane;  // (a lane whose source is outside its row, or masked off by row_mask, adds 0)
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

// lane L's value to every lane (L wave-uniform, every lane active): v_readlane (an SGPR, no LDS
// crossbar round trip)
__device__ __forceinline__ uint32_t lane_value(uint32_t x, int L) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, L);
}
__device__ __forceinline__ unsigned long long lane_value64(unsigned long long x, int L) {
  return (unsigned long long)lane_value((uint32_t)x, L) | ((unsigned long long)lane_value((uint32_t)(x >> 32), L) << 32);
}

// the wave's sum in every lane (every lane active)
__device__ __forceinline__ uint32_t wave_sum(uint32_t v, int lane) {
  return lane_value(wave_incl_scan(v, lane), 63);
}

// exclusive block scan over kThreads threads (sh: kThreads/64 words); *total = block sum
__device__ inline uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t x = wave_incl_scan(v, lane);
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

// the loop itself: id[k] / rk[k] = the ids and the ranks of the pairs (k, k + 1) (kInf past n - 1)
template <bool kWide, bool k16, int N>
__device__ __forceinline__ uint32_t lane_merge_reg_loop(const DevTable& t, uint32_t (&id)[N], uint32_t (&rk)[N], int n,
                                                        int* iters = nullptr) {
  using RK = RegKey<k16>;
  constexpr uint32_t NONE = 0xFFFFFFFFu;  // no right neighbour
  uint32_t rid[N];
#pragma unroll
  for (int k = 0; k < N; ++k) rid[k] = (k + 1 < n) ? id[(k + 1) % N] : NONE;
  uint32_t alive = (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
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

// The same loop for a WELL-FORMED table with 16-bit ids (every trained table; SW_INFO_SPLIT):
// a value names exactly one pair, so the winning pair's occurrences are the alive slots whose
// rank equals it (no id compares, no fetch of the pair's ids), and the ranks are kept as
// min-ready keys rank << 5 | slot (rank 0xFFFF: no pair -- a dead slot or the last one), so a
// step's argmin is one min per slot.  About a quarter fewer VALU instructions per step.
template <bool kWide, int N>
__device__ __forceinline__ uint32_t lane_merge_reg_loop_wf(const DevTable& t, uint32_t (&id)[N], uint32_t (&rk)[N], int n,
                                                           int* iters = nullptr) {
  constexpr uint32_t NONE = 0xFFFFFFFFu;  // no right neighbour
  constexpr uint32_t KINF = 0xFFFFu << 5;
  uint32_t rid[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    rid[k] = (k + 1 < n) ? id[(k + 1) % N] : NONE;
    rk[k] = ((k + 1 < n) ? (min(rk[k], 0xFFFFu) << 5) : KINF) | (uint32_t)k;
  }
  uint32_t alive = (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
  int it = 0;
  while (true) {
    uint32_t best = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < N; ++k) best = min(best, rk[k]);
    const uint32_t nv = best >> 5;
    if (nv >= 0xFFFFu) break;
    ++it;
    // left-to-right: every non-overlapping occurrence of the winning pair (base.py:29-35)
    bool took = false;
    uint32_t changed = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const bool al = (alive >> k) & 1u;
      const bool consume = al && took;
      const bool match = al && !took && (rk[k] >> 5) == nv;
      alive = consume ? (alive & ~(1u << k)) : alive;
      id[k] = match ? nv : id[k];
      changed |= match ? (1u << k) : 0u;
      took = al ? match : took;
    }
    // right-to-left: new right neighbours; dead slots and the last alive one get no pair; pairs
    // touching a new token need a new rank
    uint32_t carry = NONE, need = 0;
    bool carry_chg = false;
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
      const bool al = (alive >> k) & 1u;
      const bool chg = (changed >> k) & 1u;
      rid[k] = al ? carry : rid[k];
      need |= (al && carry != NONE && (chg || carry_chg)) ? (1u << k) : 0u;
      rk[k] = (!al || carry == NONE) ? (KINF | (uint32_t)k) : rk[k];
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
      const uint32_t k1 = (min(lookup<kWide>(t, a1, b1), 0xFFFFu) << 5) | (uint32_t)j1;
      const uint32_t k2 = (min(lookup<kWide>(t, a2, b2), 0xFFFFu) << 5) | (uint32_t)j2;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        rk[k] = (k == j1) ? k1 : rk[k];
        rk[k] = (k == j2) ? k2 : rk[k];
      }
    }
  }
  if (iters) *iters = it;
  return alive;
}

// the initial ranks of slots g .. g + 3 are in registers before any later slot's lookups issue
// (lane_merge_lds_wf: the compiler otherwise hoisted all N lookups -- 8 registers each in
// flight -- to the front: 239 VGPRs at N = 32, 132 with this)
template <int N, int G = 4>
__device__ __forceinline__ void rank_group_done(uint32_t (&rk)[N], int g) {
  if constexpr (G == 8) {  // (groups of 8 lookups: lane_merge_lds_wfq, N = 8, 16)
    asm volatile("" : "+v"(rk[g]), "+v"(rk[g + 1]), "+v"(rk[g + 2]), "+v"(rk[g + 3]), "+v"(rk[g + 4]), "+v"(rk[g + 5]),
                      "+v"(rk[g + 6]), "+v"(rk[g + 7])::"memory");
  } else if constexpr (N >= 4) {
    asm volatile("" : "+v"(rk[g]), "+v"(rk[g + 1]), "+v"(rk[g + 2]), "+v"(rk[g + 3])::"memory");
  } else {
    asm volatile("" ::: "memory");
  }
}

// min / rank-match mask over a lane's N keys as balanced trees: a left-to-right chain is N
// dependent instructions per step, and the loop's steps are short enough that those RAW stalls
// were most of its issue time (k_lp_encode / k_merge_bucket: 52-71% of wave cycles in
// SQ_WAIT_INST_ANY)
template <int N, int L = 0, int R = N>
__device__ __forceinline__ uint32_t tree_min(const uint32_t (&x)[N]) {
  if constexpr (R - L == 1) return x[L];
  else return min(tree_min<N, L, (L + R) / 2>(x), tree_min<N, (L + R) / 2, R>(x));
}
template <int N, int L = 0, int R = N>
__device__ __forceinline__ uint32_t tree_below(const uint32_t (&x)[N], uint32_t bound) {  // bit k: x[k] < bound
  if constexpr (R - L == 1) return (x[L] < bound ? 1u : 0u) << L;
  else return tree_below<N, L, (L + R) / 2>(x, bound) | tree_below<N, (L + R) / 2, R>(x, bound);
}

// Alive-set arithmetic on a lane's position mask A (bit k: position k holds a token):
// next_alive(A, S): for each position of S (a subset of A) the next alive position after it
// (none past bit 31): the bits just above S, carried through the gaps of A by one addition.
__device__ __forceinline__ uint32_t next_alive(uint32_t A, uint32_t S) {
  const uint32_t T = S << 1, G = ~A;
  return (T & A) | ((G + (T & G)) & A);
}
__device__ __forceinline__ uint32_t prev_alive(uint32_t A, uint32_t S) {
  return __builtin_bitreverse32(next_alive(__builtin_bitreverse32(A), __builtin_bitreverse32(S)));
}

// The merge loop for a WELL-FORMED table with 16-bit ids, with the ids in LDS and the pairs'
// ranks in registers as min-ready keys (rank << 5 | slot), every step done on bit masks:
//   - the winning rank: one min per slot;
//   - its occurrences M: the slots whose key has that rank (a value names one pair);
//   - their right partners: next_alive(A, M).  Occurrences overlap only for an (a, a) pair
//     (two adjacent occurrences of one pair are a, a, a); then they are taken left to right,
//     each one removing its partner, as merge() does (base.py:29-35);
//   - the partners die, the occurrences take the new id (LDS stores at their slots), and only the
//     pairs of the occurrences and of the alive slots before them are looked up again.
// So a step costs a few instructions per slot (the min, the rank compare, the key updates)
// instead of two sweeps that carry ids along, and the ids hold no registers.  s_id: this wave's
// ids, slot k of lane l at s_id[64 k + l] (a wave's accesses to one slot hit 64 banks).
// Returns the alive mask; the surviving ids are s_id[64 k + lane] for its set bits, in order.
template <bool kWide, int N>
__device__ __forceinline__ uint32_t lane_merge_lds_wf(const DevTable& t, const uint32_t (&u)[N / 4], int n,
                                                      uint32_t* s_id, int lane) {
  static_assert(N <= 32, "alive masks are 32 bits");
  constexpr uint32_t KINF = 0xFFFFu << 5;
  uint32_t rk[N];
#pragma unroll
  for (int k = 0; k < N; ++k) s_id[64 * k + lane] = (u[k >> 2] >> (8 * (k & 3))) & 0xFFu;
  // initial ranks: four lookups in flight at a time
#pragma unroll
  for (int g = 0; g < N; g += 4) {
#pragma unroll
    for (int k = g; k < g + 4 && k < N; ++k) {
      const uint32_t b0 = (u[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      const uint32_t b1 = (k + 1 < N) ? (u[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu : 0u;
      rk[k] = lookup<kWide>(t, b0, b1);
    }
#pragma unroll
    for (int k = g; k < g + 4 && k < N; ++k) rk[k] = ((k + 1 < n) ? (min(rk[k], 0xFFFFu) << 5) : KINF) | (uint32_t)k;
    rank_group_done<N>(rk, g);
  }
  uint32_t alive = (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
  while (true) {
    const uint32_t best = tree_min<N>(rk);
    const uint32_t nv = best >> 5;
    if (nv >= 0xFFFFu) break;
    const uint32_t bound = (nv + 1) << 5;  // (every key is >= best: rank nv <=> key < bound)
    const uint32_t m0 = tree_below<N>(rk, bound);
    uint32_t match = m0, cons = next_alive(alive, m0);
    if (cons & m0) {  // an (a, a) pair with adjacent occurrences: left to right
      match = 0;
      for (uint32_t av = m0; av;) {
        const uint32_t s = av & (0u - av);
        match |= s;
        av &= ~(s | next_alive(alive, s));
      }
      cons = next_alive(alive, match);
    }
    alive &= ~cons;
    for (uint32_t m = match; m; m &= m - 1) s_id[64 * (__ffs(m) - 1) + lane] = nv;
    // a partner that was the last alive slot leaves its occurrence without a right neighbour
    const uint32_t last = 1u << (31 - __clz(alive));
    const uint32_t kill = cons | (match & last);
    uint32_t need = (match | prev_alive(alive, match)) & alive & ~last;
#pragma unroll
    for (int k = 0; k < N; ++k) rk[k] = ((kill >> k) & 1u) ? (KINF | (uint32_t)k) : rk[k];
    while (need) {  // two lookups in flight per round
      const int j1 = __ffs(need) - 1;
      need &= need - 1;
      const int j2 = need ? __ffs(need) - 1 : j1;
      need &= need - 1;
      const int x1 = __ffs(next_alive(alive, 1u << j1)) - 1, x2 = __ffs(next_alive(alive, 1u << j2)) - 1;
      const uint32_t a1 = s_id[64 * j1 + lane], b1 = s_id[64 * x1 + lane];
      const uint32_t a2 = s_id[64 * j2 + lane], b2 = s_id[64 * x2 + lane];
      const uint32_t k1 = (min(lookup<kWide>(t, a1, b1), 0xFFFFu) << 5) | (uint32_t)j1;
      const uint32_t k2 = (min(lookup<kWide>(t, a2, b2), 0xFFFFu) << 5) | (uint32_t)j2;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        rk[k] = (k == j1) ? k1 : rk[k];
        rk[k] = (k == j2) ? k2 : rk[k];
      }
    }
  }
  return alive;
}

// lane_merge_lds_wf for Q chunks per lane (2 or 4), run side by side: every step of every loop
// issues its lookups before any waits, so a lane keeps Q times the lookups in flight (the merge loop
// without memoisation is a chain of dependent L2-hit lookups per chunk, not work: 66-71% of its
// wave cycles were issue stalls, profiles/r3n_none.md; the short buckets take 4 per lane: their
// loops are a few steps each, almost all waiting).  Chunk q's ids at s_id[64 (q N + k) + l].
template <bool kWide, int N, int Q>
__device__ __forceinline__ void lane_merge_lds_wfq(const DevTable& t, const uint32_t (&u)[Q][N / 4], const int (&n)[Q],
                                                   uint32_t* s_id, int lane, uint32_t (&alive)[Q]) {
  static_assert(N <= 32, "alive masks are 32 bits");
  constexpr uint32_t KINF = 0xFFFFu << 5;
  uint32_t rk[Q][N];
#pragma unroll
  for (int q = 0; q < Q; ++q)
#pragma unroll
    for (int k = 0; k < N; ++k) s_id[64 * (q * N + k) + lane] = (u[q][k >> 2] >> (8 * (k & 3))) & 0xFFu;
  // initial ranks: four lookups of each chunk in flight at a time
  constexpr int G = 4;  // (lookups of a chunk in flight per group)
#pragma unroll
  for (int g = 0; g < N; g += G) {
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int k = g; k < g + G && k < N; ++k) {
        const uint32_t b0 = (u[q][k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t b1 = (k + 1 < N) ? (u[q][(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu : 0u;
        rk[q][k] = lookup<kWide>(t, b0, b1);
      }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
#pragma unroll
      for (int k = g; k < g + G && k < N; ++k)
        rk[q][k] = ((k + 1 < n[q]) ? (min(rk[q][k], 0xFFFFu) << 5) : KINF) | (uint32_t)k;
      rank_group_done<N, G>(rk[q], g);
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) alive[q] = (n[q] >= 32) ? 0xFFFFFFFFu : ((1u << n[q]) - 1u);
  while (true) {
    uint32_t need[Q];
    bool any = false;
#pragma unroll
    for (int q = 0; q < Q; ++q) {  // one step of each chunk's loop (base.py:10-36), as lane_merge_lds_wf
      const uint32_t best = tree_min<N>(rk[q]);
      const uint32_t nv = best >> 5;
      need[q] = 0;
      if (nv >= 0xFFFFu) continue;
      any = true;
      const uint32_t bound = (nv + 1) << 5;
      const uint32_t m0 = tree_below<N>(rk[q], bound);
      uint32_t match = m0, cons = next_alive(alive[q], m0);
      if (cons & m0) {  // an (a, a) pair with adjacent occurrences: left to right
        match = 0;
        for (uint32_t av = m0; av;) {
          const uint32_t s = av & (0u - av);
          match |= s;
          av &= ~(s | next_alive(alive[q], s));
        }
        cons = next_alive(alive[q], match);
      }
      alive[q] &= ~cons;
      for (uint32_t m = match; m; m &= m - 1) s_id[64 * (q * N + __ffs(m) - 1) + lane] = nv;
      const uint32_t last = 1u << (31 - __clz(alive[q]));
      const uint32_t kill = cons | (match & last);
      need[q] = (match | prev_alive(alive[q], match)) & alive[q] & ~last;
#pragma unroll
      for (int k = 0; k < N; ++k) rk[q][k] = ((kill >> k) & 1u) ? (KINF | (uint32_t)k) : rk[q][k];
    }
    if (!any) break;
    while (true) {  // two lookups of each chunk in flight per round
      uint32_t pend = 0;
#pragma unroll
      for (int q = 0; q < Q; ++q) pend |= need[q];
      if (!pend) break;
      int j1[Q], j2[Q];
      uint32_t k1[Q], k2[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        j1[q] = need[q] ? __ffs(need[q]) - 1 : -1;
        need[q] &= need[q] - 1;
        j2[q] = need[q] ? __ffs(need[q]) - 1 : j1[q];
        need[q] &= need[q] - 1;
        k1[q] = k2[q] = 0;
        if (j1[q] < 0) continue;
        const int a1 = j1[q], a2 = j2[q];
        const int x1 = __ffs(next_alive(alive[q], 1u << a1)) - 1, x2 = __ffs(next_alive(alive[q], 1u << a2)) - 1;
        const uint32_t ia1 = s_id[64 * (q * N + a1) + lane], ib1 = s_id[64 * (q * N + x1) + lane];
        const uint32_t ia2 = s_id[64 * (q * N + a2) + lane], ib2 = s_id[64 * (q * N + x2) + lane];
        k1[q] = (min(lookup<kWide>(t, ia1, ib1), 0xFFFFu) << 5) | (uint32_t)a1;
        k2[q] = (min(lookup<kWide>(t, ia2, ib2), 0xFFFFu) << 5) | (uint32_t)a2;
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (j1[q] < 0) continue;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          rk[q][k] = (k == j1[q]) ? k1[q] : rk[q][k];
          rk[q][k] = (k == j2[q]) ? k2[q] : rk[q][k];
        }
      }
    }
  }
}

template <bool kWide, bool k16, int N, bool kWF = false>
__device__ __forceinline__ uint32_t lane_merge_reg(const DevTable& t, uint32_t (&id)[N], int n, int* iters = nullptr) {
  uint32_t rk[N];
  // initial ranks: four lookups in flight at a time (sched barriers cap the live registers)
#pragma unroll
  for (int g = 0; g < N; g += 4) {
#pragma unroll
    for (int k = g; k < g + 4 && k < N; ++k) rk[k] = lookup<kWide>(t, id[k], id[(k + 1) % N]);
#pragma unroll
    for (int k = g; k < g + 4 && k < N; ++k) rk[k] = (k + 1 < n) ? rk[k] : kInf;
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (kWF && k16 && !kWide) return lane_merge_reg_loop_wf<kWide, N>(t, id, rk, n, iters);
  else return lane_merge_reg_loop<kWide, k16, N>(t, id, rk, n, iters);
}

// ---------------------------------------------------------------------------------------
// wave-cooperative exact merge loop on id[0..n), rk[0..n-1) (any n; global memory)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync_mem() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

template <bool kWide>
__device__ __forceinline__ int64_t coop_merge(const DevTable& t, uint32_t* id, uint32_t* rk, int64_t n, int lane) {
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
// special-token occurrences of a launch (E1; sw_encode_ex): ascending, non-overlapping, each
// inside one string and one chunk of its own; tile_sp[t] (t <= n_tiles): the first one starting at
// or after tile t's first byte (k_tile_specials), so tile_sp[n_tiles] is the live count -- the
// host's, or the one the device finder left in device memory (n is then only the capacity)
struct SpArgs {
  const int64_t* pos;
  const int32_t* len;
  const int32_t* id;
  int64_t n;                 // > 0: the launch has occurrences (at most n)
  const int64_t* tile_sp;    // [n_tiles + 1]
  const int64_t* tile_spw;   // [n_tiles + 1] the first occurrence ending at or after tile t's first byte - 64
                             // (the start of k_split_classify's and k_edges' windows; k_tile_specials)
};

struct EncArgs {
  const uint8_t* bytes;
  int64_t n_bytes;
  const uint64_t* bits;
  int64_t n_words;
  const int64_t* str_off;
  int64_t n_str;
  DevTable table;
  DevChunkTable chunks;
  int32_t* scratch;          // [n_bytes] one slot per chunk, tile t's at t * kTile (slot_ref)
  uint32_t* res;             // [2 n_bytes] merge results (slot_ref); long chunks' work area
  uint32_t* tile_cnt;        // [n_tiles] ids per tile (k_tile_count)
  uint32_t* tile_slots;      // [n_tiles] chunks (= slots) per tile
  uint32_t* tile_nref;       // [n_tiles] reference slots per tile
  uint32_t* rlist;           // [n_tiles * kTile] per tile: the result positions its references use
  int64_t* out_off;          // [n_str+1] string -> chunk index in its tile (k_compact converts)
  const int64_t* tile_slo;   // [n_tiles] first string starting at or after the tile start
  int64_t n_tiles;
  uint32_t* qtmp;            // [n_bytes] tile-local queue entries, position space (aliases res)
  uint32_t* bcnt;            // [kNumBuckets * n_tiles] queued chunks per (bucket, tile)
  const int64_t* boff;       // [kNumBuckets * n_tiles] exclusive scan of bcnt (bucket-major)
  const int64_t* q_total;    // queued chunks in all
  uint64_t* queue;           // dense merge queue, bucket-major: start << 33 | len << 27 | dense result
  uint64_t* dtab;            // chunk dedupe table (dedupe_claim), dmask + 1 entries, cleared per launch
  uint32_t dmask;
  uint32_t dfp_mask;         // fingerprint bits in use (all 26 except in collision tests)
  uint32_t dedupe;           // 0: every queued chunk runs its own merge loop
  uint32_t dexact;           // longest exact dedupe key (kDdExactMax, or 0: every key verified)
  uint4* dres;               // [dmask + 1] dense result heads (slot_dref), by table entry
  uint8_t* dcnt;             // [dmask + 1] their id counts (<= 32): k_tile_count's reads stay in L2
  unsigned long long* dd_full;  // dedupable chunks of the launch that found no free candidate (k_scatter)
  uint64_t* llist;           // chunks over kShort bytes, as k_classify finds them: start << 32 | length
                             // (kNoDid: too long for the field, or running past its tile: k_lp_prep
                             // finds the end in the bitmap); any order.  Count in *l_count
  unsigned long long* l_count;  // (zeroed by k_tile_strings)
  unsigned long long* stamps;  // SW_STAMPS builds: cycles per phase, summed
  const uint2* inv;          // [n_inv] merge value -> its pair (a, b); well-formed tables only
  uint32_t n_inv;
  // the long chunks (> kShort bytes) for the per-chunk kernels, listed by k_lp_prep (any order)
  const uint32_t* lstart;    // first byte
  const uint32_t* llen;      // bytes
  const int64_t* n_long;     // how many (device)
  int64_t lcap;              // list capacity
  uint32_t* big_list;        // long chunks over kLongLds bytes (their index in the long list)
  uint32_t* big_count;       // ... how many (cleared per launch)
  uint32_t ids16;            // every id fits 16 bits (dres layout)
  uint32_t staged_heads;     // k_tile_count_staged wrote each tile's first kStageCap result heads into its rlist
                             // range (k_compact reads them there, in order, instead of gathering them)
  SpArgs sp;                 // special-token occurrences (sp.n == 0: none)
};

#ifdef SW_STAMPS
#define SW_STAMP(k)                                                                 \
  do {                                                                              \
    if (threadIdx.x == 0) {                                                         \
      const unsigned long long now_ = __builtin_readcyclecounter();                 \
      atomicAdd(&a.stamps[(k) * 64 + (blockIdx.x & 63)], now_ - stamp_prev_);       \
      stamp_prev_ = now_;                                                           \
    }                                                                               \
  } while (0)
#define SW_STAMP_INIT unsigned long long stamp_prev_ = __builtin_readcyclecounter()
#define SW_COUNT(k, v)                                                              \
  do {                                                                              \
    if (threadIdx.x == 0) atomicAdd(&a.stamps[(k) * 64 + (blockIdx.x & 63)], (unsigned long long)(v)); \
  } while (0)
#else
#define SW_COUNT(k, v) do {} while (0)
#define SW_STAMP(k) do {} while (0)
#define SW_STAMP_INIT do {} while (0)
#endif


// ---------------------------------------------------------------------------------------
// Batch-wide dedupe of queued chunks (in k_classify).  Real text repeats its multi-token words
// endlessly, and a chunk's encoding depends on its bytes alone, so the merge loop needs to run
// once per DISTINCT chunk of the launch.  The table (cleared before every launch) holds one
// word per claimed chunk, 8 candidates per chunk in one 64-byte line:
//   exact keys, chunks of <= 7 bytes:  bytes | length << 56 | 1 << 63
//   longer chunks:                     26-bit fingerprint << 37 | length << 31 | position
// The first occurrence claims an entry with a CAS on w0 and is merged; its result head lands in
// dres at the entry's index, which every later occurrence refers to (slot_dref): nothing has to
// be read back from the claimant.  Exact keys decide equality by themselves; a fingerprint match
// is confirmed by comparing the bytes with the claimant's bytes in the (immutable) input, so no
// hash collision can change a result.  A chunk that finds no free candidate merges itself.
// Only the CAS needs cross-XCD coherence.  (Two-word entries with exact keys up to 14 bytes, the
// second word stored after the claim, drop the verification reads of 8..14-byte chunks but were
// not faster: round 3 in k_classify, 2.32 -> 2.50 ms; round 5 in k_split_classify, C2 3.16 ->
// 3.21 ms, ENTROPY 14.0 -> 14.8 ms per step, r6o.)  u: the chunk's bytes as zero-padded LE words.
// ---------------------------------------------------------------------------------------
constexpr uint64_t kDdExact = 1ULL << 63;
struct DdOut {
  int kind;    // 0: merge on its own (no claim); 1: claimed entry `v`; 2: shares entry `v`'s result
  uint32_t v;
};

__device__ __forceinline__ DdOut dedupe_claim(const EncArgs& a, const SW_AS_GLOBAL uint32_t* words, int64_t last_word, int64_t mis,
                                              int64_t start, int n, const uint32_t (&u)[kShort / 4]) {
  const int nw = (n + 3) >> 2;
  uint32_t h = 0x9E3779B9u ^ ((uint32_t)n << 24);
#pragma unroll
  for (int q = 0; q < kShort / 4; ++q) {
    if (!__ballot(q < nw)) break;  // (no lane has word q: the wave stops at its longest chunk)
    if (q < nw) {
      h = (h ^ u[q]) * 0x85EBCA77u;
      h ^= h >> 13;
    }
  }
  const uint32_t h2 = (h ^ (h >> 16)) * 0x7FEB352Du;
  const bool exact = n <= (int)a.dexact;
  const uint64_t lo7 = (uint64_t)u[0] | ((uint64_t)(u[1] & 0xFFFFFFu) << 32);
  const uint64_t tag = exact ? (lo7 | ((uint64_t)n << 56) | kDdExact)
                             : ((uint64_t)((h2 >> 6) & a.dfp_mask & 0x3FFFFFFu) << 37 | (uint64_t)n << 31);
  const uint64_t mine = exact ? tag : (tag | (uint64_t)start);
  const uint32_t grp = h & a.dmask & ~(kDdGroup - 1);
  for (int j = 0; j < (int)kDdGroup; ++j) {
    const uint32_t idx = grp | ((h2 + j) & (kDdGroup - 1));
    unsigned long long* p = (unsigned long long*)a.dtab + (size_t)kDdWords * idx;
    // an entry changes once (0 -> final), so a cached plain load is safe: a stale 0 only sends
    // this lane to the CAS, which returns the live value
    uint64_t cur = *p;
    if (cur == 0) {
      cur = atomicCAS(p, 0ULL, (unsigned long long)mine);
      if (cur == 0) return DdOut{1, idx};  // claimed: this chunk is merged and shared
    }
    if (exact) {
      if (cur == mine) return DdOut{2, idx};
      continue;
    }
    if ((cur & ~0x7FFFFFFFULL) != tag) continue;
    const int64_t other = (int64_t)(cur & 0x7FFFFFFFULL);
    // compare with the claimant's bytes in the input, realigned
    const int64_t g = other + mis, w0 = g >> 2;
    const uint32_t sh = (uint32_t)(g & 3);
    bool same = true;
    if ((((uintptr_t)words & 15) == 0) && ((g + n - 1) >> 4) <= ((last_word + 1) >> 2) - 1) {
      // 16-byte aligned loads: one memory request per 16-byte block the chunk touches (1-3),
      // not one per word; then the words from the chunk's first word on (selects, no
      // dynamically indexed registers)
      const uint4* q16 = (const uint4*)words;
      const int64_t b0 = g >> 4;
      const int span = (int)(g & 15) + n;
      const uint4 x0 = q16[b0];
      const uint4 x1 = span > 16 ? q16[b0 + 1] : make_uint4(0, 0, 0, 0);
      const uint4 x2 = span > 32 ? q16[b0 + 2] : make_uint4(0, 0, 0, 0);
      const uint32_t W[12] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w, x2.x, x2.y, x2.z, x2.w};
      const int k = (int)(w0 & 3);
      uint32_t R[kShort / 4 + 1];
#pragma unroll
      for (int i = 0; i <= kShort / 4; ++i) R[i] = k == 0 ? W[i] : k == 1 ? W[i + 1] : k == 2 ? W[i + 2] : W[i + 3];
#pragma unroll
      for (int q = 0; q < kShort / 4; ++q) {
        if (q < nw) {
          const int keep = n - 4 * q;
          const uint32_t x = __builtin_amdgcn_alignbyte(R[q + 1], R[q], sh);
          const uint32_t m = keep >= 4 ? ~0u : ((1u << (8 * keep)) - 1u);
          same = same && ((x & m) == u[q]);
        }
      }
    } else {  // (unaligned input, or the batch's last bytes): word by word
      uint32_t prev = words[min(w0, last_word)];
#pragma unroll
      for (int q = 0; q < kShort / 4; ++q) {
        if (q < nw) {
          const uint32_t next = words[min(w0 + q + 1, last_word)];
          const int keep = n - 4 * q;
          const uint32_t x = __builtin_amdgcn_alignbyte(next, prev, sh);
          const uint32_t m = keep >= 4 ? ~0u : ((1u << (8 * keep)) - 1u);
          same = same && ((x & m) == u[q]);
          prev = next;
        }
      }
    }
    if (!same) continue;
    return DdOut{2, idx};
  }
  return DdOut{0, 0};  // (the table's overflow: counted by k_scatter for grow_dedupe)
}

// ---------------------------------------------------------------------------------------
// k_classify: one WAVE per 2 KiB tile (4 tiles per workgroup, no block barriers).  A prose
// tile holds ~380 chunks, so chunks go 64 per round (chunk 64r + lane): coalesced slot stores,
// and the per-bucket queue counts come from wave ballots (no atomics).
static_assert(kTile <= 0x10000, "chunk starts are uint16");
// ---------------------------------------------------------------------------------------
// two rounds of table probes in flight per wave: 5.52 -> 5.46 ms per C2 launch (one round or
// three: 5.55 / 5.75 ms; four cap the kernel at 5 waves per SIMD)
constexpr int kLookRounds = 2;
constexpr int kQBuf = 64 * (kLookRounds + 1);        // dedupe buffer: one batch + a group of rounds
constexpr int kWinWords = kWin / 4 + 8;

// k_classify waits on memory most of the time: 6 waves per SIMD (80 VGPRs, 12 spilled bytes
// per lane) beat the compiler's 5 (81 VGPRs): 2.81 vs 3.05 ms (profiles/r2_e_ab.txt).  k_compact:
// capped at 6 it spilled 24 B per lane (+0.9 GB of writes, not faster); with its body as a
// function of (tile, base) (compact_tile) the compiler fits 78 VGPRs, 6 waves, no spill: 1.11 ->
// 0.95 ms (profiles/r2_k.md).
// Round 5: the chunk-start list capped at kClsCsCap (a tile with more goes to k_classify_big),
// so a block fits 7 per CU: 7 waves per SIMD (as k_split_classify, split_classify.h kScCsCap).
constexpr int kClsCsCap = 1456;
// (a last chunk that runs more than kShort bytes past its tile, end unknown to the tile: long,
// its length found from the complete bitmap by k_lp_prep)
constexpr int kRelEndLong = 1 << 30;
template <bool kSp>  // kSp: the launch has special-token occurrences (a.sp)
__device__ __forceinline__ void classify_chunks(const EncArgs& a, int64_t tile, const uint32_t* s_b32,
                                                uint16_t* s_cstart, uint16_t* s_qbuf, uint32_t myhalf, int rel_end,
                                                int64_t s_first, int64_t sp_lo, int64_t sp_hi, int cap = kTile + 1,
                                                unsigned int* ov_count = nullptr, int64_t* ov_tiles = nullptr);

// one tile (the body of k_classify's tile loop): the chunk starts from the uploaded bitmap
template <bool kSp>
__device__ __forceinline__ void classify_tile(const EncArgs& a, int64_t tile, uint32_t* s_b32, uint16_t* s_cstart,
                                              uint16_t* s_qbuf, int cap, unsigned int* ov_count, int64_t* ov_tiles) {
  const int lane = threadIdx.x & 63;
  const int64_t t0 = tile * kTile;
  const int64_t t1 = tile_end(t0, a.n_bytes);
  const int64_t w0 = t0 >> 6;

  // 1. stage the window's bytes (1-KiB coalesced 16-byte loads) and the bitmap words (in
  //    registers)
  if (((uintptr_t)a.bytes & 15) == 0 && t0 + kWin <= a.n_bytes) {
#pragma unroll
    for (int q = 0; q < (kWin / 16 + 63) / 64; ++q) {
      const int i = lane + 64 * q;
      if (i < kWin / 16) {
        const u32x4 x = SW_LDNT((const u32x4*)(a.bytes + t0 + 16 * (int64_t)i));
        *(uint4*)(s_b32 + 4 * i) = make_uint4(x[0], x[1], x[2], x[3]);
      }
    }
  } else {
    for (int i = lane; i < kWin / 4; i += 64) {
      const int64_t g = t0 + 4 * (int64_t)i;
      uint32_t v = 0;
      for (int k = 0; k < 4; ++k) v |= (g + k < a.n_bytes ? (uint32_t)a.bytes[g + k] : 0u) << (8 * k);
      s_b32[i] = v;
    }
  }
  if (lane < 8) s_b32[kWin / 4 + lane] = 0;
  const uint64_t bw = (lane < kTileWords && w0 + lane < a.n_words) ? SW_LDNT2(&a.bits[w0 + lane]) : 0ULL;
  const int64_t s_first = a.tile_slo[tile];  // (prefetched: used by step 6)
  const int64_t sp_lo = kSp ? a.sp.tile_sp[tile] : 0, sp_hi = kSp ? a.sp.tile_sp[tile + 1] : 0;  // (... by step 2)

  // 2. chunk starts in [t0, t1): lane l owns bits 32 l .. 32 l + 31 of the tile (half of bitmap
  //    word l / 2: all 64 lanes enumerate, half as many starts each as with a word per lane)
  static_assert(kTile == 64 * 32, "a tile's bits are 64 lanes x 32");
  uint32_t myhalf;
  {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)bw, lane >> 1, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(bw >> 32), lane >> 1, 64);
    myhalf = (lane & 1) ? hi : lo;
    const int64_t lim = t1 - (t0 + 32 * lane);  // bits at or beyond t1 belong to the next tile
    if (lim <= 0) myhalf = 0;
    else if (lim < 32) myhalf &= (1u << lim) - 1u;
  }
  // end of the last chunk, tile-relative: the first chunk start at or after t1 (staged halo
  // word first; a launch is < 2^31 bytes, so tile-relative positions fit an int)
  int64_t last_end = a.n_bytes;
  {
    uint64_t hw = 0;
    const int64_t bit0 = t0 + 64 * (int64_t)lane;
    if (lane < kTileWords && bit0 + 64 > t1) {
      hw = bw;
      if (bit0 < t1) hw &= ~0ULL << (t1 - bit0);
    }
    const uint64_t has = __ballot(hw != 0);
    if (has) {
      const int src = __ffsll((long long)has) - 1;
      const int64_t q = t0 + 64 * (int64_t)src + __ffsll((long long)__shfl(hw, src, 64)) - 1;
      last_end = min(q, a.n_bytes);
    } else if (__ballot(myhalf != 0)) {
      // (a chunk running past the halo)
      const int64_t q = next_set_bit(a.bits, a.n_words, t0 + 64 * kTileWords, a.n_bytes);
      last_end = min(q, a.n_bytes);
    }
  }
  classify_chunks<kSp>(a, tile, s_b32, s_cstart, s_qbuf, myhalf, (int)(last_end - t0), s_first, sp_lo, sp_hi, cap,
                       ov_count, ov_tiles);
}

// The tile's chunks from its chunk-start bits on: lane l holds bits 32 l .. 32 l + 31 of the tile
// (cut at the tile's end), rel_end is the end of the tile's last chunk relative to t0 (or
// kRelEndLong), s_b32 the tile's bytes from t0 in LDS (with kWin - kTile bytes of halo).
template <bool kSp>
__device__ __forceinline__ void classify_chunks(const EncArgs& a, int64_t tile, const uint32_t* s_b32,
                                                uint16_t* s_cstart, uint16_t* s_qbuf, uint32_t myhalf, int rel_end,
                                                int64_t s_first, int64_t sp_lo, int64_t sp_hi, int cap,
                                                unsigned int* ov_count, int64_t* ov_tiles) {
  SW_STAMP_INIT;
  const int lane = threadIdx.x & 63;
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  const int64_t t0 = tile * kTile;
  const int64_t t1 = tile_end(t0, a.n_bytes);
  const uint32_t cnt = (uint32_t)__popc(myhalf);
  const uint32_t incl = wave_incl_scan(cnt, lane);
  const int C = (int)lane_value(incl, 63);
  if (C > cap) {  // (more chunk starts than the LDS list holds: nothing is written; k_classify_big does it)
    if (lane == 0) ov_tiles[atomicAdd(ov_count, 1u)] = tile;
    return;
  }
  {
    uint32_t x = myhalf;
    uint32_t k = incl - cnt;
    while (x) {
      s_cstart[k++] = (uint16_t)(32 * lane + __ffs(x) - 1);
      x &= x - 1;
    }
  }
  wave_sync_mem();
  if (kSp) {  // the special-token occurrences starting in the tile (each one whole chunk): their
              // slots get the specials' ids, their chunks the flag the lookups skip -- once per tile
    // (sp_lo, sp_hi: tile_sp[tile], tile_sp[tile + 1] -- loaded by k_classify at its start, here
    // for k_split_classify (-1))
    if (sp_lo < 0) {
      sp_lo = a.sp.tile_sp[tile];
      sp_hi = a.sp.tile_sp[tile + 1];
    }
    for (int64_t j = sp_lo + lane; j < sp_hi; j += 64) {
      const int p = (int)(a.sp.pos[j] - t0);
      int lo = 0, hi = C;  // (its chunk: the first whose start is >= p, and it starts at p)
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if ((int)(s_cstart[m] & kCsPos) < p) lo = m + 1; else hi = m;
      }
      if (lo < C && (int)s_cstart[lo] == p) {
        s_cstart[lo] = (uint16_t)(p | kCsSpecial);
        SW_STNT(&a.scratch[t0 + lo], (int32_t)a.sp.id[j]);
      }
    }
    wave_sync_mem();
  }
  SW_STAMP(0);

  // 3. settle single bytes and whole-chunk-table hits (their slots written here).  The rest
  //    collect in a small per-wave buffer and are deduped 64 at a time (full waves): repeats
  //    point their slot at the first occurrence's result, the others are queued for the merge
  //    kernels and counted per length bucket (lane b: bucket b).
  int32_t* dst = a.scratch + t0;
  const int rounds = (C + 63) >> 6;
#ifdef SW_DIAG_NO_LOOKUP  // (diagnostic, wrong ids: every multi-byte chunk "hits" token 0, no memory access)
  const bool use_table = false;
#else
  const bool use_table = a.chunks.enabled != 0;
#endif
  const int64_t mis = (int64_t)((uintptr_t)a.bytes & 3);
  const SW_AS_GLOBAL uint32_t* gwords = (const SW_AS_GLOBAL uint32_t*)((uintptr_t)a.bytes - mis);
  const int64_t last_word = (mis + a.n_bytes - 1) >> 2;
  uint32_t bcount = 0;
  int nq = 0;    // wave-uniform: chunks waiting in s_qbuf
  int nown = 0;  // wave-uniform: chunks queued for the merge kernels
  int nref = 0;  // wave-uniform: slots that refer to a merge result (k_tile_count's list)
  // kLookRounds rounds of lookups are issued together (independent chains, one wait)
  for (int r0 = 0; r0 < rounds || nq > 0; r0 += kLookRounds) {
    if (r0 < rounds) {
      uint32_t tok[kLookRounds];
      if (use_table) {
        table_lookups<kLookRounds, kSp>(a.chunks, s_b32, s_cstart, C, rel_end, r0, lane, tok);
      } else {
#pragma unroll
        for (int u = 0; u < kLookRounds; ++u) {  // (no table: single bytes only)
          const int k = ((r0 + u) << 6) + lane;
          const bool valid = k < C;
          const uint32_t cs = valid ? s_cstart[k] : 0u;
          const int ls = (int)(cs & kCsPos);
          const int end = (k + 1 < C) ? (int)(s_cstart[k + 1] & kCsPos) : rel_end;
          tok[u] = (kSp && (cs & kCsSpecial)) ? kSpDone
                   : (valid && end - ls == 1) ? (s_b32[ls >> 2] >> (8 * (ls & 3))) & 0xFFu
#ifdef SW_DIAG_NO_LOOKUP
                   : (valid && end - ls <= kShort) ? 0u
#endif
                   : kInf;
        }
      }
#pragma unroll
      for (int u = 0; u < kLookRounds; ++u) {
        const int k = ((r0 + u) << 6) + lane;
        const bool valid = k < C;
        const bool queued = valid && tok[u] == kInf;
        if (valid && !queued && (!kSp || tok[u] != kSpDone)) SW_STNT(&dst[k], (int32_t)tok[u]);
        const uint64_t mq = __ballot(queued);
        if (queued) s_qbuf[nq + __popcll(mq & lt_mask)] = (uint16_t)k;
        nq += __popcll(mq);
      }
    }
    // dedupe full batches of 64 queued chunks (and, after the last round, the remainder)
    while (nq >= 64 || (r0 + kLookRounds >= rounds && nq > 0)) {
      wave_sync_mem();
      SW_STAMP(1);
      const bool act = lane < nq;
      const int k = act ? s_qbuf[lane] : 0;
      uint16_t rest[kQBuf / 64 - 1];
#pragma unroll
      for (int q = 1; q < kQBuf / 64; ++q) rest[q - 1] = (64 * q + lane < nq) ? s_qbuf[64 * q + lane] : 0;
#pragma unroll
      for (int q = 1; q < kQBuf / 64; ++q)
        if (64 * q + lane < nq) s_qbuf[64 * (q - 1) + lane] = rest[q - 1];
      nq = nq > 64 ? nq - 64 : 0;
      const int ls = act ? (int)(s_cstart[k] & kCsPos) : 0;
      const int end = (k + 1 < C) ? (int)(s_cstart[k + 1] & kCsPos) : rel_end;
      const int len = act ? end - ls : 0;
      DdOut dd{0, 0};
      if (act && a.dedupe && len <= kShort) {
        uint32_t u[kShort / 4];
        window_words(s_b32, ls, min(len, 16), *(uint32_t(*)[4])u);
        if (len > 16) window_words(s_b32, ls + 16, len - 16, *(uint32_t(*)[4])(u + 4));
        else
#pragma unroll
          for (int q = 4; q < kShort / 4; ++q) u[q] = 0;
        dd = dedupe_claim(a, gwords, last_word, mis, t0 + ls, len, u);
      }
      const uint32_t did = dd.kind ? dd.v : kNoDid;
      if (act) {
        const int64_t own = t0 + ls;
        dst[k] = dd.kind ? slot_dref(did) : slot_ref(own);
        SW_STNT2(&a.rlist[t0 + nref + lane], dd.kind ? (kRlDense | did) : (uint32_t)own);  // (act lanes are 0 .. n-1: coalesced)
      }
      nref += (int)__popcll(__ballot(act));
      // chunks over kShort bytes go to the long list (the long-chunk passes start from it right
      // after this kernel, beside the scan, the scatter and the merge kernels); the rest to the
      // tile-local queue
      const bool longc = act && len > kShort;
      const uint64_t lm = __ballot(longc);
      if (lm) {
        unsigned long long lb = 0;
        if (lane == 0) lb = atomicAdd(a.l_count, (unsigned long long)__popcll(lm));
        lb = lane_value64(lb, 0);
        if (longc)
          a.llist[lb + __popcll(lm & lt_mask)] =
              ((uint64_t)(t0 + ls) << 32) | (len < (int)kNoDid ? (uint32_t)len : kNoDid);
      }
      const bool queued = act && dd.kind != 2 && !longc;
      const int b = queued ? bucket_of(len) : 15;
      uint64_t pend = __ballot(queued);
      // tile-local queue entry (any order; k_scatter routes by length): chunk start in tile
      // (kTileBits) | chunk index (kTileBits) | length (6 bits, 0 = long); its dense result
      // (or kNoDid) kTile / 2 entries on (a tile queues at most kTile / 2 chunks of >= 2 bytes)
      if (queued) {
        const int64_t qi = t0 + nown + __popcll(pend & lt_mask);
        SW_STNT2(&a.qtmp[qi], (uint32_t)ls | ((uint32_t)k << kTileBits) | ((uint32_t)len << (2 * kTileBits)));
        SW_STNT2(&a.qtmp[qi + kTile / 2], did);
      }
      nown += __popcll(pend);
      while (pend) {  // one ballot per bucket present
        const int bb = (int)lane_value((uint32_t)b, __ffsll((long long)pend) - 1);
        const uint64_t m = __ballot(b == bb);
        if (lane == bb) bcount += (uint32_t)__popcll(m);
        pend &= ~m;
      }
      wave_sync_mem();
      SW_STAMP(7);
    }
  }
  SW_STAMP(1);

  // 4. per-bucket counts of the queued chunks (k_scan -> k_scatter)
  if (lane < kNumBuckets) a.bcnt[(int64_t)lane * a.n_tiles + tile] = bcount;
  if (lane == 0) {
    a.tile_slots[tile] = (uint32_t)C;
    a.tile_nref[tile] = (uint32_t)nref;
  }
  SW_STAMP(2);

  // 6. strings starting in this tile: chunk (= slot) index within the tile (k_compact converts)
  //    (the first one read here, not held in a register through the tile: with a scalar tile index
  //    this is a scalar load)
  (void)s_first;
  const int64_t s_first_now = a.tile_slo[tile];
  for (int64_t s = s_first_now + lane; s < a.n_str; s += 64) {
    const int64_t p = a.str_off[s];
    if (p >= t1) break;
    int lo = 0, hi = C;  // first chunk with start >= p
    const int lp = (int)(p - t0);
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if ((int)(s_cstart[m] & kCsPos) < lp) lo = m + 1; else hi = m;
    }
    a.out_off[s] = (int64_t)lo;
  }
  SW_STAMP(3);
  wave_sync_mem();  // (the next tile reuses the wave's LDS)
}

// one wave per tile
template <bool kSp>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(7, 7))) k_classify(EncArgs a, unsigned int* ov_count, int64_t* ov_tiles) {
  __shared__ __attribute__((aligned(16))) uint32_t s_b32_all[kWaves][kWinWords];  // window bytes (+ zero tail)
  __shared__ uint16_t s_cs_all[kWaves][kClsCsCap + 1];  // chunk starts (tile-relative), up to kClsCsCap
  __shared__ uint16_t s_qb_all[kWaves][kQBuf];       // chunks not settled by a lookup, to dedupe
  const int wv = wave_in_block_s();
  const int64_t tile = (int64_t)blockIdx.x * kWaves + wv;
  if (tile < a.n_tiles)
    classify_tile<kSp>(a, tile, s_b32_all[wv], s_cs_all[wv], s_qb_all[wv], kClsCsCap, ov_count, ov_tiles);
}

// the tiles k_classify could not hold (more than kClsCsCap chunks), one wave each with the whole
// list in LDS, the waves of a fixed grid taking them in turn
template <bool kSp>
__global__ void __launch_bounds__(kThreads) k_classify_big(EncArgs a, const unsigned int* ov_count, const int64_t* ov_tiles) {
  __shared__ __attribute__((aligned(16))) uint32_t s_b32_all[kWaves][kWinWords];
  __shared__ uint16_t s_cs_all[kWaves][kTile + 1];
  __shared__ uint16_t s_qb_all[kWaves][kQBuf];
  const int wv = wave_in_block_s();
  // (this launch's list, written by k_classify: read coherently, never through the scalar cache)
  const int64_t n = (int64_t)__hip_atomic_load(ov_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int64_t i = (int64_t)blockIdx.x * kWaves + wv; i < n; i += (int64_t)gridDim.x * kWaves) {
    const int64_t tile = __hip_atomic_load(&ov_tiles[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    classify_tile<kSp>(a, tile, s_b32_all[wv], s_cs_all[wv], s_qb_all[wv], kTile + 1, nullptr, nullptr);
  }
}

// ---------------------------------------------------------------------------------------
// k_scatter: tile-local queue entries -> the dense bucket-major queue
// ---------------------------------------------------------------------------------------
// one round of k_scatter's routing: lanes with act hold a tile-local entry (e, did); lanes of a
// group of kG lanes serve one tile, whose lane b < kNumBuckets holds bucket b's next destination
// (dst); one ballot per bucket present in each group, the groups side by side
template <int kG>
__device__ __forceinline__ void scatter_round(const EncArgs& a, int64_t t0, bool act, uint32_t e, uint32_t did,
                                              int64_t& dst) {
  const int lane = threadIdx.x & 63, g = lane / kG;
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  const uint64_t gmask = (kG == 64 ? ~0ULL : ((1ULL << kG) - 1ULL)) << (kG * g);
  const uint32_t ns = e >> (2 * kTileBits);
  const int b = act ? (ns ? bucket_of(ns) : kLongBucket) : 15;
  if (a.dedupe) {  // (a dedupable chunk queued without an entry: its table line was full, see grow_dedupe)
    const uint64_t full = __ballot(act && ns != 0 && did == kNoDid);
    if (full && lane == 0) atomicAdd(a.dd_full, (unsigned long long)__popcll(full));
  }
  int64_t d = 0;
  uint64_t pend = __ballot(act);
  while (pend) {
    const uint64_t pg = pend & gmask;  // (this lane's group: its first pending lane's bucket)
    const int bb = pg ? __shfl(b, __ffsll((long long)pg) - 1, 64) : -1;
    const bool mine = act && b == bb && ((pend >> lane) & 1);
    const uint64_t m = __ballot(mine);
    const int64_t db = __shfl(dst, kG * g + (bb < 0 ? 0 : bb), 64);
    if (mine) d = db + __popcll(m & gmask & lt_mask);
    if (lane - kG * g == bb) dst += __popcll(m & gmask);
    pend &= ~m;
  }
  if (act) {
    const uint64_t start = (uint64_t)(t0 + (e & (kTile - 1)));
    a.queue[d] = (start << 33) | ((uint64_t)ns << 27) | did;
  }
}

__global__ void __launch_bounds__(kThreads) k_scatter(EncArgs a) {
  // four tiles per wave, their bucket counts in one load: a tile that queued <= 16 chunks (C2: ~1.4
  // on average; a wave per tile spent its life on two dependent loads) is routed by its 16-lane
  // group, the four side by side; a larger tile (every chunk queued: the memo-off runs) by the
  // whole wave, 64 entries a round, after them
  constexpr int kG = 16;
  const int lane = threadIdx.x & 63, g = lane >> 4, gl = lane & (kG - 1);
  const int64_t tb = ((int64_t)blockIdx.x * kWaves + wave_in_block()) * (64 / kG);
  const int64_t t = tb + g;
  const bool tile_ok = t < a.n_tiles;
  uint32_t c = 0;
  int64_t dst = 0;
  if (tile_ok && gl < kNumBuckets) {
    c = a.bcnt[(int64_t)gl * a.n_tiles + t];
    dst = a.boff[(int64_t)gl * a.n_tiles + t];
  }
  uint32_t n = c;
#pragma unroll
  for (int off = 1; off < kG; off <<= 1) n += __shfl_xor(n, off, 64);  // (the group's total, in every lane of it)
  {  // the small tiles, side by side
    const bool act = tile_ok && n <= (uint32_t)kG && (uint32_t)gl < n;
    const uint32_t e = act ? SW_LDNT2(&a.qtmp[t * kTile + gl]) : 0u;
    const uint32_t did = act ? SW_LDNT2(&a.qtmp[t * kTile + kTile / 2 + gl]) : kNoDid;
    scatter_round<kG>(a, t * kTile, act, e, did, dst);
  }
  for (int q = 0; q < 64 / kG; ++q) {  // the large ones, one by one (wave-uniform)
    const uint32_t nq = (uint32_t)__shfl((int)n, kG * q, 64);
    if (nq <= (uint32_t)kG) continue;
    const int64_t tq = tb + q, tq0 = tq * kTile;
    int64_t dq = __shfl(dst, kG * q + (lane < kNumBuckets ? lane : 0), 64);  // (lane b: bucket b)
    for (uint32_t i0 = 0; i0 < nq; i0 += 64) {
      const uint32_t i = i0 + lane;
      const bool act = i < nq;
      const uint32_t e = act ? SW_LDNT2(&a.qtmp[tq0 + i]) : 0u;
      const uint32_t did = act ? SW_LDNT2(&a.qtmp[tq0 + kTile / 2 + i]) : kNoDid;
      scatter_round<64>(a, tq0, act, e, did, dq);
    }
  }
}

// [lo, hi) of the dense queue holding buckets b_lo..b_hi
__device__ __forceinline__ void bucket_range(const EncArgs& a, int b_lo, int b_hi, int64_t* lo, int64_t* hi) {
  *lo = a.boff[(int64_t)b_lo * a.n_tiles];
  *hi = (b_hi + 1 < kNumBuckets) ? a.boff[(int64_t)(b_hi + 1) * a.n_tiles] : *a.q_total;
}

// long chunks listed by k_lp_prep (clamped to the list's capacity)
__device__ __forceinline__ int64_t long_count(const EncArgs& a) {
  const int64_t v = *a.n_long;
  return v < a.lcap ? (v < 0 ? 0 : v) : a.lcap;
}

// the chunk bytes [g, g + n) of the word-aligned input as N/4 zero-padded LE words
template <int N>
__device__ __forceinline__ void chunk_words(const SW_AS_GLOBAL uint32_t* words, int64_t last_word, int64_t g, int n,
                                            uint32_t (&u)[N / 4]) {
  constexpr int W = N / 4 + 1;  // aligned words covering any N-byte span
  const int64_t w0 = g >> 2;
  uint32_t w[W];
#pragma unroll
  for (int k = 0; k < W; ++k) w[k] = words[min(w0 + k, last_word)];
  const uint32_t sh = (uint32_t)(g & 3);
#pragma unroll
  for (int q = 0; q < N / 4; ++q) {
    const uint32_t x = __builtin_amdgcn_alignbyte(w[q + 1], w[q], sh);
    const int keep = n - 4 * q;
    u[q] = keep >= 4 ? x : keep <= 0 ? 0u : (x & ((1u << (8 * keep)) - 1u));
  }
}

// merge loop for the queue entry e of this lane (act); result at res[2 * start ..)
// (kLds: the well-formed 16-bit loop with the ids in LDS, lane_merge_lds_wf; s_id: the wave's ids)
// (u: the chunk's bytes, chunk_words<N> of the entry -- loaded by the caller, a batch ahead)
template <bool kWide, bool k16, int N, bool kWF>
__device__ __forceinline__ void merge_entry(const EncArgs& a, const uint32_t (&u)[N / 4], uint64_t e, bool act,
                                            uint32_t* s_id) {
  constexpr bool kLds = kWF && k16 && !kWide;
  const int64_t start = (int64_t)(e >> 33);
  const int n = act ? (int)((e >> 27) & 63u) : 0;
  const uint32_t did = (uint32_t)e & kNoDid;
  const int lane = threadIdx.x & 63;
  uint32_t id[kLds ? 1 : N];
  uint32_t alive;
  if constexpr (kLds) {
    alive = lane_merge_lds_wf<kWide, N>(a.table, u, n, s_id, lane);
  } else {
#pragma unroll
    for (int q = 0; q < N / 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) id[4 * q + r] = (u[q] >> (8 * r)) & 0xFFu;
    alive = lane_merge_reg<kWide, k16, N, kWF>(a.table, id, n);
  }
  if (!act) return;
  uint32_t* dst = a.res + 2 * start;
  int m = 0;
  // the dense result head (the first 7 ids as 16 bits, or 3 as 32 bits; see dres)
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
  if constexpr (kLds) {
    for (uint32_t al = alive; al; al &= al - 1) {
      const uint32_t x = s_id[64 * (__ffs(al) - 1) + lane];
      dst[1 + m] = x;
      h0 |= m == 0 ? x << 16 : 0u;
      h1 |= m == 1 ? x : m == 2 ? x << 16 : 0u;
      h2 |= m == 3 ? x : m == 4 ? x << 16 : 0u;
      h3 |= m == 5 ? x : m == 6 ? x << 16 : 0u;
      ++m;
    }
  } else {
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if ((alive >> k) & 1u) {
      dst[1 + m] = id[k];
      if (k16) {
        h0 |= m == 0 ? id[k] << 16 : 0u;
        h1 |= m == 1 ? id[k] : m == 2 ? id[k] << 16 : 0u;
        h2 |= m == 3 ? id[k] : m == 4 ? id[k] << 16 : 0u;
        h3 |= m == 5 ? id[k] : m == 6 ? id[k] << 16 : 0u;
      } else {
        h1 = m == 0 ? id[k] : h1;
        h2 = m == 1 ? id[k] : h2;
        h3 = m == 2 ? id[k] : h3;
      }
      ++m;
    }
  }
  }
  dst[0] = (uint32_t)m;
  if (did != kNoDid) {
    if (k16) a.dres[did] = make_uint4((uint32_t)m | h0, m <= 7 ? h1 : (uint32_t)start, h2, h3);
    else a.dres[did] = make_uint4((uint32_t)m, h1, h2, m <= 3 ? h3 : (uint32_t)start);
    a.dcnt[did] = (uint8_t)m;
  }
}

// the result of a chunk merged by lane_merge_lds_wf2 (ids in LDS at s_q[64 k + lane], k in alive)
// to res and, when it is shared, its dense head -- merge_entry's kLds branch
__device__ __forceinline__ void put_lds_result(const EncArgs& a, uint64_t e, uint32_t alive, const uint32_t* s_q,
                                               int lane) {
  const int64_t start = (int64_t)(e >> 33);
  const uint32_t did = (uint32_t)e & kNoDid;
  uint32_t* dst = a.res + 2 * start;
  int m = 0;
  uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
  for (uint32_t al = alive; al; al &= al - 1) {
    const uint32_t x = s_q[64 * (__ffs(al) - 1) + lane];
    dst[1 + m] = x;
    h0 |= m == 0 ? x << 16 : 0u;
    h1 |= m == 1 ? x : m == 2 ? x << 16 : 0u;
    h2 |= m == 3 ? x : m == 4 ? x << 16 : 0u;
    h3 |= m == 5 ? x : m == 6 ? x << 16 : 0u;
    ++m;
  }
  dst[0] = (uint32_t)m;
  if (did != kNoDid) {
    a.dres[did] = make_uint4((uint32_t)m | h0, m <= 7 ? h1 : (uint32_t)start, h2, h3);
    a.dcnt[did] = (uint8_t)m;
  }
}

// ---------------------------------------------------------------------------------------
// k_merge_bucket<N>: queued chunks of buckets [b_lo, b_hi] (length <= N), one per lane;
// persistent grid-stride over 64-entry batches of the bucket-major queue
// ---------------------------------------------------------------------------------------
// (capping the short buckets at 5, 6 or 8 waves per SIMD -- 64-96 VGPRs, some spilled -- was
// slower on memo-off: 18.7 -> 19.2-20.5 ms, r7x)
template <bool kWide, bool k16, int N, bool kWF = false>  // kWF: a well-formed table (lane_merge_lds_wf)
__global__ void __launch_bounds__(kThreads) k_merge_bucket(EncArgs a, int b_lo, int b_hi) {
  SW_STAMP_INIT;
  const int64_t gw = ((int64_t)blockIdx.x * kWaves + wave_in_block());  // global wave id
  const int64_t n_waves = ((int64_t)gridDim.x * kThreads) >> 6;
  const int lane = threadIdx.x & 63;
  int64_t lo, hi;
  bucket_range(a, b_lo, b_hi, &lo, &hi);
  const int64_t mis = (int64_t)((uintptr_t)a.bytes & 3);
  const SW_AS_GLOBAL uint32_t* words = (const SW_AS_GLOBAL uint32_t*)((uintptr_t)a.bytes - mis);
  const int64_t last_word = (mis + a.n_bytes - 1) >> 2;  // last word holding input bytes
  constexpr bool kLds = kWF && k16 && !kWide;
  // two or four chunks per lane (lane_merge_lds_wfq) for the short buckets of well-formed 16-bit tables
  constexpr int kPer = !kLds ? 1 : N <= kQuadMaxN ? 4 : N <= kPairMaxN ? 2 : 1;
  __shared__ uint32_t s_ids[kLds ? kWaves * 64 * N * kPer : 1];  // (lane_merge_lds_wf: the waves' ids)
  uint32_t* s_id = s_ids + (kLds ? wave_in_block() * 64 * N * kPer : 0);
  if constexpr (kPer > 1) {  // batches of 64 kPer entries per wave: entries base + 64 q + lane
    constexpr int kB = 64 * kPer;
    int64_t i = lo + gw * kB + lane;
    uint64_t e[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) e[q] = i + 64 * q < hi ? a.queue[i + 64 * q] : 0;
    for (int64_t base = lo + gw * kB; base < hi; base += n_waves * kB) {
      uint32_t u[kPer][N / 4];
      int n[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) {
        n[q] = i + 64 * q < hi ? (int)((e[q] >> 27) & 63u) : 0;
        chunk_words<N>(words, last_word, (int64_t)(e[q] >> 33) + mis, n[q], u[q]);
      }
      const int64_t i2 = i + n_waves * kB;
      uint64_t f[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) f[q] = i2 + 64 * q < hi ? a.queue[i2 + 64 * q] : 0;
      uint32_t alive[kPer];
      lane_merge_lds_wfq<kWide, N, kPer>(a.table, u, n, s_id, lane, alive);
#pragma unroll
      for (int q = 0; q < kPer; ++q)
        if (i + 64 * q < hi) put_lds_result(a, e[q], alive[q], s_id + 64 * N * q, lane);
      i = i2;
#pragma unroll
      for (int q = 0; q < kPer; ++q) e[q] = f[q];
    }
    return;
  }
  // software-pipelined: the next batch's queue entry and chunk bytes load before this batch's
  // merge loop runs (two dependent round trips per batch off the critical path)
  int64_t i = lo + gw * 64 + lane;
  uint64_t e = i < hi ? a.queue[i] : 0;
  for (int64_t base = lo + gw * 64; base < hi; base += n_waves * 64) {
    uint32_t u[N / 4];
    chunk_words<N>(words, last_word, (int64_t)(e >> 33) + mis, i < hi ? (int)((e >> 27) & 63u) : 0, u);
    const int64_t i2 = i + n_waves * 64;
    const uint64_t e2 = i2 < hi ? a.queue[i2] : 0;
    merge_entry<kWide, k16, N, kWF>(a, u, e, i < hi, s_id);
    i = i2;
    e = e2;
  }
#ifdef SW_STAMPS
  SW_STAMP(N >= 16 ? 5 : 4);
#endif
}

// long chunks (> kShort bytes): one wave each, wave-cooperative loop.  Chunks up to kLongLds
// bytes keep their ids and ranks in LDS (one 64-thread workgroup = one wave per chunk); longer
// ones work in the global work area (res, position space).
constexpr int kLongLds = 4096;

// ---------------------------------------------------------------------------------------
// Exact merge loop for one chunk of up to kLongLds bytes, one wave, without compaction: lane j
// owns the S positions [S j, S j + S), S = ceil(n / 64) (so every lane has work however short
// the chunk), and keeps in registers their ALIVE mask (merged-away positions die; "adjacent"
// means the next alive position), the smallest (rank, position) key of its pairs and the mask
// of the positions holding that rank.  Per step of the reference loop (base.py:10-36):
//   - the global minimum key is one wave min: the lowest rank, first occurrence (the pair of
//     the earliest position with that rank, as min() over the first-occurrence-ordered stats);
//   - its occurrences can only sit at positions of lanes whose minimum rank is that rank, in
//     their min-rank masks (a pair's rank is its value; ill-formed tables may give two pairs
//     one value, so the ids are compared too);
//   - all occurrences are replaced, left to right, non-overlapping: for (a, b) with a != b
//     occurrences cannot overlap; for (a, a) the runs are resolved in position order, lane
//     after lane;
//   - the right partners die, and only the ranks of the new tokens and of their alive
//     predecessors are looked up again (eight lookups in flight per lane); only the lanes whose
//     positions changed recompute their minimum.
// So a step costs a few wave-wide operations plus the changed segments, not two passes over
// the whole chunk.  Position p = S j + k lives in LDS at k * 64 + j: a wave's reads of "position
// k of every lane" hit 64 distinct banks.  The chunk's bytes are read from src.  Returns the
// surviving count; their ids are written to out.
// ---------------------------------------------------------------------------------------
template <bool kWide, typename T>  // T: uint16_t when every id and value fits 16 bits (half the LDS)
__device__ int seg_merge(const DevTable& t, const uint8_t* src, T* id, T* rk, uint64_t* s_kill, uint64_t* s_dirty,
                         int n, int lane, uint32_t* out) {
  const int S = n <= 64 ? 1 : (n + 63) >> 6;  // segment length (<= 64: n <= kLongLds)
  const int base = lane * S;
  auto own = [&](int k) -> int { return k * 64 + lane; };   // LDS index of my position base + k
  auto at = [&](int p) -> int {                              // LDS index of any position p
    if (p >= base && p < base + S) return own(p - base);
    const int j = p / S;
    return (p - j * S) * 64 + j;
  };
  auto rank_own = [&](int k) -> uint32_t {  // (16-bit storage: 0xFFFF is +inf)
    const uint32_t r = rk[own(k)];
    return (sizeof(T) == 2 && r == 0xFFFFu) ? kInf : r;
  };
  uint64_t am;
  {
    const int c = min(n - base, S);
    am = c >= 64 ? ~0ULL : c <= 0 ? 0ULL : ((1ULL << c) - 1ULL);
  }
  for (int k = 0; k < S; ++k)
    if (base + k < n) id[own(k)] = (T)src[base + k];
  s_kill[lane] = 0;
  s_dirty[lane] = 0;
  wave_sync_mem();
  // exclusive scans over the lanes: first alive position after my segment (n: none), last
  // alive position before it (-1: none)
  int nxt_after = n, prv_before = -1;
  auto scans = [&]() {
    int f = am ? base + __builtin_ctzll(am) : n;
    int l = am ? base + 63 - __builtin_clzll(am) : -1;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int fy = __shfl_down(f, off, 64);
      const int ly = __shfl_up(l, off, 64);
      if (lane + off < 64) f = min(f, fy);
      if (lane >= off) l = max(l, ly);
    }
    nxt_after = __shfl_down(f, 1, 64);
    if (lane == 63) nxt_after = n;
    prv_before = __shfl_up(l, 1, 64);
    if (lane == 0) prv_before = -1;
  };
  auto next_of = [&](int k) -> int {  // next alive position after base + k (mine)
    const uint64_t m = k == 63 ? 0ULL : (am & (~0ULL << (k + 1)));
    return m ? base + __builtin_ctzll(m) : nxt_after;
  };
  auto prev_of = [&](int k) -> int {  // last alive position before base + k (mine)
    const uint64_t m = am & ((1ULL << k) - 1ULL);
    return m ? base + 63 - __builtin_clzll(m) : prv_before;
  };
  uint64_t smin = ~0ULL, mmask = 0;  // my minimum key (rank << 32 | position), its positions
  auto seg_min = [&]() {  // (16 entries read at a time, independent loads: one LDS wait per 16)
    smin = ~0ULL;
    mmask = 0;
#pragma unroll 1
    for (int k0 = 0; k0 < S; k0 += 16) {
      uint32_t rr[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) rr[u] = rank_own(k0 + u);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int k = k0 + u;
        const uint32_t r = ((am >> k) & 1ULL) ? rr[u] : kInf;
        const uint32_t cur = (uint32_t)(smin >> 32);
        if (r < cur) {
          smin = ((uint64_t)r << 32) | (uint32_t)(base + k);
          mmask = 1ULL << k;
        } else if (r == cur) {
          mmask |= 1ULL << k;
        }
      }
    }
    if ((uint32_t)(smin >> 32) == kInf) mmask = 0;
  };
  scans();
  // initial ranks: every pair (p, p + 1), eight lookups in flight per lane
  for (int k0 = 0; k0 < S; k0 += 8) {
    uint32_t r[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u, p = base + k;
      const int nx = k + 1 < S ? own(k + 1) : lane + 1;  // (the next segment's first position)
      r[u] = (k < S && p + 1 < n) ? lookup<kWide>(t, id[own(k)], id[nx]) : kInf;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k0 + u < S && base + k0 + u < n) rk[own(k0 + u)] = (T)r[u];
  }
  seg_min();
  wave_sync_mem();
  while (true) {
    const uint64_t key = wave_min_u64(smin);
    const uint32_t r = (uint32_t)(key >> 32);
    if (r == kInf) break;
    const int pm = (int)(uint32_t)key;
    // the pair at pm (lane pm / S owns it)
    const int lm = pm / S, km = pm - lm * S;
    const uint64_t am_m = __shfl(am, lm, 64);
    const int na_m = __shfl(nxt_after, lm, 64);
    const uint64_t mq = km == 63 ? 0ULL : (am_m & (~0ULL << (km + 1)));
    const int qm = mq ? lm * S + __builtin_ctzll(mq) : na_m;
    const uint32_t p0 = id[km * 64 + lm], p1 = id[at(qm)];
    // my occurrences of (p0, p1): among my min-rank positions
    uint64_t take = 0;
    if ((uint32_t)(smin >> 32) == r) {
      for (uint64_t m = mmask; m; m &= m - 1) {
        const int k = __builtin_ctzll(m);
        if ((uint32_t)id[own(k)] == p0 && (uint32_t)id[at(next_of(k))] == p1) take |= 1ULL << k;
      }
    }
    if (p0 == p1) {  // runs of (a, a): left to right, a taken position consumes its next
      uint64_t lanes = __ballot(take != 0);
      int consumed = -1;
      uint64_t tk = 0;
      while (lanes) {
        const int L = __builtin_ctzll(lanes);
        lanes &= lanes - 1;
        if (lane == L) {
          for (uint64_t m = take; m; m &= m - 1) {
            const int k = __builtin_ctzll(m);
            if (base + k != consumed) {
              tk |= 1ULL << k;
              consumed = next_of(k);
            }
          }
        }
        consumed = __shfl(consumed, L, 64);
      }
      take = tk;
    }
    // new ids; the right partners die (a partner in a later segment is that segment's first
    // alive position: its bit goes through LDS)
    uint64_t kill = 0;
    for (uint64_t m = take; m; m &= m - 1) {
      const int k = __builtin_ctzll(m);
      id[own(k)] = (T)r;
      const int nc = next_of(k);
      if (nc < base + S) {
        kill |= 1ULL << (nc - base);
      } else {
        const int j = nc / S;
        __hip_atomic_fetch_or(&s_kill[j], 1ULL << (nc - j * S), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    wave_sync_mem();
    kill |= s_kill[lane];
    am &= ~kill;
    s_kill[lane] = 0;
    scans();
    // ranks to look up again: every new token and its alive predecessor
    uint64_t dirty = take;
    for (uint64_t m = take; m; m &= m - 1) {
      const int pv = prev_of(__builtin_ctzll(m));
      if (pv < 0) continue;
      if (pv >= base) {
        dirty |= 1ULL << (pv - base);
      } else {
        const int j = pv / S;
        __hip_atomic_fetch_or(&s_dirty[j], 1ULL << (pv - j * S), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    wave_sync_mem();
    dirty |= s_dirty[lane];
    s_dirty[lane] = 0;
    dirty &= am;
    for (uint64_t m = dirty; m;) {  // eight lookups in flight (branch-free: spare slots look up (0, 0))
      int ks[8];
      uint32_t rr[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool v = m != 0ULL;
        const int k = v ? __builtin_ctzll(m) : 0;
        m = v ? (m & (m - 1)) : m;
        const int nx = v ? next_of(k) : n;
        ks[u] = v ? k : -1;
        const uint32_t x = v ? (uint32_t)id[own(k)] : 0u;
        const uint32_t y = (v && nx < n) ? (uint32_t)id[at(nx)] : 0u;
        rr[u] = lookup<kWide>(t, x, y);
        rr[u] = nx < n ? rr[u] : kInf;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (ks[u] >= 0) rk[own(ks[u])] = (T)rr[u];
    }
    if (dirty | kill) seg_min();
    wave_sync_mem();
  }
  // the surviving ids, in order
  const uint32_t cnt = (uint32_t)__popcll(am);
  const uint32_t incl = wave_incl_scan(cnt, lane);
  uint32_t o = incl - cnt;
  for (uint64_t m = am; m; m &= m - 1) out[o++] = id[own(__builtin_ctzll(m))];
  return (int)lane_value(incl, 63);
}

// one 64-thread workgroup (one wave) per chunk; launched with a grid far larger than the
// usual long-chunk count, so the dispatcher hands chunks to free CUs as others finish
template <bool kWide, bool k16>
__global__ void __launch_bounds__(64) k_merge_long_lds(EncArgs a) {
  typedef typename std::conditional<k16, uint16_t, uint32_t>::type T;
  __shared__ T s_id[kLongLds];
  __shared__ T s_rk[kLongLds];
  __shared__ uint64_t s_kill[64], s_dirty[64];
  const int lane = threadIdx.x;
  const int64_t n_long = long_count(a);
  for (int64_t i = blockIdx.x; i < n_long; i += gridDim.x) {
    const int64_t start = a.lstart[i], len = a.llen[i];
    if (len > kLongLds) {  // (k_merge_long, from the list)
      if (lane == 0) a.big_list[atomicAdd(a.big_count, 1u)] = (uint32_t)i;
      continue;
    }
    uint32_t* gid = a.res + 2 * start + 1;
    const int m = seg_merge<kWide, T>(a.table, a.bytes + start, s_id, s_rk, s_kill, s_dirty, (int)len, lane, gid);
    if (lane == 0) gid[-1] = (uint32_t)m;
    wave_sync_mem();
  }
}

// ---------------------------------------------------------------------------------------
// Long chunks by exact SPLIT + VERIFY (well-formed tables; DESIGN.md §4.2 has the proof).
//
// A table is well-formed when every value is >= 256, unique, and larger than both ids of its
// pair.  Then the reference loop (base.py:10-36) applies ranks in strictly increasing order,
// and a token's id is the step that created it.  Cut a chunk into pieces A | B and encode them
// on their own: until a merge joins the last token of A with the first token of B, the joint
// state is the concatenation of the two states.  The last token of A over time is the RIGHT
// spine of A's final last token in the merge tree (a_0 < a_1 < ... ids = creation steps), the
// first token of B the LEFT spine of B's final first token.  The pair (a_i, b_j) exists from
// max(a_i, b_j) until min(a_{i+1}, b_{j+1}); the joint loop merges it iff its rank R comes
// before either token is replaced: R < a_{i+1} and R <= b_{j+1} (R == a_{i+1} means the same
// (x, x) pair also ends A, and left to right takes A's occurrence first).  If no coexisting pair
// of the two spines satisfies that, the joint encoding IS the concatenation; otherwise the two
// pieces are joined into one window and encoded again, and its new neighbours are checked
// (long_split.h runs this over all long chunks of a launch at once).  Cut points are chosen where
// the byte pair ranks highest (ideally not a merge at all), which leaves ~2% of the junctions
// in conflict.
// ---------------------------------------------------------------------------------------
constexpr int kPieceN = 16;  // per-lane register loop size (12-byte loops with 8-byte pieces: C5 106.9 -> 104.1 GB/s)
constexpr int kPieceW = 12;  // cut spacing
constexpr int kCutHalf = 2;  // cuts in [W k - H, W k + H)
static_assert(kPieceW + 2 * kCutHalf - 1 <= kPieceN && kPieceW + kCutHalf <= kPieceN, "pieces fit the loop");

// May the joint encoding of two adjacent segments differ from their separate encodings?  a: the
// left segment's last token, b: the right segment's first token (both encoded on their own).
// Walks the coexisting pairs of the two spines from the final state backwards: one pair lookup
// and one inverse-table load (issued together) per step.
template <bool kWide>
__device__ __forceinline__ bool junction_conflict(const DevTable& t, const uint2* inv, uint32_t n_inv, uint32_t a,
                                                  uint32_t b) {
  uint32_t na = kInf, nb = kInf;  // the ids (= creation steps) of the tokens that replace a / b
  for (int it = 0; it < 128; ++it) {
    const bool ra = a >= 256 && (b < 256 || a > b);  // the later-created one is reverted next
    const uint32_t x = ra ? a : b;
    if (x >= 256 && x >= n_inv) return true;  // (not a merge value: cannot happen; be conservative)
    const uint2 pr = x >= 256 ? inv[x] : make_uint2(0u, 0u);
    const uint32_t R = lookup<kWide>(t, a, b);
    if (R != kInf && R < na && R <= nb) return true;
    if (a < 256 && b < 256) return false;
    if (ra) { na = a; a = pr.y; } else { nb = b; b = pr.x; }
  }
  return true;
}

// The exact loop (any table) on a window of n <= 64 ids held one per lane (lane = position):
// rk = the rank of the pair (lane, lane + 1), kInf for the last.  Per step one wave min of
// (rank, position), the occurrences of that pair by ballot ((a, a) runs resolved left to right in
// alive order), the right partners die, and only the pairs touching a new token are looked up
// again -- all lanes at once.  Returns the alive mask; the survivors' ids stay in `id`.
template <bool kWide>
__device__ uint64_t wave_merge64(const DevTable& t, uint32_t& id, uint32_t& rk, int n, int lane) {
  uint64_t alive = n >= 64 ? ~0ULL : ((1ULL << n) - 1ULL);
  auto next_alive = [&](int j) -> int {
    const uint64_t m = j >= 63 ? 0ULL : (alive & (~0ULL << (j + 1)));
    return m ? __builtin_ctzll(m) : 64;
  };
  while (true) {
    const bool al = (alive >> lane) & 1ULL;
    const uint64_t key = (al && rk != kInf) ? (((uint64_t)rk << 6) | (uint64_t)lane) : ~0ULL;
    const uint64_t kmin = wave_min_u64(key);
    if (kmin == ~0ULL) break;
    const uint32_t r = (uint32_t)(kmin >> 6);
    const int pm = (int)(kmin & 63);
    const int nx = next_alive(lane);
    const uint32_t nid = (uint32_t)__shfl((int)id, nx & 63, 64);
    const uint32_t p0 = (uint32_t)__shfl((int)id, pm, 64), p1 = (uint32_t)__shfl((int)nid, pm, 64);
    const uint64_t M = __ballot(al && nx < 64 && id == p0 && nid == p1);
    uint64_t T = M;
    if (p0 == p1) {  // (a, a): a taken position consumes its next alive one
      T = 0;
      int consumed = -1;
      for (uint64_t m = M; m; m &= m - 1) {
        const int q = __builtin_ctzll(m);
        if (q != consumed) {
          T |= 1ULL << q;
          consumed = next_alive(q);
        }
      }
    }
    const uint64_t below = alive & ((1ULL << lane) - 1ULL);
    const int pv = below ? 63 - __builtin_clzll(below) : -1;
    const bool dies = al && pv >= 0 && ((T >> pv) & 1ULL);
    const bool took = (T >> lane) & 1ULL;
    if (took) id = r;
    alive &= ~__ballot(dies);
    const bool al2 = (alive >> lane) & 1ULL;
    const int nx2 = next_alive(lane);
    const uint32_t nid2 = (uint32_t)__shfl((int)id, nx2 & 63, 64);
    if (al2) {
      if (nx2 >= 64) rk = kInf;
      else if (took || ((T >> nx2) & 1ULL)) rk = lookup<kWide>(t, id, nid2);
    }
  }
  return alive;
}

template <bool kWide>
__global__ void __launch_bounds__(kThreads) k_merge_long(EncArgs a) {
  SW_STAMP_INIT;
  const int64_t gw = ((int64_t)blockIdx.x * kWaves + wave_in_block());
  const int64_t n_waves = ((int64_t)gridDim.x * kThreads) >> 6;
  const int lane = threadIdx.x & 63;
  const uint32_t n_big = *a.big_count;  // (listed by k_merge_long_lds)
  for (int64_t b = gw; b < (int64_t)n_big; b += n_waves) {
    const int64_t i = a.big_list[b];
    const int64_t start = a.lstart[i], len = a.llen[i];
    uint32_t* gid = a.res + 2 * start + 1;  // ids: len words, then ranks: len - 1 words
    uint32_t* grk = gid + len;
    for (int64_t j = lane; j < len; j += 64) gid[j] = a.bytes[start + j];
    wave_sync_mem();
    const int64_t m = coop_merge<kWide>(a.table, gid, grk, len, lane);
    if (lane == 0) gid[-1] = (uint32_t)m;  // (coop_merge ends wave-synchronised)
    wave_sync_mem();
  }
#ifdef SW_STAMPS
  SW_STAMP(6);
#endif
}

// first string starting at or after each tile's first byte (binary search per tile)
// (zero: a launch's counter to clear before its k_classify, or NULL)
__global__ void k_tile_strings(const int64_t* str_off, int64_t n_str, int64_t n_tiles, int64_t* tile_slo,
                               unsigned long long* zero) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0 && zero) *zero = 0;
  if (t >= n_tiles) return;
  const int64_t t0 = t * kTile;
  int64_t lo = 0, hi = n_str;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (str_off[m] < t0) lo = m + 1; else hi = m;
  }
  tile_slo[t] = lo;
}

// tile_sp[t], t in [0, n_tiles]: the first special-token occurrence starting at or after byte
// t * kTile; the count is n, or *n_dev (the device finder's) when n_dev is given
__global__ void k_tile_specials(const int64_t* pos, const int32_t* len, int64_t n, const int64_t* n_dev, int64_t n_tiles,
                                int64_t* tile_sp, int64_t* tile_spw) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > n_tiles) return;
  const int64_t cnt = n_dev ? min(max(*n_dev, (int64_t)0), n) : n;
  const int64_t t0 = t * kTile, w0 = t0 - 64;
  int64_t lo = 0, hi = cnt, lw = 0, hw = cnt;  // (the two searches side by side: starts, then ends)
  while (lo < hi || lw < hw) {
    if (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (pos[m] < t0) lo = m + 1; else hi = m;
    }
    if (lw < hw) {
      const int64_t m = (lw + hw) >> 1;
      if (pos[m] + len[m] < w0) lw = m + 1; else hw = m;  // (ends ascend: the occurrences do not overlap)
    }
  }
  tile_sp[t] = lo;
  tile_spw[t] = lw;
}

// ---------------------------------------------------------------------------------------
// tile-count scan (3 small kernels)
// ---------------------------------------------------------------------------------------
constexpr int kScanPer = 16;                      // tiles per thread in the scan kernels
constexpr int kScanBlock = kThreads * kScanPer;   // tiles per scan block

// (n_dev: when not null the count is min(n, *n_dev), read on the device -- a grid sized for a
// capacity n whose blocks past the live count return at once)
__device__ __forceinline__ int64_t scan_count(int64_t n, const int64_t* n_dev) {
  if (!n_dev) return n;
  const int64_t d = *n_dev;
  return d < n ? (d < 0 ? 0 : d) : n;
}

// (the counts read striped: every load instruction one contiguous 1 KB of the wave, not 64 lines)
__global__ void __launch_bounds__(kThreads) k_scan_reduce(const uint32_t* cnt, int64_t n_max, const int64_t* n_dev,
                                                          int64_t* part) {
  const int64_t n = scan_count(n_max, n_dev);
  if ((int64_t)blockIdx.x * kScanBlock >= n) {
    if (threadIdx.x == 0) part[blockIdx.x] = 0;
    return;
  }
  const int64_t b0 = (int64_t)blockIdx.x * kScanBlock;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int64_t i = b0 + k * kThreads + threadIdx.x;
    s += i < n ? cnt[i] : 0u;
  }
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

// (striped through LDS: the counts loaded and the offsets stored one contiguous run per wave
// instruction, each thread scanning kScanPer consecutive counts in between -- a thread's own 16
// counts and 16 offsets straight from memory were 16 instructions touching 64 lines each)
// Each block sums the partial sums of the blocks before it itself (<= a few thousand: one load
// per thread per 256) -- no k_scan_parts pass between -- and block 0 writes the total.
__global__ void __launch_bounds__(kThreads) k_scan_apply(const uint32_t* cnt, int64_t n_max, const int64_t* n_dev,
                                                         const int64_t* part, int64_t* base_out, int64_t* total) {
  const int64_t n = scan_count(n_max, n_dev);
  if (blockIdx.x > 0 && (int64_t)blockIdx.x * kScanBlock >= n) return;  // (block 0 writes the total, 0 too)
  __shared__ int64_t s_pre[2];
  {
    const int64_t n_parts = (n + kScanBlock - 1) / kScanBlock;
    const int64_t upto = blockIdx.x == 0 ? n_parts : (int64_t)blockIdx.x;  // (block 0: all, for the total)
    int64_t a = 0;
    for (int64_t j = threadIdx.x; j < upto; j += kThreads) a += part[j];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off, 64);
    __shared__ int64_t s_red[kThreads / 64];
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t t = 0;
      for (int k = 0; k < kThreads / 64; ++k) t += s_red[k];
      s_pre[0] = blockIdx.x == 0 ? 0 : t;
      if (blockIdx.x == 0) *total = t;
    }
  }
  __shared__ uint32_t s_c[kScanBlock + kScanBlock / 32];  // (one pad word per 32: conflict-free rows)
  auto at = [](int i) { return i + (i >> 5); };
  const int64_t b0 = (int64_t)blockIdx.x * kScanBlock;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int i = k * kThreads + threadIdx.x;
    s_c[at(i)] = b0 + i < n ? cnt[b0 + i] : 0u;
  }
  __syncthreads();
  uint32_t v[kScanPer];
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    v[k] = s_c[at(threadIdx.x * kScanPer + k)];
    s += v[k];
  }
  uint32_t x = s;  // (a block's counts sum below 2^31: at most the launch's bytes)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  x = wave_incl_scan(x, lane);
  __shared__ uint32_t sw[kThreads / 64];
  if (lane == 63) sw[wid] = x;
  __syncthreads();
  uint32_t wb = 0;
  for (int k = 0; k < wid; ++k) wb += sw[k];
  uint32_t run = wb + x - s;  // block-relative exclusive offset of this thread's first count
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    s_c[at(threadIdx.x * kScanPer + k)] = run;
    run += v[k];
  }
  __syncthreads();
  const int64_t p = s_pre[0];
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const int i = k * kThreads + threadIdx.x;
    if (b0 + i < n) base_out[b0 + i] = p + (int64_t)s_c[at(i)];
  }
}

// The same scan over a count that lives in device memory (n = min(*n_dev, n_max)), on a fixed grid
// of kDscanGrid blocks whatever the capacity: block b scans the b-th of kDscanGrid equal ranges.
constexpr int kDscanGrid = 512;
__device__ __forceinline__ void dscan_range(int64_t n, int64_t* lo, int64_t* hi) {
  const int64_t per = ((n + kDscanGrid - 1) / kDscanGrid + kScanBlock - 1) / kScanBlock * kScanBlock;
  *lo = min((int64_t)blockIdx.x * per, n);
  *hi = min(*lo + per, n);
}

__global__ void __launch_bounds__(kThreads) k_dscan_reduce(const uint32_t* cnt, int64_t n_max, const int64_t* n_dev,
                                                           int64_t* part) {
  int64_t lo, hi;
  dscan_range(scan_count(n_max, n_dev), &lo, &hi);
  uint64_t s = 0;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) s += cnt[i];
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

__global__ void __launch_bounds__(kDscanGrid) k_dscan_parts(int64_t* part, int64_t* total) {
  __shared__ int64_t sh[kDscanGrid];
  const int64_t v = part[threadIdx.x];
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int off = 1; off < kDscanGrid; off <<= 1) {
    const int64_t y = threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
    __syncthreads();
    sh[threadIdx.x] += y;
    __syncthreads();
  }
  part[threadIdx.x] = sh[threadIdx.x] - v;
  if (threadIdx.x == kDscanGrid - 1) *total = sh[threadIdx.x];
}

__global__ void __launch_bounds__(kThreads) k_dscan_apply(const uint32_t* cnt, int64_t n_max, const int64_t* n_dev,
                                                          const int64_t* part, int64_t* base_out) {
  int64_t lo, hi;
  dscan_range(scan_count(n_max, n_dev), &lo, &hi);
  __shared__ uint64_t sw[kThreads / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t carry = part[blockIdx.x];
  for (int64_t t0 = lo; t0 < hi; t0 += kScanBlock) {  // kScanPer consecutive items per thread
    const int64_t base = t0 + (int64_t)threadIdx.x * kScanPer;
    uint32_t v[kScanPer];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      v[k] = base + k < hi ? cnt[base + k] : 0u;
      s += v[k];
    }
    uint64_t x = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint64_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) sw[wid] = x;
    __syncthreads();
    uint64_t wb = 0, tot = 0;
    for (int k = 0; k < kThreads / 64; ++k) {
      if (k < wid) wb += sw[k];
      tot += sw[k];
    }
    __syncthreads();
    int64_t run = carry + (int64_t)(wb + x - s);
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      if (base + k < hi) base_out[base + k] = run;
      run += v[k];
    }
    carry += (int64_t)tot;
  }
}

// ---------------------------------------------------------------------------------------
// k_tile_count / k_compact: one WAVE per tile (a tile has <= kTile chunks, ~380 on prose), the
// tile's slots taken 64 at a time in order (slot 64r + lane in round r), so every slot load
// is one 256-byte coalesced access and the ids of consecutive slots land at consecutive
// output positions (near-coalesced stores without staging).  A reference costs one gather
// from res (count + first 3 ids in one 16-byte load).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint4 res_head(const uint32_t* res, int64_t p) {
  // res + 2p is 8-byte aligned; a dword-aligned 16-byte global load is legal on CDNA
  uint4 q;
  __builtin_memcpy(&q, res + 2 * p, sizeof(q));
  return q;
}
// the head {count, id0, id1, id2 | p} of the result a reference slot names
// (one load from a selected address: a branch per kind would wait for one load before the other)
__device__ __forceinline__ uint4 ref_head(const EncArgs& a, int32_t v) {
  const SW_AS_GLOBAL uint32_t* src =
      slot_is_dref(v) ? gptr((const uint32_t*)(a.dres + slot_did(v))) : gptr((const uint32_t*)a.res + 2 * slot_pos(v));
  const uint32_t x0 = src[0], x1 = src[1], x2 = src[2], x3 = src[3];  // (dword-aligned 16 bytes)
  return make_uint4(x0, x1, x2, x3);
}

constexpr int kRoundsInFlight = 8;  // slot rounds whose loads (then gathers) issue together

// id count of the result a reference-list entry names
// (a dense result's count from the byte array: 4 MiB at most, so these random reads mostly hit
// L2 where the 16-byte heads (64 MiB) went to the Infinity Cache; both loads issue together)
__device__ __forceinline__ uint32_t ref_count(const EncArgs& a, uint32_t r) {
  const bool dn = (r & kRlDense) != 0;
  const uint32_t c8 = a.dcnt[dn ? (r & ~kRlDense) : 0u];
  const uint32_t c32 = a.res[dn ? 0 : 2 * (int64_t)r];
  return dn ? c8 : c32;
}

// k_tile_count: kTcTiles tiles per wave, their first 64 list entries and sizes loaded together,
// then their counts: one dependent round trip serves kTcTiles tiles (a tile holds ~58
// references on prose, so one wave per tile spent most of its life waiting)
constexpr int kTcTiles = 2;  // (4: no faster, r4s)
__global__ void __launch_bounds__(kThreads) k_tile_count(EncArgs a) {
  const int64_t tb = (((int64_t)blockIdx.x * kWaves + wave_in_block())) * kTcTiles;
  const int lane = threadIdx.x & 63;
  if (tb >= a.n_tiles) return;
  uint32_t p0[kTcTiles], c[kTcTiles];
  int C[kTcTiles], nr[kTcTiles];
#pragma unroll
  for (int k = 0; k < kTcTiles; ++k) {
    const int64_t t = min(tb + k, a.n_tiles - 1);  // (a clamped duplicate is not stored)
    p0[k] = SW_LDNT2(&a.rlist[t * kTile + lane]);
    C[k] = (int)a.tile_slots[t];
    nr[k] = (int)a.tile_nref[t];
  }
#pragma unroll
  for (int k = 0; k < kTcTiles; ++k) c[k] = lane < nr[k] ? ref_count(a, p0[k]) : 0u;
#pragma unroll
  for (int k = 0; k < kTcTiles; ++k) {
    const uint32_t* rl = a.rlist + min(tb + k, a.n_tiles - 1) * kTile;
    for (int i0 = 64; i0 < nr[k]; i0 += 64)  // (long lists: the rest a round at a time)
      if (i0 + lane < nr[k]) c[k] += ref_count(a, SW_LDNT2(&rl[i0 + lane]));
  }
#pragma unroll
  for (int k = 0; k < kTcTiles; ++k) {
    const uint32_t v = wave_sum(c[k], lane);
    if (lane == 0 && tb + k < a.n_tiles) a.tile_cnt[tb + k] = v + (uint32_t)(C[k] - nr[k]);
  }
}

// k_tile_count_staged (launches whose dedupe table has grown past the caches: the low-repetition
// corpora, where every reference's 16-byte head is a random HBM read): the tile's ids per tile as
// k_tile_count, but from the heads themselves -- gathered once here, in the tile's reference order,
// and written over the tile's own reference list (2048 words: room for kStageCap heads), so that
// k_compact reads them back as one coalesced run instead of gathering them a second time.  One wave
// per tile; every list entry is read before the first head is written over the list.
constexpr int kStageCap = kTile / 4;  // heads staged per tile (the list's 2048 words)
constexpr int kStageRounds = kStageCap / 64;
__global__ void __launch_bounds__(kThreads) k_tile_count_staged(EncArgs a) {
  const int64_t t = (int64_t)blockIdx.x * kWaves + wave_in_block();
  const int lane = threadIdx.x & 63;
  if (t >= a.n_tiles) return;
  uint32_t* rl = a.rlist + t * kTile;
  const int C = (int)a.tile_slots[t], nr = (int)a.tile_nref[t];
  const int ns = min(nr, kStageCap);
  uint32_t e[kStageRounds];
#pragma unroll
  for (int j = 0; j < kStageRounds; ++j) e[j] = (64 * j < ns && 64 * j + lane < ns) ? SW_LDNT2(&rl[64 * j + lane]) : 0u;
  uint32_t c = 0;
  for (int i0 = kStageCap; i0 < nr; i0 += 64)  // (beyond the staged ones: counts only, read before any head is written)
    if (i0 + lane < nr) c += ref_count(a, SW_LDNT2(&rl[i0 + lane]));
  uint4 q[kStageRounds];
#pragma unroll
  for (int j = 0; j < kStageRounds; ++j) {
    q[j] = make_uint4(0u, 0u, 0u, 0u);
    if (64 * j < ns && 64 * j + lane < ns) {
      const uint32_t r = e[j];
      q[j] = ref_head(a, (r & kRlDense) ? slot_dref(r & ~kRlDense) : slot_ref((int64_t)r));
    }
  }
#pragma unroll
  for (int j = 0; j < kStageRounds; ++j) {
    if (64 * j < ns && 64 * j + lane < ns) {
      const bool dense = (e[j] & kRlDense) != 0;
      c += dense && a.ids16 ? (q[j].x & 0xFFFFu) : q[j].x;
    }
  }
  wave_sync_mem();  // (every lane's reads of the list are done: its words are rewritten now)
  uint4* hd = (uint4*)rl;
#pragma unroll
  for (int j = 0; j < kStageRounds; ++j)
    if (64 * j < ns && 64 * j + lane < ns) hd[64 * j + lane] = q[j];
  const uint32_t v = wave_sum(c, lane);
  if (lane == 0) a.tile_cnt[t] = v + (uint32_t)(C - nr);
}

constexpr int kRefCap = 128;    // references per 8-round group gathered through LDS
constexpr int kOutCapW = 1024;  // ids per group staged in LDS (the rest are stored directly)
// k_compact7: the same at 7 waves per SIMD with 768 staged ids a group (70 VGPRs, 22.5 KB of LDS a
// block), for launches whose tiles hold few ids (the host chooses from the last launch's ids per
// tile): C2 0.855 -> 0.803 ms, C5 0.794 -> 0.749, but 11% slower on ENTROPY's 1293 ids a tile
// (its groups overflow the staging; r7j in profiles/r5_ab.txt)
constexpr int kOutCap7 = 768;
constexpr int kCompact7MaxIdsPerTile = 900;  // (the host's threshold on the last launch's average)
constexpr int kCompactTypedMaxIdsPerTile = 640;  // (... below which it takes the typed one, see compact_tile)
constexpr uint32_t kLaneCopy = 64;  // results longer than this are copied by the whole wave

// tile t's ids to out + base (base: the ids of the tiles before it); per wave: the group's
// references, gathered with full lanes before any store (a store ahead of a load in the wave's
// vmcnt order would make the load wait for it)
// kTyped: the staging / direct stores and the staged-head loads as separate LDS and global
// instructions; else one generic (FLAT) access with a per-lane address, which costs every access
// both counters but is one instruction where a group's ids overflow the staging (ENTROPY, C5).
// r8d: C2 k_compact7 0.797 -> 0.755 ms typed; ENTROPY's k_compact 3.39 -> 3.94 and C5's k_compact7
// 0.754 -> 0.796 typed -- so the host takes the typed kernel only for launches with few ids a tile.
template <typename OutT, int kOutCap, bool kTyped>  // OutT: int32_t, or uint16_t (SW_OPT_OUT_BITS 16: every id of the table fits)
__device__ __forceinline__ void compact_tile(const EncArgs& a, int64_t t, int64_t base, OutT* out, uint32_t* s_rp_g,
                                             uint4* s_rq_g, int32_t* s_out_g) {
  SW_AS_LDS uint32_t* s_rp = lptr(s_rp_g);
  SW_AS_LDS u32x4* s_rq = lptr((u32x4*)s_rq_g);
  SW_AS_LDS int32_t* s_out = lptr(s_out_g);
  OutT* const dst_p = out + base;
  auto put_id = [&](uint32_t l, uint32_t o_, int32_t id) {  // staged id l, or straight to output o_
    if constexpr (kTyped) {
      if (l < (uint32_t)kOutCap) s_out[l] = id;
      else gptr(dst_p)[o_] = (OutT)id;
    } else {
      if (l < (uint32_t)kOutCap) s_out_g[l] = id;
      else dst_p[o_] = (OutT)id;
    }
  };
  SW_STAMP_INIT;
  const int lane = threadIdx.x & 63;
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  constexpr int R = kRoundsInFlight;
  const SW_AS_GLOBAL int32_t* src = gptr((const int32_t*)a.scratch + t * kTile);
  const int C = (int)a.tile_slots[t];
  SW_AS_GLOBAL OutT* dst = gptr(out + base);
  // strings starting in this tile: lane i holds string s_lo + i's chunk index (k_classify)
  const int64_t t1 = tile_end(t * kTile, a.n_bytes);
  const int64_t s_lo = a.tile_slo[t];
  const int64_t s_hi = (t + 1 < a.n_tiles) ? a.tile_slo[t + 1] : a.n_str;
  const int64_t my_s = s_lo + lane;
  // a string's chunk index loads with its offset, not after it (one dependent round trip
  // less); the out_off of a string past this tile may be being rewritten by its own tile's
  // wave: the value is read but not used then
  const int64_t ms = min(my_s, a.n_str);
  const int64_t s_at = a.str_off[ms], s_cj = a.out_off[ms];
  const bool has_s = my_s < s_hi && s_at < t1;
  const int sj = has_s ? (int)s_cj : -1;
  const bool many = s_hi - s_lo > 64;  // rare: slot offsets go through scratch instead
  uint32_t s_off = 0, carry = 0;
  int refs_before = 0;  // (wave-uniform) references of the groups before this one
#ifdef SW_STAMPS
  if (sj == -12345) s_off = 1;  // (forces the string loads to land here in stamp builds)
  SW_STAMP(8);
#endif
  for (int r0 = 0; r0 * 64 < C; r0 += R) {
    int32_t v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) v[u] = SW_LDNT(&src[min(((r0 + u) << 6) + lane, kTile - 1)]);
    // dense list of the group's references (their index in the list per round and lane)
    uint32_t ridx[R];
    int nref = 0;  // wave-uniform
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const bool ref = ((r0 + u) << 6) + lane < C && v[u] < 0;
      const uint64_t mk = __ballot(ref);
      ridx[u] = (uint32_t)(nref + __popcll(mk & lt_mask));
      if (ref && ridx[u] < (uint32_t)kRefCap) s_rp[ridx[u]] = (uint32_t)v[u];
      nref += __popcll(mk);
    }
    wave_sync_mem();
    {  // (both gathers of a group in flight before either lands in LDS)
      static_assert(kRefCap == 128, "two gathers per lane");
      const int nr = min(nref, kRefCap);
      uint4 q0 = make_uint4(0, 0, 0, 0), q1 = make_uint4(0, 0, 0, 0);
      // (staged: the group's references are the tile's refs_before + 0 .. nr - 1, in order)
      const SW_AS_GLOBAL u32x4* sth = gptr((const u32x4*)(a.rlist + t * kTile)) + refs_before;
      auto st4 = [&](int i) { const u32x4 x = sth[i]; return make_uint4(x[0], x[1], x[2], x[3]); };
      if (lane < nr) {
        if (a.staged_heads && refs_before + lane < kStageCap) q0 = st4(lane);
        else q0 = ref_head(a, (int32_t)s_rp[lane]);
      }
      if (lane + 64 < nr) {
        if (a.staged_heads && refs_before + lane + 64 < kStageCap) q1 = st4(lane + 64);
        else q1 = ref_head(a, (int32_t)s_rp[lane + 64]);
      }
      if (lane < nr) s_rq[lane] = u32x4{q0.x, q0.y, q0.z, q0.w};
      if (lane + 64 < nr) s_rq[lane + 64] = u32x4{q1.x, q1.y, q1.z, q1.w};
    }
    wave_sync_mem();
    SW_STAMP(9);
    const uint32_t gbase = carry;  // the group's first id, tile-relative
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int r = r0 + u;
      if ((r << 6) >= C) break;  // (wave-uniform)
      const int j = (r << 6) + lane;
      const bool valid = j < C;
      const bool ref = valid && v[u] < 0;
      uint4 q = make_uint4(0, 0, 0, 0);
      // (a group's references past kRefCap: gathered here -- from the staged heads when there are)
      const bool staged = a.staged_heads && refs_before + (int)ridx[u] < kStageCap;
      if constexpr (kTyped) {
        if (ref) {
          if (ridx[u] < (uint32_t)kRefCap) {
            const u32x4 x = s_rq[ridx[u]];
            q = make_uint4(x[0], x[1], x[2], x[3]);
          } else if (staged) {
            const u32x4 x = gptr((const u32x4*)(a.rlist + t * kTile))[refs_before + ridx[u]];
            q = make_uint4(x[0], x[1], x[2], x[3]);
          } else {
            q = ref_head(a, v[u]);
          }
        }
      } else {
        if (ref) {
          if (ridx[u] < (uint32_t)kRefCap) q = s_rq_g[ridx[u]];
          else if (staged) q = ((const uint4*)(a.rlist + t * kTile))[refs_before + ridx[u]];
          else q = ref_head(a, v[u]);
        }
      }
      const bool dense = ref && slot_is_dref(v[u]);
      const bool d16 = dense && a.ids16 != 0;
      const uint32_t m = ref ? (dense ? (q.x & 0xFFFFu) : q.x) : (valid ? 1u : 0u);
      const uint32_t incl = wave_incl_scan(m, lane);
      const uint32_t o = carry + incl - m;
      carry += lane_value(incl, 63);
      const uint32_t lo = o - gbase;
      if (valid && !ref) {
        put_id(lo, o, v[u]);
      }
      // ids from the head while it has them (nh), then from res at the merged occurrence's p
      const uint32_t nh = d16 ? (m <= 7 ? m : 1u) : dense ? (m <= 3 ? 3u : 2u) : 3u;
      const int64_t p = !ref ? 0 : d16 ? (int64_t)q.y : dense ? (int64_t)q.w : slot_pos(v[u]);
      if (ref) {
        const uint32_t mm = m > kLaneCopy ? 3u : m;  // (long results: the head here, the rest below)
        const uint32_t hm = min(mm, nh);
        auto put = [&](uint32_t k, uint32_t id) {
          put_id(lo + k, o + k, (int32_t)id);
        };
        if (d16) {
          const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (uint32_t k = 0; k < 7; ++k)
            if (k < hm) put(k, (w[(k + 1) >> 1] >> (16 * ((k + 1) & 1))) & 0xFFFFu);
        } else {
          if (hm > 0) put(0, q.y);
          if (hm > 1) put(1, q.z);
          if (hm > 2) put(2, q.w);
        }
        for (uint32_t k0 = hm; k0 < mm; k0 += 4) {  // (four loads in flight, then their stores)
          uint32_t x[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) x[q] = k0 + q < mm ? a.res[2 * p + 1 + k0 + q] : 0u;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (k0 + q < mm) put(k0 + q, x[q]);
        }
      }
      // long results (C5: whole 4 KiB chunks): one coalesced copy by the whole wave each
      for (uint64_t lm = __ballot(ref && m > kLaneCopy); lm; lm &= lm - 1) {
        const int L = __ffsll((long long)lm) - 1;
        const int64_t pL = (int64_t)lane_value64((unsigned long long)p, L);
        const uint32_t oL = lane_value(o, L), mL = lane_value(m, L);
        const uint32_t loL = oL - gbase;
        for (uint32_t k0 = 3; k0 < mL; k0 += 256) {  // (four loads in flight per lane, then the stores)
          int32_t id[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t k = k0 + 64 * q + lane;
            id[q] = k < mL ? (int32_t)a.res[2 * pL + 1 + k] : 0;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t k = k0 + 64 * q + lane;
            if (k >= mL) break;
            put_id(loL + k, oL + k, id[q]);
          }
        }
      }
      const uint32_t got = (uint32_t)__shfl((int)o, sj & 63, 64);
      if ((sj >> 6) == r) s_off = got;
      if (many && valid) a.scratch[t * kTile + j] = (int32_t)o;  // (this wave's own slots)
    }
    wave_sync_mem();
    // the staged ids: one contiguous 256-byte store per 64 ids, each lane reading its own LDS word
    // (round 6: 16-byte stores of four ids a lane read those words at a 4-word lane stride, and the
    // bank conflicts cost more than the stores saved -- C2 k_compact7 0.832 -> 0.813 ms, r9zi)
    const uint32_t staged = min(carry - gbase, (uint32_t)kOutCap);
    for (uint32_t i = lane; i < staged; i += 64) SW_STNT(&dst[gbase + i], (OutT)s_out[i]);
    refs_before += nref;
    wave_sync_mem();  // (s_rp / s_rq / s_out are rewritten by the next group)
#ifdef SW_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    SW_STAMP(10);
#endif
  }
  if (has_s) a.out_off[my_s] = ~(base + (int64_t)(sj >= C ? carry : s_off));
  if (many) {
    wave_sync_mem();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    for (int64_t s = s_lo + 64 + lane; s < s_hi; s += 64) {
      if (a.str_off[s] >= t1) break;
      const int jj = (int)a.out_off[s];
      const uint32_t oo = jj >= C ? carry
                                  : (uint32_t)__hip_atomic_load(&a.scratch[t * kTile + jj], __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT);
      a.out_off[s] = ~(base + (int64_t)oo);
    }
  }
#ifdef SW_STAMPS
  SW_STAMP(11);
#endif
}

template <typename OutT>
__global__ void __launch_bounds__(kThreads)
k_compact(EncArgs a, const int64_t* tile_base, OutT* out) {
  __shared__ uint32_t s_rp_all[kWaves][kRefCap];
  __shared__ uint4 s_rq_all[kWaves][kRefCap];
  __shared__ int32_t s_out_all[kWaves][kOutCapW];  // a group's ids, staged for 256-B stores
  const int wv = wave_in_block();
  const int64_t t = ((int64_t)blockIdx.x * kWaves + wave_in_block());
  if (t >= a.n_tiles) return;
  compact_tile<OutT, kOutCapW, false>(a, t, tile_base[t], out, s_rp_all[wv], s_rq_all[wv], s_out_all[wv]);
}

template <typename OutT, bool kTyped>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(7, 7)))
k_compact7(EncArgs a, const int64_t* tile_base, OutT* out) {
  __shared__ uint32_t s_rp_all[kWaves][kRefCap];
  __shared__ uint4 s_rq_all[kWaves][kRefCap];
  __shared__ int32_t s_out_all[kWaves][kOutCap7];
  const int wv = wave_in_block();
  const int64_t t = ((int64_t)blockIdx.x * kWaves + wave_in_block());
  if (t >= a.n_tiles) return;
  compact_tile<OutT, kOutCap7, kTyped>(a, t, tile_base[t], out, s_rp_all[wv], s_rq_all[wv], s_out_all[wv]);
}

// every string offset: a complemented value is one k_compact finished; strings starting at or
// past n_bytes (trailing empty strings) and the end sentinel get the total
// (and the launch's dedupe overflow count to host memory, zeroed for the next launch)
__global__ void k_string_offsets(const int64_t* str_off, int64_t n_str, int64_t n_bytes, const int64_t* total,
                                 int64_t* out_off, unsigned long long* dd_full, unsigned long long* h_dd_full,
                                 const int64_t* q_total) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s == 0 && dd_full) {
    const unsigned long long v = *dd_full;
    *dd_full = 0;
    __hip_atomic_store(h_dd_full, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // (and the launch's id count: the next launch picks its k_compact from the ids per tile)
    __hip_atomic_store(h_dd_full + 1, (unsigned long long)*total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // (and its merge loops run -- the distinct queued chunks: the next launch stages the result heads
    // when they are too many for the caches)
    __hip_atomic_store(h_dd_full + 2, q_total ? (unsigned long long)*q_total : 0ULL, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (s > n_str) return;
  if (s == n_str || str_off[s] >= n_bytes) {
    out_off[s] = *total;
    return;
  }
  out_off[s] = ~out_off[s];
}

}  // namespace sw
