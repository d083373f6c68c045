// The device pre-split and k_classify in ONE kernel (SW_OPT_FUSED_PRESPLIT, the default of the
// full path): a workgroup pre-splits its 8 KiB block (presplit_block, one 32-byte chunk per
// thread: apply_regex, shredword/base.py:38-58) and then each of its four waves classifies one
// 2 KiB tile of that block (classify_tile) with the chunk-start bits straight from LDS.  The
// pre-split's VALU work and the classification's memory waits now run side by side on every CU
// (separate kernels filled the CUs with one kind at a time), and the bitmap round trip through
// HBM between them is gone from the critical path.  Included by encode.hip only.
//
// A tile's last chunk ends at the next chunk start, which for the block's last tile (and for a
// chunk running past the block) lies in the NEXT block, pre-split by another workgroup.  Such a
// chunk is deferred: k_classify_deferred, one lane per tile after the fused kernel, gives it the
// same treatment k_classify would have (single byte, whole-chunk table, dedupe, queue), appended
// after the tile's other chunks -- it is the tile's last chunk, so slot order, reference-list
// order and queue contents are exactly those of the two-kernel path.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "presplit_kernel.h"

namespace sw {

static_assert(kPbThreads == kThreads && kPbBlock == kWaves * kTile, "one classify tile per pre-split wave");

__global__ void __launch_bounds__(kPbThreads, 4) k_presplit_classify(PbArgs g, int pattern, uint32_t* bits32,
                                                                     EncArgs a) {
  struct PsLds {  // the pre-split's class masks
    uint32_t m[9][kPbChunks];
  };
  struct ClLds {  // k_classify's per-wave window, chunk starts and dedupe buffer
    uint32_t b32[kWaves][kWinWords];
    uint16_t cs[kWaves][kTile + 1];
    uint16_t qb[kWaves][kQBuf];
  };
  union Lds {
    PsLds ps;
    ClLds cl;
  };
  __shared__ __attribute__((aligned(16))) Lds sh;
  __shared__ uint32_t s_ss[kPbSsWords];
  __shared__ uint32_t s_bits[kPbThreads];  // the block's chunk-start bits, 32 bytes per dword
  s_bits[threadIdx.x] = presplit_block(g, pattern, bits32, sh.ps.m, s_ss);
  __syncthreads();  // (every thread is past the pre-split's reads of sh.ps before sh.cl is written)
  const int wv = threadIdx.x >> 6;
  const int64_t tile = (int64_t)blockIdx.x * kWaves + wv;
  if (tile < a.n_tiles)
    classify_tile<true>(a, tile, sh.cl.b32[wv], sh.cl.cs[wv], sh.cl.qb[wv], s_bits, wv,
                        (int64_t)(blockIdx.x + 1) * kPbBlock);
}

// the single token of a 2..16-byte chunk from the whole-chunk table, or kInf (one lane; the
// compares of table_lookups)
__device__ __forceinline__ uint32_t chunk_lookup1(const DevChunkTable& c, const uint32_t (&w)[4], int len) {
  if (len <= 8) {
    const uint32_t h = chunk_hash(w[0], w[1], 0, 0, len, c.s_m1);
    uint4 q = c.sb[chunk_b1(h, c.s_shift)];
    if (q.x == w[0] && q.y == w[1] && (q.z >> 24) == (uint32_t)len) return q.z & 0xFFFFFFu;
    if (!(q.w & 1u)) return kInf;
    q = c.sb[chunk_b2(h, c.s_m2, c.s_shift)];
    return (q.x == w[0] && q.y == w[1] && (q.z >> 24) == (uint32_t)len) ? (q.z & 0xFFFFFFu) : kInf;
  }
  const uint32_t h = chunk_hash(w[0], w[1], w[2], w[3], len, c.l_m1);
  const uint4* p = &c.lb[2 * chunk_b1(h, c.l_shift)];
  for (int probe = 0; probe < 2; ++probe) {
    const uint4 qa = p[0], qb = p[1];
    if (qa.x == w[0] && qa.y == w[1] && qa.z == w[2] && qa.w == w[3] && (qb.x >> 24) == (uint32_t)len)
      return qb.x & 0xFFFFFFu;
    if (!(qb.y & 1u)) return kInf;
    p = &c.lb[2 * chunk_b2(h, c.l_m2, c.l_shift)];
  }
  return kInf;
}

// the deferred last chunks of k_presplit_classify, one lane per tile (the bitmap is complete now)
__global__ void __launch_bounds__(kThreads) k_classify_deferred(EncArgs a) {
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (t >= a.n_tiles) return;
  const uint32_t ds = a.tdefer[t];
  if (ds == 0xFFFFu) return;
  const int64_t t0 = t * kTile, start = t0 + ds;
  const int64_t end = min(next_set_bit(a.bits, a.n_words, start + 1, a.n_bytes), a.n_bytes);
  const int len = (int)(end - start);
  const int k = (int)a.tile_slots[t] - 1;  // (the tile's last chunk)
  const int64_t mis = (int64_t)((uintptr_t)a.bytes & 3);
  const uint32_t* gwords = (const uint32_t*)((uintptr_t)a.bytes - mis);
  const int64_t last_word = (mis + a.n_bytes - 1) >> 2;
  int32_t* dst = a.scratch + t0;
  uint32_t tok = kInf;
  if (len == 1) {
    tok = a.bytes[start];
  } else if (a.chunks.enabled && len <= 16) {
    uint32_t w[4];
    chunk_words<16>(gwords, last_word, start + mis, len, w);
    tok = chunk_lookup1(a.chunks, w, len);
  }
  if (tok != kInf) {
    dst[k] = (int32_t)tok;
    return;
  }
  DdOut dd{0, 0};
  if (a.dedupe && len <= kShort) {
    uint32_t u[kShort / 4];
    chunk_words<kShort>(gwords, last_word, start + mis, len, u);
    dd = dedupe_claim(a, gwords, last_word, mis, start, len, u);
  }
  const uint32_t did = dd.kind ? dd.v : kNoDid;
  dst[k] = dd.kind ? slot_dref(did) : slot_ref(start);
  const uint32_t nref = a.tile_nref[t];
  a.rlist[t0 + nref] = dd.kind ? (kRlDense | did) : (uint32_t)start;
  a.tile_nref[t] = nref + 1;
  if (dd.kind != 2) {  // queued for the merge kernels: appended to the tile-local queue
    uint32_t nown = 0;
    for (int b = 0; b < kNumBuckets; ++b) nown += a.bcnt[(int64_t)b * a.n_tiles + t];
    const int64_t qi = t0 + nown;
    a.qtmp[qi] = ds | ((uint32_t)k << kTileBits) | ((uint32_t)(len <= kShort ? len : 0) << (2 * kTileBits));
    a.qtmp[qi + kTile / 2] = len > kShort ? (len < (int)kNoDid ? (uint32_t)len : kNoDid) : did;
    a.bcnt[(int64_t)bucket_of(len) * a.n_tiles + t] += 1;
  }
}

}  // namespace sw
