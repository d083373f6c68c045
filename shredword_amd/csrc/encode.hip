// MI355X (gfx950) batched BPE encode: kernels + host orchestration + the C-ABI.
//
// Semantics (exact, for ANY merge table): per pre-split chunk, ids = chunk bytes; while at
// least two ids remain, find the adjacent pair with the lowest merges-value (first occurrence
// wins ties), stop if no pair is in merges, else replace every non-overlapping occurrence of
// that pair, left to right, by the value.  This is the loop the reference's primitives
// compose: get_stats (shredword/base.py:10-20), min over merges.get (base.py:107-108 leaves
// encode abstract), merge (base.py:22-36).
//
// Device pipeline (all on one stream; inputs resident in HBM):
//   k_encode_tiles   one 256-thread workgroup per 2 KiB tile of input bytes.  Chunk starts
//                    come from the pre-split bitmap.  Chunks <= kShort bytes run the merge
//                    loop one-per-lane on LDS arrays; longer chunks run a wave-cooperative
//                    loop (ballot/popcount compaction, 64-bit wave argmin) on a
//                    position-indexed global work area.  Per-tile token counts + outputs
//                    are written tile-locally (position space, tokens <= bytes).
//   k_scan_tiles     exclusive scan of the per-tile counts
//   k_compact        tile outputs -> contiguous out_ids
//   k_string_offsets per-string output offsets
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "shredword_hip.h"
#include "table.h"

using namespace sw;

// ------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------
static thread_local std::string g_err;
static int32_t fail(int32_t code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(SW_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

extern "C" const char* sw_last_error(void) { return g_err.c_str(); }
extern "C" const char* sw_version(void) { return "shredword_hip 0.1 gfx950"; }
extern "C" int32_t sw_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------
constexpr int kTile = 2048;           // input bytes per workgroup
constexpr int kThreads = 256;         // 4 waves
constexpr int kShort = 16;            // per-lane path for chunks up to this many bytes
constexpr int kTileWords = kTile / 64 + 1;  // bitmap words loaded (tile + 64-byte halo)
constexpr int kHalo = kShort;         // bytes loaded past the tile for short chunks

__device__ __forceinline__ uint32_t lookup(const DevTable& t, uint32_t a, uint32_t b) {
  if (!t.wide) {
    if ((a | b) > 0xFFFFu) return kInf;
    const uint2* s = (const uint2*)t.slots;
    uint32_t key = (a << 16) | b;
    uint32_t h = hash_narrow(key, t.shift);
    while (true) {
      uint2 e = s[h];
      if (e.x == key) return e.y;
      if (e.x == kEmptyKey) return kInf;
      h = (h + 1) & t.mask;
    }
  } else {
    const uint4* s = (const uint4*)t.slots;
    uint32_t h = hash_wide(a, b, t.shift);
    while (true) {
      uint4 e = s[h];
      if (e.x == a && e.y == b) return e.z;
      if (e.x == kEmptyKey) return kInf;
      h = (h + 1) & t.mask;
    }
  }
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    uint64_t o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

// First set bit at position >= pos (global bit index), or n_bits if none.
__device__ int64_t next_set_bit(const uint64_t* bits, int64_t n_words, int64_t pos, int64_t n_bits) {
  int64_t w = pos >> 6;
  if (w >= n_words) return n_bits;
  uint64_t word = bits[w] & (~0ULL << (pos & 63));
  while (!word) {
    if (++w >= n_words) return n_bits;
    word = bits[w];
  }
  int64_t q = (w << 6) + __ffsll((long long)word) - 1;
  return q < n_bits ? q : n_bits;
}

// Wave-cooperative exact merge loop over W[0..n): W[i].x = id, W[i].y = rank of the pair
// (W[i].x, W[i+1].x), or kRecomp if it must be looked up.  Compacts in place; returns the
// final length.  Works on any length (W is position-indexed global scratch).
__device__ int64_t coop_merge(const DevTable& t, uint2* W, int64_t n, int lane) {
  const uint64_t lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
  while (n >= 2) {
    // pass 1: resolve pending ranks, argmin over (rank, index)
    uint64_t best = ~0ULL;
    for (int64_t i = lane; i + 1 < n; i += 64) {
      uint32_t r = W[i].y;
      if (r == kRecomp) {
        r = lookup(t, W[i].x, W[i + 1].x);
        W[i].y = r;
      }
      uint64_t key = ((uint64_t)r << 32) | (uint32_t)i;
      best = key < best ? key : best;
    }
    best = wave_min_u64(best);
    const uint32_t rank = (uint32_t)(best >> 32);
    if (rank == kInf) break;
    const int64_t b = (int64_t)(uint32_t)best;
    __threadfence_block();
    const uint32_t p0 = W[b].x, p1 = W[b + 1].x;
    // pass 2: replace every non-overlapping occurrence of (p0, p1), left to right
    int64_t w = 0;
    bool prev_taken = false;
    for (int64_t seg = 0; seg < n; seg += 64) {
      const int64_t i = seg + lane;
      const bool valid = i < n;
      uint2 e = valid ? W[i] : make_uint2(kInf, kInf);
      uint32_t nid = __shfl_down(e.x, 1, 64);
      if (lane == 63) nid = (i + 1 < n) ? W[i + 1].x : kInf;
      const bool match = valid && (i + 1 < n) && e.x == p0 && nid == p1;
      uint64_t M = __ballot(match);
      if (prev_taken) M &= ~1ULL;  // position seg is the right half of the previous take
      uint64_t T = M;
      if (p0 == p1) {  // runs of (a,a): take even offsets from each run start
        const uint64_t E = 0x5555555555555555ULL;
        uint64_t S = M & ~(M << 1);
        uint64_t runs_even = M & ~(M + (S & E));
        T = (runs_even & E) | (M & ~runs_even & ~E);
      }
      const uint64_t consumed = (T << 1) | (prev_taken ? 1ULL : 0ULL);
      const uint64_t keep = __ballot(valid) & ~consumed;
      const bool take = (T >> lane) & 1ULL;
      const bool next_take = lane < 63 ? ((T >> (lane + 1)) & 1ULL) : true;
      const int64_t pos = w + __popcll(keep & lt_mask);
      __threadfence_block();  // every lane's loads of this segment precede the stores
      if ((keep >> lane) & 1ULL)
        W[pos] = make_uint2(take ? rank : e.x, (take || next_take) ? kRecomp : e.y);
      w += __popcll(keep);
      prev_taken = (T >> 63) & 1ULL;
    }
    n = w;
    __threadfence_block();
  }
  return n;
}

struct TileArgs {
  const uint8_t* bytes;
  int64_t n_bytes;
  const uint64_t* bits;
  int64_t n_words;
  const int64_t* str_off;
  int64_t n_str;
  DevTable table;
  int32_t* scratch;      // [n_bytes] tile outputs, position space
  uint2* lw;             // [n_bytes] long-chunk work area, position space
  uint32_t* tile_cnt;    // [n_tiles]
  int64_t* tile_first;   // [n_tiles] first chunk start in tile (or -1)
  int64_t* out_off;      // [n_str+1] tile-local offsets, fixed by k_string_offsets
};

// exclusive block scan of v over kThreads threads; returns the exclusive prefix, *total set
__device__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kThreads / 64; ++k) {
    uint32_t s = sh[k];
    if (k < wid) base += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

__global__ void __launch_bounds__(kThreads) k_encode_tiles(TileArgs a) {
  __shared__ uint8_t s_bytes[kTile + kHalo];
  __shared__ uint64_t s_bits[kTileWords];
  __shared__ uint16_t s_cstart[kTile];
  __shared__ uint32_t s_cnt[kTile + 1];
  __shared__ uint32_t s_stage[kTile + kHalo];
  __shared__ uint32_t s_id[kShort * kThreads];
  __shared__ uint32_t s_rk[kShort * kThreads];
  __shared__ uint32_t s_wsum[kThreads / 64];
  __shared__ uint32_t s_nchunks;
  __shared__ uint32_t s_nlong;
  __shared__ uint16_t s_long[kTile];
  __shared__ uint32_t s_isl[kTile / 32];
  __shared__ int64_t s_slo;

  const int tid = threadIdx.x;
  const int64_t tile = blockIdx.x;
  const int64_t t0 = tile * kTile;
  const int64_t t1 = min(t0 + (int64_t)kTile, a.n_bytes);
  const int64_t w0 = t0 >> 6;

  // 1. stage bytes (tile + halo) and bitmap words
  for (int i = tid; i < kTile + kHalo; i += kThreads) {
    int64_t g = t0 + i;
    s_bytes[i] = g < a.n_bytes ? a.bytes[g] : 0;
  }
  if (tid < kTileWords) s_bits[tid] = (w0 + tid < a.n_words) ? a.bits[w0 + tid] : 0ULL;
  if (tid == 0) s_nlong = 0;
  for (int i = tid; i < kTile / 32; i += kThreads) s_isl[i] = 0;
  __syncthreads();

  // 2. enumerate chunk starts in [t0, t1): one thread per bitmap word
  const int nw_tile = kTile / 64;
  uint64_t myword = 0;
  if (tid < nw_tile) {
    myword = s_bits[tid];
    int64_t lim = t1 - (t0 + 64 * tid);  // bits at or beyond t1 do not belong to this tile
    if (lim <= 0) myword = 0;
    else if (lim < 64) myword &= (1ULL << lim) - 1;
  }
  uint32_t total_chunks;
  uint32_t wbase = block_excl_scan((uint32_t)__popcll(myword), s_wsum, &total_chunks);
  if (tid < nw_tile) {
    uint64_t x = myword;
    uint32_t k = wbase;
    while (x) {
      int b = __ffsll((long long)x) - 1;
      s_cstart[k++] = (uint16_t)(64 * tid + b);
      x &= x - 1;
    }
  }
  if (tid == 0) s_nchunks = total_chunks;
  __syncthreads();
  const int C = (int)s_nchunks;

  // end of the last chunk: next chunk start at or after t1 (halo words, then global bitmap)
  // computed lazily by the owning lane below.

  // 3. per-lane merge loop for short chunks; long chunks are queued for the waves
  for (int k = tid; k < C; k += kThreads) {
    const int64_t start = t0 + s_cstart[k];
    int64_t end;
    if (k + 1 < C) end = t0 + s_cstart[k + 1];
    else {
      // search the staged halo word(s) first
      int64_t q = -1;
      for (int w = (int)((t1 - t0) >> 6); w < kTileWords && q < 0; ++w) {
        uint64_t word = s_bits[w];
        int64_t bit0 = t0 + 64 * w;
        if (bit0 < t1) word &= ~0ULL << (t1 - bit0);
        if (word) q = bit0 + __ffsll((long long)word) - 1;
      }
      if (q < 0) q = next_set_bit(a.bits, a.n_words, t0 + 64 * kTileWords, a.n_bytes);
      end = min(q, a.n_bytes);
    }
    const int len = (int)min(end - start, (int64_t)0x7FFFFFFF);
    if (end - start > kShort) {
      uint32_t slot = atomicAdd(&s_nlong, 1u);
      s_long[slot] = (uint16_t)k;
      atomicOr(&s_isl[k >> 5], 1u << (k & 31));
      continue;
    }
    const int ls = (int)(start - t0);
    uint32_t* id = s_id + tid;
    uint32_t* rk = s_rk + tid;
    int n = len;
    for (int j = 0; j < n; ++j) {
      id[j * kThreads] = s_bytes[ls + j];
      rk[j * kThreads] = kRecomp;
    }
    while (n >= 2) {
      uint32_t best = kInf;
      int bi = -1;
      for (int j = 0; j + 1 < n; ++j) {
        uint32_t r = rk[j * kThreads];
        if (r == kRecomp) {
          r = lookup(a.table, id[j * kThreads], id[(j + 1) * kThreads]);
          rk[j * kThreads] = r;
        }
        if (r < best) { best = r; bi = j; }
      }
      if (bi < 0) break;
      const uint32_t p0 = id[bi * kThreads], p1 = id[(bi + 1) * kThreads];
      int w = 0;
      for (int j = 0; j < n;) {
        uint32_t x = id[j * kThreads];
        if (j + 1 < n && x == p0 && id[(j + 1) * kThreads] == p1) {
          id[w * kThreads] = best;
          rk[w * kThreads] = kRecomp;
          if (w > 0) rk[(w - 1) * kThreads] = kRecomp;
          ++w; j += 2;
        } else {
          id[w * kThreads] = x;
          rk[w * kThreads] = rk[j * kThreads];
          ++w; ++j;
        }
      }
      n = w;
    }
    for (int j = 0; j < n; ++j) s_stage[ls + j] = id[j * kThreads];
    s_cnt[k] = (uint32_t)n;
  }
  __syncthreads();

  // 4. long chunks: one wave per chunk, exact wave-cooperative loop in the global work area
  {
    const int wid = tid >> 6, lane = tid & 63;
    const int nl = (int)s_nlong;
    for (int q = wid; q < nl; q += kThreads / 64) {
      const int k = s_long[q];
      const int64_t start = t0 + s_cstart[k];
      int64_t end;
      if (k + 1 < C) end = t0 + s_cstart[k + 1];
      else end = next_set_bit(a.bits, a.n_words, t1, a.n_bytes);
      const int64_t len = end - start;
      uint2* W = a.lw + start;
      for (int64_t i = lane; i < len; i += 64) W[i] = make_uint2(a.bytes[start + i], kRecomp);
      __threadfence_block();
      int64_t n = coop_merge(a.table, W, len, lane);
      if (lane == 0) s_cnt[k] = (uint32_t)n;
    }
  }
  __syncthreads();

  // 5. tile-local offsets (exclusive scan over chunk counts), written in position space
  //    starting at the tile's first chunk start
  uint32_t local_sum = 0;
  const int per = (C + kThreads - 1) / kThreads;  // contiguous chunks per thread
  const int c0 = min(C, tid * per), c1 = min(C, c0 + per);
  for (int k = c0; k < c1; ++k) local_sum += s_cnt[k];
  uint32_t tile_total;
  uint32_t off = block_excl_scan(local_sum, s_wsum, &tile_total);
  for (int k = c0; k < c1; ++k) {
    uint32_t c = s_cnt[k];
    s_cnt[k] = off;  // now: exclusive offset
    off += c;
  }
  if (tid == 0) s_cnt[C] = tile_total;
  __syncthreads();
  const int64_t first = C > 0 ? t0 + s_cstart[0] : -1;
  if (tid == 0) {
    a.tile_cnt[tile] = tile_total;
    a.tile_first[tile] = first;
  }
  // 6. write tokens: short chunks from the LDS stage, long chunks from the work area
  for (int k = tid; k < C; k += kThreads) {
    if ((s_isl[k >> 5] >> (k & 31)) & 1u) continue;
    const uint32_t o = s_cnt[k], cnt = s_cnt[k + 1] - o;
    const int ls = s_cstart[k];
    int32_t* dst = a.scratch + first + o;
    for (uint32_t j = 0; j < cnt; ++j) dst[j] = (int32_t)s_stage[ls + j];
  }
  {
    const int wid = tid >> 6, lane = tid & 63;
    const int nl = (int)s_nlong;
    for (int q = wid; q < nl; q += kThreads / 64) {
      const int k = s_long[q];
      const uint32_t o = s_cnt[k], cnt = s_cnt[k + 1] - o;
      const uint2* W = a.lw + t0 + s_cstart[k];
      int32_t* dst = a.scratch + first + o;
      for (uint32_t j = lane; j < cnt; j += 64) dst[j] = (int32_t)W[j].x;
    }
  }
  // 7. strings starting in this tile: tile-local output offset (k_string_offsets rebases)
  if (tid == 0) {
    int64_t lo = 0, hi = a.n_str;  // first s with str_off[s] >= t0
    while (lo < hi) { int64_t m = (lo + hi) >> 1; if (a.str_off[m] < t0) lo = m + 1; else hi = m; }
    s_slo = lo;
  }
  __syncthreads();
  for (int64_t s = s_slo + tid; s < a.n_str; s += kThreads) {
    const int64_t p = a.str_off[s];
    if (p >= t1) break;
    int lo = 0, hi = C;  // first chunk with start >= p
    const int lp = (int)(p - t0);
    while (lo < hi) { int m = (lo + hi) >> 1; if (s_cstart[m] < lp) lo = m + 1; else hi = m; }
    a.out_off[s] = (int64_t)s_cnt[lo];
  }
}

__global__ void __launch_bounds__(1024) k_scan_tiles(const uint32_t* cnt, int64_t n, int64_t* base,
                                                    int64_t* total) {
  __shared__ int64_t sh[1024];
  const int tid = threadIdx.x;
  const int64_t per = (n + 1023) / 1024;
  const int64_t i0 = min(n, tid * per), i1 = min(n, i0 + per);
  int64_t s = 0;
  for (int64_t i = i0; i < i1; ++i) s += cnt[i];
  sh[tid] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    int64_t v = tid >= off ? sh[tid - off] : 0;
    __syncthreads();
    sh[tid] += v;
    __syncthreads();
  }
  int64_t run = sh[tid] - s;
  for (int64_t i = i0; i < i1; ++i) {
    base[i] = run;
    run += cnt[i];
  }
  if (tid == 1023) *total = sh[1023];
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

__global__ void k_string_offsets(const int64_t* str_off, int64_t n_str, int64_t n_bytes,
                                 const int64_t* tile_base, const int64_t* total, int64_t* out_off) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n_str) return;
  if (s == n_str) { out_off[s] = *total; return; }
  const int64_t p = str_off[s];
  if (p >= n_bytes) out_off[s] = *total;
  else out_off[s] += tile_base[p / kTile];
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
struct sw_encoder {
  int device = 0;
  hipStream_t stream = nullptr;
  DevTable table{};
  void* d_table = nullptr;
  int64_t n_merges = 0;
  // workspace
  int64_t cap_bytes = -1, cap_str = -1;
  int32_t* d_scratch = nullptr;
  uint2* d_lw = nullptr;
  uint32_t* d_tile_cnt = nullptr;
  int64_t* d_tile_first = nullptr;
  int64_t* d_tile_base = nullptr;
  int64_t* d_total = nullptr;
  // host-path staging
  int64_t io_bytes = -1, io_str = -1;
  uint8_t* d_bytes = nullptr;
  int64_t* d_str_off = nullptr;
  uint64_t* d_bits = nullptr;
  int32_t* d_out = nullptr;
  int64_t* d_out_off = nullptr;
  // dominant-kernel timing: one event pair per launch since sw_encoder_set_timing(h, 1)
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;  // pairs recorded
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

void free_workspace(sw_encoder* h) {
  (void)hipFree(h->d_scratch); (void)hipFree(h->d_lw); (void)hipFree(h->d_tile_cnt);
  (void)hipFree(h->d_tile_first); (void)hipFree(h->d_tile_base); (void)hipFree(h->d_total);
  h->d_scratch = nullptr; h->d_lw = nullptr; h->d_tile_cnt = nullptr;
  h->d_tile_first = nullptr; h->d_tile_base = nullptr; h->d_total = nullptr;
  h->cap_bytes = -1; h->cap_str = -1;
}

void free_io(sw_encoder* h) {
  (void)hipFree(h->d_bytes); (void)hipFree(h->d_str_off); (void)hipFree(h->d_bits);
  (void)hipFree(h->d_out); (void)hipFree(h->d_out_off);
  h->d_bytes = nullptr; h->d_str_off = nullptr; h->d_bits = nullptr; h->d_out = nullptr; h->d_out_off = nullptr;
  h->io_bytes = -1; h->io_str = -1;
}

int32_t ensure_workspace(sw_encoder* h, int64_t n_bytes) {
  if (n_bytes <= h->cap_bytes) return SW_OK;
  free_workspace(h);
  const int64_t nb = std::max<int64_t>(n_bytes, 1);
  const int64_t n_tiles = (nb + kTile - 1) / kTile;
  HIP_TRY(hipMalloc(&h->d_scratch, sizeof(int32_t) * nb));
  HIP_TRY(hipMalloc(&h->d_lw, sizeof(uint2) * nb));
  HIP_TRY(hipMalloc(&h->d_tile_cnt, sizeof(uint32_t) * n_tiles));
  HIP_TRY(hipMalloc(&h->d_tile_first, sizeof(int64_t) * n_tiles));
  HIP_TRY(hipMalloc(&h->d_tile_base, sizeof(int64_t) * n_tiles));
  HIP_TRY(hipMalloc(&h->d_total, sizeof(int64_t)));
  h->cap_bytes = nb;
  return SW_OK;
}

}  // namespace

extern "C" int32_t sw_encoder_create(const int32_t* pairs, const int32_t* vals, int64_t n, int32_t device,
                                     sw_encoder** out) {
  if (!out || n < 0 || (n > 0 && (!pairs || !vals))) return fail(SW_ERR_ARG, "sw_encoder_create: bad arguments");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(SW_ERR_NODEV, "sw_encoder_create: no HIP device visible");
  if (device < 0 || device >= ndev) return fail(SW_ERR_ARG, "sw_encoder_create: bad device ordinal");
  // dict semantics: the last value of a duplicated pair wins (base.py:145-148)
  std::unordered_map<uint64_t, int32_t> dict;
  dict.reserve((size_t)n * 2);
  std::vector<uint64_t> order;
  order.reserve((size_t)n);
  bool wide = false;
  for (int64_t i = 0; i < n; ++i) {
    int32_t a = pairs[2 * i], b = pairs[2 * i + 1], v = vals[i];
    if (a < 0 || b < 0) return fail(SW_ERR_ARG, "sw_encoder_create: negative token id in a pair");
    if (v < 0 || (uint32_t)v >= kRecomp) return fail(SW_ERR_ARG, "sw_encoder_create: merge value out of range");
    uint64_t k = ((uint64_t)(uint32_t)a << 32) | (uint32_t)b;
    auto it = dict.find(k);
    if (it == dict.end()) { dict.emplace(k, v); order.push_back(k); }
    else it->second = v;
    if (a > 0xFFFF || b > 0xFFFF || (a == 0xFFFF && b == 0xFFFF)) wide = true;
  }
  uint32_t log2cap = 4;
  while ((1ull << log2cap) < 2 * (uint64_t)order.size() + 2) ++log2cap;
  const uint64_t cap = 1ull << log2cap;
  sw_encoder* h = new sw_encoder();
  h->device = device;
  h->n_merges = (int64_t)order.size();
  h->table.mask = (uint32_t)(cap - 1);
  h->table.wide = wide ? 1u : 0u;
  std::vector<uint8_t> host;
  if (!wide) {
    h->table.shift = 32 - log2cap;
    std::vector<uint2> s(cap, make_uint2(kEmptyKey, 0));
    for (uint64_t k : order) {
      uint32_t key = (uint32_t)(((k >> 32) << 16) | (k & 0xFFFF));
      uint32_t p = hash_narrow(key, h->table.shift);
      while (s[p].x != kEmptyKey) p = (p + 1) & h->table.mask;
      s[p] = make_uint2(key, (uint32_t)dict[k]);
    }
    host.resize(cap * sizeof(uint2));
    std::memcpy(host.data(), s.data(), host.size());
  } else {
    h->table.shift = 64 - log2cap;
    std::vector<uint4> s(cap, make_uint4(kEmptyKey, 0, 0, 0));
    for (uint64_t k : order) {
      uint32_t a = (uint32_t)(k >> 32), b = (uint32_t)k;
      uint32_t p = hash_wide(a, b, h->table.shift);
      while (s[p].x != kEmptyKey) p = (p + 1) & h->table.mask;
      s[p] = make_uint4(a, b, (uint32_t)dict[k], 0);
    }
    host.resize(cap * sizeof(uint4));
    std::memcpy(host.data(), s.data(), host.size());
  }
  DeviceGuard g(device);
  hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&h->d_table, host.size());
  if (e == hipSuccess) e = hipMemcpy(h->d_table, host.data(), host.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    sw_encoder_destroy(h);
    return fail(SW_ERR_HIP, std::string("sw_encoder_create: ") + hipGetErrorString(e));
  }
  h->table.slots = h->d_table;
  *out = h;
  return SW_OK;
}

extern "C" void sw_encoder_destroy(sw_encoder* h) {
  if (!h) return;
  {
    DeviceGuard g(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    free_workspace(h);
    free_io(h);
    (void)hipFree(h->d_table);
    for (hipEvent_t ev : h->ev_pool) (void)hipEventDestroy(ev);
    if (h->stream) (void)hipStreamDestroy(h->stream);
  }
  delete h;
}

extern "C" int32_t sw_encoder_reserve(sw_encoder* h, int64_t max_bytes, int64_t max_strings) {
  if (!h || max_bytes < 0 || max_strings < 0) return fail(SW_ERR_ARG, "sw_encoder_reserve: bad arguments");
  DeviceGuard g(h->device);
  return ensure_workspace(h, max_bytes);
}

extern "C" int32_t sw_encoder_set_timing(sw_encoder* h, int32_t on) {
  if (!h) return fail(SW_ERR_ARG, "sw_encoder_set_timing: null handle");
  h->timing = on != 0;
  h->ev_used = 0;
  return SW_OK;
}

// Average device time of k_encode_tiles over the launches recorded since the last
// sw_encoder_set_timing(h, 1); synchronises on the last recorded event.
extern "C" double sw_encoder_last_kernel_ms(const sw_encoder* h) {
  if (!h || h->ev_used == 0) return -1.0;
  DeviceGuard g(h->device);
  if (hipEventSynchronize(h->ev_pool[2 * h->ev_used - 1]) != hipSuccess) return -1.0;
  double sum = 0;
  for (size_t i = 0; i < h->ev_used; ++i) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, h->ev_pool[2 * i], h->ev_pool[2 * i + 1]) != hipSuccess) return -1.0;
    sum += ms;
  }
  return sum / (double)h->ev_used;
}

extern "C" int32_t sw_encode_device(sw_encoder* h, const uint8_t* d_bytes, int64_t n_bytes, const int64_t* d_str_off,
                                    int64_t n_str, const uint64_t* d_chunk_bits, int32_t* d_out_ids,
                                    int64_t* d_out_off, void* stream, int64_t* n_tokens_host) {
  if (!h || n_bytes < 0 || n_str < 0 || !d_str_off || !d_out_off || (n_bytes > 0 && (!d_bytes || !d_chunk_bits || !d_out_ids)))
    return fail(SW_ERR_ARG, "sw_encode_device: bad arguments");
  DeviceGuard g(h->device);
  hipStream_t st = stream ? (hipStream_t)stream : h->stream;
  int32_t rc = ensure_workspace(h, n_bytes);
  if (rc) return rc;
  const int64_t n_tiles = (n_bytes + kTile - 1) / kTile;
  if (n_tiles > 0) {
    TileArgs a;
    a.bytes = d_bytes; a.n_bytes = n_bytes; a.bits = d_chunk_bits; a.n_words = (n_bytes + 63) / 64;
    a.str_off = d_str_off; a.n_str = n_str; a.table = h->table;
    a.scratch = h->d_scratch; a.lw = h->d_lw; a.tile_cnt = h->d_tile_cnt; a.tile_first = h->d_tile_first;
    a.out_off = d_out_off;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->timing) {
      while (h->ev_pool.size() < 2 * (h->ev_used + 1)) {
        hipEvent_t ev;
        HIP_TRY(hipEventCreate(&ev));
        h->ev_pool.push_back(ev);
      }
      e0 = h->ev_pool[2 * h->ev_used];
      e1 = h->ev_pool[2 * h->ev_used + 1];
      HIP_TRY(hipEventRecord(e0, st));
    }
    hipLaunchKernelGGL(k_encode_tiles, dim3((unsigned)n_tiles), dim3(kThreads), 0, st, a);
    HIP_TRY(hipGetLastError());
    if (h->timing) {
      HIP_TRY(hipEventRecord(e1, st));
      ++h->ev_used;
    }
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, st, h->d_tile_cnt, n_tiles, h->d_tile_base, h->d_total);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_compact, dim3((unsigned)n_tiles), dim3(256), 0, st, h->d_scratch, h->d_tile_cnt,
                       h->d_tile_first, h->d_tile_base, d_out_ids);
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hipMemsetAsync(h->d_total, 0, sizeof(int64_t), st));
  }
  hipLaunchKernelGGL(k_string_offsets, dim3((unsigned)((n_str + 1 + 255) / 256)), dim3(256), 0, st, d_str_off, n_str,
                     n_bytes, h->d_tile_base, h->d_total, d_out_off);
  HIP_TRY(hipGetLastError());
  if (n_tokens_host) {
    HIP_TRY(hipMemcpyAsync(n_tokens_host, h->d_total, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  return SW_OK;
}

extern "C" int32_t sw_encode_batch(sw_encoder* h, const uint8_t* bytes, const int64_t* str_off, int64_t n_str,
                                   int32_t pattern, const uint64_t* chunk_bits, int32_t* out_ids, int64_t out_cap,
                                   int64_t* out_off, sw_stats* stats) {
  auto T0 = std::chrono::steady_clock::now();
  if (!h || !str_off || !out_off || n_str < 0) return fail(SW_ERR_ARG, "sw_encode_batch: bad arguments");
  const int64_t b0 = n_str > 0 ? str_off[0] : 0;
  const int64_t n_bytes = n_str > 0 ? str_off[n_str] - b0 : 0;
  if (n_bytes < 0 || (n_bytes > 0 && !bytes)) return fail(SW_ERR_ARG, "sw_encode_batch: bad string offsets");
  for (int64_t s = 0; s < n_str; ++s)
    if (str_off[s + 1] < str_off[s]) return fail(SW_ERR_ARG, "sw_encode_batch: string offsets not monotone");
  if (n_bytes > 0 && !out_ids) return fail(SW_ERR_ARG, "sw_encode_batch: null out_ids");
  const int64_t n_words = (n_bytes + 63) / 64;
  std::vector<uint64_t> own_bits;
  double ms_pre = 0;
  int64_t n_chunks = -1;
  if (!chunk_bits) {
    own_bits.resize((size_t)std::max<int64_t>(n_words, 1));
    auto a = std::chrono::steady_clock::now();
    n_chunks = sw_presplit_host(bytes, str_off, n_str, pattern, own_bits.data(), 0);
    if (n_chunks < 0) return fail((int32_t)n_chunks, "sw_encode_batch: bad pattern or offsets");
    ms_pre = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    chunk_bits = own_bits.data();
  }
  DeviceGuard g(h->device);
  // device staging (grown on demand)
  if (n_bytes > h->io_bytes || n_str > h->io_str) {
    free_io(h);
    const int64_t nb = std::max<int64_t>(n_bytes, 1), ns = std::max<int64_t>(n_str, 1);
    HIP_TRY(hipMalloc(&h->d_bytes, nb));
    HIP_TRY(hipMalloc(&h->d_str_off, sizeof(int64_t) * (ns + 1)));
    HIP_TRY(hipMalloc(&h->d_bits, sizeof(uint64_t) * ((nb + 63) / 64)));
    HIP_TRY(hipMalloc(&h->d_out, sizeof(int32_t) * nb));
    HIP_TRY(hipMalloc(&h->d_out_off, sizeof(int64_t) * (ns + 1)));
    h->io_bytes = nb; h->io_str = ns;
  }
  std::vector<int64_t> rel((size_t)n_str + 1);
  for (int64_t s = 0; s <= n_str; ++s) rel[s] = n_str > 0 ? str_off[s] - b0 : 0;
  auto a = std::chrono::steady_clock::now();
  hipStream_t st = h->stream;
  if (n_bytes > 0) {
    HIP_TRY(hipMemcpyAsync(h->d_bytes, bytes + b0, n_bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(h->d_bits, chunk_bits, sizeof(uint64_t) * n_words, hipMemcpyHostToDevice, st));
  }
  HIP_TRY(hipMemcpyAsync(h->d_str_off, rel.data(), sizeof(int64_t) * (n_str + 1), hipMemcpyHostToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));
  double ms_h2d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  int64_t n_tok = 0;
  const bool was_timing = h->timing;
  const size_t was_used = h->ev_used;
  h->timing = true;
  h->ev_used = 0;
  int32_t rc = sw_encode_device(h, h->d_bytes, n_bytes, h->d_str_off, n_str, h->d_bits, h->d_out, h->d_out_off,
                                st, &n_tok);
  const double k_ms = sw_encoder_last_kernel_ms(h);
  h->timing = was_timing;
  h->ev_used = was_timing ? was_used : 0;
  if (rc) return rc;
  if (n_tok > out_cap) return fail(SW_ERR_CAP, "sw_encode_batch: out_cap too small");
  a = std::chrono::steady_clock::now();
  if (n_tok > 0) HIP_TRY(hipMemcpyAsync(out_ids, h->d_out, sizeof(int32_t) * n_tok, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(out_off, h->d_out_off, sizeof(int64_t) * (n_str + 1), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  double ms_d2h = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  if (stats) {
    stats->n_bytes = n_bytes;
    stats->n_chunks = n_chunks;
    stats->n_tokens = n_tok;
    stats->ms_presplit = ms_pre;
    stats->ms_h2d = ms_h2d;
    stats->ms_kernels = k_ms;
    stats->ms_d2h = ms_d2h;
    stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count();
  }
  return SW_OK;
}
