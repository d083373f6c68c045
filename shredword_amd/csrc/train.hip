// MI355X-accelerated BPE trainer (include/shredword_train.h): the reference trainer's corpus-
// wide passes on the device, its heap and change bookkeeping on the host.
//
// Device layout (one corpus, resident for the whole training run):
//   ids    int32 [symbols]   every distinct word's symbols, words back to back in corpus order
//                            (word w from woff[w]; its live length len[w] shrinks as merges
//                            rewrite it in place)
//   wcnt   uint64 [words]    occurrences of each distinct word
//   ptab   pair histogram    open addressing, 24-byte slots {pair, frequency, first position}
//   dtab   change table      open addressing, 24-byte slots {pair hash, delta, first call}
// One thread per distinct word in both passes: words are short (a few symbols) and the rewrite
// of one word is sequential by definition (left to right, non-overlapping).  A pass reads every
// symbol once (~5 B per symbol with the lengths), so it is HBM/latency bound; the hash-table
// updates are 64-bit atomics on ~1 slot per occurrence of the merged pair.
//
// Host: the max-heap with lazy versions and the FreqChangeMap application order of the
// reference (bpe.cpp:486-517: hash % 1024 buckets ascending, newest first within a bucket),
// fed by the device's compacted change list: (pair hash, summed delta, first call).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "capi.h"
#include "shredword_hip.h"
#include "shredword_train.h"

namespace swt {

constexpr uint64_t kEmpty = 0x7FFFFFFFFFFFFFFFULL;  // no pair key or pair hash takes this value
constexpr int kBlock = 256;

struct Slot {  // (histogram: key, freq, first position; change table: hash, delta, first call)
  unsigned long long key;
  unsigned long long val;
  unsigned long long first;
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

// the slot holding key (claimed on first sight; its index appended to `used`)
__device__ __forceinline__ uint64_t slot_of(Slot* tab, uint64_t mask, uint64_t key, uint32_t* used,
                                            unsigned long long* n_used) {
  uint64_t i = mix64(key) & mask;
  for (;;) {
    unsigned long long cur = tab[i].key;
    if (cur == kEmpty) {
      cur = atomicCAS(&tab[i].key, kEmpty, (unsigned long long)key);
      if (cur == kEmpty) {
        used[atomicAdd(n_used, 1ULL)] = (uint32_t)i;
        return i;
      }
    }
    if (cur == key) return i;
    i = (i + 1) & mask;
  }
}

// slot_of with the first candidate's key already loaded (cur = tab[i].key, i = the key's home)
__device__ __forceinline__ uint64_t slot_of_from(Slot* tab, uint64_t mask, uint64_t key, uint64_t i,
                                                 unsigned long long cur, uint32_t* used, unsigned long long* n_used) {
  for (;;) {
    if (cur == kEmpty) {
      cur = atomicCAS(&tab[i].key, kEmpty, (unsigned long long)key);
      if (cur == kEmpty) {
        used[atomicAdd(n_used, 1ULL)] = (uint32_t)i;
        return i;
      }
    }
    if (cur == key) return i;
    i = (i + 1) & mask;
    cur = tab[i].key;
  }
}

__global__ void k_init(Slot* tab, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    tab[i].key = kEmpty;
    tab[i].val = 0;
    tab[i].first = ~0ULL;
  }
}

// bpe_count_bigrams (bpe.cpp:329-355): every pair without an unk member, weighted by the word's
// count; `first` = the pair's first position in corpus order (the BIMap insertion order)
__global__ void k_count_pairs(const int32_t* ids, const int64_t* woff, const int32_t* len, const uint64_t* wcnt,
                              int64_t nw, int32_t unk, Slot* tab, uint64_t mask, uint32_t* used,
                              unsigned long long* n_used) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  const int64_t base = woff[w];
  const int L = len[w];
  const unsigned long long wc = wcnt[w];
  int32_t a = L > 0 ? ids[base] : 0;
  for (int k = 0; k + 1 < L; ++k) {
    const int32_t b = ids[base + k + 1];
    if (a != unk && b != unk) {
      const uint64_t key = ((uint64_t)(uint32_t)a << 32) | (uint32_t)b;
      const uint64_t s = slot_of(tab, mask, key, used, n_used);
      atomicAdd(&tab[s].val, wc);
      atomicMin(&tab[s].first, (unsigned long long)(base + k));
    }
    a = b;
  }
}

// the reference's change key: ((u64)(i64)first << 32) | (u64)(i64)second (bpe.cpp:456-467)
__device__ __forceinline__ uint64_t phash(int32_t f, int32_t s) {
  return ((uint64_t)(int64_t)f << 32) | (uint64_t)(int64_t)s;
}

// bpe_merge_batch's rewrite (bpe.cpp:437-483) of every word containing (A, B): in place, left
// to right; each replaced pair's left neighbour (already rewritten) and right neighbour (not
// yet) move their frequency to the pairs with X.  A change's `first` is its call's rank in the
// reference's freq_change_add order: 4 * (word start) + call index within the word.
__device__ __forceinline__ uint64_t sym_bit(int32_t id) { return 1ULL << ((uint32_t)id & 63u); }

// per word: a 64-bit filter of the symbol ids it holds (bit id % 64); a merge reads only the
// filters of the words that cannot hold its pair, ~5 B per symbol less
__global__ void k_bloom_init(const int32_t* ids, const int64_t* woff, const int32_t* len, int64_t nw, uint64_t* bloom) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  uint64_t f = 0;
  for (int k = 0, L = len[w]; k < L; ++k) f |= sym_bit(ids[woff[w] + k]);
  bloom[w] = f;
}

// (bl, base, L, wcw: the word's filter, start, live length and count, loaded by the caller)
__device__ __forceinline__ bool merge_word_pre(int32_t* ids, int32_t* len, uint64_t* bloom, int64_t w, uint64_t bl,
                                               int64_t base, int L, uint64_t wcw, int32_t A, int32_t B, int32_t X,
                                               Slot* tab, uint64_t mask, uint32_t* used, unsigned long long* n_used) {
  const uint64_t need = sym_bit(A) | sym_bit(B);
  if ((bl & need) != need) return false;
  int32_t* s = ids + base;
  int r = 0;
  while (r + 1 < L && !(s[r] == A && s[r + 1] == B)) ++r;  // (most words: read only)
  if (r + 1 >= L) return false;
  const long long wc = (long long)wcw;
  unsigned long long call = 4ULL * (unsigned long long)base;
  // an occurrence's (up to) four changes, in the reference's call order: their home slots' keys
  // are loaded together (one memory round trip instead of four), then each is resolved
  auto add4 = [&](bool left, int32_t pv, bool right, int32_t nx) {
    uint64_t h[4], home[4];
    unsigned long long cur[4];
    const bool on[4] = {left, left, right, right};
    h[0] = phash(pv, A); h[1] = phash(pv, X); h[2] = phash(B, nx); h[3] = phash(X, nx);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      home[k] = mix64(h[k]) & mask;
      cur[k] = on[k] ? tab[home[k]].key : 0ULL;
    }
    const long long d[4] = {-wc, wc, -wc, wc};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!on[k]) continue;
      const uint64_t i = slot_of_from(tab, mask, h[k], home[k], cur[k], used, n_used);
      atomicAdd(&tab[i].val, (unsigned long long)d[k]);
      atomicMin(&tab[i].first, call++);
    }
  };
  int o = r;
  while (r < L) {
    if (r + 1 < L && s[r] == A && s[r + 1] == B) {
      add4(o > 0, o > 0 ? s[o - 1] : 0, r + 2 < L, r + 2 < L ? s[r + 2] : 0);
      s[o++] = X;
      r += 2;
    } else {
      s[o++] = s[r++];
    }
  }
  len[w] = o;
  uint64_t f = 0;
  for (int k = 0; k < o; ++k) f |= sym_bit(s[k]);
  bloom[w] = f;
  return true;
}

__device__ __forceinline__ bool merge_word(int32_t* ids, const int64_t* woff, int32_t* len, const uint64_t* wcnt,
                                           uint64_t* bloom, int64_t w, int32_t A, int32_t B, int32_t X, Slot* tab,
                                           uint64_t mask, uint32_t* used, unsigned long long* n_used) {
  const uint64_t need = sym_bit(A) | sym_bit(B);
  const uint64_t bl = bloom[w];
  if ((bl & need) != need) return false;
  return merge_word_pre(ids, len, bloom, w, bl, woff[w], len[w], wcnt[w], A, B, X, tab, mask, used, n_used);
}

// the rewrite of every word containing (A, B): one thread per word
__global__ void __launch_bounds__(kBlock) k_merge_words(int32_t* ids, const int64_t* woff, int32_t* len,
                                                        const uint64_t* wcnt, uint64_t* bloom, int64_t nw, int32_t A,
                                                        int32_t B, int32_t X, Slot* tab, uint64_t mask, uint32_t* used,
                                                        unsigned long long* n_used) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < nw) merge_word(ids, woff, len, wcnt, bloom, w, A, B, X, tab, mask, used, n_used);
}

__device__ __forceinline__ void merge_cand(int32_t* ids, const int64_t* woff, int32_t* len, const uint64_t* wcnt,
                                           uint64_t* bloom, const uint32_t* c0, int64_t n0, const uint32_t* c1,
                                           int64_t n1, const uint32_t* c2, int64_t n2, uint32_t* stamp, uint32_t seq,
                                           int32_t A, int32_t B, int32_t X, Slot* tab, uint64_t mask, uint32_t* used,
                                           unsigned long long* n_used, uint32_t* pool, unsigned long long* pool_n,
                                           uint64_t pool_cap, unsigned int* overflow, int64_t i) {
  bool done = false;
  uint32_t w = 0;
  if (i < n0 + n1 + n2) {
    w = i < n0 ? c0[i] : i < n0 + n1 ? c1[i - n0] : c2[i - n0 - n1];
    // the word's filter, start, length and count in one round trip; a word whose filter lacks A
    // or B is dropped before any atomic.  The others load their first kRegIds symbols beside the
    // stamp claim (one more round trip: nothing else rewrites the word in this step, so reading
    // before the claim is safe) and a word without the pair among them is read only once.
    const uint64_t bl = bloom[w];
    const int64_t base = woff[w];
    const int L = len[w];
    const uint64_t wcw = wcnt[w];
    const uint64_t need = sym_bit(A) | sym_bit(B);
    if ((bl & need) == need) {
      constexpr int kRegIds = 16;
      int32_t v[kRegIds];
#pragma unroll
      for (int k = 0; k < kRegIds; ++k) v[k] = k < L ? ids[base + k] : 0;
      bool has = L > kRegIds;  // (longer words: the scan in merge_word_pre decides)
#pragma unroll
      for (int k = 0; k + 1 < kRegIds; ++k) has |= k + 1 < L && v[k] == A && v[k + 1] == B;
      if (atomicExch(&stamp[w], seq) != seq && has)
        done = merge_word_pre(ids, len, bloom, w, bl, base, L, wcw, A, B, X, tab, mask, used, n_used);
    }
  }
  const uint64_t m = __ballot(done);  // (one pool append per wave)
  if (!m) return;
  const int lane = threadIdx.x & 63;
  unsigned long long base = 0;
  if (lane == __builtin_ctzll(m)) base = atomicAdd(pool_n, (unsigned long long)__popcll(m));
  base = __shfl(base, __builtin_ctzll(m), 64);
  if (done) {
    const uint64_t k = base + __popcll(m & ((1ULL << lane) - 1ULL));
    if (k < pool_cap) pool[k] = w;
    else atomicOr(overflow, 1u);
  }
}

// Per-pair word lists: the words that can hold (A, B) at a merge are those where A and B were
// adjacent in the loaded corpus (`init`: every adjacent pair's words, sorted by pair), those
// where the merge that created A rewrote something, and those where B's did (`pool`: the words
// each merge rewrote, in merge order) -- a merge only ever makes pairs with the token it creates.
// One thread per candidate (three ranges); a word listed twice is taken once (its stamp).
__global__ void __launch_bounds__(kBlock) k_merge_cand(int32_t* ids, const int64_t* woff, int32_t* len,
                                                       const uint64_t* wcnt, uint64_t* bloom, const uint32_t* c0,
                                                       int64_t n0, const uint32_t* c1, int64_t n1, const uint32_t* c2,
                                                       int64_t n2, uint32_t* stamp, uint32_t seq, int32_t A, int32_t B,
                                                       int32_t X, Slot* tab, uint64_t mask, uint32_t* used,
                                                       unsigned long long* n_used, uint32_t* pool,
                                                       unsigned long long* pool_n, uint64_t pool_cap,
                                                       unsigned int* overflow) {
  merge_cand(ids, woff, len, wcnt, bloom, c0, n0, c1, n1, c2, n2, stamp, seq, A, B, X, tab, mask, used, n_used, pool,
             pool_n, pool_cap, overflow, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// the initial pair -> words list: every adjacent pair's key and its word (then sorted by key)
__global__ void k_pair_words(const int32_t* ids, const int64_t* woff, const int32_t* len, int64_t nw,
                             uint64_t* keys, uint32_t* words) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  const int64_t base = woff[w];
  for (int k = 0, L = len[w]; k + 1 < L; ++k) {  // (entry base + k - w: every word's first position skipped)
    keys[base + k - w] = ((uint64_t)(uint32_t)ids[base + k] << 32) | (uint32_t)ids[base + k + 1];
    words[base + k - w] = (uint32_t)w;
  }
}

// a merge step's changes, by ONE workgroup after k_merge_words: the claimed slots, densely (the
// first `hcap` straight into host-coherent memory), cleared with their counter; then the record
// count and the step's sequence number for the host, which spins on it instead of synchronising
// the stream.  (One workgroup: a grid would need a device-scope fence per block to know when all
// are done, which on a multi-XCD part costs more than the whole step.)
__device__ __forceinline__ void collect_step(Slot* tab, const uint32_t* used, unsigned long long* n_used, Slot* out,
                                             Slot* hout, unsigned long long* hcount, unsigned long long* hseq,
                                             unsigned long long seq, uint64_t hcap, const unsigned long long* pool_n,
                                             const unsigned int* overflow) {
  const uint64_t n = __hip_atomic_load(n_used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    Slot& sl = tab[used[i]];
    Slot v;  // (atomic loads: the slots were updated by atomics of other workgroups)
    v.key = __hip_atomic_load(&sl.key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v.val = __hip_atomic_load(&sl.val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v.first = __hip_atomic_load(&sl.first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (i < hcap) hout[i] = v;
    else out[i] = v;
    sl.key = kEmpty;
    sl.val = 0;
    sl.first = ~0ULL;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    *n_used = 0;
    hcount[0] = n;
    hcount[2] = __hip_atomic_load(pool_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (words rewritten so far,
    hcount[3] = __hip_atomic_load(overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // list overflow)
    __threadfence_system();
    __hip_atomic_store(hseq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void __launch_bounds__(1024) k_collect_step(Slot* tab, const uint32_t* used, unsigned long long* n_used,
                                                       Slot* out, Slot* hout, unsigned long long* hcount,
                                                       unsigned long long* hseq, unsigned long long seq, uint64_t hcap,
                                                       const unsigned long long* pool_n, const unsigned int* overflow) {
  collect_step(tab, used, n_used, out, hout, hcount, hseq, seq, hcap, pool_n, overflow);
}

// a merge over few candidates (<= kFuseBlocks workgroups) in ONE launch: the candidates, then the
// last workgroup to finish (a ticket after a device-scope fence: a few fences, not thousands)
// collects the changes and publishes them
constexpr unsigned kFuseBlocks = 16;
__global__ void __launch_bounds__(kBlock) k_merge_cand_fused(
    int32_t* ids, const int64_t* woff, int32_t* len, const uint64_t* wcnt, uint64_t* bloom, const uint32_t* c0,
    int64_t n0, const uint32_t* c1, int64_t n1, const uint32_t* c2, int64_t n2, uint32_t* stamp, uint32_t seq, int32_t A,
    int32_t B, int32_t X, Slot* tab, uint64_t mask, uint32_t* used, unsigned long long* n_used, uint32_t* pool,
    unsigned long long* pool_n, uint64_t pool_cap, unsigned int* overflow, unsigned int* ticket, Slot* out, Slot* hout,
    unsigned long long* hcount, unsigned long long* hseq, unsigned long long hseq_val, uint64_t hcap) {
  merge_cand(ids, woff, len, wcnt, bloom, c0, n0, c1, n1, c2, n2, stamp, seq, A, B, X, tab, mask, used, n_used, pool,
             pool_n, pool_cap, overflow, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  __shared__ bool last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  if (threadIdx.x == 0) *ticket = 0;
  collect_step(tab, used, n_used, out, hout, hcount, hseq, hseq_val, hcap, pool_n, overflow);
}

// the table's claimed slots, densely (the first `hcap` also into host-mapped memory, with the
// count), then cleared for the next pass; n_used counts this pass, next_used (the next pass's
// counter) is reset here, so no separate memset runs between passes
__global__ void k_collect(Slot* tab, const uint32_t* used, const unsigned long long* n_used,
                          unsigned long long* next_used, Slot* out, Slot* hout, unsigned long long* hcount,
                          uint64_t hcap) {
  const uint64_t n = *n_used;
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid == 0) {
    *next_used = 0;
    *hcount = n;
  }
  for (uint64_t i = gid; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    Slot& t = tab[used[i]];
    const Slot v = t;
    out[i] = v;
    if (i < hcap) hout[i] = v;
    t.key = kEmpty;
    t.val = 0;
    t.first = ~0ULL;
  }
}

// final token frequencies over the rewritten corpus (bpe_save :703-712; negative ids skipped)
__global__ void k_tok_freq(const int32_t* ids, const int64_t* woff, const int32_t* len, const uint64_t* wcnt, int64_t nw,
                           int64_t n_tok, unsigned long long* freq) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  const unsigned long long c = wcnt[w];
  for (int k = 0, L = len[w]; k < L; ++k) {
    const int32_t id = ids[woff[w] + k];
    if (id >= 0 && id < n_tok) atomicAdd(&freq[id], c);
  }
}

// ---------------------------------------------------------------------------------------------
// corpus load on the device (bpe_load_corpus, bpe.cpp:208-297): words = maximal runs of
// non-delimiter bytes, counted per distinct word (first occurrence = smallest offset), ordered
// as the reference's StrMap iterates (djb2 & 4095 bucket, then first occurrence), the character
// histogram over the distinct words, then the symbols written in that order
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool d_delim(uint8_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }

// word starts (a non-delimiter after a delimiter or at 0); a NUL byte anywhere sets *bad
__global__ void k_word_flags(const uint8_t* text, int64_t n, uint8_t* flags, unsigned int* bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t c = text[i];
    if (c == 0) atomicOr(bad, 1u);
    flags[i] = (!d_delim(c) && (i == 0 || d_delim(text[i - 1]))) ? 1 : 0;
  }
}

__device__ __forceinline__ uint64_t d_word_hash(const uint8_t* p, int64_t n) {  // FNV-1a 64 + finaliser
  uint64_t h = 1469598103934665603ULL;
  for (int64_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ULL;
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ULL;
  return h ^ (h >> 32);
}

__global__ void k_iota(uint32_t* v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = (uint32_t)i;
}

// every word occurrence's 64-bit hash (the sort key) and start
__global__ void k_word_hash(const uint8_t* text, int64_t n, const int64_t* starts, const int64_t* n_words,
                            uint64_t* keys, uint64_t* vals) {
  const int64_t nwd = *n_words;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwd; w += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = starts[w];
    int64_t e = s;
    while (e < n && !d_delim(text[e])) ++e;
    keys[w] = d_word_hash(text + s, e - s);
    vals[w] = (uint64_t)s;
  }
}

// after the (stable) sort by hash: run heads (an occurrence whose hash differs from the one before)
__global__ void k_run_heads(const uint64_t* skeys, int64_t m, int64_t* head) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
    head[i] = (i == 0 || skeys[i] != skeys[i - 1]) ? i : 0;
}

// exactness: every occurrence equals its run's first occurrence byte for byte (a 64-bit hash
// collision between two distinct words sets *bad, and the load falls back to the host)
__global__ void k_word_verify(const uint8_t* text, int64_t n, const uint64_t* svals, const int64_t* headidx, int64_t m,
                              unsigned int* bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = (int64_t)svals[i], r = (int64_t)svals[headidx[i]];
    if (s == r) continue;
    int64_t q = 0;
    while (s + q < n && r + q < n && !d_delim(text[s + q]) && text[s + q] == text[r + q]) ++q;
    const bool end_s = s + q >= n || d_delim(text[s + q]), end_r = r + q >= n || d_delim(text[r + q]);
    if (!(end_s && end_r)) atomicOr(bad, 1u);
  }
}

// the distinct words (one per run): first occurrence (the run's first: the sort is stable and
// the occurrences were in corpus order), count, length, and the StrMap order key (djb2 & 4095,
// then the first occurrence: hash.cpp:29-53, 61-72)
__global__ void k_word_runs(const uint8_t* text, int64_t n, const uint64_t* svals, const int64_t* roff,
                            const int64_t* n_runs, uint64_t* first, uint64_t* cnt, uint32_t* wlen, uint64_t* keys) {
  const int64_t nd = *n_runs;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nd; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t f = svals[roff[r]];
    uint64_t h = 5381;
    int64_t e = (int64_t)f;
    while (e < n && !d_delim(text[e])) {
      h = (h << 5) + h + text[e];
      ++e;
    }
    first[r] = f;
    cnt[r] = (uint64_t)(roff[r + 1] - roff[r]);
    wlen[r] = (uint32_t)(e - (int64_t)f);
    keys[r] = ((h & 4095u) << 52) | f;
  }
}

// the character histogram over the distinct words (histogram.cpp:30-36: each distinct word's
// bytes once), per block in LDS; and each word's length and count in StrMap order
__global__ void k_word_hist(const uint8_t* text, const uint64_t* first, const uint32_t* wlen, const uint64_t* cnt,
                            const uint32_t* order, int64_t nd, unsigned long long* hist, int64_t* len_out,
                            int32_t* len32, uint64_t* cnt_out) {
  __shared__ unsigned int h[256];
  for (int c = threadIdx.x; c < 256; c += blockDim.x) h[c] = 0;
  __syncthreads();
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nd; j += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = order[j];
    const uint64_t f = first[r];
    const uint32_t L = wlen[r];
    for (uint32_t q = 0; q < L; ++q) atomicAdd(&h[text[f + q]], 1u);
    len_out[j] = L;
    len32[j] = (int32_t)L;
    cnt_out[j] = cnt[r];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 256; c += blockDim.x)
    if (h[c]) atomicAdd(&hist[c], (unsigned long long)h[c]);
}

// the symbols: word j's bytes through the coverage map, at woff[j]
__global__ void k_word_ids(const uint8_t* text, const uint64_t* first, const uint32_t* wlen, const uint32_t* order,
                           const int64_t* woff, int64_t nd, const int32_t* map, int32_t* ids) {
  __shared__ int32_t m[256];
  for (int c = threadIdx.x; c < 256; c += blockDim.x) m[c] = map[c];
  __syncthreads();
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nd; j += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = order[j];
    const uint64_t f = first[r];
    int32_t* d = ids + woff[j];
    for (uint32_t q = 0, L = wlen[r]; q < L; ++q) d[q] = m[text[f + q]];
  }
}

// ---------------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------------
struct HeapEntry {
  int32_t a, b;
  uint64_t freq;
  uint32_t version;
};

// heap_push / heap_pop (heap.cpp:53-114): ties fall where these sift rules put them.  The same
// binary heap (parent >= child on push, the larger child taken only if strictly larger on pop),
// laid out for the cache: 16-byte nodes {a, b, freq << 24 | version}, 1-based in a 64-byte
// aligned array, so a node's two children share a half line and its four grandchildren one line,
// prefetched two levels ahead of the sift-down (a pop walks ~20 levels of a 1 M-entry heap of
// mostly stale entries; the stale pops outnumber the merges ~16:1).  freq < 2^40 and
// version < 2^24 (checked: overflow() -> SW_ERR_CAP).
struct MaxHeap {
  struct Node {
    int32_t a, b;
    uint64_t fv;
  };
  static_assert(sizeof(Node) == 16, "16-byte heap nodes");
  static constexpr int kVerBits = 24;
  Node* d = nullptr;
  size_t n = 0, cap = 0;
  bool over = false;
  MaxHeap() = default;
  MaxHeap(const MaxHeap&) = delete;
  MaxHeap& operator=(const MaxHeap&) = delete;
  ~MaxHeap() { std::free(d); }
  static uint64_t freq_of(uint64_t fv) { return fv >> kVerBits; }
  bool empty() const { return n == 0; }
  size_t size() const { return n; }
  bool overflow() const { return over; }
  void reserve(size_t want) {
    if (want + 1 <= cap) return;
    size_t c = 1024;
    while (c < want + 1) c <<= 1;
    Node* nd = static_cast<Node*>(std::aligned_alloc(64, c * sizeof(Node)));
    if (!nd) throw std::bad_alloc();
    if (d) std::memcpy(nd, d, (n + 1) * sizeof(Node));
    std::free(d);
    d = nd;
    cap = c;
  }
  HeapEntry top() const { return decode(d[1]); }
  static HeapEntry decode(const Node& x) {
    return HeapEntry{x.a, x.b, freq_of(x.fv), (uint32_t)(x.fv & ((1u << kVerBits) - 1u))};
  }
  void push(int32_t a, int32_t b, uint64_t freq, uint32_t version) {
    if ((freq >> (64 - kVerBits)) != 0 || (version >> kVerBits) != 0) over = true;
    if (n + 2 > cap) reserve(2 * n + 2);
    const Node x{a, b, (freq << kVerBits) | (version & ((1u << kVerBits) - 1u))};
    const uint64_t f = freq_of(x.fv);
    size_t i = ++n;
    while (i > 1) {
      const size_t p = i >> 1;
      if (freq_of(d[p].fv) >= f) break;
      d[i] = d[p];
      i = p;
    }
    d[i] = x;
  }
  HeapEntry pop() {
    const Node top = d[1];
    const Node x = d[n];
    --n;
    if (n > 0) {
      const uint64_t f = freq_of(x.fv);
      size_t i = 1;
      for (;;) {
        if (8 * i + 4 < cap) {
          __builtin_prefetch(&d[8 * i]);
          __builtin_prefetch(&d[8 * i + 4]);
        }
        const size_t l = 2 * i, r = l + 1;
        size_t best = i;
        uint64_t bf = f;
        if (l <= n && freq_of(d[l].fv) > bf) { best = l; bf = freq_of(d[l].fv); }
        if (r <= n && freq_of(d[r].fv) > bf) best = r;
        if (best == i) break;
        d[i] = d[best];
        i = best;
      }
      d[i] = x;
    }
    return decode(top);
  }
};

struct PairInfo {
  uint64_t freq = 0;
  uint32_t version = 0;
};

// pair -> PairInfo, open addressing (the BIMap's role, hash.cpp:104-130; its iteration order
// only matters for the heap seed, which is sorted explicitly).  Key and value in one 24-byte
// entry (one cache miss a lookup); prefetch() lets the change pass issue its misses early.
class PairMap {
 public:
  explicit PairMap(size_t n) { rehash(n); }
  PairInfo& operator[](uint64_t key) {  // get or create (freq 0, version 0)
    if (2 * (n_ + 1) > e_.size()) rehash(e_.size());
    size_t i = slot(key);
    if (e_[i].key != key) {
      e_[i].key = key;
      e_[i].v = PairInfo{};
      ++n_;
    }
    return e_[i].v;
  }
  void prefetch(uint64_t key) const { __builtin_prefetch(&e_[(size_t)mix(key) & (e_.size() - 1)], 1); }

 private:
  struct E {
    uint64_t key;
    PairInfo v;
  };
  static uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    return x ^ (x >> 33);
  }
  size_t slot(uint64_t key) const {
    size_t i = (size_t)mix(key) & (e_.size() - 1);
    while (e_[i].key != key && e_[i].key != kEmpty) i = (i + 1) & (e_.size() - 1);
    return i;
  }
  void rehash(size_t n) {
    size_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    std::vector<E> old;
    old.swap(e_);
    e_.assign(cap, E{kEmpty, PairInfo{}});
    n_ = 0;
    for (const E& x : old)
      if (x.key != kEmpty) (*this)[x.key] = x.v;
  }
  std::vector<E> e_;
  size_t n_ = 0;
};

inline uint64_t pkey(int32_t a, int32_t b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

// BIMap bucket (hash.cpp:7-16, 109-110): FNV-1a over the 8-byte PairKey, 4096 buckets
inline uint32_t bimap_bucket(int32_t a, int32_t b) {
  uint8_t by[8];
  std::memcpy(by, &a, 4);
  std::memcpy(by + 4, &b, 4);
  uint32_t h = 2166136261u;
  for (uint8_t c : by) {
    h ^= c;
    h *= 16777619u;
  }
  return h & 4095u;
}

inline bool is_delim(uint8_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace swt

using namespace swt;

struct sw_trainer {
  sw_train_config cfg{};
  int device = 0;
  hipStream_t st = nullptr;
  // the loaded corpus, on the device (training rewrites copies of ids and len): every distinct
  // word's symbols back to back in StrMap order, its offset, length and count
  int32_t* d_ids0 = nullptr;
  int64_t* d_woff0 = nullptr;
  int32_t* d_len0 = nullptr;
  uint64_t* d_wcnt0 = nullptr;
  int64_t nw = 0, ns = 0;
  bool loaded = false;
  bool host_load = false;             // the last load took the host path (SW_TRAIN_HOST_LOAD, or a hash collision)
  // results
  std::vector<int32_t> merges;   // 3 per merge
  std::vector<uint64_t> tok_freq;
  double stats[8] = {0};
  // device
  int32_t* d_ids = nullptr;
  int64_t* d_woff = nullptr;
  int32_t* d_len = nullptr;
  uint64_t* d_wcnt = nullptr;
  uint64_t* d_bloom = nullptr;        // per word: symbol-id filter (k_bloom_init)
  Slot* d_tab = nullptr;
  Slot* d_out = nullptr;
  uint32_t* d_used = nullptr;
  unsigned long long* d_nused = nullptr;  // two pass counters, used alternately
  int pass = 0;
  uint64_t tab_mask = 0;
  Slot* h_out = nullptr;          // pinned, device-mapped: the first kPinnedRecords changes
  unsigned long long* h_nused = nullptr;
  Slot* h_out_dev = nullptr;      // (their device-side addresses)
  unsigned long long* h_nused_dev = nullptr;
  int64_t out_cap = 0;
  // merge steps (k_merge_words + k_collect_step): device counter, and host-coherent records + count + sequence
  unsigned long long* d_step_used = nullptr;
  // per-pair word lists (k_merge_cand): the initial pair -> words list, the rewritten-words pool
  uint32_t* d_pwords = nullptr;
  unsigned int* d_ticket = nullptr;
  uint32_t* d_stamp = nullptr;
  uint32_t* d_pool = nullptr;
  unsigned long long* d_pool_n = nullptr;
  unsigned int* d_overflow = nullptr;
  Slot* h_rec = nullptr;
  unsigned long long* h_cnt = nullptr;   // [0] record count, [1] sequence number
  Slot* h_rec_dev = nullptr;
  unsigned long long* h_cnt_dev = nullptr;
};

namespace {

constexpr int64_t kPinnedRecords = 4096;  // change records fetched with the count (more: a second copy)

void free_corpus(sw_trainer* t) {
  (void)hipFree(t->d_ids0); (void)hipFree(t->d_woff0); (void)hipFree(t->d_len0); (void)hipFree(t->d_wcnt0);
  t->d_ids0 = nullptr; t->d_woff0 = nullptr; t->d_len0 = nullptr; t->d_wcnt0 = nullptr;
  t->nw = t->ns = 0;
  t->loaded = false;
}

void free_device(sw_trainer* t) {
  (void)hipFree(t->d_ids); (void)hipFree(t->d_woff); (void)hipFree(t->d_len); (void)hipFree(t->d_wcnt);
  (void)hipFree(t->d_bloom);
  t->d_bloom = nullptr;
  (void)hipFree(t->d_tab); (void)hipFree(t->d_out); (void)hipFree(t->d_used); (void)hipFree(t->d_nused);
  (void)hipHostFree(t->h_out); (void)hipHostFree(t->h_nused);
  (void)hipFree(t->d_step_used);
  (void)hipFree(t->d_pwords); (void)hipFree(t->d_stamp); (void)hipFree(t->d_pool); (void)hipFree(t->d_pool_n);
  (void)hipFree(t->d_overflow); (void)hipFree(t->d_ticket);
  t->d_ticket = nullptr;
  t->d_pwords = nullptr; t->d_stamp = nullptr; t->d_pool = nullptr; t->d_pool_n = nullptr; t->d_overflow = nullptr;
  (void)hipHostFree(t->h_rec); (void)hipHostFree(t->h_cnt);
  t->d_step_used = nullptr; t->h_rec = nullptr; t->h_cnt = nullptr;
  t->h_rec_dev = nullptr; t->h_cnt_dev = nullptr;
  t->d_ids = nullptr; t->d_woff = nullptr; t->d_len = nullptr; t->d_wcnt = nullptr; t->d_tab = nullptr;
  t->d_out = nullptr; t->d_used = nullptr; t->d_nused = nullptr; t->h_out = nullptr; t->h_nused = nullptr;
  t->h_out_dev = nullptr; t->h_nused_dev = nullptr;
}

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

// distinct words of one text range: open addressing over (64-bit hash, first offset, length, count)
struct WordTable {
  struct E {
    uint64_t h;
    int64_t off;
    int64_t len;
    uint64_t cnt;
  };
  std::vector<E> e;
  size_t n = 0;
  explicit WordTable(size_t cap) {
    size_t c = 1024;
    while (c < 2 * cap) c <<= 1;
    e.assign(c, E{0, -1, 0, 0});
  }
  void grow(const uint8_t* text) {
    std::vector<E> old;
    old.swap(e);
    e.assign(old.size() * 2, E{0, -1, 0, 0});
    n = 0;
    for (const E& x : old)
      if (x.off >= 0) add(text, x.h, x.off, x.len, x.cnt);
  }
  // count cnt occurrences of text[off, off + len) (first seen at off if new)
  void add(const uint8_t* text, uint64_t h, int64_t off, int64_t len, uint64_t cnt) {
    if (2 * (n + 1) > e.size()) grow(text);
    size_t i = (size_t)(h & (e.size() - 1));
    for (;;) {
      E& x = e[i];
      if (x.off < 0) {
        x = E{h, off, len, cnt};
        ++n;
        return;
      }
      if (x.h == h && x.len == len && std::memcmp(text + x.off, text + off, (size_t)len) == 0) {
        x.cnt += cnt;
        if (off < x.off) x.off = off;
        return;
      }
      i = (i + 1) & (e.size() - 1);
    }
  }
};

inline uint64_t word_hash(const uint8_t* p, int64_t n) {  // FNV-1a 64, then a finaliser
  uint64_t h = 1469598103934665603ULL;
  for (int64_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ULL;
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ULL;
  return h ^ (h >> 32);
}

// bpe_load_corpus (bpe.cpp:208-297) restated over a buffer: the text's ranges are counted by
// host threads in parallel (the first occurrence of a word = its smallest offset), then merged
// character coverage (bpe.cpp:256-279): chars in StrMap order ((c + 165) & 255), stable by
// count, the first (size_t)(n * coverage) kept; the others map to unk_id
void coverage_map(const uint64_t (&ch)[256], const sw_train_config& cfg, int32_t (&map)[256]) {
  std::vector<int> chars;
  for (int b = 0; b < 256; ++b) {
    const int c = (b + 91) & 255;
    if (ch[c]) chars.push_back(c);
  }
  std::stable_sort(chars.begin(), chars.end(), [&](int x, int y) { return ch[x] > ch[y]; });
  float cov = cfg.character_coverage;
  if (!(cov > 0.0f && cov < 1.0f)) cov = 0.995f;
  const size_t keep = (size_t)((float)chars.size() * cov);
  for (int c = 0; c < 256; ++c) map[c] = cfg.unk_id;
  for (size_t k = 0; k < keep && k < chars.size(); ++k) map[chars[k]] = chars[k];
}

int32_t load_words(sw_trainer* t, const uint8_t* text, int64_t n) {
  if (n > 0 && std::memchr(text, 0, (size_t)n)) return sw::set_error(SW_ERR_ARG, "sw_trainer: the corpus holds NUL bytes");
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(),
                                                           n / (1 << 20) + 1}));
  std::vector<int64_t> cut(T + 1, n);
  cut[0] = 0;
  for (int k = 1; k < T; ++k) {  // range starts moved past the word in progress
    int64_t c = std::max(cut[k - 1], n * k / T);
    while (c < n && c > 0 && !is_delim(text[c - 1])) ++c;
    cut[k] = c;
  }
  std::vector<WordTable> local;
  local.reserve(T);
  for (int k = 0; k < T; ++k) local.emplace_back((size_t)((cut[k + 1] - cut[k]) / 64 + 16));
  auto count_range = [&](int k) {
    for (int64_t i = cut[k], e = cut[k + 1]; i < e;) {
      while (i < e && is_delim(text[i])) ++i;
      const int64_t s = i;
      while (i < e && !is_delim(text[i])) ++i;
      if (i > s) local[k].add(text, word_hash(text + s, i - s), s, i - s, 1);
    }
  };
  auto run = [&](auto&& fn) {
    std::vector<std::thread> th;
    for (int k = 1; k < T; ++k) th.emplace_back(fn, k);
    fn(0);
    for (auto& x : th) x.join();
  };
  run(count_range);
  // merge by hash partition: every range scatters its words by hash % T (in range order, so the
  // smallest offset of a word arrives first), then partition p merges its share
  struct Item {
    uint64_t h;
    int64_t off, len;
    uint64_t cnt;
  };
  std::vector<std::vector<std::vector<Item>>> out((size_t)T, std::vector<std::vector<Item>>((size_t)T));
  run([&](int k) {
    for (const auto& x : local[k].e)
      if (x.off >= 0) out[k][(size_t)((x.h >> 40) % (uint64_t)T)].push_back(Item{x.h, x.off, x.len, x.cnt});
    std::vector<WordTable::E>().swap(local[k].e);
  });
  std::vector<WordTable> part;
  part.reserve(T);
  for (int p = 0; p < T; ++p) {
    size_t m = 16;
    for (int k = 0; k < T; ++k) m += out[k][p].size();
    part.emplace_back(m);
  }
  run([&](int p) {
    for (int k = 0; k < T; ++k)
      for (const Item& x : out[k][p]) part[p].add(text, x.h, x.off, x.len, x.cnt);
  });
  std::vector<int64_t> pbase(T + 1, 0);
  for (int p = 0; p < T; ++p) pbase[p + 1] = pbase[p] + (int64_t)part[p].n;
  const int64_t nw = pbase[T];
  std::vector<int64_t> woff0((size_t)nw), wlen0((size_t)nw), first((size_t)nw);
  std::vector<uint64_t> counts((size_t)nw);
  std::vector<uint32_t> bucket((size_t)nw);
  std::vector<std::array<uint64_t, 256>> chs((size_t)T);
  // StrMap iteration order (hash.cpp:29-53, 61-72) needs djb2 & 4095 of every word; the
  // character histogram (histogram.cpp:30-36) counts the chars of every distinct word once
  run([&](int p) {
    auto& ch = chs[(size_t)p];
    ch.fill(0);
    int64_t k = pbase[p];
    for (const auto& x : part[p].e) {
      if (x.off < 0) continue;
      const uint8_t* w = text + x.off;
      uint64_t h = 5381;
      for (int64_t q = 0; q < x.len; ++q) {
        h = (h << 5) + h + w[q];
        ch[w[q]]++;
      }
      woff0[(size_t)k] = x.off;
      wlen0[(size_t)k] = x.len;
      first[(size_t)k] = x.off;
      counts[(size_t)k] = x.cnt;
      bucket[(size_t)k] = (uint32_t)(h & 4095u);
      ++k;
    }
  });
  // (counting sort by bucket, then each bucket's few words by first offset)
  std::vector<int64_t> start(4097, 0), order((size_t)nw);
  for (uint32_t b : bucket) start[b + 1]++;
  for (int b = 0; b < 4096; ++b) start[b + 1] += start[b];
  {
    std::vector<int64_t> fill(start.begin(), start.end() - 1);
    for (int64_t k = 0; k < nw; ++k) order[(size_t)fill[bucket[(size_t)k]]++] = k;
  }
  run([&](int p) {
    for (int b = p; b < 4096; b += T)
      std::sort(order.begin() + start[b], order.begin() + start[b + 1],
                [&](int64_t x, int64_t y) { return first[(size_t)x] < first[(size_t)y]; });
  });
  uint64_t ch[256] = {0};
  for (const auto& a : chs)
    for (int c = 0; c < 256; ++c) ch[c] += a[(size_t)c];
  int32_t map[256];
  coverage_map(ch, t->cfg, map);
  // symbols, words in StrMap order (filled by the threads), then onto the device
  std::vector<int64_t> woff((size_t)nw);
  std::vector<int32_t> wlen((size_t)nw);
  std::vector<uint64_t> wcnt((size_t)nw);
  int64_t total = 0;
  for (int64_t r = 0; r < nw; ++r) {
    const int64_t k = order[(size_t)r];
    woff[(size_t)r] = total;
    wlen[(size_t)r] = (int32_t)wlen0[(size_t)k];
    wcnt[(size_t)r] = counts[(size_t)k];
    total += wlen0[(size_t)k];
  }
  std::vector<int32_t> ids((size_t)total);
  run([&](int p) {
    for (int64_t r = nw * p / T, e = nw * (p + 1) / T; r < e; ++r) {
      const int64_t k = order[(size_t)r];
      const uint8_t* w = text + woff0[(size_t)k];
      int32_t* d = ids.data() + woff[(size_t)r];
      for (int64_t q = 0; q < wlen0[(size_t)k]; ++q) d[q] = map[w[q]];
    }
  });
  free_corpus(t);
  SW_HIP_TRY(hipMalloc(&t->d_ids0, sizeof(int32_t) * std::max<int64_t>(total, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_woff0, sizeof(int64_t) * std::max<int64_t>(nw, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_len0, sizeof(int32_t) * std::max<int64_t>(nw, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_wcnt0, sizeof(uint64_t) * std::max<int64_t>(nw, 1)));
  if (total) SW_HIP_TRY(hipMemcpy(t->d_ids0, ids.data(), sizeof(int32_t) * total, hipMemcpyHostToDevice));
  if (nw) {
    SW_HIP_TRY(hipMemcpy(t->d_woff0, woff.data(), sizeof(int64_t) * nw, hipMemcpyHostToDevice));
    SW_HIP_TRY(hipMemcpy(t->d_len0, wlen.data(), sizeof(int32_t) * nw, hipMemcpyHostToDevice));
    SW_HIP_TRY(hipMemcpy(t->d_wcnt0, wcnt.data(), sizeof(uint64_t) * nw, hipMemcpyHostToDevice));
  }
  t->nw = nw;
  t->ns = total;
  t->host_load = true;
  t->loaded = true;
  t->merges.clear();
  t->tok_freq.clear();
  return SW_OK;
}

// device temporaries freed together
struct TempBufs {
  std::vector<void*> p;
  ~TempBufs() { for (void* x : p) (void)hipFree(x); }
  template <typename T>
  hipError_t get(T** out, size_t bytes) {
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, std::max<size_t>(bytes, 16));
    if (e == hipSuccess) p.push_back(q);
    *out = (T*)q;
    return e;
  }
};

// bpe_load_corpus on the device (the kernels above); returns 1 when a 64-bit hash collision
// between two distinct words makes it give way to the host path, and for corpora whose byte or
// word counts pass the int item counts of the hipcub passes (the host path is int64 throughout)
int32_t load_words_device(sw_trainer* t, const uint8_t* text, int64_t n) {
  if (n > (int64_t)INT32_MAX) return 1;
  hipStream_t st = t->st;
  TempBufs b;  // (temporaries, freed on every return)
  uint8_t* d_text;
  uint8_t* d_flags;
  int64_t *d_starts, *d_cnt;
  unsigned int* d_bad;
  SW_HIP_TRY(b.get(&d_text, (size_t)n));
  SW_HIP_TRY(b.get(&d_flags, (size_t)n));
  SW_HIP_TRY(b.get(&d_cnt, 4 * sizeof(int64_t)));
  SW_HIP_TRY(b.get(&d_bad, sizeof(unsigned int)));
  SW_HIP_TRY(hipMemsetAsync(d_bad, 0, sizeof(unsigned int), st));
  if (n) SW_HIP_TRY(hipMemcpyAsync(d_text, text, (size_t)n, hipMemcpyHostToDevice, st));
  const unsigned g = 4096;
  hipLaunchKernelGGL(k_word_flags, dim3(g), dim3(kBlock), 0, st, d_text, n, d_flags, d_bad);
  // word starts (in corpus order)
  size_t tmp_bytes = 0;
  hipcub::CountingInputIterator<int64_t> pos(0);
  SW_HIP_TRY(hipcub::DeviceSelect::Flagged(nullptr, tmp_bytes, pos, d_flags, (int64_t*)nullptr, d_cnt, n, st));
  void* d_tmp;
  SW_HIP_TRY(b.get(&d_tmp, tmp_bytes));
  // (an upper bound of the word count without a round trip: at most one word per 2 bytes + 1)
  const int64_t wmax = n / 2 + 1;
  SW_HIP_TRY(b.get(&d_starts, sizeof(int64_t) * (size_t)wmax));
  SW_HIP_TRY(hipcub::DeviceSelect::Flagged(d_tmp, tmp_bytes, pos, d_flags, d_starts, d_cnt, n, st));
  int64_t nwords = 0;
  unsigned int bad = 0;
  SW_HIP_TRY(hipMemcpyAsync(&nwords, d_cnt, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  SW_HIP_TRY(hipMemcpyAsync(&bad, d_bad, sizeof(unsigned int), hipMemcpyDeviceToHost, st));
  SW_HIP_TRY(hipStreamSynchronize(st));
  if (bad) return sw::set_error(SW_ERR_ARG, "sw_trainer: the corpus holds NUL bytes");
  // distinct words: the occurrences sorted by hash (stable: corpus order within a run), one
  // run per distinct word, every occurrence checked against its run's first
  const int64_t m = nwords;
  if (m > (int64_t)INT32_MAX) return 1;  // (cannot happen below 2^31 bytes; kept with the sorts' int counts)
  uint64_t *d_hk, *d_hk2, *d_hv, *d_hv2;
  int64_t *d_head, *d_roff, *d_rcnt64;
  SW_HIP_TRY(b.get(&d_hk, sizeof(uint64_t) * (size_t)std::max<int64_t>(m, 1)));
  SW_HIP_TRY(b.get(&d_hk2, sizeof(uint64_t) * (size_t)std::max<int64_t>(m, 1)));
  SW_HIP_TRY(b.get(&d_hv, sizeof(uint64_t) * (size_t)std::max<int64_t>(m, 1)));
  SW_HIP_TRY(b.get(&d_hv2, sizeof(uint64_t) * (size_t)std::max<int64_t>(m, 1)));
  hipLaunchKernelGGL(k_word_hash, dim3(g), dim3(kBlock), 0, st, d_text, n, d_starts, d_cnt, d_hk, d_hv);
  size_t tb1 = 0;
  SW_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb1, d_hk, d_hk2, d_hv, d_hv2, (int)m, 0, 64, st));
  void* d_tmp1;
  SW_HIP_TRY(b.get(&d_tmp1, tb1));
  SW_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp1, tb1, d_hk, d_hk2, d_hv, d_hv2, (int)m, 0, 64, st));
  int64_t* d_headidx;
  SW_HIP_TRY(b.get(&d_head, sizeof(int64_t) * (size_t)std::max<int64_t>(m, 1)));
  SW_HIP_TRY(b.get(&d_headidx, sizeof(int64_t) * (size_t)std::max<int64_t>(m, 1)));
  hipLaunchKernelGGL(k_run_heads, dim3(g), dim3(kBlock), 0, st, d_hk2, m, d_head);
  size_t tb2 = 0;  // (every occurrence's run head: a max-scan of the head positions)
  SW_HIP_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, tb2, d_head, d_headidx, hipcub::Max(), (int)m, st));
  void* d_tmp2;
  SW_HIP_TRY(b.get(&d_tmp2, tb2));
  SW_HIP_TRY(hipcub::DeviceScan::InclusiveScan(d_tmp2, tb2, d_head, d_headidx, hipcub::Max(), (int)m, st));
  hipLaunchKernelGGL(k_word_verify, dim3(g), dim3(kBlock), 0, st, d_text, n, d_hv2, d_headidx, m, d_bad);
  // runs: their lengths (counts), then offsets
  uint64_t* d_ukeys;
  SW_HIP_TRY(b.get(&d_ukeys, sizeof(uint64_t) * (size_t)std::max<int64_t>(m, 1)));
  SW_HIP_TRY(b.get(&d_rcnt64, sizeof(int64_t) * (size_t)(m + 1)));
  SW_HIP_TRY(b.get(&d_roff, sizeof(int64_t) * (size_t)(m + 1)));
  size_t tb3 = 0;
  SW_HIP_TRY(hipcub::DeviceRunLengthEncode::Encode(nullptr, tb3, d_hk2, d_ukeys, d_rcnt64, d_cnt + 1, (int)m, st));
  void* d_tmp3;
  SW_HIP_TRY(b.get(&d_tmp3, tb3));
  SW_HIP_TRY(hipcub::DeviceRunLengthEncode::Encode(d_tmp3, tb3, d_hk2, d_ukeys, d_rcnt64, d_cnt + 1, (int)m, st));
  int64_t nd = 0;
  SW_HIP_TRY(hipMemcpyAsync(&nd, d_cnt + 1, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  SW_HIP_TRY(hipMemcpyAsync(&bad, d_bad, sizeof(unsigned int), hipMemcpyDeviceToHost, st));
  SW_HIP_TRY(hipStreamSynchronize(st));
  if (bad) return 1;  // (a hash collision: the host path)
  SW_HIP_TRY(hipMemsetAsync(d_rcnt64 + nd, 0, sizeof(int64_t), st));
  size_t tb4 = 0;
  SW_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb4, d_rcnt64, d_roff, (int)(nd + 1), st));
  void* d_tmp4;
  SW_HIP_TRY(b.get(&d_tmp4, tb4));
  SW_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(d_tmp4, tb4, d_rcnt64, d_roff, (int)(nd + 1), st));
  // StrMap order
  uint64_t *d_first, *d_wcnt, *d_keys, *d_keys2;
  uint32_t *d_wlen, *d_ridx, *d_order;
  SW_HIP_TRY(b.get(&d_first, sizeof(uint64_t) * (size_t)std::max<int64_t>(nd, 1)));
  SW_HIP_TRY(b.get(&d_wcnt, sizeof(uint64_t) * (size_t)std::max<int64_t>(nd, 1)));
  SW_HIP_TRY(b.get(&d_wlen, sizeof(uint32_t) * (size_t)std::max<int64_t>(nd, 1)));
  SW_HIP_TRY(b.get(&d_keys, sizeof(uint64_t) * (size_t)std::max<int64_t>(nd, 1)));
  SW_HIP_TRY(b.get(&d_keys2, sizeof(uint64_t) * (size_t)std::max<int64_t>(nd, 1)));
  SW_HIP_TRY(b.get(&d_ridx, sizeof(uint32_t) * (size_t)std::max<int64_t>(nd, 1)));
  SW_HIP_TRY(b.get(&d_order, sizeof(uint32_t) * (size_t)std::max<int64_t>(nd, 1)));
  hipLaunchKernelGGL(k_word_runs, dim3(g), dim3(kBlock), 0, st, d_text, n, d_hv2, d_roff, d_cnt + 1, d_first, d_wcnt,
                     d_wlen, d_keys);
  hipLaunchKernelGGL(k_iota, dim3(g), dim3(kBlock), 0, st, d_ridx, nd);
  size_t tb5 = 0;
  SW_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb5, d_keys, d_keys2, d_ridx, d_order, (int)nd, 0, 64, st));
  void* d_tmp5;
  SW_HIP_TRY(b.get(&d_tmp5, tb5));
  SW_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp5, tb5, d_keys, d_keys2, d_ridx, d_order, (int)nd, 0, 64, st));
  // histogram, lengths, counts; then the offsets
  unsigned long long* d_hist;
  int64_t* d_len64;
  SW_HIP_TRY(b.get(&d_hist, 256 * sizeof(unsigned long long)));
  SW_HIP_TRY(b.get(&d_len64, sizeof(int64_t) * (size_t)std::max<int64_t>(nd, 1) + sizeof(int64_t)));
  free_corpus(t);
  SW_HIP_TRY(hipMalloc(&t->d_woff0, sizeof(int64_t) * (size_t)std::max<int64_t>(nd + 1, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_len0, sizeof(int32_t) * (size_t)std::max<int64_t>(nd, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_wcnt0, sizeof(uint64_t) * (size_t)std::max<int64_t>(nd, 1)));
  SW_HIP_TRY(hipMemsetAsync(d_hist, 0, 256 * sizeof(unsigned long long), st));
  SW_HIP_TRY(hipMemsetAsync(d_len64 + nd, 0, sizeof(int64_t), st));
  hipLaunchKernelGGL(k_word_hist, dim3(g), dim3(kBlock), 0, st, d_text, d_first, d_wlen, d_wcnt, d_order, nd, d_hist,
                     d_len64, t->d_len0, t->d_wcnt0);
  size_t tb6 = 0;
  SW_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb6, d_len64, t->d_woff0, (int)(nd + 1), st));
  void* d_tmp6;
  SW_HIP_TRY(b.get(&d_tmp6, tb6));
  SW_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(d_tmp6, tb6, d_len64, t->d_woff0, (int)(nd + 1), st));
  unsigned long long hist[256];
  int64_t total = 0;
  SW_HIP_TRY(hipMemcpyAsync(hist, d_hist, sizeof(hist), hipMemcpyDeviceToHost, st));
  SW_HIP_TRY(hipMemcpyAsync(&total, t->d_woff0 + nd, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  SW_HIP_TRY(hipStreamSynchronize(st));
  uint64_t ch[256];
  for (int c = 0; c < 256; ++c) ch[c] = hist[c];
  int32_t map[256];
  coverage_map(ch, t->cfg, map);
  int32_t* d_map;
  SW_HIP_TRY(b.get(&d_map, sizeof(map)));
  SW_HIP_TRY(hipMemcpyAsync(d_map, map, sizeof(map), hipMemcpyHostToDevice, st));
  SW_HIP_TRY(hipMalloc(&t->d_ids0, sizeof(int32_t) * (size_t)std::max<int64_t>(total, 1)));
  hipLaunchKernelGGL(k_word_ids, dim3(g), dim3(kBlock), 0, st, d_text, d_first, d_wlen, d_order, t->d_woff0, nd, d_map,
                     t->d_ids0);
  SW_HIP_TRY(hipGetLastError());
  SW_HIP_TRY(hipStreamSynchronize(st));  // (the temporaries are freed on return)
  t->nw = nd;
  t->ns = total;
  t->host_load = false;
  return SW_OK;
}

// k_collect for the current pass, then its records on the host: the first kPinnedRecords come
// through mapped memory (one stream synchronisation, no copy command), the rest by a copy
int32_t collect(sw_trainer* t, std::vector<Slot>* out) {
  unsigned long long* cnt = t->d_nused + (t->pass & 1);
  unsigned long long* nxt = t->d_nused + ((t->pass + 1) & 1);
  hipLaunchKernelGGL(k_collect, dim3(1024), dim3(kBlock), 0, t->st, t->d_tab, t->d_used, cnt, nxt, t->d_out,
                     t->h_out_dev, t->h_nused_dev, (uint64_t)kPinnedRecords);
  SW_HIP_TRY(hipGetLastError());
  SW_HIP_TRY(hipStreamSynchronize(t->st));
  ++t->pass;
  const int64_t n = (int64_t)*(volatile unsigned long long*)t->h_nused;
  out->assign(t->h_out, t->h_out + std::min(n, kPinnedRecords));
  if (n > kPinnedRecords) {
    out->resize((size_t)n);
    SW_HIP_TRY(hipMemcpy(out->data() + kPinnedRecords, t->d_out + kPinnedRecords, sizeof(Slot) * (n - kPinnedRecords),
                         hipMemcpyDeviceToHost));
  }
  return SW_OK;
}

// the host side of k_collect_step: spin on the step's sequence number in host-coherent memory
// (no stream synchronisation), then take the records; bounded, so a failed launch is reported
int32_t wait_step(sw_trainer* t, unsigned long long seq, std::vector<Slot>* out) {
  volatile unsigned long long* vs = t->h_cnt + 1;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 0; *vs != seq; ++spin) {
    if ((spin & 0xFFFF) == 0xFFFF) {
      const hipError_t e = hipStreamQuery(t->st);
      if (e != hipSuccess && e != hipErrorNotReady)
        return sw::set_error(SW_ERR_HIP, std::string("sw_trainer_train: merge step: ") + hipGetErrorString(e));
      if (e == hipSuccess && *vs != seq)
        return sw::set_error(SW_ERR_HIP, "sw_trainer_train: merge step finished without publishing its records");
      if (ms_since(t0) > 60000.0) return sw::set_error(SW_ERR_HIP, "sw_trainer_train: merge step timed out");
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  const int64_t n = (int64_t)((volatile unsigned long long*)t->h_cnt)[0];
  out->assign(t->h_rec, t->h_rec + std::min(n, kPinnedRecords));
  if (n > kPinnedRecords) {
    out->resize((size_t)n);
    SW_HIP_TRY(hipMemcpy(out->data() + kPinnedRecords, t->d_out + kPinnedRecords, sizeof(Slot) * (n - kPinnedRecords),
                         hipMemcpyDeviceToHost));
  }
  return SW_OK;
}

int64_t train(sw_trainer* t) {
  using clk = std::chrono::steady_clock;
  const auto t_up = clk::now();
  const int64_t nw = t->nw, ns = t->ns;
  uint64_t min_freq = t->cfg.min_pair_freq ? t->cfg.min_pair_freq : 2000;  // MIN_PAIR_FREQ (bpe.cpp:128-130)
  free_device(t);
  // tables: room for twice the distinct pairs a pass can touch (<= symbols; a merge's changes
  // <= 2 per rewritten symbol)
  uint64_t cap = 1024;
  while (cap < 4 * (uint64_t)std::max<int64_t>(ns, 1)) cap <<= 1;
  if (cap > (1ULL << 32))  // (slot indices and word lengths are 32-bit)
    return sw::set_error(SW_ERR_CAP, "sw_trainer_train: more than 2^30 symbols in distinct words");
  t->tab_mask = cap - 1;
  t->out_cap = (int64_t)cap / 2;
  SW_HIP_TRY(hipMalloc(&t->d_ids, sizeof(int32_t) * std::max<int64_t>(ns, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_woff, sizeof(int64_t) * std::max<int64_t>(nw, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_len, sizeof(int32_t) * std::max<int64_t>(nw, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_wcnt, sizeof(uint64_t) * std::max<int64_t>(nw, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_bloom, sizeof(uint64_t) * std::max<int64_t>(nw, 1)));
  SW_HIP_TRY(hipMalloc(&t->d_tab, sizeof(Slot) * cap));
  SW_HIP_TRY(hipMalloc(&t->d_out, sizeof(Slot) * std::max<int64_t>(t->out_cap, kPinnedRecords)));
  SW_HIP_TRY(hipMalloc(&t->d_used, sizeof(uint32_t) * t->out_cap));
  SW_HIP_TRY(hipMalloc(&t->d_nused, 2 * sizeof(unsigned long long)));
  SW_HIP_TRY(hipHostMalloc(&t->h_out, sizeof(Slot) * kPinnedRecords, hipHostMallocMapped));
  SW_HIP_TRY(hipHostMalloc(&t->h_nused, sizeof(unsigned long long), hipHostMallocMapped));
  SW_HIP_TRY(hipHostGetDevicePointer((void**)&t->h_out_dev, t->h_out, 0));
  SW_HIP_TRY(hipMalloc(&t->d_step_used, sizeof(unsigned long long)));
  SW_HIP_TRY(hipMemsetAsync(t->d_step_used, 0, sizeof(unsigned long long), t->st));
  SW_HIP_TRY(hipHostMalloc(&t->h_rec, sizeof(Slot) * kPinnedRecords, hipHostMallocMapped | hipHostMallocCoherent));
  SW_HIP_TRY(hipHostMalloc(&t->h_cnt, 4 * sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent));
  for (int k = 0; k < 4; ++k) t->h_cnt[k] = 0;
  SW_HIP_TRY(hipHostGetDevicePointer((void**)&t->h_rec_dev, t->h_rec, 0));
  SW_HIP_TRY(hipHostGetDevicePointer((void**)&t->h_cnt_dev, t->h_cnt, 0));
  SW_HIP_TRY(hipHostGetDevicePointer((void**)&t->h_nused_dev, t->h_nused, 0));
  t->pass = 0;
  // the working copies of the loaded corpus (training rewrites ids and len in place)
  if (ns) SW_HIP_TRY(hipMemcpyAsync(t->d_ids, t->d_ids0, sizeof(int32_t) * ns, hipMemcpyDeviceToDevice, t->st));
  if (nw) {
    SW_HIP_TRY(hipMemcpyAsync(t->d_woff, t->d_woff0, sizeof(int64_t) * nw, hipMemcpyDeviceToDevice, t->st));
    SW_HIP_TRY(hipMemcpyAsync(t->d_len, t->d_len0, sizeof(int32_t) * nw, hipMemcpyDeviceToDevice, t->st));
    SW_HIP_TRY(hipMemcpyAsync(t->d_wcnt, t->d_wcnt0, sizeof(uint64_t) * nw, hipMemcpyDeviceToDevice, t->st));
  }
  SW_HIP_TRY(hipMemsetAsync(t->d_nused, 0, 2 * sizeof(unsigned long long), t->st));
  hipLaunchKernelGGL(k_init, dim3(2048), dim3(kBlock), 0, t->st, t->d_tab, cap);
  SW_HIP_TRY(hipGetLastError());
  SW_HIP_TRY(hipStreamSynchronize(t->st));
  t->stats[1] = ms_since(t_up);

  // pair histogram on the device, heap seeded in BIMap order (bpe.cpp:357-366)
  const auto t_cnt = clk::now();
  const unsigned grid = (unsigned)std::max<int64_t>((nw + kBlock - 1) / kBlock, 1);
  if (nw) hipLaunchKernelGGL(k_bloom_init, dim3(grid), dim3(kBlock), 0, t->st, t->d_ids, t->d_woff, t->d_len, nw,
                             t->d_bloom);
  if (nw) hipLaunchKernelGGL(k_count_pairs, dim3(grid), dim3(kBlock), 0, t->st, t->d_ids, t->d_woff, t->d_len, t->d_wcnt,
                             nw, t->cfg.unk_id, t->d_tab, t->tab_mask, t->d_used, t->d_nused + (t->pass & 1));
  std::vector<Slot> rec;
  if (int32_t rc = collect(t, &rec)) return rc;
  PairMap info(rec.size() * 2 + 1024);
  struct Seed { uint32_t bucket; uint64_t first; int32_t a, b; uint64_t freq; };
  std::vector<Seed> seeds;
  seeds.reserve(rec.size());
  for (const Slot& s : rec) {
    const int32_t a = (int32_t)(s.key >> 32), b = (int32_t)(s.key & 0xFFFFFFFFu);
    info[s.key].freq = s.val;
    if (s.val >= min_freq) seeds.push_back(Seed{bimap_bucket(a, b), s.first, a, b, s.val});
  }
  std::sort(seeds.begin(), seeds.end(),
            [](const Seed& x, const Seed& y) { return x.bucket != y.bucket ? x.bucket < y.bucket : x.first < y.first; });
  MaxHeap heap;
  heap.reserve(seeds.size() * 2 + 16);
  for (const Seed& s : seeds) heap.push(s.a, s.b, s.freq, 0);
  // per-pair word lists (k_merge_cand): the loaded corpus's adjacent pairs sorted by pair, their
  // distinct keys and run lengths on the host; SW_TRAIN_FULL_SCAN=1 keeps every merge on the
  // word filters of all words instead (A/B, tests)
  const char* fs_env = std::getenv("SW_TRAIN_FULL_SCAN");
  bool lists = !(fs_env && fs_env[0] == '1') && ns > nw;
  std::vector<uint64_t> ukeys;
  std::vector<int64_t> uoff;
  std::vector<std::pair<uint64_t, uint64_t>> touched;  // per merge: its rewritten words in the pool
  const int64_t pool_cap = ns + 64;                    // (every rewrite shortens its word: <= ns in all)
  if (lists) {
    const int64_t np = ns - nw;
    TempBufs b;
    uint64_t *d_k, *d_k2;
    uint32_t* d_w;
    int64_t* d_nrun;
    SW_HIP_TRY(b.get(&d_k, sizeof(uint64_t) * np));
    SW_HIP_TRY(b.get(&d_k2, sizeof(uint64_t) * np));
    SW_HIP_TRY(b.get(&d_w, sizeof(uint32_t) * np));
    SW_HIP_TRY(hipMalloc(&t->d_pwords, sizeof(uint32_t) * np));
    hipLaunchKernelGGL(k_pair_words, dim3(grid), dim3(kBlock), 0, t->st, t->d_ids, t->d_woff, t->d_len, nw, d_k, d_w);
    size_t tb = 0;
    SW_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d_k, d_k2, d_w, t->d_pwords, (int)np, 0, 64, t->st));
    void* d_tmp;
    SW_HIP_TRY(b.get(&d_tmp, tb));
    SW_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp, tb, d_k, d_k2, d_w, t->d_pwords, (int)np, 0, 64, t->st));
    uint64_t* d_u;
    int64_t* d_c;
    SW_HIP_TRY(b.get(&d_u, sizeof(uint64_t) * np));
    SW_HIP_TRY(b.get(&d_c, sizeof(int64_t) * np));
    SW_HIP_TRY(b.get(&d_nrun, sizeof(int64_t)));
    size_t tb2 = 0;
    SW_HIP_TRY(hipcub::DeviceRunLengthEncode::Encode(nullptr, tb2, d_k2, d_u, d_c, d_nrun, (int)np, t->st));
    void* d_tmp2;
    SW_HIP_TRY(b.get(&d_tmp2, tb2));
    SW_HIP_TRY(hipcub::DeviceRunLengthEncode::Encode(d_tmp2, tb2, d_k2, d_u, d_c, d_nrun, (int)np, t->st));
    int64_t nrun = 0;
    SW_HIP_TRY(hipMemcpyAsync(&nrun, d_nrun, sizeof(int64_t), hipMemcpyDeviceToHost, t->st));
    SW_HIP_TRY(hipStreamSynchronize(t->st));
    ukeys.resize((size_t)nrun);
    std::vector<int64_t> cnt((size_t)nrun);
    SW_HIP_TRY(hipMemcpy(ukeys.data(), d_u, sizeof(uint64_t) * nrun, hipMemcpyDeviceToHost));
    SW_HIP_TRY(hipMemcpy(cnt.data(), d_c, sizeof(int64_t) * nrun, hipMemcpyDeviceToHost));
    uoff.resize((size_t)nrun + 1);
    uoff[0] = 0;
    for (int64_t k = 0; k < nrun; ++k) uoff[(size_t)k + 1] = uoff[(size_t)k] + cnt[(size_t)k];
    SW_HIP_TRY(hipMalloc(&t->d_stamp, sizeof(uint32_t) * nw));
    SW_HIP_TRY(hipMalloc(&t->d_pool, sizeof(uint32_t) * pool_cap));
    SW_HIP_TRY(hipMalloc(&t->d_pool_n, sizeof(unsigned long long)));
    SW_HIP_TRY(hipMalloc(&t->d_overflow, sizeof(unsigned int)));
    SW_HIP_TRY(hipMalloc(&t->d_ticket, sizeof(unsigned int)));
    SW_HIP_TRY(hipMemsetAsync(t->d_ticket, 0, sizeof(unsigned int), t->st));
    SW_HIP_TRY(hipMemsetAsync(t->d_stamp, 0, sizeof(uint32_t) * nw, t->st));
    SW_HIP_TRY(hipMemsetAsync(t->d_pool_n, 0, sizeof(unsigned long long), t->st));
    SW_HIP_TRY(hipMemsetAsync(t->d_overflow, 0, sizeof(unsigned int), t->st));
    SW_HIP_TRY(hipStreamSynchronize(t->st));  // (the temporaries are freed on leaving this block)
  }
  t->stats[2] = ms_since(t_cnt);

  // merges (bpe_train / bpe_merge_batch: batch boundaries do not change the result)
  const int64_t target = (int64_t)t->cfg.target_vocab_size - 256;
  t->merges.clear();
  double dev_ms = 0, host_ms = 0, ahead_ms = 0;
  struct Push { uint32_t bucket; uint64_t first; int32_t a, b; uint64_t freq; uint32_t version; };
  std::vector<Push> pl, pl2;
  std::vector<uint32_t> bstart(1025), bfill(1024);
  int64_t nm = 0;
  unsigned long long seq = 0;
  uint64_t n_pops = 0, n_changes = 0, n_pushes = 0, n_ahead = 0;  // (SW_TRAIN_DEBUG)
  double launch_ms = 0;
  const char* ov_env = std::getenv("SW_TRAIN_NO_AHEAD");
  const bool ahead_ok = !(ov_env && ov_env[0] == '1');
  const char* fb_env = std::getenv("SW_TRAIN_FUSE_BLOCKS");  // (A/B: the one-launch threshold)
  const unsigned fuse_blocks = fb_env ? (unsigned)std::max(1, std::atoi(fb_env)) : kFuseBlocks;
  // one merge's rewrite on the device (X - 256 merges done before it)
  auto launch = [&](int32_t A, int32_t B, int32_t X) -> int32_t {
    const auto tl = clk::now();
    const int64_t before = (int64_t)X - 256;
    ++seq;
    if (lists) {  // the candidate words: the initial list of (A, B), the words A's and B's merges rewrote
      const uint64_t key = pkey(A, B);
      const auto it = std::lower_bound(ukeys.begin(), ukeys.end(), key);
      int64_t o0 = 0, n0 = 0, o1 = 0, n1 = 0, o2 = 0, n2 = 0;
      if (it != ukeys.end() && *it == key) {
        const size_t k = (size_t)(it - ukeys.begin());
        o0 = uoff[k];
        n0 = uoff[k + 1] - uoff[k];
      }
      if (A >= 256 && A - 256 < before) {
        o1 = (int64_t)touched[(size_t)(A - 256)].first;
        n1 = (int64_t)touched[(size_t)(A - 256)].second;
      }
      if (B >= 256 && B - 256 < before && B != A) {
        o2 = (int64_t)touched[(size_t)(B - 256)].first;
        n2 = (int64_t)touched[(size_t)(B - 256)].second;
      }
      const int64_t nc = n0 + n1 + n2;
      const unsigned g = (unsigned)std::max<int64_t>((nc + kBlock - 1) / kBlock, 1);
      if (g <= fuse_blocks) {  // (one launch)
        hipLaunchKernelGGL(k_merge_cand_fused, dim3(g), dim3(kBlock), 0, t->st, t->d_ids, t->d_woff, t->d_len,
                           t->d_wcnt, t->d_bloom, t->d_pwords + o0, n0, t->d_pool + o1, n1, t->d_pool + o2, n2,
                           t->d_stamp, (uint32_t)seq, A, B, X, t->d_tab, t->tab_mask, t->d_used, t->d_step_used,
                           t->d_pool, t->d_pool_n, (uint64_t)pool_cap, t->d_overflow, t->d_ticket, t->d_out,
                           t->h_rec_dev, t->h_cnt_dev, t->h_cnt_dev + 1, seq, (uint64_t)kPinnedRecords);
      } else {
        hipLaunchKernelGGL(k_merge_cand, dim3(g), dim3(kBlock), 0, t->st, t->d_ids, t->d_woff, t->d_len, t->d_wcnt,
                           t->d_bloom, t->d_pwords + o0, n0, t->d_pool + o1, n1, t->d_pool + o2, n2, t->d_stamp,
                           (uint32_t)seq, A, B, X, t->d_tab, t->tab_mask, t->d_used, t->d_step_used, t->d_pool,
                           t->d_pool_n, (uint64_t)pool_cap, t->d_overflow);
        hipLaunchKernelGGL(k_collect_step, dim3(1), dim3(1024), 0, t->st, t->d_tab, t->d_used, t->d_step_used,
                           t->d_out, t->h_rec_dev, t->h_cnt_dev, t->h_cnt_dev + 1, seq, (uint64_t)kPinnedRecords,
                           t->d_pool_n, t->d_overflow);
      }
    } else {
      hipLaunchKernelGGL(k_merge_words, dim3(grid), dim3(kBlock), 0, t->st, t->d_ids, t->d_woff, t->d_len, t->d_wcnt,
                         t->d_bloom, nw, A, B, X, t->d_tab, t->tab_mask, t->d_used, t->d_step_used);
      hipLaunchKernelGGL(k_collect_step, dim3(1), dim3(1024), 0, t->st, t->d_tab, t->d_used, t->d_step_used, t->d_out,
                         t->h_rec_dev, t->h_cnt_dev, t->h_cnt_dev + 1, seq, (uint64_t)kPinnedRecords, t->d_step_used,
                         (const unsigned int*)t->d_step_used);  // (full scan: no pool; these two fields unused)
    }
    SW_HIP_TRY(hipGetLastError());
    launch_ms += ms_since(tl);
    return SW_OK;
  };
  // The reference loop (bpe.cpp:486-535) pops the heap top, merges it, pushes the changed pairs'
  // new entries in FreqChangeMap order (hash % 1024 ascending, newest first within a bucket), and
  // pops again.  The next pop is known before those pushes whenever it is provably the heap root
  // after them: a push reaches the root iff its frequency is above the root's (the sift-up
  // stops at a parent >= it), so the root after the pushes is the first pushed entry with the
  // largest pushed frequency if that beats the current root, else the current root -- taken
  // only if it is live (its version current, its frequency >= min).  Then the next merge is
  // launched first and the pushes (and that pop, checked) run on the host while the device
  // rewrites; every heap operation still happens in the reference's order.
  bool ahead = false;  // the next merge was launched before the pushes (cur = its entry)
  HeapEntry cur{};
  while (true) {
    if (!ahead) {
      if (nm >= target || heap.empty()) break;
      const auto tp = clk::now();
      const HeapEntry top = heap.pop();
      ++n_pops;
      const PairInfo& pi = info[pkey(top.a, top.b)];
      if (top.version != pi.version || pi.freq < min_freq) {  // stale / below the threshold
        host_ms += ms_since(tp);
        continue;
      }
      cur = top;
      if (int32_t rc = launch(cur.a, cur.b, (int32_t)(256 + nm))) return rc;
      host_ms += ms_since(tp);
    }
    ahead = false;
    const int32_t A = cur.a, B = cur.b, X = (int32_t)(256 + nm);
    {
      const auto tw = clk::now();
      if (int32_t rc = wait_step(t, seq, &rec)) return rc;
      dev_ms += ms_since(tw);
    }
    const auto t1 = clk::now();
    if (lists) {
      const uint64_t pn = ((volatile unsigned long long*)t->h_cnt)[2];
      const uint64_t before = touched.empty() ? 0 : touched.back().first + touched.back().second;
      if (((volatile unsigned long long*)t->h_cnt)[3]) lists = false;  // (cannot happen: <= ns rewrites)
      touched.emplace_back(before, pn - before);
    }
    // the changes' new frequencies (each pair once per merge: the device table is keyed by it)
    for (const Slot& s : rec) info.prefetch(s.key);
    n_changes += rec.size();
    pl.clear();
    for (const Slot& s : rec) {
      const int32_t pa = (int32_t)(s.key >> 32), pb = (int32_t)(s.key & 0xFFFFFFFFu);
      if (pa == A && pb == B) continue;
      PairInfo& q = info[s.key];
      const int64_t delta = (int64_t)s.val;
      if (delta < 0) {
        const uint64_t ad = (uint64_t)(-delta);
        q.freq = q.freq >= ad ? q.freq - ad : 0;
      } else {
        q.freq += (uint64_t)delta;
      }
      if (q.freq >= min_freq) {
        q.version++;
        pl.push_back(Push{(uint32_t)(s.key % 1024u), s.first, pa, pb, q.freq, q.version});
      }
    }
    PairInfo& done = info[pkey(A, B)];
    done.freq = 0;
    done.version++;
    t->merges.push_back(A);
    t->merges.push_back(B);
    t->merges.push_back(X);
    ++nm;
    // the next pop, if it is provable now
    if (ahead_ok && nm < target && (!pl.empty() || !heap.empty())) {
      const Push* best = nullptr;
      for (const Push& p : pl)
        if (!best || p.freq > best->freq ||
            (p.freq == best->freq && (p.bucket < best->bucket || (p.bucket == best->bucket && p.first > best->first))))
          best = &p;
      if (best && (heap.empty() || best->freq > heap.top().freq)) {
        cur = HeapEntry{best->a, best->b, best->freq, best->version};
        ahead = true;
      } else if (!heap.empty()) {
        const HeapEntry r = heap.top();
        const PairInfo& ri = info[pkey(r.a, r.b)];
        if (r.version == ri.version && ri.freq >= min_freq) {
          cur = r;
          ahead = true;
        }
      }
      if (ahead) {
        if (int32_t rc = launch(cur.a, cur.b, (int32_t)(256 + nm))) return rc;
        ++n_ahead;
      }
    }
    const auto t2 = clk::now();
    // the pushes in FreqChangeMap order
    if (pl.size() <= 256) {
      std::sort(pl.begin(), pl.end(),
                [](const Push& x, const Push& y) { return x.bucket != y.bucket ? x.bucket < y.bucket : x.first > y.first; });
    } else {  // (many changes: a counting sort by bucket, then each bucket's few by first call)
      std::fill(bstart.begin(), bstart.end(), 0u);
      for (const Push& c : pl) bstart[c.bucket + 1]++;
      for (int q = 0; q < 1024; ++q) bstart[q + 1] += bstart[q];
      pl2.resize(pl.size());
      std::copy(bstart.begin(), bstart.begin() + 1024, bfill.begin());
      for (const Push& c : pl) pl2[bfill[c.bucket]++] = c;
      for (int q = 0; q < 1024; ++q)
        if (bstart[q + 1] - bstart[q] > 1)
          std::sort(pl2.begin() + bstart[q], pl2.begin() + bstart[q + 1],
                    [](const Push& x, const Push& y) { return x.first > y.first; });
      pl.swap(pl2);
    }
    for (const Push& p : pl) heap.push(p.a, p.b, p.freq, p.version);
    n_pushes += pl.size();
    if (ahead) {  // the pop the reference makes next: the entry already launched
      const HeapEntry top = heap.pop();
      ++n_pops;
      if (top.a != cur.a || top.b != cur.b || top.version != cur.version)
        return sw::set_error(SW_ERR_HIP, "sw_trainer_train: internal error: the merge launched ahead is not the heap's next pop");
      ahead_ms += ms_since(t2);
      host_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
    } else {
      host_ms += ms_since(t1);
    }
  }
  if (heap.overflow())
    return sw::set_error(SW_ERR_CAP, "sw_trainer_train: a pair frequency >= 2^40 or more than 2^24 merges");
  if (const char* dbg = std::getenv("SW_TRAIN_DEBUG"); dbg && dbg[0] == '1')
    std::fprintf(stderr, "sw_trainer: %lld merges (%llu launched ahead), %llu heap pops, %llu change records, "
                 "%llu heap pushes, heap %zu, launch calls %.1f ms, host work behind the device %.1f ms\n",
                 (long long)nm, (unsigned long long)n_ahead, (unsigned long long)n_pops, (unsigned long long)n_changes,
                 (unsigned long long)n_pushes, heap.size(), launch_ms, ahead_ms);
  t->stats[3] = dev_ms;
  t->stats[4] = host_ms;
  t->stats[5] = (double)nm;
  t->stats[6] = (double)nw;
  t->stats[7] = (double)ns;
  // final token frequencies over the rewritten corpus (bpe_save :703-712; negative ids skipped),
  // on the device
  t->tok_freq.assign((size_t)(256 + nm), 0);
  unsigned long long* d_freq = nullptr;
  SW_HIP_TRY(hipMalloc(&d_freq, sizeof(unsigned long long) * (size_t)(256 + nm)));
  struct FreeOnExit {
    void* p;
    ~FreeOnExit() { (void)hipFree(p); }
  } free_freq{d_freq};
  SW_HIP_TRY(hipMemsetAsync(d_freq, 0, sizeof(unsigned long long) * (size_t)(256 + nm), t->st));
  if (nw) hipLaunchKernelGGL(k_tok_freq, dim3(grid), dim3(kBlock), 0, t->st, t->d_ids, t->d_woff, t->d_len, t->d_wcnt,
                             nw, (int64_t)(256 + nm), d_freq);
  SW_HIP_TRY(hipGetLastError());
  SW_HIP_TRY(hipMemcpyAsync(t->tok_freq.data(), d_freq, sizeof(uint64_t) * (size_t)(256 + nm), hipMemcpyDeviceToHost,
                            t->st));
  SW_HIP_TRY(hipStreamSynchronize(t->st));
  free_device(t);
  return nm;
}

}  // namespace

extern "C" int32_t sw_trainer_create(const sw_train_config* config, int32_t device, sw_trainer** out) {
  if (!config || !out) return sw::set_error(SW_ERR_ARG, "sw_trainer_create: null argument");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return sw::set_error(SW_ERR_NODEV, "sw_trainer_create: no HIP device");
  if (device < 0 || device >= n) return sw::set_error(SW_ERR_ARG, "sw_trainer_create: bad device ordinal");
  DeviceGuard g(device);
  sw_trainer* t = new sw_trainer();
  t->cfg = *config;
  t->device = device;
  if (hipStreamCreateWithFlags(&t->st, hipStreamNonBlocking) != hipSuccess) {
    delete t;
    return sw::set_error(SW_ERR_HIP, "sw_trainer_create: stream creation failed");
  }
  *out = t;
  return SW_OK;
}

extern "C" void sw_trainer_destroy(sw_trainer* t) {
  if (!t) return;
  DeviceGuard g(t->device);
  free_device(t);
  free_corpus(t);
  if (t->st) (void)hipStreamDestroy(t->st);
  delete t;
}

extern "C" int32_t sw_trainer_load_text(sw_trainer* t, const uint8_t* text, int64_t n) {
  if (!t || n < 0 || (n > 0 && !text)) return sw::set_error(SW_ERR_ARG, "sw_trainer_load_text: bad arguments");
  DeviceGuard g(t->device);
  const auto t0 = std::chrono::steady_clock::now();
  t->merges.clear();
  t->tok_freq.clear();
  // the device path; the host threads when asked (SW_TRAIN_HOST_LOAD=1, for A/B and tests) or
  // when two distinct words share a 64-bit hash
  const char* env = std::getenv("SW_TRAIN_HOST_LOAD");
  int32_t rc = (env && env[0] == '1') ? 1 : load_words_device(t, text, n);
  if (rc == 1) rc = load_words(t, text, n);
  t->loaded = rc == SW_OK;
  t->stats[0] = ms_since(t0);
  return rc;
}

extern "C" int32_t sw_trainer_load_corpus(sw_trainer* t, const char* path) {
  if (!t || !path) return sw::set_error(SW_ERR_ARG, "sw_trainer_load_corpus: bad arguments");
  FILE* f = std::fopen(path, "rb");
  if (!f) return sw::set_error(SW_ERR_ARG, std::string("sw_trainer_load_corpus: cannot open ") + path);
  std::vector<uint8_t> buf;
  if (std::fseek(f, 0, SEEK_END) == 0) {  // (one read of the whole file when its size is known)
    const long sz = std::ftell(f);
    if (sz > 0) buf.resize((size_t)sz);
    std::rewind(f);
    buf.resize(std::fread(buf.data(), 1, buf.size(), f));
  }
  uint8_t tmp[1 << 16];
  size_t got;
  while ((got = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);  // (pipes)
  std::fclose(f);
  return sw_trainer_load_text(t, buf.data(), (int64_t)buf.size());
}

extern "C" int64_t sw_trainer_train(sw_trainer* t) {
  if (!t) return sw::set_error(SW_ERR_ARG, "sw_trainer_train: null handle");
  if (!t->loaded) return sw::set_error(SW_ERR_ARG, "sw_trainer_train: no corpus loaded");
  DeviceGuard g(t->device);
  const int64_t rc = train(t);
  if (rc < 0) free_device(t);
  return rc;
}

extern "C" int64_t sw_trainer_merges(const sw_trainer* t, int32_t* rows, int64_t cap) {
  if (!t || cap < 0 || (cap > 0 && !rows)) return sw::set_error(SW_ERR_ARG, "sw_trainer_merges: bad arguments");
  const int64_t n = (int64_t)t->merges.size() / 3;
  std::memcpy(rows, t->merges.data(), sizeof(int32_t) * 3 * (size_t)std::min(n, cap));
  return n;
}

extern "C" int64_t sw_trainer_token_freq(const sw_trainer* t, uint64_t* freq, int64_t cap) {
  if (!t || cap < 0 || (cap > 0 && !freq)) return sw::set_error(SW_ERR_ARG, "sw_trainer_token_freq: bad arguments");
  const int64_t n = (int64_t)t->tok_freq.size();
  std::memcpy(freq, t->tok_freq.data(), sizeof(uint64_t) * (size_t)std::min(n, cap));
  return n;
}

extern "C" int32_t sw_trainer_save(const sw_trainer* t, const char* model_path, const char* vocab_path) {
  if (!t) return sw::set_error(SW_ERR_ARG, "sw_trainer_save: null handle");
  const size_t M = t->merges.size() / 3;
  if (vocab_path) {  // tokens as the reference's C strings (bpe.cpp:686-701): byte 0 is ""
    std::vector<std::string> toks(256 + M);
    for (int i = 1; i < 256; ++i) toks[(size_t)i] = std::string(1, (char)i);
    // a member can be the UNK id (< 0 with a negative unk_id: bpe.cpp:486-516 does not filter
    // such pairs); the reference then reads toks[-1] (undefined), here it is the empty string
    auto tok = [&](int32_t id) -> std::string { return id >= 0 && (size_t)id < 256 + M ? toks[(size_t)id] : std::string(); };
    for (size_t m = 0; m < M; ++m) toks[256 + m] = tok(t->merges[3 * m]) + tok(t->merges[3 * m + 1]);
    FILE* f = std::fopen(vocab_path, "wb");
    if (!f) return sw::set_error(SW_ERR_ARG, std::string("sw_trainer_save: cannot write ") + vocab_path);
    for (size_t i = 0; i < toks.size(); ++i)
      std::fprintf(f, "%s %llu\n", toks[i].c_str(),
                   (unsigned long long)(i < t->tok_freq.size() ? t->tok_freq[i] : 0ULL));
    std::fclose(f);
  }
  if (model_path) {
    FILE* f = std::fopen(model_path, "wb");
    if (!f) return sw::set_error(SW_ERR_ARG, std::string("sw_trainer_save: cannot write ") + model_path);
    if (M) std::fwrite(t->merges.data(), sizeof(int32_t), 3 * M, f);
    std::fclose(f);
  }
  return SW_OK;
}

extern "C" int32_t sw_trainer_stats(const sw_trainer* t, double* out8) {
  if (!t || !out8) return sw::set_error(SW_ERR_ARG, "sw_trainer_stats: bad arguments");
  for (int i = 0; i < 8; ++i) out8[i] = t->stats[i];
  return SW_OK;
}
