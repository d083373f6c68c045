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
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

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

__global__ void k_merge_words(int32_t* ids, const int64_t* woff, int32_t* len, const uint64_t* wcnt, uint64_t* bloom,
                              int64_t nw, int32_t A, int32_t B, int32_t X, Slot* tab, uint64_t mask, uint32_t* used,
                              unsigned long long* n_used) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nw) return;
  const uint64_t need = sym_bit(A) | sym_bit(B);
  if ((bloom[w] & need) != need) return;
  const int64_t base = woff[w];
  int32_t* s = ids + base;
  const int L = len[w];
  int r = 0;
  while (r + 1 < L && !(s[r] == A && s[r + 1] == B)) ++r;  // (most words: read only)
  if (r + 1 >= L) return;
  const long long wc = (long long)wcnt[w];
  unsigned long long call = 4ULL * (unsigned long long)base;
  auto add = [&](uint64_t h, long long d) {
    const uint64_t i = slot_of(tab, mask, h, used, n_used);
    atomicAdd(&tab[i].val, (unsigned long long)d);
    atomicMin(&tab[i].first, call++);
  };
  int o = r;
  while (r < L) {
    if (r + 1 < L && s[r] == A && s[r + 1] == B) {
      if (o > 0) {
        add(phash(s[o - 1], A), -wc);
        add(phash(s[o - 1], X), wc);
      }
      if (r + 2 < L) {
        add(phash(B, s[r + 2]), -wc);
        add(phash(X, s[r + 2]), wc);
      }
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

// ---------------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------------
struct HeapEntry {
  int32_t a, b;
  uint64_t freq;
  uint32_t version;
};

// heap_push / heap_pop (heap.cpp:53-114): ties fall where these sift rules put them
struct MaxHeap {
  std::vector<HeapEntry> d;
  void push(int32_t a, int32_t b, uint64_t freq, uint32_t version) {
    d.push_back(HeapEntry{a, b, freq, version});
    size_t i = d.size() - 1;
    while (i > 0) {
      const size_t p = (i - 1) >> 1;
      if (d[p].freq >= d[i].freq) break;
      std::swap(d[p], d[i]);
      i = p;
    }
  }
  HeapEntry pop() {
    const HeapEntry top = d[0];
    d[0] = d.back();
    d.pop_back();
    size_t i = 0;
    const size_t n = d.size();
    for (;;) {
      const size_t l = 2 * i + 1, r = l + 1;
      size_t best = i;
      if (l < n && d[l].freq > d[best].freq) best = l;
      if (r < n && d[r].freq > d[best].freq) best = r;
      if (best == i) break;
      std::swap(d[i], d[best]);
      i = best;
    }
    return top;
  }
};

struct PairInfo {
  uint64_t freq = 0;
  uint32_t version = 0;
};

// pair -> PairInfo, open addressing (the BIMap's role, hash.cpp:104-130; its iteration order
// only matters for the heap seed, which is sorted explicitly)
class PairMap {
 public:
  explicit PairMap(size_t n) { rehash(n); }
  PairInfo& operator[](uint64_t key) {  // get or create (freq 0, version 0)
    if (2 * (n_ + 1) > keys_.size()) rehash(keys_.size());
    size_t i = slot(key);
    if (keys_[i] != key) {
      keys_[i] = key;
      vals_[i] = PairInfo{};
      ++n_;
    }
    return vals_[i];
  }

 private:
  static uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    return x ^ (x >> 33);
  }
  size_t slot(uint64_t key) const {
    size_t i = (size_t)mix(key) & (keys_.size() - 1);
    while (keys_[i] != key && keys_[i] != kEmpty) i = (i + 1) & (keys_.size() - 1);
    return i;
  }
  void rehash(size_t n) {
    size_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    std::vector<uint64_t> ok;
    std::vector<PairInfo> ov;
    ok.swap(keys_);
    ov.swap(vals_);
    keys_.assign(cap, kEmpty);
    vals_.assign(cap, PairInfo{});
    n_ = 0;
    for (size_t i = 0; i < ok.size(); ++i)
      if (ok[i] != kEmpty) (*this)[ok[i]] = ov[i];
  }
  std::vector<uint64_t> keys_;
  std::vector<PairInfo> vals_;
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
  // corpus (host copy of the initial symbols; the device copy is rewritten by training)
  std::vector<int32_t> ids;
  std::vector<int64_t> woff;
  std::vector<int32_t> wlen;
  std::vector<uint64_t> wcnt;
  bool loaded = false;
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
};

namespace {

constexpr int64_t kPinnedRecords = 4096;  // change records fetched with the count (more: a second copy)

void free_device(sw_trainer* t) {
  (void)hipFree(t->d_ids); (void)hipFree(t->d_woff); (void)hipFree(t->d_len); (void)hipFree(t->d_wcnt);
  (void)hipFree(t->d_bloom);
  t->d_bloom = nullptr;
  (void)hipFree(t->d_tab); (void)hipFree(t->d_out); (void)hipFree(t->d_used); (void)hipFree(t->d_nused);
  (void)hipHostFree(t->h_out); (void)hipHostFree(t->h_nused);
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
  // character coverage (bpe.cpp:256-279): chars in StrMap order ((c + 165) & 255), stable by
  // count, the first (size_t)(n * coverage) kept
  uint64_t ch[256] = {0};
  for (const auto& a : chs)
    for (int c = 0; c < 256; ++c) ch[c] += a[(size_t)c];
  std::vector<int> chars;
  for (int b = 0; b < 256; ++b) {
    const int c = (b + 91) & 255;
    if (ch[c]) chars.push_back(c);
  }
  std::stable_sort(chars.begin(), chars.end(), [&](int x, int y) { return ch[x] > ch[y]; });
  float cov = t->cfg.character_coverage;
  if (!(cov > 0.0f && cov < 1.0f)) cov = 0.995f;
  const size_t keep = (size_t)((float)chars.size() * cov);
  int32_t map[256];
  for (int c = 0; c < 256; ++c) map[c] = t->cfg.unk_id;
  for (size_t k = 0; k < keep && k < chars.size(); ++k) map[chars[k]] = chars[k];
  // symbols, words in corpus order (filled by the threads)
  t->woff.assign((size_t)nw, 0);
  t->wlen.assign((size_t)nw, 0);
  t->wcnt.assign((size_t)nw, 0);
  int64_t total = 0;
  for (int64_t r = 0; r < nw; ++r) {
    const int64_t k = order[(size_t)r];
    t->woff[(size_t)r] = total;
    t->wlen[(size_t)r] = (int32_t)wlen0[(size_t)k];
    t->wcnt[(size_t)r] = counts[(size_t)k];
    total += wlen0[(size_t)k];
  }
  t->ids.assign((size_t)total, 0);
  run([&](int p) {
    for (int64_t r = nw * p / T, e = nw * (p + 1) / T; r < e; ++r) {
      const int64_t k = order[(size_t)r];
      const uint8_t* w = text + woff0[(size_t)k];
      int32_t* d = t->ids.data() + t->woff[(size_t)r];
      for (int64_t q = 0; q < wlen0[(size_t)k]; ++q) d[q] = map[w[q]];
    }
  });
  t->loaded = true;
  t->merges.clear();
  t->tok_freq.clear();
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

int64_t train(sw_trainer* t) {
  using clk = std::chrono::steady_clock;
  const auto t_up = clk::now();
  const int64_t nw = (int64_t)t->wlen.size(), ns = (int64_t)t->ids.size();
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
  SW_HIP_TRY(hipHostGetDevicePointer((void**)&t->h_nused_dev, t->h_nused, 0));
  t->pass = 0;
  if (ns) SW_HIP_TRY(hipMemcpyAsync(t->d_ids, t->ids.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice, t->st));
  if (nw) {
    SW_HIP_TRY(hipMemcpyAsync(t->d_woff, t->woff.data(), sizeof(int64_t) * nw, hipMemcpyHostToDevice, t->st));
    SW_HIP_TRY(hipMemcpyAsync(t->d_len, t->wlen.data(), sizeof(int32_t) * nw, hipMemcpyHostToDevice, t->st));
    SW_HIP_TRY(hipMemcpyAsync(t->d_wcnt, t->wcnt.data(), sizeof(uint64_t) * nw, hipMemcpyHostToDevice, t->st));
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
  heap.d.reserve(seeds.size() * 2 + 16);
  for (const Seed& s : seeds) heap.push(s.a, s.b, s.freq, 0);
  t->stats[2] = ms_since(t_cnt);

  // merges (bpe_train / bpe_merge_batch: batch boundaries do not change the result)
  const int64_t target = (int64_t)t->cfg.target_vocab_size - 256;
  t->merges.clear();
  double dev_ms = 0, host_ms = 0;
  struct Change { uint32_t bucket; uint64_t first; uint64_t h; int64_t delta; };
  std::vector<Change> ch;
  int64_t nm = 0;
  while (nm < target && !heap.d.empty()) {
    const HeapEntry top = heap.pop();
    PairInfo& pi = info[pkey(top.a, top.b)];
    if (top.version != pi.version) continue;  // stale
    if (pi.freq < min_freq) continue;
    const int32_t A = top.a, B = top.b, X = (int32_t)(256 + nm);
    const auto t0 = clk::now();
    hipLaunchKernelGGL(k_merge_words, dim3(grid), dim3(kBlock), 0, t->st, t->d_ids, t->d_woff, t->d_len, t->d_wcnt,
                       t->d_bloom, nw,
                       A, B, X, t->d_tab, t->tab_mask, t->d_used, t->d_nused + (t->pass & 1));
    if (int32_t rc = collect(t, &rec)) return rc;
    const auto t1 = clk::now();
    dev_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    // FreqChangeMap order: hash % 1024 ascending, newest first within a bucket
    ch.clear();
    for (const Slot& s : rec) ch.push_back(Change{(uint32_t)(s.key % 1024u), s.first, s.key, (int64_t)s.val});
    std::sort(ch.begin(), ch.end(),
              [](const Change& x, const Change& y) { return x.bucket != y.bucket ? x.bucket < y.bucket : x.first > y.first; });
    for (const Change& c : ch) {
      const int32_t pa = (int32_t)(c.h >> 32), pb = (int32_t)(c.h & 0xFFFFFFFFu);
      if (pa == A && pb == B) continue;
      PairInfo& q = info[pkey(pa, pb)];
      if (c.delta < 0) {
        const uint64_t ad = (uint64_t)(-c.delta);
        q.freq = q.freq >= ad ? q.freq - ad : 0;
      } else {
        q.freq += (uint64_t)c.delta;
      }
      if (q.freq >= min_freq) {
        q.version++;
        heap.push(pa, pb, q.freq, q.version);
      }
    }
    PairInfo& done = info[pkey(A, B)];
    done.freq = 0;
    done.version++;
    t->merges.push_back(A);
    t->merges.push_back(B);
    t->merges.push_back(X);
    ++nm;
    host_ms += ms_since(t1);
  }
  t->stats[3] = dev_ms;
  t->stats[4] = host_ms;
  t->stats[5] = (double)nm;
  t->stats[6] = (double)nw;
  t->stats[7] = (double)ns;
  // final token frequencies over the rewritten corpus (bpe_save :703-712; negative ids skipped)
  std::vector<int32_t> ids((size_t)ns), len((size_t)nw);
  if (ns) SW_HIP_TRY(hipMemcpy(ids.data(), t->d_ids, sizeof(int32_t) * ns, hipMemcpyDeviceToHost));
  if (nw) SW_HIP_TRY(hipMemcpy(len.data(), t->d_len, sizeof(int32_t) * nw, hipMemcpyDeviceToHost));
  t->tok_freq.assign((size_t)(256 + nm), 0);
  for (int64_t w = 0; w < nw; ++w)
    for (int32_t k = 0; k < len[(size_t)w]; ++k) {
      const int32_t id = ids[(size_t)(t->woff[(size_t)w] + k)];
      if (id >= 0 && id < 256 + nm) t->tok_freq[(size_t)id] += t->wcnt[(size_t)w];
    }
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
  if (t->st) (void)hipStreamDestroy(t->st);
  delete t;
}

extern "C" int32_t sw_trainer_load_text(sw_trainer* t, const uint8_t* text, int64_t n) {
  if (!t || n < 0 || (n > 0 && !text)) return sw::set_error(SW_ERR_ARG, "sw_trainer_load_text: bad arguments");
  const auto t0 = std::chrono::steady_clock::now();
  const int32_t rc = load_words(t, text, n);
  t->stats[0] = ms_since(t0);
  return rc;
}

extern "C" int32_t sw_trainer_load_corpus(sw_trainer* t, const char* path) {
  if (!t || !path) return sw::set_error(SW_ERR_ARG, "sw_trainer_load_corpus: bad arguments");
  FILE* f = std::fopen(path, "rb");
  if (!f) return sw::set_error(SW_ERR_ARG, std::string("sw_trainer_load_corpus: cannot open ") + path);
  std::vector<uint8_t> buf;
  uint8_t tmp[1 << 16];
  size_t got;
  while ((got = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
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
