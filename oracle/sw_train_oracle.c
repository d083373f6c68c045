/* ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, CPU-only restatement of shredword's BPE trainer (the C++ core,
 * shredword/csrc/bpe/), with two of its defects fixed.  It CHECKS the GPU trainer
 * (shredword_amd/csrc/train.hip) and is timed as its CPU baseline; the product never links
 * or calls it.  Pinned against the reference trainer's own output (tests/golden/toy500.bin,
 * made by oracle/make_golden.py from the reference sources, and tests/golden/train_*.bin,
 * made by oracle/make_train_golden.py).
 *
 * Behaviour restated (reference file:line), including every iteration order a result depends on:
 *   corpus      bpe_load_corpus        bpe.cpp:208-297   words = maximal runs of bytes other than
 *               ' ', '\t', '\r', '\n' (strtok :247-251); counted per distinct word; word order =
 *               StrMap iteration: djb2(word) & 4095 buckets, first occurrence within a bucket
 *               (hash.cpp:29-53, 61-72; INITIAL_STR_BUFFER buckets, bpe.cpp:214)
 *   coverage    char_hist/collect/qsort histogram.cpp:30-53, bpe.cpp:256-279: per distinct word
 *               (not weighted by its count), chars collected in StrMap bucket order
 *               ((c + 165) & 255 with 256 buckets), stably sorted by count (glibc qsort, a merge
 *               sort), the first (size_t)((float)n * coverage) kept; the rest map to unk_id
 *               (histogram.cpp:15); coverage outside (0, 1) defaults to 0.995 (bpe.cpp:124-126)
 *   count       bpe_count_bigrams      bpe.cpp:315-370   pairs with no unk_id member, weighted by
 *               word count; heap seeded in BIMap order: FNV-1a over the 8-byte pair & 4095
 *               (hash.cpp:7-16, 104-130; MIN_HEAP_SIZE buckets), insertion order within a bucket
 *   heap        heap_push / heap_pop   heap.cpp:53-114   (ties resolved by the sift rules)
 *   merge       bpe_merge_batch        bpe.cpp:391-535   lazy version check, min_pair_freq check,
 *               left-to-right non-overlapping replacement in every word (the replaced pair's left
 *               neighbour is the already-rewritten one), neighbour deltas accumulated per
 *               ((u64)(i64)first << 32 | (u64)(i64)second) and applied in FreqChangeMap order
 *               (hash % 1024 buckets ascending, newest first within a bucket, bpe.cpp:29-46,
 *               486-517), with the clamp at 0, the re-push rule and the merged pair reset
 *   train       bpe_train              bpe.cpp:597-655   merges until target_vocab_size - 256 or
 *               the heap runs dry (batch boundaries do not change the result)
 *   ids         new id = 256 + merge index (bpe.cpp:424); model rows (a, b, id) (bpe.cpp:722-731)
 * Defects fixed:
 *   Symbol.deleted is never initialised (histogram.cpp:14-22): here no symbol starts deleted,
 *     which is what the reference computes whenever the allocator hands it zeroed memory;
 *   bpe_save counts freq[s->id] with s->id == unk_id (bpe.cpp:709), out of bounds for a
 *     negative unk_id: here token frequencies skip negative ids.
 * Inputs with NUL bytes are rejected (-2): the reference's fgets/strlen line reader truncates
 * them in ways that are not part of the trainer's behaviour.
 */
#include "sw_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- small hash maps */
typedef struct {
  uint64_t* keys;
  int64_t* vals;  /* index into a side array */
  uint8_t* used;
  int64_t cap;    /* power of two */
  int64_t n;
} u64map;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

static int u64map_init(u64map* m, int64_t cap) {
  m->cap = 16;
  while (m->cap < 2 * cap) m->cap <<= 1;
  m->keys = (uint64_t*)malloc(sizeof(uint64_t) * m->cap);
  m->vals = (int64_t*)malloc(sizeof(int64_t) * m->cap);
  m->used = (uint8_t*)calloc((size_t)m->cap, 1);
  m->n = 0;
  return m->keys && m->vals && m->used ? 0 : -1;
}

static void u64map_free(u64map* m) { free(m->keys); free(m->vals); free(m->used); }

/* slot of key, or of the empty slot where it belongs */
static int64_t u64map_slot(const u64map* m, uint64_t key) {
  int64_t i = (int64_t)(mix64(key) & (uint64_t)(m->cap - 1));
  while (m->used[i] && m->keys[i] != key) i = (i + 1) & (m->cap - 1);
  return i;
}

static int u64map_grow(u64map* m) {
  u64map g;
  if (u64map_init(&g, m->cap) != 0) return -1;
  for (int64_t i = 0; i < m->cap; ++i)
    if (m->used[i]) {
      const int64_t s = u64map_slot(&g, m->keys[i]);
      g.used[s] = 1; g.keys[s] = m->keys[i]; g.vals[s] = m->vals[i]; g.n++;
    }
  u64map_free(m);
  *m = g;
  return 0;
}

/* ---------------------------------------------------------------- pairs */
typedef struct {
  int32_t a, b;
  uint64_t freq;
  uint32_t version;
  int64_t seq;  /* insertion order (BIMap chain order) */
} pair_info;

typedef struct {
  u64map map;
  pair_info* v;
  int64_t n, cap;
} pair_table;

static uint64_t pkey(int32_t a, int32_t b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; }

/* get-or-create (bimap_get, hash.cpp:104-130): a new pair starts at freq 0, version 0 */
static int64_t pair_get(pair_table* t, int32_t a, int32_t b) {
  const uint64_t k = pkey(a, b);
  int64_t s = u64map_slot(&t->map, k);
  if (t->map.used[s]) return t->map.vals[s];
  if (2 * (t->map.n + 1) > t->map.cap) {
    if (u64map_grow(&t->map) != 0) return -1;
    s = u64map_slot(&t->map, k);
  }
  if (t->n == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 1024;
    pair_info* nv = (pair_info*)realloc(t->v, sizeof(pair_info) * t->cap);
    if (!nv) return -1;
    t->v = nv;
  }
  const int64_t i = t->n++;
  t->v[i].a = a; t->v[i].b = b; t->v[i].freq = 0; t->v[i].version = 0; t->v[i].seq = i;
  t->map.used[s] = 1; t->map.keys[s] = k; t->map.vals[s] = i; t->map.n++;
  return i;
}

/* ---------------------------------------------------------------- heap (heap.cpp:53-114) */
typedef struct {
  int32_t a, b;
  uint64_t freq;
  uint32_t version;
} heap_entry;

typedef struct {
  heap_entry* d;
  int64_t n, cap;
} max_heap;

static int heap_push(max_heap* h, int32_t a, int32_t b, uint64_t freq, uint32_t version) {
  if (h->n == h->cap) {
    h->cap = h->cap ? 2 * h->cap : 4096;
    heap_entry* nd = (heap_entry*)realloc(h->d, sizeof(heap_entry) * h->cap);
    if (!nd) return -1;
    h->d = nd;
  }
  int64_t i = h->n++;
  h->d[i].a = a; h->d[i].b = b; h->d[i].freq = freq; h->d[i].version = version;
  while (i > 0) {  /* up while the parent is strictly smaller */
    const int64_t p = (i - 1) >> 1;
    if (h->d[p].freq >= h->d[i].freq) break;
    const heap_entry t = h->d[p]; h->d[p] = h->d[i]; h->d[i] = t;
    i = p;
  }
  return 0;
}

static heap_entry heap_pop(max_heap* h) {
  const heap_entry top = h->d[0];
  h->d[0] = h->d[--h->n];
  int64_t i = 0;
  for (;;) {  /* down to the larger child, left first on equal children */
    const int64_t l = 2 * i + 1, r = l + 1;
    int64_t best = i;
    if (l < h->n && h->d[l].freq > h->d[best].freq) best = l;
    if (r < h->n && h->d[r].freq > h->d[best].freq) best = r;
    if (best == i) break;
    const heap_entry t = h->d[i]; h->d[i] = h->d[best]; h->d[best] = t;
    i = best;
  }
  return top;
}

/* ---------------------------------------------------------------- orders */
static uint32_t fnv1a_pair(int32_t a, int32_t b) {
  uint8_t by[8];
  memcpy(by, &a, 4);
  memcpy(by + 4, &b, 4);
  uint32_t h = 2166136261u;
  for (int i = 0; i < 8; ++i) { h ^= by[i]; h *= 16777619u; }
  return h;
}

static uint64_t djb2(const uint8_t* s, int64_t n) {
  uint64_t h = 5381;
  for (int64_t i = 0; i < n; ++i) h = (h << 5) + h + s[i];
  return h;
}

typedef struct { uint64_t k1; int64_t k2; int64_t i; } sort_item;
static int cmp_item_asc(const void* x, const void* y) {
  const sort_item *a = (const sort_item*)x, *b = (const sort_item*)y;
  if (a->k1 != b->k1) return a->k1 < b->k1 ? -1 : 1;
  if (a->k2 != b->k2) return a->k2 < b->k2 ? -1 : 1;
  return 0;
}

static int is_delim(uint8_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }

/* ---------------------------------------------------------------- corpus */
int64_t orc_train_words(const uint8_t* text, int64_t n, int32_t unk_id, float coverage, uint8_t* keep_out,
                        int64_t* word_off, int64_t* word_len, uint64_t* word_count, int64_t cap) {
  /* distinct words in StrMap order; returns their number (or -1 / -2 for NUL bytes / -3 if
   * cap is too small); keep_out[256]: the kept characters */
  (void)unk_id;
  for (int64_t i = 0; i < n; ++i)
    if (text[i] == 0) return -2;
  u64map m;
  if (u64map_init(&m, 1024) != 0) return -1;
  int64_t nw = 0, wcap = 1024;
  int64_t* off = (int64_t*)malloc(sizeof(int64_t) * wcap);
  int64_t* len = (int64_t*)malloc(sizeof(int64_t) * wcap);
  uint64_t* cnt = (uint64_t*)malloc(sizeof(uint64_t) * wcap);
  int64_t i = 0;
  while (i < n) {
    while (i < n && is_delim(text[i])) ++i;
    const int64_t s = i;
    while (i < n && !is_delim(text[i])) ++i;
    if (i == s) break;
    const int64_t L = i - s;
    const uint64_t h = djb2(text + s, L);
    /* key: hash; collisions resolved by probing on the full key below */
    int64_t slot = (int64_t)(mix64(h ^ (uint64_t)L) & (uint64_t)(m.cap - 1));
    int64_t found = -1;
    while (m.used[slot]) {
      const int64_t w = m.vals[slot];
      if (len[w] == L && memcmp(text + off[w], text + s, (size_t)L) == 0) { found = w; break; }
      slot = (slot + 1) & (m.cap - 1);
    }
    if (found >= 0) { cnt[found]++; continue; }
    if (nw == wcap) {
      wcap *= 2;
      off = (int64_t*)realloc(off, sizeof(int64_t) * wcap);
      len = (int64_t*)realloc(len, sizeof(int64_t) * wcap);
      cnt = (uint64_t*)realloc(cnt, sizeof(uint64_t) * wcap);
    }
    off[nw] = s; len[nw] = L; cnt[nw] = 1;
    m.used[slot] = 1; m.keys[slot] = h; m.vals[slot] = nw; m.n++;
    ++nw;
    if (2 * m.n > m.cap) {  /* rehash by the same (hash, length) key */
      u64map g;
      u64map_init(&g, m.cap);
      for (int64_t k = 0; k < m.cap; ++k)
        if (m.used[k]) {
          const int64_t w = m.vals[k];
          int64_t t = (int64_t)(mix64(m.keys[k] ^ (uint64_t)len[w]) & (uint64_t)(g.cap - 1));
          while (g.used[t]) t = (t + 1) & (g.cap - 1);
          g.used[t] = 1; g.keys[t] = m.keys[k]; g.vals[t] = w; g.n++;
        }
      u64map_free(&m);
      m = g;
    }
  }
  u64map_free(&m);
  /* StrMap order: djb2 & 4095, first occurrence within a bucket */
  sort_item* it = (sort_item*)malloc(sizeof(sort_item) * (nw ? nw : 1));
  for (int64_t w = 0; w < nw; ++w) {
    it[w].k1 = djb2(text + off[w], len[w]) & 4095u;
    it[w].k2 = w;
    it[w].i = w;
  }
  qsort(it, (size_t)nw, sizeof(sort_item), cmp_item_asc);
  /* character histogram over distinct words, collected in (c + 165) & 255 order, stably sorted */
  uint64_t ch[256] = {0};
  for (int64_t w = 0; w < nw; ++w)
    for (int64_t k = 0; k < len[w]; ++k) ch[text[off[w] + k]]++;
  sort_item cs[256];
  int nc = 0;
  for (int b = 0; b < 256; ++b) {
    const int c = (b + 91) & 255;  /* bucket b holds the char with (c + 165) & 255 == b */
    if (ch[c]) { cs[nc].k1 = ~ch[c]; cs[nc].k2 = nc; cs[nc].i = c; ++nc; }
  }
  qsort(cs, (size_t)nc, sizeof(sort_item), cmp_item_asc);
  if (!(coverage > 0.0f && coverage < 1.0f)) coverage = 0.995f;
  const size_t keep = (size_t)((float)nc * coverage);
  memset(keep_out, 0, 256);
  for (size_t k = 0; k < keep && k < (size_t)nc; ++k) keep_out[cs[k].i] = 1;
  int64_t rc = nw;
  if (nw > cap) rc = -3;
  else
    for (int64_t w = 0; w < nw; ++w) {
      word_off[w] = off[it[w].i];
      word_len[w] = len[it[w].i];
      word_count[w] = cnt[it[w].i];
    }
  free(it); free(off); free(len); free(cnt);
  return rc;
}

/* ---------------------------------------------------------------- training */
typedef struct { uint64_t h; int64_t delta; int64_t seq; } change;

int64_t orc_train(const uint8_t* text, int64_t n, int64_t target_vocab_size, int32_t unk_id, float coverage,
                  uint64_t min_pair_freq, int32_t* merges_out, int64_t merges_cap, uint64_t* tok_freq) {
  if (min_pair_freq == 0) min_pair_freq = 2000;  /* MIN_PAIR_FREQ (bpe.cpp:128-130) */
  int64_t cap = n / 2 + 16;
  int64_t* woff = (int64_t*)malloc(sizeof(int64_t) * cap);
  int64_t* wlen = (int64_t*)malloc(sizeof(int64_t) * cap);
  uint64_t* wcnt = (uint64_t*)malloc(sizeof(uint64_t) * cap);
  uint8_t keep[256];
  const int64_t nw = orc_train_words(text, n, unk_id, coverage, keep, woff, wlen, wcnt, cap);
  if (nw < 0) { free(woff); free(wlen); free(wcnt); return nw; }
  /* symbols: word w at [sym_off[w], sym_off[w] + cur_len[w]) */
  int64_t total = 0;
  for (int64_t w = 0; w < nw; ++w) total += wlen[w];
  int32_t* ids = (int32_t*)malloc(sizeof(int32_t) * (total ? total : 1));
  int64_t* soff = (int64_t*)malloc(sizeof(int64_t) * (nw + 1));
  int64_t* slen = (int64_t*)malloc(sizeof(int64_t) * (nw ? nw : 1));
  total = 0;
  for (int64_t w = 0; w < nw; ++w) {
    soff[w] = total;
    slen[w] = wlen[w];
    for (int64_t k = 0; k < wlen[w]; ++k) {
      const uint8_t c = text[woff[w] + k];
      ids[total + k] = keep[c] ? (int32_t)c : unk_id;
    }
    total += wlen[w];
  }
  soff[nw] = total;
  free(woff); free(wlen);

  /* bigram counts (bpe_count_bigrams) and the heap seed in BIMap order */
  pair_table pt = {0};
  u64map_init(&pt.map, 1024);
  for (int64_t w = 0; w < nw; ++w)
    for (int64_t k = 0; k + 1 < slen[w]; ++k) {
      const int32_t a = ids[soff[w] + k], b = ids[soff[w] + k + 1];
      if (a == unk_id || b == unk_id) continue;
      const int64_t p = pair_get(&pt, a, b);
      pt.v[p].freq += wcnt[w];
    }
  max_heap hp = {0};
  {
    sort_item* it = (sort_item*)malloc(sizeof(sort_item) * (pt.n ? pt.n : 1));
    for (int64_t p = 0; p < pt.n; ++p) {
      it[p].k1 = fnv1a_pair(pt.v[p].a, pt.v[p].b) & 4095u;
      it[p].k2 = pt.v[p].seq;
      it[p].i = p;
    }
    qsort(it, (size_t)pt.n, sizeof(sort_item), cmp_item_asc);
    for (int64_t q = 0; q < pt.n; ++q) {
      const pair_info* pi = &pt.v[it[q].i];
      if (pi->freq >= min_pair_freq) heap_push(&hp, pi->a, pi->b, pi->freq, pi->version);
    }
    free(it);
  }

  /* merges */
  const int64_t target = target_vocab_size - 256;
  int64_t nm = 0;
  u64map cm;
  u64map_init(&cm, 1024);
  int64_t ccap = 1024, nch = 0;
  change* chg = (change*)malloc(sizeof(change) * ccap);
  sort_item* ord = NULL;
  int64_t ocap = 0;
  while (nm < target && hp.n > 0) {
    const heap_entry top = heap_pop(&hp);
    const int64_t pk = pair_get(&pt, top.a, top.b);
    if (top.version != pt.v[pk].version) continue;  /* stale */
    if (pt.v[pk].freq < min_pair_freq) continue;
    const int32_t A = top.a, B = top.b, X = (int32_t)(256 + nm);
    /* every word, left to right; FreqChangeMap restated as (hash -> delta, first-insert seq) */
    for (int64_t q = 0; q < cm.cap; ++q) cm.used[q] = 0;
    cm.n = 0;
    nch = 0;
    int64_t seq = 0;
#define ADD_CHANGE(HASH, DELTA)                                                     \
    do {                                                                            \
      const uint64_t h_ = (HASH);                                                   \
      int64_t s_ = u64map_slot(&cm, h_);                                            \
      if (cm.used[s_]) { chg[cm.vals[s_]].delta += (DELTA); ++seq; break; }         \
      if (nch == ccap) { ccap *= 2; chg = (change*)realloc(chg, sizeof(change) * ccap); } \
      chg[nch].h = h_; chg[nch].delta = (DELTA); chg[nch].seq = seq++;             \
      cm.used[s_] = 1; cm.keys[s_] = h_; cm.vals[s_] = nch++; cm.n++;               \
      if (2 * cm.n > cm.cap) u64map_grow(&cm);                                      \
    } while (0)
#define PHASH(F, S) (((uint64_t)(int64_t)(F) << 32) | (uint64_t)(int64_t)(S))
    for (int64_t w = 0; w < nw; ++w) {
      int32_t* s = ids + soff[w];
      const int64_t L = slen[w];
      const int64_t wc = (int64_t)wcnt[w];
      int64_t r = 0, o = 0;
      while (r < L) {
        if (r + 1 < L && s[r] == A && s[r + 1] == B) {
          if (o > 0) {  /* left neighbour: the rewritten symbol before */
            ADD_CHANGE(PHASH(s[o - 1], A), -wc);
            ADD_CHANGE(PHASH(s[o - 1], X), wc);
          }
          if (r + 2 < L) {  /* right neighbour: the next original symbol */
            ADD_CHANGE(PHASH(B, s[r + 2]), -wc);
            ADD_CHANGE(PHASH(X, s[r + 2]), wc);
          }
          s[o++] = X;
          r += 2;
        } else {
          s[o++] = s[r++];
        }
      }
      slen[w] = o;
    }
#undef ADD_CHANGE
    /* apply in FreqChangeMap order: hash % 1024 ascending, newest first */
    if (ocap < nch) { ocap = nch; ord = (sort_item*)realloc(ord, sizeof(sort_item) * ocap); }
    for (int64_t c = 0; c < nch; ++c) {
      ord[c].k1 = chg[c].h % 1024u;
      ord[c].k2 = -chg[c].seq;
      ord[c].i = c;
    }
    qsort(ord, (size_t)nch, sizeof(sort_item), cmp_item_asc);
    for (int64_t q = 0; q < nch; ++q) {
      const change* c = &chg[ord[q].i];
      const int32_t pa = (int32_t)(c->h >> 32), pb = (int32_t)(c->h & 0xFFFFFFFFu);
      if (pa == A && pb == B) continue;
      const int64_t p = pair_get(&pt, pa, pb);
      pair_info* pi = &pt.v[p];
      if (c->delta < 0) {
        const uint64_t ad = (uint64_t)(-c->delta);
        pi->freq = pi->freq >= ad ? pi->freq - ad : 0;
      } else {
        pi->freq += (uint64_t)c->delta;
      }
      if (pi->freq >= min_pair_freq) {
        pi->version++;
        heap_push(&hp, pa, pb, pi->freq, pi->version);
      }
    }
    {
      pair_info* pi = &pt.v[pair_get(&pt, A, B)];
      pi->freq = 0;
      pi->version++;
    }
    if (nm < merges_cap) {
      merges_out[3 * nm] = A;
      merges_out[3 * nm + 1] = B;
      merges_out[3 * nm + 2] = X;
    }
    ++nm;
  }
#undef PHASH
  if (tok_freq) {  /* final token frequencies (bpe_save :703-712), negative ids skipped */
    memset(tok_freq, 0, sizeof(uint64_t) * (size_t)(256 + nm));
    for (int64_t w = 0; w < nw; ++w)
      for (int64_t k = 0; k < slen[w]; ++k) {
        const int32_t id = ids[soff[w] + k];
        if (id >= 0 && id < 256 + nm) tok_freq[id] += wcnt[w];
      }
  }
  free(ord); free(chg); u64map_free(&cm);
  free(hp.d); u64map_free(&pt.map); free(pt.v);
  free(ids); free(soff); free(slen); free(wcnt);
  return nm;
}
