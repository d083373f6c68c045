/* ORACLE -- TEST INFRASTRUCTURE ONLY (see sw_oracle.h for the contract and citations).
 *
 * Written for obviousness, not speed: every step mirrors one reference primitive.
 * Pinned by tests/test_oracle_golden.py against vectors produced by the reference's own
 * Python (shredword/base.py) in oracle/make_golden.py.
 */
#include "sw_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "ucd_ranges.h"

/* ------------------------------------------------------------------------------------ */
/* merges dict: (a, b) -> value.  Open addressing on the 64-bit key.                      */
/* ------------------------------------------------------------------------------------ */
struct orc_model {
  uint64_t* keys;  /* (a << 32) | b, UINT64_MAX = empty */
  int32_t* vals;
  uint64_t mask;
  int well_formed; /* every value >= 256, unique and larger than both ids of its pair */
};

static uint64_t orc_mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

orc_model* orc_model_new(const int32_t* pairs, const int32_t* vals, int64_t n) {
  orc_model* m = (orc_model*)calloc(1, sizeof(orc_model));
  if (!m) return NULL;
  uint64_t cap = 16;
  while (cap < (uint64_t)(n * 2 + 2)) cap <<= 1;
  m->keys = (uint64_t*)malloc(cap * sizeof(uint64_t));
  m->vals = (int32_t*)malloc(cap * sizeof(int32_t));
  if (!m->keys || !m->vals) { orc_model_free(m); return NULL; }
  memset(m->keys, 0xff, cap * sizeof(uint64_t));
  m->mask = cap - 1;
  for (int64_t i = 0; i < n; ++i) {
    uint64_t key = ((uint64_t)(uint32_t)pairs[2 * i] << 32) | (uint32_t)pairs[2 * i + 1];
    uint64_t h = orc_mix(key) & m->mask;
    while (m->keys[h] != UINT64_MAX && m->keys[h] != key) h = (h + 1) & m->mask;
    m->keys[h] = key;          /* dict assignment: a later duplicate overwrites (base.py:147) */
    m->vals[h] = vals[i];
  }
  /* well-formed? (over the dict's final values) */
  m->well_formed = 1;
  int32_t vmax = 0;
  for (uint64_t h = 0; h <= m->mask; ++h) {
    if (m->keys[h] == UINT64_MAX) continue;
    const int32_t v = m->vals[h], a = (int32_t)(m->keys[h] >> 32), b = (int32_t)(uint32_t)m->keys[h];
    if (v < 256 || v <= a || v <= b) m->well_formed = 0;
    if (v > vmax) vmax = v;
  }
  if (m->well_formed) {
    uint8_t* seen = (uint8_t*)calloc((size_t)vmax + 1, 1);
    for (uint64_t h = 0; h <= m->mask && seen; ++h) {
      if (m->keys[h] == UINT64_MAX) continue;
      if (seen[m->vals[h]]++) m->well_formed = 0;
    }
    if (!seen) m->well_formed = 0;
    free(seen);
  }
  return m;
}

int orc_model_well_formed(const orc_model* m) { return m->well_formed; }

void orc_model_free(orc_model* m) {
  if (!m) return;
  free(m->keys); free(m->vals); free(m);
}

int64_t orc_model_get(const orc_model* m, int32_t a, int32_t b) {
  uint64_t key = ((uint64_t)(uint32_t)a << 32) | (uint32_t)b;
  uint64_t h = orc_mix(key) & m->mask;
  while (m->keys[h] != UINT64_MAX) {
    if (m->keys[h] == key) return m->vals[h];
    h = (h + 1) & m->mask;
  }
  return -1;
}

/* ------------------------------------------------------------------------------------ */
/* Unicode classes (regex-module tables, tools/gen_ucd.py)                               */
/* ------------------------------------------------------------------------------------ */
enum { C_OTHER = 0, C_L = 1, C_N = 2, C_S = 3 };
#define CP_INVALID 0xFFFFFFFFu /* an undecodable byte: class other, never matches a literal */

int orc_ucd_class(uint32_t cp) {
  int lo = 0, hi = ORC_UCD_NRANGES - 1;
  if (cp > 0x10FFFF) return C_OTHER;
  while (lo <= hi) {
    int mid = (lo + hi) / 2;
    if (cp < ORC_UCD_RANGES[mid][0]) hi = mid - 1;
    else if (cp > ORC_UCD_RANGES[mid][1]) lo = mid + 1;
    else return (int)ORC_UCD_RANGES[mid][2];
  }
  return C_OTHER;
}

static int in_set(uint32_t cp, const unsigned int* set, int n) {
  for (int i = 0; i < n; ++i) if (set[i] == cp) return 1;
  return 0;
}
#define IN_CI(cp, X) in_set((cp), ORC_CI_##X, (int)(sizeof(ORC_CI_##X) / sizeof(unsigned int)))

/* Strict UTF-8 decode of one code point at s[i]; returns its byte length. Invalid -> 1 byte. */
static int utf8_next(const uint8_t* s, int64_t n, int64_t i, uint32_t* cp) {
  uint8_t c = s[i];
  if (c < 0x80) { *cp = c; return 1; }
  int len; uint32_t v; uint8_t lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) { len = 2; v = c & 0x1F; }
  else if (c >= 0xE0 && c <= 0xEF) {
    len = 3; v = c & 0x0F;
    if (c == 0xE0) lo = 0xA0;
    if (c == 0xED) hi = 0x9F;
  } else if (c >= 0xF0 && c <= 0xF4) {
    len = 4; v = c & 0x07;
    if (c == 0xF0) lo = 0x90;
    if (c == 0xF4) hi = 0x8F;
  } else { *cp = CP_INVALID; return 1; }
  if (i + len > n) { *cp = CP_INVALID; return 1; }
  for (int k = 1; k < len; ++k) {
    uint8_t d = s[i + k];
    if (k == 1 ? (d < lo || d > hi) : (d < 0x80 || d > 0xBF)) { *cp = CP_INVALID; return 1; }
    v = (v << 6) | (d & 0x3F);
  }
  *cp = v;
  return len;
}

/* ------------------------------------------------------------------------------------ */
/* E2: pre-split -- each alternative of the pattern restated as a matcher over code points */
/* ------------------------------------------------------------------------------------ */
typedef struct { const uint32_t* cp; const int* cl; int64_t n; } cps_t;

static int64_t run_end(const cps_t* t, int64_t j, int cls) {
  while (j < t->n && t->cl[j] == cls) ++j;
  return j;
}
static int is_crlf(uint32_t c) { return c == '\r' || c == '\n'; }

/* cl100k: '(?i:[sdmt]|ll|ve|re)|[^\r\n\p{L}\p{N}]?+\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]++[\r\n]*|\s*[\r\n]|\s+(?!\S)|\s+ */
static int64_t match_cl100k(const cps_t* t, int64_t i) {
  const uint32_t* cp = t->cp; const int* cl = t->cl; int64_t n = t->n;
  /* '(?i:[sdmt]|ll|ve|re) */
  if (cp[i] == '\'' && i + 1 < n) {
    uint32_t c = cp[i + 1];
    if (IN_CI(c, S) || IN_CI(c, D) || IN_CI(c, M) || IN_CI(c, T)) return i + 2;
    if (i + 2 < n) {
      uint32_t d = cp[i + 2];
      if ((IN_CI(c, L) && IN_CI(d, L)) || (IN_CI(c, V) && IN_CI(d, E)) || (IN_CI(c, R) && IN_CI(d, E)))
        return i + 3;
    }
  }
  /* [^\r\n\p{L}\p{N}]?+\p{L}+  (possessive optional: taken whenever it can be) */
  {
    int64_t j = i;
    if (!is_crlf(cp[i]) && cl[i] != C_L && cl[i] != C_N) j = i + 1;
    if (j < n && cl[j] == C_L) return run_end(t, j, C_L);
  }
  /* \p{N}{1,3} */
  if (cl[i] == C_N) {
    int64_t j = i;
    while (j < n && j < i + 3 && cl[j] == C_N) ++j;
    return j;
  }
  /*  ?[^\s\p{L}\p{N}]++[\r\n]*  */
  {
    int64_t j = -1;
    if (cp[i] == ' ' && i + 1 < n && cl[i + 1] == C_OTHER) j = i + 1;
    else if (cl[i] == C_OTHER) j = i;
    if (j >= 0) {
      int64_t k = run_end(t, j, C_OTHER);
      while (k < n && is_crlf(cp[k])) ++k;
      return k;
    }
  }
  if (cl[i] == C_S) {
    int64_t j = run_end(t, i, C_S);
    /* \s*[\r\n] : longest prefix of the whitespace run ending in \r or \n */
    for (int64_t k = j - 1; k >= i; --k)
      if (is_crlf(cp[k])) return k + 1;
    /* \s+(?!\S) */
    if (j == n) return j;
    if (j - i >= 2) return j - 1;
    /* \s+ */
    return j;
  }
  return -1; /* unreachable: every class is covered above */
}

/* GPT-2: '(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+ */
static int64_t match_gpt2(const cps_t* t, int64_t i) {
  const uint32_t* cp = t->cp; const int* cl = t->cl; int64_t n = t->n;
  if (cp[i] == '\'' && i + 1 < n) {
    uint32_t c = cp[i + 1];
    if (c == 's' || c == 'd' || c == 'm' || c == 't') return i + 2;
    if (i + 2 < n) {
      uint32_t d = cp[i + 2];
      if ((c == 'l' && d == 'l') || (c == 'v' && d == 'e') || (c == 'r' && d == 'e')) return i + 3;
    }
  }
  static const int classes[3] = {C_L, C_N, C_OTHER};
  for (int a = 0; a < 3; ++a) {
    int want = classes[a];
    if (cp[i] == ' ' && i + 1 < n && cl[i + 1] == want) return run_end(t, i + 1, want);
    if (cl[i] == want) return run_end(t, i, want);
  }
  if (cl[i] == C_S) {
    int64_t j = run_end(t, i, C_S);
    if (j == n) return j;
    if (j - i >= 2) return j - 1;
    return j;
  }
  return -1;
}

int64_t orc_presplit(const uint8_t* s, int64_t n, int pattern, int64_t* starts, int64_t cap) {
  if (n <= 0) return 0;
  if (pattern == ORC_PAT_NONE) {
    if (cap < 1) return -1;
    starts[0] = 0;
    return 1;
  }
  uint32_t* cp = (uint32_t*)malloc(sizeof(uint32_t) * n);
  int* cl = (int*)malloc(sizeof(int) * n);
  int64_t* off = (int64_t*)malloc(sizeof(int64_t) * (n + 1));
  int64_t ncp = 0;
  for (int64_t i = 0; i < n;) {
    uint32_t c;
    int len = utf8_next(s, n, i, &c);
    cp[ncp] = c;
    cl[ncp] = c == CP_INVALID ? C_OTHER : orc_ucd_class(c);
    off[ncp] = i;
    ++ncp;
    i += len;
  }
  off[ncp] = n;
  cps_t t = {cp, cl, ncp};
  int64_t nch = 0;
  for (int64_t i = 0; i < ncp;) {
    int64_t e = pattern == ORC_PAT_GPT2 ? match_gpt2(&t, i) : match_cl100k(&t, i);
    if (e <= i) e = i + 1; /* defensive; no position is unmatched by either pattern */
    if (nch >= cap) { nch = -1; break; }
    starts[nch++] = off[i];
    i = e;
  }
  free(cp); free(cl); free(off);
  return nch;
}

/* ------------------------------------------------------------------------------------ */
/* E3/E4: the merge loop over one chunk                                                  */
/* ------------------------------------------------------------------------------------ */
/* The same loop for a LONG chunk of a well-formed table, in O(n log n): a min-heap of the
 * adjacent pairs keyed by (rank, position) over a linked list of the symbols.  Equal to the
 * loop above (and so to the reference) for well-formed tables: ranks are unique, so the step
 * of rank r takes exactly the occurrences of one pair, and every pair a merge creates holds
 * the new id r and so ranks above r -- the heap pops all of step r's occurrences, left to
 * right, before anything else; an occurrence whose left or right symbol was consumed by the
 * previous one (the (a, a) overlap rule of base.py:29-35) no longer matches and is skipped.
 * tests/test_oracle_golden.py checks it against the loop above on long chunks of every table. */
typedef struct { int64_t rank, pos; int32_t a, b; } orc_hent;
static int orc_hless(const orc_hent* x, const orc_hent* y) {
  return x->rank < y->rank || (x->rank == y->rank && x->pos < y->pos);
}
static void orc_hpush(orc_hent* h, int64_t* n, orc_hent e) {
  int64_t i = (*n)++;
  while (i > 0) {
    int64_t p = (i - 1) / 2;
    if (!orc_hless(&e, &h[p])) break;
    h[i] = h[p];
    i = p;
  }
  h[i] = e;
}
static orc_hent orc_hpop(orc_hent* h, int64_t* n) {
  orc_hent top = h[0], last = h[--(*n)];
  int64_t i = 0;
  for (;;) {
    int64_t l = 2 * i + 1, r = l + 1, c = i;
    const orc_hent* best = &last;
    if (l < *n && orc_hless(&h[l], best)) { c = l; best = &h[l]; }
    if (r < *n && orc_hless(&h[r], best)) { c = r; best = &h[r]; }
    if (c == i) break;
    h[i] = h[c];
    i = c;
  }
  if (*n > 0) h[i] = last;
  return top;
}

int64_t orc_encode_chunk_heap(const orc_model* m, const uint8_t* b, int64_t len, int32_t* out) {
  int32_t* id = (int32_t*)malloc(sizeof(int32_t) * len);
  int64_t* nx = (int64_t*)malloc(sizeof(int64_t) * len);
  int64_t* pv = (int64_t*)malloc(sizeof(int64_t) * len);
  orc_hent* h = (orc_hent*)malloc(sizeof(orc_hent) * (2 * len + 2));
  int64_t nh = 0;
  for (int64_t i = 0; i < len; ++i) { id[i] = b[i]; nx[i] = i + 1 < len ? i + 1 : -1; pv[i] = i - 1; }
  for (int64_t i = 0; i + 1 < len; ++i) {
    int64_t r = orc_model_get(m, id[i], id[i + 1]);
    if (r >= 0) { orc_hent e = {r, i, id[i], id[i + 1]}; orc_hpush(h, &nh, e); }
  }
  while (nh > 0) {
    orc_hent e = orc_hpop(h, &nh);
    const int64_t i = e.pos, j = nx[i];
    if (id[i] != e.a || j < 0 || id[j] != e.b || pv[i] == -2) continue;  /* stale */
    id[i] = (int32_t)e.rank;                       /* merge (base.py:22-36) */
    nx[i] = nx[j];
    if (nx[j] >= 0) pv[nx[j]] = i;
    pv[j] = -2;                                     /* j consumed */
    id[j] = -1;
    if (pv[i] >= 0) {
      int64_t r = orc_model_get(m, id[pv[i]], id[i]);
      if (r >= 0) { orc_hent f = {r, pv[i], id[pv[i]], id[i]}; orc_hpush(h, &nh, f); }
    }
    if (nx[i] >= 0) {
      int64_t r = orc_model_get(m, id[i], id[nx[i]]);
      if (r >= 0) { orc_hent f = {r, i, id[i], id[nx[i]]}; orc_hpush(h, &nh, f); }
    }
  }
  int64_t n = 0;
  for (int64_t i = 0; i >= 0; i = nx[i]) out[n++] = id[i];
  free(id); free(nx); free(pv); free(h);
  return n;
}

#define ORC_HEAP_MIN 256 /* chunks at least this long take the heap form (well-formed tables) */

int64_t orc_encode_chunk(const orc_model* m, const uint8_t* b, int64_t len, int32_t* out) {
  if (m->well_formed && len >= ORC_HEAP_MIN) return orc_encode_chunk_heap(m, b, len, out);
  return orc_encode_chunk_naive(m, b, len, out);
}

int64_t orc_encode_chunk_naive(const orc_model* m, const uint8_t* b, int64_t len, int32_t* out) {
  int32_t* ids = out;
  int64_t n = len;
  for (int64_t i = 0; i < n; ++i) ids[i] = b[i];               /* chunk.encode("utf-8") */
  while (n >= 2) {
    /* get_stats (base.py:10-20) + min(stats, key=merges.get(p, inf)): pairs are visited in
     * first-occurrence order, so the first strictly-smaller rank wins ties like min() does */
    int64_t best = -1, best_rank = 0;
    for (int64_t i = 0; i + 1 < n; ++i) {
      int64_t r = orc_model_get(m, ids[i], ids[i + 1]);
      if (r >= 0 && (best < 0 || r < best_rank)) { best = i; best_rank = r; }
    }
    if (best < 0) break;                                        /* pair not in merges */
    int32_t p0 = ids[best], p1 = ids[best + 1], idx = (int32_t)best_rank;
    /* merge (base.py:22-36): left to right, non-overlapping */
    int64_t w = 0;
    for (int64_t i = 0; i < n;) {
      if (i + 1 < n && ids[i] == p0 && ids[i + 1] == p1) { ids[w++] = idx; i += 2; }
      else { ids[w++] = ids[i]; i += 1; }
    }
    n = w;
  }
  return n;
}

int64_t orc_encode_ordinary(const orc_model* m, const uint8_t* s, int64_t n, int pattern, int32_t* out) {
  if (n <= 0) return 0;
  int64_t* starts = (int64_t*)malloc(sizeof(int64_t) * n);
  int64_t nch = orc_presplit(s, n, pattern, starts, n);
  if (nch < 0) { free(starts); return -1; }
  int64_t w = 0;
  for (int64_t c = 0; c < nch; ++c) {
    int64_t a = starts[c], e = c + 1 < nch ? starts[c + 1] : n;
    w += orc_encode_chunk(m, s + a, e - a, out + w);
  }
  free(starts);
  return w;
}

typedef struct {
  const orc_model* m; const uint8_t* bytes; const int64_t* off; int64_t s0, s1; int pattern;
  int32_t* out; int64_t* cnt;
  const uint8_t* spec_bytes; const int64_t* spec_off; const int32_t* spec_ids; int64_t n_spec;
} orc_job;

static void* orc_worker(void* p) {
  orc_job* j = (orc_job*)p;
  for (int64_t s = j->s0; s < j->s1; ++s) {
    int64_t a = j->off[s], e = j->off[s + 1];
    j->cnt[s] = j->n_spec > 0 ? orc_encode_with_specials(j->m, j->bytes + a, e - a, j->pattern, j->spec_bytes,
                                                         j->spec_off, j->spec_ids, j->n_spec, j->out + a)
                              : orc_encode_ordinary(j->m, j->bytes + a, e - a, j->pattern, j->out + a);
  }
  return NULL;
}

int64_t orc_encode_batch(const orc_model* m, const uint8_t* bytes, const int64_t* off, int64_t n_str,
                         int pattern, int32_t* out, int64_t* out_off, int n_threads) {
  return orc_encode_batch_specials(m, bytes, off, n_str, pattern, NULL, NULL, NULL, 0, out, out_off, n_threads);
}

int64_t orc_encode_batch_specials(const orc_model* m, const uint8_t* bytes, const int64_t* off, int64_t n_str,
                                  int pattern, const uint8_t* spec_bytes, const int64_t* spec_off,
                                  const int32_t* spec_ids, int64_t n_spec, int32_t* out, int64_t* out_off,
                                  int n_threads) {
  if (n_threads < 1) n_threads = 1;
  int64_t* cnt = (int64_t*)calloc(n_str > 0 ? n_str : 1, sizeof(int64_t));
  /* each string writes its ids at its own byte offset (tokens <= bytes), then compact */
  pthread_t th[256];
  orc_job jobs[256];
  if (n_threads > 256) n_threads = 256;
  int64_t total_bytes = n_str > 0 ? off[n_str] - off[0] : 0;
  int64_t s = 0;
  for (int t = 0; t < n_threads; ++t) {
    int64_t target = off[0] + total_bytes * (t + 1) / n_threads, s1 = s;
    while (s1 < n_str && (t == n_threads - 1 || off[s1 + 1] <= target)) ++s1;
    jobs[t] = (orc_job){m, bytes, off, s, s1, pattern, out - off[0], cnt, spec_bytes, spec_off, spec_ids, n_spec};
    s = s1;
  }
  for (int t = 1; t < n_threads; ++t) pthread_create(&th[t], NULL, orc_worker, &jobs[t]);
  orc_worker(&jobs[0]);
  for (int t = 1; t < n_threads; ++t) pthread_join(th[t], NULL);
  int64_t w = 0;
  out_off[0] = 0;
  for (int64_t i = 0; i < n_str; ++i) {
    if (cnt[i] < 0) { free(cnt); return -1; }
    memmove(out + w, out + (off[i] - off[0]), sizeof(int32_t) * cnt[i]);
    w += cnt[i];
    out_off[i + 1] = w;
  }
  free(cnt);
  return w;
}

/* ------------------------------------------------------------------------------------ */
/* E1: special tokens (build-defined; leftmost occurrence, dictionary order on ties)    */
/* ------------------------------------------------------------------------------------ */
int64_t orc_encode_with_specials(const orc_model* m, const uint8_t* s, int64_t n, int pattern,
                                 const uint8_t* spec_bytes, const int64_t* spec_off,
                                 const int32_t* spec_ids, int64_t n_spec, int32_t* out) {
  int64_t w = 0, seg = 0;
  for (int64_t i = 0; i < n;) {
    int64_t hit = -1;
    for (int64_t k = 0; k < n_spec && hit < 0; ++k) {
      int64_t L = spec_off[k + 1] - spec_off[k];
      if (L > 0 && i + L <= n && memcmp(s + i, spec_bytes + spec_off[k], (size_t)L) == 0) hit = k;
    }
    if (hit < 0) { ++i; continue; }
    int64_t r = orc_encode_ordinary(m, s + seg, i - seg, pattern, out + w);
    if (r < 0) return -1;
    w += r;
    out[w++] = spec_ids[hit];
    i += spec_off[hit + 1] - spec_off[hit];
    seg = i;
  }
  int64_t r = orc_encode_ordinary(m, s + seg, n - seg, pattern, out + w);
  if (r < 0) return -1;
  return w + r;
}
