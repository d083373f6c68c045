// Special tokens (E1).  The reference stores `special_tokens` (str -> id, shredword/base.py:103,
// written/read by save/load at :120-121 / :142-144) but defines no split; the build's rule (the
// minbpe convention, the one Tokenizer._split_specials states): scanning each string left to
// right, the first position where some special matches starts an occurrence; at one position the
// first special in dict order wins; the scan resumes after it.  The text between occurrences is
// encoded on its own (pre-split included: an occurrence is a boundary, as a string start is).
//
// Host side, multithreaded over byte-balanced ranges of strings:
//   sw_find_specials_host      the occurrences (position, length, id), ascending
//   sw_presplit_host_specials  the chunk-start bitmap of the pieces, one chunk per occurrence
#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "presplit.h"
#include "shredword_hip.h"

namespace {

struct SpTable {
  const uint8_t* bytes;
  const int64_t* off;
  const int32_t* ids;
  int64_t n;
  bool first[256] = {};                 // some special starts with this byte
  std::vector<int32_t> by_first[256];   // specials starting with that byte, in dict order
  int n_first = 0;
  uint8_t only = 0;                     // the first byte when there is exactly one
};

bool build_table(const sw_specials* sp, SpTable* t) {
  t->bytes = sp->bytes; t->off = sp->off; t->ids = sp->ids; t->n = sp->n;
  for (int64_t k = 0; k < sp->n; ++k) {
    const int64_t len = sp->off[k + 1] - sp->off[k];
    if (len < 0) return false;
    if (len == 0) continue;  // (an empty special never matches: _split_specials drops it)
    const uint8_t b = sp->bytes[sp->off[k]];
    if (!t->first[b]) { t->first[b] = true; ++t->n_first; t->only = b; }
    t->by_first[b].push_back((int32_t)k);
  }
  return true;
}

// occurrences in [a, e) (absolute offsets), appended as positions relative to base
void scan_string(const SpTable& t, const uint8_t* s, int64_t a, int64_t e, int64_t base, std::vector<int64_t>* pos,
                 std::vector<int32_t>* len, std::vector<int32_t>* id) {
  int64_t i = a;
  while (i < e) {
    if (t.n_first == 1) {  // one distinct first byte (e.g. every special is "<|...|>"): memchr
      const void* q = std::memchr(s + i, t.only, (size_t)(e - i));
      if (!q) return;
      i = (const uint8_t*)q - s;
    } else {
      while (i < e && !t.first[s[i]]) ++i;
      if (i >= e) return;
    }
    int32_t hit = -1;
    for (int32_t k : t.by_first[s[i]]) {
      const int64_t L = t.off[k + 1] - t.off[k];
      if (i + L <= e && std::memcmp(s + i, t.bytes + t.off[k], (size_t)L) == 0) { hit = k; break; }
    }
    if (hit < 0) { ++i; continue; }
    const int64_t L = t.off[hit + 1] - t.off[hit];
    pos->push_back(i - base);
    len->push_back((int32_t)L);
    id->push_back(t.ids[hit]);
    i += L;
  }
}

int threads_for(int64_t nbytes, int32_t n_threads) {
  int nt = n_threads > 0 ? n_threads : (int)std::min(64u, std::max(1u, std::thread::hardware_concurrency()));
  return nbytes < (1 << 20) ? 1 : nt;
}

// strings [s0, s1) of thread t of nt (byte-balanced)
void thread_strings(const int64_t* str_off, int64_t n_str, int t, int nt, int64_t* s0, int64_t* s1) {
  const int64_t b0 = str_off[0], nb = str_off[n_str] - b0;
  *s0 = std::lower_bound(str_off, str_off + n_str, b0 + nb * t / nt) - str_off;
  *s1 = t == nt - 1 ? n_str : std::lower_bound(str_off, str_off + n_str, b0 + nb * (t + 1) / nt) - str_off;
}

}  // namespace

extern "C" int64_t sw_find_specials_host(const uint8_t* bytes, const int64_t* str_off, int64_t n_str,
                                         const sw_specials* sp, int64_t* sp_pos, int32_t* sp_len, int32_t* sp_id,
                                         int64_t cap, int32_t n_threads) {
  if (!str_off || n_str < 0 || !sp || sp->n < 0 || (sp->n > 0 && (!sp->bytes || !sp->off || !sp->ids)) || cap < 0)
    return SW_ERR_ARG;
  if (cap > 0 && (!sp_pos || !sp_len || !sp_id)) return SW_ERR_ARG;
  if (n_str == 0 || sp->n == 0) return 0;
  if (str_off[n_str] > str_off[0] && !bytes) return SW_ERR_ARG;
  for (int64_t s = 0; s < n_str; ++s)
    if (str_off[s + 1] < str_off[s]) return SW_ERR_ARG;
  SpTable t;
  if (!build_table(sp, &t)) return SW_ERR_ARG;
  if (t.n_first == 0) return 0;
  const int nt = threads_for(str_off[n_str] - str_off[0], n_threads);
  std::vector<std::vector<int64_t>> pos(nt);
  std::vector<std::vector<int32_t>> len(nt), id(nt);
  auto work = [&](int k) {
    int64_t s0, s1;
    thread_strings(str_off, n_str, k, nt, &s0, &s1);
    for (int64_t s = s0; s < s1; ++s) scan_string(t, bytes, str_off[s], str_off[s + 1], str_off[0], &pos[k], &len[k], &id[k]);
  };
  std::vector<std::thread> th;
  for (int k = 1; k < nt; ++k) th.emplace_back(work, k);
  work(0);
  for (auto& x : th) x.join();
  int64_t total = 0;
  for (int k = 0; k < nt; ++k) total += (int64_t)pos[k].size();
  if (cap == 0) return total;
  if (total > cap) return SW_ERR_CAP;
  int64_t w = 0;
  for (int k = 0; k < nt; ++k) {
    std::copy(pos[k].begin(), pos[k].end(), sp_pos + w);
    std::copy(len[k].begin(), len[k].end(), sp_len + w);
    std::copy(id[k].begin(), id[k].end(), sp_id + w);
    w += (int64_t)pos[k].size();
  }
  return total;
}

extern "C" int64_t sw_presplit_host_specials(const uint8_t* bytes, const int64_t* str_off, int64_t n_str,
                                             int32_t pattern, const int64_t* sp_pos, const int32_t* sp_len,
                                             int64_t n_sp, uint64_t* chunk_bits, int32_t n_threads) {
  if (n_sp < 0 || (n_sp > 0 && (!sp_pos || !sp_len))) return SW_ERR_ARG;
  if (n_sp == 0) return sw_presplit_host(bytes, str_off, n_str, pattern, chunk_bits, n_threads);
  if (!str_off || n_str < 0 || (n_str > 0 && (!bytes || !chunk_bits))) return SW_ERR_ARG;
  if (pattern != SW_PAT_CL100K && pattern != SW_PAT_GPT2 && pattern != SW_PAT_NONE) return SW_ERR_ARG;
  if (n_str == 0) return 0;
  const int64_t b0 = str_off[0], nbytes = str_off[n_str] - b0;
  if (nbytes < 0) return SW_ERR_ARG;
  for (int64_t s = 0; s < n_str; ++s)
    if (str_off[s + 1] < str_off[s]) return SW_ERR_ARG;
  for (int64_t j = 0; j < n_sp; ++j)  // (ascending, non-overlapping, inside the batch)
    if (sp_len[j] <= 0 || sp_pos[j] < 0 || sp_pos[j] + sp_len[j] > nbytes || (j > 0 && sp_pos[j] < sp_pos[j - 1] + sp_len[j - 1]))
      return SW_ERR_ARG;
  const int nt = threads_for(nbytes, n_threads);
  const int64_t nwords = (nbytes + 63) / 64;
  std::atomic<int64_t> total{0};
  std::atomic<bool> bad{false};
  {
    std::vector<std::thread> th;
    auto zero = [&](int k) {
      const int64_t w0 = nwords * k / nt, w1 = nwords * (k + 1) / nt;
      std::memset(chunk_bits + w0, 0, sizeof(uint64_t) * (size_t)(w1 - w0));
    };
    for (int k = 1; k < nt; ++k) th.emplace_back(zero, k);
    zero(0);
    for (auto& x : th) x.join();
  }
  auto split = [&](int k) {
    int64_t s0, s1;
    thread_strings(str_off, n_str, k, nt, &s0, &s1);
    // this thread's occurrences: those starting in its strings
    int64_t j = std::lower_bound(sp_pos, sp_pos + n_sp, str_off[s0] - b0) - sp_pos;
    int64_t c = 0;
    for (int64_t s = s0; s < s1; ++s) {
      const int64_t a = str_off[s] - b0, e = str_off[s + 1] - b0;
      int64_t seg = a;
      for (; j < n_sp && sp_pos[j] < e; ++j) {
        if (sp_pos[j] < seg || sp_pos[j] + sp_len[j] > e) { bad = true; return; }  // (crosses a string)
        c += sw::presplit_string(bytes + b0 + seg, sp_pos[j] - seg, pattern, chunk_bits, seg);
        __atomic_fetch_or(&chunk_bits[sp_pos[j] >> 6], 1ULL << (sp_pos[j] & 63), __ATOMIC_RELAXED);
        ++c;
        seg = sp_pos[j] + sp_len[j];
      }
      c += sw::presplit_string(bytes + b0 + seg, e - seg, pattern, chunk_bits, seg);
    }
    total += c;
  };
  std::vector<std::thread> th;
  for (int k = 1; k < nt; ++k) th.emplace_back(split, k);
  split(0);
  for (auto& x : th) x.join();
  if (bad) return SW_ERR_ARG;
  return total.load();
}
