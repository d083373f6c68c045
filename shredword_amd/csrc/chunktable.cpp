// Host builder of the whole-chunk table (see chunktable.h).
#include "chunktable.h"

#include <algorithm>
#include <string>
#include <unordered_set>

namespace sw {

std::vector<int32_t> host_encode_chunk(const std::unordered_map<uint64_t, int32_t>& dict, const uint8_t* b, int n) {
  std::vector<int32_t> ids(b, b + n);
  while (ids.size() >= 2) {
    int64_t best = -1;
    int32_t best_v = 0;
    for (size_t i = 0; i + 1 < ids.size(); ++i) {
      auto it = dict.find(((uint64_t)(uint32_t)ids[i] << 32) | (uint32_t)ids[i + 1]);
      if (it != dict.end() && (best < 0 || it->second < best_v)) { best = (int64_t)i; best_v = it->second; }
    }
    if (best < 0) break;
    const int32_t p0 = ids[best], p1 = ids[best + 1];
    size_t w = 0;
    for (size_t i = 0; i < ids.size();) {
      if (i + 1 < ids.size() && ids[i] == p0 && ids[i + 1] == p1) { ids[w++] = best_v; i += 2; }
      else ids[w++] = ids[i++];
    }
    ids.resize(w);
  }
  return ids;
}

namespace {

struct Entry {
  uint64_t k0, k1;
  uint32_t len, token;
};

uint64_t le64(const std::string& s, size_t at) {
  uint64_t v = 0;
  for (size_t i = 0; i < 8 && at + i < s.size(); ++i) v |= (uint64_t)(uint8_t)s[at + i] << (8 * i);
  return v;
}

// two-choice cuckoo over `slots_per_entry`-uint4 entries, one entry per bucket
bool place(const std::vector<Entry>& es, bool is_long, std::vector<uint4>* out, uint32_t* shift, uint32_t* m1,
           uint32_t* m2) {
  const int w = is_long ? 2 : 1;
  uint32_t log2b = 4;
  constexpr double kLoad = 0.10;  // the cuckoo's maximum load: a sparse table leaves few spilled buckets, so few wave batches pay a second probe
  // sparse up to 2^22 buckets (64 MB of short entries); a larger vocabulary fills them to 0.45
  while ((double)(1ull << log2b) * kLoad < (double)es.size() &&
         (log2b < 22 || (double)(1ull << log2b) * 0.45 < (double)es.size()))
    ++log2b;
  uint64_t rng = is_long ? 0x13198A2E03707344ULL : 0xA4093822299F31D0ULL;
  auto next = [&]() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; };
  for (int attempt = 0; attempt < 64; ++attempt) {
    if (attempt && attempt % 4 == 0 && log2b < 28) ++log2b;
    const size_t nb = (size_t)1 << log2b;
    *shift = 32 - log2b;
    *m1 = (uint32_t)next() | 1u;
    *m2 = (uint32_t)next() | 1u;
    std::vector<int64_t> slot(nb, -1);  // entry index per bucket
    bool ok = true;
    // entries come in token order (lower token = earlier merge = more frequent in the table's
    // training text), each to its first candidate when free: the frequent chunks are answered
    // by the first probe
    for (size_t e = 0; e < es.size() && ok; ++e) {
      int64_t cur = (int64_t)e;
      for (int kick = 0;; ++kick) {
        if (kick > 500) { ok = false; break; }
        const Entry& x = es[cur];
        const uint32_t f = chunk_hash((uint32_t)x.k0, (uint32_t)(x.k0 >> 32), (uint32_t)x.k1, (uint32_t)(x.k1 >> 32),
                                      x.len, *m1);
        const uint32_t c1 = chunk_b1(f, *shift), c2 = chunk_b2(f, *m2, *shift);
        if (slot[c1] < 0) { slot[c1] = cur; break; }
        if (slot[c2] < 0) { slot[c2] = cur; break; }
        const uint32_t victim = (next() & 1) ? c1 : c2;
        std::swap(cur, slot[victim]);
      }
    }
    if (!ok) continue;
    out->assign(nb * w, make_uint4(0, 0, 0, 0));
    std::vector<uint32_t> spill(nb, 0);  // 1: some entry whose first candidate is this bucket sits in its second
    for (size_t bk = 0; bk < nb; ++bk) {
      if (slot[bk] < 0) continue;
      const Entry& x = es[slot[bk]];
      const uint32_t f = chunk_hash((uint32_t)x.k0, (uint32_t)(x.k0 >> 32), (uint32_t)x.k1, (uint32_t)(x.k1 >> 32),
                                    x.len, *m1);
      if (chunk_b1(f, *shift) != bk) spill[chunk_b1(f, *shift)] = 1;
    }
    for (size_t bk = 0; bk < nb; ++bk) {
      if (!is_long) (*out)[bk].w = spill[bk];
      else (*out)[2 * bk + 1].y = spill[bk];
      if (slot[bk] < 0) continue;
      const Entry& x = es[slot[bk]];
      const uint32_t tag = (x.len << 24) | x.token;
      if (!is_long) {
        (*out)[bk] = make_uint4((uint32_t)x.k0, (uint32_t)(x.k0 >> 32), tag, spill[bk]);
      } else {
        (*out)[2 * bk] = make_uint4((uint32_t)x.k0, (uint32_t)(x.k0 >> 32), (uint32_t)x.k1, (uint32_t)(x.k1 >> 32));
        (*out)[2 * bk + 1] = make_uint4(tag, spill[bk], 0, 0);
      }
    }
    return true;
  }
  return false;
}

}  // namespace

bool build_chunk_table(const std::unordered_map<uint64_t, int32_t>& dict, const std::vector<uint64_t>& order,
                       ChunkTableHost* out) {
  // vocabulary byte strings in dict order (build_vocab semantics; pairs whose members are not
  // yet defined are skipped instead of raising)
  std::unordered_map<int32_t, std::string> vocab;
  for (int i = 0; i < 256; ++i) vocab[i] = std::string(1, (char)i);
  for (uint64_t k : order) {
    const int32_t a = (int32_t)(k >> 32), b = (int32_t)(uint32_t)k, v = dict.at(k);
    auto ia = vocab.find(a), ib = vocab.find(b);
    if (ia == vocab.end() || ib == vocab.end()) continue;
    vocab[v] = ia->second + ib->second;
  }
  std::unordered_set<std::string> seen;
  std::vector<Entry> es_short, es_long;
  for (const auto& kv : vocab) {
    const std::string& s = kv.second;
    if (s.size() < 2 || s.size() > 16 || !seen.insert(s).second) continue;
    const std::vector<int32_t> e = host_encode_chunk(dict, (const uint8_t*)s.data(), (int)s.size());
    if (e.size() != 1 || e[0] < 0 || e[0] >= (1 << 24)) continue;
    Entry x{le64(s, 0), le64(s, 8), (uint32_t)s.size(), (uint32_t)e[0]};
    (s.size() <= 8 ? es_short : es_long).push_back(x);
  }
  auto by_token = [](const Entry& x, const Entry& y) { return x.token < y.token; };
  std::stable_sort(es_short.begin(), es_short.end(), by_token);
  std::stable_sort(es_long.begin(), es_long.end(), by_token);
  out->n_short = es_short.size();
  out->n_long = es_long.size();
  return place(es_short, false, &out->sb, &out->s_shift, &out->s_m1, &out->s_m2) &&
         place(es_long, true, &out->lb, &out->l_shift, &out->l_m1, &out->l_m2);
}

}  // namespace sw
