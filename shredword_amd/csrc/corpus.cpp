// Deterministic synthetic UTF-8 corpora for the benchmark configs.
//
// The reference ships no corpus; these generators define the inputs every bench / parity
// run uses.  Everything derives from splitmix64 streams keyed by (seed, string index), so
// the bytes are identical on any machine and for any thread count.
//
//   SW_CORPUS_ASCII  (C1)  ASCII prose lines over a Zipf lexicon (5-20 words/line)
//   SW_CORPUS_MIXED  (C2)  ~85% ASCII / 8% Latin-1 / 5% CJK / 2% emoji bytes, punctuation,
//                          digit runs, whitespace runs, contractions
//   SW_CORPUS_STRESS (C5)  Zipf string lengths 4..4096 B, >=1% strings that are a single
//                          4096-B letter run, long whitespace runs, (a,a) runs
//   SW_CORPUS_ENTROPY      low-repetition text: a flat Zipf over 1 M words -- mixed-case Latin
//                          pseudo-words with accents, and Cyrillic, Greek, CJK, Hangul, Devanagari
//                          letter strings -- so that many multi-token chunks are distinct and the
//                          merge loop itself, not the memoisation, carries much of the encode
//
// sw_synth_splice_specials inserts special tokens into such a corpus (the C3 workload: a
// document separator at every string's end and others at random code-point boundaries).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "shredword_hip.h"

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
};

uint64_t key(uint64_t a, uint64_t b) { return Rng(a * 0x100000001B3ULL ^ (b + 0x632BE59BD9B4E019ULL)).next(); }

void put_utf8(std::string& s, uint32_t cp) {
  if (cp < 0x80) s += (char)cp;
  else if (cp < 0x800) { s += (char)(0xC0 | (cp >> 6)); s += (char)(0x80 | (cp & 63)); }
  else if (cp < 0x10000) {
    s += (char)(0xE0 | (cp >> 12)); s += (char)(0x80 | ((cp >> 6) & 63)); s += (char)(0x80 | (cp & 63));
  } else {
    s += (char)(0xF0 | (cp >> 18)); s += (char)(0x80 | ((cp >> 12) & 63));
    s += (char)(0x80 | ((cp >> 6) & 63)); s += (char)(0x80 | (cp & 63));
  }
}

// Syllable inventory for pronounceable pseudo-words (weights in parentheses are implicit:
// earlier entries are drawn more often).  Real-text-like words give BPE the sub-word structure
// it learns on natural language, so merge depth per chunk resembles real corpora.
const char* kOnset[] = {"", "t", "s", "r", "n", "l", "d", "m", "c", "p", "b", "h", "f", "g", "w", "v", "k",
                        "th", "st", "tr", "pr", "ch", "sh", "br", "cr", "gr", "fr", "pl", "cl", "sp", "bl",
                        "dr", "wh", "j", "qu", "sl", "fl", "sc", "y", "str", "gl", "sm", "sn", "sw", "z"};
const char* kVowel[] = {"e", "a", "i", "o", "u", "ea", "ou", "io", "ee", "ai", "oo", "ie", "y", "oa", "au"};
const char* kCoda[] = {"", "", "n", "r", "s", "t", "l", "d", "m", "nd", "ng", "st", "nt", "ck", "rs", "th",
                       "ll", "ss", "ct", "rt", "ns", "sh", "x", "ld", "ts", "ch", "ght", "ble", "tion", "ment"};
const uint32_t kLatin1[] = {0xE9, 0xE8, 0xEA, 0xE0, 0xE2, 0xE7, 0xF4, 0xEE, 0xFC, 0xF6,
                            0xE4, 0xF1, 0xDF, 0xE1, 0xED, 0xF3, 0xFA, 0xF8, 0xE5, 0xE6};

template <size_t N>
const char* pick(Rng& r, const char* (&arr)[N]) {  // ~geometric preference for early entries
  double u = r.uni();
  size_t i = (size_t)(N * u * u);
  return arr[i < N ? i : N - 1];
}

struct Alias {  // Vose alias table: O(1) draws from a fixed discrete distribution
  std::vector<double> prob;
  std::vector<uint32_t> alias;
  void build(const std::vector<double>& w) {
    size_t n = w.size();
    prob.assign(n, 0.0); alias.assign(n, 0);
    double sum = 0; for (double x : w) sum += x;
    std::vector<double> p(n);
    std::vector<uint32_t> small, large;
    for (size_t i = 0; i < n; ++i) { p[i] = w[i] * n / sum; (p[i] < 1.0 ? small : large).push_back((uint32_t)i); }
    while (!small.empty() && !large.empty()) {
      uint32_t s = small.back(), l = large.back(); small.pop_back();
      prob[s] = p[s]; alias[s] = l; p[l] = (p[l] + p[s]) - 1.0;
      if (p[l] < 1.0) { large.pop_back(); small.push_back(l); }
    }
    for (uint32_t i : large) prob[i] = 1.0;
    for (uint32_t i : small) prob[i] = 1.0;
  }
  uint32_t draw(Rng& r) const {
    uint32_t i = r.below((uint32_t)prob.size());
    return r.uni() < prob[i] ? i : alias[i];
  }
};

struct Lexicon {
  std::vector<std::string> words;
  Alias zipf;
  int kind;
  Lexicon(uint64_t seed, int kind_) : kind(kind_) {
    Rng r(key(seed, 0xC0FFEE));
    if (kind == SW_CORPUS_ENTROPY) {
      build_entropy(r);
      return;
    }
    size_t n = kind == SW_CORPUS_ASCII ? 50000 : 200000;
    words.reserve(n);
    for (size_t i = 0; i < n; ++i) {
      std::string w;
      double u = r.uni();
      int type = 0;  // 0 ascii, 1 latin-1, 2 cjk, 3 emoji
      if (kind != SW_CORPUS_ASCII) type = u < 0.80 ? 0 : u < 0.90 ? 1 : u < 0.97 ? 2 : 3;
      if (type == 2) {
        int len = 1 + r.below(3);
        for (int k = 0; k < len; ++k) put_utf8(w, 0x4E00 + r.below(0x51A6));
      } else if (type == 3) {
        int len = 1 + r.below(2);
        for (int k = 0; k < len; ++k) put_utf8(w, 0x1F300 + r.below(0x350));
      } else {
        double v = r.uni();
        int syl = v < 0.40 ? 1 : v < 0.75 ? 2 : v < 0.93 ? 3 : 4;
        for (int k = 0; k < syl; ++k) {
          w += pick(r, kOnset);
          if (type == 1 && r.uni() < 0.35) put_utf8(w, kLatin1[r.below(20)]);
          else w += pick(r, kVowel);
          if (k + 1 == syl || r.uni() < 0.3) w += pick(r, kCoda);
        }
      }
      words.push_back(std::move(w));
    }
    std::vector<double> zw(n);
    for (size_t i = 0; i < n; ++i) zw[i] = 1.0 / std::pow((double)i + 2.7, 1.07);
    zipf.build(zw);
  }
  // 1 M words: 62% pseudo-words of 1..5 syllables (the MIXED syllables, accented vowels; prose()
  // flips their case per occurrence), the rest random letters of Cyrillic / Greek (2..10,
  // random case), CJK (1..4), Hangul (1..3), Devanagari (2..6); a digit inside 3% of the words; a
  // flat Zipf (exponent 0.8) -- the word list is large and mixed-case enough that most chunks the
  // merge loop gets are distinct in a 1 GiB batch
  void build_entropy(Rng& r) {
    const size_t n = 1000000;
    words.reserve(n);
    for (size_t i = 0; i < n; ++i) {
      std::string w;
      const double u = r.uni();
      if (u < 0.62) {
        const double v = r.uni();
        const int syl = v < 0.25 ? 1 : v < 0.55 ? 2 : v < 0.80 ? 3 : v < 0.93 ? 4 : 5;
        for (int k = 0; k < syl; ++k) {
          w += pick(r, kOnset);
          if (r.uni() < 0.10) put_utf8(w, kLatin1[r.below(20)]);
          else w += pick(r, kVowel);
          if (k + 1 == syl || r.uni() < 0.3) w += pick(r, kCoda);
        }
      } else {
        const int script = u < 0.72 ? 1 : u < 0.80 ? 2 : u < 0.89 ? 3 : u < 0.95 ? 4 : 5;
        static const uint32_t kBase[] = {0, 0x430, 0x3B1, 0x4E00, 0xAC00, 0x915};
        static const uint32_t kSpan[] = {0, 32, 24, 0x51A6, 11172, 37};
        const int len = script <= 2 ? 2 + (int)r.below(9) : script == 3 ? 1 + (int)r.below(4)
                                                           : script == 4 ? 1 + (int)r.below(3) : 2 + (int)r.below(5);
        for (int k = 0; k < len; ++k) {
          uint32_t cp = kBase[script] + r.below(kSpan[script]);
          if (script == 2 && cp >= 0x3C2) ++cp;              // (skip final sigma's slot: U+03A2 upper is unassigned)
          if (script <= 2 && r.uni() < 0.3) cp -= 0x20;      // upper case
          put_utf8(w, cp);
        }
      }
      if (r.uni() < 0.03) {  // a digit at a code-point boundary
        size_t at = r.below((uint32_t)w.size() + 1);
        while (at < w.size() && ((unsigned char)w[at] & 0xC0) == 0x80) ++at;
        w.insert(at, 1, (char)('0' + r.below(10)));
      }
      words.push_back(std::move(w));
    }
    std::vector<double> zw(n);
    for (size_t i = 0; i < n; ++i) zw[i] = 1.0 / std::pow((double)i + 2.7, 0.8);
    zipf.build(zw);
  }
};

const char* kContractions[] = {"'s", "'t", "'re", "'ve", "'ll", "'d", "'m", "'S", "'LL"};
const char* kPunct[] = {",", ".", "!", "?", ";", ":", "\"", ")", "...", "-", "--", "%", "&"};

// Emits prose until s.size() >= len, then trims to exactly len bytes at a code point edge.
// (SW_CORPUS_ENTROPY: every ASCII letter of every occurrence upper-cased with probability 0.12,
// so a word's occurrences are rarely byte-equal)
void prose(const Lexicon& lx, Rng& r, std::string& s, size_t len, bool ascii_lines) {
  const bool flip = lx.kind == SW_CORPUS_ENTROPY;
  bool sentence_start = true;
  int words_in_line = 0, line_len = 5 + r.below(16);
  while (s.size() < len) {
    double u = r.uni();
    if (u < 0.07) {  // number: 1-7 digits, sometimes with a separator
      int nd = 1 + r.below(7);
      for (int k = 0; k < nd; ++k) s += (char)('0' + r.below(10));
      if (r.uni() < 0.2) { s += (r.uni() < 0.5 ? '.' : ','); s += (char)('0' + r.below(10)); s += (char)('0' + r.below(10)); }
    } else {
      const std::string& w = lx.words[lx.zipf.draw(r)];
      size_t at = s.size();
      if (!ascii_lines && r.uni() < 0.03) s += (r.uni() < 0.5 ? '(' : '"');
      s += w;
      if (flip)
        for (size_t k = s.size() - w.size(); k < s.size(); ++k)
          if (s[k] >= 'a' && s[k] <= 'z' && r.uni() < 0.12) s[k] = (char)(s[k] - 32);
      if ((sentence_start && r.uni() < 0.9) || r.uni() < 0.05) {
        char& c = s[at + (s[at] == '(' || s[at] == '"')];
        if (c >= 'a' && c <= 'z') c = (char)(c - 32);
      }
      if (r.uni() < 0.02) s += kContractions[r.below(ascii_lines ? 7 : 9)];
    }
    sentence_start = false;
    double p = r.uni();
    if (p < 0.08) { s += '.'; sentence_start = true; }
    else if (p < 0.13) s += kPunct[r.below(ascii_lines ? 6 : 13)];
    ++words_in_line;
    if (ascii_lines ? words_in_line >= line_len : r.uni() < 0.03) {
      s += '\n';
      if (!ascii_lines && r.uni() < 0.3) s += '\n';
      words_in_line = 0; line_len = 5 + r.below(16);
      sentence_start = true;
    } else {
      double q = r.uni();
      if (!ascii_lines && q < 0.02) s += "  ";
      else if (!ascii_lines && q < 0.025) s += '\t';
      else if (!ascii_lines && q < 0.027) s += " \n ";
      else s += ' ';
    }
  }
  // trim to len bytes without splitting a multi-byte sequence: pad with ASCII if needed
  size_t cut = len;
  while (cut > 0 && cut < s.size() && ((unsigned char)s[cut] & 0xC0) == 0x80) --cut;
  s.resize(cut);
  while (s.size() < len) s += (char)('a' + r.below(26));
}

void stress(const Lexicon& lx, Rng& r, std::string& s, size_t len) {
  double u = r.uni();
  if (u < 0.012) {  // one 4096-byte letter run: a single pre-split chunk
    for (size_t k = 0; k < len; ++k) s += (char)('a' + r.below(26));
    return;
  }
  if (u < 0.02) {  // (a,a) runs
    while (s.size() < len) {
      char c = (char)('a' + r.below(26));
      size_t run = 2 + r.below(200);
      for (size_t k = 0; k < run && s.size() < len; ++k) s += c;
      if (s.size() < len) s += ' ';
    }
    s.resize(len);
    return;
  }
  if (u < 0.03) {  // whitespace runs
    static const char ws[] = {' ', ' ', ' ', '\n', '\t', '\r'};
    while (s.size() < len) {
      size_t run = 1 + r.below(300);
      for (size_t k = 0; k < run && s.size() < len; ++k) s += ws[r.below(6)];
      if (s.size() < len) s += lx.words[lx.zipf.draw(r)];
    }
    size_t cut = len;
    while (cut > 0 && cut < s.size() && ((unsigned char)s[cut] & 0xC0) == 0x80) --cut;
    s.resize(cut);
    while (s.size() < len) s += ' ';
    return;
  }
  prose(lx, r, s, len, false);
}

size_t string_len(int kind, Rng& r, double mean) {
  if (kind == SW_CORPUS_STRESS) {
    // Zipf over 4..4096 (P(L) ~ 1/L), and the dedicated 4096-B letter-run strings
    double lo = std::log(4.0), hi = std::log(4097.0);
    size_t L = (size_t)std::exp(lo + (hi - lo) * r.uni());
    return std::min<size_t>(4096, std::max<size_t>(4, L));
  }
  // lognormal around the requested mean, sigma 0.6, clamped
  double g = std::sqrt(-2.0 * std::log(1.0 - r.uni())) * std::cos(6.283185307179586 * r.uni());
  double L = mean * std::exp(0.6 * g - 0.18);
  return (size_t)std::max(1.0, std::min(L, mean * 8));
}

}  // namespace

extern "C" int64_t sw_synth_corpus(uint64_t seed, int32_t kind, int64_t n_strings, int64_t mean_len,
                                   uint8_t* out_bytes, int64_t cap, int64_t* out_off, int32_t n_threads) {
  if (n_strings < 0 || mean_len < 1 || !out_off) return -1;
  if (kind != SW_CORPUS_ASCII && kind != SW_CORPUS_MIXED && kind != SW_CORPUS_STRESS && kind != SW_CORPUS_ENTROPY)
    return -1;
  // lengths first (cheap, serial, deterministic)
  out_off[0] = 0;
  for (int64_t i = 0; i < n_strings; ++i) {
    Rng r(key(seed, 2 * (uint64_t)i + 1));
    size_t L = kind == SW_CORPUS_STRESS ? (r.uni() < 0.012 ? 4096 : string_len(kind, r, (double)mean_len))
                                        : string_len(kind, r, (double)mean_len);
    out_off[i + 1] = out_off[i] + (int64_t)L;
  }
  if (!out_bytes) return out_off[n_strings];
  if (cap < out_off[n_strings]) return -1;
  // The lexicon is the corpus' "language": fixed per kind, shared by every seed, so a merge
  // table trained on one seed's sample compresses another seed's text like real BPE does.
  Lexicon lx(0x5EED0000ULL + (uint64_t)kind, kind);
  int nt = n_threads > 0 ? n_threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  auto work = [&](int t) {
    std::string s;
    for (int64_t i = t; i < n_strings; i += nt) {
      Rng r(key(seed, 2 * (uint64_t)i + 2));
      size_t L = (size_t)(out_off[i + 1] - out_off[i]);
      s.clear();
      if (kind == SW_CORPUS_STRESS && L == 4096 && r.uni() < 0.75) {
        for (size_t k = 0; k < L; ++k) s += (char)('a' + r.below(26));
      } else if (kind == SW_CORPUS_STRESS) {
        stress(lx, r, s, L);
      } else {
        prose(lx, r, s, L, kind == SW_CORPUS_ASCII);
      }
      std::memcpy(out_bytes + out_off[i], s.data(), L);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  return out_off[n_strings];
}

extern "C" int64_t sw_synth_splice_specials(uint64_t seed, const uint8_t* bytes, const int64_t* off, int64_t n_strings,
                                           const sw_specials* sp, double per_kib, int32_t end_special,
                                           uint8_t* out_bytes, int64_t cap, int64_t* out_off, int32_t n_threads) {
  if (n_strings < 0 || !off || !out_off || !sp || sp->n <= 0 || !sp->bytes || !sp->off || per_kib < 0) return -1;
  if (end_special >= sp->n) return -1;
  if (n_strings > 0 && off[n_strings] > off[0] && !bytes) return -1;
  // per string: how many random insertions (deterministic), and the bytes they add
  auto plan = [&](int64_t i, Rng& r) -> int64_t {
    const double want = (double)(off[i + 1] - off[i]) / 1024.0 * per_kib;
    return (int64_t)want + (r.uni() < want - (double)(int64_t)want ? 1 : 0);
  };
  auto sp_len = [&](int64_t k) { return sp->off[k + 1] - sp->off[k]; };
  out_off[0] = 0;
  for (int64_t i = 0; i < n_strings; ++i) {
    Rng r(key(seed, 3 * (uint64_t)i + 1));
    int64_t add = end_special >= 0 ? sp_len(end_special) : 0;
    for (int64_t c = plan(i, r); c > 0; --c) add += sp_len(r.below((uint32_t)sp->n));
    out_off[i + 1] = out_off[i] + (off[i + 1] - off[i]) + add;
  }
  if (!out_bytes) return out_off[n_strings];
  if (cap < out_off[n_strings]) return -1;
  int nt = n_threads > 0 ? n_threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  auto work = [&](int t) {
    std::vector<std::pair<int64_t, int64_t>> ins;  // (position in the string, special)
    for (int64_t i = t; i < n_strings; i += nt) {
      Rng r(key(seed, 3 * (uint64_t)i + 1));
      const int64_t n = plan(i, r);
      ins.clear();
      for (int64_t c = 0; c < n; ++c) ins.emplace_back(0, r.below((uint32_t)sp->n));
      const uint8_t* src = bytes + off[i];
      const int64_t L = off[i + 1] - off[i];
      Rng q(key(seed, 3 * (uint64_t)i + 2));
      for (auto& x : ins) {  // a random code-point boundary
        int64_t p = L > 0 ? (int64_t)q.below((uint32_t)(L + 1)) : 0;
        while (p > 0 && p < L && (src[p] & 0xC0) == 0x80) --p;
        x.first = p;
      }
      std::stable_sort(ins.begin(), ins.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
      uint8_t* dst = out_bytes + out_off[i];
      int64_t at = 0;
      for (const auto& x : ins) {
        std::memcpy(dst, src + at, (size_t)(x.first - at));
        dst += x.first - at;
        at = x.first;
        std::memcpy(dst, sp->bytes + sp->off[x.second], (size_t)sp_len(x.second));
        dst += sp_len(x.second);
      }
      std::memcpy(dst, src + at, (size_t)(L - at));
      dst += L - at;
      if (end_special >= 0) std::memcpy(dst, sp->bytes + sp->off[end_special], (size_t)sp_len(end_special));
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  return out_off[n_strings];
}
