// Whole-chunk table: byte strings of 2..16 bytes whose exact encoding is ONE token.
//
// Built once per merge table at encoder creation (host side, chunktable.cpp).  Candidates are
// the byte strings of the vocabulary (build_vocab, shredword/base.py:60-79); each candidate B
// is encoded with the exact merge loop and kept iff encode(B) == [T].  At encode time a chunk
// whose bytes are in the table is answered with T directly, and every other chunk runs the
// merge loop -- so the result is identical by construction: a chunk that encodes to a single
// token T necessarily has bytes(T) == chunk, so the table is a perfect classifier of
// single-token chunks.  This is the same shortcut tiktoken takes ("piece is itself a token").
//
// Device layout: two two-choice cuckoo tables keyed by (bytes, length):
//   short (2..8 bytes):  16-byte entries {bytes 0-3, bytes 4-7, len << 24 | token, spill}
//   long  (9..16 bytes): 32-byte entries {bytes 0-3, 4-7, 8-11, 12-15}{len << 24 | token, spill, 0,0}
// Unused key bytes are zero; an empty entry has len 0.  Tokens >= 2^24 are not tabled.
// spill = 1 marks a bucket that is the FIRST candidate of some key stored in its second: a
// lookup whose first probe neither matches nor sees spill is a certain miss, so most lookups
// cost one memory request instead of two (entries are placed in token order, first candidate
// preferred, so the frequent chunks sit in their first bucket).  The tables are kept at most
// 10% full (kLoad, up to 2^22 buckets): one lane that needs its second candidate costs
// its whole wave batch a second dependent round trip, so few spilled buckets matter more than
// the table's size (C2 at 0.45: 2.99 ms of k_split_classify, at 0.10: 2.76; profiles/r5_ab.txt).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <unordered_map>
#include <vector>

namespace sw {

struct DevChunkTable {
  const uint4* sb;  // short buckets
  const uint4* lb;  // long buckets (2 uint4 each)
  uint32_t s_shift, s_m1, s_m2;  // m1: hash seed, m2: second-candidate multiplier
  uint32_t l_shift, l_m1, l_m2;
  uint32_t enabled;
};

// 32-bit hash of a chunk key (its bytes as LE words w0..w3, zero padded): three 32-bit
// multiplies for <= 8 bytes, five for 9..16.  `seed` is drawn per table build (m1 below).
__host__ __device__ inline uint32_t chunk_hash(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t len,
                                               uint32_t seed) {
  uint32_t h = seed ^ (len << 24);
  h = (h ^ w0) * 0x85EBCA77u;
  h ^= h >> 13;
  h = (h ^ w1) * 0xC2B2AE3Du;
  h ^= h >> 16;
  if (len > 8) {
    h = (h ^ w2) * 0x27D4EB2Fu;
    h ^= h >> 13;
    h = (h ^ w3) * 0x165667B1u;
    h ^= h >> 16;
  }
  return h;
}
// the two cuckoo candidates of a hash (shift = 32 - log2(buckets); m2 odd, per build)
__host__ __device__ inline uint32_t chunk_b1(uint32_t h, uint32_t shift) { return h >> shift; }
__host__ __device__ inline uint32_t chunk_b2(uint32_t h, uint32_t m2, uint32_t shift) {
  return ((h ^ (h >> 15)) * m2) >> shift;
}

struct ChunkTableHost {
  std::vector<uint4> sb, lb;
  uint32_t s_shift = 0, s_m1 = 0, s_m2 = 0, l_shift = 0, l_m1 = 0, l_m2 = 0;
  size_t n_short = 0, n_long = 0;
};

// dict: (a << 32 | b) -> value; order: first-insertion order of the pairs (dict order).
bool build_chunk_table(const std::unordered_map<uint64_t, int32_t>& dict, const std::vector<uint64_t>& order,
                       ChunkTableHost* out);

// Exact encode of one chunk on the host (the semantics of shredword/base.py:10-36); used by
// the table builder.
std::vector<int32_t> host_encode_chunk(const std::unordered_map<uint64_t, int32_t>& dict, const uint8_t* b, int n);

}  // namespace sw
