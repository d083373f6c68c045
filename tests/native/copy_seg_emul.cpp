// CPU harness for the pipeline's copy kernels (csrc/copy_seg.h): runs the device template
// copy_seg_t itself, lane by lane, with recording memory operations, for a grid of whole waves.
// The one cross-lane operation (the realigning shuffle) is emulated exactly: each of a wave's 64
// lanes runs as a fiber (ucontext) that parks at the shuffle; when every lane has parked, lane l
// receives lane l + 1's value (lane 63 its own, as __shfl_down(x, 1, 64)) and all resume.
//
// For every case it checks the access ranges DESIGN.md §4.5 states:
//   - every write lies in [dst, dst + n), every byte of it written exactly once, with src's byte;
//   - every read lies inside [src, src + n) rounded out to 16-byte aligned blocks, and each
//     16-byte read holds at least one byte of [src, src + n) (so it is on one of the range's pages).
// It also runs the round-4 copy (unaligned 16-byte loads and stores at src + 16 i / dst + 16 i,
// then single bytes), restated here as it was in encode.hip before commit 0685c92, under the
// stricter rule that every read lies inside [src, src + n) itself.
//
// Built by tests/test_copy_seg.py with g++; entry point copy_seg_check().
#include <ucontext.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define __host__
#define __device__
#include "copy_seg.h"

namespace {

struct V4 {
  uint32_t w[4] = {0, 0, 0, 0};
  uint32_t& operator[](int i) { return w[i]; }
  const uint32_t& operator[](int i) const { return w[i]; }
};

struct Case {
  const uint8_t* src;
  uint8_t* dst;
  int64_t n;
  std::vector<int>* writes;  // per dst byte
  const char* err = nullptr;
  int64_t bad_addr = 0;
  bool strict_reads = false;  // (round-4 rule: reads inside [src, src + n))
};

struct Wave;
struct EmuOps {
  using V = V4;
  Case* c;
  Wave* w;
  int lane;
  void read(const uint8_t* p, int64_t size) {
    const uintptr_t a = (uintptr_t)p, lo = (uintptr_t)c->src, hi = lo + (uintptr_t)c->n;
    const uintptr_t lo16 = lo & ~(uintptr_t)15, hi16 = (hi + 15) & ~(uintptr_t)15;
    bool ok;
    if (c->strict_reads) ok = a >= lo && a + size <= hi;
    else ok = a >= lo16 && a + size <= hi16 && a < hi && a + size > lo;  // (overlaps the range)
    if (!ok && !c->err) { c->err = "read outside the source range"; c->bad_addr = (int64_t)(a - lo); }
  }
  void write(uint8_t* p, int64_t size) {
    const uintptr_t a = (uintptr_t)p, lo = (uintptr_t)c->dst, hi = lo + (uintptr_t)c->n;
    if (a < lo || a + size > hi) {
      if (!c->err) { c->err = "write outside the destination range"; c->bad_addr = (int64_t)(a - lo); }
      return;
    }
    for (int64_t k = 0; k < size; ++k) ++(*c->writes)[a - lo + k];
  }
  V ld16(const uint8_t* p) { read(p, 16); V v; std::memcpy(v.w, p, 16); return v; }
  void st16(uint8_t* p, const V& v) { write(p, 16); if (!c->err) std::memcpy(p, v.w, 16); }
  uint8_t ld1(const uint8_t* p) { read(p, 1); return *p; }
  void st1(uint8_t* p, uint8_t v) { write(p, 1); if (!c->err) *p = v; }
  uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) { return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh)); }
  V shfl_down1(const V& x);
};

// one wave of 64 fibers
struct Wave {
  ucontext_t main_ctx, ctx[64];
  std::vector<char> stacks;
  V4 slot[64], got[64];
  bool parked[64], done[64];
  Case* c;
  int64_t t0, nt;
  int version;  // 0: copy_seg_t, 1: the round-4 copy
  Wave() : stacks(64 * 65536) {}
};

// the round-4 copy (encode.hip before 0685c92): unaligned 16-byte accesses, then the tail bytes
void copy_seg_r4(EmuOps& o, const uint8_t* src, uint8_t* dst, int64_t n, int64_t t, int64_t nt) {
  const int64_t n16 = n >> 4;
  for (int64_t i = t; i < n16; i += nt) o.st16(dst + 16 * i, o.ld16(src + 16 * i));
  for (int64_t i = (n16 << 4) + t; i < n; i += nt) o.st1(dst + i, o.ld1(src + i));
}

Wave* g_wave = nullptr;

V4 EmuOps::shfl_down1(const V4& x) {
  w->slot[lane] = x;
  w->parked[lane] = true;
  swapcontext(&w->ctx[lane], &w->main_ctx);  // (resumed once every lane has parked)
  return w->got[lane];
}

void lane_entry(int lane) {
  Wave* w = g_wave;
  EmuOps o{w->c, w, lane};
  const int64_t t = w->t0 + lane;
  if (w->version == 0) sw::copy_seg_t(o, w->c->src, w->c->dst, w->c->n, t, w->nt, lane);
  else copy_seg_r4(o, w->c->src, w->c->dst, w->c->n, t, w->nt);
  w->done[lane] = true;
  swapcontext(&w->ctx[lane], &w->main_ctx);
}

// run one wave to completion; false if the lanes did not all meet at a shuffle (not wave-uniform)
bool run_wave(Wave* w) {
  g_wave = w;
  for (int l = 0; l < 64; ++l) {
    w->parked[l] = w->done[l] = false;
    getcontext(&w->ctx[l]);
    w->ctx[l].uc_stack.ss_sp = w->stacks.data() + (size_t)l * 65536;
    w->ctx[l].uc_stack.ss_size = 65536;
    w->ctx[l].uc_link = nullptr;
    makecontext(&w->ctx[l], (void (*)())lane_entry, 1, l);
  }
  while (true) {
    int n_parked = 0, n_done = 0;
    for (int l = 0; l < 64; ++l) {
      if (!w->parked[l] && !w->done[l]) swapcontext(&w->main_ctx, &w->ctx[l]);
      n_parked += w->parked[l];
      n_done += w->done[l];
    }
    if (n_done == 64) return true;
    if (n_parked + n_done != 64 || n_done != 0) return false;  // (some lanes finished while others shuffle)
    for (int l = 0; l < 64; ++l) {  // (all parked: exchange -- lane l gets lane l + 1's value -- then resume them all)
      w->got[l] = w->slot[l < 63 ? l + 1 : l];
      w->parked[l] = false;
    }
  }
}

}  // namespace

extern "C" int copy_seg_check(int version, int64_t n, int src_mis, int dst_mis, int64_t nt, char* msg, int msg_len) {
  static Wave wave;
  // buffers with 64 bytes of guard before and after; src / dst at the requested misalignment
  std::vector<uint8_t> sbuf((size_t)n + 256), dbuf((size_t)n + 256);
  uint8_t* s0 = (uint8_t*)(((uintptr_t)sbuf.data() + 63) & ~(uintptr_t)63) + 64 + src_mis;
  uint8_t* d0 = (uint8_t*)(((uintptr_t)dbuf.data() + 63) & ~(uintptr_t)63) + 64 + dst_mis;
  for (size_t i = 0; i < sbuf.size(); ++i) sbuf[i] = (uint8_t)(i * 131 + 7);
  std::memset(dbuf.data(), 0xEE, dbuf.size());
  std::vector<int> writes((size_t)n, 0);
  Case c{s0, d0, n, &writes};
  c.strict_reads = version == 1;
  wave.c = &c;
  wave.version = version;
  wave.nt = nt;
  for (int64_t t0 = 0; t0 < nt; t0 += 64) {
    wave.t0 = t0;
    if (!run_wave(&wave)) {
      std::snprintf(msg, msg_len, "lanes diverged at a shuffle (n=%lld)", (long long)n);
      return 1;
    }
    if (c.err) {
      std::snprintf(msg, msg_len, "%s at offset %lld (n=%lld src_mis=%d dst_mis=%d nt=%lld)", c.err,
                    (long long)c.bad_addr, (long long)n, src_mis, dst_mis, (long long)nt);
      return 1;
    }
  }
  for (int64_t i = 0; i < n; ++i) {
    if (writes[i] != 1 || d0[i] != s0[i]) {
      std::snprintf(msg, msg_len, "byte %lld written %d times / wrong value (n=%lld src_mis=%d dst_mis=%d)", (long long)i,
                    writes[i], (long long)n, src_mis, dst_mis);
      return 1;
    }
  }
  for (uint8_t* p = dbuf.data(); p < dbuf.data() + dbuf.size(); ++p)
    if ((p < d0 || p >= d0 + n) && *p != 0xEE) {
      std::snprintf(msg, msg_len, "guard byte changed at %lld", (long long)(p - d0));
      return 1;
    }
  return 0;
}
