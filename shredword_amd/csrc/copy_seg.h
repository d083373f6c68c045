// copy_seg: the pipeline's PCIe copies as kernels (encode.hip: k_copy_segs uploads a run's input,
// k_push_direct / k_push_run write its ids and offsets into pinned host memory).  Staging buffers
// are hipHostMalloc'd (page aligned) and device buffers hipMalloc'd, but two paths hand over
// arbitrary offsets: the caller's pinned input (a run starts at any byte) and the caller's pinned
// output (a run's ids start at any id), so the copy aligns the destination with a head of single
// bytes and then reads the source as aligned 16-byte blocks, each lane taking its neighbour's
// block (a shuffle) to realign.
//
// Access ranges (checked for every src / dst misalignment and length class by
// tests/native/copy_seg_emul.cpp, which runs this same template with recording memory operations
// and a 64-lane emulation of the shuffle):
//   - writes: exactly [dst, dst + n), each byte once;
//   - reads: inside [src, src + n) rounded out to whole 16-byte aligned blocks, and every block read
//     holds at least one byte of [src, src + n) -- an aligned block never crosses a page, so no read
//     touches a page that holds no byte of the source range.
//
// Ops supplies the memory and lane operations: DevCopyOps below on the device; the emulation's
// recording operations in the CPU harness.
#pragma once
#include <cstdint>

namespace sw {

template <class Ops>
__host__ __device__ inline typename Ops::V copy_realign16(Ops& o, const typename Ops::V& lo, const typename Ops::V& hi,
                                                          uint32_t r) {  // bytes [r, r + 16) of lo | hi (0 < r < 16)
  const uint32_t w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  const uint32_t sh = r & 3;
  typename Ops::V v{};
  switch (r >> 2) {  // (uniform: no dynamically indexed registers)
    case 0: v[0] = o.alignbyte(w[1], w[0], sh); v[1] = o.alignbyte(w[2], w[1], sh);
            v[2] = o.alignbyte(w[3], w[2], sh); v[3] = o.alignbyte(w[4], w[3], sh); break;
    case 1: v[0] = o.alignbyte(w[2], w[1], sh); v[1] = o.alignbyte(w[3], w[2], sh);
            v[2] = o.alignbyte(w[4], w[3], sh); v[3] = o.alignbyte(w[5], w[4], sh); break;
    case 2: v[0] = o.alignbyte(w[3], w[2], sh); v[1] = o.alignbyte(w[4], w[3], sh);
            v[2] = o.alignbyte(w[5], w[4], sh); v[3] = o.alignbyte(w[6], w[5], sh); break;
    default: v[0] = o.alignbyte(w[4], w[3], sh); v[1] = o.alignbyte(w[5], w[4], sh);
             v[2] = o.alignbyte(w[6], w[5], sh); v[3] = o.alignbyte(w[7], w[6], sh); break;
  }
  return v;
}

// dst[0, n) = src[0, n); t / nt: this thread's index in the grid and the grid's size (whole waves);
// lane: t's lane in its wave (t - lane is the wave's first thread)
template <class Ops>
__host__ __device__ inline void copy_seg_t(Ops& o, const uint8_t* src, uint8_t* dst, int64_t n, int64_t t, int64_t nt,
                                           int lane) {
  using V = typename Ops::V;
  const int64_t to16 = (int64_t)((16 - ((uintptr_t)dst & 15)) & 15);
  const int64_t head = n < to16 ? n : to16;
  for (int64_t i = t; i < head; i += nt) o.st1(dst + i, o.ld1(src + i));
  src += head;
  dst += head;
  n -= head;
  const int64_t n16 = n >> 4;
  const uint32_t mis = (uint32_t)((uintptr_t)src & 15);
  if (mis == 0) {
    for (int64_t i = t; i < n16; i += nt) o.st16(dst + 16 * i, o.ld16(src + 16 * i));
  } else {
    // block i of dst = bytes [mis, mis + 16) of the aligned source blocks i, i + 1 (block n16 holds
    // the last bytes block n16 - 1 needs: it begins inside the range, so it lies on one of its pages)
    const uint8_t* s = src - mis;
    for (int64_t i0 = t - lane; i0 < n16; i0 += nt) {  // (wave-uniform: every lane takes the shuffle)
      const int64_t i = i0 + lane;
      V x{};
      if (i <= n16) x = o.ld16(s + 16 * i);
      V y = o.shfl_down1(x);
      if (lane == 63 && i + 1 <= n16) y = o.ld16(s + 16 * (i + 1));
      if (i < n16) o.st16(dst + 16 * i, copy_realign16(o, x, y, mis));
    }
  }
  for (int64_t i = (n16 << 4) + t; i < n; i += nt) o.st1(dst + i, o.ld1(src + i));
}

#ifdef __HIPCC__
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
struct DevCopyOps {
  using V = v4u32;
  __device__ V ld16(const uint8_t* p) { return __builtin_nontemporal_load((const V*)p); }
  __device__ void st16(uint8_t* p, const V& v) { *(V*)p = v; }
  __device__ uint8_t ld1(const uint8_t* p) { return *p; }
  __device__ void st1(uint8_t* p, uint8_t v) { *p = v; }
  __device__ V shfl_down1(const V& x) {
    V y;
    y[0] = (uint32_t)__shfl_down((int)x[0], 1, 64); y[1] = (uint32_t)__shfl_down((int)x[1], 1, 64);
    y[2] = (uint32_t)__shfl_down((int)x[2], 1, 64); y[3] = (uint32_t)__shfl_down((int)x[3], 1, 64);
    return y;
  }
  __device__ uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) { return __builtin_amdgcn_alignbyte(hi, lo, sh); }
};

__device__ inline void copy_seg(const uint8_t* src, uint8_t* dst, int64_t n, int64_t t, int64_t nt) {
  DevCopyOps o;
  copy_seg_t(o, src, dst, n, t, nt, (int)(threadIdx.x & 63));
}
#endif

}  // namespace sw
