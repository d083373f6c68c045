// Multi-GPU reassembly, step 4 of the doc-sharded encode; the reference has no
// multi-device path (its trainer is single-threaded, shredword/csrc/bpe), so this layer is the
// build's own.  After the RCCL all-gathers (shredword_amd/shard.py) every rank holds, per rank r,
// a padded block of its ids (r * width ..) and of its string offsets (r * width_s ..); one pass
// here turns them into the batch's contiguous int32 ids (16-bit transport widened on the way)
// and its rebased string offsets, on the device and without a host synchronisation (the counts
// come from the counts all-gather, in device memory).
//
// Streaming kernels: every gathered id is read once and every output written once (coalesced:
// consecutive threads own consecutive ids of one rank, and a rank's ids land contiguously).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "capi.h"
#include "shredword_hip.h"

namespace {

constexpr int kRaThreads = 256;
constexpr int kRaPer = 8;        // ids per thread (a block covers kRaThreads * kRaPer consecutive ids)
constexpr int kMaxWorld = 1024;  // ranks (displacements are computed per block in LDS)

// exclusive prefix of min(counts[r], width) over r < world into s_disp (world + 1 entries)
__device__ inline void rank_displacements(const int64_t* counts, int64_t width, int world, int64_t* s_disp) {
  if (threadIdx.x == 0) {
    int64_t d = 0;
    for (int r = 0; r < world; ++r) {
      s_disp[r] = d;
      const int64_t c = counts[r];
      d += c < 0 ? 0 : (c > width ? width : c);
    }
    s_disp[world] = d;
  }
  __syncthreads();
}

// blockIdx.y = rank; block x covers ids [x * kRaThreads * kRaPer, ..) of that rank, lane-interleaved
template <typename T>
__global__ void __launch_bounds__(kRaThreads) k_reassemble_ids(const T* __restrict__ recv, const int64_t* counts,
                                                               int64_t width, int world, int32_t* __restrict__ out) {
  __shared__ int64_t s_disp[kMaxWorld + 1];
  rank_displacements(counts, width, world, s_disp);
  const int r = blockIdx.y;
  const int64_t n = s_disp[r + 1] - s_disp[r];
  const int64_t j0 = (int64_t)blockIdx.x * kRaThreads * kRaPer + threadIdx.x;
  if (j0 >= n) return;
  const T* src = recv + (int64_t)r * width;
  int32_t* dst = out + s_disp[r];
  uint32_t v[kRaPer];  // (every load issued before the first store)
#pragma unroll
  for (int k = 0; k < kRaPer; ++k) {
    const int64_t j = j0 + (int64_t)k * kRaThreads;
    v[k] = j < n ? (sizeof(T) == 2 ? (uint32_t)(uint16_t)__builtin_nontemporal_load(src + j)
                                   : (uint32_t)__builtin_nontemporal_load(src + j))
                 : 0u;
  }
#pragma unroll
  for (int k = 0; k < kRaPer; ++k) {
    const int64_t j = j0 + (int64_t)k * kRaThreads;
    if (j < n) __builtin_nontemporal_store((int32_t)v[k], dst + j);
  }
}

// string offsets: rank r's offsets rebased by the ids before it; the last one = the total
__global__ void __launch_bounds__(kRaThreads) k_reassemble_offsets(const int64_t* recv_off, const int64_t* n_strs,
                                                                   int64_t width_s, const int64_t* counts, int64_t width,
                                                                   int world, int64_t* out_off) {
  __shared__ int64_t s_disp[kMaxWorld + 1];
  __shared__ int64_t s_sdisp[kMaxWorld + 1];
  rank_displacements(counts, width, world, s_disp);
  rank_displacements(n_strs, width_s, world, s_sdisp);
  const int r = blockIdx.y;
  const int64_t n = s_sdisp[r + 1] - s_sdisp[r];
  const int64_t j = (int64_t)blockIdx.x * kRaThreads + threadIdx.x;
  if (r == world - 1 && j == 0) out_off[s_sdisp[world]] = s_disp[world];
  if (j >= n) return;
  out_off[s_sdisp[r] + j] = recv_off[(int64_t)r * width_s + j] + s_disp[r];
}

}  // namespace

extern "C" int32_t sw_reassemble_device(const void* d_recv, int32_t id_bits, const int64_t* d_counts, int64_t width,
                                        const int64_t* d_recv_off, const int64_t* d_n_strs, int64_t width_s,
                                        int32_t world, int32_t* d_out_ids, int64_t* d_out_off, void* stream) {
  if (world < 1 || world > kMaxWorld || width < 0 || width_s < 0 || (id_bits != 16 && id_bits != 32) || !d_counts ||
      !d_n_strs || !d_out_off || (width > 0 && (!d_recv || !d_out_ids)) || (width_s > 0 && !d_recv_off))
    return sw::set_error(SW_ERR_ARG, "sw_reassemble_device: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (width > 0) {
    const int64_t per_block = (int64_t)kRaThreads * kRaPer;
    const dim3 grid((unsigned)((width + per_block - 1) / per_block), (unsigned)world);
    if (id_bits == 16)
      hipLaunchKernelGGL(k_reassemble_ids<uint16_t>, grid, dim3(kRaThreads), 0, st, (const uint16_t*)d_recv, d_counts,
                         width, (int)world, d_out_ids);
    else
      hipLaunchKernelGGL(k_reassemble_ids<int32_t>, grid, dim3(kRaThreads), 0, st, (const int32_t*)d_recv, d_counts,
                         width, (int)world, d_out_ids);
  }
  const dim3 grid_s((unsigned)((std::max<int64_t>(width_s, 1) + kRaThreads - 1) / kRaThreads), (unsigned)world);
  hipLaunchKernelGGL(k_reassemble_offsets, grid_s, dim3(kRaThreads), 0, st, d_recv_off, d_n_strs, width_s, d_counts,
                     width, (int)world, d_out_off);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sw::set_error(SW_ERR_HIP, std::string("sw_reassemble_device: ") + hipGetErrorString(e));
  return SW_OK;
}
