// MI355X decode: token ids -> the bytes of their vocabulary entries, per string (the byte join
// of a tokenizer's decode over build_vocab, shredword/base.py:60-79).  The UTF-8 decoding with
// errors="replace" stays with the caller (Python's bytes.decode), as it is per string.
//
// Device pipeline (one stream):
//   k_decode_len      byte length of every id (0 and an error flag for an id not in the vocab)
//   launch_scan       exclusive scan of the lengths: every id's output position
//   k_decode_copy     each id's bytes to its position (one lane per id, vocab bytes L2-resident)
//   k_decode_offsets  per-string byte offsets from the per-string id offsets
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "capi.h"
#include "shredword_hip.h"

using namespace sw;

namespace {

constexpr uint32_t kUndef = 0xFFFFFFFFu;  // vocabulary entry: no such id

__global__ void __launch_bounds__(256) k_decode_len(const int32_t* ids, int64_t n, const uint2* vtab, int64_t n_vocab,
                                                    uint32_t* len, int32_t* err) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int32_t t = ids[i];
  uint32_t L = 0;
  if (t >= 0 && t < n_vocab) {
    const uint2 e = vtab[t];
    if (e.y != kUndef) L = e.y;
    else atomicOr(err, 1);
  } else {
    atomicOr(err, 1);
  }
  len[i] = L;
}

__global__ void __launch_bounds__(256) k_decode_copy(const int32_t* ids, int64_t n, const uint2* vtab,
                                                     int64_t n_vocab, const uint8_t* vbytes, const int64_t* base,
                                                     uint8_t* out, int64_t cap) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int32_t t = ids[i];
  if (t < 0 || t >= n_vocab) return;
  const uint2 e = vtab[t];
  if (e.y == kUndef) return;
  const int64_t p = base[i];
  if (p + (int64_t)e.y > cap) return;  // (the call reports SW_ERR_CAP)
  const uint8_t* src = vbytes + e.x;
  for (uint32_t k = 0; k < e.y; ++k) out[p + k] = src[k];
}

__global__ void k_decode_offsets(const int64_t* id_off, int64_t n_str, int64_t n_ids, const int64_t* base,
                                 const int64_t* total, int64_t* out_off) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n_str) return;
  const int64_t j = id_off[s];
  out_off[s] = j >= n_ids ? *total : base[j];
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

}  // namespace

struct sw_decoder {
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t n_vocab = 0;
  uint2* d_vtab = nullptr;       // [n_vocab] (start, length) into d_vbytes; length kUndef: not an id
  uint8_t* d_vbytes = nullptr;
  // workspace, grown on demand
  int64_t cap_ids = -1;
  uint32_t* d_len = nullptr;
  int64_t* d_base = nullptr;
  int64_t* d_part = nullptr;
  int64_t* d_total = nullptr;
  int32_t* d_err = nullptr;
  // host-path staging
  int64_t io_ids = -1, io_str = -1, io_bytes = -1;
  int32_t* d_ids = nullptr;
  int64_t* d_id_off = nullptr;
  int64_t* d_out_off = nullptr;
  uint8_t* d_out = nullptr;
};

static void free_decoder_ws(sw_decoder* d) {
  (void)hipFree(d->d_len); (void)hipFree(d->d_base); (void)hipFree(d->d_part); (void)hipFree(d->d_total);
  (void)hipFree(d->d_err);
  d->d_len = nullptr; d->d_base = nullptr; d->d_part = nullptr; d->d_total = nullptr; d->d_err = nullptr;
  d->cap_ids = -1;
}

static void free_decoder_io(sw_decoder* d) {
  (void)hipFree(d->d_ids); (void)hipFree(d->d_id_off); (void)hipFree(d->d_out_off); (void)hipFree(d->d_out);
  d->d_ids = nullptr; d->d_id_off = nullptr; d->d_out_off = nullptr; d->d_out = nullptr;
  d->io_ids = d->io_str = d->io_bytes = -1;
}

static int32_t ensure_decoder_ws(sw_decoder* d, int64_t n_ids) {
  if (n_ids <= d->cap_ids) return SW_OK;
  free_decoder_ws(d);
  const int64_t n = std::max<int64_t>(n_ids, 1024);
  const int64_t parts = (n + scan_block() - 1) / scan_block();
  SW_HIP_TRY(hipMalloc(&d->d_len, sizeof(uint32_t) * n));
  SW_HIP_TRY(hipMalloc(&d->d_base, sizeof(int64_t) * n));
  SW_HIP_TRY(hipMalloc(&d->d_part, sizeof(int64_t) * (parts + 1)));
  SW_HIP_TRY(hipMalloc(&d->d_total, sizeof(int64_t)));
  SW_HIP_TRY(hipMalloc(&d->d_err, sizeof(int32_t)));
  d->cap_ids = n;
  return SW_OK;
}

extern "C" int32_t sw_decoder_create(const uint8_t* vocab_bytes, const int64_t* vocab_off, const uint8_t* defined,
                                     int64_t n_vocab, int32_t device, sw_decoder** out) {
  if (!out || n_vocab < 0 || (n_vocab > 0 && (!vocab_off || !defined)) || n_vocab > 0x7FFFFFFF)
    return set_error(SW_ERR_ARG, "sw_decoder_create: bad arguments");
  *out = nullptr;
  const int64_t total = n_vocab > 0 ? vocab_off[n_vocab] - vocab_off[0] : 0;
  if (total < 0 || total >= (int64_t)kUndef || (total > 0 && !vocab_bytes))
    return set_error(SW_ERR_ARG, "sw_decoder_create: bad vocabulary offsets");
  std::vector<uint2> tab((size_t)std::max<int64_t>(n_vocab, 1));
  for (int64_t t = 0; t < n_vocab; ++t) {
    const int64_t a = vocab_off[t] - vocab_off[0], b = vocab_off[t + 1] - vocab_off[0];
    if (b < a || b > total) return set_error(SW_ERR_ARG, "sw_decoder_create: vocabulary offsets not ascending");
    tab[t] = defined[t] ? make_uint2((uint32_t)a, (uint32_t)(b - a)) : make_uint2(0, kUndef);
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return set_error(SW_ERR_NODEV, "sw_decoder_create: no HIP device visible");
  if (device < 0 || device >= ndev) return set_error(SW_ERR_ARG, "sw_decoder_create: bad device ordinal");
  DeviceGuard g(device);
  sw_decoder* d = new sw_decoder();
  d->device = device;
  d->n_vocab = n_vocab;
  hipError_t e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&d->d_vtab, sizeof(uint2) * tab.size());
  if (e == hipSuccess) e = hipMalloc(&d->d_vbytes, (size_t)std::max<int64_t>(total, 1));
  if (e == hipSuccess) e = hipMemcpy(d->d_vtab, tab.data(), sizeof(uint2) * tab.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && total > 0)
    e = hipMemcpy(d->d_vbytes, vocab_bytes + vocab_off[0], (size_t)total, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    sw_decoder_destroy(d);
    return set_error(SW_ERR_HIP, std::string("sw_decoder_create: ") + hipGetErrorString(e));
  }
  *out = d;
  return SW_OK;
}

extern "C" void sw_decoder_destroy(sw_decoder* d) {
  if (!d) return;
  DeviceGuard g(d->device);
  free_decoder_ws(d);
  free_decoder_io(d);
  (void)hipFree(d->d_vtab);
  (void)hipFree(d->d_vbytes);
  if (d->stream) (void)hipStreamDestroy(d->stream);
  delete d;
}

extern "C" int32_t sw_decode_device(sw_decoder* d, const int32_t* d_ids, int64_t n_ids, const int64_t* d_id_off,
                                    int64_t n_str, uint8_t* d_out, int64_t out_cap, int64_t* d_out_off, void* stream,
                                    int64_t* n_bytes_host) {
  if (!d || n_ids < 0 || n_str < 0 || out_cap < 0 || !d_id_off || !d_out_off || (n_ids > 0 && !d_ids) ||
      (out_cap > 0 && !d_out))
    return set_error(SW_ERR_ARG, "sw_decode_device: bad arguments");
  DeviceGuard g(d->device);
  hipStream_t st = (hipStream_t)stream;  // (NULL: the null stream)
  int32_t rc = ensure_decoder_ws(d, n_ids);
  if (rc) return rc;
  SW_HIP_TRY(hipMemsetAsync(d->d_err, 0, sizeof(int32_t), st));
  if (n_ids > 0) {
    const dim3 grid((unsigned)((n_ids + 255) / 256));
    hipLaunchKernelGGL(k_decode_len, grid, dim3(256), 0, st, d_ids, n_ids, d->d_vtab, d->n_vocab, d->d_len, d->d_err);
    SW_HIP_TRY(launch_scan(st, d->d_len, n_ids, d->d_part, d->d_base, d->d_total));
    hipLaunchKernelGGL(k_decode_copy, grid, dim3(256), 0, st, d_ids, n_ids, d->d_vtab, d->n_vocab, d->d_vbytes,
                       d->d_base, d_out, out_cap);
  } else {
    SW_HIP_TRY(hipMemsetAsync(d->d_total, 0, sizeof(int64_t), st));
  }
  hipLaunchKernelGGL(k_decode_offsets, dim3((unsigned)((n_str + 1 + 255) / 256)), dim3(256), 0, st, d_id_off, n_str,
                     n_ids, d->d_base, d->d_total, d_out_off);
  SW_HIP_TRY(hipGetLastError());
  if (n_bytes_host) {
    int64_t total = 0;
    int32_t err = 0;
    SW_HIP_TRY(hipMemcpyAsync(&total, d->d_total, sizeof(total), hipMemcpyDeviceToHost, st));
    SW_HIP_TRY(hipMemcpyAsync(&err, d->d_err, sizeof(err), hipMemcpyDeviceToHost, st));
    SW_HIP_TRY(hipStreamSynchronize(st));
    *n_bytes_host = total;
    if (err) return set_error(SW_ERR_ARG, "sw_decode_device: an id is not in the vocabulary");
    if (total > out_cap) return set_error(SW_ERR_CAP, "sw_decode_device: output capacity too small");
  }
  return SW_OK;
}

extern "C" int32_t sw_decode_batch(sw_decoder* d, const int32_t* ids, const int64_t* id_off, int64_t n_str,
                                   uint8_t* out, int64_t out_cap, int64_t* out_off) {
  if (!d || n_str < 0 || !id_off || !out_off || out_cap < 0 || (out_cap > 0 && !out))
    return set_error(SW_ERR_ARG, "sw_decode_batch: bad arguments");
  const int64_t i0 = id_off[0], n_ids = id_off[n_str] - i0;
  if (n_ids < 0 || (n_ids > 0 && !ids)) return set_error(SW_ERR_ARG, "sw_decode_batch: bad id offsets");
  DeviceGuard g(d->device);
  if (n_ids > d->io_ids || n_str > d->io_str || out_cap > d->io_bytes) {
    free_decoder_io(d);
    SW_HIP_TRY(hipMalloc(&d->d_ids, sizeof(int32_t) * std::max<int64_t>(n_ids, 1)));
    SW_HIP_TRY(hipMalloc(&d->d_id_off, sizeof(int64_t) * (n_str + 1)));
    SW_HIP_TRY(hipMalloc(&d->d_out_off, sizeof(int64_t) * (n_str + 1)));
    SW_HIP_TRY(hipMalloc(&d->d_out, (size_t)std::max<int64_t>(out_cap, 1)));
    d->io_ids = n_ids; d->io_str = n_str; d->io_bytes = out_cap;
  }
  std::vector<int64_t> rel((size_t)n_str + 1);
  for (int64_t s = 0; s <= n_str; ++s) rel[s] = id_off[s] - i0;
  hipStream_t st = d->stream;
  if (n_ids > 0) SW_HIP_TRY(hipMemcpyAsync(d->d_ids, ids + i0, sizeof(int32_t) * n_ids, hipMemcpyHostToDevice, st));
  SW_HIP_TRY(hipMemcpyAsync(d->d_id_off, rel.data(), sizeof(int64_t) * (n_str + 1), hipMemcpyHostToDevice, st));
  int64_t total = 0;
  int32_t rc = sw_decode_device(d, d->d_ids, n_ids, d->d_id_off, n_str, d->d_out, out_cap, d->d_out_off, st, &total);
  if (rc) return rc;
  if (total > 0) SW_HIP_TRY(hipMemcpyAsync(out, d->d_out, (size_t)total, hipMemcpyDeviceToHost, st));
  SW_HIP_TRY(hipMemcpyAsync(out_off, d->d_out_off, sizeof(int64_t) * (n_str + 1), hipMemcpyDeviceToHost, st));
  SW_HIP_TRY(hipStreamSynchronize(st));
  return SW_OK;
}
