// PCIe probe for sw_encode_batch's pipeline: host<->device copy rates for one 64 MiB run by
// SDMA (hipMemcpyAsync, one stream or split over several) and by a kernel reading/writing the
// pinned host buffer directly, plus host-side staging rates.  Not part of the library.
//   hipcc --offload-arch=gfx950 -O2 -o tools/h2d_probe tools/h2d_probe.hip -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void k_pull(const v4u* __restrict__ src, v4u* __restrict__ dst, long n16) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x)
    dst[i] = __builtin_nontemporal_load(src + i);
}

__global__ void k_push(const v4u* __restrict__ src, v4u* __restrict__ dst, long n16) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(src[i], dst + i);
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t N = 64ull << 20;
  const int reps = 8;
  uint8_t *h_a, *h_b, *d_a, *d_b;
  CK(hipHostMalloc((void**)&h_a, N, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&h_b, N, hipHostMallocDefault));
  CK(hipMalloc(&d_a, N));
  CK(hipMalloc(&d_b, N));
  std::memset(h_a, 1, N);
  std::memset(h_b, 2, N);
  hipStream_t s[4];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  auto gbs = [&](double ms, double bytes) { return bytes / ms / 1e6; };

  // each configuration twice (the first pass of a kind can include one-time setup)
  auto sdma = [&](int dir, size_t lo, size_t hi, hipStream_t st) {
    if (dir == 0) CK(hipMemcpyAsync(d_a + lo, h_a + lo, hi - lo, hipMemcpyHostToDevice, st));
    else CK(hipMemcpyAsync(h_b + lo, d_b + lo, hi - lo, hipMemcpyDeviceToHost, st));
  };
  auto kern = [&](int dir, size_t bytes, int blocks, hipStream_t st) {
    if (dir == 0) hipLaunchKernelGGL(k_pull, dim3(blocks), dim3(256), 0, st, (const v4u*)h_a, (v4u*)d_a, (long)(bytes / 16));
    else hipLaunchKernelGGL(k_push, dim3(blocks), dim3(256), 0, st, (const v4u*)d_b, (v4u*)h_b, (long)(bytes / 16));
  };
  auto timed = [&](const char* name, double bytes, const std::function<void()>& body) {
    for (int pass = 0; pass < 2; ++pass) {
      CK(hipDeviceSynchronize());
      double t = now_ms();
      for (int r = 0; r < reps; ++r) body();
      CK(hipDeviceSynchronize());
      t = now_ms() - t;
      std::printf("%-48s pass %d: %6.1f GB/s  (%.3f ms per rep)\n", name, pass, gbs(t, bytes * reps), t / reps);
    }
  };
  timed("sdma H2D 64M", N, [&] { sdma(0, 0, N, s[0]); });
  timed("sdma D2H 64M", N, [&] { sdma(1, 0, N, s[0]); });
  timed("sdma H2D 64M as 2 streams", N, [&] { sdma(0, 0, N / 2, s[0]); sdma(0, N / 2, N, s[1]); });
  timed("sdma H2D 64M as 4 streams", N, [&] { for (int k = 0; k < 4; ++k) sdma(0, N * k / 4, N * (k + 1) / 4, s[k]); });
  timed("sdma H2D 64M + sdma D2H 32M", 1.5 * N, [&] { sdma(0, 0, N, s[0]); sdma(1, 0, N / 2, s[1]); });
  for (int blocks : {32, 64, 128, 256}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "kernel pull 64M, %d blocks", blocks);
    timed(nm, N, [&] { kern(0, N, blocks, s[0]); });
    std::snprintf(nm, sizeof nm, "kernel push 64M, %d blocks", blocks);
    timed(nm, N, [&] { kern(1, N, blocks, s[0]); });
  }
  timed("kernel pull 64M + sdma D2H 32M", 1.5 * N, [&] { kern(0, N, 128, s[0]); sdma(1, 0, N / 2, s[1]); });
  timed("kernel pull 64M + kernel push 32M", 1.5 * N, [&] { kern(0, N, 128, s[0]); kern(1, N / 2, 64, s[1]); });
  timed("sdma H2D 64M + kernel push 32M", 1.5 * N, [&] { sdma(0, 0, N, s[0]); kern(1, N / 2, 64, s[1]); });
  // host side: pageable -> pinned staging, and first-touch writes into fresh pageable memory
  {
    std::vector<uint8_t> src(N, 3);
    for (int th : {1, 4, 8, 16}) {
      double t = now_ms();
      for (int r = 0; r < reps; ++r) {
        std::vector<std::thread> ts;
        for (int k = 0; k < th; ++k)
          ts.emplace_back([&, k] { std::memcpy(h_a + N * k / th, src.data() + N * k / th, N / th); });
        for (auto& x : ts) x.join();
      }
      t = now_ms() - t;
      std::printf("host memcpy pageable->pinned %d threads: %.1f GB/s\n", th, gbs(t, (double)N * reps));
    }
    for (int th : {1, 8, 16}) {
      const size_t M = 256ull << 20;
      uint8_t* fresh = (uint8_t*)std::malloc(M);
      double t = now_ms();
      std::vector<std::thread> ts;
      for (int k = 0; k < th; ++k)
        ts.emplace_back([&, k] { std::memset(fresh + M * k / th, 5, M / th); });
      for (auto& x : ts) x.join();
      t = now_ms() - t;
      std::printf("host first-touch write 256M %d threads: %.1f GB/s\n", th, gbs(t, (double)M));
      std::free(fresh);
    }
  }
  std::printf("done\n");
  return 0;
}
