// Shared by the C-ABI translation units (encode.hip, decode.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace sw {

// records msg as this thread's sw_last_error() and returns code
int32_t set_error(int32_t code, const std::string& msg);

// exclusive scan of cnt[0..n) into base[0..n), the sum into *total; part: ceil(n / scan_block())
// int64 scratch words (encode.hip: k_scan_reduce / k_scan_parts / k_scan_apply).  n_dev: the
// count is min(n, *n_dev), read on the device (the grids are sized for n)
hipError_t launch_scan(hipStream_t st, const uint32_t* cnt, int64_t n, int64_t* part, int64_t* base, int64_t* total,
                       const int64_t* n_dev = nullptr);
int64_t scan_block();

}  // namespace sw

#define SW_HIP_TRY(expr)                                                                          \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return sw::set_error(SW_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)
