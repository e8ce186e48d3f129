// common.h -- shared internals of libgcg_spmm.so (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "../../include/gcg_spmm.h"

namespace gcg {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

// Record a printf-style message as this thread's gcg_last_error() and return `st`.
gcg_status fail(gcg_status st, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define GCG_HIP_CHECK(expr)                                                            \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return ::gcg::fail(GCG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));  \
  } while (0)

inline bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }
inline int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  return static_cast<int>(std::min<int64_t>(std::max<int64_t>(g, 1), 4096));
}
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
inline int bits_for(int64_t n) {
  int b = 1;
  while (b < 31 && (int64_t{1} << b) < n) ++b;
  return b;
}

namespace {  // small device helpers, one copy per translation unit

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

}  // namespace
}  // namespace gcg
