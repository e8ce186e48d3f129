// index_kernels.h -- index helpers shared by csr_ops.hip and spgemm.hip (internal).
#pragma once

#include "common.h"

namespace gcg {
namespace {

__global__ void iota_kernel(int32_t* __restrict__ out, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = static_cast<int32_t>(i);
}

// Row id of every nonzero (expanded indptr).
__global__ void expand_rows_kernel(int64_t n_rows, const int32_t* __restrict__ indptr,
                                   int32_t* __restrict__ row_of) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < n_rows; r += stride)
    for (int32_t j = indptr[r]; j < indptr[r + 1]; ++j) row_of[j] = static_cast<int32_t>(r);
}

}  // namespace
}  // namespace gcg
