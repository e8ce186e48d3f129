// graph_build.hip -- the normalized graph operator H = D^-1/2 (A+I) D^-1/2 built on the
// device from an undirected edge list (tensormain.py:170-181; see gcg_normalize_adjacency_f32).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "common.h"

using namespace gcg;

namespace {

// ---- graph operator construction (tensormain.py:170-180) -------------------------------
// Edge (u, v) -> keys u*n+v and v*n+u, plus i*n+i for every node (setdiag(1)).
__global__ void edge_keys_kernel(int64_t n, int64_t n_edges, const int32_t* __restrict__ u,
                                 const int32_t* __restrict__ v, int self_loops,
                                 uint64_t* __restrict__ keys, int32_t* __restrict__ status) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < n_edges; e += stride) {
    const int64_t a = u[e], b = v[e];
    if (a < 0 || b < 0 || a >= n || b >= n) {
      atomicMax(status, int32_t(GCG_ERR_BAD_CSR));
      keys[2 * e] = keys[2 * e + 1] = static_cast<uint64_t>(n) * n;  // sorts past every real key
      continue;
    }
    keys[2 * e] = static_cast<uint64_t>(a) * n + b;
    keys[2 * e + 1] = static_cast<uint64_t>(b) * n + a;
  }
  if (self_loops)
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
      keys[2 * n_edges + i] = static_cast<uint64_t>(i) * n + i;
}

// Sorted unique keys -> CSR: indices, and row_start flags via lower bound on rows.
__global__ void keys_to_csr_kernel(int64_t n, const uint64_t* __restrict__ keys,
                                   const int64_t* __restrict__ n_unique,
                                   int32_t* __restrict__ indices) {
  const int64_t m = *n_unique;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < m; k += stride)
    indices[k] = static_cast<int32_t>(keys[k] % static_cast<uint64_t>(n));
}

__global__ void row_ptr_from_keys_kernel(int64_t n, const uint64_t* __restrict__ keys,
                                         const int64_t* __restrict__ n_unique,
                                         int32_t* __restrict__ indptr) {
  const int64_t m = *n_unique;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r <= n; r += stride) {
    const uint64_t target = static_cast<uint64_t>(r) * n;  // first key of row r
    int64_t lo = 0, hi = m;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < target) lo = mid + 1; else hi = mid;
    }
    indptr[r] = static_cast<int32_t>(lo);
  }
}

// d_i^-1/2 in float64 exactly as numpy: 1.0 / sqrt(double(deg)), inf -> 0.
__global__ void dinv_kernel(int64_t n, const int32_t* __restrict__ indptr, double* __restrict__ dinv) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const double d = static_cast<double>(indptr[i + 1] - indptr[i]);
    dinv[i] = d > 0.0 ? 1.0 / sqrt(d) : 0.0;
  }
}

// H_ij = float32( float64(d_i^-1/2 * d_j^-1/2) ): the D*adj*D entry, then .astype(float32).
__global__ void norm_vals_kernel(int64_t n, const int32_t* __restrict__ indptr,
                                 const int32_t* __restrict__ indices,
                                 const double* __restrict__ dinv, float* __restrict__ vals) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < n; r += stride) {
    const double di = dinv[r];
    for (int32_t k = indptr[r]; k < indptr[r + 1]; ++k)
      vals[k] = static_cast<float>(di * dinv[indices[k]]);
  }
}

}  // namespace

extern "C" {

gcg_status gcg_normalize_adjacency_f32(int64_t n, int64_t n_edges, const int32_t* u,
                                       const int32_t* v, int self_loops, int32_t* indptr,
                                       int32_t* indices, float* vals, int64_t* nnz_dev,
                                       void* workspace, size_t workspace_bytes,
                                       size_t* workspace_needed, int32_t* status_dev,
                                       gcg_stream_t stream) {
  if (n < 0 || n >= INT32_MAX || n_edges < 0 || (n > 0 && static_cast<double>(n) * n > 1.8e19))
    return fail(GCG_ERR_INVALID_ARG, "bad sizes");
  const int64_t m = 2 * n_edges + (self_loops ? n : 0);
  if (m > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "too many entries for int32 CSR");
  int end_bit = 1;
  while (end_bit < 64 && (uint64_t{1} << end_bit) <= static_cast<uint64_t>(n) * n) ++end_bit;
  size_t t_sort = 0, t_uniq = 0;
  {
    uint64_t* k = nullptr;
    int64_t* cnt = nullptr;
    if (hipcub::DeviceRadixSort::SortKeys(nullptr, t_sort, k, k, static_cast<int>(m), 0, end_bit) != hipSuccess ||
        hipcub::DeviceSelect::Unique(nullptr, t_uniq, k, k, cnt, static_cast<int>(m)) != hipSuccess)
      return fail(GCG_ERR_HIP, "hipcub sizing failed");
  }
  const size_t kb = align_up(static_cast<size_t>(m) * sizeof(uint64_t), 256);
  const size_t db = align_up(static_cast<size_t>(n) * sizeof(double), 256);
  const size_t need = 2 * kb + db + align_up(std::max(t_sort, t_uniq), 256);
  if (workspace_needed) *workspace_needed = need;
  if (indptr == nullptr && indices == nullptr && vals == nullptr) return GCG_OK;  // sizing
  if (indptr == nullptr || nnz_dev == nullptr || status_dev == nullptr ||
      (m > 0 && (indices == nullptr || vals == nullptr)) || (n_edges > 0 && (u == nullptr || v == nullptr)))
    return fail(GCG_ERR_INVALID_ARG, "NULL buffer");
  if (workspace_bytes < need || workspace == nullptr)
    return fail(GCG_ERR_WORKSPACE, "workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = static_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(workspace);
  uint64_t* keys = reinterpret_cast<uint64_t*>(w);
  uint64_t* sorted = reinterpret_cast<uint64_t*>(w + kb);
  double* dinv = reinterpret_cast<double*>(w + 2 * kb);
  void* tmp = w + 2 * kb + db;
  GCG_HIP_CHECK(hipMemsetAsync(status_dev, 0, sizeof(int32_t), st));
  GCG_HIP_CHECK(hipMemsetAsync(nnz_dev, 0, sizeof(int64_t), st));
  if (m > 0) {
    hipLaunchKernelGGL(edge_keys_kernel, dim3(grid_for(std::max(n_edges, n))), dim3(256), 0, st, n,
                       n_edges, u, v, self_loops, keys, status_dev);
    GCG_HIP_CHECK(hipGetLastError());
    size_t ts = t_sort;
    GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp, ts, keys, sorted, static_cast<int>(m), 0, end_bit, st));
    size_t tu = t_uniq;
    // Duplicate edges collapse (binary adjacency, as networkx holds one edge per pair).
    GCG_HIP_CHECK(hipcub::DeviceSelect::Unique(tmp, tu, sorted, keys, nnz_dev, static_cast<int>(m), st));
    hipLaunchKernelGGL(keys_to_csr_kernel, dim3(grid_for(m)), dim3(256), 0, st, n, keys, nnz_dev, indices);
    GCG_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(row_ptr_from_keys_kernel, dim3(grid_for(n + 1)), dim3(256), 0, st, n, keys,
                     nnz_dev, indptr);
  GCG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(dinv_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, indptr, dinv);
  GCG_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(norm_vals_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, indptr, indices, dinv, vals);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}


}  // extern "C"
