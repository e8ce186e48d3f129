// csr_ops.hip -- device CSR utilities around the SpMM: validation (scipy check_format on
// upload), CSR transpose (the X^T of Theano's grad of S.dot(X, W), mlpconv.py:71), and the
// deterministic scatter-add of rows (grad of Y[target_indices], mlpconv.py:94, with the
// duplicates tensormain.py:226 draws).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "common.h"
#include "index_kernels.h"

using namespace gcg;

namespace {


__global__ void validate_kernel(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                const int32_t* __restrict__ indptr,
                                const int32_t* __restrict__ indices, int32_t* status) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i <= n_rows; i += stride) {
    const int32_t v = indptr[i];
    bool bad = (i == 0 && v != 0) || (i == n_rows && v != nnz) || v < 0 || v > nnz ||
               (i < n_rows && indptr[i + 1] < v);
    if (bad) atomicMax(status, int32_t(GCG_ERR_BAD_CSR));
  }
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < nnz; j += stride) {
    const int32_t c = indices[j];
    if (c < 0 || c >= n_cols) atomicMax(status, int32_t(GCG_ERR_BAD_CSR));
  }
}

// seg_ptr[r] = number of sorted keys < r (lower bound), r in [0, n_rows].
__global__ void lower_bound_kernel(const int32_t* __restrict__ sorted_keys, int64_t n,
                                   int64_t n_rows, int32_t* __restrict__ seg_ptr) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r <= n_rows; r += stride) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (sorted_keys[mid] < r) lo = mid + 1; else hi = mid;
    }
    seg_ptr[r] = static_cast<int32_t>(lo);
  }
}

// out[r] += sum over i in segment r (ascending i) of src[sorted_pos[i]]; one wave per row.
__global__ __launch_bounds__(kBlock) void scatter_add_kernel(int64_t n_rows,
                                                             const int32_t* __restrict__ seg_ptr,
                                                             const int32_t* __restrict__ sorted_pos,
                                                             const float* __restrict__ src,
                                                             int64_t lds, int64_t K,
                                                             float* __restrict__ out, int64_t ldo) {
  const int64_t r = uniform(static_cast<int>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6));
  if (r >= n_rows) return;
  const int s = uniform(seg_ptr[r]), e = uniform(seg_ptr[r + 1]);
  if (s == e) return;
  const int lane = threadIdx.x & (kWave - 1);
  float* orow = out + r * ldo;
  for (int64_t c = lane; c < K; c += kWave) {
    float acc = orow[c];
    for (int i = s; i < e; ++i) acc = acc + src[static_cast<int64_t>(sorted_pos[i]) * lds + c];
    orow[c] = acc;
  }
}

__global__ void permute_transpose_kernel(int64_t nnz, const int32_t* __restrict__ perm,
                                         const int32_t* __restrict__ row_of,
                                         const float* __restrict__ vals,
                                         int32_t* __restrict__ out_indices,
                                         float* __restrict__ out_vals) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < nnz; k += stride) {
    const int32_t j = perm[k];
    out_indices[k] = row_of[j];
    out_vals[k] = vals[j];
  }
}

// Stable sort of int32 keys carrying int32 values (iota) -> sorted keys + permutation.
// Workspace layout: [keys_out n][vals_in n][vals_out n][cub temp].
gcg_status sort_pairs_ws(int64_t n, int end_bit, size_t* temp_bytes) {
  uint32_t* dk = nullptr;
  int32_t* dv = nullptr;
  size_t tb = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, dk, dk, dv, dv,
                                                    static_cast<int>(n), 0, end_bit);
  if (e != hipSuccess) return fail(GCG_ERR_HIP, "SortPairs sizing: %s", hipGetErrorString(e));
  *temp_bytes = tb;
  return GCG_OK;
}



}  // namespace

extern "C" {


gcg_status gcg_csr_validate(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t* indptr,
                            const int32_t* indices, int32_t* status_dev, gcg_stream_t stream) {
  if (n_rows < 0 || n_cols < 0 || nnz < 0 || indptr == nullptr || status_dev == nullptr ||
      (nnz > 0 && indices == nullptr))
    return fail(GCG_ERR_INVALID_ARG, "bad args to gcg_csr_validate");
  hipStream_t st = static_cast<hipStream_t>(stream);
  GCG_HIP_CHECK(hipMemsetAsync(status_dev, 0, sizeof(int32_t), st));
  hipLaunchKernelGGL(validate_kernel, dim3(grid_for(std::max(n_rows + 1, nnz))), dim3(256), 0, st,
                     n_rows, n_cols, nnz, indptr, indices, status_dev);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

gcg_status gcg_index_csr(int64_t n_idx, const int32_t* idx, int64_t n_rows, int32_t* seg_ptr,
                         int32_t* sorted_pos, void* workspace, size_t workspace_bytes,
                         size_t* workspace_needed, gcg_stream_t stream) {
  if (n_idx < 0 || n_idx > INT32_MAX || n_rows < 0 || n_rows >= INT32_MAX)
    return fail(GCG_ERR_INVALID_ARG, "bad sizes");
  const int end_bit = bits_for(n_rows + 1);
  size_t temp = 0;
  if (gcg_status s = sort_pairs_ws(n_idx, end_bit, &temp)) return s;
  const size_t nb = align_up(static_cast<size_t>(n_idx) * sizeof(int32_t), 256);
  const size_t need = 2 * nb + align_up(temp, 256);
  if (workspace_needed) *workspace_needed = need;
  if (seg_ptr == nullptr && sorted_pos == nullptr) return GCG_OK;  // sizing query
  if (seg_ptr == nullptr || (n_idx > 0 && (idx == nullptr || sorted_pos == nullptr)))
    return fail(GCG_ERR_INVALID_ARG, "NULL buffer");
  if (workspace_bytes < need || (need > 0 && workspace == nullptr))
    return fail(GCG_ERR_WORKSPACE, "workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = static_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(workspace);
  int32_t* keys_out = reinterpret_cast<int32_t*>(w);
  int32_t* vals_in = reinterpret_cast<int32_t*>(w + nb);
  void* cub_tmp = w + 2 * nb;
  if (n_idx > 0) {
    hipLaunchKernelGGL(iota_kernel, dim3(grid_for(n_idx)), dim3(256), 0, st, vals_in, n_idx);
    GCG_HIP_CHECK(hipGetLastError());
    GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(cub_tmp, temp, reinterpret_cast<const uint32_t*>(idx), reinterpret_cast<uint32_t*>(keys_out), vals_in, sorted_pos,
                                                     static_cast<int>(n_idx), 0, end_bit, st));
  }
  hipLaunchKernelGGL(lower_bound_kernel, dim3(grid_for(n_rows + 1)), dim3(256), 0, st, keys_out,
                     n_idx, n_rows, seg_ptr);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

gcg_status gcg_scatter_add_rows_f32(int64_t n_rows, const int32_t* seg_ptr,
                                    const int32_t* sorted_pos, const float* src, int64_t lds,
                                    int64_t K, float* out, int64_t ldo, gcg_stream_t stream) {
  if (n_rows < 0 || n_rows > INT32_MAX || K < 0 || lds < K || ldo < K || seg_ptr == nullptr ||
      (K > 0 && out == nullptr))
    return fail(GCG_ERR_INVALID_ARG, "bad args to gcg_scatter_add_rows_f32");
  if (n_rows == 0 || K == 0) return GCG_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(scatter_add_kernel, dim3((n_rows + kWavesPerBlock - 1) / kWavesPerBlock),
                     dim3(kBlock), 0, st, n_rows, seg_ptr, sorted_pos, src, lds, K, out, ldo);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

gcg_status gcg_csr_transpose_f32(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                 const int32_t* indptr, const int32_t* indices,
                                 const float* vals, int32_t* out_indptr, int32_t* out_indices,
                                 float* out_vals, void* workspace, size_t workspace_bytes,
                                 size_t* workspace_needed, gcg_stream_t stream) {
  if (n_rows < 0 || n_cols < 0 || nnz < 0 || nnz > INT32_MAX || n_cols >= INT32_MAX)
    return fail(GCG_ERR_INVALID_ARG, "bad sizes");
  const int end_bit = bits_for(n_cols + 1);
  size_t temp = 0;
  if (gcg_status s = sort_pairs_ws(nnz, end_bit, &temp)) return s;
  const size_t nb = align_up(static_cast<size_t>(nnz) * sizeof(int32_t), 256);
  // [sorted cols][iota][perm][row_of][cub temp]
  const size_t need = 4 * nb + align_up(temp, 256);
  if (workspace_needed) *workspace_needed = need;
  if (out_indptr == nullptr && out_indices == nullptr && out_vals == nullptr) return GCG_OK;
  if (out_indptr == nullptr || indptr == nullptr ||
      (nnz > 0 && (indices == nullptr || vals == nullptr || out_indices == nullptr || out_vals == nullptr)))
    return fail(GCG_ERR_INVALID_ARG, "NULL buffer");
  if (workspace_bytes < need || (need > 0 && workspace == nullptr))
    return fail(GCG_ERR_WORKSPACE, "workspace %zu < %zu", workspace_bytes, need);
  hipStream_t st = static_cast<hipStream_t>(stream);
  char* w = static_cast<char*>(workspace);
  int32_t* keys_out = reinterpret_cast<int32_t*>(w);
  int32_t* iota = reinterpret_cast<int32_t*>(w + nb);
  int32_t* perm = reinterpret_cast<int32_t*>(w + 2 * nb);
  int32_t* row_of = reinterpret_cast<int32_t*>(w + 3 * nb);
  void* cub_tmp = w + 4 * nb;
  if (nnz > 0) {
    hipLaunchKernelGGL(iota_kernel, dim3(grid_for(nnz)), dim3(256), 0, st, iota, nnz);
    GCG_HIP_CHECK(hipGetLastError());
    GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(cub_tmp, temp, reinterpret_cast<const uint32_t*>(indices), reinterpret_cast<uint32_t*>(keys_out), iota, perm,
                                                     static_cast<int>(nnz), 0, end_bit, st));
    hipLaunchKernelGGL(expand_rows_kernel, dim3(grid_for(n_rows)), dim3(256), 0, st, n_rows, indptr, row_of);
    GCG_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(permute_transpose_kernel, dim3(grid_for(nnz)), dim3(256), 0, st, nnz, perm,
                       row_of, vals, out_indices, out_vals);
    GCG_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(lower_bound_kernel, dim3(grid_for(n_cols + 1)), dim3(256), 0, st, keys_out,
                     nnz, n_cols, out_indptr);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}


}  // extern "C"
