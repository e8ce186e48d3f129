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




// Rectify backward + bias gradient in one pass (Theano's grad of
// rectify(S.dot(H, Z) + b), mlpconv.py:75-77): g = gY where Y > 0 else 0, written to g_out
// (may alias gY), and per-block column partial sums of g. Block = 4 waves; wave w takes rows
// r0 + w, r0 + w + 4, ...; lanes span the columns in dwordx4 (or dword) pieces. MASK = false:
// column sums of gY only (Y and g_out unused) -- the bias gradient of a dense projection.
constexpr int kReluMinRows = 512;   // rows per block at least ...
constexpr int kReluMaxBlocks = 1024;  // ... and at most this many blocks (partial rows)
constexpr int kReluMaxK4 = 4;       // dwordx4 column pieces per lane (K <= 1024 on the vector path)

int64_t relu_rows_per_block(int64_t M) {
  const int64_t r = (M + kReluMaxBlocks - 1) / kReluMaxBlocks;
  return std::max<int64_t>(kReluMinRows, (r + 3) / 4 * 4);
}

// GATE: the mask comes from the gate bytes of the SpMM epilogue (2 / 1 / 0 -> g, g/2, 0:
// Theano's 0.5*(1 + sgn(x)) rectify gradient) instead of Y > 0.
__device__ __forceinline__ float gate_apply(float g, uint32_t code) {
  return code == 2u ? g : (code == 1u ? 0.5f * g : 0.0f);
}

template <int VEC, bool MASK, bool GATE = false>
__global__ __launch_bounds__(256) void relu_backward_kernel(
    int64_t M, int K, int64_t rows_per_block, const float* gY, int64_t ldg,
    const float* __restrict__ Y, int64_t ldy, float* g_out, int64_t ldo,
    float* __restrict__ partial, const uint8_t* __restrict__ gate = nullptr,
    int64_t ldgate = 0) {
  __shared__ float red[4][kReluMaxK4 * 64 * 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  const int pieces = (K + 64 * VEC - 1) / (64 * VEC);
  float acc[kReluMaxK4][VEC];
#pragma unroll
  for (int p = 0; p < kReluMaxK4; ++p)
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[p][e] = 0.f;
#pragma unroll 2
  for (int64_t r = r0 + w; r < r1; r += 4) {
    const float* gr = gY + r * ldg;
    const float* yr = (MASK && !GATE) ? Y + r * ldy : nullptr;
    const uint8_t* gt = GATE ? gate + r * ldgate : nullptr;
    float* orow = MASK ? g_out + r * ldo : nullptr;
#pragma unroll
    for (int p = 0; p < kReluMaxK4; ++p) {
      if (p >= pieces) break;
      const int c = (p * 64 + lane) * VEC;
      if (c >= K) continue;
      if constexpr (VEC == 4) {
        if (c + 4 > K) {  // ragged tail: element-wise, never touches columns >= K
          for (int e = 0; e < 4; ++e)
            if (c + e < K) {
              float o = gr[c + e];
              if constexpr (GATE) {
                o = gate_apply(o, gt[c + e]);
                orow[c + e] = o;
              } else if constexpr (MASK) {
                o = yr[c + e] > 0.f ? o : 0.f;
                orow[c + e] = o;
              }
              acc[p][e] += o;
            }
          continue;
        }
        float4 o = *reinterpret_cast<const float4*>(gr + c);
        if constexpr (GATE) {
          const uint32_t gv = *reinterpret_cast<const uint32_t*>(gt + c);
          o = make_float4(gate_apply(o.x, gv & 0xffu), gate_apply(o.y, (gv >> 8) & 0xffu),
                          gate_apply(o.z, (gv >> 16) & 0xffu), gate_apply(o.w, gv >> 24));
          *reinterpret_cast<float4*>(orow + c) = o;
        } else if constexpr (MASK) {
          const float4 yv = *reinterpret_cast<const float4*>(yr + c);
          o = make_float4(yv.x > 0.f ? o.x : 0.f, yv.y > 0.f ? o.y : 0.f,
                          yv.z > 0.f ? o.z : 0.f, yv.w > 0.f ? o.w : 0.f);
          *reinterpret_cast<float4*>(orow + c) = o;
        }
        acc[p][0] += o.x; acc[p][1] += o.y; acc[p][2] += o.z; acc[p][3] += o.w;
      } else {
        float o = gr[c];
        if constexpr (GATE) {
          o = gate_apply(o, gt[c]);
          orow[c] = o;
        } else if constexpr (MASK) {
          o = yr[c] > 0.f ? o : 0.f;
          orow[c] = o;
        }
        acc[p][0] += o;
      }
    }
  }
  // combine the 4 waves (fixed order), one partial row per block
#pragma unroll
  for (int p = 0; p < kReluMaxK4; ++p)
#pragma unroll
    for (int e = 0; e < VEC; ++e) red[w][(p * 64 + lane) * VEC + e] = acc[p][e];
  __syncthreads();
  for (int c = threadIdx.x; c < K; c += 256) {
    const float v = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
    partial[static_cast<int64_t>(blockIdx.x) * K + c] = v;
  }
}

// out[c] = sum over the partial rows of partial[b][c], in a fixed order: workgroup = 16 waves
// over 64 columns; wave w sums rows w, w + 16, ... in order, then wave 0 adds the 16 in order.
__global__ __launch_bounds__(1024) void column_sum_kernel(int64_t n_blocks, int K,
                                                         const float* __restrict__ partial,
                                                         float* __restrict__ out) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int cc = c < K ? c : K - 1;
  float s = 0.f;
#pragma unroll 4
  for (int64_t b = w; b < n_blocks; b += 16) s += partial[b * K + cc];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < K) {
    float t = red[0][lane];
#pragma unroll
    for (int i = 1; i < 16; ++i) t += red[i][lane];
    out[c] = t;
  }
}

// lasagne.updates.adam (mlpconv.py:263) for one parameter, every elementwise op of the step in
// one pass (the trainer's update otherwise runs ~8 torch kernels per parameter):
//   m = b1*m + (1-b1)*g;  v = b2*v + (1-b2)*g*g;  p -= a_t*m / (sqrt(v) + eps)
// a_t = lr*sqrt(1-b2^t)/(1-b1^t) is read on the device (a captured HIP graph replays it).
__global__ __launch_bounds__(256) void adam_kernel(int64_t n, float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   const float* __restrict__ step_dev, float b1,
                                                   float b2, float eps) {
  const float a_t = *step_dev;
  const float c1 = 1.0f - b1, c2 = 1.0f - b2;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gi = g[i];
    const float mi = b1 * m[i] + c1 * gi;
    const float vi = b2 * v[i] + c2 * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = p[i] - (a_t * mi) / (sqrtf(vi) + eps);
  }
}

// lasagne.regularization l1 / l2 of one weight (mlpconv.py:235-243): partial sums of |w| and
// w*w over a fixed grid (kPenBlocks blocks, grid-stride order fixed by the grid), one pair per
// block; then ONE thread adds the pairs in block order -- deterministic, graph-capturable.
constexpr int kPenBlocks = 256;

__global__ __launch_bounds__(256) void l1l2_partial_kernel(int64_t n, const float* __restrict__ w,
                                                           float* __restrict__ part) {
  __shared__ float s1[256], s2[256];
  float a = 0.f, q = 0.f;
  const int64_t stride = static_cast<int64_t>(kPenBlocks) * 256;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) {
    const float x = w[i];
    a += fabsf(x);
    q += x * x;
  }
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = q;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (static_cast<int>(threadIdx.x) < h) {
      s1[threadIdx.x] += s1[threadIdx.x + h];
      s2[threadIdx.x] += s2[threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s1[0];
    part[2 * blockIdx.x + 1] = s2[0];
  }
}

// out = ((acc_in ? *acc_in : 0) + l1 * sum|w|) + l2 * sum w^2 (acc_in may alias out).
__global__ __launch_bounds__(64) void l1l2_finish_kernel(const float* __restrict__ part, float l1,
                                                         float l2, const float* acc_in,
                                                         float* out) {
  if (threadIdx.x != 0) return;
  float a = 0.f, q = 0.f;
  for (int b = 0; b < kPenBlocks; ++b) {
    a += part[2 * b];
    q += part[2 * b + 1];
  }
  const float base = acc_in != nullptr ? *acc_in : 0.f;
  out[0] = (base + a * l1) + q * l2;
}

// d/dw of l1 * sum|w| + l2 * sum w^2, times the upstream gradient: s * (l1 sgn(w) + 2 l2 w)
// (Theano's grad of abs is sgn, 0 at 0).
__global__ __launch_bounds__(256) void l1l2_grad_kernel(int64_t n, const float* __restrict__ w,
                                                        float l1, float l2,
                                                        const float* __restrict__ scale_dev,
                                                        float* __restrict__ dw) {
  const float s = scale_dev != nullptr ? *scale_dev : 1.0f;
  const float c1 = s * l1, c2 = s * (2.0f * l2);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float x = w[i];
    const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
    dw[i] = c1 * sg + c2 * x;
  }
}

}  // namespace

extern "C" {

gcg_status gcg_adam_step_f32(int64_t n, float* p, const float* g, float* m, float* v,
                             const float* step_dev, float beta1, float beta2, float eps,
                             gcg_stream_t stream) {
  if (n < 0 || (n > 0 && (p == nullptr || g == nullptr || m == nullptr || v == nullptr ||
                          step_dev == nullptr)))
    return fail(GCG_ERR_INVALID_ARG, "gcg_adam_step_f32: bad arguments");
  if (n == 0) return GCG_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     n, p, g, m, v, step_dev, beta1, beta2, eps);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

gcg_status gcg_l1l2_penalty_f32(int64_t n, const float* W, float l1, float l2,
                                const float* acc_in, float* out, void* workspace,
                                size_t workspace_bytes, gcg_stream_t stream) {
  if (n < 0 || (n > 0 && W == nullptr) || out == nullptr || workspace == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "gcg_l1l2_penalty_f32: bad arguments");
  if (workspace_bytes < GCG_L1L2_WORKSPACE_BYTES || !aligned(workspace, 4))
    return fail(GCG_ERR_INVALID_ARG, "gcg_l1l2_penalty_f32: workspace needs %d aligned bytes",
                GCG_L1L2_WORKSPACE_BYTES);
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(l1l2_partial_kernel, dim3(kPenBlocks), dim3(256), 0, st, n, W, part);
  hipLaunchKernelGGL(l1l2_finish_kernel, dim3(1), dim3(64), 0, st, part, l1, l2, acc_in, out);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

gcg_status gcg_l1l2_grad_f32(int64_t n, const float* W, float l1, float l2,
                             const float* scale_dev, float* dW, gcg_stream_t stream) {
  if (n < 0 || (n > 0 && (W == nullptr || dW == nullptr)))
    return fail(GCG_ERR_INVALID_ARG, "gcg_l1l2_grad_f32: bad arguments");
  if (n == 0) return GCG_OK;
  hipLaunchKernelGGL(l1l2_grad_kernel, dim3(grid_for(n)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), n, W, l1, l2, scale_dev, dW);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

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


gcg_status gcg_relu_backward_f32_workspace_bytes(int64_t M, int64_t K, size_t* bytes) {
  if (M < 0 || K < 0 || bytes == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "gcg_relu_backward_f32_workspace_bytes: bad args");
  const int64_t rpb = relu_rows_per_block(M);
  *bytes = sizeof(float) * static_cast<size_t>((M + rpb - 1) / rpb) * K;
  return GCG_OK;
}

namespace {

// shared by gcg_relu_backward_f32 (MASK: Y), gcg_relu_backward_gate_f32 (MASK: gate bytes)
// and gcg_column_sum_f32 (no mask)
gcg_status relu_colsum(const char* fn, bool mask, int64_t M, int64_t K, const float* gY,
                       int64_t ldg, const float* Y, int64_t ldy, float* g_out, int64_t ldo,
                       float* bias_grad, void* workspace, size_t workspace_bytes,
                       gcg_stream_t stream, const uint8_t* gate = nullptr, int64_t ldgate = 0) {
  if (M < 0 || K < 0 || K > 64 * 4 * kReluMaxK4)
    return fail(GCG_ERR_INVALID_ARG, "%s: bad sizes M=%lld K=%lld (K <= %d)", fn,
                static_cast<long long>(M), static_cast<long long>(K), 64 * 4 * kReluMaxK4);
  auto st = static_cast<hipStream_t>(stream);
  if (M == 0 || K == 0) {
    if (bias_grad != nullptr && K > 0)
      GCG_HIP_CHECK(hipMemsetAsync(bias_grad, 0, sizeof(float) * K, st));
    return GCG_OK;
  }
  const bool use_gate = mask && gate != nullptr;
  if (use_gate) {  // the gate stands in for Y
    if (ldgate < K || ldgate % 4 != 0 || !aligned(gate, 4))
      return fail(GCG_ERR_MISALIGNED, "%s: gate needs ldgate >= K, ldgate %% 4 == 0, 4-B base", fn);
    Y = gY;
    ldy = ldg;
  }
  if (gY == nullptr || (mask && (Y == nullptr || g_out == nullptr)) ||
      (!mask && bias_grad == nullptr))
    return fail(GCG_ERR_INVALID_ARG, "%s: null operand", fn);
  if (ldg < K || (mask && (ldy < K || ldo < K)))
    return fail(GCG_ERR_INVALID_ARG, "%s: ld < K", fn);
  if (!aligned(gY, 4) || (mask && (!aligned(Y, 4) || !aligned(g_out, 4))))
    return fail(GCG_ERR_MISALIGNED, "%s: operand not 4-B aligned", fn);
  const int64_t rpb = relu_rows_per_block(M);
  const int64_t n_blocks = (M + rpb - 1) / rpb;
  const size_t need = sizeof(float) * static_cast<size_t>(n_blocks) * K;
  if (workspace == nullptr || workspace_bytes < need)  // the kernel always writes partials
    return fail(GCG_ERR_WORKSPACE, "%s: workspace %zu < %zu bytes", fn, workspace_bytes, need);
  if (!aligned(workspace, 4)) return fail(GCG_ERR_MISALIGNED, "%s: workspace alignment", fn);
  float* part = static_cast<float*>(workspace);
  const bool vec = ldg % 4 == 0 && aligned(gY, 16) &&
                   (!mask || (ldy % 4 == 0 && ldo % 4 == 0 && aligned(Y, 16) && aligned(g_out, 16)));
  if (!vec && K > 64 * kReluMaxK4)
    return fail(GCG_ERR_MISALIGNED, "%s: K > %d needs 16-B rows (ld %% 4 == 0)", fn,
                64 * kReluMaxK4);
  const dim3 grid(static_cast<unsigned>(n_blocks));
#define GCG_RELU_LAUNCH(V, MK, GT)                                                              \
  hipLaunchKernelGGL((relu_backward_kernel<V, MK, GT>), grid, dim3(256), 0, st, M, int(K), rpb,  \
                     gY, ldg, Y, ldy, g_out, ldo, part, gate, ldgate)
  if (vec) {
    if (use_gate) GCG_RELU_LAUNCH(4, true, true);
    else if (mask) GCG_RELU_LAUNCH(4, true, false);
    else GCG_RELU_LAUNCH(4, false, false);
  } else {
    if (use_gate) GCG_RELU_LAUNCH(1, true, true);
    else if (mask) GCG_RELU_LAUNCH(1, true, false);
    else GCG_RELU_LAUNCH(1, false, false);
  }
#undef GCG_RELU_LAUNCH
  GCG_HIP_CHECK(hipGetLastError());
  if (bias_grad != nullptr) {
    hipLaunchKernelGGL(column_sum_kernel, dim3(static_cast<unsigned>((K + 63) / 64)), dim3(1024),
                       0, st, n_blocks, int(K), part, bias_grad);
    GCG_HIP_CHECK(hipGetLastError());
  }
  return GCG_OK;
}

}  // namespace

gcg_status gcg_relu_backward_f32(int64_t M, int64_t K, const float* gY, int64_t ldg,
                                 const float* Y, int64_t ldy, float* g_out, int64_t ldo,
                                 float* bias_grad, void* workspace, size_t workspace_bytes,
                                 gcg_stream_t stream) {
  return relu_colsum("gcg_relu_backward_f32", true, M, K, gY, ldg, Y, ldy, g_out, ldo, bias_grad,
                     workspace, workspace_bytes, stream);
}

gcg_status gcg_relu_backward_gate_f32(int64_t M, int64_t K, const float* gY, int64_t ldg,
                                      const uint8_t* gate, int64_t ldgate, float* g_out,
                                      int64_t ldo, float* bias_grad, void* workspace,
                                      size_t workspace_bytes, gcg_stream_t stream) {
  if (M > 0 && K > 0 && gate == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "gcg_relu_backward_gate_f32: gate is NULL");
  return relu_colsum("gcg_relu_backward_gate_f32", true, M, K, gY, ldg, nullptr, 0, g_out, ldo,
                     bias_grad, workspace, workspace_bytes, stream, gate, ldgate);
}

gcg_status gcg_column_sum_f32(int64_t M, int64_t K, const float* X, int64_t ldx, float* out,
                              void* workspace, size_t workspace_bytes, gcg_stream_t stream) {
  return relu_colsum("gcg_column_sum_f32", false, M, K, X, ldx, nullptr, 0, nullptr, 0, out,
                     workspace, workspace_bytes, stream);
}

}  // extern "C"
