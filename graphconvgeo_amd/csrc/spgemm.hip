// spgemm.hip -- C = A . B for the host "input convolution" X_conv = H * X (main.py:530,
// tensormain.py:114), expand-sort-reduce with scipy csr_matmat's summation order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "common.h"
#include "index_kernels.h"

using namespace gcg;

namespace {

// ---- SpGEMM C = A . B (main.py:530 / tensormain.py:114 "input convolution") -----------
// Expand-sort-reduce: every product a_ij * b_jk becomes (key = i*p + k, seq); a stable
// radix sort by key keeps equal keys in traversal order (A row order, then B row order),
// so each C entry is summed exactly in scipy csr_matmat's order: sums[k] += v * Bx[kk].
__global__ void spgemm_count_kernel(int64_t nnz_a, const int32_t* __restrict__ a_idx,
                                    const int32_t* __restrict__ b_ptr, int64_t* __restrict__ cnt) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < nnz_a; j += stride) {
    const int32_t r = a_idx[j];
    cnt[j] = b_ptr[r + 1] - b_ptr[r];
  }
}

template <typename TA, typename TACC>
__global__ void spgemm_expand_kernel(int64_t nnz_a, int64_t p, const int32_t* __restrict__ row_of,
                                     const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val,
                                     const int32_t* __restrict__ b_ptr, const int32_t* __restrict__ b_idx,
                                     const float* __restrict__ b_val, const int64_t* __restrict__ off,
                                     uint64_t* __restrict__ keys, int32_t* __restrict__ seq,
                                     TACC* __restrict__ prod) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < nnz_a; j += stride) {
    const uint64_t base_key = static_cast<uint64_t>(row_of[j]) * static_cast<uint64_t>(p);
    const TACC a = static_cast<TACC>(a_val[j]);
    const int32_t r = a_idx[j];
    int64_t o = off[j];
    for (int32_t kk = b_ptr[r]; kk < b_ptr[r + 1]; ++kk, ++o) {
      keys[o] = base_key + static_cast<uint64_t>(b_idx[kk]);
      seq[o] = static_cast<int32_t>(o);
      prod[o] = a * static_cast<TACC>(b_val[kk]);
    }
  }
}

__global__ void run_flags_kernel(int64_t n, const uint64_t* __restrict__ keys, int32_t* __restrict__ flags) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t s = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; s < n; s += stride)
    flags[s] = (s == 0 || keys[s] != keys[s - 1]) ? 1 : 0;
}

// One thread per run: sequential sum in traversal order; zero sums are dropped (scipy
// `if (sums[head] != 0)`), surviving runs get keep = 1.
template <typename TACC>
__global__ void run_sum_kernel(int64_t n_runs, int64_t n, const int32_t* __restrict__ run_start,
                               const int32_t* __restrict__ seq, const TACC* __restrict__ prod,
                               TACC* __restrict__ sums, int32_t* __restrict__ keep) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < n_runs; r += stride) {
    const int64_t s0 = run_start[r], s1 = (r + 1 < n_runs) ? run_start[r + 1] : n;
    TACC acc = 0;
    for (int64_t s = s0; s < s1; ++s) acc = acc + prod[seq[s]];
    sums[r] = acc;
    keep[r] = acc != TACC(0) ? 1 : 0;
  }
}

template <typename TACC>
__global__ void spgemm_emit_kernel(int64_t p, const uint64_t* __restrict__ keys,
                                   const TACC* __restrict__ sums, const int64_t* __restrict__ n_out,
                                   int32_t* __restrict__ out_idx, float* __restrict__ out_val) {
  const int64_t m = *n_out;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < m; k += stride) {
    out_idx[k] = static_cast<int32_t>(keys[k] % static_cast<uint64_t>(p));
    out_val[k] = static_cast<float>(sums[k]);
  }
}

__global__ void row_ptr_from_rowkeys_kernel(int64_t n_rows, int64_t p, const uint64_t* __restrict__ keys,
                                            const int64_t* __restrict__ n_out, int32_t* __restrict__ indptr) {
  const int64_t m = *n_out;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r <= n_rows; r += stride) {
    const uint64_t target = static_cast<uint64_t>(r) * static_cast<uint64_t>(p);
    int64_t lo = 0, hi = m;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < target) lo = mid + 1; else hi = mid;
    }
    indptr[r] = static_cast<int32_t>(lo);
  }
}

struct DevBuf {
  void* p = nullptr;
  hipStream_t s = nullptr;
  ~DevBuf() { if (p) (void)hipFreeAsync(p, s); }
};

template <typename TA, typename TACC>
gcg_status spgemm_impl(int64_t m, int64_t n, int64_t p, int64_t nnz_a, const int32_t* a_ptr,
                       const int32_t* a_idx, const TA* a_val, int64_t nnz_b, const int32_t* b_ptr,
                       const int32_t* b_idx, const float* b_val, int64_t n_products, int32_t* c_ptr,
                       int32_t* c_idx, float* c_val, int64_t* nnz_c_dev, hipStream_t st) {
  (void)n; (void)nnz_b;
  const int64_t P = n_products;
  GCG_HIP_CHECK(hipMemsetAsync(nnz_c_dev, 0, sizeof(int64_t), st));
  if (P == 0 || nnz_a == 0) {
    GCG_HIP_CHECK(hipMemsetAsync(c_ptr, 0, (m + 1) * sizeof(int32_t), st));
    return GCG_OK;
  }
  int end_bit = 1;
  while (end_bit < 64 && (uint64_t{1} << end_bit) <= static_cast<uint64_t>(m) * static_cast<uint64_t>(p)) ++end_bit;
  size_t t_sort = 0, t_sel = 0, t_scan = 0;
  {
    uint64_t* k = nullptr; int32_t* v = nullptr; int64_t* c = nullptr; int64_t* o = nullptr;
    TACC* f = nullptr;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, k, k, v, v, static_cast<int>(P), 0, end_bit) != hipSuccess ||
        hipcub::DeviceSelect::Flagged(nullptr, t_sel, k, v, k, c, static_cast<int>(P)) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, o, o, static_cast<int>(nnz_a)) != hipSuccess)
      return fail(GCG_ERR_HIP, "hipcub sizing failed");
    size_t t2 = 0;
    if (hipcub::DeviceSelect::Flagged(nullptr, t2, f, v, f, c, static_cast<int>(P)) != hipSuccess)
      return fail(GCG_ERR_HIP, "hipcub sizing failed");
    t_sel = std::max(t_sel, t2);
  }
  const size_t tmp_bytes = std::max({t_sort, t_sel, t_scan});
  DevBuf b_row, b_off, b_keys, b_keys2, b_seq, b_seq2, b_prod, b_flags, b_starts, b_sums, b_tmp, b_cnt;
  auto alloc = [&](DevBuf& b, size_t bytes) -> hipError_t {
    b.s = st;
    return hipMallocAsync(&b.p, std::max<size_t>(bytes, 16), st);
  };
  hipError_t e = hipSuccess;
  if (e == hipSuccess) e = alloc(b_row, nnz_a * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_off, nnz_a * sizeof(int64_t));
  if (e == hipSuccess) e = alloc(b_keys, P * sizeof(uint64_t));
  if (e == hipSuccess) e = alloc(b_keys2, P * sizeof(uint64_t));
  if (e == hipSuccess) e = alloc(b_seq, P * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_seq2, P * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_prod, P * sizeof(TACC));
  if (e == hipSuccess) e = alloc(b_flags, P * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_starts, P * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_sums, P * sizeof(TACC));
  if (e == hipSuccess) e = alloc(b_tmp, tmp_bytes);
  if (e == hipSuccess) e = alloc(b_cnt, 2 * sizeof(int64_t));
  if (e != hipSuccess) return fail(GCG_ERR_ALLOC, "SpGEMM temporaries (%lld products): %s", (long long)P, hipGetErrorString(e));
  auto* row_of = static_cast<int32_t*>(b_row.p);
  auto* off = static_cast<int64_t*>(b_off.p);
  auto* keys = static_cast<uint64_t*>(b_keys.p);
  auto* keys2 = static_cast<uint64_t*>(b_keys2.p);
  auto* seq = static_cast<int32_t*>(b_seq.p);
  auto* seq2 = static_cast<int32_t*>(b_seq2.p);
  auto* prod = static_cast<TACC*>(b_prod.p);
  auto* flags = static_cast<int32_t*>(b_flags.p);
  auto* starts = static_cast<int32_t*>(b_starts.p);
  auto* sums = static_cast<TACC*>(b_sums.p);
  auto* cnts = static_cast<int64_t*>(b_cnt.p);
  size_t tb = tmp_bytes;
  hipLaunchKernelGGL(expand_rows_kernel, dim3(grid_for(m)), dim3(256), 0, st, m, a_ptr, row_of);
  hipLaunchKernelGGL(spgemm_count_kernel, dim3(grid_for(nnz_a)), dim3(256), 0, st, nnz_a, a_idx, b_ptr, off);
  GCG_HIP_CHECK(hipGetLastError());
  GCG_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(b_tmp.p, tb, off, off, static_cast<int>(nnz_a), st));
  hipLaunchKernelGGL((spgemm_expand_kernel<TA, TACC>), dim3(grid_for(nnz_a)), dim3(256), 0, st, nnz_a, p,
                     row_of, a_idx, a_val, b_ptr, b_idx, b_val, off, keys, seq, prod);
  GCG_HIP_CHECK(hipGetLastError());
  tb = tmp_bytes;
  GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(b_tmp.p, tb, keys, keys2, seq, seq2, static_cast<int>(P), 0, end_bit, st));
  hipLaunchKernelGGL(run_flags_kernel, dim3(grid_for(P)), dim3(256), 0, st, P, keys2, flags);
  GCG_HIP_CHECK(hipGetLastError());
  // run starts (positions) and run keys
  hipLaunchKernelGGL(iota_kernel, dim3(grid_for(P)), dim3(256), 0, st, seq, P);  // reuse seq as positions
  tb = tmp_bytes;
  GCG_HIP_CHECK(hipcub::DeviceSelect::Flagged(b_tmp.p, tb, seq, flags, starts, cnts, static_cast<int>(P), st));
  tb = tmp_bytes;
  GCG_HIP_CHECK(hipcub::DeviceSelect::Flagged(b_tmp.p, tb, keys2, flags, keys, cnts, static_cast<int>(P), st));
  int64_t n_runs = 0;
  GCG_HIP_CHECK(hipMemcpyAsync(&n_runs, cnts, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  hipLaunchKernelGGL((run_sum_kernel<TACC>), dim3(grid_for(n_runs)), dim3(256), 0, st, n_runs, P, starts,
                     seq2, prod, sums, flags);
  GCG_HIP_CHECK(hipGetLastError());
  // drop exact zeros: compact keys and sums by keep flags
  tb = tmp_bytes;
  GCG_HIP_CHECK(hipcub::DeviceSelect::Flagged(b_tmp.p, tb, keys, flags, keys2, nnz_c_dev, static_cast<int>(n_runs), st));
  tb = tmp_bytes;
  GCG_HIP_CHECK(hipcub::DeviceSelect::Flagged(b_tmp.p, tb, sums, flags, prod, cnts + 1, static_cast<int>(n_runs), st));
  hipLaunchKernelGGL((spgemm_emit_kernel<TACC>), dim3(grid_for(n_runs)), dim3(256), 0, st, p, keys2,
                     prod, nnz_c_dev, c_idx, c_val);
  hipLaunchKernelGGL(row_ptr_from_rowkeys_kernel, dim3(grid_for(m + 1)), dim3(256), 0, st, m, p, keys2,
                     nnz_c_dev, c_ptr);
  GCG_HIP_CHECK(hipGetLastError());
  GCG_HIP_CHECK(hipStreamSynchronize(st));  // temporaries are freed stream-ordered on return
  return GCG_OK;
}
}  // namespace

extern "C" {

gcg_status gcg_spgemm_products(int64_t m, int64_t nnz_a, const int32_t* a_ptr, const int32_t* a_idx,
                               int64_t n, const int32_t* b_ptr, int64_t* n_products,
                               gcg_stream_t stream) {
  if (m < 0 || nnz_a < 0 || n < 0 || n_products == nullptr || a_ptr == nullptr || b_ptr == nullptr ||
      (nnz_a > 0 && a_idx == nullptr))
    return fail(GCG_ERR_INVALID_ARG, "bad args to gcg_spgemm_products");
  *n_products = 0;
  if (nnz_a == 0) return GCG_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  DevBuf cnt, tot, tmp;
  cnt.s = tot.s = tmp.s = st;
  size_t tb = 0;
  int64_t* dummy = nullptr;
  GCG_HIP_CHECK(hipcub::DeviceReduce::Sum(nullptr, tb, dummy, dummy, static_cast<int>(nnz_a)));
  GCG_HIP_CHECK(hipMallocAsync(&cnt.p, nnz_a * sizeof(int64_t), st));
  GCG_HIP_CHECK(hipMallocAsync(&tot.p, sizeof(int64_t), st));
  GCG_HIP_CHECK(hipMallocAsync(&tmp.p, std::max<size_t>(tb, 16), st));
  hipLaunchKernelGGL(spgemm_count_kernel, dim3(grid_for(nnz_a)), dim3(256), 0, st, nnz_a, a_idx, b_ptr,
                     static_cast<int64_t*>(cnt.p));
  GCG_HIP_CHECK(hipGetLastError());
  GCG_HIP_CHECK(hipcub::DeviceReduce::Sum(tmp.p, tb, static_cast<int64_t*>(cnt.p), static_cast<int64_t*>(tot.p),
                                          static_cast<int>(nnz_a), st));
  GCG_HIP_CHECK(hipMemcpyAsync(n_products, tot.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  return GCG_OK;
}

gcg_status gcg_spgemm(int64_t m, int64_t n, int64_t p, int64_t nnz_a, const int32_t* a_ptr,
                      const int32_t* a_idx, const void* a_val, int a_is_f64, int64_t nnz_b,
                      const int32_t* b_ptr, const int32_t* b_idx, const float* b_val,
                      int accumulate_f64, int64_t n_products, int32_t* c_ptr, int32_t* c_idx,
                      float* c_val, int64_t* nnz_c_dev, gcg_stream_t stream) {
  if (m < 0 || n < 0 || p < 0 || nnz_a < 0 || nnz_b < 0 || n_products < 0 || c_ptr == nullptr ||
      nnz_c_dev == nullptr || a_ptr == nullptr || b_ptr == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "bad args to gcg_spgemm");
  if (n_products > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "%lld products exceed int32 CSR", (long long)n_products);
  if (n_products > 0 && (c_idx == nullptr || c_val == nullptr || a_idx == nullptr || a_val == nullptr ||
                         b_idx == nullptr || b_val == nullptr))
    return fail(GCG_ERR_INVALID_ARG, "NULL buffer");
  if (a_is_f64 && !accumulate_f64) return fail(GCG_ERR_INVALID_ARG, "float64 A needs accumulate_f64");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (a_is_f64)
    return spgemm_impl<double, double>(m, n, p, nnz_a, a_ptr, a_idx, static_cast<const double*>(a_val), nnz_b,
                                       b_ptr, b_idx, b_val, n_products, c_ptr, c_idx, c_val, nnz_c_dev, st);
  if (accumulate_f64)
    return spgemm_impl<float, double>(m, n, p, nnz_a, a_ptr, a_idx, static_cast<const float*>(a_val), nnz_b,
                                      b_ptr, b_idx, b_val, n_products, c_ptr, c_idx, c_val, nnz_c_dev, st);
  return spgemm_impl<float, float>(m, n, p, nnz_a, a_ptr, a_idx, static_cast<const float*>(a_val), nnz_b,
                                   b_ptr, b_idx, b_val, n_products, c_ptr, c_idx, c_val, nnz_c_dev, st);
}

}  // extern "C"
