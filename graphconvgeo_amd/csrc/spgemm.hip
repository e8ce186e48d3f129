// spgemm.hip -- C = A . B for the host "input convolution" X_conv = H * X (main.py:530,
// tensormain.py:114), expand-sort-reduce with scipy csr_matmat's summation order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <vector>

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
                                            const int64_t* __restrict__ n_out, int64_t base,
                                            int32_t* __restrict__ indptr) {
  const int64_t m = *n_out;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r <= n_rows; r += stride) {
    const uint64_t target = static_cast<uint64_t>(r) * static_cast<uint64_t>(p);
    int64_t lo = 0, hi = m;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < target) lo = mid + 1; else hi = mid;
    }
    indptr[r] = static_cast<int32_t>(base + lo);
  }
}

// Rebased row pointers of rows [r0, r0 + n] (chunk-local nonzero offsets).
__global__ void rebase_ptr_kernel(int64_t n, const int32_t* __restrict__ a_ptr, int64_t r0,
                                  int32_t* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int32_t b = a_ptr[r0];
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i <= n; i += stride)
    out[i] = a_ptr[r0 + i] - b;
}

// Products before row i: off[a_ptr[i]] (off = exclusive scan of per-nonzero products).
__global__ void row_products_kernel(int64_t m, const int32_t* __restrict__ a_ptr,
                                    const int64_t* __restrict__ off, int64_t nnz_a, int64_t total,
                                    int64_t* __restrict__ row_off) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i <= m; i += stride) {
    const int64_t j = a_ptr[i];
    row_off[i] = j < nnz_a ? off[j] : total;
  }
}

struct DevBuf {
  void* p = nullptr;
  hipStream_t s = nullptr;
  ~DevBuf() { if (p) (void)hipFreeAsync(p, s); }
};

// Products per row chunk: the expand-sort-reduce temporaries are ~40 B per product, so a
// chunk of 2^29 products holds ~21 GB of HBM; row chunks also keep every hipcub item count
// and the int32 permutation within range. Twitter-World H.X (2.65e9 products) -> 5 chunks.
// GCG_SPGEMM_CHUNK (products, > 0) overrides it -- the tests use it to force many chunks.
int64_t chunk_products() {
  if (const char* v = std::getenv("GCG_SPGEMM_CHUNK")) {
    const long long c = std::atoll(v);
    if (c > 0) return c;
  }
  return int64_t{1} << 29;
}

template <typename TA, typename TACC>
gcg_status spgemm_impl(int64_t m, int64_t n, int64_t p, int64_t nnz_a, const int32_t* a_ptr,
                       const int32_t* a_idx, const TA* a_val, int64_t nnz_b, const int32_t* b_ptr,
                       const int32_t* b_idx, const float* b_val, int64_t n_products, int32_t* c_ptr,
                       int32_t* c_idx, float* c_val, int64_t* nnz_c_dev, hipStream_t st) {
  (void)n; (void)nnz_b;
  GCG_HIP_CHECK(hipMemsetAsync(nnz_c_dev, 0, sizeof(int64_t), st));
  if (n_products == 0 || nnz_a == 0) {
    GCG_HIP_CHECK(hipMemsetAsync(c_ptr, 0, (m + 1) * sizeof(int32_t), st));
    return GCG_OK;
  }
  if (nnz_a > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "nnz(A) exceeds int32");
  auto alloc = [&](DevBuf& b, size_t bytes) -> hipError_t {
    b.s = st;
    return hipMallocAsync(&b.p, std::max<size_t>(bytes, 16), st);
  };
  // ---- products per nonzero / per row, row chunks (host) ----
  DevBuf b_off, b_rowoff, b_tmp0;
  size_t t_scan = 0;
  {
    int64_t* o = nullptr;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, o, o, static_cast<int>(nnz_a)) != hipSuccess)
      return fail(GCG_ERR_HIP, "hipcub sizing failed");
  }
  hipError_t e = alloc(b_off, nnz_a * sizeof(int64_t));
  if (e == hipSuccess) e = alloc(b_rowoff, (m + 1) * sizeof(int64_t));
  if (e == hipSuccess) e = alloc(b_tmp0, t_scan);
  if (e != hipSuccess) return fail(GCG_ERR_ALLOC, "SpGEMM row offsets: %s", hipGetErrorString(e));
  auto* off = static_cast<int64_t*>(b_off.p);
  auto* rowoff_dev = static_cast<int64_t*>(b_rowoff.p);
  hipLaunchKernelGGL(spgemm_count_kernel, dim3(grid_for(nnz_a)), dim3(256), 0, st, nnz_a, a_idx, b_ptr, off);
  GCG_HIP_CHECK(hipGetLastError());
  size_t tb = t_scan;
  GCG_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(b_tmp0.p, tb, off, off, static_cast<int>(nnz_a), st));
  hipLaunchKernelGGL(row_products_kernel, dim3(grid_for(m + 1)), dim3(256), 0, st, m, a_ptr, off, nnz_a,
                     n_products, rowoff_dev);
  GCG_HIP_CHECK(hipGetLastError());
  std::vector<int64_t> rowoff(m + 1);
  std::vector<int32_t> aptr(m + 1);
  GCG_HIP_CHECK(hipMemcpyAsync(rowoff.data(), rowoff_dev, (m + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipMemcpyAsync(aptr.data(), a_ptr, (m + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  if (rowoff[m] != n_products)
    return fail(GCG_ERR_INVALID_ARG, "n_products %lld != %lld (from gcg_spgemm_products)",
                (long long)n_products, (long long)rowoff[m]);
  const int64_t kChunkProducts = chunk_products();
  std::vector<int64_t> cuts{0};  // greedy row chunks of <= kChunkProducts products (>= 1 row)
  while (cuts.back() < m) {
    const int64_t r0 = cuts.back();
    int64_t r1 = std::upper_bound(rowoff.begin() + r0 + 1, rowoff.end(), rowoff[r0] + kChunkProducts) -
                 rowoff.begin() - 1;
    if (r1 <= r0) r1 = r0 + 1;  // one row alone
    if (rowoff[r1] - rowoff[r0] > INT32_MAX)
      return fail(GCG_ERR_INVALID_ARG, "row %lld alone has %lld products (> int32)", (long long)r0,
                  (long long)(rowoff[r1] - rowoff[r0]));
    cuts.push_back(r1);
  }
  int64_t P_max = 0, m_max = 0, nnz_max = 0;
  for (size_t c = 0; c + 1 < cuts.size(); ++c) {
    P_max = std::max(P_max, rowoff[cuts[c + 1]] - rowoff[cuts[c]]);
    m_max = std::max(m_max, cuts[c + 1] - cuts[c]);
    nnz_max = std::max<int64_t>(nnz_max, aptr[cuts[c + 1]] - aptr[cuts[c]]);
  }
  P_max = std::max<int64_t>(P_max, 1);

  // ---- temporaries sized for the largest chunk, reused ----
  size_t t_sort = 0, t_sel = 0;
  {
    uint64_t* k = nullptr; int32_t* v = nullptr; int64_t* c = nullptr; int64_t* o = nullptr;
    TACC* f = nullptr;
    size_t t2 = 0, t3 = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, k, k, v, v, static_cast<int>(P_max), 0, 64) != hipSuccess ||
        hipcub::DeviceSelect::Flagged(nullptr, t_sel, k, v, k, c, static_cast<int>(P_max)) != hipSuccess ||
        hipcub::DeviceSelect::Flagged(nullptr, t2, f, v, f, c, static_cast<int>(P_max)) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, t3, o, o, static_cast<int>(std::max<int64_t>(nnz_max, 1))) != hipSuccess)
      return fail(GCG_ERR_HIP, "hipcub sizing failed");
    t_sel = std::max({t_sel, t2, t3});
  }
  const size_t tmp_bytes = std::max({t_sort, t_sel, t_scan});
  DevBuf b_cp, b_row, b_coff, b_keys, b_keys2, b_seq, b_seq2, b_prod, b_flags, b_starts, b_sums, b_tmp, b_cnt;
  e = alloc(b_cp, (m_max + 1) * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_row, nnz_max * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_coff, nnz_max * sizeof(int64_t));
  if (e == hipSuccess) e = alloc(b_keys, P_max * sizeof(uint64_t));
  if (e == hipSuccess) e = alloc(b_keys2, P_max * sizeof(uint64_t));
  if (e == hipSuccess) e = alloc(b_seq, P_max * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_seq2, P_max * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_prod, P_max * sizeof(TACC));
  if (e == hipSuccess) e = alloc(b_flags, P_max * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_starts, P_max * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_sums, P_max * sizeof(TACC));
  if (e == hipSuccess) e = alloc(b_tmp, tmp_bytes);
  if (e == hipSuccess) e = alloc(b_cnt, 2 * sizeof(int64_t));
  if (e != hipSuccess)
    return fail(GCG_ERR_ALLOC, "SpGEMM temporaries (%lld products per chunk): %s", (long long)P_max,
                hipGetErrorString(e));
  auto* cptr = static_cast<int32_t*>(b_cp.p);
  auto* row_of = static_cast<int32_t*>(b_row.p);
  auto* coff = static_cast<int64_t*>(b_coff.p);
  auto* keys = static_cast<uint64_t*>(b_keys.p);
  auto* keys2 = static_cast<uint64_t*>(b_keys2.p);
  auto* seq = static_cast<int32_t*>(b_seq.p);
  auto* seq2 = static_cast<int32_t*>(b_seq2.p);
  auto* prod = static_cast<TACC*>(b_prod.p);
  auto* flags = static_cast<int32_t*>(b_flags.p);
  auto* starts = static_cast<int32_t*>(b_starts.p);
  auto* sums = static_cast<TACC*>(b_sums.p);
  auto* cnts = static_cast<int64_t*>(b_cnt.p);

  int64_t nnz_done = 0;
  for (size_t c = 0; c + 1 < cuts.size(); ++c) {
    const int64_t r0 = cuts[c], mc = cuts[c + 1] - r0;
    const int64_t base = aptr[r0], nnz_c = aptr[r0 + mc] - base;
    const int64_t P = rowoff[r0 + mc] - rowoff[r0];
    if (P == 0 || nnz_c == 0) {  // every row of the chunk is empty in C
      std::vector<int32_t> z(mc + 1, static_cast<int32_t>(nnz_done));
      GCG_HIP_CHECK(hipMemcpyAsync(c_ptr + r0, z.data(), (mc + 1) * sizeof(int32_t), hipMemcpyHostToDevice, st));
      GCG_HIP_CHECK(hipStreamSynchronize(st));
      continue;
    }
    int end_bit = 1;
    while (end_bit < 64 && (uint64_t{1} << end_bit) <= static_cast<uint64_t>(mc) * static_cast<uint64_t>(p)) ++end_bit;
    hipLaunchKernelGGL(rebase_ptr_kernel, dim3(grid_for(mc + 1)), dim3(256), 0, st, mc, a_ptr, r0, cptr);
    hipLaunchKernelGGL(expand_rows_kernel, dim3(grid_for(mc)), dim3(256), 0, st, mc, cptr, row_of);
    hipLaunchKernelGGL(spgemm_count_kernel, dim3(grid_for(nnz_c)), dim3(256), 0, st, nnz_c, a_idx + base, b_ptr, coff);
    GCG_HIP_CHECK(hipGetLastError());
    tb = tmp_bytes;
    GCG_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(b_tmp.p, tb, coff, coff, static_cast<int>(nnz_c), st));
    hipLaunchKernelGGL((spgemm_expand_kernel<TA, TACC>), dim3(grid_for(nnz_c)), dim3(256), 0, st, nnz_c, p,
                       row_of, a_idx + base, a_val + base, b_ptr, b_idx, b_val, coff, keys, seq, prod);
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
    GCG_HIP_CHECK(hipcub::DeviceSelect::Flagged(b_tmp.p, tb, keys, flags, keys2, cnts, static_cast<int>(n_runs), st));
    tb = tmp_bytes;
    GCG_HIP_CHECK(hipcub::DeviceSelect::Flagged(b_tmp.p, tb, sums, flags, prod, cnts + 1, static_cast<int>(n_runs), st));
    hipLaunchKernelGGL((spgemm_emit_kernel<TACC>), dim3(grid_for(n_runs)), dim3(256), 0, st, p, keys2,
                       prod, cnts, c_idx + nnz_done, c_val + nnz_done);
    hipLaunchKernelGGL(row_ptr_from_rowkeys_kernel, dim3(grid_for(mc + 1)), dim3(256), 0, st, mc, p, keys2,
                       cnts, nnz_done, c_ptr + r0);
    GCG_HIP_CHECK(hipGetLastError());
    int64_t kept = 0;
    GCG_HIP_CHECK(hipMemcpyAsync(&kept, cnts, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    GCG_HIP_CHECK(hipStreamSynchronize(st));
    nnz_done += kept;
    if (nnz_done > INT32_MAX)
      return fail(GCG_ERR_INVALID_ARG, "nnz(C) exceeds int32 CSR (%lld after row %lld)", (long long)nnz_done,
                  (long long)(r0 + mc));
  }
  GCG_HIP_CHECK(hipMemcpyAsync(nnz_c_dev, &nnz_done, sizeof(int64_t), hipMemcpyHostToDevice, st));
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
