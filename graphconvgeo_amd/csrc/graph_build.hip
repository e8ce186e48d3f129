// graph_build.hip -- graph construction on the device: the mention-graph projection
// (data.py:226-250, gcg_project_mention_graph) and the normalized operator
// H = D^-1/2 (A+I) D^-1/2 from an undirected edge list (tensormain.py:170-181,
// gcg_normalize_adjacency_f32).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

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


// ---- mention-graph projection (data.py:226-250 after the celebrity filter, data.py:364-370)
// g: undirected graph over n_nodes ids; ids < n_targets are users (each with a self loop, as
// get_graph adds), ids >= n_targets are mention-only nodes. Projection: for every surviving
// node m, connect every pair of its user neighbours (m itself included when m is a user,
// through its self loop). Edges are unweighted and deduplicated.

// Incidence (a, b) -> both directed keys a*M+b, b*M+a; self pairs and bad ids -> sentinel.
__global__ void incidence_keys_kernel(int64_t n_nodes, int64_t n_inc, const int32_t* __restrict__ a,
                                      const int32_t* __restrict__ b, uint64_t* __restrict__ keys,
                                      int32_t* __restrict__ status) {
  const uint64_t M = static_cast<uint64_t>(n_nodes), sentinel = M * M;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < n_inc; e += stride) {
    const int64_t x = a[e], y = b[e];
    if (x < 0 || y < 0 || x >= n_nodes || y >= n_nodes) {
      atomicMax(status, int32_t(GCG_ERR_BAD_CSR));
      keys[2 * e] = keys[2 * e + 1] = sentinel;
    } else if (x == y) {
      keys[2 * e] = keys[2 * e + 1] = sentinel;  // self loops are implicit for users
    } else {
      keys[2 * e] = static_cast<uint64_t>(x) * M + y;
      keys[2 * e + 1] = static_cast<uint64_t>(y) * M + x;
    }
  }
}

// CSR (over all M nodes) of the deduplicated keys; sentinel keys sort last and are excluded.
__global__ void adj_ptr_kernel(int64_t n_nodes, const uint64_t* __restrict__ keys,
                               const int64_t* __restrict__ n_unique, int64_t* __restrict__ ptr) {
  const uint64_t M = static_cast<uint64_t>(n_nodes);
  const int64_t m = *n_unique;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r <= n_nodes; r += stride) {
    const uint64_t target = static_cast<uint64_t>(r) * M;
    int64_t lo = 0, hi = m;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < target) lo = mid + 1; else hi = mid;
    }
    ptr[r] = lo;
  }
}

// Per node m: alive? (users always; mention nodes iff 1 < degree <= threshold, data.py:364-369)
// and t(m) = number of user neighbours that survive, + 1 for m itself when m is a user.
__global__ void target_count_kernel(int64_t n_targets, int64_t n_nodes, int celebrity,
                                    const int64_t* __restrict__ ptr, const uint64_t* __restrict__ keys,
                                    int64_t* __restrict__ tcount, int64_t* __restrict__ npairs) {
  const uint64_t M = static_cast<uint64_t>(n_nodes);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t m = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; m < n_nodes; m += stride) {
    const int64_t deg = ptr[m + 1] - ptr[m];
    const bool alive = m < n_targets || (deg != 1 && deg <= celebrity);
    int64_t t = 0;
    if (alive) {
      for (int64_t k = ptr[m]; k < ptr[m + 1]; ++k)
        if (static_cast<int64_t>(keys[k] % M) < n_targets) ++t;
      if (m < n_targets) ++t;
    }
    tcount[m] = t;
    npairs[m] = t * (t - 1) / 2;
  }
}

// Sorted list T(m) of user neighbours (+ m itself for users) at toff[m].
__global__ void target_fill_kernel(int64_t n_targets, int64_t n_nodes, const int64_t* __restrict__ ptr,
                                   const uint64_t* __restrict__ keys, const int64_t* __restrict__ tcount,
                                   const int64_t* __restrict__ toff, int32_t* __restrict__ tlist) {
  const uint64_t M = static_cast<uint64_t>(n_nodes);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t m = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; m < n_nodes; m += stride) {
    if (tcount[m] == 0) continue;
    int64_t o = toff[m];
    bool self_done = m >= n_targets;
    for (int64_t k = ptr[m]; k < ptr[m + 1]; ++k) {
      const int64_t nb = static_cast<int64_t>(keys[k] % M);
      if (nb >= n_targets) continue;
      if (!self_done && m < nb) { tlist[o++] = static_cast<int32_t>(m); self_done = true; }
      tlist[o++] = static_cast<int32_t>(nb);
    }
    if (!self_done) tlist[o++] = static_cast<int32_t>(m);
  }
}

// Pair q of node m's list (row-major over i < j) -> key T[i]*N + T[j] (T sorted, so T[i] < T[j]).
__global__ void pair_keys_kernel(int64_t n_nodes, int64_t n_targets, int64_t total,
                                 const int64_t* __restrict__ poff, const int64_t* __restrict__ tcount,
                                 const int64_t* __restrict__ toff, const int32_t* __restrict__ tlist,
                                 uint64_t* __restrict__ keys) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total; g += stride) {
    int64_t lo = 0, hi = n_nodes;  // last m with poff[m] <= g
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (poff[mid] <= g) lo = mid; else hi = mid;
    }
    const int64_t m = lo, t = tcount[m];
    int64_t q = g - poff[m];
    // row i holds (t - 1 - i) pairs; i from the closed form, then fixed up in integers
    double disc = static_cast<double>(2 * t - 1) * (2 * t - 1) - 8.0 * static_cast<double>(q);
    int64_t i = static_cast<int64_t>((static_cast<double>(2 * t - 1) - sqrt(disc > 0 ? disc : 0.0)) / 2.0);
    if (i < 0) i = 0;
    auto row_start = [t](int64_t r) { return r * (2 * t - r - 1) / 2; };
    while (i > 0 && row_start(i) > q) --i;
    while (i + 1 < t && row_start(i + 1) <= q) ++i;
    const int64_t j = i + 1 + (q - row_start(i));
    const int64_t base = toff[m];
    keys[g] = static_cast<uint64_t>(tlist[base + i]) * static_cast<uint64_t>(n_targets) +
              static_cast<uint64_t>(tlist[base + j]);
  }
}

__global__ void decode_pairs_kernel(int64_t n_targets, const uint64_t* __restrict__ keys,
                                    const int64_t* __restrict__ n_unique, int32_t* __restrict__ u,
                                    int32_t* __restrict__ v) {
  const int64_t m = *n_unique;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t k = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k < m; k += stride) {
    u[k] = static_cast<int32_t>(keys[k] / static_cast<uint64_t>(n_targets));
    v[k] = static_cast<int32_t>(keys[k] % static_cast<uint64_t>(n_targets));
  }
}

struct DevMem {
  void* p = nullptr;
  hipStream_t s = nullptr;
  ~DevMem() { if (p) (void)hipFreeAsync(p, s); }
  hipError_t alloc(size_t bytes, hipStream_t st) { s = st; return hipMallocAsync(&p, std::max<size_t>(bytes, 16), st); }
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

int key_bits(uint64_t max_key) {
  int b = 1;
  while (b < 64 && (uint64_t{1} << b) <= max_key) ++b;
  return b;
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



gcg_status gcg_project_mention_graph(int64_t n_targets, int64_t n_nodes, int64_t n_inc,
                                     const int32_t* a, const int32_t* b, int celebrity_threshold,
                                     int32_t* out_u, int32_t* out_v, int64_t capacity,
                                     int64_t* n_edges, int32_t* status_dev, gcg_stream_t stream) {
  if (n_targets < 0 || n_nodes < n_targets || n_nodes >= INT32_MAX || n_inc < 0 ||
      n_edges == nullptr || status_dev == nullptr || (n_inc > 0 && (a == nullptr || b == nullptr)) ||
      2 * n_inc > INT32_MAX || (out_u == nullptr) != (out_v == nullptr))
    return fail(GCG_ERR_INVALID_ARG, "bad args to gcg_project_mention_graph");
  const bool sizing = out_u == nullptr;
  *n_edges = 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  GCG_HIP_CHECK(hipMemsetAsync(status_dev, 0, sizeof(int32_t), st));
  if (n_targets < 2) return GCG_OK;
  const int64_t m2 = 2 * n_inc;
  const uint64_t M = static_cast<uint64_t>(n_nodes);
  DevMem keys, keys2, cnt, ptr, tcount, npairs, toff, poff, tmp;
  size_t tb = 0;
  // 1. symmetric, deduplicated adjacency of g
  {
    uint64_t* k = nullptr; int64_t* c = nullptr; int64_t* o = nullptr;
    size_t t1 = 0, t2 = 0, t3 = 0;
    GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, t1, k, k, static_cast<int>(std::max<int64_t>(m2, 1)), 0, key_bits(M * M)));
    GCG_HIP_CHECK(hipcub::DeviceSelect::Unique(nullptr, t2, k, k, c, static_cast<int>(std::max<int64_t>(m2, 1))));
    GCG_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, t3, o, o, static_cast<int>(n_nodes)));
    tb = std::max({t1, t2, t3});
  }
  GCG_HIP_CHECK(keys.alloc(m2 * sizeof(uint64_t), st));
  GCG_HIP_CHECK(keys2.alloc(m2 * sizeof(uint64_t), st));
  GCG_HIP_CHECK(cnt.alloc(2 * sizeof(int64_t), st));
  GCG_HIP_CHECK(ptr.alloc((n_nodes + 1) * sizeof(int64_t), st));
  GCG_HIP_CHECK(tcount.alloc(n_nodes * sizeof(int64_t), st));
  GCG_HIP_CHECK(npairs.alloc(n_nodes * sizeof(int64_t), st));
  GCG_HIP_CHECK(toff.alloc(n_nodes * sizeof(int64_t), st));
  GCG_HIP_CHECK(poff.alloc(n_nodes * sizeof(int64_t), st));
  GCG_HIP_CHECK(tmp.alloc(tb, st));
  GCG_HIP_CHECK(hipMemsetAsync(cnt.p, 0, 2 * sizeof(int64_t), st));
  if (m2 > 0) {
    hipLaunchKernelGGL(incidence_keys_kernel, dim3(grid_for(n_inc)), dim3(256), 0, st, n_nodes, n_inc, a, b,
                       keys.as<uint64_t>(), status_dev);
    GCG_HIP_CHECK(hipGetLastError());
    size_t t = tb;
    GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp.p, t, keys.as<uint64_t>(), keys2.as<uint64_t>(),
                                                    static_cast<int>(m2), 0, key_bits(M * M), st));
    t = tb;
    GCG_HIP_CHECK(hipcub::DeviceSelect::Unique(tmp.p, t, keys2.as<uint64_t>(), keys.as<uint64_t>(),
                                               cnt.as<int64_t>(), static_cast<int>(m2), st));
  }
  hipLaunchKernelGGL(adj_ptr_kernel, dim3(grid_for(n_nodes + 1)), dim3(256), 0, st, n_nodes,
                     keys.as<uint64_t>(), cnt.as<int64_t>(), ptr.as<int64_t>());
  // 2-3. celebrity filter, user-neighbour lists, pair counts
  hipLaunchKernelGGL(target_count_kernel, dim3(grid_for(n_nodes)), dim3(256), 0, st, n_targets, n_nodes,
                     celebrity_threshold, ptr.as<int64_t>(), keys.as<uint64_t>(), tcount.as<int64_t>(),
                     npairs.as<int64_t>());
  GCG_HIP_CHECK(hipGetLastError());
  size_t t = tb;
  GCG_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, t, tcount.as<int64_t>(), toff.as<int64_t>(),
                                                 static_cast<int>(n_nodes), st));
  t = tb;
  GCG_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, t, npairs.as<int64_t>(), poff.as<int64_t>(),
                                                 static_cast<int>(n_nodes), st));
  int64_t last[4] = {0, 0, 0, 0};  // toff[M-1], tcount[M-1], poff[M-1], npairs[M-1]
  GCG_HIP_CHECK(hipMemcpyAsync(&last[0], toff.as<int64_t>() + n_nodes - 1, 8, hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipMemcpyAsync(&last[1], tcount.as<int64_t>() + n_nodes - 1, 8, hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipMemcpyAsync(&last[2], poff.as<int64_t>() + n_nodes - 1, 8, hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipMemcpyAsync(&last[3], npairs.as<int64_t>() + n_nodes - 1, 8, hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  const int64_t n_tlist = last[0] + last[1], P = last[2] + last[3];
  if (sizing) {  // capacity query: the number of pairs bounds the number of edges
    *n_edges = P;
    return GCG_OK;
  }
  if (P == 0) return GCG_OK;
  if (P > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "%lld projected pairs exceed the int32 sort range", (long long)P);
  DevMem tlist, pk, pk2, ucnt, tmp2;
  GCG_HIP_CHECK(tlist.alloc(n_tlist * sizeof(int32_t), st));
  GCG_HIP_CHECK(pk.alloc(P * sizeof(uint64_t), st));
  GCG_HIP_CHECK(pk2.alloc(P * sizeof(uint64_t), st));
  GCG_HIP_CHECK(ucnt.alloc(sizeof(int64_t), st));
  hipLaunchKernelGGL(target_fill_kernel, dim3(grid_for(n_nodes)), dim3(256), 0, st, n_targets, n_nodes,
                     ptr.as<int64_t>(), keys.as<uint64_t>(), tcount.as<int64_t>(), toff.as<int64_t>(),
                     tlist.as<int32_t>());
  hipLaunchKernelGGL(pair_keys_kernel, dim3(grid_for(P)), dim3(256), 0, st, n_nodes, n_targets, P,
                     poff.as<int64_t>(), tcount.as<int64_t>(), toff.as<int64_t>(), tlist.as<int32_t>(),
                     pk.as<uint64_t>());
  GCG_HIP_CHECK(hipGetLastError());
  // 4. dedupe pairs
  const uint64_t N = static_cast<uint64_t>(n_targets);
  size_t t4 = 0, t5 = 0;
  {
    uint64_t* k = nullptr; int64_t* c = nullptr;
    GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, t4, k, k, static_cast<int>(P), 0, key_bits(N * N)));
    GCG_HIP_CHECK(hipcub::DeviceSelect::Unique(nullptr, t5, k, k, c, static_cast<int>(P)));
  }
  GCG_HIP_CHECK(tmp2.alloc(std::max(t4, t5), st));
  t4 = std::max(t4, t5);
  size_t tt = t4;
  GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp2.p, tt, pk.as<uint64_t>(), pk2.as<uint64_t>(),
                                                  static_cast<int>(P), 0, key_bits(N * N), st));
  tt = t4;
  GCG_HIP_CHECK(hipcub::DeviceSelect::Unique(tmp2.p, tt, pk2.as<uint64_t>(), pk.as<uint64_t>(),
                                             ucnt.as<int64_t>(), static_cast<int>(P), st));
  int64_t n_unique = 0;
  GCG_HIP_CHECK(hipMemcpyAsync(&n_unique, ucnt.p, 8, hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  if (n_unique > capacity)
    return fail(GCG_ERR_WORKSPACE, "output capacity %lld < %lld edges", (long long)capacity, (long long)n_unique);
  hipLaunchKernelGGL(decode_pairs_kernel, dim3(grid_for(n_unique)), dim3(256), 0, st, n_targets,
                     pk.as<uint64_t>(), ucnt.as<int64_t>(), out_u, out_v);
  GCG_HIP_CHECK(hipGetLastError());
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  *n_edges = n_unique;
  return GCG_OK;
}


}  // extern "C"
