// gcg_spmm.hip -- MI355X (gfx950 / CDNA4) CSR x dense SpMM for the graphconvgeo GCN hot path.
//
// Implements include/gcg_spmm.h. The reference computes Y = act(H . Z + b) with
// theano.sparse.dot (mlpconv.py:71,73,90) on the host CPU via scipy `csr_matvecs`;
// here the product is a memory-bound row gather on the GPU:
//
//   * One 64-lane wave owns one output row at a time. Lanes span the dense width K
//     in VEC-float vectors (16-byte dwordx4 loads when K, ldz, ldy and the pointers
//     allow), so one nonzero costs one coalesced read of a whole Z row (1200 B at
//     K = 300: 64 lanes x 16 B + 11 lanes x 16 B).
//   * The row's (column, value) pairs are wave-uniform: they are read through the
//     scalar unit (s_load) and the Z row base is an SGPR, so there is no per-lane
//     index traffic and no divergence.
//   * U nonzeros are gathered per batch before any is consumed (U x row bytes in
//     flight per wave) and then accumulated in storage order, mul and add rounded
//     separately (-ffp-contract=off): bitwise scipy float32.
//   * Widths beyond one panel (64 lanes x VEC x NCH <= 512 floats) are split into
//     column panels on grid.y; each panel re-reads only the 8-byte (col, val) stream.
//   * Load balance (power-law degrees, data.py:245-249 co-mention cliques): the plan
//     groups consecutive rows into tasks of ~task_nnz nonzeros, and splits longer rows
//     into segments whose partial sums go to a workspace; a fix-up kernel adds the
//     segments of each split row in order and applies the epilogue.
//   * Epilogue fused: + bias (mlpconv.py:75-76,92-93), rectify = 0.5*(x+|x|) as
//     Theano's nnet.relu computes it (mlpconv.py:77 via lasagne.nonlinearities.rectify),
//     and the target_indices row subset (mlpconv.py:94) via out_rows.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "../../include/gcg_spmm.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kPanelMax = 512;  // floats per column panel
constexpr int64_t kDefaultTaskNnz = 512;
constexpr int64_t kRowCost = 2;  // planner: per-row overhead in nonzero-equivalents

thread_local std::string g_last_error;

gcg_status fail(gcg_status st, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
gcg_status fail(gcg_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return st;
}

#define GCG_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      return fail(GCG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));     \
  } while (0)

inline bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

// ------------------------------------------------------------------------------------
// Vector helpers. Explicit per-component arithmetic keeps the rounding sequence
// exactly acc = acc + (v * z) per element.
// ------------------------------------------------------------------------------------
template <int VEC>
struct Vec {
  float x[VEC];
};

template <int VEC>
__device__ __forceinline__ Vec<VEC> load_vec(const float* __restrict__ p) {
  Vec<VEC> r;
  if constexpr (VEC == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    r.x[0] = t.x; r.x[1] = t.y; r.x[2] = t.z; r.x[3] = t.w;
  } else if constexpr (VEC == 2) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    r.x[0] = t.x; r.x[1] = t.y;
  } else {
    r.x[0] = *p;
  }
  return r;
}

template <int VEC>
__device__ __forceinline__ void store_vec(float* __restrict__ p, const Vec<VEC>& v) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v.x[0], v.x[1], v.x[2], v.x[3]);
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v.x[0], v.x[1]);
  } else {
    *p = v.x[0];
  }
}

__device__ __forceinline__ float apply_act(float y, int act) {
  // lasagne.nonlinearities.rectify -> theano.tensor.nnet.relu(x) = 0.5 * (x + abs(x))
  return act == GCG_ACT_RELU ? 0.5f * (y + fabsf(y)) : y;
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Accumulate nonzeros [s, e) of one row into acc, storage order, U gathers in flight.
template <int VEC, int NCH, int U>
__device__ __forceinline__ void accumulate_range(int s, int e, const int32_t* __restrict__ indices,
                                                 const float* __restrict__ vals,
                                                 const float* __restrict__ Z, int64_t ldz,
                                                 const int (&col)[NCH], Vec<VEC> (&acc)[NCH]) {
  // `col` is pre-clamped for lanes past K (they re-read a column of the same row, which
  // coalesces with lane 0's line): no exec-mask branches, so hipcc can count vmcnt.
  int j = s;
  for (; j + U <= e; j += U) {
    int c[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = indices[j + u];
      v[u] = vals[j + u];
    }
    Vec<VEC> z[U][NCH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* zrow = Z + static_cast<int64_t>(c[u]) * ldz;
#pragma unroll
      for (int k = 0; k < NCH; ++k)
        z[u][k] = load_vec<VEC>(zrow + col[k]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < NCH; ++k)
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[k].x[q] = acc[k].x[q] + v[u] * z[u][k].x[q];
  }
  const int rem = e - j;  // wave-uniform, < U
  if (rem > 0) {
    int c[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      if (u < rem) {
        c[u] = indices[j + u];
        v[u] = vals[j + u];
      }
    Vec<VEC> z[U][NCH];
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      if (u < rem) {
        const float* zrow = Z + static_cast<int64_t>(c[u]) * ldz;
#pragma unroll
        for (int k = 0; k < NCH; ++k)
          z[u][k] = load_vec<VEC>(zrow + col[k]);
      }
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      if (u < rem)
#pragma unroll
        for (int k = 0; k < NCH; ++k)
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[k].x[q] = acc[k].x[q] + v[u] * z[u][k].x[q];
  }
}

// Main kernel. One wave per task; grid.y = column panel.
//   tasks == nullptr : task w = rows of positions [w, w+1)           (plan-less path)
//   task.w <  0      : rows of positions [task.x, task.y)            (short rows)
//   task.w >= 0      : position task.x, nonzeros [task.y, task.z) -> workspace slot task.w
template <int VEC, int NCH, int U, int WPB = kWavesPerBlock>
__global__ __launch_bounds__(kWave * WPB) void spmm_rows_kernel(
    const int4* __restrict__ tasks, int n_tasks, const int32_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const float* __restrict__ vals,
    const int32_t* __restrict__ out_rows, const float* __restrict__ Z, int64_t ldz, int K,
    float* __restrict__ Y, int64_t ldy, const float* __restrict__ bias, int act,
    float* __restrict__ ws, int64_t ldws) {
  const int w = uniform(static_cast<int>(blockIdx.x) * WPB + (threadIdx.x >> 6));
  if (w >= n_tasks) return;
  const int lane = threadIdx.x & (kWave - 1);
  const int panel0 = static_cast<int>(blockIdx.y) * (kWave * VEC * NCH);

  int col[NCH], gcol[NCH];  // output column / clamped gather column
  bool on[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    col[k] = panel0 + (k * kWave + lane) * VEC;
    on[k] = col[k] < K;
    gcol[k] = on[k] ? col[k] : panel0;
  }

  int4 t;
  if (tasks != nullptr) {
    t = tasks[w];
    t.x = uniform(t.x); t.y = uniform(t.y); t.z = uniform(t.z); t.w = uniform(t.w);
  } else {
    t = make_int4(w, w + 1, -1, -1);
  }

  Vec<VEC> acc[NCH];
  if (t.w >= 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[k].x[q] = 0.0f;
    accumulate_range<VEC, NCH, U>(t.y, t.z, indices, vals, Z, ldz, gcol, acc);
    float* dst = ws + static_cast<int64_t>(t.w) * ldws;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
      if (on[k]) store_vec<VEC>(dst + col[k], acc[k]);
    return;
  }

  for (int p = t.x; p < t.y; ++p) {
    const int r = out_rows ? uniform(out_rows[p]) : p;
    const int s = uniform(indptr[r]);
    const int e = uniform(indptr[r + 1]);
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[k].x[q] = 0.0f;
    accumulate_range<VEC, NCH, U>(s, e, indices, vals, Z, ldz, gcol, acc);
    float* yrow = Y + static_cast<int64_t>(p) * ldy;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (!on[k]) continue;
      if (bias != nullptr) {
        const Vec<VEC> b = load_vec<VEC>(bias + col[k]);
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[k].x[q] = acc[k].x[q] + b.x[q];
      }
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[k].x[q] = apply_act(acc[k].x[q], act);
      store_vec<VEC>(yrow + col[k], acc[k]);
    }
  }
}

// Fix-up for split rows: Y[p] = act(sum_{s in slots, in order} ws[s] + bias).
// One wave per (split row, 64-column strip).
__global__ __launch_bounds__(kBlock) void spmm_fixup_kernel(const int4* __restrict__ longs,
                                                            int n_long,
                                                            const float* __restrict__ ws,
                                                            int64_t ldws, int K,
                                                            float* __restrict__ Y, int64_t ldy,
                                                            const float* __restrict__ bias,
                                                            int act) {
  const int w = uniform(static_cast<int>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6));
  if (w >= n_long) return;
  const int c = static_cast<int>(blockIdx.y) * kWave + (threadIdx.x & (kWave - 1));
  if (c >= K) return;
  const int4 L = longs[w];
  const float* src = ws + static_cast<int64_t>(L.y) * ldws + c;
  float acc = src[0];
  for (int s = 1; s < L.z; ++s) acc = acc + src[static_cast<int64_t>(s) * ldws];
  if (bias != nullptr) acc = acc + bias[c];
  Y[static_cast<int64_t>(L.x) * ldy + c] = apply_act(acc, act);
}

// ------------------------------------------------------------------------------------
// Launch dispatch: pick VEC (vector width) and NCH (vectors per lane per panel).
// ------------------------------------------------------------------------------------
struct LaunchArgs {
  const int4* tasks;
  int n_tasks;
  const int32_t* indptr;
  const int32_t* indices;
  const float* vals;
  const int32_t* out_rows;
  const float* Z;
  int64_t ldz;
  int K;
  float* Y;
  int64_t ldy;
  const float* bias;
  int act;
  float* ws;
  int64_t ldws;
  int64_t task_nnz;  // plan task size (0 = plan-less, one row per wave)
};

template <int VEC, int NCH, int U, int WPB>
void launch_rows_u(const LaunchArgs& a, int n_panels, hipStream_t stream) {
  const dim3 grid((a.n_tasks + WPB - 1) / WPB, n_panels);
  hipLaunchKernelGGL((spmm_rows_kernel<VEC, NCH, U, WPB>), grid, dim3(kWave * WPB), 0, stream,
                     a.tasks, a.n_tasks, a.indptr, a.indices, a.vals, a.out_rows, a.Z, a.ldz, a.K,
                     a.Y, a.ldy, a.bias, a.act, a.ws, a.ldws);
}

// Experiment knobs (GCG_UNROLL = gathers per lane per batch, GCG_WPB = waves per workgroup),
// instantiated for the K = 300 variant only; 0 / unset = the defaults below.
int env_int(const char* name) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : 0;
}

// Gathers in flight per lane: INFLIGHT floats of Z per lane per batch (U = INFLIGHT/(VEC*NCH)
// nonzeros). Measured (MI355X, same box, K = 300 variant VEC = 4 / NCH = 2): 192 floats
// (U = 24, 210 VGPRs, 2 waves/SIMD) vs 64 (U = 8, 92 VGPRs, 5 waves/SIMD): Twitter-World
// power-law 6.67 vs 6.97 ms, Twitter-US 1.70 vs 1.81 ms, uniform equal; but slower on the
// small GEOTEXT graph (32-nnz tasks: 39 vs 26 us) and for the narrower variants (K = 64, 128,
// 129). 256 floats (U = 32) drops to 1 wave/SIMD and halves throughput. So the deep batch is
// used for the VEC 4 x 2 variant with >= 256-nnz tasks only; GCG_INFLIGHT=64 forces the shallow.
template <int VEC, int NCH, int INFLIGHT>
void launch_rows_f(const LaunchArgs& a, int n_panels, hipStream_t stream) {
  constexpr int U0 = INFLIGHT / (VEC * NCH);
  constexpr int U = U0 > 24 ? 24 : (U0 < 2 ? 2 : U0);
  launch_rows_u<VEC, NCH, U, kWavesPerBlock>(a, n_panels, stream);
}

template <int VEC, int NCH>
void launch_rows(const LaunchArgs& a, int n_panels, hipStream_t stream) {
  if constexpr (VEC == 4 && NCH == 2) {
    static const int u = env_int("GCG_UNROLL"), inflight = env_int("GCG_INFLIGHT");
    if (u == 16) return launch_rows_u<4, 2, 16, kWavesPerBlock>(a, n_panels, stream);
    if (inflight != 64 && a.task_nnz >= 256) return launch_rows_f<4, 2, 192>(a, n_panels, stream);
  }
  launch_rows_f<VEC, NCH, 64>(a, n_panels, stream);
}

int pick_vec(const float* Z, int64_t ldz, const float* Y, int64_t ldy, int64_t K,
             const float* bias, const float* ws, int64_t ldws) {
  for (int vec : {4, 2}) {
    const size_t bytes = sizeof(float) * vec;
    if (K % vec == 0 && ldz % vec == 0 && ldy % vec == 0 && aligned(Z, bytes) &&
        aligned(Y, bytes) && (bias == nullptr || aligned(bias, bytes)) &&
        (ws == nullptr || (aligned(ws, bytes) && ldws % vec == 0)))
      return vec;
  }
  return 1;
}

// Returns panel width (floats) and launches.
int panel_override() {
  static const int v = [] {
    const char* e = std::getenv("GCG_PANEL");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

gcg_status launch_spmm(const LaunchArgs& a, int vec, hipStream_t stream) {
  const int64_t K = a.K;
  const int req = panel_override();  // experiment knob: panel width in floats
  if (req > 0)
    while (vec > 1 && kWave * vec > req) vec /= 2;
  const int per_chunk = kWave * vec;
  const int nch_max = req > 0 ? std::max(1, std::min(kPanelMax, req) / per_chunk) : kPanelMax / per_chunk;
  int nch = static_cast<int>((K + per_chunk - 1) / per_chunk);
  if (nch > nch_max) nch = nch_max;
  if (nch < 1) nch = 1;
  const int panel = per_chunk * nch;
  const int n_panels = static_cast<int>((K + panel - 1) / panel);
  if (a.n_tasks <= 0 || K <= 0) return GCG_OK;
  switch (vec * 16 + nch) {
    case 4 * 16 + 1: launch_rows<4, 1>(a, n_panels, stream); break;
    case 4 * 16 + 2: launch_rows<4, 2>(a, n_panels, stream); break;
    case 2 * 16 + 1: launch_rows<2, 1>(a, n_panels, stream); break;
    case 2 * 16 + 2: launch_rows<2, 2>(a, n_panels, stream); break;
    case 2 * 16 + 3: launch_rows<2, 3>(a, n_panels, stream); break;
    case 2 * 16 + 4: launch_rows<2, 4>(a, n_panels, stream); break;
    case 1 * 16 + 1: launch_rows<1, 1>(a, n_panels, stream); break;
    case 1 * 16 + 2: launch_rows<1, 2>(a, n_panels, stream); break;
    case 1 * 16 + 3: launch_rows<1, 3>(a, n_panels, stream); break;
    case 1 * 16 + 4: launch_rows<1, 4>(a, n_panels, stream); break;
    case 1 * 16 + 5: launch_rows<1, 5>(a, n_panels, stream); break;
    case 1 * 16 + 6: launch_rows<1, 6>(a, n_panels, stream); break;
    case 1 * 16 + 7: launch_rows<1, 7>(a, n_panels, stream); break;
    case 1 * 16 + 8: launch_rows<1, 8>(a, n_panels, stream); break;
    default: return fail(GCG_ERR_INVALID_ARG, "internal: no kernel for vec=%d nch=%d", vec, nch);
  }
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

gcg_status check_dense(const float* Z, int64_t ldz, float* Y, int64_t ldy, int64_t K,
                       const float* bias, int act) {
  if (K < 0 || K > (int64_t{1} << 30)) return fail(GCG_ERR_INVALID_ARG, "bad K=%lld", (long long)K);
  if (K > 0 && (Z == nullptr || Y == nullptr)) return fail(GCG_ERR_INVALID_ARG, "Z or Y is NULL");
  if (ldz < K || ldy < K) return fail(GCG_ERR_INVALID_ARG, "ldz=%lld / ldy=%lld < K=%lld",
                                      (long long)ldz, (long long)ldy, (long long)K);
  if (!aligned(Z, 4) || !aligned(Y, 4) || (bias && !aligned(bias, 4)))
    return fail(GCG_ERR_MISALIGNED, "Z/Y/bias not 4-byte aligned");
  if (act != GCG_ACT_NONE && act != GCG_ACT_RELU) return fail(GCG_ERR_INVALID_ARG, "bad act=%d", act);
  return GCG_OK;
}

// ------------------------------------------------------------------------------------
// Host planner.
// ------------------------------------------------------------------------------------
struct HostPlan {
  std::vector<int32_t> tasks;  // quadruples
  std::vector<int32_t> longs;  // quadruples
  int64_t n_slots = 0;
  int64_t max_task_nnz = 0;
};

// Default task size: 512 nonzeros, smaller on small graphs so the launch still has
// >= ~8k waves (256 CUs x 32 waves) to spread; never below 32.
int64_t default_task_nnz(int64_t nnz) {
  int64_t w = nnz / 8192;
  return w < 32 ? 32 : (w > kDefaultTaskNnz ? kDefaultTaskNnz : w);
}

gcg_status build_host_plan(int64_t n_rows, const int32_t* indptr, const int32_t* out_rows,
                           int64_t n_out, int64_t task_nnz, int ordered, HostPlan* hp) {
  if (task_nnz <= 0) task_nnz = default_task_nnz(indptr[n_rows]);
  if (indptr[0] != 0) return fail(GCG_ERR_BAD_CSR, "indptr[0] = %d != 0", indptr[0]);
  for (int64_t r = 0; r < n_rows; ++r)
    if (indptr[r + 1] < indptr[r]) return fail(GCG_ERR_BAD_CSR, "indptr decreases at row %lld", (long long)r);
  hp->tasks.clear();
  hp->longs.clear();
  hp->n_slots = 0;
  hp->max_task_nnz = 0;
  std::vector<int32_t> seg_tasks;
  std::vector<std::pair<int64_t, int64_t>> long_rows;  // (nnz, position), ordered mode
  int64_t cur_begin = -1, cur_cost = 0, cur_nnz = 0;
  auto close = [&](int64_t end) {
    if (cur_begin >= 0) {
      hp->tasks.insert(hp->tasks.end(), {int32_t(cur_begin), int32_t(end), -1, -1});
      hp->max_task_nnz = std::max(hp->max_task_nnz, cur_nnz);
    }
    cur_begin = -1;
    cur_cost = 0;
    cur_nnz = 0;
  };
  for (int64_t p = 0; p < n_out; ++p) {
    const int64_t r = out_rows ? out_rows[p] : p;
    if (r < 0 || r >= n_rows) return fail(GCG_ERR_INVALID_ARG, "out_rows[%lld]=%lld out of range", (long long)p, (long long)r);
    const int64_t s = indptr[r], e = indptr[r + 1], len = e - s;
    if (!ordered && len > task_nnz) {
      close(p);
      const int64_t nseg = (len + task_nnz - 1) / task_nnz;
      // Equal-sized segments (differ by at most one nonzero).
      hp->longs.insert(hp->longs.end(), {int32_t(p), int32_t(hp->n_slots), int32_t(nseg), 0});
      for (int64_t k = 0; k < nseg; ++k) {
        const int64_t b = s + (len * k) / nseg, f = s + (len * (k + 1)) / nseg;
        seg_tasks.insert(seg_tasks.end(), {int32_t(p), int32_t(b), int32_t(f), int32_t(hp->n_slots + k)});
        hp->max_task_nnz = std::max(hp->max_task_nnz, f - b);
      }
      hp->n_slots += nseg;
      continue;
    }
    if (ordered && len > task_nnz) {
      // Unsplittable long row (bitwise mode): its own task, scheduled first (LPT) so the
      // serial tail of a hub row overlaps the bulk instead of ending the launch.
      close(p);
      long_rows.push_back({len, p});
      continue;
    }
    const int64_t cost = len + kRowCost;
    if (cur_begin >= 0 && cur_cost + cost > task_nnz) close(p);
    if (cur_begin < 0) cur_begin = p;
    cur_cost += cost;
    cur_nnz += len;
  }
  close(n_out);
  // Longest work first: unsplit long rows (ordered mode) by descending length, then the
  // segments of split rows, then the short-row tasks in row order.
  std::stable_sort(long_rows.begin(), long_rows.end(),
                   [](const std::pair<int64_t, int64_t>& a, const std::pair<int64_t, int64_t>& b) {
                     return a.first > b.first;
                   });
  std::vector<int32_t> head;
  head.reserve(long_rows.size() * 4 + seg_tasks.size());
  for (const auto& lr : long_rows) {
    head.insert(head.end(), {int32_t(lr.second), int32_t(lr.second + 1), -1, -1});
    hp->max_task_nnz = std::max(hp->max_task_nnz, lr.first);
  }
  head.insert(head.end(), seg_tasks.begin(), seg_tasks.end());
  hp->tasks.insert(hp->tasks.begin(), head.begin(), head.end());
  if (hp->tasks.size() / 4 > static_cast<size_t>(INT32_MAX)) return fail(GCG_ERR_INVALID_ARG, "too many tasks");
  return GCG_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------
// Plan object.
// ------------------------------------------------------------------------------------
struct gcg_spmm_plan {
  int64_t n_rows = 0, n_cols = 0, nnz = 0, n_out = 0;
  int ordered = 0;
  int64_t task_nnz = 0;
  int n_tasks = 0, n_long = 0;
  int64_t n_slots = 0, max_task_nnz = 0;
  int4* tasks = nullptr;     // device
  int4* longs = nullptr;     // device
  int32_t* out_rows = nullptr;  // device copy (nullptr = identity)
};

extern "C" {

const char* gcg_version(void) { return "0.1.0"; }
const char* gcg_last_error(void) { return g_last_error.c_str(); }

gcg_status gcg_spmm_csr_f32(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t* indptr,
                            const int32_t* indices, const float* vals, const float* Z,
                            int64_t ldz, int64_t K, float* Y, int64_t ldy, const float* bias,
                            int act, const int32_t* out_rows, int64_t n_out,
                            gcg_stream_t stream) {
  if (n_rows < 0 || n_cols < 0 || nnz < 0 || n_rows > INT32_MAX || nnz > INT32_MAX)
    return fail(GCG_ERR_INVALID_ARG, "bad CSR shape n_rows=%lld n_cols=%lld nnz=%lld",
                (long long)n_rows, (long long)n_cols, (long long)nnz);
  if (out_rows == nullptr) n_out = n_rows;
  if (n_out < 0 || n_out > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "bad n_out=%lld", (long long)n_out);
  if (gcg_status st = check_dense(Z, ldz, Y, ldy, K, bias, act)) return st;
  if (n_out > 0 && indptr == nullptr) return fail(GCG_ERR_INVALID_ARG, "indptr is NULL");
  if (nnz > 0 && (indices == nullptr || vals == nullptr)) return fail(GCG_ERR_INVALID_ARG, "indices/vals NULL");
  if (n_out == 0 || K == 0) return GCG_OK;
  LaunchArgs a{nullptr, int(n_out), indptr, indices, vals, out_rows, Z, ldz, int(K), Y, ldy,
               bias, act, nullptr, 0, 0};
  return launch_spmm(a, pick_vec(Z, ldz, Y, ldy, K, bias, nullptr, 0),
                     static_cast<hipStream_t>(stream));
}

gcg_status gcg_spmm_plan_host(int64_t n_rows, const int32_t* indptr_host,
                              const int32_t* out_rows_host, int64_t n_out, int64_t task_nnz,
                              int ordered, int32_t* tasks_host, int64_t tasks_cap,
                              int64_t* n_tasks, int32_t* long_host, int64_t long_cap,
                              int64_t* n_long, int64_t* n_slots) {
  if (n_rows < 0 || indptr_host == nullptr) return fail(GCG_ERR_INVALID_ARG, "bad n_rows/indptr");
  if (out_rows_host == nullptr) n_out = n_rows;
  HostPlan hp;
  try {
    if (gcg_status st = build_host_plan(n_rows, indptr_host, out_rows_host, n_out, task_nnz, ordered, &hp)) return st;
  } catch (const std::bad_alloc&) {
    return fail(GCG_ERR_ALLOC, "host allocation failed");
  }
  const int64_t nt = hp.tasks.size() / 4, nl = hp.longs.size() / 4;
  if (n_tasks) *n_tasks = nt;
  if (n_long) *n_long = nl;
  if (n_slots) *n_slots = hp.n_slots;
  if (tasks_host) {
    if (tasks_cap < nt) return fail(GCG_ERR_INVALID_ARG, "tasks_cap %lld < %lld", (long long)tasks_cap, (long long)nt);
    std::memcpy(tasks_host, hp.tasks.data(), hp.tasks.size() * sizeof(int32_t));
  }
  if (long_host) {
    if (long_cap < nl) return fail(GCG_ERR_INVALID_ARG, "long_cap %lld < %lld", (long long)long_cap, (long long)nl);
    std::memcpy(long_host, hp.longs.data(), hp.longs.size() * sizeof(int32_t));
  }
  return GCG_OK;
}

gcg_status gcg_spmm_plan_create(gcg_spmm_plan** plan, int64_t n_rows, int64_t n_cols,
                                int64_t nnz, const int32_t* indptr, const int32_t* out_rows,
                                int64_t n_out, int64_t task_nnz, int ordered,
                                gcg_stream_t stream) {
  if (plan == nullptr) return fail(GCG_ERR_INVALID_ARG, "plan is NULL");
  *plan = nullptr;
  if (n_rows < 0 || n_cols < 0 || nnz < 0 || n_rows > INT32_MAX - 1 || nnz > INT32_MAX || indptr == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "bad CSR shape");
  if (out_rows == nullptr) n_out = n_rows;
  if (n_out < 0 || n_out > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "bad n_out");
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<int32_t> h_indptr, h_rows;
  HostPlan hp;
  try {
    h_indptr.resize(n_rows + 1);
    if (out_rows) h_rows.resize(n_out);
  } catch (const std::bad_alloc&) {
    return fail(GCG_ERR_ALLOC, "host allocation failed");
  }
  GCG_HIP_CHECK(hipMemcpyAsync(h_indptr.data(), indptr, (n_rows + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  if (out_rows && n_out > 0)
    GCG_HIP_CHECK(hipMemcpyAsync(h_rows.data(), out_rows, n_out * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  if (h_indptr[n_rows] != nnz)
    return fail(GCG_ERR_BAD_CSR, "indptr[n_rows]=%d != nnz=%lld", h_indptr[n_rows], (long long)nnz);
  if (gcg_status s = build_host_plan(n_rows, h_indptr.data(), out_rows ? h_rows.data() : nullptr,
                                     n_out, task_nnz, ordered, &hp))
    return s;
  gcg_spmm_plan* p = new (std::nothrow) gcg_spmm_plan();
  if (p == nullptr) return fail(GCG_ERR_ALLOC, "plan allocation failed");
  p->n_rows = n_rows; p->n_cols = n_cols; p->nnz = nnz; p->n_out = n_out;
  p->ordered = ordered; p->task_nnz = task_nnz > 0 ? task_nnz : default_task_nnz(nnz);
  p->n_tasks = static_cast<int>(hp.tasks.size() / 4);
  p->n_long = static_cast<int>(hp.longs.size() / 4);
  p->n_slots = hp.n_slots;
  p->max_task_nnz = hp.max_task_nnz;
  auto cleanup = [&]() { gcg_spmm_plan_destroy(p); };
  hipError_t e = hipSuccess;
  if (p->n_tasks > 0) e = hipMalloc(&p->tasks, hp.tasks.size() * sizeof(int32_t));
  if (e == hipSuccess && p->n_long > 0) e = hipMalloc(&p->longs, hp.longs.size() * sizeof(int32_t));
  if (e == hipSuccess && out_rows && n_out > 0) e = hipMalloc(&p->out_rows, n_out * sizeof(int32_t));
  if (e != hipSuccess) { cleanup(); return fail(GCG_ERR_ALLOC, "hipMalloc: %s", hipGetErrorString(e)); }
  if (p->n_tasks > 0) e = hipMemcpyAsync(p->tasks, hp.tasks.data(), hp.tasks.size() * sizeof(int32_t), hipMemcpyHostToDevice, st);
  if (e == hipSuccess && p->n_long > 0) e = hipMemcpyAsync(p->longs, hp.longs.data(), hp.longs.size() * sizeof(int32_t), hipMemcpyHostToDevice, st);
  if (e == hipSuccess && p->out_rows) e = hipMemcpyAsync(p->out_rows, h_rows.data(), n_out * sizeof(int32_t), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) { cleanup(); return fail(GCG_ERR_HIP, "plan upload: %s", hipGetErrorString(e)); }
  *plan = p;
  return GCG_OK;
}

gcg_status gcg_spmm_plan_destroy(gcg_spmm_plan* plan) {
  if (plan == nullptr) return GCG_OK;
  hipError_t e1 = plan->tasks ? hipFree(plan->tasks) : hipSuccess;
  hipError_t e2 = plan->longs ? hipFree(plan->longs) : hipSuccess;
  hipError_t e3 = plan->out_rows ? hipFree(plan->out_rows) : hipSuccess;
  delete plan;
  if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess)
    return fail(GCG_ERR_HIP, "hipFree failed in plan destroy");
  return GCG_OK;
}

gcg_status gcg_spmm_plan_workspace_bytes(const gcg_spmm_plan* plan, int64_t K, size_t* bytes) {
  if (plan == nullptr || bytes == nullptr || K < 0) return fail(GCG_ERR_INVALID_ARG, "bad args");
  // Row stride rounded up to 4 floats so the workspace never forces a narrower vector width.
  const int64_t ldws = (K + 3) & ~int64_t{3};
  *bytes = static_cast<size_t>(plan->n_slots) * ldws * sizeof(float);
  return GCG_OK;
}

gcg_status gcg_spmm_plan_info(const gcg_spmm_plan* plan, int64_t* n_tasks, int64_t* n_long_rows,
                              int64_t* n_segments, int64_t* max_task_nnz) {
  if (plan == nullptr) return fail(GCG_ERR_INVALID_ARG, "plan is NULL");
  if (n_tasks) *n_tasks = plan->n_tasks;
  if (n_long_rows) *n_long_rows = plan->n_long;
  if (n_segments) *n_segments = plan->n_slots;
  if (max_task_nnz) *max_task_nnz = plan->max_task_nnz;
  return GCG_OK;
}

gcg_status gcg_spmm_csr_f32_planned(const gcg_spmm_plan* plan, const int32_t* indptr,
                                    const int32_t* indices, const float* vals, const float* Z,
                                    int64_t ldz, int64_t K, float* Y, int64_t ldy,
                                    const float* bias, int act, void* workspace,
                                    size_t workspace_bytes, gcg_stream_t stream) {
  if (plan == nullptr) return fail(GCG_ERR_INVALID_ARG, "plan is NULL");
  if (gcg_status st = check_dense(Z, ldz, Y, ldy, K, bias, act)) return st;
  if (plan->n_out > 0 && indptr == nullptr) return fail(GCG_ERR_INVALID_ARG, "indptr is NULL");
  if (plan->nnz > 0 && (indices == nullptr || vals == nullptr)) return fail(GCG_ERR_INVALID_ARG, "indices/vals NULL");
  if (K == 0 || plan->n_tasks == 0) return GCG_OK;
  size_t need = 0;
  gcg_spmm_plan_workspace_bytes(plan, K, &need);
  if (need > 0 && (workspace == nullptr || workspace_bytes < need))
    return fail(GCG_ERR_WORKSPACE, "workspace %zu bytes < %zu needed", workspace_bytes, need);
  if (need > 0 && !aligned(workspace, 16)) return fail(GCG_ERR_MISALIGNED, "workspace not 16-byte aligned");
  const int64_t ldws = (K + 3) & ~int64_t{3};
  float* ws = need > 0 ? static_cast<float*>(workspace) : nullptr;
  hipStream_t st = static_cast<hipStream_t>(stream);
  LaunchArgs a{plan->tasks, plan->n_tasks, indptr, indices, vals, plan->out_rows, Z, ldz, int(K),
               Y, ldy, bias, act, ws, ldws, plan->task_nnz};
  if (gcg_status s = launch_spmm(a, pick_vec(Z, ldz, Y, ldy, K, bias, ws, ldws), st)) return s;
  if (plan->n_long > 0) {
    const dim3 grid((plan->n_long + kWavesPerBlock - 1) / kWavesPerBlock, (K + kWave - 1) / kWave);
    hipLaunchKernelGGL(spmm_fixup_kernel, grid, dim3(kBlock), 0, st, plan->longs, plan->n_long,
                       ws, ldws, int(K), Y, ldy, bias, act);
    GCG_HIP_CHECK(hipGetLastError());
  }
  return GCG_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// CSR validation, index CSR + scatter-add, transpose.
// ------------------------------------------------------------------------------------
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

__global__ void iota_kernel(int32_t* __restrict__ out, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = static_cast<int32_t>(i);
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

// Row id of every nonzero (expanded indptr).
__global__ void expand_rows_kernel(int64_t n_rows, const int32_t* __restrict__ indptr,
                                   int32_t* __restrict__ row_of) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < n_rows; r += stride)
    for (int32_t j = indptr[r]; j < indptr[r + 1]; ++j) row_of[j] = static_cast<int32_t>(r);
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

inline int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > 4096) g = 4096;
  return static_cast<int>(g);
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

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

int bits_for(int64_t n) {
  int b = 1;
  while (b < 31 && (int64_t{1} << b) < n) ++b;
  return b;
}


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
__global__ void spgemm_emit_kernel(int64_t n_keep, int64_t p, const uint64_t* __restrict__ keys,
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
  hipLaunchKernelGGL((spgemm_emit_kernel<TACC>), dim3(grid_for(n_runs)), dim3(256), 0, st, n_runs, p, keys2,
                     prod, nnz_c_dev, c_idx, c_val);
  hipLaunchKernelGGL(row_ptr_from_rowkeys_kernel, dim3(grid_for(m + 1)), dim3(256), 0, st, m, p, keys2,
                     nnz_c_dev, c_ptr);
  GCG_HIP_CHECK(hipGetLastError());
  GCG_HIP_CHECK(hipStreamSynchronize(st));  // temporaries are freed stream-ordered on return
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
