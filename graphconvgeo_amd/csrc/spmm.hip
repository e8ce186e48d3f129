// spmm.hip -- MI355X (gfx950 / CDNA4) CSR x dense SpMM for the graphconvgeo GCN hot path.
//
// Implements the SpMM part of include/gcg_spmm.h. The reference computes Y = act(H . Z + b) with
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

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

#include "common.h"

using namespace gcg;

#ifndef GCG_SPMM_IDX_PREFETCH
#define GCG_SPMM_IDX_PREFETCH 1
#endif

namespace {

constexpr int kPanelMax = 512;  // floats per column panel
constexpr int64_t kDefaultTaskNnz = 512;
constexpr int64_t kRowCost = 2;  // planner: per-row overhead in nonzero-equivalents

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

// Non-temporal load: the gather hint's cold columns (HC = 1, gcg_spmm_csr_f32_planned_hint).
template <int VEC>
__device__ __forceinline__ Vec<VEC> load_vec_nt(const float* __restrict__ p) {
  Vec<VEC> r;
  if constexpr (VEC == 4) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    r.x[0] = t[0]; r.x[1] = t[1]; r.x[2] = t[2]; r.x[3] = t[3];
  } else {
#pragma unroll
    for (int q = 0; q < VEC; ++q) r.x[q] = __builtin_nontemporal_load(p + q);
  }
  return r;
}

// Round 5: the dwordx4 output rows are stored non-temporal -- Y is written once and read by
// the next kernel long after L2 has turned over, and the default policy let it evict the gather
// hint's hot Z rows: World power-law 6.19-6.25 -> 6.15-6.18 ms, uniform 9.20-9.21 -> 9.13-9.16,
// the Twitter-US step's SpMMs -0.5..-1.3 % (profiles/r05/spmm_nontemporal_y.jsonl). Round 2
// measured the same change neutral, before the gather hint kept a hot set in L2.
template <int VEC>
__device__ __forceinline__ void store_vec(float* __restrict__ p, const Vec<VEC>& v) {
  if constexpr (VEC == 4) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{v.x[0], v.x[1], v.x[2], v.x[3]}, reinterpret_cast<f4v*>(p));
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

// Rectify gate of a pre-activation x: Theano's relu(x) = 0.5*(x + |x|) has the gradient
// 0.5*g*(1 + sgn(x)) (mlpconv.py:77 via lasagne rectify), i.e. g, g/2 or 0 for x > 0, x == 0,
// x < 0. The byte keeps 2 * that factor: 2, 1, 0 (NaN -> 0). Read by gcg_relu_backward_gate_f32.
__device__ __forceinline__ uint32_t gate_code(float x) {
  return x > 0.0f ? 2u : (x == 0.0f ? 1u : 0u);
}

template <int VEC>
__device__ __forceinline__ void store_gate(uint8_t* __restrict__ p, const Vec<VEC>& v) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<uint32_t*>(p) = gate_code(v.x[0]) | (gate_code(v.x[1]) << 8) |
                                      (gate_code(v.x[2]) << 16) | (gate_code(v.x[3]) << 24);
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<uint16_t*>(p) =
        static_cast<uint16_t>(gate_code(v.x[0]) | (gate_code(v.x[1]) << 8));
  } else {
    *p = static_cast<uint8_t>(gate_code(v.x[0]));
  }
}

// Masked last vector (round 4, TL = 1): a width K that is not a multiple of VEC still runs the
// VEC-wide gathers when Z's rows are padded to a multiple of VEC (empty_dense: K = 930 -> 932
// floats). The last vector of a row reads Z's padding columns [K, roundVEC(K)) -- products
// that are never stored -- while bias loads, Y stores and gate bytes past K are masked.
// Full vectors (c + VEC <= K) take the plain path; TL = 0 compiles exactly the old code.
template <int VEC, int TL>
__device__ __forceinline__ Vec<VEC> load_bias(const float* __restrict__ b, int c, int K) {
  if (!TL || c + VEC <= K) return load_vec<VEC>(b + c);
  Vec<VEC> r;
#pragma unroll
  for (int q = 0; q < VEC; ++q) r.x[q] = c + q < K ? b[c + q] : 0.0f;
  return r;
}

template <int VEC, int TL>
__device__ __forceinline__ void store_out(float* __restrict__ yrow, int c, int K,
                                          const Vec<VEC>& v) {
  if (!TL || c + VEC <= K) {
    store_vec<VEC>(yrow + c, v);
    return;
  }
#pragma unroll
  for (int q = 0; q < VEC; ++q)
    if (c + q < K) yrow[c + q] = v.x[q];
}

template <int VEC, int TL>
__device__ __forceinline__ void store_gate_t(uint8_t* __restrict__ grow, int c, int K,
                                             const Vec<VEC>& v) {
  if (!TL || c + VEC <= K) return store_gate<VEC>(grow + c, v);
#pragma unroll
  for (int q = 0; q < VEC; ++q)
    if (c + q < K) grow[c + q] = static_cast<uint8_t>(gate_code(v.x[q]));
}

// Accumulate nonzeros [s, e) of one row into acc, storage order, U gathers in flight.
template <int VEC, int NCH, int U, int HC = 0>
__device__ __forceinline__ void accumulate_range(int s, int e, const int32_t* __restrict__ indices,
                                                 const float* __restrict__ vals,
                                                 const float* __restrict__ Z, int64_t ldz,
                                                 const int (&col)[NCH], Vec<VEC> (&acc)[NCH]) {
  // `col` is pre-clamped for lanes past K (they re-read a column of the same row, which
  // coalesces with lane 0's line): no exec-mask branches, so hipcc can count vmcnt.
  int j = s;
#if GCG_SPMM_IDX_PREFETCH
  // software-pipelined (col, val) stream: the next batch's scalar loads are issued after this
  // batch's gathers, from a clamped base (always inside the row), so they land while the
  // gathers are in flight
  int cn[U];
  float vn[U];
  if (j + U <= e) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cn[u] = indices[j + u];
      vn[u] = vals[j + u];
    }
  }
#endif
  for (; j + U <= e; j += U) {
    int c[U];
    float v[U];
#if GCG_SPMM_IDX_PREFETCH
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = cn[u];
      v[u] = vn[u];
    }
#else
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = indices[j + u];
      v[u] = vals[j + u];
    }
#endif
    Vec<VEC> z[U][NCH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (HC) {  // gather hint: sign bit = cold column -> non-temporal gather
        const float* zrow = Z + static_cast<int64_t>(c[u] & 0x7fffffff) * ldz;
        if (c[u] < 0) {
#pragma unroll
          for (int k = 0; k < NCH; ++k) z[u][k] = load_vec_nt<VEC>(zrow + col[k]);
        } else {
#pragma unroll
          for (int k = 0; k < NCH; ++k) z[u][k] = load_vec<VEC>(zrow + col[k]);
        }
      } else {
        const float* zrow = Z + static_cast<int64_t>(c[u]) * ldz;
#pragma unroll
        for (int k = 0; k < NCH; ++k)
          z[u][k] = load_vec<VEC>(zrow + col[k]);
      }
    }
#if GCG_SPMM_IDX_PREFETCH
    {
      const int jn = min(j + U, e - U);  // in-row base; unused when no full batch follows
#pragma unroll
      for (int u = 0; u < U; ++u) {
        cn[u] = indices[jn + u];
        vn[u] = vals[jn + u];
      }
    }
#endif
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
        const float* zrow = Z + static_cast<int64_t>(HC ? (c[u] & 0x7fffffff) : c[u]) * ldz;
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

// Narrow rows (round 3): K <= 256 / SUB floats, so a row needs only 64 / SUB lanes and a wave
// accumulates SUB rows at once, one lane group per row (the whole-wave loop above would leave
// 3/4 of the lanes idle at K = 64). Each group walks its own row [s, e) in storage order; the
// (col, val) pairs are per-lane vector loads (one address per group), U gathers in flight, the
// next batch's pairs loaded behind this batch's gathers. The wave runs to its longest row
// (mlen, wave-uniform); a group past its row end loads row 0 / column 0 (valid addresses) and
// keeps its sum by a select, so every row's additions are exactly the single-row sequence.
template <int U>
__device__ __forceinline__ void accumulate_sub(int s, int e, int mlen,
                                               const int32_t* __restrict__ indices,
                                               const float* __restrict__ vals,
                                               const float* __restrict__ Z, int64_t ldz, int gcol,
                                               Vec<4>& acc) {
  int cn[U];
  float vn[U];
  auto load_idx = [&](int j0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = s + j0 + u;
      const int ix = idx < e ? idx : 0;
      cn[u] = indices[ix];
      vn[u] = vals[ix];
    }
  };
  if (mlen > 0) load_idx(0);
  for (int j = 0; j < mlen; j += U) {
    int c[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = cn[u];
      v[u] = vn[u];
    }
    Vec<4> z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) z[u] = load_vec<4>(Z + static_cast<int64_t>(c[u]) * ldz + gcol);
    if (j + U < mlen) load_idx(j + U);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = s + j + u < e;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float t = acc.x[q] + v[u] * z[u].x[q];
        acc.x[q] = ok ? t : acc.x[q];
      }
    }
  }
}

// Barrier for LDS hand-over between the waves of a workgroup: retires this wave's LDS
// operations only (the gathers stay in flight across it), then s_barrier.
__device__ __forceinline__ void lds_handover_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One long row of the bitwise 'ordered' mode, by a whole workgroup (round 3). A hub row of a
// power-law graph on a single wave is bound by that wave's U gathers in flight (~12k nonzeros
// take ~1.5 ms, longer than a whole 8-way row block's SpMM). Here the WPB waves gather WPB x U
// consecutive nonzeros per batch -- WPB times the row bytes in flight -- and the storage-order
// sum is handed from wave to wave: wave w adds its U products (nonzeros w*U .. w*U+U-1 of the
// batch) to the running row sum in LDS, in order, then wave w+1 continues. Every addition is
// the one the single-wave loop makes, in the same order: bitwise equal (scipy csr_matvecs).
// A wave issues its next batch's gathers right after its own hand-over, so they fly while the
// later waves of this batch add. LDS: one row sum (<= 512 floats).
//
template <int VEC, int NCH, int U, int WPB, int HC = 0, int TL = 0>
__device__ __forceinline__ void coop_row(int p, const int32_t* __restrict__ indptr,
                                         const int32_t* __restrict__ indices,
                                         const float* __restrict__ vals,
                                         const int32_t* __restrict__ out_rows,
                                         const float* __restrict__ Z, int64_t ldz,
                                         const int (&col)[NCH], const int (&gcol)[NCH],
                                         const bool (&on)[NCH], int K, float* __restrict__ Y,
                                         int64_t ldy, const float* __restrict__ bias, int act,
                                         uint8_t* __restrict__ gate, int64_t ldgate,
                                         float* __restrict__ sacc) {
  const int wave = uniform(static_cast<int>(threadIdx.x >> 6));
  const int lane = threadIdx.x & (kWave - 1);
  const int r = out_rows ? uniform(out_rows[p]) : p;
  const int s = uniform(indptr[r]);
  const int e = uniform(indptr[r + 1]);
  constexpr int B = WPB * U;  // nonzeros per batch
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int q = 0; q < VEC; ++q) sacc[(k * kWave + lane) * VEC + q] = 0.0f;
  }
  // (col, val) of this wave's nonzeros of a batch: one VECTOR load per wave (lane u holds
  // nonzero u, indices clamped into the row -- coop rows are never empty), prefetched one batch
  // ahead and moved to SGPRs with readlane when the batch is gathered. (Scalar-loaded pairs,
  // as in accumulate_range, spill to VGPR lanes here -- 160 SGPRs -- and every spill waits for
  // its s_load: one scalar-load latency per hand-over stage, 5.7 us per batch.)
  int c[U];
  float v[U];
  Vec<VEC> z[U][NCH];
  static_assert(U <= kWave, "one lane per nonzero of a wave's batch");
  const int lu = min(lane, U - 1);
  auto load_idx = [&](int j0, int& ci, float& vi) {
    const int jj = min(j0 + lu, e - 1);
    ci = indices[jj];
    vi = vals[jj];
  };
  auto gather = [&](int ci, float vi) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = __builtin_amdgcn_readlane(ci, u);
      if constexpr (HC) c[u] &= 0x7fffffff;  // the gather hint's cold-column bit
      v[u] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vi), u));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* zrow = Z + static_cast<int64_t>(c[u]) * ldz;
#pragma unroll
      for (int k = 0; k < NCH; ++k) z[u][k] = load_vec<VEC>(zrow + gcol[k]);
    }
  };
  // products v * z formed in place (z <- v * z, rounded as in acc + v * z), then added in
  // storage order; both as packed f32 ops where VEC allows (v_pk_mul_f32 / v_pk_add_f32: half
  // the VALU issue of a hand-over stage, which the waves of a batch take in turn)
  auto multiply = [&]() {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < NCH; ++k)
#pragma unroll
        for (int q = 0; q < VEC; ++q) z[u][k].x[q] = v[u] * z[u][k].x[q];
  };
  auto add = [&](Vec<VEC>& a, const Vec<VEC>& t) {
    if constexpr (VEC % 2 == 0) {  // packed f32 adds (v_pk_add_f32), each lane rounded alone
      typedef float f2v __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int q = 0; q < VEC; q += 2) {
        f2v x = {a.x[q], a.x[q + 1]};
        const f2v y = {t.x[q], t.x[q + 1]};
        x = x + y;
        a.x[q] = x[0];
        a.x[q + 1] = x[1];
      }
    } else {
#pragma unroll
      for (int q = 0; q < VEC; ++q) a.x[q] = a.x[q] + t.x[q];
    }
  };
  int ci, cin;
  float vi, vin;
  load_idx(s + wave * U, ci, vi);
  gather(ci, vi);
  load_idx(s + B + wave * U, cin, vin);
  lds_handover_barrier();
  for (int b = s; b < e; b += B) {
    for (int st = 0; st < WPB; ++st) {
      if (st == wave) {
        const int n = min(U, max(0, e - (b + wave * U)));  // this wave's nonzeros, uniform
        Vec<VEC> acc[NCH];
#pragma unroll
        for (int k = 0; k < NCH; ++k)
          acc[k] = *reinterpret_cast<const Vec<VEC>*>(sacc + (k * kWave + lane) * VEC);
        multiply();
        if (n == U) {
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < NCH; ++k) add(acc[k], z[u][k]);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (u < n)
#pragma unroll
              for (int k = 0; k < NCH; ++k) add(acc[k], z[u][k]);
        }
#pragma unroll
        for (int k = 0; k < NCH; ++k)
          *reinterpret_cast<Vec<VEC>*>(sacc + (k * kWave + lane) * VEC) = acc[k];
        // the next batch's gathers fly while the later waves of this batch add
        gather(cin, vin);
        load_idx(b + 2 * B + wave * U, cin, vin);
      }
      lds_handover_barrier();
    }
  }
  if (wave != 0) return;
  float* yrow = Y + static_cast<int64_t>(p) * ldy;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    if (!on[k]) continue;
    Vec<VEC> a = *reinterpret_cast<const Vec<VEC>*>(sacc + (k * kWave + lane) * VEC);
    if (bias != nullptr) {
      const Vec<VEC> bv = load_bias<VEC, TL>(bias, col[k], K);
#pragma unroll
      for (int q = 0; q < VEC; ++q) a.x[q] = a.x[q] + bv.x[q];
    }
    if (gate != nullptr) store_gate_t<VEC, TL>(gate + static_cast<int64_t>(p) * ldgate, col[k], K, a);
#pragma unroll
    for (int q = 0; q < VEC; ++q) a.x[q] = apply_act(a.x[q], act);
    store_out<VEC, TL>(yrow, col[k], K, a);
  }
}

// Column-sliced hub rows (round 5). One CU's ordered sum of a hub row is bound by the rows it
// has in flight (~19 GB/s for 1216-B random rows: 0.66 ms for a 12k-nonzero row of a P = 8
// World block, longer than the rest of that block's launch). The columns are independent, so
// a row of a two-chunk launch (NCH = 2) is cut into two column slices, each a whole-workgroup
// task on its own CU that runs coop_sum over ALL the row's nonzeros for its half of the
// columns: every column's additions are the single-wave loop's, in storage order (bitwise).
// Half the floats per gathered row let a wave keep twice the rows in flight (coop_row over one
// chunk with 2U rows per batch, the same registers), so each slice streams its row in ~0.6
// the time. (A chained design -- row chunks on several CUs handing the running sum over
// through a flag -- was built and measured first: 1.66 ms for the P = 8 block vs 1.04
// whole-row, its phase that adds stored products being as latency-bound as the gather;
// profiles/HISTORY.md §1.1.) Task {position, slice, -4, slices}. Launches of one chunk (NCH = 1: K <= 256
// at dwordx4) gain nothing from a slice, and the wider-chunk dword / dwordx2 launches (rows
// whose stride is not a multiple of 4 floats) are not cut: slice 0 runs the whole row, the
// others exit. Compiled only into the SLC = 1 kernels, which run plans with cut rows: inlined
// beside the bulk path, its deeper batch changes that path's register allocation (the K = 300
// kernel's row tasks: X.W1 on Twitter-US 1.71 -> 2.08 ms with no cut row in the launch).
template <int VEC, int NCH, int U, int WPB, int HC = 0, int TL = 0>
__device__ __forceinline__ void coop_slice(int p, int sl, int n_sl,
                                           const int32_t* __restrict__ indptr,
                                           const int32_t* __restrict__ indices,
                                           const float* __restrict__ vals,
                                           const int32_t* __restrict__ out_rows,
                                           const float* __restrict__ Z, int64_t ldz,
                                           const int (&col)[NCH], const int (&gcol)[NCH],
                                           const bool (&on)[NCH], int K, float* __restrict__ Y,
                                           int64_t ldy, const float* __restrict__ bias, int act,
                                           uint8_t* __restrict__ gate, int64_t ldgate,
                                           float* __restrict__ sacc) {
  if constexpr (NCH != 2) {
    if (sl == 0)
      coop_row<VEC, NCH, U, WPB, HC, TL>(p, indptr, indices, vals, out_rows, Z, ldz, col, gcol,
                                         on, K, Y, ldy, bias, act, gate, ldgate, sacc);
  } else {
    constexpr int US = 2 * U > kWave ? kWave : 2 * U;  // rows in flight per wave: one chunk
    const int lane = threadIdx.x & (kWave - 1);
    const int panel0 = static_cast<int>(blockIdx.y) * (kWave * VEC * NCH);
    const int wp = min(kWave * VEC * NCH, K - panel0);  // panel width (floats)
    const int ws = min(kWave * VEC, ((wp + n_sl - 1) / n_sl + VEC - 1) / VEC * VEC);
    const int c0 = panel0 + sl * ws;
    const int c1 = min(c0 + ws, panel0 + wp);
    if (c0 >= c1) return;  // an empty slice (narrow last panel)
    int scol[1], sgcol[1];
    bool son[1];
    scol[0] = c0 + lane * VEC;
    son[0] = scol[0] < c1;
    sgcol[0] = son[0] ? scol[0] : c0;
    coop_row<VEC, 1, US, WPB, HC, TL>(p, indptr, indices, vals, out_rows, Z, ldz, scol, sgcol,
                                      son, K, Y, ldy, bias, act, gate, ldgate, sacc);
  }
}

// Main kernel. One wave per task; grid.y = column panel.
//   tasks == nullptr : task w = rows of positions [w, w+1)           (plan-less path)
//   task.w <  0      : rows of positions [task.x, task.y)            (short rows)
//   task.w >= 0      : position task.x, nonzeros [task.y, task.z) -> workspace slot task.w
// The first n_coop tasks ('ordered' long rows, longest first) take a whole workgroup each
// (coop_row); the other tasks one wave each, in the blocks after them.
template <int VEC, int NCH, int U, int WPB = kWavesPerBlock, int SUB = 1, int HC = 0, int TL = 0,
          int SLC = 0>
__global__ __launch_bounds__(kWave * WPB) void spmm_rows_kernel(
    const int4* __restrict__ tasks, int n_tasks, int n_coop, int n_out,
    const int32_t* __restrict__ indptr,
    const int32_t* __restrict__ indices, const float* __restrict__ vals,
    const int32_t* __restrict__ out_rows, const float* __restrict__ Z, int64_t ldz, int K,
    float* __restrict__ Y, int64_t ldy, const float* __restrict__ bias, int act,
    float* __restrict__ ws, int64_t ldws, uint8_t* __restrict__ gate, int64_t ldgate) {
  // (An XCD-aware block -> task mapping was measured and not kept: a random gather has no
  // per-XCD locality, and it breaks the longest-first task order; profiles/HISTORY.md §1.1.)
  const int blk = static_cast<int>(blockIdx.x);
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
  if (blk < n_coop) {  // a whole-workgroup long row or slice of one (uniform across the block)
    __shared__ __attribute__((aligned(16))) float sacc[kWave * VEC * NCH];
    const int4 t0 = tasks[blk];
    if constexpr (SLC) {
      if (uniform(t0.z) == -4) {  // {position, slice, -4, slices}
        coop_slice<VEC, NCH, U, WPB, HC, TL>(uniform(t0.x), uniform(t0.y), uniform(t0.w), indptr,
                                             indices, vals, out_rows, Z, ldz, col, gcol, on, K, Y,
                                             ldy, bias, act, gate, ldgate, sacc);
        return;
      }
    } else {
      // a sliced plan launched on a kernel without slices (a narrower K or a dword / dwordx2
      // gather): slice 0 runs the whole row, the others exit (both used to run it)
      if (uniform(t0.z) == -4 && uniform(t0.y) != 0) return;
    }
    coop_row<VEC, NCH, U, WPB, HC, TL>(uniform(t0.x), indptr, indices, vals, out_rows, Z,
                                       ldz, col, gcol, on, K, Y, ldy, bias, act, gate, ldgate,
                                       sacc);
    return;
  }
  const int w = uniform(n_coop + (blk - n_coop) * WPB + (threadIdx.x >> 6));
  if (w >= n_tasks) return;

  int4 t;
  if (tasks != nullptr) {
    t = tasks[w];
    t.x = uniform(t.x); t.y = uniform(t.y); t.z = uniform(t.z); t.w = uniform(t.w);
  } else {  // plan-less: SUB consecutive rows per wave
    t = make_int4(w * SUB, min(w * SUB + SUB, n_out), -1, -1);
  }

  Vec<VEC> acc[NCH];
  if (t.w >= 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[k].x[q] = 0.0f;
    accumulate_range<VEC, NCH, U, HC>(t.y, t.z, indices, vals, Z, ldz, gcol, acc);
    float* dst = ws + static_cast<int64_t>(t.w) * ldws;
#pragma unroll
    for (int k = 0; k < NCH; ++k)
      if (on[k]) store_vec<VEC>(dst + col[k], acc[k]);
    return;
  }

  if constexpr (SUB > 1) {
    static_assert(VEC == 4 && NCH == 1, "narrow rows: one dwordx4 per lane");
    constexpr int LG = kWave / SUB;  // lanes per row
    const int g = lane / LG;
    const int scol = (lane % LG) * 4;  // one panel: K <= 4 * LG
    const bool son = scol < K;
    const int sgcol = son ? scol : 0;
    Vec<4> sbv;
#pragma unroll
    for (int q = 0; q < 4; ++q) sbv.x[q] = 0.0f;
    if (bias != nullptr) sbv = load_bias<4, TL>(bias, sgcol, K);
    for (int pb = t.x; pb < t.y; pb += SUB) {
      const int p = pb + g;
      const bool live = p < t.y;
      const int pp = live ? p : t.x;
      const int r = out_rows ? out_rows[pp] : pp;
      const int rs = indptr[r];
      const int re = live ? indptr[r + 1] : rs;
      int mlen = re - rs;  // the longest of the wave's SUB rows (every group's first lane)
#pragma unroll
      for (int o = LG; o < kWave; o <<= 1) mlen = max(mlen, __shfl_xor(mlen, o, kWave));
      mlen = uniform(mlen);
      Vec<4> acc;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc.x[q] = 0.0f;
      accumulate_sub<U>(rs, re, mlen, indices, vals, Z, ldz, sgcol, acc);
      if (!(live && son)) continue;
      if (bias != nullptr) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc.x[q] = acc.x[q] + sbv.x[q];
      }
      if (gate != nullptr) store_gate_t<4, TL>(gate + static_cast<int64_t>(p) * ldgate, scol, K, acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc.x[q] = apply_act(acc.x[q], act);
      store_out<4, TL>(Y + static_cast<int64_t>(p) * ldy, scol, K, acc);
    }
    return;
  }

  // The bias depends on the column only: loaded once per wave, before the row loop. (Loaded
  // after each row's gathers it was a dependent global load per row: +8 % on Twitter-US
  // H.Z1 + b1, +5 % at World.)
  Vec<VEC> bv[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    if (bias != nullptr) {
      bv[k] = load_bias<VEC, TL>(bias, gcol[k], K);
    } else {
#pragma unroll
      for (int q = 0; q < VEC; ++q) bv[k].x[q] = 0.0f;
    }
  }

  for (int p = t.x; p < t.y; ++p) {
    const int r = out_rows ? uniform(out_rows[p]) : p;
    const int s = uniform(indptr[r]);
    const int e = uniform(indptr[r + 1]);
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[k].x[q] = 0.0f;
    accumulate_range<VEC, NCH, U, HC>(s, e, indices, vals, Z, ldz, gcol, acc);
    float* yrow = Y + static_cast<int64_t>(p) * ldy;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (!on[k]) continue;
      if (bias != nullptr) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[k].x[q] = acc[k].x[q] + bv[k].x[q];
      }
      if (gate != nullptr)
        store_gate_t<VEC, TL>(gate + static_cast<int64_t>(p) * ldgate, col[k], K, acc[k]);
#pragma unroll
      for (int q = 0; q < VEC; ++q) acc[k].x[q] = apply_act(acc[k].x[q], act);
      store_out<VEC, TL>(yrow, col[k], K, acc[k]);
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
                                                            int act, uint8_t* __restrict__ gate,
                                                            int64_t ldgate) {
  const int w = uniform(static_cast<int>(blockIdx.x) * kWavesPerBlock + (threadIdx.x >> 6));
  if (w >= n_long) return;
  const int c = static_cast<int>(blockIdx.y) * kWave + (threadIdx.x & (kWave - 1));
  if (c >= K) return;
  const int4 L = longs[w];
  const float* src = ws + static_cast<int64_t>(L.y) * ldws + c;
  float acc = src[0];
  for (int s = 1; s < L.z; ++s) acc = acc + src[static_cast<int64_t>(s) * ldws];
  if (bias != nullptr) acc = acc + bias[c];
  if (gate != nullptr) gate[static_cast<int64_t>(L.x) * ldgate + c] = static_cast<uint8_t>(gate_code(acc));
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
  uint8_t* gate = nullptr;  // rectify gate bytes (nullable), row stride ldgate
  int64_t ldgate = 0;
  int n_coop = 0;  // leading tasks run by a whole workgroup each (ordered long rows)
  // gather hint: the column indices with a cold-column sign bit (nullable); used by the
  // dwordx4 launches (NCH 1 and 2), every other launch reads `indices`
  const int32_t* hint = nullptr;
  // K % VEC != 0 on VEC-padded rows: the last vector of a row is masked (TL = 1 kernels)
  int tail = 0;
  // the plan cuts rows into column slices (coop_slice): the SLC = 1 kernels
  int sliced = 0;
};

template <int VEC, int NCH, int U, int WPB, int SUB = 1, int HC = 0>
void launch_rows_u(const LaunchArgs& a, int n_panels, hipStream_t stream) {
  // plan-less: one wave per SUB consecutive rows
  const int n_tasks = a.tasks == nullptr ? (a.n_tasks + SUB - 1) / SUB : a.n_tasks;
  const dim3 grid(a.n_coop + (n_tasks - a.n_coop + WPB - 1) / WPB, n_panels);
  if constexpr (VEC == 4 && NCH == 2 && SUB == 1) {  // column-sliced hub rows
    if (a.sliced) {
      if (a.tail)
        hipLaunchKernelGGL((spmm_rows_kernel<VEC, NCH, U, WPB, SUB, HC, 1, 1>), grid,
                           dim3(kWave * WPB), 0, stream, a.tasks, n_tasks, a.n_coop, a.n_tasks,
                           a.indptr, a.indices, a.vals, a.out_rows, a.Z, a.ldz, a.K, a.Y, a.ldy,
                           a.bias, a.act, a.ws, a.ldws, a.gate, a.ldgate);
      else
        hipLaunchKernelGGL((spmm_rows_kernel<VEC, NCH, U, WPB, SUB, HC, 0, 1>), grid,
                           dim3(kWave * WPB), 0, stream, a.tasks, n_tasks, a.n_coop, a.n_tasks,
                           a.indptr, a.indices, a.vals, a.out_rows, a.Z, a.ldz, a.K, a.Y, a.ldy,
                           a.bias, a.act, a.ws, a.ldws, a.gate, a.ldgate);
      return;
    }
  }
  if constexpr (VEC == 4) {
    if (a.tail) {
      hipLaunchKernelGGL((spmm_rows_kernel<VEC, NCH, U, WPB, SUB, HC, 1>), grid, dim3(kWave * WPB),
                         0, stream, a.tasks, n_tasks, a.n_coop, a.n_tasks, a.indptr, a.indices,
                         a.vals, a.out_rows, a.Z, a.ldz, a.K, a.Y, a.ldy, a.bias, a.act, a.ws,
                         a.ldws, a.gate, a.ldgate);
      return;
    }
  }
  hipLaunchKernelGGL((spmm_rows_kernel<VEC, NCH, U, WPB, SUB, HC>), grid, dim3(kWave * WPB), 0, stream,
                     a.tasks, n_tasks, a.n_coop, a.n_tasks, a.indptr, a.indices, a.vals, a.out_rows,
                     a.Z, a.ldz, a.K, a.Y, a.ldy, a.bias, a.act, a.ws, a.ldws, a.gate,
                     a.ldgate);
}

// Gathers in flight per lane: INFLIGHT floats of Z per lane per batch (U = INFLIGHT/(VEC*NCH)
// nonzeros). Measured (MI355X, same box, K = 300 variant VEC = 4 / NCH = 2): 192 floats
// (U = 24, 210 VGPRs, 2 waves/SIMD) vs 64 (U = 8, 92 VGPRs, 5 waves/SIMD): Twitter-World
// power-law 6.67 vs 6.97 ms, Twitter-US 1.70 vs 1.81 ms, uniform equal; but slower on the
// small GEOTEXT graph (32-nnz tasks: 39 vs 26 us) and for the narrower variants (K = 64, 128,
// 129). 256 floats (U = 32) drops to 1 wave/SIMD and halves throughput. So the deep batch is
// used for the VEC 4 x 2 variant with >= 256-nnz tasks only.
template <int VEC, int NCH, int INFLIGHT>
void launch_rows_f(const LaunchArgs& a, int n_panels, hipStream_t stream) {
  constexpr int U0 = INFLIGHT / (VEC * NCH);
  constexpr int U = U0 > 24 ? 24 : (U0 < 2 ? 2 : U0);
  launch_rows_u<VEC, NCH, U, kWavesPerBlock>(a, n_panels, stream);
}

template <int VEC, int NCH>
void launch_rows(const LaunchArgs& a, int n_panels, hipStream_t stream) {
  if constexpr (VEC == 4 && NCH == 1) {
    // Narrow rows, plan-less (rowwise) only: 4 rows per wave at K <= 64, 2 at K <= 96. The wave
    // runs to its longest row, so this pays where rows are alike -- 'auto' takes rowwise only
    // on hub-free graphs -- and loses on a planned power-law task (ordered, World: K = 96 2.08
    // -> 2.54 ms) and at K = 128 (3.09 -> 3.20); World uniform: K = 16 / 32 / 64 1.93 / 1.94 /
    // 2.19 -> 0.91 / 0.93 / 1.48 ms, K = 96 2.50 -> 2.39 (tools/exp_spmm_narrow.py).
    if (a.hint != nullptr) {  // gather hint (planned only)
      LaunchArgs h = a;
      h.indices = a.hint;
      return launch_rows_u<4, 1, 16, kWavesPerBlock, 1, 1>(h, n_panels, stream);
    }
    if (a.tasks == nullptr && a.K <= 64) return launch_rows_u<4, 1, 16, kWavesPerBlock, 4>(a, n_panels, stream);
    if (a.tasks == nullptr && a.K <= 96) return launch_rows_u<4, 1, 16, kWavesPerBlock, 2>(a, n_panels, stream);
  }
  if constexpr (VEC == 4 && NCH == 2) {
    // planned tasks of >= 256 nnz: U = 16 since the (col, val) stream is software-pipelined
    // (late round 2): 163 VGPRs / 3 waves per SIMD and fewer SGPR spills than U = 24 (222 VGPRs,
    // 2 waves): World power-law 6.60 vs 6.71 ms (three alternating runs each, one box)
    // gather hint: cold columns' rows gathered non-temporally (gcg_spmm_csr_f32_planned_hint)
    if (a.hint != nullptr) {
      LaunchArgs h = a;
      h.indices = a.hint;
      return launch_rows_u<4, 2, 16, kWavesPerBlock, 1, 1>(h, n_panels, stream);
    }
    if (a.task_nnz >= 256) return launch_rows_u<4, 2, 16, kWavesPerBlock>(a, n_panels, stream);
    // plan-less, one row per wave, on a large graph (sparse.resolve_auto picks it for graphs
    // without hub rows): U = 16, 3 waves/SIMD -- Twitter-World uniform 9.35-9.36 vs 9.41-9.44 ms
    // at U = 8 (two boxes)
    if (a.tasks == nullptr && a.n_tasks >= 65536)
      return launch_rows_u<4, 2, 16, kWavesPerBlock>(a, n_panels, stream);
  }
  launch_rows_f<VEC, NCH, 64>(a, n_panels, stream);
}

// Vector width of the gathers. K % 4 != 0 on rows padded to a multiple of 4 floats (ldz % 4 == 0
// implies ldz >= round4(K): the last vector's padding columns are inside the row) runs dwordx4
// with a masked last vector (*tail = 1) instead of dwordx2 / dword gathers. Measured before
// (profiles/r03/spmm_k_odd.jsonl, World): C = 930 uniform 29.6 ms as dwordx2 vs 26.5 ms for the
// 932-wide dwordx4 product on the same rows. (Operands whose row stride is not a multiple of 4
// floats still gather dwordx2 / dword vectors: the same products, bitwise.)
int pick_vec(const float* Z, int64_t ldz, const float* Y, int64_t ldy, int64_t K,
             const float* bias, const float* ws, int64_t ldws, int* tail) {
  *tail = 0;
  for (int vec : {4, 2}) {
    const size_t bytes = sizeof(float) * vec;
    if (ldz % vec == 0 && ldy % vec == 0 && aligned(Z, bytes) && aligned(Y, bytes) &&
        (bias == nullptr || aligned(bias, bytes)) &&
        (ws == nullptr || (aligned(ws, bytes) && ldws % vec == 0))) {
      if (K % vec == 0) return vec;
      if (vec == 4) {
        *tail = 1;
        return 4;
      }
    }
  }
  return 1;
}

// Panel width (floats): up to kPanelMax per launch column (grid.y for the rest).
gcg_status launch_spmm(const LaunchArgs& a, int vec, hipStream_t stream) {
  const int64_t K = a.K;
  const int per_chunk = kWave * vec;
  const int nch_max = kPanelMax / per_chunk;
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
  // grid.y of the fix-up kernel is ceil(K / 64) <= 65535
  if (K < 0 || K > int64_t{65535} * kWave) return fail(GCG_ERR_INVALID_ARG, "bad K=%lld", (long long)K);
  if (K > 0 && (Z == nullptr || Y == nullptr)) return fail(GCG_ERR_INVALID_ARG, "Z or Y is NULL");
  if (ldz < K || ldy < K) return fail(GCG_ERR_INVALID_ARG, "ldz=%lld / ldy=%lld < K=%lld",
                                      (long long)ldz, (long long)ldy, (long long)K);
  if (!aligned(Z, 4) || !aligned(Y, 4) || (bias && !aligned(bias, 4)))
    return fail(GCG_ERR_MISALIGNED, "Z/Y/bias not 4-byte aligned");
  if (act != GCG_ACT_NONE && act != GCG_ACT_RELU) return fail(GCG_ERR_INVALID_ARG, "bad act=%d", act);
  return GCG_OK;
}

gcg_status check_gate(const uint8_t* gate, int64_t ldgate, int64_t K, int act) {
  if (gate == nullptr) return GCG_OK;
  if (act != GCG_ACT_RELU) return fail(GCG_ERR_INVALID_ARG, "gate needs act = GCG_ACT_RELU");
  if (ldgate < K || ldgate % 4 != 0) return fail(GCG_ERR_INVALID_ARG, "ldgate=%lld: need >= K and %% 4 == 0", (long long)ldgate);
  if (!aligned(gate, 4)) return fail(GCG_ERR_MISALIGNED, "gate not 4-byte aligned");
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
  int64_t n_coop = 0;        // leading whole-workgroup tasks: column slices, then whole rows
  int64_t n_coop_rows = 0;   // rows on whole workgroups (sliced or not)
  int64_t n_sliced = 0;      // ... of which cut into column slices (coop_slice)
};

// Column slices per cut row. A whole-workgroup row is cut (ordered == 1; ordered == 2 keeps
// every row whole) when it is also longer than 1/kSliceDivisor of the plan's nonzeros: where
// one CU's sum of it would outlast the rest of the launch (~55 ns per 1216-B row on one CU vs
// ~5.8 G rows/s for the bulk: rows past ~1/320 of the work). Cutting every whole-workgroup row
// costs throughput -- two half rows fetch ~10 % more lines than one, twice the per-row issue
// -- and a launch of many of them (X^T.g's Zipf-tail features on Twitter-US) ran 1.69 -> 1.98
// ms. World P = 8 blocks cut their ~12k-nonzero hub rows; the whole graph cuts none.
constexpr int kHubSlices = 2;
constexpr int64_t kSliceDivisor = 768;

// 'ordered' rows longer than this many nonzeros run on a whole workgroup (coop_row); shorter
// long rows stay single-wave tasks scheduled first: 8 x task_nnz (1024 with the ordered default task of 128). Measured (World power-law,
// K = 300, slowest of P row blocks, tools/exp_block_modes.py): P = 4 2.12 -> 1.70 ms, P = 8
// 1.59 -> 1.16 ms, P = 1 and 2 unchanged; thresholds 1024 / 2048 / 4096 within noise of each
// other. One hub row alone is bound by its CU (~19 GB/s per CU for 1216-B random rows: 0.77 ms
// for 12,189 nonzeros on 4 waves vs 0.83 on one), so the gain is that hub rows now get a CU
// each instead of sharing one four to a workgroup.
int64_t coop_min_nnz(int64_t task_nnz) { return 8 * task_nnz; }

// Default task size: 512 nonzeros, smaller on small graphs so the launch still has
// >= ~8k waves (256 CUs x 32 waves) to spread; never below 32. Ordered plans (round 5): 128,
// from 32k nonzeros per 1/32768 of the work -- four times the tasks, whole-workgroup rows from
// 1,024 nonzeros, and the U = 8 batch (5 waves per SIMD) of the < 256-nonzero tasks. World
// power-law K = 300, slowest of P row blocks (tools/exp_block_modes.py, one box, ordered at
// 512 / 256 / 128 / 64): P = 1 6.344 / 6.313 / 6.285 / 6.376 ms, P = 4 1.666 / 1.634 / 1.620 /
// 1.636, P = 8 0.919 / 0.854 / 0.822 / 0.821 (`fast` 7.238 / 1.824 / 0.942 on that box): the
// rows of 512..4096 nonzeros no longer run on one wave (up to ~0.5 ms each).
constexpr int64_t kDefaultOrderedTaskNnz = 128;
// ... and 256 for matrices whose rows average >= 256 nonzeros (the W1 gradient's CSR(X^T) tail:
// Twitter-US 11.6M nonzeros over 10k rows, ordered 2.21 ms at 128 vs 2.06 at 256 = `fast`;
// Twitter-World 43.5M over 50k rows 7.86-7.88 either way; profiles/r05/xt_tail_modes.jsonl):
// with 128, every row from 1,024 nonzeros is a whole-workgroup hand-over row, most of such a
// matrix.
constexpr int64_t kLongRowsOrderedTaskNnz = 256;
int64_t default_task_nnz(int64_t nnz, int ordered, int64_t n_rows) {
  const bool long_rows = n_rows > 0 && nnz >= 256 * n_rows;
  const int64_t cap = ordered ? (long_rows ? kLongRowsOrderedTaskNnz : kDefaultOrderedTaskNnz)
                              : kDefaultTaskNnz;
  int64_t w = nnz / (ordered ? 32768 : 8192);
  return w < 32 ? 32 : (w > cap ? cap : w);
}

gcg_status build_host_plan(int64_t n_rows, const int32_t* indptr, const int32_t* out_rows,
                           int64_t n_out, int64_t task_nnz, int ordered, HostPlan* hp) {
  if (task_nnz <= 0) task_nnz = default_task_nnz(indptr[n_rows], ordered, n_rows);
  if (indptr[0] != 0) return fail(GCG_ERR_BAD_CSR, "indptr[0] = %d != 0", indptr[0]);
  for (int64_t r = 0; r < n_rows; ++r)
    if (indptr[r + 1] < indptr[r]) return fail(GCG_ERR_BAD_CSR, "indptr decreases at row %lld", (long long)r);
  hp->tasks.clear();
  hp->longs.clear();
  hp->n_slots = 0;
  hp->max_task_nnz = 0;
  hp->n_coop = 0;
  hp->n_coop_rows = 0;
  hp->n_sliced = 0;
  const int64_t coop_min = coop_min_nnz(task_nnz);
  std::vector<int32_t> seg_tasks;
  std::vector<std::pair<int64_t, int64_t>> long_rows;  // (nnz, position), ordered mode
  std::vector<std::pair<int64_t, int64_t>> coop_rows;  // (nnz, position), ordered mode
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
  int64_t work = 0;  // nonzeros of the output rows
  for (int64_t p = 0; p < n_out; ++p) {
    const int64_t r = out_rows ? out_rows[p] : p;
    if (r < 0 || r >= n_rows) return fail(GCG_ERR_INVALID_ARG, "out_rows[%lld]=%lld out of range", (long long)p, (long long)r);
    work += indptr[r + 1] - indptr[r];
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
      // serial tail of a hub row overlaps the bulk instead of ending the launch; the longest
      // ones on a whole workgroup (coop_row).
      close(p);
      (len > coop_min ? coop_rows : long_rows).push_back({len, p});
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
  auto longest_first = [](const std::pair<int64_t, int64_t>& a,
                          const std::pair<int64_t, int64_t>& b) { return a.first > b.first; };
  std::stable_sort(coop_rows.begin(), coop_rows.end(), longest_first);
  std::stable_sort(long_rows.begin(), long_rows.end(), longest_first);
  std::vector<int32_t> head;
  head.reserve((coop_rows.size() * kHubSlices + long_rows.size()) * 4 + seg_tasks.size());
  // whole-workgroup rows first, longest first: cut into column slices or whole
  const int64_t slice_min = std::max(coop_min, work / kSliceDivisor);
  for (const auto& lr : coop_rows) {
    if (ordered == 1 && lr.first >= slice_min) {
      for (int k = 0; k < kHubSlices; ++k)
        head.insert(head.end(), {int32_t(lr.second), k, -4, kHubSlices});
      ++hp->n_sliced;
    } else {
      head.insert(head.end(), {int32_t(lr.second), int32_t(lr.second + 1), -2, -1});
    }
    hp->max_task_nnz = std::max(hp->max_task_nnz, lr.first);
  }
  hp->n_coop_rows = static_cast<int64_t>(coop_rows.size());
  hp->n_coop = hp->n_coop_rows + hp->n_sliced * (kHubSlices - 1);
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
struct gcg_spmm_plan {
  int64_t n_rows = 0, n_cols = 0, nnz = 0, n_out = 0;
  int ordered = 0;
  int64_t task_nnz = 0;
  int n_tasks = 0, n_long = 0, n_coop = 0, n_coop_rows = 0, n_sliced = 0;
  int64_t n_slots = 0, max_task_nnz = 0;
  int4* tasks = nullptr;     // device
  int4* longs = nullptr;     // device
  int32_t* out_rows = nullptr;  // device copy (nullptr = identity)
};

extern "C" {

gcg_status gcg_spmm_csr_f32(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t* indptr,
                            const int32_t* indices, const float* vals, const float* Z,
                            int64_t ldz, int64_t K, float* Y, int64_t ldy, const float* bias,
                            int act, const int32_t* out_rows, int64_t n_out,
                            gcg_stream_t stream) {
  return gcg_spmm_csr_f32_gate(n_rows, n_cols, nnz, indptr, indices, vals, Z, ldz, K, Y, ldy,
                               bias, act, out_rows, n_out, nullptr, 0, stream);
}

gcg_status gcg_spmm_csr_f32_gate(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                 const int32_t* indptr, const int32_t* indices,
                                 const float* vals, const float* Z, int64_t ldz, int64_t K,
                                 float* Y, int64_t ldy, const float* bias, int act,
                                 const int32_t* out_rows, int64_t n_out, uint8_t* gate,
                                 int64_t ldgate, gcg_stream_t stream) {
  if (n_rows < 0 || n_cols < 0 || nnz < 0 || n_rows > INT32_MAX || nnz > INT32_MAX)
    return fail(GCG_ERR_INVALID_ARG, "bad CSR shape n_rows=%lld n_cols=%lld nnz=%lld",
                (long long)n_rows, (long long)n_cols, (long long)nnz);
  if (out_rows == nullptr) n_out = n_rows;
  if (n_out < 0 || n_out > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "bad n_out=%lld", (long long)n_out);
  if (gcg_status st = check_dense(Z, ldz, Y, ldy, K, bias, act)) return st;
  if (gcg_status st = check_gate(gate, ldgate, K, act)) return st;
  if (n_out > 0 && indptr == nullptr) return fail(GCG_ERR_INVALID_ARG, "indptr is NULL");
  if (nnz > 0 && (indices == nullptr || vals == nullptr)) return fail(GCG_ERR_INVALID_ARG, "indices/vals NULL");
  if (n_out == 0 || K == 0) return GCG_OK;
  LaunchArgs a{nullptr, int(n_out), indptr, indices, vals, out_rows, Z, ldz, int(K), Y, ldy,
               bias, act, nullptr, 0, 0, gate, ldgate};
  const int vec = pick_vec(Z, ldz, Y, ldy, K, bias, nullptr, 0, &a.tail);
  return launch_spmm(a, vec, static_cast<hipStream_t>(stream));
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
  p->ordered = ordered; p->task_nnz = task_nnz > 0 ? task_nnz : default_task_nnz(nnz, ordered, n_rows);
  p->n_tasks = static_cast<int>(hp.tasks.size() / 4);
  p->n_long = static_cast<int>(hp.longs.size() / 4);
  p->n_coop = static_cast<int>(hp.n_coop);
  p->n_coop_rows = static_cast<int>(hp.n_coop_rows);
  p->n_sliced = static_cast<int>(hp.n_sliced);
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
  // One row per split-row segment (fast mode; ordered plans need none).
  const int64_t ldws = (K + 3) & ~int64_t{3};
  *bytes = static_cast<size_t>(plan->n_slots) * ldws * sizeof(float);
  return GCG_OK;
}

gcg_status gcg_spmm_plan_info(const gcg_spmm_plan* plan, int64_t* n_tasks, int64_t* n_long_rows,
                              int64_t* n_segments, int64_t* max_task_nnz) {
  if (plan == nullptr) return fail(GCG_ERR_INVALID_ARG, "plan is NULL");
  if (n_tasks) *n_tasks = plan->n_tasks;
  // split (fast) + whole-workgroup rows (ordered)
  if (n_long_rows) *n_long_rows = plan->n_long + plan->n_coop_rows;
  if (n_segments) *n_segments = plan->n_slots;
  if (max_task_nnz) *max_task_nnz = plan->max_task_nnz;
  return GCG_OK;
}

gcg_status gcg_spmm_plan_hub_rows(const gcg_spmm_plan* plan, int64_t* n_coop_rows,
                                  int64_t* n_sliced_rows, int64_t* n_slices) {
  if (plan == nullptr) return fail(GCG_ERR_INVALID_ARG, "plan is NULL");
  if (n_coop_rows) *n_coop_rows = plan->n_coop_rows;
  if (n_sliced_rows) *n_sliced_rows = plan->n_sliced;
  if (n_slices) *n_slices = kHubSlices;
  return GCG_OK;
}

gcg_status gcg_spmm_csr_f32_planned(const gcg_spmm_plan* plan, const int32_t* indptr,
                                    const int32_t* indices, const float* vals, const float* Z,
                                    int64_t ldz, int64_t K, float* Y, int64_t ldy,
                                    const float* bias, int act, void* workspace,
                                    size_t workspace_bytes, gcg_stream_t stream) {
  return gcg_spmm_csr_f32_planned_gate(plan, indptr, indices, vals, Z, ldz, K, Y, ldy, bias, act,
                                       nullptr, 0, workspace, workspace_bytes, stream);
}

gcg_status gcg_spmm_csr_f32_planned_gate(const gcg_spmm_plan* plan, const int32_t* indptr,
                                         const int32_t* indices, const float* vals,
                                         const float* Z, int64_t ldz, int64_t K, float* Y,
                                         int64_t ldy, const float* bias, int act, uint8_t* gate,
                                         int64_t ldgate, void* workspace,
                                         size_t workspace_bytes, gcg_stream_t stream) {
  return gcg_spmm_csr_f32_planned_hint(plan, indptr, indices, vals, Z, ldz, K, Y, ldy, bias, act,
                                       gate, ldgate, workspace, workspace_bytes, nullptr, stream);
}

gcg_status gcg_spmm_csr_f32_planned_hint(const gcg_spmm_plan* plan, const int32_t* indptr,
                                         const int32_t* indices, const float* vals,
                                         const float* Z, int64_t ldz, int64_t K, float* Y,
                                         int64_t ldy, const float* bias, int act, uint8_t* gate,
                                         int64_t ldgate, void* workspace,
                                         size_t workspace_bytes, const int32_t* gather_hint,
                                         gcg_stream_t stream) {
  if (plan == nullptr) return fail(GCG_ERR_INVALID_ARG, "plan is NULL");
  if (gcg_status st = check_dense(Z, ldz, Y, ldy, K, bias, act)) return st;
  if (gcg_status st = check_gate(gate, ldgate, K, act)) return st;
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
               Y, ldy, bias, act, ws, ldws, plan->task_nnz, gate, ldgate, plan->n_coop,
               gather_hint};
  a.sliced = plan->n_sliced > 0 ? 1 : 0;
  const int vec = pick_vec(Z, ldz, Y, ldy, K, bias, ws, ldws, &a.tail);
  if (gcg_status s = launch_spmm(a, vec, st)) return s;
  if (plan->n_long > 0) {
    const dim3 grid((plan->n_long + kWavesPerBlock - 1) / kWavesPerBlock, (K + kWave - 1) / kWave);
    hipLaunchKernelGGL(spmm_fixup_kernel, grid, dim3(kBlock), 0, st, plan->longs, plan->n_long,
                       ws, ldws, int(K), Y, ldy, bias, act, gate, ldgate);
    GCG_HIP_CHECK(hipGetLastError());
  }
  return GCG_OK;
}

}  // extern "C"
