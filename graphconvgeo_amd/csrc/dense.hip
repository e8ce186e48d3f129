// dense.hip -- the dense side of the GCN output layer on the CDNA4 matrix cores.
//
// Reference (Theano graph, host BLAS):
//   ConvolutionDenseLayer.get_output_for   T.dot(h, W) + b, softmax     mlpconv.py:86-95
//   MLPCONV.fit loss                        categorical_crossentropy(    mlpconv.py:229-230
//                                           softmax(logits), y).mean()
//   Theano grads of both                    (softmax - onehot)/T, g.W^T, h^T.g
//
// Kernels:
//   gemm_kernel<RT, G, WR, WC, EPI>  C = A.B (+ bias, rectify) with v_mfma_f32_16x16x4_f32
//       (exact f32 in / f32 accumulate). EPI = 1 fuses the whole output row: bias, softmax,
//       cross-entropy against int32 labels, first-index argmax, and writes either
//       (softmax - onehot) * scale (the logits gradient) or the probabilities.
//   gemm_bl_kernel<G, WC, EPI>       the same product with B staged through LDS and shared by
//       4 row bands (the plain products' default; see pick_shape).
//   softmax_xent_rows_kernel<NV>     the same row epilogue for logits that already exist
//       (the reference order, where the logits come out of the H SpMM, mlpconv.py:90-94).
//
// Work decomposition (64-wide waves, 4 per workgroup, WR x WC of them):
//   workgroup tile  BM = 16*RT*WR rows  x  BN = 64*G*WC columns
//   wave tile       16*RT rows x 64*G columns = RT x (4G) MFMA 16x16 tiles
// A (rows x K) is staged through LDS in KC-deep chunks (double-buffered through registers),
// shared by the WC waves of a row band. B (K x N, row-major, e.g. W: 1.1 MB at K=300,
// C=930, L2-resident) is read straight into VGPRs: lane (j = l&15, q = l>>4) loads ONE
// dwordx4 B[k][c0 + 4j .. 4j+3] per k-step and uses its 4 floats as the B fragment of 4
// different 16-column tiles (tile e covers columns c0 + 4j + e). The accumulator registers
// then hold 4 adjacent columns per lane for every row -> dwordx4 stores, no shuffles.
// The k order inside a 16-deep step is permuted consistently for A and B (step e uses
// k = k0 + 4q + e), so each lane reads A as one dwordx4 from LDS as well.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <type_traits>

#include "common.h"

using namespace gcg;

namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// f32 products on the bf16 matrix cores ("bf16x6", MX = 1 below): x = x0 + x1 + x2 with each
// plane the round-to-nearest bf16 of what the planes before it left (8 significant bits each,
// |x1| <= 2^-9 |x|, |x2| <= 2^-17 |x|, x - (x0 + x1 + x2) <= 2^-26 |x|). a . b keeps the six
// plane products of order <= 2^-16 -- a0b0, a0b1, a1b0, a0b2, a1b1, a2b0 -- each exact in the
// f32 accumulator; the dropped a1b2 + a2b1 + a2b2 are <= 2^-25 |a||b|, below f32 rounding. NaN
// propagates (through plane 0 and the NaN residuals); an infinite or > 3.39e38 operand gives a
// non-finite tile, which f32_tile below recomputes with f32 products (f32 semantics).
using f8 = __attribute__((ext_vector_type(8))) float;
using bf8 = __attribute__((ext_vector_type(8))) __bf16;

using f2 = __attribute__((ext_vector_type(2))) float;
using bf2 = __attribute__((ext_vector_type(2))) __bf16;
using u4v = __attribute__((ext_vector_type(4))) unsigned;

// one pair: packed bf16 (v_cvt_pk_bf16_f32) and the f32 residual x - bf16(x), unpacked from the
// packed word by a shift / mask instead of a second conversion
__device__ __forceinline__ unsigned split_pair(f2& x) {
  const unsigned p = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf2));
  const f2 h = {__builtin_bit_cast(float, p << 16), __builtin_bit_cast(float, p & 0xffff0000u)};
  x = x - h;
  return p;
}
__device__ __forceinline__ void split3(const f8 x, bf8& h0, bf8& h1, bf8& h2) {
  u4v p0, p1, p2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f2 r = {x[2 * i], x[2 * i + 1]};
    p0[i] = split_pair(r);
    p1[i] = split_pair(r);
    p2[i] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf2));
  }
  h0 = __builtin_bit_cast(bf8, p0);
  h1 = __builtin_bit_cast(bf8, p1);
  h2 = __builtin_bit_cast(bf8, p2);
}
__device__ __forceinline__ f4 mfma_bf(bf8 a, bf8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// The six plane products of one A fragment (planes a[0] a[1] a[2]) and one B fragment (b0 b1
// b2) into c, smallest planes first. A lane's 32-deep fragment holds k = kc0 + 4q + i (low
// half, elements 0-3) and kc0 + 16 + 4q + i (high half). TP = the packed K tail (round 6): a
// chunk with r = K - kc0 <= 16 live k has both fragments' high halves zero, so every MFMA
// carries two plane products instead -- the high half holding another plane of the low half's
// k: a2b0 + a1b1, a0b2 + a1b0, a0b1 + a0b0, 3 MFMAs instead of 6. K = 300 ends in such a chunk
// (12 live k): the projection and the fused layer issue 57 MFMAs per output tile, not 60.
// The A side is packed once per chunk in place (pack_tail_a: the same three registers per
// fragment), the B side per slot. Every bf16x6 kernel packs the same way (bitwise equal).
// Kernels take the packed tail as a template flag the host sets from K, and peel the last
// chunk out of the K loop: a runtime branch between the two MFMA paths inside one kernel
// doubled the register pressure (100s of VGPRs spilled). Measured (one box, three rounds,
// profiles/r06/tail_packed_fence_ab.jsonl): NT projection 191.4 -> 199.0 TF, dP 179.7 ->
// 183.5 TF, fused layer unchanged (its last chunk waits on the weight-plane loads).
__device__ __forceinline__ bf8 lohi(bf8 lo, bf8 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 8, 9, 10, 11);
}
__device__ __forceinline__ void pack_tail_a(bf8 (&a)[3]) {
  const bf8 a0 = a[0], a1 = a[1], a2 = a[2];
  a[0] = lohi(a2, a1);
  a[1] = lohi(a0, a1);
  a[2] = lohi(a0, a0);
}
template <bool TP>
__device__ __forceinline__ f4 mfma6(const bf8 (&a)[3], bf8 b0, bf8 b1, bf8 b2, f4 c) {
  if constexpr (TP) {  // a packed by pack_tail_a
    c = mfma_bf(a[0], lohi(b0, b1), c);
    c = mfma_bf(a[1], lohi(b2, b0), c);
    return mfma_bf(a[2], lohi(b1, b0), c);
  } else {
    c = mfma_bf(a[2], b0, c);
    c = mfma_bf(a[1], b1, c);
    c = mfma_bf(a[0], b2, c);
    c = mfma_bf(a[1], b0, c);
    c = mfma_bf(a[0], b1, c);
    return mfma_bf(a[0], b0, c);
  }
}

// f32 semantics for the bf16x6 kernels (round 5). Three bf16 planes cannot carry an infinite
// operand (plane 0 = +-Inf, the residual Inf - Inf = NaN) nor one above bf16's largest finite
// value, 3.39e38 < FLT_MAX (plane 0 rounds to Inf); either leaves a NaN or Inf in the wave's
// accumulators, and so does a product or sum that overflows. A wave whose tile holds any
// non-finite value after the K loop (a wave-uniform ballot) recomputes its tile with f32 MFMA
// products (v_mfma_f32_16x16x4_f32) straight from global memory, in the f32 kernels' k order
// (16-deep steps, step s takes k = k0 + 4q + s, k >= K zeroed): Inf propagates, Inf * 0 and
// Inf - Inf give NaN, overflow gives Inf -- the f32 MFMA kernel's result for that tile. Finite
// data of sane range never takes the branch (~1 v_cmp_class per accumulator element).
// Padding rows never count: every kernel clamps the rows it loads past M (and NT kernels the
// weight rows past N) to the last valid one, so a padding row is non-finite only when a valid
// row is. MASKCOL: only columns < N count -- for the fused layer's in-register weight split
// (FX = 0), whose last vector reads the weight's padding columns [N, round4(N)), which may hold
// anything (a NaN there must not send the tile down the slow f32 path); every other
// kernel reads zeros or clamped columns past N and keeps the one-compare-per-element check (the
// masked form costs the fused layer ~2 % at the end of its K loop, PMC r06).
template <int RT, int G, bool MASKCOL = false>
__device__ __forceinline__ bool tile_nonfinite(const f4 (&acc)[RT][G][4], int N, int colw, int j) {
  if constexpr (!MASKCOL) {
    // x * 0 is 0 for finite x and NaN for Inf / NaN: one packed FMA per two accumulators
    // (round 6: the fused layer +2 % against a v_cmp_class per accumulator and the SGPR ors;
    // profiles/r06/dense_ab.jsonl)
    f2 s = {0.f, 0.f};
    const f2 z = {0.f, 0.f};
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s = __builtin_elementwise_fma(f2{acc[t][g][e][0], acc[t][g][e][1]}, z, s);
          s = __builtin_elementwise_fma(f2{acc[t][g][e][2], acc[t][g][e][3]}, z, s);
        }
    return __builtin_amdgcn_ballot_w64(s[0] != s[0] || s[1] != s[1]) != 0;
  }
  bool bad = false;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool col_in = !MASKCOL || colw + 64 * g + 4 * j + e < N;
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) bad |= col_in && !__builtin_isfinite(acc[t][g][e][r]);
    }
  return __builtin_amdgcn_ballot_w64(bad) != 0;
}
// B element (k, column n) at B + n * bn + k * bk (NT: Bt, bn = ldbt, bk = 1; fused: W, bn = 1,
// bk = ldw). rowb = the first row of the wave's 16 RT-row band; columns colw + 64 g + 4 j + e.
template <int RT, int G>
__device__ __forceinline__ void f32_tile(f4 (&acc)[RT][G][4], int M, int N, int K,
                                         const float* __restrict__ A, int64_t lda, int64_t rowb,
                                         const float* __restrict__ B, int64_t bn, int64_t bk,
                                         int colw, int j, int q) {
  int64_t ar[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const int64_t r = rowb + 16 * t + j;
    ar[t] = (r < M ? r : M - 1) * lda;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][g][e] = f4{0.f, 0.f, 0.f, 0.f};
  }
  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = k0 + 4 * q + s;
      const bool kin = k < K;
      float a[RT];
#pragma unroll
      for (int t = 0; t < RT; ++t) a[t] = kin ? A[ar[t] + k] : 0.f;
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = colw + 64 * g + 4 * j + e;
          const float b = (kin && c < N) ? B[c * bn + static_cast<int64_t>(k) * bk] : 0.f;
#pragma unroll
          for (int t = 0; t < RT; ++t) acc[t][g][e] = mfma4(a[t], b, acc[t][g][e]);
        }
    }
  }
}

template <int W>
__device__ __forceinline__ float reduce16_max(float v) {
#pragma unroll
  for (int o = 1; o < W; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
template <int W>
__device__ __forceinline__ float reduce16_sum(float v) {
#pragma unroll
  for (int o = 1; o < W; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int W>
__device__ __forceinline__ int reduce16_min(int v) {
#pragma unroll
  for (int o = 1; o < W; o <<= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

constexpr float kNegInf = -std::numeric_limits<float>::infinity();

// Reductions over the 16 lanes of a DPP row (lanes 16q .. 16q + 15: one output row of the
// MFMA layout) with DPP lane swaps -- quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror -- instead of ds_bpermute shuffles. Every lane of the row ends with the same
// value (each step combines a and b as op(a, b) in one lane and op(b, a) in its partner).
// Round 6: each step is ONE DPP-sourced VALU op (v_add_f32_dpp / v_min_i32_dpp / v_max_f32_dpp)
// instead of a v_mov_b32_dpp and the op -- the row reductions are 64 of the fused epilogue's
// per-wave steps. update_dpp with bound_ctrl lets the compiler fold the permute into the add /
// min (every lane of these row-internal permutations is valid, so bound_ctrl never applies).
// fmaxf keeps canonicalising maxes around a folded permute, so the max is written out: the
// s_nop 1 covers the VALU-write -> DPP-read hazard the compiler cannot see inside the asm. Same
// values as the two-instruction forms: a + b == b + a, min / max commute (max over quiet NaNs
// keeps fmaxf's maxNum: a NaN operand gives the other).
template <int CTRL>
__device__ __forceinline__ float upd_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ int upd_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
#define GCG_MAX_DPP(v, CTRL_ASM)                                                             \
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %1 " CTRL_ASM                              \
               " row_mask:0xf bank_mask:0xf bound_ctrl:1"                                  \
               : "=v"(v) : "v"(v))
__device__ __forceinline__ float row16_max(float v) {
  GCG_MAX_DPP(v, "quad_perm:[1,0,3,2]");
  GCG_MAX_DPP(v, "quad_perm:[2,3,0,1]");
  GCG_MAX_DPP(v, "row_half_mirror");
  GCG_MAX_DPP(v, "row_mirror");
  return v;
}
#undef GCG_MAX_DPP
__device__ __forceinline__ float row16_sum(float v) {
  v = v + upd_f<0xB1>(v);
  v = v + upd_f<0x4E>(v);
  v = v + upd_f<0x141>(v);
  return v + upd_f<0x140>(v);
}
__device__ __forceinline__ int row16_min(int v) {
  v = min(v, upd_i<0xB1>(v));
  v = min(v, upd_i<0x4E>(v));
  v = min(v, upd_i<0x141>(v));
  return min(v, upd_i<0x140>(v));
}


template <int RT, int G, int WR, int WC, int EPI, int PF>
__global__ __launch_bounds__(64 * WR * WC, (PF == 1 && WR * WC == 4) ? 1 : 2) void gemm_kernel(
    int M, int N, int K, const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
    int64_t ldb, const float* __restrict__ bias, int act, float* __restrict__ Cout, int64_t ldc,
    const int32_t* __restrict__ labels, float scale, const float* __restrict__ scale_dev,
    float* __restrict__ loss_rows, float* __restrict__ correct_rows,
    const float* __restrict__ row_w) {
  constexpr int NT = 64 * WR * WC;  // threads per workgroup (4 or 8 waves)
  static_assert(WR * WC == 4 || WR * WC == 8, "4 or 8 waves per workgroup");
  constexpr int BM = 16 * RT * WR;
  constexpr int BN = 64 * G * WC;
  constexpr int KC = 32;                   // k depth of one LDS chunk
  constexpr int A4 = BM * KC / 4 / NT;     // A dwordx4 per thread per chunk
  static_assert(A4 >= 1 && BM * KC / 4 % NT == 0, "A chunk must split evenly");
  // A chunk image: unpadded 128-B rows of 8 slots (16 B each), slot s of row r stored at slot
  // s ^ ((r >> 1) & 7). A fragment ds_read_b128 is serviced in 4 lane groups of 16, each
  // holding every j = 0..15 once with two q values ({0-3,12-15} with q, {4-11} with q + 1 or
  // the reverse, MI355X_MICROARCH.md §LDS): with this key the 16 starting dwords of a group
  // are 16 distinct multiples of 4 mod 64 -- conflict-free (the 36-float padded rows of round
  // 1-2 gave 2-way conflicts there: 13 % of the LDS cycles, PMC r02). The 8-lane groups of
  // the ds_write_b128 still cover one whole row each: conflict-free too.
  __shared__ float As[2][BM][KC];
  auto aslot = [](int r, int slot) { return (slot ^ ((r >> 1) & 7)) * 4; };
  __shared__ float red[4][WC][BM];  // epilogue row reductions: sum, label logit, argmax, max
  // EPI = 1: the bias of the workgroup's columns and the labels of its rows, staged in LDS
  // at the start so the epilogue reads them from LDS instead of waiting on global loads
  __shared__ float sbias[EPI == 1 ? BN : 1];
  __shared__ int slab[EPI == 1 ? BM : 1];
  __shared__ float srw[EPI == 1 ? BM : 1];  // row weights (target multiplicities), 1 if none

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: uniform branches
  const int wr = wave / WC, wc = wave % WC;
  const int j = lane & 15, q = lane >> 4;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
  const int colw = blockIdx.y * BN + wc * G * 64;  // this wave's first column
  const int n4 = (N + 3) & ~3;                     // columns B may be read at (<= ldb)

  // Per-lane B column offsets (clamped in range; out-of-range columns are never stored).
  int bcol[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int c = colw + 64 * g + 4 * j;
    bcol[g] = c < n4 ? c : 0;
  }

  f4 acc[RT][G][4];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][g][e] = f4{0.f, 0.f, 0.f, 0.f};

  // ---- A staging: chunk c covers k in [c*KC, c*KC + KC) ----
  // Branch-free: row and column are clamped into the operand and out-of-range elements are
  // zeroed by selects, so the loop body is straight-line and hipcc keeps counted vmcnt waits
  // (a branchy load makes it drain every load in flight). A 16-B load at a clamped column
  // stays inside the 16-B aligned block of a valid element, hence inside the allocation.
  const int kmax4 = (K - 1) & ~3;  // last 4-aligned column start with a valid element
  // The out-of-range elements are zeroed when the registers are written to LDS (store_a), not
  // right after the load: a select on the loaded value makes hipcc wait for the load there,
  // at the top of the chunk, instead of at the chunk's end.
  f4 areg[A4];
  int avalid[A4];  // valid elements of areg[i]: 0..4 (0 for a row past M)
  auto load_a = [&](int kc0) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int idx = tid + NT * i;
      const int r = idx / (KC / 4), k = kc0 + (idx % (KC / 4)) * 4;
      const int64_t gr = row0 + r;
      const int64_t rr = gr < M ? gr : M - 1;
      const int kk = k < kmax4 ? k : kmax4;
      areg[i] = *reinterpret_cast<const f4*>(A + rr * lda + kk);
      avalid[i] = gr < M ? min(max(K - k, 0), 4) : 0;
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int idx = tid + NT * i;
      const int r = idx / (KC / 4), slot = idx % (KC / 4);
      f4 v = areg[i];
      v.x = avalid[i] > 0 ? v.x : 0.f;
      v.y = avalid[i] > 1 ? v.y : 0.f;
      v.z = avalid[i] > 2 ? v.z : 0.f;
      v.w = avalid[i] > 3 ? v.w : 0.f;
      *reinterpret_cast<f4*>(&As[buf][r][aslot(r, slot)]) = v;
    }
  };
  // Workgroup barrier for the LDS hand-off only: waits for this wave's LDS traffic, not for
  // its global loads (a __syncthreads() fence would drain the B prefetch every chunk).
  auto lds_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- B fragments for one 16-deep k-step: bf[g][e] = B[k0 + 4q + e][bcol[g] .. +3] ----
  // Fragments (g, e) with unit u = 4g + e in [u0, u1) only (the split ping-pong body loads
  // one part of the set at a time).
  // B is read through a buffer descriptor re-based at row k0 for every step (scalar work): the
  // range check returns 0 for rows past K (A is 0 there as well), so the per-lane row clamp and
  // 64-bit row addresses of round 2 (~48 VALU per 16-deep step, VALU that lowered the clock this
  // MFMA loop holds) are gone; the per-lane byte offsets are constants. Host: K * ldb * 4 < 2^31.
  uint32_t boff[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      boff[g][e] = static_cast<uint32_t>(((4 * q + e) * static_cast<int>(ldb) + bcol[g]) * 4);
  auto load_b = [&](f4 (&bf)[G][4], int k0, int u0 = 0, int u1 = 4 * G) {
    const int kb = k0 < K ? k0 : K;  // a prefetch past K gets an empty range: zeros
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(B + static_cast<int64_t>(kb) * ldb), static_cast<short>(0),
        (K - kb) * static_cast<int>(ldb) * 4, 0x00020000);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (4 * g + e >= u0 && 4 * g + e < u1)
          bf[g][e] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, boff[g][e], 0, 0));
  };

  const int arow = wr * 16 * RT + j;
  // Skipping groups past N (a wave-uniform branch per step and group) measured faster with the
  // register-prefetch (PF = 1) body -- without it hipcc shuffles the accumulators through
  // AGPR copies and spills -- and slower with the single-buffer body.
  constexpr bool SKIP = PF != 0;
  const int ngv = min(G, max(0, (N - colw + 63) / 64));  // groups with a column < N
  auto compute = [&](const f4 (&bf)[G][4], int buf, int s, int u0 = 0, int u1 = 4 * G) {
    f4 af[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t)
      af[t] = *reinterpret_cast<const f4*>(&As[buf][arow + 16 * t][aslot(arow + 16 * t, 4 * s + q)]);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (4 * g + e < u0 || 4 * g + e >= u1) continue;  // compile-time after unrolling
        if (SKIP && g >= ngv) continue;  // scalar branch: group entirely past N
#pragma unroll
        for (int t = 0; t < RT; ++t) {
          acc[t][g][0] = mfma4(af[t][e], bf[g][e].x, acc[t][g][0]);
          acc[t][g][1] = mfma4(af[t][e], bf[g][e].y, acc[t][g][1]);
          acc[t][g][2] = mfma4(af[t][e], bf[g][e].z, acc[t][g][2]);
          acc[t][g][3] = mfma4(af[t][e], bf[g][e].w, acc[t][g][3]);
        }
      }
  };

  // Main loop, one 32-deep chunk (two 16-deep steps) per iteration, straight-line: B
  // ping-pongs between two register sets (step 2c in b0, 2c+1 in b1, each loaded one step
  // ahead), A chunk c+1 is loaded to registers during chunk c and written to the other LDS
  // buffer after it.
  static_assert(KC == 32, "two 16-deep steps per chunk");
  __builtin_assume(K > 0);  // checked on the host: the main loop runs at least once
  const int n_chunks = (K + KC - 1) / KC;
  load_a(0);
  if constexpr (EPI == 1) {
    for (int c = tid; c < BN; c += NT) {
      const int gc = blockIdx.y * BN + c;
      // columns past N: -inf, so their softmax weight is exactly 0 (no mask in the epilogue)
      sbias[c] = gc < N ? (bias != nullptr ? bias[gc] : 0.f) : kNegInf;
    }
    for (int r = tid; r < BM; r += NT) {
      const int64_t row = row0 + r;
      int y = (labels != nullptr && row < M) ? labels[row] : -1;
      // -1: no label; a label outside [0, N) becomes -2: NaN loss, no hit, no onehot
      if (labels != nullptr && (y < 0 || y >= N)) y = -2;
      slab[r] = y;
      srw[r] = (row_w != nullptr && row < M) ? row_w[row] : 1.f;
    }
    // (issued beside the first A chunk's loads; visible after the barrier below)
  }
  store_a(0);
  lds_barrier();
  f4 b0[G][4];
  if constexpr (PF >= 2) {
    // Split ping-pong in one register set: b0's 4G fragments (g, e) are cut into NP = PF
    // parts that rotate, each part loaded for the next 16-deep step as soon as its MFMAs for
    // this step are issued, so a wave computes the other parts while a part's loads are in
    // flight (PF = 1's latency hiding at PF = 0's register count, which keeps 2 workgroups
    // per CU). Every accumulator still sees e = 0..3 in order: bitwise equal to PF = 0.
    constexpr int NP = PF, NU = 4 * G;
    static_assert(NU % NP == 0, "parts split the fragments evenly");
    // The prologue issues the parts in ring order (scheduling barriers; K > 0 is assumed so
    // the loads are not sunk past a zero-trip branch): hipcc merges the preheader's and the
    // back-edge's outstanding loads at the loop header and otherwise drains the ring there
    // (vmcnt(2)); now every wait is counted (vmcnt(15..16)). Measured neutral (the kernel runs
    // at a power-limited clock), kept for the cleaner schedule. Pinning the loop body as well
    // measured slower: 93.0-95.0 vs 96.2 TFLOP/s.
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      load_b(b0, 0, p * NU / NP, (p + 1) * NU / NP);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int c = 0; c < n_chunks; ++c) {
      const int buf = c & 1;
      const int k0 = c * KC;
      load_a(k0 + KC);  // past K: clamped and zeroed, never used
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        // the second 16-deep step of the last chunk lies wholly past K (A is zero there):
        // skip its MFMAs and the refills, which would only fetch rows past K
        if (st == 1 && k0 + 16 >= K) break;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          compute(b0, buf, st, p * NU / NP, (p + 1) * NU / NP);
          load_b(b0, k0 + 16 * (st + 1), p * NU / NP, (p + 1) * NU / NP);
        }
      }
      store_a(buf ^ 1);
      lds_barrier();
    }
  } else if constexpr (PF) {
    f4 b1[G][4];
    load_b(b0, 0);
    for (int c = 0; c < n_chunks; ++c) {
      const int buf = c & 1;
      const int k0 = c * KC;
      load_a(k0 + KC);  // past K: clamped and zeroed, never used
      load_b(b1, k0 + 16);
      compute(b0, buf, 0);
      load_b(b0, k0 + 32);
      if (k0 + 16 < K) compute(b1, buf, 1);
      store_a(buf ^ 1);
      lds_barrier();
    }
  } else {
    // One B register set: a wave waits for its step's loads while the other wave(s) on
    // its SIMD compute (8-wave workgroups, 2 waves per SIMD).
    for (int c = 0; c < n_chunks; ++c) {
      const int buf = c & 1;
      const int k0 = c * KC;
      load_a(k0 + KC);
      load_b(b0, k0);
      compute(b0, buf, 0);
      if (k0 + 16 < K) {
        load_b(b0, k0 + 16);
        compute(b0, buf, 1);
      }
      store_a(buf ^ 1);
      lds_barrier();
    }
  }

#define GCG_EPI_BV_READY
#define GCG_EPI_LABELS_LDS
  f4 bv[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if constexpr (EPI == 1) {
      bv[g] = *reinterpret_cast<const f4*>(&sbias[wc * G * 64 + 64 * g + 4 * j]);
    } else {
      bv[g] = f4{0.f, 0.f, 0.f, 0.f};
      const int c = colw + 64 * g + 4 * j;
      if (bias != nullptr) {
        if (c < N) bv[g].x = bias[c];
        if (c + 1 < N) bv[g].y = bias[c + 1];
        if (c + 2 < N) bv[g].z = bias[c + 2];
        if (c + 3 < N) bv[g].w = bias[c + 3];
      }
    }
  }
#include "gemm_epilogue.inc"
#undef GCG_EPI_BV_READY
#undef GCG_EPI_LABELS_LDS
}

// ---------------------------------------------------------------------------------------
// gemm_bl_kernel<G, WC, EPI>: the same product and epilogues with B staged through LDS.
// Workgroup = 4 row bands (WR = 4) x WC column waves, wave tile 16 rows x 64*G columns
// (RT = 1), workgroup tile 64 x 64*G*WC. Per 32-deep k chunk the workgroup copies A[64 x 32]
// and B[32 x BN] to LDS once; the 4 row bands share every B fragment, so B leaves L2 once per
// 64 rows (gemm_kernel: once per 16*RT rows per wave) and a fragment read costs LDS latency
// instead of L2 latency. The next chunk's loads are issued into registers before the current
// chunk's MFMAs and written to LDS after them (one LDS buffer, two barriers per chunk).
// LDS B image: row k at k*BN floats; lanes (j, q) of one ds_read_b128 group read rows
// k0+4q+e, columns 4j..4j+3: BN % 16 == 0 keeps every 16-lane group on 64 distinct banks.
// ---------------------------------------------------------------------------------------
template <int G, int WC, int EPI>
__global__ __launch_bounds__(256 * WC, WC == 1 ? 2 : 1) void gemm_bl_kernel(
    int M, int N, int K, const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
    int64_t ldb, const float* __restrict__ bias, int act, float* __restrict__ Cout, int64_t ldc,
    const int32_t* __restrict__ labels, float scale, const float* __restrict__ scale_dev,
    float* __restrict__ loss_rows, float* __restrict__ correct_rows,
    const float* __restrict__ row_w) {
  constexpr int RT = 1, WR = 4;
  constexpr int NT = 64 * WR * WC;
  constexpr int BM = 16 * RT * WR;  // 64
  constexpr int BN = 64 * G * WC;
  constexpr int KC = BN >= 512 ? 16 : 32;  // k depth of one chunk: wide B -> fewer staging VGPRs
  constexpr int KP = KC + 4;
  constexpr int AT = BM * KC / 4 < NT ? BM * KC / 4 : NT;  // threads staging A (whole waves)
  constexpr int A4 = BM * KC / 4 / AT;
  constexpr int B4 = KC * BN / 4 / NT;
  static_assert(AT % 64 == 0 && A4 >= 1 && BM * KC / 4 % AT == 0, "A chunk must split evenly");
  static_assert(B4 >= 1 && KC * BN / 4 % NT == 0, "B chunk must split evenly");
  static_assert(BN % 16 == 0, "conflict-free B fragment reads");
  // NB = 2 LDS buffers (one barrier per chunk) for the 8-wave tiles, which hold a CU alone
  // anyway; the 4-wave tiles keep one buffer (two barriers) so 2-3 workgroups share a CU
  constexpr int NB = (WC >= 2 && (2 * (BM * KP + KC * BN) + 4 * WC * BM) * 4 <= 160 * 1024) ? 2 : 1;
  __shared__ float As[NB][BM][KP];
  __shared__ float Bs[NB][KC][BN];
  __shared__ float red[4][WC][BM];  // epilogue row reductions: sum, label logit, argmax, max

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int j = lane & 15, q = lane >> 4;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
  const int colb = blockIdx.y * BN;          // workgroup's first column
  const int colw = colb + wc * G * 64;       // this wave's first column
  const int n4 = (N + 3) & ~3;

  f4 acc[RT][G][4];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[0][g][e] = f4{0.f, 0.f, 0.f, 0.f};

  // Branch-free staging loads (clamped addresses, zeroed by selects): see gemm_kernel.
  const int kmax4 = (K - 1) & ~3;
  f4 areg[A4], breg[B4];
  const bool a_stager = tid < AT;  // wave-uniform
  auto load_chunk = [&](int kc0) {
#pragma unroll
    for (int i = 0; i < A4; ++i) {
      const int idx = (a_stager ? tid : tid - AT) + AT * i;  // non-stagers: a harmless copy
      const int r = idx / (KC / 4), k = kc0 + (idx % (KC / 4)) * 4;
      const int64_t gr = row0 + r;
      const int64_t rr = gr < M ? gr : M - 1;
      const int kk = k < kmax4 ? k : kmax4;
      f4 v = *reinterpret_cast<const f4*>(A + rr * lda + kk);
      const bool rowok = gr < M;
      v.x = (rowok && k < K) ? v.x : 0.f;
      v.y = (rowok && k + 1 < K) ? v.y : 0.f;
      v.z = (rowok && k + 2 < K) ? v.z : 0.f;
      v.w = (rowok && k + 3 < K) ? v.w : 0.f;
      areg[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B4; ++i) {
      const int idx = tid + NT * i;
      const int kr = idx / (BN / 4), c = colb + (idx % (BN / 4)) * 4;
      int k = kc0 + kr;
      k = k < K ? k : K - 1;         // A is zero there; any finite B row does
      const int cc = c < n4 ? c : 0;  // columns past N: never stored (masked in EPI = 1)
      breg[i] = *reinterpret_cast<const f4*>(B + static_cast<int64_t>(k) * ldb + cc);
    }
  };
  auto store_chunk = [&](int buf) {
    if (a_stager) {
#pragma unroll
      for (int i = 0; i < A4; ++i) {
        const int idx = tid + AT * i;
        *reinterpret_cast<f4*>(&As[buf][idx / (KC / 4)][(idx % (KC / 4)) * 4]) = areg[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B4; ++i) {
      const int idx = tid + NT * i;
      *reinterpret_cast<f4*>(&Bs[buf][idx / (BN / 4)][(idx % (BN / 4)) * 4]) = breg[i];
    }
  };
  auto lds_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  const int arow = wr * 16 + j;
  const int bl = wc * G * 64 + 4 * j;  // this lane's column inside the LDS B image
  auto compute_step = [&](int buf, int s) {
    const f4 af = *reinterpret_cast<const f4*>(&As[buf][arow][s * 16 + 4 * q]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      // all G fragments of this k first (no branch between them: the reads stay in flight
      // together), then 4G MFMAs; groups past N compute on clamped columns, never stored
      const float* brow = &Bs[buf][s * 16 + 4 * q + e][bl];
      f4 bf[G];
#pragma unroll
      for (int g = 0; g < G; ++g) bf[g] = *reinterpret_cast<const f4*>(brow + 64 * g);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        acc[0][g][0] = mfma4(af[e], bf[g].x, acc[0][g][0]);
        acc[0][g][1] = mfma4(af[e], bf[g].y, acc[0][g][1]);
        acc[0][g][2] = mfma4(af[e], bf[g].z, acc[0][g][2]);
        acc[0][g][3] = mfma4(af[e], bf[g].w, acc[0][g][3]);
      }
    }
  };

  const int n_chunks = (K + KC - 1) / KC;
  load_chunk(0);
  store_chunk(0);
  lds_barrier();
  for (int c = 0; c < n_chunks; ++c) {
    const int k0 = c * KC;
    const int buf = NB == 2 ? (c & 1) : 0;
    const bool more = c + 1 < n_chunks;
    if (more) load_chunk(k0 + KC);  // in flight during this chunk's MFMAs
    compute_step(buf, 0);
    if (KC == 32 && k0 + 16 < K) compute_step(buf, 1);
    if (more) {
      // two buffers: the other one was last read in chunk c-1, before the barrier that
      // ended it; one buffer: wait until every wave is done reading this chunk
      if (NB == 1) lds_barrier();
      store_chunk(NB == 2 ? buf ^ 1 : 0);
      lds_barrier();
    }
  }
#include "gemm_epilogue.inc"
}

// ---------------------------------------------------------------------------------------
// gemm_nt_kernel<RT, G, WR, WC, S, PF, KC>: C = act(A . Bt^T + bias), both operands
// k-contiguous (A: M x K row-major, Bt: N x K row-major -- the weight stored transposed, as
// graphconvgeo_amd.dense keeps it), staged into LDS by the async LDS-DMA
// (global_load_lds_dwordx4) through an S-deep ring of KC-deep k chunks (KC = 32 or 16).
//
//   * LDS image per stage: [BM + BN rows][KC floats], SL = KC/4 slots of 16 B per row, slot s
//     of image row r stored at slot s ^ key(r): key = r & 7 for 8-slot rows, a permutation of
//     (r >> 2) & 3 for 4-slot rows -- chosen so that each 16-lane group of a fragment read
//     (16 consecutive image rows, slots q) hits 16 distinct bank quads: conflict-free
//     ds_read_b128. The DMA writes LDS linearly (wave base + 16 B per lane), so the swizzle is
//     applied to the per-lane GLOBAL source address (the involution s' <-> s ^ key(r)).
//   * B image row order: within each 64-column group, row 16e + j holds column 4j + e, so
//     the fragment of the strided MFMA tile e (columns 4j + e, j = 0..15) is 16 consecutive
//     image rows, and a lane ends up with 4 ADJACENT output columns (acc[t][g][0..3]) ->
//     dwordx4 stores; the register layout of gemm_kernel (gemm_epilogue.inc).
//   * A fragment: one ds_read_b128 per 16-row tile per 16-deep step gives the lane its 4
//     k-values of the 4 v_mfma_f32_16x16x4_f32 substeps (k = k0 + 4q + e, permuted
//     identically for A and B); B likewise, one ds_read_b128 per 16-column tile.
//   * Sync: ONE raw s_barrier per chunk, after a counted `s_waitcnt vmcnt` that retires the
//     chunk's own DMA (S = 2: vmcnt(0); S = 3: the next stage stays in flight). The barrier
//     also fences the buffer the next DMA overwrites: every wave finished reading it (its
//     MFMAs consumed the reads) before arriving. All LDS is one __shared__ array (a second
//     object makes hipcc drain the DMA queue before every ds_read).
//   * K tail: source addresses are clamped into the row; in the step that reaches past K the
//     fragment elements at k >= K are zeroed in registers (both operands, so garbage in the
//     operands' padding never meets a finite factor). Until round 2 the last chunk's k >= K
//     elements were zeroed in LDS by a 24-iteration loop per thread plus an extra barrier, once
//     per tile (~10 % of a K = 300 tile). Rows past M / columns past N read clamped rows and
//     are never stored.
//   * XCD-aware order (MI355X_MICROARCH.md: workgroup b runs on XCD b % 8): workgroup b takes
//     logical tile remap(b), each XCD walking one contiguous range of tiles in row-block-major
//     order, so the N / BN column tiles of a row block share one XCD's L2 copy of its A rows.
// Numerics: exact f32 products, f32 accumulation in k order k0 + 4q + e inside each 16-deep
// step (as gemm_kernel): equal to BLAS sgemm within f32 rounding.
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) const void* glds_src_t;
typedef __attribute__((address_space(3))) void* glds_dst_t;

// 16 B per lane into LDS through a buffer descriptor (base + byte range; reads past the range
// return 0), lane byte offset voff
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), static_cast<short>(0), bytes,
                                           0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, float* lds_wave_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds_wave_base),
                                           16, voff, 0, 0, 0);
}

// the same with the non-temporal policy (a stream read once, e.g. the fused layer's A rows)
__device__ __forceinline__ void blds16_nt(__amdgpu_buffer_rsrc_t r, float* lds_wave_base, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds_wave_base),
                                           16, voff, 0, 0, 2);
}

__device__ __forceinline__ void glds16(const float* src, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(reinterpret_cast<glds_src_t>(reinterpret_cast<uintptr_t>(src)),
                                   (glds_dst_t)(lds_wave_base), 16, 0, 0);
}

template <int RT, int G, int WR, int WC, int S, int KC>
struct NtCfg {
  static constexpr int NW = WR * WC;
  static constexpr int NT = 64 * NW;
  static constexpr int BM = 16 * RT * WR;
  static constexpr int BN = 64 * G * WC;
  static constexpr int SL = KC / 4;               // 16-B slots per image row
  static constexpr int RPI = 64 / SL;             // image rows per DMA instruction (1 KB)
  static constexpr int ROWS = BM + BN;            // image rows per stage
  static constexpr int STAGE = ROWS * KC;         // floats per stage
  static constexpr int NGLDS = ROWS / RPI;        // DMA wave-instructions per stage
  static constexpr int PER_WAVE = NGLDS / NW;     // (exact when S >= 3)
  static constexpr int FLOATS = S * STAGE;
  static constexpr int LDS_BYTES = FLOATS * 4;
  static constexpr int OCC_LDS = (160 * 1024) / LDS_BYTES;  // workgroups per CU the LDS allows
  static constexpr int OCC = OCC_LDS < 1 ? 1 : (OCC_LDS > 4 ? 4 : OCC_LDS);
  static_assert(KC == 16 || KC == 32, "4- or 8-slot image rows");
  static_assert(ROWS % RPI == 0, "whole DMA instructions per stage");
  static_assert(S == 2 || NGLDS % NW == 0, "S >= 3 needs the same DMA count on every wave");
  static_assert(S >= 2 && S <= 6, "2..6 stages");
};

// Swizzle key of image row r (see above). 4-slot rows: pi((r >> 2) & 3), pi = {0, 2, 3, 1},
// the permutation that makes every ds_read_b128 lane group {0-3,12-15,20-27}, ... of rows
// j = 0..15 x slots q land on distinct bank quads.
template <int SL>
__device__ __forceinline__ int nt_key(int r) {
  if constexpr (SL == 8) return r & 7;
  else return (0x78 >> (2 * ((r >> 2) & 3))) & 3;  // pi packed 2 bits each: 0, 2, 3, 1
}

template <int RT, int G, int WR, int WC, int S, int PF, int KC, int MX = 0>
__global__ __launch_bounds__(64 * WR * WC, (NtCfg<RT, G, WR, WC, S, KC>::OCC)) void
gemm_nt_kernel(int M, int N, int K, const float* __restrict__ A, int64_t lda,
               const float* __restrict__ Bt, int64_t ldb, const float* __restrict__ bias, int act,
               float* __restrict__ Cout, int64_t ldc, int n_col_tiles) {
  constexpr bool TP = (MX & 2) != 0;  // the packed K tail (mfma6; MX & 1: bf16x6)
  using Cfg = NtCfg<RT, G, WR, WC, S, KC>;
  constexpr int EPI = 0;  // plain epilogue only (gemm_epilogue.inc names the EPI = 1 operands)
  const int32_t* labels = nullptr;
  float scale = 0.f;
  const float* scale_dev = nullptr;
  float* loss_rows = nullptr;
  float* correct_rows = nullptr;
  const float* row_w = nullptr;
  (void)labels; (void)scale; (void)scale_dev; (void)loss_rows; (void)correct_rows; (void)row_w;
  constexpr int NT = Cfg::NT, BM = Cfg::BM, BN = Cfg::BN, STAGE = Cfg::STAGE;
  constexpr int SL = Cfg::SL, RPI = Cfg::RPI;
  __shared__ __attribute__((aligned(16))) float smem[Cfg::FLOATS];
  float (*red)[WC][BM] = nullptr;  // (EPI = 1 only)
  (void)red;

  // XCD-aware bijective remap of the 1-D grid (cdna_hip_programming.md T1).
  const int nwg = static_cast<int>(gridDim.x);
  const int b = static_cast<int>(blockIdx.x);
  const int xcd = b % 8, qq = nwg / 8, rr = nwg % 8;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
  const int row_tile = tile / n_col_tiles, col_tile = tile % n_col_tiles;
  const int64_t row0 = static_cast<int64_t>(row_tile) * BM;
  const int col0 = col_tile * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int j = lane & 15, q = lane >> 4;
  const int colw = col0 + wc * G * 64;  // this wave's first output column (epilogue)

  // ---- DMA source rows: this wave's instructions i = wave + NW * u cover image rows
  // RPI*i .. RPI*i + RPI-1; lane -> row RPI*i + lane / SL, LDS slot lane % SL, global slot
  // (lane % SL) ^ key(row).
  constexpr int NU = (Cfg::NGLDS + Cfg::NW - 1) / Cfg::NW;  // instructions per wave (max)
  const float* src[NU];
  int kofs[NU];  // 4 * global slot
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int i = wave + Cfg::NW * u;
    const int r = RPI * i + lane / SL;
    const int sl = (lane % SL) ^ nt_key<SL>(r);
    kofs[u] = 4 * sl;
    if (r < BM) {
      const int64_t gr = row0 + r;
      src[u] = A + (gr < M ? gr : static_cast<int64_t>(M) - 1) * lda;
    } else {
      const int rb = r - BM;                       // B image row: group, tile e, lane j
      const int n = col0 + (rb & ~63) + 4 * (rb & 15) + ((rb >> 4) & 3);
      src[u] = Bt + static_cast<int64_t>(n < N ? n : N - 1) * ldb;
    }
  }
  const int kmax4 = (K - 1) & ~3;  // last 16-B segment holding a valid k
  auto issue = [&](int chunk) {
    float* stage = smem + (chunk % S) * STAGE;
    const int kc0 = chunk * KC;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = wave + Cfg::NW * u;
      if (NU * Cfg::NW != Cfg::NGLDS && i >= Cfg::NGLDS) break;  // wave-uniform
      int k = kc0 + kofs[u];
      k = k < kmax4 ? k : kmax4;
      glds16(src[u] + k, stage + i * 256);  // instruction i fills 1 KB of the image
    }
  };
  auto lds_barrier = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f4 acc[RT][G][4];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][g][e] = f4{0.f, 0.f, 0.f, 0.f};

  // bias of this lane's output columns, loaded now so its latency hides behind the K loop
  f4 bv[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    bv[g] = f4{0.f, 0.f, 0.f, 0.f};
    const int c = colw + 64 * g + 4 * j;
    if (bias != nullptr) {
      if (c + 3 < N) {
        bv[g] = f4{bias[c], bias[c + 1], bias[c + 2], bias[c + 3]};
      } else {
        if (c < N) bv[g].x = bias[c];
        if (c + 1 < N) bv[g].y = bias[c + 1];
        if (c + 2 < N) bv[g].z = bias[c + 2];
      }
    }
  }

  const int n_chunks = (K + KC - 1) / KC;
  const int arow0 = wr * 16 * RT + j;       // A image row of tile 0 (lane j)
  const int brow0 = BM + wc * G * 64 + j;   // B image row of group 0, tile e = 0 (lane j)
  auto frag = [&](const float* stage, int row, int slot) -> f4 {
    return *reinterpret_cast<const f4*>(stage + row * KC + 4 * (slot ^ nt_key<SL>(row)));
  };
  auto mfma_step = [&](const f4 (&af)[RT], const f4 (&bf)[G][4]) {
#pragma unroll
    for (int ss = 0; ss < 4; ++ss)
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[t][g][e] = mfma4(af[t][ss], bf[g][e][ss], acc[t][g][e]);
  };
  // zero the elements of a step's fragments at k >= K: lane (j, q) holds k = kb + 4q + e
  auto mask_step = [&](f4 (&af)[RT], f4 (&bf)[G][4], int kb) {
    const int lim = K - kb - 4 * q;  // elements e < lim are inside K
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool in = e < lim;
#pragma unroll
      for (int t = 0; t < RT; ++t) af[t][e] = in ? af[t][e] : 0.f;
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) bf[g][e2][e] = in ? bf[g][e2][e] : 0.f;
    }
  };
  auto read_step = [&](const float* stage, int h, f4 (&af)[RT], f4 (&bf)[G][4]) {
#pragma unroll
    for (int t = 0; t < RT; ++t) af[t] = frag(stage, arow0 + 16 * t, 4 * h + q);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) bf[g][e] = frag(stage, brow0 + 64 * g + 16 * e, 4 * h + q);
  };

#pragma unroll
  for (int c = 0; c < S - 1; ++c)
    if (c < n_chunks) issue(c);
  // one chunk; tp: the packed K tail (mfma6), only the peeled last chunk of a TP kernel (MX & 2,
  // chosen by the host when that chunk holds <= 16 live k)
  auto chunk_body = [&](int c, auto tp) {
    // retire this chunk's DMA (leave the later stages in flight), then one barrier
    if constexpr (S == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (c + S - 2 < n_chunks) {
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"((S - 2) * Cfg::PER_WAVE) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    lds_barrier();
    const float* stage = smem + (c % S) * STAGE;
    const int kc0 = c * KC;
    if (c + S - 1 < n_chunks) issue(c + S - 1);
    // K tail: a step reaching past K has its k >= K fragment elements zeroed in registers
    // (wave-uniform branch, last chunk only); the LDS there holds clamped re-reads / padding
    if constexpr (KC == 16) {
      f4 af[RT], bf[G][4];
      read_step(stage, 0, af, bf);
      if (kc0 + 16 > K) mask_step(af, bf, kc0);
      mfma_step(af, bf);
    } else if constexpr ((MX & 1) != 0) {
      // bf16x6: the chunk's two 16-deep fragment sets are one 32-deep bf16 MFMA operand (lane
      // (j, q) holds k = kc0 + 4q + {0..3} and kc0 + 16 + 4q + {0..3}, the same for A and B)
      f4 af0[RT], bf0[G][4], af1[RT], bf1[G][4];
      read_step(stage, 0, af0, bf0);
      read_step(stage, 1, af1, bf1);
      if (kc0 + 16 > K) mask_step(af0, bf0, kc0);
      if (kc0 + 32 > K) mask_step(af1, bf1, kc0 + 16);
      bf8 ap[RT][3];
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const f8 x = {af0[t][0], af0[t][1], af0[t][2], af0[t][3],
                      af1[t][0], af1[t][1], af1[t][2], af1[t][3]};
        split3(x, ap[t][0], ap[t][1], ap[t][2]);
      }
      auto mm = [&](auto tp) {  // tp: the packed K tail (mfma6)
        constexpr bool TPC = decltype(tp)::value;
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f8 y = {bf0[g][e][0], bf0[g][e][1], bf0[g][e][2], bf0[g][e][3],
                          bf1[g][e][0], bf1[g][e][1], bf1[g][e][2], bf1[g][e][3]};
            bf8 b0, b1, b2;
            split3(y, b0, b1, b2);
#pragma unroll
            for (int t = 0; t < RT; ++t)
              acc[t][g][e] = mfma6<TPC>(ap[t], b0, b1, b2, acc[t][g][e]);
          }
      };
      if constexpr (decltype(tp)::value) {
#pragma unroll
        for (int t = 0; t < RT; ++t) pack_tail_a(ap[t]);
      }
      mm(tp);
    } else if constexpr (PF) {
      // both 16-deep steps' fragments first: the second step's LDS reads are in flight
      // during the first step's MFMAs (counted lgkmcnt waits)
      f4 af0[RT], bf0[G][4], af1[RT], bf1[G][4];
      read_step(stage, 0, af0, bf0);
      read_step(stage, 1, af1, bf1);
      if (kc0 + 16 > K) mask_step(af0, bf0, kc0);
      mfma_step(af0, bf0);
      if (kc0 + 16 < K) {
        if (kc0 + 32 > K) mask_step(af1, bf1, kc0 + 16);
        mfma_step(af1, bf1);
      }
    } else {
      f4 af[RT], bf[G][4];
      read_step(stage, 0, af, bf);
      if (kc0 + 16 > K) mask_step(af, bf, kc0);
      mfma_step(af, bf);
      if (kc0 + 16 < K) {
        read_step(stage, 1, af, bf);
        if (kc0 + 32 > K) mask_step(af, bf, kc0 + 16);
        mfma_step(af, bf);
      }
    }
  };
  const int n_full = TP ? n_chunks - 1 : n_chunks;
  for (int c = 0; c < n_full; ++c) chunk_body(c, std::false_type{});
  if constexpr (TP) chunk_body(n_full, std::true_type{});
  if constexpr (MX != 0) {  // bf16x6: f32 semantics for Inf / huge operands (f32_tile)
    if (tile_nonfinite<RT, G>(acc, N, colw, j))
      f32_tile<RT, G>(acc, M, N, K, A, lda, row0 + wr * 16 * RT, Bt, ldb, 1, colw, j, q);
  }
#define GCG_EPI_BV_READY
#include "gemm_epilogue.inc"
#undef GCG_EPI_BV_READY
}

// ---------------------------------------------------------------------------------------
// bf16x6 NT GEMM with the weight side pre-split (round 4): C = act(A . Bt^T + bias) with
// Bt's three bf16 planes written once per call by split3_rows_kernel into a workspace laid out
// [N][Kc][3][32] bf16 (Kc = ceil(K / 32) chunks, zeros past K), each 32-element plane chunk in
// the k order of the MFMA operand (position 8q + w holds k = 4q + w for w < 4, 16 + 4q + w - 4
// after), so a lane's B fragment of one plane is ONE 16-B LDS read and no B conversion is left
// in the loop. A stays f32 (staged exactly as gemm_nt_kernel's KC = 32 image) and is split in
// registers. LDS stage: [BM rows][8 slots] f32, then per plane [BN rows][4 slots] (64-B rows,
// swizzle nt_key<4>, the conflict-free 4-slot layout of the KC = 16 kernel), all through the
// LDS-DMA ring. The B image keeps gemm_nt_kernel's strided row order (row 16e + j of a 64-column
// group holds column 4j + e), so the accumulator layout and the epilogue are the same.
// ---------------------------------------------------------------------------------------
// (element (n, k) at Bt + n * ldb + k * kstride: kstride = 1 for the NT weight Bt, ldw for the
// fused layer's W read column-wise; planes for n in [N, n_out) are zero)
__global__ __launch_bounds__(256) void split3_rows_kernel(int N, int K, int Kc,
                                                          const float* __restrict__ Bt, int64_t ldb,
                                                          unsigned* __restrict__ out,
                                                          int64_t kstride = 1, int n_out = 0) {
  const int n_rows = n_out > N ? n_out : N;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;  // (n, chunk, q)
  if (i >= static_cast<int64_t>(n_rows) * Kc * 4) return;
  const int q = static_cast<int>(i & 3);
  const int64_t nc = i >> 2;
  const int n = static_cast<int>(nc / Kc), c = static_cast<int>(nc % Kc);
  const float* row = Bt + static_cast<int64_t>(n < N ? n : 0) * ldb;
  f8 x;
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    const int k = 32 * c + (w < 4 ? 4 * q + w : 16 + 4 * q + (w - 4));
    x[w] = (k < K && n < N) ? row[static_cast<int64_t>(k) * kstride] : 0.f;
  }
  bf8 h[3];
  split3(x, h[0], h[1], h[2]);
  if (n_out > 0) {
    // fused layer's layout [c][plane][n / 64][n % 4][(n % 64) / 4][q]: the 16 lanes j of one
    // (column group, slot e, plane) read 16 x 64 contiguous bytes
    const int gq = n >> 6, e = n & 3, jj = (n & 63) >> 2, ng = (n_rows + 63) >> 6;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int64_t pos = ((((static_cast<int64_t>(c) * 3 + p) * ng + gq) * 4 + e) * 16 + jj) * 16 + 4 * q;
      *reinterpret_cast<u4v*>(out + pos) = __builtin_bit_cast(u4v, h[p]);
    }
    return;
  }
  // [n][c][plane][32 bf16]: plane p's lane-q fragment is the 16 B at (nc * 3 + p) * 64 + 16 q
#pragma unroll
  for (int p = 0; p < 3; ++p)
    *reinterpret_cast<u4v*>(out + (nc * 3 + p) * 16 + 4 * q) = __builtin_bit_cast(u4v, h[p]);
}

template <int RT, int G, int WR, int WC, int S>
struct Nt3Cfg {
  static constexpr int NW = WR * WC;
  static constexpr int BM = 16 * RT * WR;
  static constexpr int BN = 64 * G * WC;
  static constexpr int A_FLOATS = BM * 32;          // [BM][8 slots of 16 B]
  static constexpr int P_FLOATS = BN * 16;          // one plane: [BN][4 slots of 16 B]
  static constexpr int STAGE = A_FLOATS + 3 * P_FLOATS;
  static constexpr int NGA = BM / 8;                // DMA wave-instructions (1 KB each)
  static constexpr int NGP = BN / 16;               // ... per plane
  static constexpr int NG = NGA + 3 * NGP;
  static constexpr int NU = (NG + NW - 1) / NW;
  static constexpr int PER_WAVE = NG / NW;          // (exact when S >= 3)
  static constexpr int FLOATS = S * STAGE;
  static constexpr int OCC_LDS = (160 * 1024) / (FLOATS * 4);
  static constexpr int OCC = OCC_LDS < 1 ? 1 : (OCC_LDS > 4 ? 4 : OCC_LDS);
  static_assert(S == 2 || NG % NW == 0, "S >= 3 needs the same DMA count on every wave");
  static_assert(S >= 2 && S <= 4, "2..4 stages");
};

template <int RT, int G, int WR, int WC, int S, bool TP = false>  // TP: the packed K tail
__global__ __launch_bounds__(64 * WR * WC, (Nt3Cfg<RT, G, WR, WC, S>::OCC)) void
gemm_nt3_kernel(int M, int N, int K, const float* __restrict__ A, int64_t lda,
                const unsigned* __restrict__ Bs, const float* __restrict__ Bt, int64_t ldbt, const float* __restrict__ bias, int act,
                float* __restrict__ Cout, int64_t ldc, int n_col_tiles) {
  using Cfg = Nt3Cfg<RT, G, WR, WC, S>;
  constexpr int EPI = 0;
  const int32_t* labels = nullptr;
  float scale = 0.f;
  const float* scale_dev = nullptr;
  float* loss_rows = nullptr;
  float* correct_rows = nullptr;
  const float* row_w = nullptr;
  (void)labels; (void)scale; (void)scale_dev; (void)loss_rows; (void)correct_rows; (void)row_w;
  constexpr int BM = Cfg::BM, BN = Cfg::BN, STAGE = Cfg::STAGE, NW = Cfg::NW, NU = Cfg::NU;
  __shared__ __attribute__((aligned(16))) float smem[Cfg::FLOATS];
  float (*red)[WC][BM] = nullptr;
  (void)red;

  const int nwg = static_cast<int>(gridDim.x);
  const int b = static_cast<int>(blockIdx.x);
  const int xcd = b % 8, qq = nwg / 8, rr = nwg % 8;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
  const int row_tile = tile / n_col_tiles, col_tile = tile % n_col_tiles;
  const int64_t row0 = static_cast<int64_t>(row_tile) * BM;
  const int col0 = col_tile * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int j = lane & 15, q = lane >> 4;
  const int colw = col0 + wc * G * 64;
  const int Kc = (K + 31) / 32;

  // DMA sources, through buffer descriptors re-based every chunk (scalar work only; the lane
  // offsets are constants): instruction i < NGA fills A image rows 8i .. 8i+7 (8 slots, key
  // r & 7), the others plane p = (i - NGA) / NGP, plane rows 16 ib .. 16 ib + 15 (4 slots, key
  // nt_key<4>). A's range ends at the tile's last row's round4(K): the K-tail chunk's segments
  // past it read 0 (rows inside read their neighbours' floats, zeroed in registers below).
  static_assert(Cfg::NGA % NW == 0, "A and B DMA instructions split at a whole u");
  constexpr int UA = Cfg::NGA / NW;
  int voff[NU];
  const int rows_here = static_cast<int>(M - row0 < BM ? M - row0 : BM);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int i = wave + NW * u;
    if (u < UA) {
      const int r = 8 * i + lane / 8;
      const int rl = r < rows_here ? r : rows_here - 1;
      voff[u] = (rl * static_cast<int>(lda) + 4 * ((lane % 8) ^ (r & 7))) * 4;
    } else {
      const int ib = i - Cfg::NGA;
      const int p = ib / Cfg::NGP;
      const int rb = (ib % Cfg::NGP) * 16 + lane / 4;
      const int sl = (lane % 4) ^ nt_key<4>(rb);
      int n = col0 + (rb & ~63) + 4 * (rb & 15) + ((rb >> 4) & 3);
      n = n < N ? n : N - 1;
      voff[u] = ((n * Kc) * 3 + p) * 64 + 16 * sl;
    }
  }
  const int a_bytes = ((rows_here - 1) * static_cast<int>(lda) + ((K + 3) & ~3)) * 4;
  const int b_bytes = N * Kc * 192;
  auto issue = [&](int chunk) {
    float* stage = smem + (chunk % S) * STAGE;
    const auto ra = brsrc(A + row0 * lda + 32 * chunk, a_bytes - 128 * chunk);
    const auto rbs = brsrc(Bs + 48 * chunk, b_bytes - 192 * chunk);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = wave + NW * u;
      if (NU * NW != Cfg::NG && i >= Cfg::NG) break;  // wave-uniform
      blds16(u < UA ? ra : rbs, stage + i * 256, voff[u]);
    }
  };
  auto lds_barrier = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f4 acc[RT][G][4];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][g][e] = f4{0.f, 0.f, 0.f, 0.f};

  f4 bv[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    bv[g] = f4{0.f, 0.f, 0.f, 0.f};
    const int c = colw + 64 * g + 4 * j;
    if (bias != nullptr) {
      if (c + 3 < N) {
        bv[g] = f4{bias[c], bias[c + 1], bias[c + 2], bias[c + 3]};
      } else {
        if (c < N) bv[g].x = bias[c];
        if (c + 1 < N) bv[g].y = bias[c + 1];
        if (c + 2 < N) bv[g].z = bias[c + 2];
      }
    }
  }

  const int arow0 = wr * 16 * RT + j;
  const int brow0 = wc * G * 64 + j;
  for (int c = 0; c < S - 1; ++c)
    if (c < Kc) issue(c);
  // one chunk; tp: the packed K tail (mfma6), only the peeled last chunk of a TP kernel
  auto chunk_body = [&](int c, auto tp) {
    if constexpr (S == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (c + S - 2 < Kc) {
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"((S - 2) * Cfg::PER_WAVE) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    lds_barrier();
    const float* stage = smem + (c % S) * STAGE;
    const int kc0 = c * 32;
    if (c + S - 1 < Kc) issue(c + S - 1);
    // A fragments (two 16-B reads per tile), masked past K, split into planes
    bf8 ap[RT][3];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const int r = arow0 + 16 * t;
      const f4 lo = *reinterpret_cast<const f4*>(stage + r * 32 + 4 * (q ^ (r & 7)));
      const f4 hi = *reinterpret_cast<const f4*>(stage + r * 32 + 4 * ((4 + q) ^ (r & 7)));
      f8 x = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (kc0 + 32 > K) {
        const int lim = K - kc0 - 4 * q;  // lo element w: k = kc0 + 4q + w; hi: + 16
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          x[w] = w < lim ? x[w] : 0.f;
          x[4 + w] = 16 + w < lim ? x[4 + w] : 0.f;
        }
      }
      split3(x, ap[t][0], ap[t][1], ap[t][2]);
    }
    const float* bsec = stage + Cfg::A_FLOATS;
    auto mm = [&](auto tp) {  // tp: the packed K tail (mfma6)
      constexpr bool TPC = decltype(tp)::value;
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rb = brow0 + 64 * g + 16 * e;
          const int so = rb * 16 + 4 * (q ^ nt_key<4>(rb));
          const bf8 b0 = __builtin_bit_cast(bf8, *reinterpret_cast<const f4*>(bsec + so));
          const bf8 b1 = __builtin_bit_cast(bf8, *reinterpret_cast<const f4*>(bsec + Cfg::P_FLOATS + so));
          const bf8 b2 = __builtin_bit_cast(bf8, *reinterpret_cast<const f4*>(bsec + 2 * Cfg::P_FLOATS + so));
#pragma unroll
          for (int t = 0; t < RT; ++t)
            acc[t][g][e] = mfma6<TPC>(ap[t], b0, b1, b2, acc[t][g][e]);
        }
    };
    if constexpr (decltype(tp)::value) {
#pragma unroll
      for (int t = 0; t < RT; ++t) pack_tail_a(ap[t]);
    }
    mm(tp);
  };
  const int n_full = TP ? Kc - 1 : Kc;
  for (int c = 0; c < n_full; ++c) chunk_body(c, std::false_type{});
  if constexpr (TP) chunk_body(n_full, std::true_type{});
  if (tile_nonfinite<RT, G>(acc, N, colw, j))  // f32 semantics for Inf / huge operands
    f32_tile<RT, G>(acc, M, N, K, A, lda, row0 + wr * 16 * RT, Bt, ldbt, 1, colw, j, q);
#define GCG_EPI_BV_READY
#include "gemm_epilogue.inc"
#undef GCG_EPI_BV_READY
}

// gemm_nt3r_kernel<RT, G, WR, WC>: gemm_nt3_kernel with A loaded straight into registers (each
// wave owns its 16 RT rows, so an LDS stage of A is shared by nobody when WC = 1): two
// dwordx4 buffer loads per row tile and chunk through a descriptor re-based every chunk, one
// chunk ahead (two register sets, the chunk loop unrolled by two), while only the weight's
// planes go through the LDS-DMA ring (12 KB per 64 columns and chunk, two stages), so more
// workgroups fit per CU.
template <int RT, int G, int WR, int WC>
struct Nt3rCfg {
  static constexpr int NW = WR * WC;
  static constexpr int BM = 16 * RT * WR;
  static constexpr int BN = 64 * G * WC;
  static constexpr int P_FLOATS = BN * 16;
  static constexpr int STAGE = 3 * P_FLOATS;
  static constexpr int NGP = BN / 16;
  static constexpr int NG = 3 * NGP;
  static constexpr int NU = (NG + NW - 1) / NW;
  static constexpr int FLOATS = 2 * STAGE;
  static constexpr int OCC_LDS = (160 * 1024) / (FLOATS * 4);
  static constexpr int OCC_REG = RT * G >= 4 ? 2 : 4;  // 4 x 4 accumulator tiles: <= 256 VGPRs
  static constexpr int OCC = OCC_LDS < 1 ? 1 : (OCC_LDS > OCC_REG ? OCC_REG : OCC_LDS);
};

template <int RT, int G, int WR, int WC, int V = 0>
__global__ __launch_bounds__(64 * WR * WC, (Nt3rCfg<RT, G, WR, WC>::OCC)) void
gemm_nt3r_kernel(int M, int N, int K, const float* __restrict__ A, int64_t lda,
                 const unsigned* __restrict__ Bs, const float* __restrict__ Bt, int64_t ldbt, const float* __restrict__ bias, int act,
                 float* __restrict__ Cout, int64_t ldc, int n_col_tiles) {
  using Cfg = Nt3rCfg<RT, G, WR, WC>;
  constexpr bool PL = (V & 1) != 0;
  constexpr bool TP = (V & 2) != 0;
  constexpr int EPI = 0;
  const int32_t* labels = nullptr;
  float scale = 0.f;
  const float* scale_dev = nullptr;
  float* loss_rows = nullptr;
  float* correct_rows = nullptr;
  const float* row_w = nullptr;
  (void)labels; (void)scale; (void)scale_dev; (void)loss_rows; (void)correct_rows; (void)row_w;
  constexpr int BM = Cfg::BM, BN = Cfg::BN, STAGE = Cfg::STAGE, NW = Cfg::NW, NU = Cfg::NU;
  __shared__ __attribute__((aligned(16))) float smem[Cfg::FLOATS];
  float (*red)[WC][BM] = nullptr;
  (void)red;

  const int nwg = static_cast<int>(gridDim.x);
  const int b = static_cast<int>(blockIdx.x);
  const int xcd = b % 8, qq = nwg / 8, rr = nwg % 8;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
  const int row_tile = tile / n_col_tiles, col_tile = tile % n_col_tiles;
  const int64_t row0 = static_cast<int64_t>(row_tile) * BM;
  const int col0 = col_tile * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int j = lane & 15, q = lane >> 4;
  const int colw = col0 + wc * G * 64;
  const int Kc = (K + 31) / 32;
  const int rows_here = static_cast<int>(M - row0 < BM ? M - row0 : BM);

  // weight planes: LDS-DMA instruction i fills plane p = i / NGP, rows 16 (i % NGP) .. + 15
  int voff[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int i = wave + NW * u;
    const int p = i / Cfg::NGP;
    const int rb = (i % Cfg::NGP) * 16 + lane / 4;
    const int sl = (lane % 4) ^ nt_key<4>(rb);
    int n = col0 + (rb & ~63) + 4 * (rb & 15) + ((rb >> 4) & 3);
    n = n < N ? n : N - 1;
    voff[u] = ((n * Kc) * 3 + p) * 64 + 16 * sl;
  }
  // A: lane (j, q) of row tile t reads row wr*16RT + 16t + j, k = 4q..4q+3 and 16+4q..16+4q+3
  int aoff[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    int r = wr * 16 * RT + 16 * t + j;
    r = r < rows_here ? r : rows_here - 1;
    aoff[t] = (r * static_cast<int>(lda) + 4 * q) * 4;
  }
  const int a_bytes = ((rows_here - 1) * static_cast<int>(lda) + ((K + 3) & ~3)) * 4;
  const int b_bytes = N * Kc * 192;
  auto issue_b = [&](int chunk) {
    float* stage = smem + (chunk & 1) * STAGE;
    const auto rbs = brsrc(Bs + 48 * chunk, b_bytes - 192 * chunk);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = wave + NW * u;
      if (NU * NW != Cfg::NG && i >= Cfg::NG) break;  // wave-uniform
      blds16(rbs, stage + i * 256, voff[u]);
    }
  };
  // (A keeps the default policy: the N / BN column tiles of a row block re-read its rows from
  // L2 -- non-temporal A loads measured 3.5-17 % slower, profiles/r05/nontemporal_streams.jsonl)
  auto load_a = [&](int chunk, f4 (&lo)[RT], f4 (&hi)[RT]) {
    const auto ra = brsrc(A + row0 * lda + 32 * chunk, a_bytes - 128 * chunk);
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      lo[t] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, aoff[t], 0, 0));
      hi[t] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, aoff[t] + 64, 0, 0));
    }
  };

  f4 acc[RT][G][4];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][g][e] = f4{0.f, 0.f, 0.f, 0.f};

  f4 bv[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    bv[g] = f4{0.f, 0.f, 0.f, 0.f};
    const int c = colw + 64 * g + 4 * j;
    if (bias != nullptr) {
      if (c + 3 < N) {
        bv[g] = f4{bias[c], bias[c + 1], bias[c + 2], bias[c + 3]};
      } else {
        if (c < N) bv[g].x = bias[c];
        if (c + 1 < N) bv[g].y = bias[c + 1];
        if (c + 2 < N) bv[g].z = bias[c + 2];
      }
    }
  }

  const int brow0 = wc * G * 64 + j;
  // tp: the packed K tail (mfma6) -- only the peeled last chunk of a TP kernel
  auto step = [&](int c, f4 (&lo)[RT], f4 (&hi)[RT], f4 (&nlo)[RT], f4 (&nhi)[RT], auto tp) {
    constexpr bool TPC = decltype(tp)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk c: its A registers and B planes
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + 1 < Kc) {
      issue_b(c + 1);
      load_a(c + 1, nlo, nhi);
    }
    const int kc0 = c * 32;
    const float* bsec = smem + (c & 1) * STAGE;
    // PL = 1: the weight planes of slot (g, e) + 1 are read from LDS before slot (g, e)'s
    // MFMAs are issued (the scheduler is fenced at each slot), so a read's latency hides behind
    // RT x 6 MFMAs instead of being waited on right before its own
    auto rd_planes = [&](int ge, bf8 (&bb)[3]) {
      const int rb = brow0 + 64 * (ge >> 2) + 16 * (ge & 3);
      const int so = rb * 16 + 4 * (q ^ nt_key<4>(rb));
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bb[p] = __builtin_bit_cast(bf8, *reinterpret_cast<const f4*>(bsec + p * Cfg::P_FLOATS + so));
    };
    bf8 bq[2][3];
    if constexpr (PL) rd_planes(0, bq[0]);
    bf8 ap[RT][3];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      f8 x = {lo[t][0], lo[t][1], lo[t][2], lo[t][3], hi[t][0], hi[t][1], hi[t][2], hi[t][3]};
      if (kc0 + 32 > K) {
        const int lim = K - kc0 - 4 * q;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          x[w] = w < lim ? x[w] : 0.f;
          x[4 + w] = 16 + w < lim ? x[4 + w] : 0.f;
        }
      }
      split3(x, ap[t][0], ap[t][1], ap[t][2]);
    }
    auto mm = [&](auto tp) {  // tp: the packed K tail (mfma6)
      constexpr bool TPC = decltype(tp)::value;
      if constexpr (PL) {
#pragma unroll
        for (int ge = 0; ge < 4 * G; ++ge) {
          if (ge + 1 < 4 * G) rd_planes(ge + 1, bq[(ge + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
          const int g = ge >> 2, e = ge & 3;
          const bf8 (&bb)[3] = bq[ge & 1];
#pragma unroll
          for (int t = 0; t < RT; ++t)
            acc[t][g][e] = mfma6<TPC>(ap[t], bb[0], bb[1], bb[2], acc[t][g][e]);
        }
        return;
      }
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rb = brow0 + 64 * g + 16 * e;
          const int so = rb * 16 + 4 * (q ^ nt_key<4>(rb));
          const bf8 b0 = __builtin_bit_cast(bf8, *reinterpret_cast<const f4*>(bsec + so));
          const bf8 b1 = __builtin_bit_cast(bf8, *reinterpret_cast<const f4*>(bsec + Cfg::P_FLOATS + so));
          const bf8 b2 = __builtin_bit_cast(bf8, *reinterpret_cast<const f4*>(bsec + 2 * Cfg::P_FLOATS + so));
#pragma unroll
          for (int t = 0; t < RT; ++t)
            acc[t][g][e] = mfma6<TPC>(ap[t], b0, b1, b2, acc[t][g][e]);
        }
    };
    if constexpr (TPC) {
#pragma unroll
      for (int t = 0; t < RT; ++t) pack_tail_a(ap[t]);
    }
    mm(tp);
  };
  f4 alo[RT], ahi[RT], blo[RT], bhi[RT];
  issue_b(0);
  load_a(0, alo, ahi);
  // TP (V & 2, chosen by the host when the last chunk holds <= 16 live k): the loop runs the
  // full chunks and the last one is peeled, packed (no branch between two MFMA paths in one
  // kernel: that doubled the register pressure and spilled)
  const int Kf = TP ? Kc - 1 : Kc;
  for (int c = 0; c < Kf; c += 2) {
    step(c, alo, ahi, blo, bhi, std::false_type{});
    if (c + 1 < Kf) step(c + 1, blo, bhi, alo, ahi, std::false_type{});
  }
  if constexpr (TP) {
    if (Kf & 1) {  // the tail's A arrived in the second set
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        alo[t] = blo[t];
        ahi[t] = bhi[t];
      }
    }
    step(Kf, alo, ahi, blo, bhi, std::true_type{});
  }
  if (tile_nonfinite<RT, G>(acc, N, colw, j))  // f32 semantics for Inf / huge operands
    f32_tile<RT, G>(acc, M, N, K, A, lda, row0 + wr * 16 * RT, Bt, ldbt, 1, colw, j, q);
#define GCG_EPI_BV_READY
// C is written once and read by the next kernel long after L2 has turned over (840k x 930 =
// 3.1 GB): non-temporal stores keep the weight planes and the row blocks' A in L2 (K = 300
// projections +4 %, K = 930 unchanged, profiles/r05/nontemporal_streams.jsonl)
#define GCG_EPI_NT true
#include "gemm_epilogue.inc"
#undef GCG_EPI_BV_READY
#undef GCG_EPI_NT
}

// ---------------------------------------------------------------------------------------
// gemm_fused6_kernel<RT, G>: the fused output layer (gemm_kernel EPI = 1: P . W + b -> softmax,
// cross-entropy, hits, logits gradient / probabilities) with the products on the bf16 matrix
// cores (bf16x6, as gcg_gemm_nt_f32_bf16x6; round 4). A workgroup owns 16 RT whole rows: 4
// waves x 64 G columns (N <= 256 G). A goes through the LDS-DMA ring (the nt3 image: [BM][8
// slots], key r & 7; each wave reads all rows) and is split in registers; the weight W
// (K x N, L2-resident) is read straight into registers as f32, one dwordx4 of 4 adjacent columns
// per lane and k row -- rows k0 + 4q + i and k0 + 16 + 4q + i (i < 4) give, per column, the 8
// k-values of the lane's bf16 operand in the A image's k order -- and split in registers; the
// next 64-column group's 8 loads are in flight while a group computes. Weight rows past K read
// as 0 (buffer range), A's elements past K are zeroed before the split, W's padding columns
// are handled by the epilogue's straddle guard. All LDS (ring, row reductions, bias, labels,
// row weights) is one array: a second __shared__ object makes hipcc drain the DMA queue.
// Round 5: A (each row read by exactly one workgroup) is DMA'd and the logits gradient stored
// with the non-temporal policy, so these streams (1 GB in, 3.1 GB out at Twitter-World) stop
// evicting the weight planes every workgroup re-reads from L2: World 139.4-140.1 -> 147.6-148.6
// TF (bf16x6), Twitter-US and the f32 forms unchanged (profiles/r05/nontemporal_streams.jsonl).
// ---------------------------------------------------------------------------------------
// CS = 1 (round 5, FX only): the A chunk is split cooperatively -- each of the workgroup's
// threads splits one 16-B k-quad of one row (BM x 8 quads = the thread count) and writes its
// three planes to an LDS image ([plane][BM rows][4 slots of 16 B], key nt_key<4>, the NT
// kernel's conflict-free B image), then every wave reads its RT x 3 plane fragments from it --
// instead of all WR x WC waves splitting all BM rows in registers; one more barrier per chunk.
// TP: the packed K tail (mfma6): the last chunk peeled, packed (host: when it holds <= 16 k).
template <int RT, int G, int WR = 1, int WC = 4, int SB = 0, int FX = 0, int CS = 0, bool TP = false>
__global__ __launch_bounds__(64 * WR * WC, WR * WC == 4 ? 2 : 1) void gemm_fused6_kernel(
    int M, int N, int K, const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
    int64_t ldb, const float* __restrict__ bias, float* __restrict__ Cout, int64_t ldc,
    const int32_t* __restrict__ labels, float scale, const float* __restrict__ scale_dev,
    float* __restrict__ loss_rows, float* __restrict__ correct_rows,
    const float* __restrict__ row_w, const unsigned* __restrict__ Wsplit = nullptr) {
  constexpr int EPI = 1, S = 2;
  constexpr int BM = 16 * RT * WR, BN = 64 * G * WC;
  constexpr int STAGE = BM * 32;                 // A image floats per stage
  constexpr int NGA = BM / 8;                    // A DMA wave-instructions per stage
  constexpr int UA = NGA / (WR * WC);
  static_assert(NGA % (WR * WC) == 0, "whole A DMA instructions per wave");
  constexpr int OFF_RED = S * STAGE, OFF_BIAS = OFF_RED + 4 * WC * BM;
  constexpr int OFF_LAB = OFF_BIAS + BN, OFF_RW = OFF_LAB + BM;
  constexpr int OFF_PL = OFF_RW + BM, PL_FLOATS = BM * 16;  // (CS) plane p image at p * PL_FLOATS
  __shared__ __attribute__((aligned(16))) float smem[OFF_PL + (CS ? 3 * PL_FLOATS : 0)];
  static_assert(!CS || (FX && BM * 8 == 64 * WR * WC), "CS: one k-quad of one row per thread");
  float (*red)[WC][BM] = reinterpret_cast<float (*)[WC][BM]>(smem + OFF_RED);
  float* sbias = smem + OFF_BIAS;
  int* slab = reinterpret_cast<int*>(smem + OFF_LAB);
  float* srw = smem + OFF_RW;
  const int act = GCG_ACT_NONE;
  (void)act;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;
  const int j = lane & 15, q = lane >> 4;
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
  const int colw = wc * G * 64;
  const int Kc = (K + 31) / 32;
  const int rows_here = static_cast<int>(M - row0 < BM ? M - row0 : BM);
  const int n4 = (N + 3) & ~3;

  // A DMA: instruction i = wave + WC u fills image rows 8i .. 8i + 7
  int voff[UA];
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int r = 8 * (wave + WR * WC * u) + lane / 8;
    const int rl = r < rows_here ? r : rows_here - 1;
    voff[u] = (rl * static_cast<int>(lda) + 4 * ((lane % 8) ^ (r & 7))) * 4;
  }
  const int a_bytes = ((rows_here - 1) * static_cast<int>(lda) + ((K + 3) & ~3)) * 4;
  auto issue_a = [&](int chunk) {
    float* stage = smem + (chunk & 1) * STAGE;
    const auto ra = brsrc(A + row0 * lda + 32 * chunk, a_bytes - 128 * chunk);
#pragma unroll
    for (int u = 0; u < UA; ++u) blds16_nt(ra, stage + (wave + WR * WC * u) * 256, voff[u]);
  };
  // W: lane offsets (row 4q, column of group g); rows i and 16 + i through the scalar offset
  int bofs[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int c = colw + 64 * g + 4 * j;
    bofs[g] = ((4 * q) * static_cast<int>(ldb) + (c < n4 ? c : 0)) * 4;
  }
  const int ldb4 = static_cast<int>(ldb) * 4;
  auto load_w = [&](int chunk, int g, f4 (&w)[8]) {
    const int k0 = 32 * chunk;
    const auto rw = brsrc(B + static_cast<int64_t>(k0) * ldb, (K - k0) * ldb4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rw, bofs[g], i * ldb4, 0));
      w[4 + i] = __builtin_bit_cast(
          f4, __builtin_amdgcn_raw_buffer_load_b128(rw, bofs[g], (16 + i) * ldb4, 0));
    }
  };

  f4 acc[RT][G][4];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][g][e] = f4{0.f, 0.f, 0.f, 0.f};

  for (int c = tid; c < BN; c += 64 * WR * WC)  // columns past N: -inf (softmax weight 0)
    sbias[c] = c < N ? (bias != nullptr ? bias[c] : 0.f) : kNegInf;
  for (int r = tid; r < BM; r += 64 * WR * WC) {
    const int64_t row = row0 + r;
    int y = (labels != nullptr && row < M) ? labels[row] : -1;
    if (labels != nullptr && (y < 0 || y >= N)) y = -2;  // outside [0, N): NaN loss, no hit
    slab[r] = y;
    srw[r] = (row_w != nullptr && row < M) ? row_w[row] : 1.f;
  }
  __syncthreads();
  // the bias is the accumulators' starting value (b + sum of products), so the epilogue adds
  // nothing per element; columns past N start at 0 and become -inf in the epilogue (round 6:
  // +3 %, every wave of the CU's one workgroup runs the epilogue with the matrix pipe idle)
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const f4 bb = *reinterpret_cast<const f4*>(&sbias[colw + 64 * g + 4 * j]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float b0 = colw + 64 * g + 4 * j + e < N ? bb[e] : 0.f;
#pragma unroll
      for (int t = 0; t < RT; ++t) acc[t][g][e] = f4{b0, b0, b0, b0};
    }
  }

  const int ngv = min(G, max(0, (N - colw + 63) / 64));  // groups with a column < N
  const int arow0 = wr * 16 * RT + j;
  f4 w0[8], w1[8];
  issue_a(0);
  if constexpr (!FX) {
    if (ngv > 0) load_w(0, 0, w0);
  }
  // (tp in the group forms below: the packed K tail, mfma6)
  auto group = [&](int c, int g, const bf8 (&ap)[RT][3], const f4 (&w)[8], f4 (&wn)[8], auto tp) {
    constexpr bool TPC = decltype(tp)::value;
    // prefetch the next group (or the next chunk's first) into the other set
    if (g + 1 < ngv) load_w(c, g + 1, wn);
    else if (c + 1 < Kc && ngv > 0) load_w(c + 1, 0, wn);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f8 y = {w[0][e], w[1][e], w[2][e], w[3][e], w[4][e], w[5][e], w[6][e], w[7][e]};
      bf8 b0, b1, b2;
      split3(y, b0, b1, b2);
#pragma unroll
      for (int t = 0; t < RT; ++t)
        acc[t][g][e] = mfma6<TPC>(ap[t], b0, b1, b2, acc[t][g][e]);
    }
  };
  // SB = 1 (one W register set, for tiles whose accumulators leave no room for two): the next
  // group's loads go into the set as soon as its last column slot is split, so they fly during
  // that slot's MFMAs and the other waves' work
  auto group_sb = [&](int c, int g, const bf8 (&ap)[RT][3], f4 (&w)[8], auto tp) {
    constexpr bool TPC = decltype(tp)::value;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const f8 y = {w[0][e], w[1][e], w[2][e], w[3][e], w[4][e], w[5][e], w[6][e], w[7][e]};
      bf8 b0, b1, b2;
      split3(y, b0, b1, b2);
      if (e == 3) {
        if (g + 1 < ngv) load_w(c, g + 1, w);
        else if (c + 1 < Kc && ngv > 0) load_w(c + 1, 0, w);
      }
#pragma unroll
      for (int t = 0; t < RT; ++t)
        acc[t][g][e] = mfma6<TPC>(ap[t], b0, b1, b2, acc[t][g][e]);
    }
  };
  // FX = 1: W's bf16 planes pre-split into a workspace [BN][Kc][3][32] (split3_rows_kernel, zero
  // past N): per group and chunk 12 loads of 16 B (4 column slots x 3 planes) and no split; the
  // slot's column n = colw + 64 g + e + 4 j gives the scalar part (colw + 64 g + e) * Kc * 192
  // layout (split3_rows_kernel, n_out = BN): [c][plane][BN / 64][e][j][q], 16 B per (j, q)
  const int wlane = 64 * j + 16 * q;
  constexpr int NG64 = BN / 64;
  // the 3 planes of slot e (columns colw + 64 g + e + 4 j) of one chunk and group
  auto load_slot = [&](int chunk, int g, int e, f4 (&wp)[12]) {
    // one chunk = 3 planes x NG64 groups x 4 slots x 1024 B
    const auto rs = brsrc(Wsplit + chunk * 3 * NG64 * 1024, (Kc - chunk) * 3 * NG64 * 4096);
    const int gq = colw / 64 + g;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      wp[3 * e + p] = __builtin_bit_cast(
          f4, __builtin_amdgcn_raw_buffer_load_b128(rs, wlane, ((p * NG64 + gq) * 4 + e) * 1024, 0));
  };
  auto load_p = [&](int chunk, int g, f4 (&wp)[12]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) load_slot(chunk, g, e, wp);
  };
  // one register set, refilled slot by slot: once slot e's MFMAs are issued its registers take
  // the next group's (or the next chunk's first group's) slot e, so each load has three slots
  // of MFMAs (and the other waves' work) to land in
  auto group_fx = [&](int c, int g, const bf8 (&ap)[RT][3], f4 (&wp)[12], auto tp) {
    constexpr bool TPC = decltype(tp)::value;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bf8 b0 = __builtin_bit_cast(bf8, wp[3 * e]);
      const bf8 b1 = __builtin_bit_cast(bf8, wp[3 * e + 1]);
      const bf8 b2 = __builtin_bit_cast(bf8, wp[3 * e + 2]);
#pragma unroll
      for (int t = 0; t < RT; ++t)
        acc[t][g][e] = mfma6<TPC>(ap[t], b0, b1, b2, acc[t][g][e]);
      if (g + 1 < ngv) load_slot(c, g + 1, e, wp);
      else if (c + 1 < Kc && ngv > 0) load_slot(c + 1, 0, e, wp);
    }
  };
  f4 wpl[FX ? 12 : 1];
  // one chunk; wa holds its first group's W on entry. G even: the next chunk's first group
  // ends in wa again, G odd (G = 1, 3): in wb, so the loop alternates the sets (a wave whose
  // live-group count has the other parity -- it straddles N -- moves it)
  auto chunk = [&](int c, f4 (&wa)[8], f4 (&wb)[8], auto tp) {
    // A(c) landed. FX with live groups: the last 12 loads issued (this chunk's first group of
    // planes, prefetched by the previous chunk's last group or the prologue) may still fly
    if (FX && ngv > 0) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (and W's prefetch)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + 1 < Kc) issue_a(c + 1);
    const int kc0 = 32 * c;
    const float* stage = smem + (c & 1) * STAGE;
    bf8 ap[RT][3];
    if constexpr (CS) {
      // thread (row r = tid / 8, quad kq = tid % 8: k = kc0 + 4 kq .. + 3) splits its 4 floats;
      // MFMA operand position of k: slot q = kq & 3, half kq >> 2 (low: k = 4q + w, high: 16 +
      // 4q + w) -- 8 B of the slot per plane
      const int r = tid >> 3, kq = tid & 7;
      f4 x = *reinterpret_cast<const f4*>(stage + r * 32 + 4 * (kq ^ (r & 7)));
      if (kc0 + 32 > K) {
        const int lim = K - kc0 - 4 * kq;
#pragma unroll
        for (int w = 0; w < 4; ++w) x[w] = w < lim ? x[w] : 0.f;
      }
      f2 lo2 = {x[0], x[1]}, hi2 = {x[2], x[3]};
      unsigned pw[3][2];
      pw[0][0] = split_pair(lo2);
      pw[0][1] = split_pair(hi2);
      pw[1][0] = split_pair(lo2);
      pw[1][1] = split_pair(hi2);
      pw[2][0] = __builtin_bit_cast(unsigned, __builtin_convertvector(lo2, bf2));
      pw[2][1] = __builtin_bit_cast(unsigned, __builtin_convertvector(hi2, bf2));
      const int so = r * 16 + 4 * ((kq & 3) ^ nt_key<4>(r)) + 2 * (kq >> 2);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        using u2v = __attribute__((ext_vector_type(2))) unsigned;
        *reinterpret_cast<u2v*>(smem + OFF_PL + p * PL_FLOATS + so) = u2v{pw[p][0], pw[p][1]};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const int rr = arow0 + 16 * t;
        const int ro = rr * 16 + 4 * (q ^ nt_key<4>(rr));
#pragma unroll
        for (int p = 0; p < 3; ++p)
          ap[t][p] = __builtin_bit_cast(bf8, *reinterpret_cast<const f4*>(smem + OFF_PL + p * PL_FLOATS + ro));
      }
    }
#pragma unroll
    for (int t = 0; t < (CS ? 0 : RT); ++t) {
      const int r = arow0 + 16 * t;
      const f4 lo = *reinterpret_cast<const f4*>(stage + r * 32 + 4 * (q ^ (r & 7)));
      const f4 hi = *reinterpret_cast<const f4*>(stage + r * 32 + 4 * ((4 + q) ^ (r & 7)));
      f8 x = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (kc0 + 32 > K) {
        const int lim = K - kc0 - 4 * q;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          x[w] = w < lim ? x[w] : 0.f;
          x[4 + w] = 16 + w < lim ? x[4 + w] : 0.f;
        }
      }
      split3(x, ap[t][0], ap[t][1], ap[t][2]);
    }
    auto groups = [&](auto tp) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (g >= ngv) break;  // wave-uniform: groups wholly past N
        if constexpr (FX) {
          group_fx(c, g, ap, wpl, tp);
        } else if constexpr (SB) {
          group_sb(c, g, ap, wa, tp);
        } else if (g % 2 == 0) {
          group(c, g, ap, wa, wb, tp);
        } else {
          group(c, g, ap, wb, wa, tp);
        }
      }
    };
    if constexpr (decltype(tp)::value) {
#pragma unroll
      for (int t = 0; t < RT; ++t) pack_tail_a(ap[t]);
    }
    groups(tp);
    // the last live group (ngv - 1) prefetched the next chunk's first into wb when ngv is odd
    if (!SB && !FX && ngv > 0 && c + 1 < Kc) {
      const bool in_b = (ngv & 1) != 0;
      if constexpr (G % 2 == 0) {
        if (in_b) {
#pragma unroll
          for (int i = 0; i < 8; ++i) wa[i] = wb[i];
        }
      } else {
        if (!in_b) {
#pragma unroll
          for (int i = 0; i < 8; ++i) wb[i] = wa[i];
        }
      }
    }
  };
  if constexpr (FX) {
    if (ngv > 0) load_p(0, 0, wpl);
  }
  const int Kf = TP ? Kc - 1 : Kc;  // full chunks; TP: the last one peeled, packed
  if constexpr (G % 2 == 0 || SB || FX) {
    for (int c = 0; c < Kf; ++c) chunk(c, w0, w1, std::false_type{});
    if constexpr (TP) chunk(Kf, w0, w1, std::true_type{});
  } else {
    for (int c = 0; c < Kf; c += 2) {
      chunk(c, w0, w1, std::false_type{});
      if (c + 1 < Kf) chunk(c + 1, w1, w0, std::false_type{});
    }
    if constexpr (TP) {
      if (Kf & 1) {  // the tail's first group arrived in the second set
#pragma unroll
        for (int i = 0; i < 8; ++i) w0[i] = w1[i];
      }
      chunk(Kf, w0, w1, std::true_type{});
    }
  }
  if (tile_nonfinite<RT, G, FX == 0>(acc, N, colw, j)) {  // f32 semantics (see tile_nonfinite)
    f32_tile<RT, G>(acc, M, N, K, A, lda, row0 + wr * 16 * RT, B, 1, ldb, colw, j, q);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = colw + 64 * g + 4 * j + e;
        const float b0 = c < N ? sbias[c] : 0.f;
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t][g][e][r] += b0;
      }
  }
#define GCG_EPI_BV_READY
#define GCG_EPI_LABELS_LDS
#define GCG_EPI_BIAS_IN_ACC
#define GCG_EPI_NT true
  f4 bv[G];
#pragma unroll
  for (int g = 0; g < G; ++g) bv[g] = *reinterpret_cast<const f4*>(&sbias[colw + 64 * g + 4 * j]);
#include "gemm_epilogue.inc"
#undef GCG_EPI_BV_READY
#undef GCG_EPI_LABELS_LDS
#undef GCG_EPI_BIAS_IN_ACC
#undef GCG_EPI_NT
}

// One wave per row: the row (N <= 256*NV) is read once into registers, then max, sum of
// exp, label logit and first-index argmax, then dlogits / probabilities. In-place safe.
template <int NV>
__global__ __launch_bounds__(256) void softmax_xent_rows_kernel(
    int M, int N, const float* __restrict__ L, int64_t ldl, const int32_t* __restrict__ labels,
    float scale, const float* __restrict__ scale_dev, float* O, int64_t ldo,
    float* __restrict__ loss_rows, float* __restrict__ correct_rows,
    const float* __restrict__ row_w, int vec) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float w = row_w != nullptr ? row_w[row] : 1.f;  // target multiplicity (1 if none)
  const float* lrow = L + row * ldl;
  f4 v[NV];
  float m = kNegInf;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * (lane + 64 * i);
    if (vec && c + 3 < N) {
      v[i] = *reinterpret_cast<const f4*>(lrow + c);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i][e] = (c + e < N) ? lrow[c + e] : kNegInf;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) m = fmaxf(m, v[i][e]);
  }
  m = reduce16_max<64>(m);
  // a label outside [0, N) gets a NaN loss (never a silent wrong class); -1 = no labels
  int y = labels ? labels[row] : -1;
  const bool bad_y = labels != nullptr && (y < 0 || y >= N);
  y = bad_y ? -1 : y;
  float s = 0.f, x = 0.f;
  int a = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 4 * (lane + 64 * i) + e;
      s += expf(v[i][e] - m);
      x += (c == y) ? v[i][e] : 0.f;
      a = (v[i][e] == m && c < a) ? c : a;
    }
  s = reduce16_sum<64>(s);
  x = reduce16_sum<64>(x);
  a = reduce16_min<64>(a);
  if (labels != nullptr && lane == 0) {
    loss_rows[row] = bad_y ? std::numeric_limits<float>::quiet_NaN() : w * ((m + logf(s)) - x);
    if (correct_rows) correct_rows[row] = (!bad_y && a == y) ? w : 0.f;
  }
  if (O == nullptr) return;  // loss / accuracy only
  if (scale_dev != nullptr) scale *= *scale_dev;
  if (labels != nullptr) scale *= w;
  const float inv = 1.0f / s;
  float* orow = O + row * ldo;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = 4 * (lane + 64 * i);
    if (c >= N) continue;
    f4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float p = expf(v[i][e] - m) * inv;
      if (labels != nullptr) p = (p - ((c + e) == y ? 1.f : 0.f)) * scale;
      o[e] = p;
    }
    if (vec && c + 3 < N) {
      *reinterpret_cast<f4*>(orow + c) = o;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c + e < N) orow[c + e] = o[e];
    }
  }
}

// ---------------------------------------------------------------------------------------
// C = scale * A^T . B, the weight gradients h^T . g / P^T . G (Theano's grad of T.dot(h, W)
// w.r.t. W, mlpconv.py:88): reduction over R ~ 10^6 rows into a small M x N output.
// Split-K: blockIdx.z owns rows [z*rows_per_split, ...); each wave keeps a 64*MG x 64*NG
// accumulator tile. Lane (j, q) loads ONE dwordx4 of A's row t and one of B's row t per
// 64-wide group (t = t0 + q): element e of the A vector is row-slot j of the MFMA tile that
// owns the C rows m0 + 4j + e, element e' of the B vector the column-slot j of the tile owning
// the C columns n0 + 4j + e' -- so 2 loads feed 16 v_mfma_f32_16x16x4_f32 and a lane's
// accumulators hold 4 adjacent C columns (dwordx4 partial stores). A ring of PD register
// sets keeps PD steps of loads in flight. Partials [split][Mp][Np] are summed in split order
// by gemm_tn_reduce_kernel (deterministic), which applies scale (a device scalar).
// ---------------------------------------------------------------------------------------
// WM = 1: the workgroup's 4 waves sit side by side along N (tile 64*MG x 256*NG): they load
// the same A rows, and each 64-row band of C re-reads B. WM > 1 (round 3): WM waves stacked
// along M (tile 64*MG*WM x 64*NG, WM = 5 covers M = 300 in one tile): B -- the wide operand,
// G at 840k x 930 -- is read once per row and shared by the WM waves through L1, and the N
// tiles of one split (same XCD, remap) share A through L2.
// WM = 0 (round 3): every wave owns its own 64*MG x 64*NG tile, enumerated m fastest over
// (m tile, n tile, split), 4 consecutive wave tiles per workgroup (the 4 waves of a workgroup
// then share their B rows through L1), one wave per SIMD: the accumulators of a wide NG (3 or
// 5: N = 930 in 960 columns instead of the 1024 of 256-column workgroup tiles) live in the
// 512-register file beside a deep load ring.
// OCC = 2 keeps a per-wave (WM = 0) tile at 2 waves per SIMD (<= 256 registers: a shallow ring),
// so it can share CUs with kernels running beside it on other streams.
template <int MG, int NG, int PD, int WM = 1, int OCC = 0>
__global__ __launch_bounds__(WM <= 1 ? 256 : 64 * WM, (WM == 0 && OCC != 2) ? 1 : 2) void gemm_tn_partial_kernel(
    int R, int M, int N, const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
    int64_t ldb, int rows_per_split, float* __restrict__ part, int Mp, int Np, int mt, int nt,
    int remap) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane & 15, q = lane >> 4;
  // 1-D grid of mt x nt x S tiles, m fastest. remap: XCD-aware bijection (workgroup b runs on
  // XCD b % 8; each XCD walks one contiguous range of tiles), so the mt x nt tiles of one
  // split -- which read the same rows of A and B -- share one XCD's L2.
  const int nwg = static_cast<int>(gridDim.x), b = static_cast<int>(blockIdx.x);
  int tile = b;
  if (remap) {
    const int xcd = b % 8, qq = nwg / 8, rr = nwg % 8;
    tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
  }
  const int wt = WM == 0 ? 4 * tile + wave : tile;  // WM = 0: the wave's own tile
  const int bx = wt % mt, by = (wt / mt) % nt, bz = wt / (mt * nt);
  const int m0 = WM == 0   ? bx * (64 * MG)
                 : WM == 1 ? bx * (64 * MG)
                           : bx * (64 * MG * WM) + wave * (64 * MG);
  const int n0 = WM == 0   ? by * (64 * NG)
                 : WM == 1 ? by * (256 * NG) + wave * (64 * NG)
                           : by * (64 * NG);
  // a wave wholly past N (or M), or past the last split, leaves at once (no LDS, no barriers)
  if (n0 >= N || (WM != 1 && m0 >= M)) return;
  if (static_cast<int64_t>(bz) * rows_per_split >= R) return;
  const int t_begin = bz * rows_per_split;
  const int t_end = min(R, t_begin + rows_per_split);
  const int m4 = (M + 3) & ~3, n4 = (N + 3) & ~3;
  int acol[MG], bcol[NG];
#pragma unroll
  for (int g = 0; g < MG; ++g) {
    const int c = m0 + 64 * g + 4 * j;
    acol[g] = c < m4 ? c : 0;  // rows of C past M: computed on a valid column, never stored
  }
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int c = n0 + 64 * g + 4 * j;
    bcol[g] = c < n4 ? c : 0;
  }
  f4 acc[MG][NG][4][4];
#pragma unroll
  for (int a = 0; a < MG; ++a)
#pragma unroll
    for (int b = 0; b < NG; ++b)
#pragma unroll
      for (int ea = 0; ea < 4; ++ea)
#pragma unroll
        for (int eb = 0; eb < 4; ++eb) acc[a][b][ea][eb] = f4{0.f, 0.f, 0.f, 0.f};

  f4 ra[PD][MG], rb[PD][NG];
  // A and B rows through buffer descriptors re-based at the step's first row (scalar work): the
  // range check covers only the rows left in the split, so rows past it read as 0 -- no per-lane
  // row clamp, select or 64-bit address arithmetic (round 3; the per-lane byte offsets are
  // constants). Host: lda, ldb < 2^27.
  uint32_t aoff[MG], boff[NG];
#pragma unroll
  for (int g = 0; g < MG; ++g) aoff[g] = static_cast<uint32_t>((q * static_cast<int>(lda) + acol[g]) * 4);
#pragma unroll
  for (int g = 0; g < NG; ++g) boff[g] = static_cast<uint32_t>((q * static_cast<int>(ldb) + bcol[g]) * 4);
  auto load = [&](int u, int t0) {
    // (readfirstlane: the descriptor must be provably wave-uniform, or hipcc emits a waterfall)
    const int left = __builtin_amdgcn_readfirstlane(min(max(t_end - t0, 0), 4));  // rows in split
    const int tb = __builtin_amdgcn_readfirstlane(left > 0 ? t0 : t_begin);
    const auto ar = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(A + static_cast<int64_t>(tb) * lda), static_cast<short>(0),
        left * static_cast<int>(lda) * 4, 0x00020000);
    const auto br = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(B + static_cast<int64_t>(tb) * ldb), static_cast<short>(0),
        left * static_cast<int>(ldb) * 4, 0x00020000);
#pragma unroll
    for (int g = 0; g < MG; ++g)
      ra[u][g] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ar, aoff[g], 0, 0));
#pragma unroll
    for (int g = 0; g < NG; ++g)
      rb[u][g] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(br, boff[g], 0, 0));
  };
  auto compute = [&](int u) {
#pragma unroll
    for (int a = 0; a < MG; ++a)
#pragma unroll
      for (int b = 0; b < NG; ++b)
#pragma unroll
        for (int ea = 0; ea < 4; ++ea)
#pragma unroll
          for (int eb = 0; eb < 4; ++eb)
            acc[a][b][ea][eb] = mfma4(ra[u][a][ea], rb[u][b][eb], acc[a][b][ea][eb]);
  };
  // steps of 4 rows; the ring is refilled PD steps ahead (loads past t_end are zeroed)
#pragma unroll
  for (int u = 0; u < PD; ++u) {
    load(u, t_begin + 4 * u);
    __builtin_amdgcn_sched_barrier(0);  // issue order = ring order (counted waits below)
  }
  // The scheduling barriers pin each refill behind its step's MFMAs: without them the machine
  // scheduler sinks every load next to its use (to cut register pressure) and the ring is gone
  // -- one exposed load latency per step (round 2, ISA: vmcnt(0) before each step's MFMAs).
  for (int t0 = t_begin; t0 < t_end; t0 += 4 * PD) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      compute(u);
      __builtin_amdgcn_sched_barrier(0);
      load(u, t0 + 4 * (u + PD));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // partial tile: lane holds C[m0 + 64a + 16q + 4r + ea][n0 + 64b + 4j + eb] in acc[a][b][ea][eb][r]
  float* dst = part + static_cast<int64_t>(bz) * Mp * Np;
#pragma unroll
  for (int a = 0; a < MG; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int ea = 0; ea < 4; ++ea) {
        const int m = m0 + 64 * a + 16 * q + 4 * r + ea;
        float* row = dst + static_cast<int64_t>(m) * Np;
#pragma unroll
        for (int b = 0; b < NG; ++b) {
          const int n = n0 + 64 * b + 4 * j;
          *reinterpret_cast<f4*>(row + n) = f4{acc[a][b][ea][0][r], acc[a][b][ea][1][r],
                                               acc[a][b][ea][2][r], acc[a][b][ea][3][r]};
        }
      }
}

// gemm_tn6_partial_kernel (round 6): gemm_tn_partial_kernel's split-K A^T . B (the weight
// gradients dW2 = P^T . G and X_head^T . G) on the bf16 matrix cores (bf16x6, mfma6). Each wave
// owns a 64 (m) x 64 (n) tile of one split: per 32-row chunk, lane (j, q) loads rows
// t0 + 4q + i and t0 + 16 + 4q + i (i < 4) of A and B as dwordx4 of 4 adjacent columns (the
// fused layer's in-register weight load), which gives, for each of its 4 column slots e
// (column m0 + 4j + e), the 8 k-values of its MFMA fragment in the bf16x6 kernels' k order;
// the fragments are split into planes in registers. The D row rho of block (eA, eB) is
// m = m0 + 4 rho + eA, its column j is n = n0 + 4j + eB, so each lane stores 4 adjacent n of
// 16 rows. Rows past the split come from a buffer range that reads 0; columns past M / N are
// computed on a clamped column and never reach C (the reduce kernel reads m < M, n < N). A tile
// whose accumulators are not finite is recomputed with f32 products (v_mfma_f32_16x16x4_f32,
// one row t per k step) -- f32 semantics, as the other bf16x6 kernels.
__global__ __launch_bounds__(256, 2) void gemm_tn6_partial_kernel(
    int R, int M, int N, const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
    int64_t ldb, int rows_per_split, float* __restrict__ part, int Mp, int Np, int mt, int nt) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane & 15, q = lane >> 4;
  const int nwg = static_cast<int>(gridDim.x), b = static_cast<int>(blockIdx.x);
  const int xcd = b % 8, qq = nwg / 8, rr = nwg % 8;  // XCD-aware order, as gemm_tn_partial
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
  const int wt = 4 * tile + wave;
  const int bx = wt % mt, by = (wt / mt) % nt, bz = wt / (mt * nt);
  const int m0 = bx * 64, n0 = by * 64;
  if (m0 >= M || n0 >= N) return;  // wave-uniform; no barriers in this kernel
  if (static_cast<int64_t>(bz) * rows_per_split >= R) return;
  const int t_begin = bz * rows_per_split;
  const int rows = min(R, t_begin + rows_per_split) - t_begin;
  const int m4 = (M + 3) & ~3, n4 = (N + 3) & ~3;
  const int ac = m0 + 4 * j < m4 ? m0 + 4 * j : 0;
  const int bc = n0 + 4 * j < n4 ? n0 + 4 * j : 0;
  const int lda4 = static_cast<int>(lda) * 4, ldb4 = static_cast<int>(ldb) * 4;
  const float* Ab = A + static_cast<int64_t>(t_begin) * lda;
  const float* Bb = B + static_cast<int64_t>(t_begin) * ldb;
  const int aoff = 4 * q * lda4 + ac * 4, boff = 4 * q * ldb4 + bc * 4;
  const int nch = (rows + 31) / 32;
  auto load = [&](int c, f4 (&xa)[8], f4 (&xb)[8]) {
    const int live = min(rows - 32 * c, 32);  // rows of this chunk inside the split
    const auto ra = brsrc(Ab + static_cast<int64_t>(32 * c) * lda, live * lda4);
    const auto rb = brsrc(Bb + static_cast<int64_t>(32 * c) * ldb, live * ldb4);
    // (the row offset in the VGPR offset, which the range check covers: rows past the split
    // must read 0, they are the next split's)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xa[i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, aoff + i * lda4, 0, 0));
      xa[4 + i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, aoff + (16 + i) * lda4, 0, 0));
      xb[i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, boff + i * ldb4, 0, 0));
      xb[4 + i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, boff + (16 + i) * ldb4, 0, 0));
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int ea = 0; ea < 4; ++ea)
#pragma unroll
    for (int eb = 0; eb < 4; ++eb) acc[ea][eb] = f4{0.f, 0.f, 0.f, 0.f};
  f4 xa[8], xb[8], na[8], nb[8];
  load(0, xa, xb);
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) load(c + 1, na, nb);  // one chunk ahead
    bf8 ap[4][3];
#pragma unroll
    for (int ea = 0; ea < 4; ++ea) {
      const f8 y = {xa[0][ea], xa[1][ea], xa[2][ea], xa[3][ea], xa[4][ea], xa[5][ea], xa[6][ea], xa[7][ea]};
      split3(y, ap[ea][0], ap[ea][1], ap[ea][2]);
    }
#pragma unroll
    for (int eb = 0; eb < 4; ++eb) {
      const f8 y = {xb[0][eb], xb[1][eb], xb[2][eb], xb[3][eb], xb[4][eb], xb[5][eb], xb[6][eb], xb[7][eb]};
      bf8 b0, b1, b2;
      split3(y, b0, b1, b2);
      // the chunk's six plane products into a fresh accumulator, then one f32 add into the
      // tile's: a split's thousands of rows cost one rounding of the running sum per 32 rows,
      // not six (accumulated straight into the running sum, World dW2 came out ~3 x less
      // accurate than the f32 kernel's, whose MFMA adds 4 rows per rounding)
#pragma unroll
      for (int ea = 0; ea < 4; ++ea)
        acc[ea][eb] += mfma6<false>(ap[ea], b0, b1, b2, f4{0.f, 0.f, 0.f, 0.f});
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      xa[i] = na[i];
      xb[i] = nb[i];
    }
  }
  // f32 semantics for Inf / huge operands (x * 0 is NaN only for a non-finite x)
  f2 sn = {0.f, 0.f};
#pragma unroll
  for (int ea = 0; ea < 4; ++ea)
#pragma unroll
    for (int eb = 0; eb < 4; ++eb) {
      sn = __builtin_elementwise_fma(f2{acc[ea][eb][0], acc[ea][eb][1]}, f2{0.f, 0.f}, sn);
      sn = __builtin_elementwise_fma(f2{acc[ea][eb][2], acc[ea][eb][3]}, f2{0.f, 0.f}, sn);
    }
  if (__builtin_amdgcn_ballot_w64(sn[0] != sn[0] || sn[1] != sn[1]) != 0) {
#pragma unroll
    for (int ea = 0; ea < 4; ++ea)
#pragma unroll
      for (int eb = 0; eb < 4; ++eb) acc[ea][eb] = f4{0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < rows; t += 4) {  // k step: row t + q
      const int live = min(rows - t, 4);
      const auto ra = brsrc(Ab + static_cast<int64_t>(t) * lda, live * lda4);
      const auto rb = brsrc(Bb + static_cast<int64_t>(t) * ldb, live * ldb4);
      const f4 a = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, q * lda4 + ac * 4, 0, 0));
      const f4 bv = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, q * ldb4 + bc * 4, 0, 0));
#pragma unroll
      for (int ea = 0; ea < 4; ++ea)
#pragma unroll
        for (int eb = 0; eb < 4; ++eb) acc[ea][eb] = mfma4(a[ea], bv[eb], acc[ea][eb]);
    }
  }
  float* pt = part + static_cast<int64_t>(bz) * Mp * Np;
#pragma unroll
  for (int ea = 0; ea < 4; ++ea)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 4 * (4 * q + r) + ea;
      const f4 o = {acc[ea][0][r], acc[ea][1][r], acc[ea][2][r], acc[ea][3][r]};
      *reinterpret_cast<f4*>(pt + static_cast<int64_t>(m) * Np + n0 + 4 * j) = o;
    }
}

// C[m][n] = scale * sum over the S split partials part[s][m][n], deterministic. One workgroup
// per (row m, 64 column quads): wave w of the 8 sums the splits s = w, w + 8, ... (4 loads in
// flight per lane), then the 8 wave sums are added in wave order through LDS. (One thread per
// output quad summing all S serially left ~1 wave per CU in flight: 0.57 ms for Twitter-US.)
constexpr int kTnRedWaves = 8;
__global__ __launch_bounds__(64 * kTnRedWaves) void gemm_tn_reduce_kernel(
    int M, int N, int S, const float* __restrict__ part, int Mp, int Np,
    const float* __restrict__ scale_dev, float* __restrict__ C, int64_t ldc, int vec) {
  __shared__ f4 red[kTnRedWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nq = (N + 3) / 4;
  for (int m = blockIdx.y; m < M; m += gridDim.y) {  // grid.y <= 65535
  if (m != static_cast<int>(blockIdx.y)) __syncthreads();  // red is reused
  const int qd = static_cast<int>(blockIdx.x) * 64 + lane;  // column quad
  const int qc = qd < nq ? qd : nq - 1;
  const float* src = part + static_cast<int64_t>(m) * Np + 4 * qc;
  const int64_t stride = static_cast<int64_t>(Mp) * Np;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  int s = w;
  for (; s + 3 * kTnRedWaves < S; s += 4 * kTnRedWaves) {
    const f4 v0 = *reinterpret_cast<const f4*>(src + s * stride);
    const f4 v1 = *reinterpret_cast<const f4*>(src + (s + kTnRedWaves) * stride);
    const f4 v2 = *reinterpret_cast<const f4*>(src + (s + 2 * kTnRedWaves) * stride);
    const f4 v3 = *reinterpret_cast<const f4*>(src + (s + 3 * kTnRedWaves) * stride);
    acc += v0;
    acc += v1;
    acc += v2;
    acc += v3;
  }
  for (; s < S; s += kTnRedWaves) acc += *reinterpret_cast<const f4*>(src + s * stride);
  red[w][lane] = acc;
  __syncthreads();
  if (w != 0 || qd >= nq) continue;
  f4 t = red[0][lane];
#pragma unroll
  for (int i = 1; i < kTnRedWaves; ++i) t += red[i][lane];
  const float sc = scale_dev ? *scale_dev : 1.0f;
  const int n = 4 * qd;
  float* crow = C + static_cast<int64_t>(m) * ldc;
  const f4 o = {t.x * sc, t.y * sc, t.z * sc, t.w * sc};
  if (vec && n + 3 < N) {
    *reinterpret_cast<f4*>(crow + n) = o;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (n + e < N) crow[n + e] = o[e];
  }
  }
}

struct TnPlan {
  int mg, ng, pd, wm = 1, occ = 0;  // tile variant (wm: waves stacked along M; occ: see kernel)
  int mt, nt, S, rows_per_split, Mp, Np;
};

// Alternative split-K layouts (gcg_gemm_tn tile 1..n): {MG, NG, PD, WM, OCC}. tools/exp_tn_*.py
// measured each; the default below is a function of the shape only.
constexpr int kTnTiles[][5] = {
    {1, 2, 8, 1, 0},   // 1: round-2 workgroup tiles (4 waves side by side, 64 x 256 NG)
    {1, 3, 8, 0, 0},   // 2: per-wave 64 x 192, 1 wave per SIMD, 8-deep ring
    {1, 2, 8, 0, 0},   // 3: per-wave 64 x 128, 1 wave per SIMD
    {1, 3, 12, 0, 0},  // 4: per-wave 64 x 192, 12-deep ring
    {1, 1, 8, 4, 0},   // 5: 4 waves stacked along M
    {1, 3, 3, 0, 2},   // 6: per-wave 64 x 192, 2 waves per SIMD (the default at N = 930)
    {1, 2, 6, 0, 2},   // 7: per-wave 64 x 128, 2 waves per SIMD
};
constexpr int kTnTileCount = sizeof(kTnTiles) / sizeof(kTnTiles[0]);

TnPlan tn_plan(int64_t R, int64_t M, int64_t N, int tile = 0, bool bf16x6 = false) {
  TnPlan p;
  // Default: per-wave 64 x 64*NG tiles (WM = 0), NG = 3 or 2, whichever pads N less (ties: 3,
  // fewer loads per MFMA). The round-2 workgroup tiles (WM = 1: 4 waves side by side, 64 x
  // 256*NG) padded N = 930 to 1024 columns -- 15 % of the MFMAs computed discarded columns.
  // World dW2 840k x 300 x 930: 960 padded columns, 105.8 -> 121.7 TFLOP/s; US dW2 270k x 300
  // x 256 (NG = 2): 87-103 -> 118 (tools/exp_tn_wave.py).
  // NG = 3 runs at 2 waves per SIMD (PD = 3: 246 VGPRs, accumulators included) over ~8192 wave
  // tiles: 129 vs 123 TFLOP/s at 1 wave per SIMD standalone, and inside the training step -- where
  // the weight gradient shares the chip with the SpMM gathers on the main stream -- the shorter,
  // CU-sharing waves overlap better: World step 44.4 -> 43.2 ms (tools/exp_tn_instep.py). NG = 2
  // (US dW2, N = 256) measured best at 1 wave per SIMD, PD = 8, ~2048 tiles, in both settings.
  p.mg = 1, p.pd = 8;
  int64_t slots = 2048;
  {
    const int64_t pad3 = (N + 191) / 192 * 192, pad2 = (N + 127) / 128 * 128;
    p.wm = 0, p.ng = pad3 <= pad2 ? 3 : 2;
    if (p.ng == 3) p.pd = 3, p.occ = 2, slots = 8192;
  }
  // M <= 256 in whole 64-row bands and N <= 512 (the X-head gradient G^T.Xh: 1.4M x 300 x 256
  // as 300 x 256 with the roles below): M/64 waves stacked along M -- A (the narrow operand) is
  // then split over the waves and B read once per row: 85-89 -> 112-115 TFLOP/s. Not for the
  // 300 x 930 dW2 (73-82 vs 106 TFLOP/s: its 8-15 N tiles re-read A), tools/exp_tn_layout.py.
  const bool stacked = M <= 256 && M % 64 == 0 && N <= 512;
  if (stacked) p.ng = 1, p.pd = 8, p.occ = 0, p.wm = static_cast<int>(M / 64), slots = 2048;
  if (tile > 0) {  // an explicit alternative (caller-checked range)
    const int* t = kTnTiles[tile - 1];
    p.mg = t[0], p.ng = t[1], p.pd = t[2], p.wm = t[3], p.occ = t[4], slots = 2048;
  }
#ifndef GCG_TN6_SLOTS  // wave tiles per launch: 4096 / 8192 / 16384 within noise, 32768 -3 %
#define GCG_TN6_SLOTS 8192  // (variant libraries, tools/gpu/tn_slots.sh, profiles/r06/tn6_slots_ab.txt)
#endif
  if (bf16x6) p.mg = 1, p.ng = 1, p.pd = 0, p.wm = 0, p.occ = 0, slots = GCG_TN6_SLOTS;  // gemm_tn6
  const int tm = 64 * p.mg * std::max(1, p.wm);          // C rows per tile
  const int tn = (p.wm == 1 ? 256 : 64) * p.ng;          // C columns per tile
  p.mt = static_cast<int>((M + tm - 1) / tm);
  p.nt = static_cast<int>((N + tn - 1) / tn);
  // ~`slots` tiles per launch (2048: 2 workgroups per CU of the 256 CUs; per-wave tiles at 1
  // wave per SIMD: 2 rounds of the 1024 SIMDs -- 1 round measured the same speed with 2x longer
  // serial sums), at least 256 rows per split, 16-row aligned
  const int64_t want = std::max<int64_t>(1, slots / std::max(1, p.mt * p.nt));
  const int64_t max_s = std::max<int64_t>(1, R / 256);
  p.S = static_cast<int>(std::min(want, max_s));
  int64_t rps = (R + p.S - 1) / p.S;
  rps = (rps + 15) / 16 * 16;
  p.rows_per_split = static_cast<int>(std::max<int64_t>(rps, 16));
  p.S = static_cast<int>((R + p.rows_per_split - 1) / p.rows_per_split);
  p.Mp = p.mt * tm;
  p.Np = p.nt * tn;
  return p;
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------

struct Shape {
  int RT, G, WR, WC, PF = 1;
  int BL = 0;  // 1: gemm_bl_kernel (B through LDS; RT = 1, WR = 4)
  int bm() const { return 16 * RT * WR; }
  int bn() const { return 64 * G * WC; }
};

// Instantiated tiles. EPI = 0 (plain products): the LDS-B tiles (gemm_bl_kernel, the default)
// and the register-B tiles (gcg_gemm tile 1). EPI = 1 (the fused output layer on the f32 MFMA):
// row bands keeping a whole output row of up to 1024 columns in one workgroup, the B register
// set split into PF rotating parts (the default 8 at G = 4, 4 below; gcg_project_softmax_xent
// tiles 1..5 = 0, 2, 4, 8, 16 parts).
template <int EPI>
gcg_status launch_gemm(const Shape& s, dim3 grid, hipStream_t st, int M, int N, int K,
                       const float* A, int64_t lda, const float* B, int64_t ldb,
                       const float* bias, int act, float* C, int64_t ldc, const int32_t* labels,
                       float scale, const float* scale_dev, float* loss_rows,
                       float* correct_rows, const float* row_w) {
#define GCG_GEMM_BL_CASE(g, wc)                                                              \
  if (s.BL && s.G == g && s.WC == wc) {                                                      \
    hipLaunchKernelGGL((gemm_bl_kernel<g, wc, EPI>), grid, dim3(256 * (wc)), 0, st, M, N, K, A, \
                       lda, B, ldb, bias, act, C, ldc, labels, scale, scale_dev, loss_rows,   \
                       correct_rows, row_w);                                                  \
    GCG_HIP_CHECK(hipGetLastError());                                                         \
    return GCG_OK;                                                                            \
  }
#define GCG_GEMM_CASE(rt, g, wr, wc, pf)                                                    \
  if (!s.BL && s.RT == rt && s.G == g && s.WR == wr && s.WC == wc && s.PF == pf) {           \
    hipLaunchKernelGGL((gemm_kernel<rt, g, wr, wc, EPI, pf>), grid, dim3(64 * (wr) * (wc)), 0, \
                       st, M, N, K, A,                                                       \
                       lda, B, ldb, bias, act, C, ldc, labels, scale, scale_dev, loss_rows,   \
                       correct_rows, row_w);                                                  \
    GCG_HIP_CHECK(hipGetLastError());                                                         \
    return GCG_OK;                                                                            \
  }
  if constexpr (EPI == 0) {
    GCG_GEMM_BL_CASE(4, 4)
    GCG_GEMM_BL_CASE(4, 2)
    GCG_GEMM_BL_CASE(5, 1)
    GCG_GEMM_BL_CASE(4, 1)
    GCG_GEMM_BL_CASE(3, 1)
    GCG_GEMM_BL_CASE(2, 1)
    GCG_GEMM_BL_CASE(1, 1)
    GCG_GEMM_CASE(4, 4, 1, 4, 1)
    GCG_GEMM_CASE(4, 2, 1, 4, 1)
    GCG_GEMM_CASE(4, 3, 1, 4, 1)
    GCG_GEMM_CASE(2, 1, 4, 1, 1)
    GCG_GEMM_CASE(2, 2, 4, 1, 1)
    GCG_GEMM_CASE(2, 3, 4, 1, 1)
    GCG_GEMM_CASE(2, 4, 4, 1, 1)
    GCG_GEMM_CASE(2, 5, 4, 1, 1)
  } else {
    GCG_GEMM_CASE(2, 1, 1, 4, 1)
    GCG_GEMM_CASE(2, 4, 1, 4, 0)
    GCG_GEMM_CASE(2, 2, 1, 4, 0)
    GCG_GEMM_CASE(2, 3, 1, 4, 0)
    GCG_GEMM_CASE(2, 4, 1, 4, 2)
    GCG_GEMM_CASE(2, 3, 1, 4, 2)
    GCG_GEMM_CASE(2, 2, 1, 4, 2)
    GCG_GEMM_CASE(2, 4, 1, 4, 4)
    GCG_GEMM_CASE(2, 4, 1, 4, 8)
    GCG_GEMM_CASE(2, 4, 1, 4, 16)
    GCG_GEMM_CASE(2, 3, 1, 4, 4)
    GCG_GEMM_CASE(2, 2, 1, 4, 4)
  }
#undef GCG_GEMM_CASE
#undef GCG_GEMM_BL_CASE
  return fail(GCG_ERR_INVALID_ARG, "gemm: no tile instantiated for RT=%d G=%d WR=%d WC=%d PF=%d",
              s.RT, s.G, s.WR, s.WC, s.PF);
}

// Plain products (gcg_gemm). Tile 0, B through LDS (gemm_bl_kernel), measured on the train
// step's shapes (tools/exp_gemm_bl.py, TFLOP/s, B-from-L2 gemm_kernel -> LDS-B):
//   840k x 300 x 930  93.5 -> 96.7 (16 waves x 256 columns)   1.4M x 300 x 930  94.5 -> 97.0
//   840k x 930 x 300  90.9 -> 105.1 (4 waves x 320 columns)   1.4M x 930 x 300  91.6 -> 105.7
// Tile 1: B from L2 straight to registers (gemm_kernel), the same k order (bitwise equal).
Shape pick_gemm_shape(int64_t N, int tile) {
  const int groups = static_cast<int>((N + 63) / 64);
  if (tile == 0) {
    if (groups <= 5) return Shape{1, std::max(groups, 1), 4, 1, 0, 1};
    if (groups <= 8) return Shape{1, 4, 4, 2, 0, 1};
    return Shape{1, 4, 4, 4, 0, 1};  // 1024 columns per workgroup, grid.y for the rest
  }
  if (groups <= 5) return Shape{2, std::max(groups, 1), 4, 1};  // one wave spans all columns
  return Shape{4, std::min(4, (groups + 3) / 4), 1, 4};         // RT = 4, 1 workgroup per CU
}

// The fused output layer on the f32 MFMA (gemm_kernel EPI = 1): the workgroup holds the whole
// row (WC = 4, G = ceil(N / 256)), measured on Twitter-World's 840k x 300 x 930 (TFLOP/s):
//   RT = 4, B ping-pong, 1 workgroup per CU          78.7
//   RT = 2, one B set, 2 workgroups per CU           85.0-87.4: the second workgroup hides B
//       latency and overlaps the other's softmax epilogue + stores
//   ... + B set split into 2 / 4 / 8 / 16 rotating parts, groups past N skipped
//                                                    92.3, 96.4, 96.8, 95.4  <- 8 parts
// `parts` (tiles 1..5: 0, 2, 4, 8, 16) only reorders MFMAs between distinct accumulators.
constexpr int kFusedParts[] = {0, 2, 4, 8, 16};
Shape pick_fused_shape(int64_t N, int parts) {
  const int groups = static_cast<int>((N + 63) / 64);
  const int g = std::min(4, (groups + 3) / 4);
  if (g < 2) return Shape{2, 1, 1, 4};
  const int sp = parts < 0 ? 8 : parts;
  const int np = sp >= 8 && g == 4 ? (sp >= 16 ? 16 : 8) : sp >= 4 ? 4 : sp >= 2 ? 2 : 0;
  return Shape{2, g, 1, 4, np};
}

gcg_status check_dense(const char* fn, const float* p, int64_t ld, int64_t cols, bool vec4) {
  if (p == nullptr) return fail(GCG_ERR_INVALID_ARG, "%s: null operand", fn);
  if (ld < cols) return fail(GCG_ERR_INVALID_ARG, "%s: leading dimension %lld < %lld", fn,
                             static_cast<long long>(ld), static_cast<long long>(cols));
  if (vec4 && (ld % 4 != 0 || !aligned(p, 16)))
    return fail(GCG_ERR_MISALIGNED, "%s: operand needs a 16-B aligned base and ld %% 4 == 0", fn);
  if (!aligned(p, 4)) return fail(GCG_ERR_MISALIGNED, "%s: operand not 4-B aligned", fn);
  return GCG_OK;
}

// Per-call arithmetic and tile: the math and tile arguments of the entry points.
gcg_status check_opts(const char* fn, int op, int math, int tile) {
  const int n = gcg_dense_tile_count(op, math);
  if (n < 0) return fail(GCG_ERR_INVALID_ARG, "%s: math %d not available for this product", fn, math);
  if (tile < 0 || tile > n)
    return fail(GCG_ERR_INVALID_ARG, "%s: tile %d outside 0..%d", fn, tile, n);
  return GCG_OK;
}

// The fused output layer on the bf16 matrix cores (gemm_fused6_kernel). ws != NULL: the weight's
// planes pre-split into it (FX = 1); tile 3 = 64 rows x 8 waves of 128 columns at N > 768 (the
// planes read once per 64 rows, half the 32-row form's L2 reads), else 32 rows x 4 waves, with
// the A chunk split cooperatively into LDS planes (CS = 1; World 144.5-145.1 -> 152.2-152.8 TF,
// Twitter-US 117-118 -> 120-122, profiles/r05/fused_cooperative_split.jsonl); tile 0 = tile 3;
// tile 1 = the 32-row form at any N with every wave splitting A in registers (bitwise the
// in-register weight split); tile 2 = the 64-row form likewise (N > 768 only). Every CS form is
// bitwise its CS = 0 form. ws == NULL: the weight split in every workgroup's registers, 32 rows x
// 4 waves.
// a gemm_fused6_kernel launch with the packed K tail when the last chunk holds <= 16 k (needs
// K in scope); TARGS is the parenthesised template argument list
#define GCG_FUSED6_UNPAREN(...) __VA_ARGS__
#define GCG_FUSED6_LAUNCH(TARGS, ...)                                                           \
  do {                                                                                        \
    if (K - 32 * ((K - 1) / 32) <= 16)                                                       \
      hipLaunchKernelGGL((gemm_fused6_kernel<GCG_FUSED6_UNPAREN TARGS, true>), __VA_ARGS__);  \
    else                                                                                      \
      hipLaunchKernelGGL((gemm_fused6_kernel<GCG_FUSED6_UNPAREN TARGS>), __VA_ARGS__);        \
  } while (0)
gcg_status launch_fused6(int64_t M, int N, int K, const float* A, int64_t lda, const float* B,
                         int64_t ldb, const float* bias, float* C, int64_t ldc,
                         const int32_t* labels, float scale, const float* scale_dev,
                         float* loss_rows, float* correct_rows, const float* row_w,
                         hipStream_t st, void* ws, int tile) {
  const int g = (N + 255) / 256;
  if (ws != nullptr && tile == 0) tile = 3;
  if (ws != nullptr) {  // the weight's planes pre-split (FX = 1) for the tile's BN columns
    const int Kc = (K + 31) / 32;
    if (tile == 2 && g != 4)
      return fail(GCG_ERR_INVALID_ARG, "fused layer: the 64-row tile needs N > 768 (N=%d)", N);
    const bool wide = g == 4 && tile != 1;
    const int bn = wide ? 1024 : 256 * g;
    const int64_t threads = int64_t{bn} * Kc * 4;
    hipLaunchKernelGGL(split3_rows_kernel, dim3(static_cast<unsigned>((threads + 255) / 256)),
                       dim3(256), 0, st, N, K, Kc, B, int64_t{1}, static_cast<unsigned*>(ws), ldb,
                       bn);
    GCG_HIP_CHECK(hipGetLastError());
    const auto* wsp = static_cast<const unsigned*>(ws);
    if (wide && tile == 3) {
      GCG_FUSED6_LAUNCH((4, 2, 1, 8, 0, 1, 1), dim3(static_cast<unsigned>((M + 63) / 64)),
                         dim3(512), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels,
                         scale, scale_dev, loss_rows, correct_rows, row_w, wsp);
    } else if (wide) {
      GCG_FUSED6_LAUNCH((4, 2, 1, 8, 0, 1, 0), dim3(static_cast<unsigned>((M + 63) / 64)),
                         dim3(512), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels,
                         scale, scale_dev, loss_rows, correct_rows, row_w, wsp);
    } else if (tile == 3) {  // the 32-row form with the cooperative A split
      const dim3 grid(static_cast<unsigned>((M + 31) / 32));
      switch (g) {
        case 1: GCG_FUSED6_LAUNCH((2, 1, 1, 4, 0, 1, 1), grid, dim3(256), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels, scale, scale_dev, loss_rows, correct_rows, row_w, wsp); break;
        case 2: GCG_FUSED6_LAUNCH((2, 2, 1, 4, 0, 1, 1), grid, dim3(256), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels, scale, scale_dev, loss_rows, correct_rows, row_w, wsp); break;
        default: GCG_FUSED6_LAUNCH((2, 3, 1, 4, 0, 1, 1), grid, dim3(256), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels, scale, scale_dev, loss_rows, correct_rows, row_w, wsp); break;
      }
    } else {
      const dim3 grid(static_cast<unsigned>((M + 31) / 32));
      switch (g) {
        case 1: GCG_FUSED6_LAUNCH((2, 1, 1, 4, 0, 1, 0), grid, dim3(256), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels, scale, scale_dev, loss_rows, correct_rows, row_w, wsp); break;
        case 2: GCG_FUSED6_LAUNCH((2, 2, 1, 4, 0, 1, 0), grid, dim3(256), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels, scale, scale_dev, loss_rows, correct_rows, row_w, wsp); break;
        case 3: GCG_FUSED6_LAUNCH((2, 3, 1, 4, 0, 1, 0), grid, dim3(256), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels, scale, scale_dev, loss_rows, correct_rows, row_w, wsp); break;
        default: GCG_FUSED6_LAUNCH((2, 4, 1, 4, 0, 1, 0), grid, dim3(256), 0, st, int(M), N, K, A, lda, B, ldb, bias, C, ldc, labels, scale, scale_dev, loss_rows, correct_rows, row_w, wsp); break;
      }
    }
    GCG_HIP_CHECK(hipGetLastError());
    return GCG_OK;
  }
  if (tile != 0)
    return fail(GCG_ERR_INVALID_ARG, "fused layer: tile %d needs the plane workspace", tile);
  const dim3 grid(static_cast<unsigned>((M + 31) / 32));
#define GCG_FUSED6_CASE(g_)                                                                    \
  if (g == g_) {                                                                              \
    GCG_FUSED6_LAUNCH((2, g_, 1, 4, 0, 0, 0), grid, dim3(256), 0, st, int(M), N, K, A, \
                       lda, B, ldb, bias, C, ldc, labels, scale, scale_dev, loss_rows,        \
                       correct_rows, row_w);                                                  \
    GCG_HIP_CHECK(hipGetLastError());                                                         \
    return GCG_OK;                                                                            \
  }
  GCG_FUSED6_CASE(1)
  GCG_FUSED6_CASE(2)
  GCG_FUSED6_CASE(3)
  GCG_FUSED6_CASE(4)
#undef GCG_FUSED6_CASE
  return fail(GCG_ERR_INVALID_ARG, "fused layer: N=%d", N);
}

// gcg_gemm / gcg_project_softmax_xent: validation, then the tile of (math, tile).
gcg_status gemm_common(const char* fn, bool fused, int64_t M, int64_t N, int64_t K,
                       const float* A, int64_t lda, const float* B, int64_t ldb,
                       const float* bias, int act, float* C, int64_t ldc,
                       const int32_t* labels, float scale, const float* scale_dev,
                       float* loss_rows, float* correct_rows, const float* row_w,
                       gcg_stream_t stream, int math, int tile, void* ws = nullptr) {
  gcg_status s;
  if ((s = check_opts(fn, fused ? GCG_DENSE_FUSED : GCG_DENSE_GEMM, math, tile)) != GCG_OK)
    return s;
  if (M < 0 || N <= 0 || K <= 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return fail(GCG_ERR_INVALID_ARG, "%s: bad sizes M=%lld N=%lld K=%lld", fn,
                static_cast<long long>(M), static_cast<long long>(N), static_cast<long long>(K));
  if (fused && N > 1024)
    return fail(GCG_ERR_INVALID_ARG, "%s: N=%lld > 1024 columns per fused row", fn,
                static_cast<long long>(N));
  if (act != GCG_ACT_NONE && act != GCG_ACT_RELU)
    return fail(GCG_ERR_INVALID_ARG, "%s: unknown act %d", fn, act);
  if ((s = check_dense(fn, A, lda, K, true)) != GCG_OK) return s;
  // B is read as dwordx4 at columns < round4(N): its row stride must cover them.
  if ((s = check_dense(fn, B, ldb, (N + 3) & ~int64_t{3}, true)) != GCG_OK) return s;
  if (!(fused && C == nullptr && labels != nullptr) &&
      (s = check_dense(fn, C, ldc, N, true)) != GCG_OK)
    return s;
  if (labels != nullptr && loss_rows == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "%s: labels given without loss_rows", fn);
  if (row_w != nullptr && !aligned(row_w, 4))
    return fail(GCG_ERR_MISALIGNED, "%s: row_weight not 4-B aligned", fn);
  if (M == 0) return GCG_OK;
  // gemm_kernel / gemm_fused6_kernel read B through a 32-bit buffer range (K * ldb * 4 bytes)
  if (K * ldb * 4 >= (int64_t{1} << 31))
    return fail(GCG_ERR_INVALID_ARG, "%s: B of %lld x %lld floats exceeds the 2 GB buffer range", fn,
                static_cast<long long>(K), static_cast<long long>(ldb));
  auto st = static_cast<hipStream_t>(stream);
  if (fused && math == GCG_MATH_BF16X6) {
    return launch_fused6(M, int(N), int(K), A, lda, B, ldb, bias, C, ldc, labels, scale,
                         scale_dev, loss_rows, correct_rows, row_w, st, ws, tile);
  }
  const Shape sh = fused ? pick_fused_shape(N, tile == 0 ? -1 : kFusedParts[tile - 1])
                         : pick_gemm_shape(N, tile);
  dim3 grid(static_cast<unsigned>((M + sh.bm() - 1) / sh.bm()),
            static_cast<unsigned>((N + sh.bn() - 1) / sh.bn()));
  if ((M + sh.bm() - 1) / sh.bm() > 0x7fffffffLL) return fail(GCG_ERR_INVALID_ARG, "%s: M too large", fn);
  if (fused)
    return launch_gemm<1>(sh, grid, st, int(M), int(N), int(K), A, lda, B, ldb, bias, act, C, ldc,
                          labels, scale, scale_dev, loss_rows, correct_rows, row_w);
  return launch_gemm<0>(sh, grid, st, int(M), int(N), int(K), A, lda, B, ldb, bias, act, C, ldc,
                        nullptr, 0.f, nullptr, nullptr, nullptr, nullptr);
}

// NT GEMM tiles on the f32 MFMA: (RT, G, WR, WC, S, PF, KC). Tile 0 = the first row.
struct NtShape {
  int RT, G, WR, WC, S, PF = 0, KC = 32, MX = 0;
  int bm() const { return 16 * RT * WR; }
  int bn() const { return 64 * G * WC; }
};

// Measured on one MI355X (tools/exp_gemm_nt.py, TFLOP/s on 840k x 300 x 930 / 840k x 930 x 300
// / 450k x 300 x 256 / 450k x 256 x 300): 16-deep chunks in a 4-stage ring (2,1,4,1,4,KC=16):
// 48 KB, 3 workgroups per CU, three chunks of DMA in flight: 118.0 / 118.0 / 114.4 / 111.2
// against 108.6 / 113.3 / 112.2 / 109.9 for the 32-deep 2-stage tile; 256 x 64 116 / 117.5;
// 128 x 128 91-115; 64 x 64 106-111. BM = 128 x BN = 64 with 48-72 KB of LDS runs 2-3
// workgroups per CU: one workgroup's barrier, DMA wait and epilogue overlap the others' MFMAs.
constexpr NtShape kNtTiles[] = {
    {2, 1, 4, 1, 4, 0, 16},  // 0: default, 128 x 64, 16-deep chunks, 4 stages
    {2, 1, 4, 1, 2, 0, 32},  // 1: 32-deep chunks, 2 stages
    {2, 1, 4, 1, 2, 1, 32},  // 2: ... both 16-deep steps' fragments read first
    {2, 1, 4, 1, 3, 1, 32},  // 3: ... 3 stages
    {4, 1, 4, 1, 2, 0, 32},  // 4: 256 x 64
    {2, 2, 4, 1, 2, 0, 32},  // 5: 128 x 128
    {2, 1, 2, 2, 2, 0, 32},  // 6: 2 x 2 waves
    {2, 1, 4, 1, 3, 0, 16},  // 7: 16-deep, 3 stages
    {4, 1, 4, 1, 4, 0, 16},  // 8: 256 x 64, 16-deep
    {2, 2, 4, 1, 4, 0, 16},  // 9: 128 x 128, 16-deep
    {1, 1, 4, 1, 4, 0, 16},  // 10: 64 x 64, 16-deep
};
constexpr int kNtTileCount = sizeof(kNtTiles) / sizeof(kNtTiles[0]) - 1;

struct NtArgs {
  int M, N, K;
  const float* A;
  int64_t lda;
  const float* Bt;
  int64_t ldb;
  const float* bias;
  int act;
  float* C;
  int64_t ldc;
};

template <int RT, int G, int WR, int WC, int S>
gcg_status launch_nt3_t(const NtArgs& a, const unsigned* Bs, hipStream_t st) {
  constexpr int BM = 16 * RT * WR, BN = 64 * G * WC;
  const int64_t rt = (a.M + BM - 1) / BM, ct = (a.N + BN - 1) / BN;
  if (rt * ct > 0x7fffffffLL) return fail(GCG_ERR_INVALID_ARG, "gemm_nt: M too large");
  if (a.K - 32 * ((a.K - 1) / 32) <= 16) {  // the last chunk packed (mfma6)
    hipLaunchKernelGGL((gemm_nt3_kernel<RT, G, WR, WC, S, true>), dim3(static_cast<unsigned>(rt * ct)),
                       dim3(64 * WR * WC), 0, st, a.M, a.N, a.K, a.A, a.lda, Bs, a.Bt, a.ldb, a.bias,
                       a.act, a.C, a.ldc, static_cast<int>(ct));
  } else {
    hipLaunchKernelGGL((gemm_nt3_kernel<RT, G, WR, WC, S>), dim3(static_cast<unsigned>(rt * ct)),
                       dim3(64 * WR * WC), 0, st, a.M, a.N, a.K, a.A, a.lda, Bs, a.Bt, a.ldb, a.bias,
                       a.act, a.C, a.ldc, static_cast<int>(ct));
  }
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

template <int RT, int G, int WR, int WC, int V = 0>
gcg_status launch_nt3r_t(const NtArgs& a, const unsigned* Bs, hipStream_t st) {
  constexpr int BM = 16 * RT * WR, BN = 64 * G * WC;
  const int64_t rt = (a.M + BM - 1) / BM, ct = (a.N + BN - 1) / BN;
  if (rt * ct > 0x7fffffffLL) return fail(GCG_ERR_INVALID_ARG, "gemm_nt: M too large");
  if (a.K - 32 * ((a.K - 1) / 32) <= 16) {  // the last chunk packed (mfma6)
    hipLaunchKernelGGL((gemm_nt3r_kernel<RT, G, WR, WC, V | 2>), dim3(static_cast<unsigned>(rt * ct)),
                       dim3(64 * WR * WC), 0, st, a.M, a.N, a.K, a.A, a.lda, Bs, a.Bt, a.ldb, a.bias,
                       a.act, a.C, a.ldc, static_cast<int>(ct));
  } else {
    hipLaunchKernelGGL((gemm_nt3r_kernel<RT, G, WR, WC, V>), dim3(static_cast<unsigned>(rt * ct)),
                       dim3(64 * WR * WC), 0, st, a.M, a.N, a.K, a.A, a.lda, Bs, a.Bt, a.ldb, a.bias,
                       a.act, a.C, a.ldc, static_cast<int>(ct));
  }
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

template <int RT, int G, int WR, int WC, int S, int PF, int KC, int MX = 0>
gcg_status launch_nt_t(const NtArgs& a, hipStream_t st) {
  constexpr int BM = 16 * RT * WR, BN = 64 * G * WC;
  const int64_t rt = (a.M + BM - 1) / BM, ct = (a.N + BN - 1) / BN;
  if (rt * ct > 0x7fffffffLL) return fail(GCG_ERR_INVALID_ARG, "gemm_nt: M too large");
  if constexpr (MX == 1) {
    if (a.K - 32 * ((a.K - 1) / 32) <= 16) {  // the last chunk packed (mfma6)
      hipLaunchKernelGGL((gemm_nt_kernel<RT, G, WR, WC, S, PF, KC, MX | 2>),
                         dim3(static_cast<unsigned>(rt * ct)), dim3(64 * WR * WC), 0, st, a.M, a.N,
                         a.K, a.A, a.lda, a.Bt, a.ldb, a.bias, a.act, a.C, a.ldc,
                         static_cast<int>(ct));
      GCG_HIP_CHECK(hipGetLastError());
      return GCG_OK;
    }
  }
  hipLaunchKernelGGL((gemm_nt_kernel<RT, G, WR, WC, S, PF, KC, MX>),
                     dim3(static_cast<unsigned>(rt * ct)), dim3(64 * WR * WC), 0, st, a.M, a.N,
                     a.K, a.A, a.lda, a.Bt, a.ldb, a.bias, a.act, a.C, a.ldc,
                     static_cast<int>(ct));
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

gcg_status launch_nt(const NtShape& sh, hipStream_t st, const NtArgs& a) {
  // bf16x6 with both operands split in the loop (no workspace): 128 x 64, 32-deep, 2 stages
  if (sh.MX == 1) return launch_nt_t<2, 1, 4, 1, 2, 1, 32, 1>(a, st);
#define GCG_NT_CASE(rt_, g_, wr_, wc_, s_, pf_, kc_)                                             \
  if (sh.RT == rt_ && sh.G == g_ && sh.WR == wr_ && sh.WC == wc_ && sh.S == s_ && sh.PF == pf_ && \
      sh.KC == kc_)                                                                              \
    return launch_nt_t<rt_, g_, wr_, wc_, s_, pf_, kc_>(a, st);
  GCG_NT_CASE(2, 1, 4, 1, 4, 0, 16)
  GCG_NT_CASE(2, 1, 4, 1, 2, 0, 32)
  GCG_NT_CASE(2, 1, 4, 1, 2, 1, 32)
  GCG_NT_CASE(2, 1, 4, 1, 3, 1, 32)
  GCG_NT_CASE(4, 1, 4, 1, 2, 0, 32)
  GCG_NT_CASE(2, 2, 4, 1, 2, 0, 32)
  GCG_NT_CASE(2, 1, 2, 2, 2, 0, 32)
  GCG_NT_CASE(2, 1, 4, 1, 3, 0, 16)
  GCG_NT_CASE(4, 1, 4, 1, 4, 0, 16)
  GCG_NT_CASE(2, 2, 4, 1, 4, 0, 16)
  GCG_NT_CASE(1, 1, 4, 1, 4, 0, 16)
#undef GCG_NT_CASE
  return fail(GCG_ERR_INVALID_ARG, "gemm_nt: no tile RT=%d G=%d WR=%d WC=%d S=%d PF=%d KC=%d",
              sh.RT, sh.G, sh.WR, sh.WC, sh.S, sh.PF, sh.KC);
}

// bf16x6 NT tiles with the weight's planes pre-split: (RT, G, WR, WC, S); S = 0:
// gemm_nt3r_kernel (A in registers), S = 2: gemm_nt3_kernel (A through the LDS-DMA ring).
struct Nt3Shape {
  int RT, G, WR, WC, S;
};
// Measured (tools/exp_gemm_bf16x6.py, one box, f32-equivalent TFLOP/s; f32 MFMA kernel 113-119):
//   shape (M x K x N)     LDS A: 2,1,4,1,2  2,2,4,1,2  2,1,4,2,2 | register A: 2,1,4,1  2,2,4,1  4,1,4,1
//   840k x 300 x 930           146          151-156     154-155  |             164-165  170-172  151-154
//   840k x 930 x 300           167          165-166     155      |             159-160  164      154-157
//   1.4M x 300 x 930           146          151-152     154-155  |             165-166  171      151
//   450k x 300 x 256           138-141      155         154-155  |             155-157  168-170  141-142
//   450k x 256 x 300           136          138-139     134-137  |             143-145  142      129
// Default: register A, 128 rows x 64 G columns, G in 1..3:
//                       G = 1      G = 2      G = 3
//   840k x 300 x 930    166-168    171-173    175-176   (N padded to 960 / 1024 / 960)
//   840k x 930 x 300    162-163    166        170-172   (320 / 384 / 384)
//   450k x 300 x 256    157-160    170-172    122       (256 / 256 / 384)
//   450k x 256 x 300    144.5      142-144    137-138   (320 / 384 / 384)
// Rule: the G padding N least (ties: the larger G -- fewer re-reads of A); for K > 512 the
// largest G within 1.25 x the least padding (a long k loop amortises the wider tile's waste).
constexpr Nt3Shape kNt3Tiles[] = {
    {2, 1, 4, 1, 0},  // 1: register A, 128 x 64
    {2, 2, 4, 1, 0},  // 2: register A, 128 x 128
    {2, 3, 4, 1, 0},  // 3: register A, 128 x 192
    {4, 1, 4, 1, 0},  // 4: register A, 256 x 64
    {2, 1, 4, 1, 2},  // 5: LDS A, 128 x 64
    {2, 2, 4, 1, 2},  // 6: LDS A, 128 x 128
    {2, 1, 4, 2, 2},  // 7: LDS A, 2 column waves
    {4, 1, 4, 1, 2},  // 8: LDS A, 256 x 64
    {2, 3, 4, 1, 1},  // 9: register A, 128 x 192, weight planes read one slot ahead (PL)
};
constexpr int kNt3TileCount = sizeof(kNt3Tiles) / sizeof(kNt3Tiles[0]);

Nt3Shape pick_nt3_shape(int64_t N, int64_t K) {
  int64_t pad[4] = {0, 0, 0, 0}, least = INT64_MAX;
  for (int g = 1; g <= 3; ++g) {
    pad[g] = (N + 64 * g - 1) / (64 * g) * (64 * g);
    least = std::min(least, pad[g]);
  }
  int best = 1;
  for (int g = 1; g <= 3; ++g)
    if (pad[g] == least || (K > 512 && 4 * pad[g] <= 5 * least)) best = g;
  // G = 3 reads the weight planes one slot ahead (PL, bitwise the same products in the same
  // order): 840k x 930 x 300 172.5-173.0 -> 176.1-176.8, 840k x 300 x 930 176.0-176.8 vs
  // 174.9-177.1 (profiles/r05/nt_planes_ahead.jsonl); at G = 1 / 2 the fenced schedule lost
  // (164 / 153 vs 169 / 172), so they keep the compiler's
  return Nt3Shape{2, best, 4, 1, best == 3 ? 1 : 0};
}
gcg_status launch_nt3(const Nt3Shape& sh, hipStream_t st, const NtArgs& a, const unsigned* Bs) {
#define GCG_NT3_CASE(rt_, g_, wr_, wc_, s_)                                                    \
  if (sh.RT == rt_ && sh.G == g_ && sh.WR == wr_ && sh.WC == wc_ && sh.S == s_)                \
    return launch_nt3_t<rt_, g_, wr_, wc_, s_>(a, Bs, st);
  GCG_NT3_CASE(2, 1, 4, 1, 2)
  GCG_NT3_CASE(2, 2, 4, 1, 2)
  GCG_NT3_CASE(2, 1, 4, 2, 2)
  GCG_NT3_CASE(4, 1, 4, 1, 2)
#undef GCG_NT3_CASE
#define GCG_NT3R_CASE(rt_, g_, wr_, wc_)                                                       \
  if (sh.RT == rt_ && sh.G == g_ && sh.WR == wr_ && sh.WC == wc_ && sh.S == 0)                 \
    return launch_nt3r_t<rt_, g_, wr_, wc_>(a, Bs, st);
  GCG_NT3R_CASE(2, 1, 4, 1)
  GCG_NT3R_CASE(2, 2, 4, 1)
  GCG_NT3R_CASE(2, 3, 4, 1)
  GCG_NT3R_CASE(4, 1, 4, 1)
#undef GCG_NT3R_CASE
  if (sh.RT == 2 && sh.G == 3 && sh.WR == 4 && sh.WC == 1 && sh.S == 1)  // planes one slot ahead
    return launch_nt3r_t<2, 3, 4, 1, 1>(a, Bs, st);
  return fail(GCG_ERR_INVALID_ARG, "gemm_nt bf16x6: no tile RT=%d G=%d WR=%d WC=%d S=%d",
              sh.RT, sh.G, sh.WR, sh.WC, sh.S);
}

gcg_status gemm_nt_impl(const char* fn, int64_t M, int64_t N, int64_t K, const float* A,
                        int64_t lda, const float* Bt, int64_t ldbt, const float* bias, int act,
                        float* C, int64_t ldc, int math, int tile, void* ws, int64_t ws_bytes,
                        gcg_stream_t stream) {
  gcg_status s;
  if ((s = check_opts(fn, GCG_DENSE_GEMM_NT, math, tile)) != GCG_OK) return s;
  if (M < 0 || N <= 0 || K <= 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return fail(GCG_ERR_INVALID_ARG, "%s: bad sizes M=%lld N=%lld K=%lld", fn,
                static_cast<long long>(M), static_cast<long long>(N), static_cast<long long>(K));
  if (act != GCG_ACT_NONE && act != GCG_ACT_RELU)
    return fail(GCG_ERR_INVALID_ARG, "%s: unknown act %d", fn, act);
  // both operands are read as 16-B k-segments up to round4(K)
  if ((s = check_dense(fn, A, lda, (K + 3) & ~int64_t{3}, true)) != GCG_OK) return s;
  if ((s = check_dense(fn, Bt, ldbt, (K + 3) & ~int64_t{3}, true)) != GCG_OK) return s;
  if ((s = check_dense(fn, C, ldc, N, true)) != GCG_OK) return s;
  if (bias != nullptr && !aligned(bias, 4)) return fail(GCG_ERR_MISALIGNED, "%s: bias", fn);
  NtArgs a{int(M), int(N), int(K), A, lda, Bt, ldbt, bias, act, C, ldc};
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (math == GCG_MATH_F32) {
    if (M == 0) return GCG_OK;
    return launch_nt(kNtTiles[tile], st, a);
  }
  // bf16x6. Planes or A tiles past the 32-bit buffer offsets: both operands split in the loop.
  if (ws != nullptr && (gcg_gemm_nt_bf16x6_workspace(N, K) > INT32_MAX || 256 * lda * 4 > INT32_MAX / 2)) {
    if (tile != 0) return fail(GCG_ERR_INVALID_ARG, "%s: operands too large for tile %d", fn, tile);
    ws = nullptr;
  }
  if (ws == nullptr) {
    if (tile != 0) return fail(GCG_ERR_INVALID_ARG, "%s: tile %d needs the plane workspace", fn, tile);
    if (M == 0) return GCG_OK;
    NtShape sh{};
    sh.MX = 1;
    return launch_nt(sh, st, a);
  }
  if (ws_bytes < gcg_gemm_nt_bf16x6_workspace(N, K))
    return fail(GCG_ERR_WORKSPACE, "%s: workspace %lld B < %lld B", fn,
                static_cast<long long>(ws_bytes),
                static_cast<long long>(gcg_gemm_nt_bf16x6_workspace(N, K)));
  if (!aligned(ws, 16)) return fail(GCG_ERR_MISALIGNED, "%s: workspace", fn);
  if (M == 0) return GCG_OK;
  const int Kc = static_cast<int>((K + 31) / 32);
  const int64_t threads = N * Kc * 4;
  hipLaunchKernelGGL(split3_rows_kernel, dim3(static_cast<unsigned>((threads + 255) / 256)), dim3(256),
                     0, st, int(N), int(K), Kc, Bt, ldbt, static_cast<unsigned*>(ws));
  GCG_HIP_CHECK(hipGetLastError());
  const auto* wsp = static_cast<const unsigned*>(ws);
  if (tile == 0) {
    // Ragged column split (round 6): the 192-column tile over N's whole 192-column blocks and
    // the narrowest tile over the rest, when that pads less than the one shape the picker
    // chose. dP = G.W2^T at N = 300, K = 930: the picker's 128 x 192 tile (two passes over A)
    // computes 384 columns; 192 + 128 computes 320, with the same two passes over A. Every
    // output element is the same products in the same order (bitwise the one-shape result).
    const Nt3Shape sh = pick_nt3_shape(N, K);
    const int64_t bn = 64 * sh.G, pad_pick = (N + bn - 1) / bn * bn;
    const int64_t n_main = N / 192 * 192, r = N - n_main, gr = (r + 63) / 64;
    if (n_main > 0 && r > 0 && n_main + 64 * gr < pad_pick) {
      NtArgs a1 = a;
      a1.N = static_cast<int>(n_main);
      gcg_status s1 = launch_nt3(Nt3Shape{2, 3, 4, 1, 1}, st, a1, wsp);
      if (s1 != GCG_OK) return s1;
      NtArgs a2 = a;  // columns n_main .. N - 1: their weight rows, planes, bias and outputs
      a2.N = static_cast<int>(r);
      a2.Bt = Bt + n_main * ldbt;
      a2.bias = bias != nullptr ? bias + n_main : nullptr;
      a2.C = C + n_main;
      return launch_nt3(Nt3Shape{2, static_cast<int>(gr), 4, 1, gr == 3 ? 1 : 0}, st, a2,
                        wsp + n_main * Kc * 48);
    }
  }
  return launch_nt3(tile == 0 ? pick_nt3_shape(N, K) : kNt3Tiles[tile - 1], st, a, wsp);
}

gcg_status gemm_tn_impl(const char* fn, int64_t R, int64_t M, int64_t N, const float* A,
                        int64_t lda, const float* B, int64_t ldb, const float* scale_dev,
                        float* C, int64_t ldc, int math, int tile, void* workspace,
                        size_t workspace_bytes, gcg_stream_t stream) {
  gcg_status st;
  if ((st = check_opts(fn, GCG_DENSE_GEMM_TN, math, tile)) != GCG_OK) return st;
  if (R < 0 || M <= 0 || N <= 0 || R > INT32_MAX || M > INT32_MAX || N > INT32_MAX)
    return fail(GCG_ERR_INVALID_ARG, "%s: bad sizes R=%lld M=%lld N=%lld", fn,
                static_cast<long long>(R), static_cast<long long>(M), static_cast<long long>(N));
  // dwordx4 row reads at columns < round4(M) / round4(N)
  if ((st = check_dense(fn, A, lda, (M + 3) & ~int64_t{3}, true)) != GCG_OK) return st;
  if ((st = check_dense(fn, B, ldb, (N + 3) & ~int64_t{3}, true)) != GCG_OK) return st;
  if ((st = check_dense(fn, C, ldc, N, false)) != GCG_OK) return st;
  if (lda >= (int64_t{1} << 27) || ldb >= (int64_t{1} << 27))  // 4-row buffer ranges < 2 GB
    return fail(GCG_ERR_INVALID_ARG, "%s: leading dimension too large", fn);
  auto s = static_cast<hipStream_t>(stream);
  if (R == 0) {
    for (int64_t m = 0; m < M; ++m)
      GCG_HIP_CHECK(hipMemsetAsync(C + m * ldc, 0, sizeof(float) * N, s));
    return GCG_OK;
  }
  const bool bf = math == GCG_MATH_BF16X6;
  const TnPlan p = tn_plan(R, M, N, tile, bf);
  const size_t need = sizeof(float) * static_cast<size_t>(p.S) * p.Mp * p.Np;
  if (workspace == nullptr || workspace_bytes < need)
    return fail(GCG_ERR_WORKSPACE, "%s: workspace %zu bytes < %zu needed", fn, workspace_bytes,
                need);
  if (!aligned(workspace, 16)) return fail(GCG_ERR_MISALIGNED, "%s: workspace not 16-B aligned", fn);
  float* part = static_cast<float*>(workspace);
  int64_t n_tiles = int64_t{p.mt} * p.nt * p.S;
  if (n_tiles > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "%s: too many tiles", fn);
  if (p.wm == 0) n_tiles = (n_tiles + 3) / 4;  // 4 wave tiles per workgroup
  const dim3 grid(static_cast<unsigned>(n_tiles));
  constexpr int remap = 1;  // XCD-aware tile order (+1-3 % dW2, +14 % X head)
  if (bf) {
    hipLaunchKernelGGL(gemm_tn6_partial_kernel, grid, dim3(256), 0, s, int(R), int(M), int(N), A,
                       lda, B, ldb, p.rows_per_split, part, p.Mp, p.Np, p.mt, p.nt);
  } else
#define GCG_TN_CASE_OCC(MG_, NG_, PD_, WM_, OCC_)                                            \
  if (p.mg == MG_ && p.ng == NG_ && p.pd == PD_ && p.wm == WM_ && p.occ == OCC_) {           \
    hipLaunchKernelGGL((gemm_tn_partial_kernel<MG_, NG_, PD_, WM_, OCC_>), grid,             \
                       dim3(WM_ <= 1 ? 256 : 64 * WM_), 0, s, int(R), int(M), int(N), A, lda, \
                       B, ldb, p.rows_per_split, part, p.Mp, p.Np, p.mt, p.nt, remap);       \
  } else
#define GCG_TN_CASE(MG_, NG_, PD_, WM_) GCG_TN_CASE_OCC(MG_, NG_, PD_, WM_, 0)
  GCG_TN_CASE(1, 2, 8, 1)
  GCG_TN_CASE(1, 1, 8, 1)
  GCG_TN_CASE(1, 1, 8, 2)
  GCG_TN_CASE(1, 1, 8, 3)
  GCG_TN_CASE(1, 1, 8, 4)
  GCG_TN_CASE(1, 2, 8, 0)
  GCG_TN_CASE(1, 3, 8, 0)
  GCG_TN_CASE(1, 3, 12, 0)
  GCG_TN_CASE_OCC(1, 3, 3, 0, 2)
  GCG_TN_CASE_OCC(1, 2, 6, 0, 2)
  { return fail(GCG_ERR_INVALID_ARG, "%s: no TN tile MG=%d NG=%d PD=%d WM=%d OCC=%d", fn, p.mg,
                p.ng, p.pd, p.wm, p.occ); }
#undef GCG_TN_CASE
#undef GCG_TN_CASE_OCC
  GCG_HIP_CHECK(hipGetLastError());
  const int vec = (ldc % 4 == 0 && aligned(C, 16)) ? 1 : 0;
  const dim3 rgrid(static_cast<unsigned>(((N + 3) / 4 + 63) / 64),
                   static_cast<unsigned>(std::min<int64_t>(M, 65535)));
  hipLaunchKernelGGL(gemm_tn_reduce_kernel, rgrid, dim3(64 * kTnRedWaves), 0, s, int(M), int(N),
                     p.S, part, p.Mp, p.Np, scale_dev, C, ldc, vec);
  GCG_HIP_CHECK(hipGetLastError());
  return GCG_OK;
}

}  // namespace

extern "C" {

int32_t gcg_dense_tile_count(int32_t op, int32_t math) {
  switch (op) {
    case GCG_DENSE_GEMM: return math == GCG_MATH_F32 ? 1 : -1;
    case GCG_DENSE_GEMM_NT:
      return math == GCG_MATH_F32 ? kNtTileCount : math == GCG_MATH_BF16X6 ? kNt3TileCount : -1;
    case GCG_DENSE_FUSED:
      return math == GCG_MATH_F32 ? 5 : math == GCG_MATH_BF16X6 ? 3 : -1;
    case GCG_DENSE_GEMM_TN:
      return math == GCG_MATH_F32 ? kTnTileCount : math == GCG_MATH_BF16X6 ? 0 : -1;
    default: return -1;
  }
}

gcg_status gcg_gemm_nt(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                       const float* Bt, int64_t ldbt, const float* bias, int act, float* C,
                       int64_t ldc, int32_t math, int32_t tile, void* ws, int64_t ws_bytes,
                       gcg_stream_t stream) {
  return gemm_nt_impl("gcg_gemm_nt", M, N, K, A, lda, Bt, ldbt, bias, act, C, ldc, math, tile, ws,
                      ws_bytes, stream);
}

int64_t gcg_gemm_nt_workspace(int64_t N, int64_t K, int32_t math) {
  return math == GCG_MATH_BF16X6 ? gcg_gemm_nt_bf16x6_workspace(N, K) : 0;
}

gcg_status gcg_gemm_nt_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                           const float* Bt, int64_t ldbt, const float* bias, int act, float* C,
                           int64_t ldc, gcg_stream_t stream) {
  return gemm_nt_impl("gcg_gemm_nt_f32", M, N, K, A, lda, Bt, ldbt, bias, act, C, ldc,
                      GCG_MATH_F32, 0, nullptr, 0, stream);
}

int64_t gcg_gemm_nt_bf16x6_workspace(int64_t N, int64_t K) {
  if (N <= 0 || K <= 0) return 0;
  return N * ((K + 31) / 32) * 192;
}

gcg_status gcg_gemm_nt_f32_bf16x6(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                  const float* Bt, int64_t ldbt, const float* bias, int act,
                                  float* C, int64_t ldc, void* ws, int64_t ws_bytes,
                                  gcg_stream_t stream) {
  return gemm_nt_impl("gcg_gemm_nt_f32_bf16x6", M, N, K, A, lda, Bt, ldbt, bias, act, C, ldc,
                      GCG_MATH_BF16X6, 0, ws, ws_bytes, stream);
}

gcg_status gcg_gemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
                    int64_t ldb, const float* bias, int act, float* C, int64_t ldc, int32_t math,
                    int32_t tile, gcg_stream_t stream) {
  return gemm_common("gcg_gemm", false, M, N, K, A, lda, B, ldb, bias, act, C, ldc, nullptr,
                     0.f, nullptr, nullptr, nullptr, nullptr, stream, math, tile);
}

gcg_status gcg_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                        const float* B, int64_t ldb, const float* bias, int act, float* C,
                        int64_t ldc, gcg_stream_t stream) {
  return gemm_common("gcg_gemm_f32", false, M, N, K, A, lda, B, ldb, bias, act, C, ldc, nullptr,
                     0.f, nullptr, nullptr, nullptr, nullptr, stream, GCG_MATH_F32, 0);
}

int64_t gcg_project_softmax_xent_workspace(int64_t N, int64_t K, int32_t math) {
  if (math != GCG_MATH_BF16X6 || N <= 0 || N > 1024 || K <= 0) return 0;
  return int64_t{1024} * ((K + 31) / 32) * 192;
}

int64_t gcg_project_softmax_xent_bf16x6_workspace(int64_t N, int64_t K) {
  return gcg_project_softmax_xent_workspace(N, K, GCG_MATH_BF16X6);
}

gcg_status gcg_project_softmax_xent(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                    const float* W, int64_t ldw, const float* bias,
                                    const int32_t* labels, float scale, const float* scale_dev,
                                    float* out, int64_t ldo, float* loss_rows,
                                    float* correct_rows, const float* row_weight, int32_t math,
                                    int32_t tile, void* ws, int64_t ws_bytes,
                                    gcg_stream_t stream) {
  const char* fn = "gcg_project_softmax_xent";
  if (math == GCG_MATH_BF16X6 && ws != nullptr) {
    if (ws_bytes < gcg_project_softmax_xent_workspace(N, K, math))
      return fail(GCG_ERR_WORKSPACE, "%s: workspace %lld B too small", fn,
                  static_cast<long long>(ws_bytes));
    if (!aligned(ws, 16)) return fail(GCG_ERR_MISALIGNED, "%s: workspace", fn);
    if (int64_t{1024} * ((K + 31) / 32) * 192 > INT32_MAX) {  // 32-bit plane offsets
      if (tile != 0) return fail(GCG_ERR_INVALID_ARG, "%s: K too large for tile %d", fn, tile);
      ws = nullptr;
    }
  }
  return gemm_common(fn, true, M, N, K, A, lda, W, ldw, bias, GCG_ACT_NONE, out, ldo, labels,
                     scale, scale_dev, loss_rows, correct_rows, row_weight, stream, math, tile, ws);
}

gcg_status gcg_project_softmax_xent_f32(int64_t M, int64_t N, int64_t K, const float* A,
                                        int64_t lda, const float* W, int64_t ldw,
                                        const float* bias, const int32_t* labels, float scale,
                                        const float* scale_dev, float* out, int64_t ldo,
                                        float* loss_rows, float* correct_rows,
                                        gcg_stream_t stream) {
  return gemm_common("gcg_project_softmax_xent_f32", true, M, N, K, A, lda, W, ldw, bias,
                     GCG_ACT_NONE, out, ldo, labels, scale, scale_dev, loss_rows, correct_rows,
                     nullptr, stream, GCG_MATH_F32, 0);
}

gcg_status gcg_project_softmax_xent_weighted_f32(int64_t M, int64_t N, int64_t K,
                                                 const float* A, int64_t lda, const float* W,
                                                 int64_t ldw, const float* bias,
                                                 const int32_t* labels, float scale,
                                                 const float* scale_dev, float* out,
                                                 int64_t ldo, float* loss_rows,
                                                 float* correct_rows, const float* row_weight,
                                                 gcg_stream_t stream) {
  return gemm_common("gcg_project_softmax_xent_weighted_f32", true, M, N, K, A, lda, W, ldw,
                     bias, GCG_ACT_NONE, out, ldo, labels, scale, scale_dev, loss_rows,
                     correct_rows, row_weight, stream, GCG_MATH_F32, 0);
}

gcg_status gcg_project_softmax_xent_weighted_ws_f32(
    int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* W, int64_t ldw,
    const float* bias, const int32_t* labels, float scale, const float* scale_dev, float* out,
    int64_t ldo, float* loss_rows, float* correct_rows, const float* row_weight, void* ws,
    int64_t ws_bytes, gcg_stream_t stream) {
  return gcg_project_softmax_xent(M, N, K, A, lda, W, ldw, bias, labels, scale, scale_dev, out,
                                  ldo, loss_rows, correct_rows, row_weight, GCG_MATH_BF16X6, 0, ws,
                                  ws_bytes, stream);
}

gcg_status gcg_softmax_xent_f32(int64_t M, int64_t N, const float* logits, int64_t ldl,
                                const int32_t* labels, float scale, const float* scale_dev,
                                float* out, int64_t ldo, float* loss_rows, float* correct_rows,
                                gcg_stream_t stream) {
  return gcg_softmax_xent_weighted_f32(M, N, logits, ldl, labels, scale, scale_dev, out, ldo,
                                       loss_rows, correct_rows, nullptr, stream);
}

gcg_status gcg_softmax_xent_weighted_f32(int64_t M, int64_t N, const float* logits, int64_t ldl,
                                         const int32_t* labels, float scale,
                                         const float* scale_dev, float* out, int64_t ldo,
                                         float* loss_rows, float* correct_rows,
                                         const float* row_weight, gcg_stream_t stream) {
  const char* fn = "gcg_softmax_xent_f32";
  if (M < 0 || N <= 0 || M > INT32_MAX || N > 4096)
    return fail(GCG_ERR_INVALID_ARG, "%s: bad sizes M=%lld N=%lld (N <= 4096)", fn,
                static_cast<long long>(M), static_cast<long long>(N));
  gcg_status s;
  if ((s = check_dense(fn, logits, ldl, N, false)) != GCG_OK) return s;
  if (out != nullptr && (s = check_dense(fn, out, ldo, N, false)) != GCG_OK) return s;
  if (labels != nullptr && loss_rows == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "%s: labels given without loss_rows", fn);
  if (out == nullptr && labels == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "%s: nothing to compute (no out, no labels)", fn);
  if (M == 0) return GCG_OK;
  const int vec = (ldl % 4 == 0 && aligned(logits, 16) &&
                   (out == nullptr || (ldo % 4 == 0 && aligned(out, 16)))) ? 1 : 0;
  const int nv = static_cast<int>((N + 255) / 256);
  dim3 grid(static_cast<unsigned>((M + 3) / 4));
  auto st = static_cast<hipStream_t>(stream);
#define GCG_SX_CASE(v)                                                                       \
  if (nv <= v) {                                                                             \
    hipLaunchKernelGGL(softmax_xent_rows_kernel<v>, grid, dim3(256), 0, st, int(M), int(N), \
                       logits, ldl, labels, scale, scale_dev, out, ldo, loss_rows,          \
                       correct_rows, row_weight, vec);                                       \
    GCG_HIP_CHECK(hipGetLastError());                                                        \
    return GCG_OK;                                                                           \
  }
  GCG_SX_CASE(1)
  GCG_SX_CASE(2)
  GCG_SX_CASE(4)
  GCG_SX_CASE(8)
  GCG_SX_CASE(16)
#undef GCG_SX_CASE
  return fail(GCG_ERR_INVALID_ARG, "%s: N too large", fn);
}

gcg_status gcg_gemm_tn_workspace_bytes(int64_t R, int64_t M, int64_t N, int32_t math,
                                       int32_t tile, size_t* bytes) {
  const char* fn = "gcg_gemm_tn_workspace_bytes";
  gcg_status s;
  if ((s = check_opts(fn, GCG_DENSE_GEMM_TN, math, tile)) != GCG_OK) return s;
  if (R < 0 || M <= 0 || N <= 0 || R > INT32_MAX || M > INT32_MAX || N > INT32_MAX ||
      bytes == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "%s: bad sizes", fn);
  if (R == 0) { *bytes = 0; return GCG_OK; }
  const TnPlan p = tn_plan(R, M, N, tile, math == GCG_MATH_BF16X6);
  *bytes = sizeof(float) * static_cast<size_t>(p.S) * p.Mp * p.Np;
  return GCG_OK;
}

gcg_status gcg_gemm_tn_f32_workspace_bytes(int64_t R, int64_t M, int64_t N, size_t* bytes) {
  return gcg_gemm_tn_workspace_bytes(R, M, N, GCG_MATH_F32, 0, bytes);
}

gcg_status gcg_gemm_tn(int64_t R, int64_t M, int64_t N, const float* A, int64_t lda,
                       const float* B, int64_t ldb, const float* scale_dev, float* C, int64_t ldc,
                       int32_t math, int32_t tile, void* workspace, size_t workspace_bytes,
                       gcg_stream_t stream) {
  return gemm_tn_impl("gcg_gemm_tn", R, M, N, A, lda, B, ldb, scale_dev, C, ldc, math, tile,
                      workspace, workspace_bytes, stream);
}

gcg_status gcg_gemm_tn_f32(int64_t R, int64_t M, int64_t N, const float* A, int64_t lda,
                           const float* B, int64_t ldb, const float* scale_dev, float* C,
                           int64_t ldc, void* workspace, size_t workspace_bytes,
                           gcg_stream_t stream) {
  return gemm_tn_impl("gcg_gemm_tn_f32", R, M, N, A, lda, B, ldb, scale_dev, C, ldc,
                      GCG_MATH_F32, 0, workspace, workspace_bytes, stream);
}

}  // extern "C"
