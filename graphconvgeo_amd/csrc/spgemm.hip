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


// ---- row-wise SpGEMM with a dense LDS accumulator (the default for p <= 8 slabs) ---------
// One 1024-thread workgroup per row of C, rows dispatched longest-first. The row's products
// are staged through LDS in traversal order (A row storage order, then B row order), NB at a
// time, and added into a dense LDS accumulator that covers a slab of `sw` output columns.
// OWN = 2 owner waves apply them (measured: 4 -> 2 owners 55.1 -> 53.8 ms at Twitter-World; 1
// owner 52.9 but Twitter-US 7.2 -> 7.6): wave w adds exactly the columns c with c % OWN == w and walks
// the steps (nonzeros of the A row) in order, so every C entry receives its products in
// scipy csr_matmat's order (sums[k] += v * Bx[kk], from 0) through no-return LDS adds that
// need no ordering beyond the wave's own program order; inside one step the columns are
// distinct (a CSR row), so the lanes of a wave never collide. Extraction
// walks the slab in column order (canonical output), keeps sums != 0 (scipy's
// `if (sums[head] != 0)`) and re-zeroes the slab. Output goes to an upper-bound layout
// (row i at rowoff[i], its product count prefix) and is compacted afterwards.
constexpr int kRowsNT = 1024;
constexpr int kRowsNB = 2048;

template <int NW>
__device__ __forceinline__ int block_excl_scan(int v, int* s_wsum, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wsum[wave] = x;
  __syncthreads();
  int wpre = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int s = s_wsum[w];
    wpre += w < wave ? s : 0;
    total += s;
  }
  __syncthreads();  // s_wsum reusable
  return wpre + x - v;
}

template <typename TA, typename TACC, int SMAX>
__global__ __launch_bounds__(kRowsNT) void spgemm_rows_kernel(
    int64_t p, int sw, const int32_t* __restrict__ order, const int32_t* __restrict__ a_ptr,
    const int32_t* __restrict__ a_idx, const TA* __restrict__ a_val, const int32_t* __restrict__ b_ptr,
    const int32_t* __restrict__ b_idx, const float* __restrict__ b_val, const int64_t* __restrict__ rowoff,
    int32_t* __restrict__ t_idx, float* __restrict__ t_val, int64_t* __restrict__ kept) {
  // NB products per staging buffer, two buffers: waves OWN.. stage window w+1 while the
  // owner waves apply window w
  constexpr int NT = kRowsNT, NB = sizeof(TACC) == 8 ? kRowsNB / 2 : kRowsNB, NW = NT / 64, OWN = 2;
  __shared__ TACC acc[SMAX];
  __shared__ int32_t s_col[2][NB];
  __shared__ TACC s_val[2][NB];
  __shared__ int32_t s_pref[NT + 1];
  __shared__ int32_t s_bst[NT];
  __shared__ TACC s_av[NT];
  __shared__ int32_t s_wsum[NW];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int k = t; k < SMAX; k += NT) acc[k] = TACC(0);
  const int64_t row = order[blockIdx.x];
  const int32_t a0 = a_ptr[row], a1 = a_ptr[row + 1];
  const int64_t out0 = rowoff[row];
  const int n_slabs = static_cast<int>((p + sw - 1) / sw);
  const int spt = sw / NT;  // columns per thread in the extraction
  int base = 0;             // outputs of this row so far (block-uniform)
  __syncthreads();
  for (int sl = 0; sl < n_slabs; ++sl) {
    const int64_t c0 = static_cast<int64_t>(sl) * sw;
    const int64_t c1 = min(p, c0 + sw);
    for (int32_t jb = a0; jb < a1; jb += NT) {
      const int ns = min(NT, a1 - jb);
      // step table (B-row starts, A values, prefix of B-row lengths); a row of at most NT
      // nonzeros keeps it from the first slab
      if (sl == 0 || a1 - a0 > NT) {
        int len = 0;
        if (t < ns) {
          const int32_t r = a_idx[jb + t];
          const int32_t b0 = b_ptr[r];
          len = b_ptr[r + 1] - b0;
          s_bst[t] = b0;
          s_av[t] = static_cast<TACC>(a_val[jb + t]);
        }
        int tot;
        const int excl = block_excl_scan<NW>(len, s_wsum, tot);
        s_pref[t] = excl;
        if (t == 0) s_pref[NT] = tot;
        __syncthreads();
      }
      const int total = s_pref[NT];
      // Step lookups are wave-parallel scans from a per-wave hint (windows only move forward):
      // 64 prefix entries per LDS read + ballot instead of a ~10-read dependent binary search.
      // first step overlapping the window starting at w0: last j in [from, ns) with
      // s_pref[j] <= w0 (s_pref[from] <= w0 holds for a hint from an earlier window)
      auto first_step = [&](int from, int w0) {
        for (int j0 = from;; j0 += 64) {
          const int j = j0 + lane;
          const uint64_t b = __ballot(j >= ns || s_pref[min(j, NT)] > w0);
          if (b) return j0 + static_cast<int>(__builtin_ctzll(b)) - 1;
        }
      };
      // first j in [from, ns] with j == ns or s_pref[j] >= target
      auto first_ge = [&](int from, int target) {
        for (int j0 = from;; j0 += 64) {
          const int j = j0 + lane;
          const uint64_t b = __ballot(j >= ns || s_pref[min(j, NT)] >= target);
          if (b) return min(j0 + static_cast<int>(__builtin_ctzll(b)), ns);
        }
      };
      int hint = 0;  // this wave's last window start step (owner and stager waves apart)
      // stage positions [w0, w0 + wn) into buffer `buf`: stager wave v of nv copies steps
      // jlo + v, jlo + v + nv, ... (one coalesced B-row read per step)
      // SU steps per round: their first 64 positions are loaded before any is stored, so a
      // stager wave keeps SU B-row reads in flight instead of one; positions past the first 64
      // of a step (B rows longer than a wave) follow in a remainder loop.
      auto stage = [&](int buf, int w0, int v, int nv) {
        constexpr int SU = 4;
        const int wn = min(NB, total - w0), wend = w0 + wn;
        hint = first_step(hint, w0);
        for (int j = hint + v; j < ns && s_pref[j] < wend; j += SU * nv) {
          int32_t ci[SU];
          float bv[SU];
          int e0[SU], e1[SU], kb[SU];
#pragma unroll
          for (int u = 0; u < SU; ++u) {
            const int jj = j + u * nv;
            const bool ok = jj < ns && s_pref[jj] < wend;
            e0[u] = ok ? max(s_pref[jj], w0) : 0;
            e1[u] = ok ? min(s_pref[jj + 1], wend) : 0;
            kb[u] = ok ? s_bst[jj] - s_pref[jj] : 0;
            const int pos = e0[u] + lane;
            if (pos < e1[u]) {
              ci[u] = b_idx[kb[u] + pos];
              bv[u] = b_val[kb[u] + pos];
            }
          }
#pragma unroll
          for (int u = 0; u < SU; ++u) {
            const int pos = e0[u] + lane;
            if (pos < e1[u]) {
              const TACC av = s_av[j + u * nv];
              s_col[buf][pos - w0] = ci[u];
              s_val[buf][pos - w0] = av * static_cast<TACC>(bv[u]);
            }
            if (e1[u] - e0[u] > 64) {
              const TACC av = s_av[j + u * nv];
              for (int q = e0[u] + 64 + lane; q < e1[u]; q += 64) {
                s_col[buf][q - w0] = b_idx[kb[u] + q];
                s_val[buf][q - w0] = av * static_cast<TACC>(b_val[kb[u] + q]);
              }
            }
          }
        }
      };
      // steps [jlo, jhi) overlap the window; their bounds go through VGPRs (readlane) in blocks
      // of 64 so the only LDS traffic per step is the entries themselves. The adds are LDS
      // atomics without return: a wave's LDS operations execute in program order, so entry
      // (j, c) lands after every (j' < j, c) with no wait on the accumulator; inside one step
      // the columns are distinct.
      auto apply = [&](int buf, int w0) {
        const int wn = min(NB, total - w0);
        const int jlo = hint = first_step(hint, w0);
        const int jhi = first_ge(jlo, w0 + wn);  // first step starting at or after w0 + wn
        // AU steps per round: their first 64 entries are read from LDS before any add is
        // issued (AU reads in flight), then added in step order; entries past the first 64
        // of a step follow in order before the next step's.
        constexpr int AU = 8;
        for (int jb2 = jlo; jb2 < jhi; jb2 += 64) {
          const int nj = min(64, jhi - jb2);
          const int p0 = lane < nj ? s_pref[jb2 + lane] : 0;
          const int p1 = lane < nj ? s_pref[jb2 + lane + 1] : 0;
          for (int q = 0; q < nj; q += AU) {
            int cc[AU], e0[AU], e1[AU];
            TACC vv[AU];
#pragma unroll
            for (int u = 0; u < AU; ++u) {
              const int qq = min(q + u, 63);
              const bool ok = q + u < nj;
              e0[u] = ok ? max(__builtin_amdgcn_readlane(p0, qq), w0) - w0 : 0;
              e1[u] = ok ? min(__builtin_amdgcn_readlane(p1, qq), w0 + wn) - w0 : 0;
              const int e = e0[u] + lane;
              cc[u] = e < e1[u] ? s_col[buf][e] : -1;
              vv[u] = e < e1[u] ? s_val[buf][e] : TACC(0);
            }
#pragma unroll
            for (int u = 0; u < AU; ++u) {
              const int c = cc[u];
              if (c >= 0 && (c & (OWN - 1)) == wave && c >= c0 && c < c1) atomicAdd(&acc[c - c0], vv[u]);
              for (int e = e0[u] + 64 + lane; e < e1[u]; e += 64) {
                const int c2 = s_col[buf][e];
                if ((c2 & (OWN - 1)) == wave && c2 >= c0 && c2 < c1) atomicAdd(&acc[c2 - c0], s_val[buf][e]);
              }
            }
          }
        }
      };
      const int n_win = (total + NB - 1) / NB;
      if (n_win > 0) {
        stage(0, 0, wave, NW);
        __syncthreads();
      }
      for (int wi = 0; wi < n_win; ++wi) {
        if (wave < OWN) apply(wi & 1, wi * NB);
        else if (wi + 1 < n_win) stage((wi + 1) & 1, (wi + 1) * NB, wave - OWN, NW - OWN);
        __syncthreads();
      }
    }
    // extraction of the slab, column order; re-zeroes it
    const int k0 = t * spt;
    const int kn = static_cast<int>(min<int64_t>(spt, max<int64_t>(0, c1 - c0 - k0)));
    int cnt = 0;
    for (int i = 0; i < kn; ++i) cnt += acc[k0 + i] != TACC(0) ? 1 : 0;
    int total;
    int o = base + block_excl_scan<NW>(cnt, s_wsum, total);
    for (int i = 0; i < kn; ++i) {
      const TACC v = acc[k0 + i];
      if (v != TACC(0)) {
        t_idx[out0 + o] = static_cast<int32_t>(c0 + k0 + i);
        t_val[out0 + o] = static_cast<float>(v);
        ++o;
        acc[k0 + i] = TACC(0);
      }
    }
    base += total;
    __syncthreads();
  }
  if (t == 0) kept[row] = base;
}


// Rows with at most kSmallSteps nonzeros and kSmallProducts products skip the slabs: the
// workgroup stages the row's products (key = column << 11 | traversal position), radix-sorts
// the keys in LDS, and sums every run of equal columns in position order -- the same
// csr_matmat order, independent of the number of output columns. 256 threads, 20-29 KB of LDS
// (several workgroups per CU); the bulk of a power-law graph's rows.
constexpr int kSmallNT = 256;
constexpr int kSmallSteps = kSmallNT;
constexpr int kSmallProducts = 2048;  // positions fit 11 bits of the sort key
constexpr int64_t kSmallMaxCols = int64_t{1} << 20;  // column < 2^21: keys stay below the pad key

template <typename TA, typename TACC>
__global__ __launch_bounds__(kSmallNT) void spgemm_small_rows_kernel(
    const int32_t* __restrict__ order, const int32_t* __restrict__ a_ptr, const int32_t* __restrict__ a_idx,
    const TA* __restrict__ a_val, const int32_t* __restrict__ b_ptr, const int32_t* __restrict__ b_idx,
    const float* __restrict__ b_val, const int64_t* __restrict__ rowoff, int32_t* __restrict__ t_idx,
    float* __restrict__ t_val, int64_t* __restrict__ kept, int64_t n_rows, int col_bits) {
  constexpr int NT = kSmallNT, NB = kSmallProducts, NW = NT / 64, KPT8 = 8;
  using Sort2 = hipcub::BlockRadixSort<uint32_t, NT, 2>;     // rows of <= 512 products
  using Sort8 = hipcub::BlockRadixSort<uint32_t, NT, KPT8>;  // <= 2,048
  // the keys are sorted in registers, so their LDS image can hold the sort's scratch
  __shared__ union {
    uint32_t key[NB];
    typename Sort2::TempStorage t2;
    typename Sort8::TempStorage t8;
  } s_u;
  uint32_t* s_key = s_u.key;
  __shared__ TACC s_val[NB];
  __shared__ int32_t s_pref[NT + 1];
  __shared__ int32_t s_bst[NT];
  __shared__ TACC s_av[NT];
  __shared__ int32_t s_wsum[NW];
  const int t = threadIdx.x;
  // one row per workgroup by default; a capped grid walks the rows (experiment knob)
  for (int64_t ri = blockIdx.x; ri < n_rows; ri += gridDim.x) {
  const int64_t row = order[ri];
  const int32_t a0 = a_ptr[row];
  const int ns = a_ptr[row + 1] - a0;  // <= NT (host-side classification)
  int len = 0;
  if (t < ns) {
    const int32_t r = a_idx[a0 + t];
    const int32_t b0 = b_ptr[r];
    len = b_ptr[r + 1] - b0;
    s_bst[t] = b0;
    s_av[t] = static_cast<TACC>(a_val[a0 + t]);
  }
  int total;
  const int excl = block_excl_scan<NW>(len, s_wsum, total);  // total <= NB
  s_pref[t] = excl;
  int sz = 64;
  while (sz < total) sz <<= 1;
  __syncthreads();
  // one position per thread (binary search for its step); measured faster than staging by
  // step with 4 B-row reads in flight per wave (World 16.2 vs 17.4 ms)
  for (int q = t; q < sz; q += NT) {
    uint32_t key = 0xffffffffu;
    if (q < total) {
      int lo = 0, hi = ns - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_pref[mid] <= q) lo = mid; else hi = mid - 1;
      }
      const int32_t kk = s_bst[lo] + (q - s_pref[lo]);
      key = (static_cast<uint32_t>(b_idx[kk]) << 11) | static_cast<uint32_t>(q);
      s_val[q] = s_av[lo] * static_cast<TACC>(b_val[kk]);
    }
    s_key[q] = key;
  }
  __syncthreads();
  // Stable LSD radix sort of the blocked keys on their column bits [11, 11 + col_bits): the
  // positions (low 11 bits) enter in traversal order, so equal columns stay in csr_matmat
  // order. Pad keys (all ones) sort last.
  if (sz <= 2 * NT) {
    uint32_t k[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) k[i] = t * 2 + i < sz ? s_key[t * 2 + i] : 0xffffffffu;
    __syncthreads();
    Sort2(s_u.t2).Sort(k, 11, 11 + col_bits);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) s_key[t * 2 + i] = k[i];
  } else {
    uint32_t k[KPT8];
#pragma unroll
    for (int i = 0; i < KPT8; ++i) k[i] = t * KPT8 + i < sz ? s_key[t * KPT8 + i] : 0xffffffffu;
    __syncthreads();
    Sort8(s_u.t8).Sort(k, 11, 11 + col_bits);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KPT8; ++i) s_key[t * KPT8 + i] = k[i];
  }
  __syncthreads();
  // runs of equal columns: thread t owns sorted positions [t*per, (t+1)*per) and sums the
  // runs that START there, in position order
  const int per = (total + NT - 1) / NT;
  const int s0 = min(total, t * per), s1 = min(total, s0 + per);
  int cnt = 0;
  for (int s = s0; s < s1; ++s) {
    const uint32_t col = s_key[s] >> 11;
    if (s > 0 && (s_key[s - 1] >> 11) == col) continue;
    TACC acc = TACC(0);
    for (int u = s; u < total && (s_key[u] >> 11) == col; ++u) acc = acc + s_val[s_key[u] & 2047u];
    cnt += acc != TACC(0) ? 1 : 0;
  }
  int n_kept;
  int o = block_excl_scan<NW>(cnt, s_wsum, n_kept);
  const int64_t out0 = rowoff[row];
  for (int s = s0; s < s1; ++s) {
    const uint32_t col = s_key[s] >> 11;
    if (s > 0 && (s_key[s - 1] >> 11) == col) continue;
    TACC acc = TACC(0);
    for (int u = s; u < total && (s_key[u] >> 11) == col; ++u) acc = acc + s_val[s_key[u] & 2047u];
    if (acc != TACC(0)) {
      t_idx[out0 + o] = static_cast<int32_t>(col);
      t_val[out0 + o] = static_cast<float>(acc);
      ++o;
    }
  }
  if (t == 0) kept[row] = n_kept;
  __syncthreads();  // LDS reuse by the next row
  }
}

// C rows from the upper-bound layout: row i's kept entries at rowoff[i] -> c_ptr[i]. One wave
// per row.
__global__ void spgemm_compact_kernel(int64_t m, const int64_t* __restrict__ rowoff,
                                      const int64_t* __restrict__ cptr64, const int32_t* __restrict__ t_idx,
                                      const float* __restrict__ t_val, int32_t* __restrict__ c_ptr,
                                      int32_t* __restrict__ c_idx, float* __restrict__ c_val) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (blockDim.x / 64);
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6); r <= m; r += waves) {
    const int64_t d = cptr64[r];
    if (lane == 0) c_ptr[r] = static_cast<int32_t>(d);
    if (r == m) continue;
    const int64_t s = rowoff[r], n = cptr64[r + 1] - d;
    for (int64_t k = lane; k < n; k += 64) {
      c_idx[d + k] = t_idx[s + k];
      c_val[d + k] = t_val[s + k];
    }
  }
}

// In-place form: rows [r0, r1) move left inside the caller's capacity-P output, from the
// upper-bound layout (rowoff) to the compact one (cptr64 <= rowoff). The host schedules the
// row ranges so every destination of a launch lies before every source it reads
// (cptr64[r1] <= rowoff[r0]); a single row may overlap itself, which a wave's forward copy
// handles (each iteration's loads complete before its stores, and d <= s). No __restrict__:
// source and destination are the same arrays.
__global__ void spgemm_compact_inplace_kernel(int64_t r0, int64_t r1, const int64_t* __restrict__ rowoff,
                                              const int64_t* __restrict__ cptr64, int32_t* idx, float* val) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (blockDim.x / 64);
  for (int64_t r = r0 + static_cast<int64_t>(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6); r < r1;
       r += waves) {
    const int64_t d = cptr64[r], s = rowoff[r], n = cptr64[r + 1] - d;
    if (d == s) continue;
    // 4 x 64 entries per round: all loads of a round before its stores (d <= s, so a round's
    // stores never reach a source entry of this or a later round)
    constexpr int R = 4;
    for (int64_t k0 = 0; k0 < n; k0 += R * 64) {
      int32_t iv[R];
      float vv[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int64_t k = k0 + u * 64 + lane;
        if (k < n) {
          iv[u] = idx[s + k];
          vv[u] = val[s + k];
        }
      }
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int64_t k = k0 + u * 64 + lane;
        if (k < n) {
          idx[d + k] = iv[u];
          val[d + k] = vv[u];
        }
      }
    }
  }
}

__global__ void cptr32_kernel(int64_t m, const int64_t* __restrict__ cptr64, int32_t* __restrict__ c_ptr) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i <= m; i += stride)
    c_ptr[i] = static_cast<int32_t>(cptr64[i]);
}

// Row ranges for the in-place compaction: rows already in place (cptr == rowoff) are skipped;
// a range starting at r0 extends while its destinations end at or before rowoff[r0]. The gap
// rowoff - cptr only grows with the row, so ranges get longer as rows merge products.
std::vector<std::pair<int64_t, int64_t>> inplace_ranges(const std::vector<int64_t>& rowoff,
                                                        const std::vector<int64_t>& cptr) {
  std::vector<std::pair<int64_t, int64_t>> out;
  const int64_t m = static_cast<int64_t>(rowoff.size()) - 1;
  int64_t r0 = 0;
  while (r0 < m && cptr[r0] == rowoff[r0]) ++r0;
  while (r0 < m) {
    int64_t r1 = r0 + 1;
    while (r1 < m && cptr[r1 + 1] <= rowoff[r0]) ++r1;
    out.emplace_back(r0, r1);
    r0 = r1;
  }
  return out;
}
constexpr size_t kMaxInplaceLaunches = 256;

// Row products (clamped to int32) for the longest-first order.
// Rows that the small-row kernel cannot take (more than kSmallSteps nonzeros) are keyed
// above kSmallProducts so they sort into the dense-slab set.
__global__ void row_products_u32_kernel(int64_t m, const int64_t* __restrict__ rowoff,
                                        const int32_t* __restrict__ a_ptr, int small_ok,
                                        uint32_t* __restrict__ key, int32_t* __restrict__ id) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < m; i += stride) {
    int64_t v = rowoff[i + 1] - rowoff[i];
    if (v <= kSmallProducts && (!small_ok || a_ptr[i + 1] - a_ptr[i] > kSmallSteps)) v = kSmallProducts + 1;
    key[i] = static_cast<uint32_t>(v > 0xffffffffLL ? 0xffffffffLL : v);
    id[i] = static_cast<int32_t>(i);
  }
}

template <typename TACC> struct RowsSlab;
template <> struct RowsSlab<float> { static constexpr int kMax = 25 * kRowsNT; };   // 100 KB
template <> struct RowsSlab<double> { static constexpr int kMax = 13 * kRowsNT; };  // 104 KB
constexpr int kRowsMaxSlabs = 8;

template <typename TA, typename TACC>
gcg_status spgemm_rows(int64_t m, int64_t p, int64_t nnz_a, const int32_t* a_ptr, const int32_t* a_idx,
                       const TA* a_val, const int32_t* b_ptr, const int32_t* b_idx, const float* b_val,
                       int64_t n_products, const int64_t* rowoff_dev, const std::vector<int64_t>& rowoff,
                       int32_t* c_ptr, int32_t* c_idx, float* c_val, int64_t* nnz_c_dev, hipStream_t st, int flags) {
  (void)nnz_a; (void)n_products;
  constexpr int SMAX = RowsSlab<TACC>::kMax;
  const int64_t n_slabs = (p + SMAX - 1) / SMAX;
  int64_t sw = (p + n_slabs - 1) / n_slabs;
  sw = std::max<int64_t>(kRowsNT, (sw + kRowsNT - 1) / kRowsNT * kRowsNT);
  // The row kernels write C in the upper-bound layout (row i at rowoff[i]) straight into the
  // caller's capacity-P c_idx / c_val, which are then compacted in place: no products-sized
  // temporary (21 GB at Twitter-World) is allocated per call.
  DevBuf b_key, b_key2, b_id, b_id2, b_kept, b_cp64, b_tmp;
  size_t t_sort = 0, t_scan = 0;
  {
    uint32_t* k = nullptr; int32_t* v = nullptr; int64_t* o = nullptr;
    if (hipcub::DeviceRadixSort::SortPairsDescending(nullptr, t_sort, k, k, v, v, static_cast<int>(m)) != hipSuccess ||
        hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, o, o, static_cast<int>(m + 1)) != hipSuccess)
      return fail(GCG_ERR_HIP, "hipcub sizing failed");
  }
  auto alloc = [&](DevBuf& b, size_t bytes) -> hipError_t {
    b.s = st;
    return hipMallocAsync(&b.p, std::max<size_t>(bytes, 16), st);
  };
  hipError_t e = alloc(b_key, m * sizeof(uint32_t));
  if (e == hipSuccess) e = alloc(b_key2, m * sizeof(uint32_t));
  if (e == hipSuccess) e = alloc(b_id, m * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_id2, m * sizeof(int32_t));
  if (e == hipSuccess) e = alloc(b_kept, (m + 1) * sizeof(int64_t));
  if (e == hipSuccess) e = alloc(b_cp64, (m + 1) * sizeof(int64_t));
  if (e == hipSuccess) e = alloc(b_tmp, std::max(t_sort, t_scan));
  if (e != hipSuccess) return fail(GCG_ERR_ALLOC, "SpGEMM row temporaries: %s", hipGetErrorString(e));
  auto* key = static_cast<uint32_t*>(b_key.p);
  auto* key2 = static_cast<uint32_t*>(b_key2.p);
  auto* id = static_cast<int32_t*>(b_id.p);
  auto* id2 = static_cast<int32_t*>(b_id2.p);
  auto* kept = static_cast<int64_t*>(b_kept.p);
  auto* cp64 = static_cast<int64_t*>(b_cp64.p);
  const int small_ok = (p <= kSmallMaxCols && !(flags & GCG_SPGEMM_DENSE_SLABS)) ? 1 : 0;
  hipLaunchKernelGGL(row_products_u32_kernel, dim3(grid_for(m)), dim3(256), 0, st, m, rowoff_dev, a_ptr, small_ok,
                     key, id);
  GCG_HIP_CHECK(hipGetLastError());
  size_t tb = t_sort;
  GCG_HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(b_tmp.p, tb, key, key2, id, id2, static_cast<int>(m), 0, 32, st));
  GCG_HIP_CHECK(hipMemsetAsync(kept + m, 0, sizeof(int64_t), st));
  // rows [0, n_big) of the longest-first order take the dense slabs, the rest the sort kernel
  std::vector<uint32_t> skey(m);
  GCG_HIP_CHECK(hipMemcpyAsync(skey.data(), key2, m * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  const int64_t n_big = std::lower_bound(skey.begin(), skey.end(), static_cast<uint32_t>(kSmallProducts),
                                         [](uint32_t a, uint32_t b) { return a > b; }) - skey.begin();
  auto* tidx = c_idx;
  auto* tval = c_val;
  // Measured (tools/exp_spgemm_knobs.py, Twitter-World): the small-row kernel on a side stream
  // beside the dense-slab kernel ran 5x SLOWER (615 vs 112 ms; the two kernels' workgroups
  // compete for LDS), and a persistent grid was no faster than one workgroup per row -- so one
  // stream, one workgroup per row.
  int col_bits = 1;  // (1 << col_bits) > p: the pad key's column bits exceed every column
  while ((int64_t{1} << col_bits) <= p) ++col_bits;
  auto small_launch = [&](auto kern, int64_t r0, int64_t r1) {
    if (r1 <= r0) return;
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(r1 - r0)),
                       dim3(kSmallNT), 0, st, id2 + r0, a_ptr, a_idx, a_val, b_ptr, b_idx, b_val, rowoff_dev, tidx,
                       tval, kept, r1 - r0, col_bits);
  };
  // measured: a second instance for rows of <= 512 products with a quarter of the LDS (8
  // workgroups per CU instead of ~5) left the small-row time unchanged (16.2 vs 16.3 ms, World)
  small_launch(spgemm_small_rows_kernel<TA, TACC>, n_big, m);
  if (n_big > 0)
    hipLaunchKernelGGL((spgemm_rows_kernel<TA, TACC, SMAX>), dim3(static_cast<unsigned>(n_big)), dim3(kRowsNT), 0, st,
                       p, static_cast<int>(sw), id2, a_ptr, a_idx, a_val, b_ptr, b_idx, b_val, rowoff_dev, tidx,
                       tval, kept);
  const hipError_t launch_err = hipGetLastError();
  if (launch_err != hipSuccess) return fail(GCG_ERR_HIP, "SpGEMM row kernels: %s", hipGetErrorString(launch_err));
  tb = t_scan;
  GCG_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(b_tmp.p, tb, kept, cp64, static_cast<int>(m + 1), st));
  std::vector<int64_t> cptr(m + 1);
  GCG_HIP_CHECK(hipMemcpyAsync(cptr.data(), cp64, (m + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));
  const int64_t nnz_c = cptr[m];
  if (nnz_c > INT32_MAX) return fail(GCG_ERR_INVALID_ARG, "nnz(C) = %lld exceeds int32 CSR", (long long)nnz_c);
  hipLaunchKernelGGL(cptr32_kernel, dim3(grid_for(m + 1)), dim3(256), 0, st, m, cp64, c_ptr);
  const auto ranges = inplace_ranges(rowoff, cptr);
  if (ranges.size() <= kMaxInplaceLaunches && !(flags & GCG_SPGEMM_COMPACT_TEMPORARY)) {
    for (const auto& rg : ranges)
      hipLaunchKernelGGL(spgemm_compact_inplace_kernel, dim3(grid_for((rg.second - rg.first) * 64)), dim3(256), 0,
                         st, rg.first, rg.second, rowoff_dev, cp64, c_idx, c_val);
  } else {  // rows that merge few products: compact through an nnz(C)-sized temporary instead
    DevBuf b_cidx, b_cval;
    e = alloc(b_cidx, nnz_c * sizeof(int32_t));
    if (e == hipSuccess) e = alloc(b_cval, nnz_c * sizeof(float));
    if (e != hipSuccess) return fail(GCG_ERR_ALLOC, "SpGEMM compaction temporary: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(spgemm_compact_kernel, dim3(grid_for(m * 64)), dim3(256), 0, st, m, rowoff_dev, cp64,
                       c_idx, c_val, c_ptr, static_cast<int32_t*>(b_cidx.p), static_cast<float*>(b_cval.p));
    GCG_HIP_CHECK(hipGetLastError());
    GCG_HIP_CHECK(hipMemcpyAsync(c_idx, b_cidx.p, nnz_c * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    GCG_HIP_CHECK(hipMemcpyAsync(c_val, b_cval.p, nnz_c * sizeof(float), hipMemcpyDeviceToDevice, st));
  }
  GCG_HIP_CHECK(hipGetLastError());
  GCG_HIP_CHECK(hipMemcpyAsync(nnz_c_dev, cp64 + m, sizeof(int64_t), hipMemcpyDeviceToDevice, st));
  GCG_HIP_CHECK(hipStreamSynchronize(st));  // temporaries are freed stream-ordered on return
  return GCG_OK;
}

// Products per row chunk: the expand-sort-reduce temporaries are ~40 B per product, so a
// chunk of 2^29 products holds ~21 GB of HBM; row chunks also keep every hipcub item count
// and the int32 permutation within range. Twitter-World H.X (2.65e9 products) -> 5 chunks.
// gcg_spgemm_ex's chunk_products (> 0) overrides it -- the tests force many chunks.
constexpr int64_t kChunkProductsDefault = int64_t{1} << 29;

template <typename TA, typename TACC>
gcg_status spgemm_impl(int64_t m, int64_t n, int64_t p, int64_t nnz_a, const int32_t* a_ptr,
                       const int32_t* a_idx, const TA* a_val, int64_t nnz_b, const int32_t* b_ptr,
                       const int32_t* b_idx, const float* b_val, int64_t n_products, int32_t* c_ptr,
                       int32_t* c_idx, float* c_val, int64_t* nnz_c_dev, hipStream_t st, int path,
                       int64_t chunk_products) {
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
  if (m <= INT32_MAX && (p + RowsSlab<TACC>::kMax - 1) / RowsSlab<TACC>::kMax <= kRowsMaxSlabs &&
      !(path & GCG_SPGEMM_EXPAND_SORT))
    return spgemm_rows<TA, TACC>(m, p, nnz_a, a_ptr, a_idx, a_val, b_ptr, b_idx, b_val, n_products, rowoff_dev,
                                 rowoff, c_ptr, c_idx, c_val, nnz_c_dev, st, path);
  const int64_t kChunkProducts = chunk_products > 0 ? chunk_products : kChunkProductsDefault;
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
  return gcg_spgemm_ex(m, n, p, nnz_a, a_ptr, a_idx, a_val, a_is_f64, nnz_b, b_ptr, b_idx, b_val,
                       accumulate_f64, n_products, c_ptr, c_idx, c_val, nnz_c_dev, 0, 0, stream);
}

gcg_status gcg_spgemm_ex(int64_t m, int64_t n, int64_t p, int64_t nnz_a, const int32_t* a_ptr,
                         const int32_t* a_idx, const void* a_val, int a_is_f64, int64_t nnz_b,
                         const int32_t* b_ptr, const int32_t* b_idx, const float* b_val,
                         int accumulate_f64, int64_t n_products, int32_t* c_ptr, int32_t* c_idx,
                         float* c_val, int64_t* nnz_c_dev, int32_t flags, int64_t chunk_products,
                         gcg_stream_t stream) {
  if (m < 0 || n < 0 || p < 0 || nnz_a < 0 || nnz_b < 0 || n_products < 0 || c_ptr == nullptr ||
      nnz_c_dev == nullptr || a_ptr == nullptr || b_ptr == nullptr)
    return fail(GCG_ERR_INVALID_ARG, "bad args to gcg_spgemm");
  if (n_products > 0 && (c_idx == nullptr || c_val == nullptr || a_idx == nullptr || a_val == nullptr ||
                         b_idx == nullptr || b_val == nullptr))
    return fail(GCG_ERR_INVALID_ARG, "NULL buffer");
  if (a_is_f64 && !accumulate_f64) return fail(GCG_ERR_INVALID_ARG, "float64 A needs accumulate_f64");
  if (flags & ~(GCG_SPGEMM_EXPAND_SORT | GCG_SPGEMM_DENSE_SLABS | GCG_SPGEMM_COMPACT_TEMPORARY))
    return fail(GCG_ERR_INVALID_ARG, "unknown gcg_spgemm_ex flags 0x%x", flags);
  if (chunk_products < 0) return fail(GCG_ERR_INVALID_ARG, "chunk_products < 0");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (a_is_f64)
    return spgemm_impl<double, double>(m, n, p, nnz_a, a_ptr, a_idx, static_cast<const double*>(a_val), nnz_b,
                                       b_ptr, b_idx, b_val, n_products, c_ptr, c_idx, c_val, nnz_c_dev, st,
                                       flags, chunk_products);
  if (accumulate_f64)
    return spgemm_impl<float, double>(m, n, p, nnz_a, a_ptr, a_idx, static_cast<const float*>(a_val), nnz_b,
                                      b_ptr, b_idx, b_val, n_products, c_ptr, c_idx, c_val, nnz_c_dev, st,
                                      flags, chunk_products);
  return spgemm_impl<float, float>(m, n, p, nnz_a, a_ptr, a_idx, static_cast<const float*>(a_val), nnz_b,
                                   b_ptr, b_idx, b_val, n_products, c_ptr, c_idx, c_val, nnz_c_dev, st,
                                   flags, chunk_products);
}

}  // extern "C"
