/*
 * spmm_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * CPU restatement of the arithmetic behind the reference's `S.dot(H, Z)`
 * (mlpconv.py:71,73,90). Theano's sparse Dot perform evaluates `x * y` with
 * scipy, i.e. scipy.sparse `_mul_multivector` -> sparsetools `csr_matvecs`
 * (third-party, not vendored in /root/reference; scipy 1.15.3 in this image):
 *
 *     Y = zeros(n_rows, K)
 *     for i in rows:
 *         for jj in indptr[i] .. indptr[i+1]-1:       (CSR storage order)
 *             a = data[jj];  x = Z[indices[jj], :]
 *             for k in 0..K-1:  Y[i,k] += a * x[k]     (product rounded, then sum rounded)
 *
 * Built with -ffp-contract=off so `y += a * x` is a rounded multiply followed by a
 * rounded add, as scipy's x86-64 build (no FMA) computes it. tests/test_oracle.py
 * pins this against scipy itself bit for bit.
 *
 * Also restates:
 *   - the epilogue of mlpconv.py:75-77 / 92-94 (+ b, rectify = 0.5*(x+|x|), [rows]);
 *   - the scatter-add (inc_subtensor) Theano uses for the gradient of Y[target_indices]
 *     (mlpconv.py:94), duplicates added in index order.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

/* Y[i] = act(sum_j vals[j] * Z[indices[j]] + bias) for output row i <- CSR row rows[i]. */
int oracle_spmm_f32(int64_t n_rows, const int32_t* indptr, const int32_t* indices,
                    const float* vals, const float* Z, int64_t ldz, int64_t K, float* Y,
                    int64_t ldy, const float* bias, int act, const int32_t* rows, int64_t n_out) {
  if (rows == NULL) n_out = n_rows;
  for (int64_t i = 0; i < n_out; ++i) {
    const int64_t r = rows ? rows[i] : i;
    if (r < 0 || r >= n_rows) return 1;
    float* y = Y + i * ldy;
    for (int64_t k = 0; k < K; ++k) y[k] = 0.0f;
    for (int32_t jj = indptr[r]; jj < indptr[r + 1]; ++jj) {
      const float a = vals[jj];
      const float* x = Z + (int64_t)indices[jj] * ldz;
      for (int64_t k = 0; k < K; ++k) y[k] += a * x[k];
    }
    if (bias)
      for (int64_t k = 0; k < K; ++k) y[k] = y[k] + bias[k];
    if (act == 1)
      for (int64_t k = 0; k < K; ++k) y[k] = 0.5f * (y[k] + fabsf(y[k]));
  }
  return 0;
}

/* Same in float64 (the "exact" reference for tolerance checks). */
int oracle_spmm_f64(int64_t n_rows, const int32_t* indptr, const int32_t* indices,
                    const double* vals, const double* Z, int64_t ldz, int64_t K, double* Y,
                    int64_t ldy) {
  for (int64_t i = 0; i < n_rows; ++i) {
    double* y = Y + i * ldy;
    for (int64_t k = 0; k < K; ++k) y[k] = 0.0;
    for (int32_t jj = indptr[i]; jj < indptr[i + 1]; ++jj) {
      const double a = vals[jj];
      const double* x = Z + (int64_t)indices[jj] * ldz;
      for (int64_t k = 0; k < K; ++k) y[k] += a * x[k];
    }
  }
  return 0;
}

/* out[idx[i]] += src[i] for i ascending (Theano AdvancedIncSubtensor1 semantics). */
int oracle_scatter_add_f32(int64_t n_idx, const int32_t* idx, const float* src, int64_t lds,
                           int64_t K, float* out, int64_t ldo, int64_t n_rows) {
  for (int64_t i = 0; i < n_idx; ++i) {
    if (idx[i] < 0 || idx[i] >= n_rows) return 1;
    float* o = out + (int64_t)idx[i] * ldo;
    const float* s = src + i * lds;
    for (int64_t k = 0; k < K; ++k) o[k] = o[k] + s[k];
  }
  return 0;
}
