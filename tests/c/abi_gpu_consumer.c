/* A plain C99 caller of include/gcg_spmm.h on the GPU: what a C / cgo / JNI binding of the
 * S.dot(H, Z) replacement (mlpconv.py:73) does -- hipMalloc the CSR and the dense operand,
 * call the C-ABI on a stream, read back, compare. No Python, no torch. The host reference is
 * scipy's csr_matvecs loop (storage order, product and sum rounded separately: build with
 * -ffp-contract=off), so the plan-less and ordered results must match it bit for bit.
 * Exit code 0 = all checks passed; prints "gpu abi ok". */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gcg_spmm.h"

#define CHECK_HIP(x)                                                       \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      return 10;                                                           \
    }                                                                      \
  } while (0)
#define CHECK_GCG(x)                                                           \
  do {                                                                         \
    gcg_status s_ = (x);                                                       \
    if (s_ != GCG_OK) {                                                        \
      printf("gcg status %d at line %d: %s\n", (int)s_, __LINE__, gcg_last_error()); \
      return 11;                                                               \
    }                                                                          \
  } while (0)

static uint32_t lcg = 12345u;
static uint32_t rnd(void) { lcg = lcg * 1664525u + 1013904223u; return lcg >> 8; }
static float frnd(void) { return (float)(rnd() % 2000001) / 1000000.0f - 1.0f; }

/* Y[i] = act(sum_j v_j * Z[c_j] + b) for rows r = rows ? rows[i] : i (csr_matvecs order) */
static void host_spmm(int n_out, const int32_t* indptr, const int32_t* idx, const float* val,
                      const float* Z, int K, const float* bias, int relu, const int32_t* rows,
                      float* Y) {
  for (int i = 0; i < n_out; ++i) {
    const int r = rows ? rows[i] : i;
    for (int c = 0; c < K; ++c) {
      float acc = 0.0f;
      for (int j = indptr[r]; j < indptr[r + 1]; ++j) {
        const float p = val[j] * Z[(size_t)idx[j] * K + c];
        acc = acc + p;
      }
      if (bias) acc = acc + bias[c];
      if (relu) acc = 0.5f * (acc + fabsf(acc));
      Y[(size_t)i * K + c] = acc;
    }
  }
}

int main(void) {
  const int n = 3000, K = 300, n_sub = 700;
  /* CSR with ragged rows: mostly 0-40 nnz, a few long rows (one of 5000) and empty rows */
  int32_t* indptr = malloc(sizeof(int32_t) * (n + 1));
  indptr[0] = 0;
  for (int r = 0; r < n; ++r) {
    int len = (int)(rnd() % 41);
    if (r % 97 == 0) len = 0;
    if (r == 11) len = 5000;
    if (r == 2000) len = 1300;
    indptr[r + 1] = indptr[r] + len;
  }
  const int nnz = indptr[n];
  int32_t* idx = malloc(sizeof(int32_t) * nnz);
  float* val = malloc(sizeof(float) * nnz);
  for (int j = 0; j < nnz; ++j) { idx[j] = (int32_t)(rnd() % n); val[j] = frnd(); }
  float* Z = malloc(sizeof(float) * n * K);
  for (int i = 0; i < n * K; ++i) Z[i] = frnd();
  float bias[300];
  for (int c = 0; c < K; ++c) bias[c] = (c % 7 == 0) ? 0.0f : 0.1f * frnd();
  int32_t rows[700];
  for (int i = 0; i < n_sub; ++i) rows[i] = (int32_t)(rnd() % n);
  rows[0] = 11;
  rows[1] = 11; /* duplicates, as train indices drawn with replacement (tensormain.py:226) */

  float* ref = malloc(sizeof(float) * n * K);
  float* got = malloc(sizeof(float) * n * K);

  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));
  int32_t *d_ptr, *d_idx, *d_rows;
  float *d_val, *d_Z, *d_Y, *d_b;
  uint8_t* d_gate;
  CHECK_HIP(hipMalloc((void**)&d_ptr, sizeof(int32_t) * (n + 1)));
  CHECK_HIP(hipMalloc((void**)&d_idx, sizeof(int32_t) * nnz));
  CHECK_HIP(hipMalloc((void**)&d_val, sizeof(float) * nnz));
  CHECK_HIP(hipMalloc((void**)&d_Z, sizeof(float) * n * K));
  CHECK_HIP(hipMalloc((void**)&d_Y, sizeof(float) * n * K));
  CHECK_HIP(hipMalloc((void**)&d_b, sizeof(float) * K));
  CHECK_HIP(hipMalloc((void**)&d_rows, sizeof(int32_t) * n_sub));
  CHECK_HIP(hipMalloc((void**)&d_gate, (size_t)n * K));
  CHECK_HIP(hipMemcpy(d_ptr, indptr, sizeof(int32_t) * (n + 1), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_idx, idx, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_val, val, sizeof(float) * nnz, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_Z, Z, sizeof(float) * n * K, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_b, bias, sizeof(float) * K, hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(d_rows, rows, sizeof(int32_t) * n_sub, hipMemcpyHostToDevice));

  int32_t status = -1, *d_status;
  CHECK_HIP(hipMalloc((void**)&d_status, sizeof(int32_t)));
  CHECK_GCG(gcg_csr_validate(n, n, nnz, d_ptr, d_idx, d_status, st));
  CHECK_HIP(hipMemcpyAsync(&status, d_status, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipStreamSynchronize(st));
  if (status != 0) { printf("validate: %d\n", status); return 20; }

  /* 1) plan-less, bias + rectify: bitwise */
  CHECK_GCG(gcg_spmm_csr_f32(n, n, nnz, d_ptr, d_idx, d_val, d_Z, K, K, d_Y, K, d_b, GCG_ACT_RELU,
                             NULL, 0, st));
  CHECK_HIP(hipMemcpyAsync(got, d_Y, sizeof(float) * n * K, hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipStreamSynchronize(st));
  host_spmm(n, indptr, idx, val, Z, K, bias, 1, NULL, ref);
  if (memcmp(got, ref, sizeof(float) * n * K) != 0) { printf("plan-less differs\n"); return 21; }

  /* 2) ordered plan: bitwise, plain product */
  gcg_spmm_plan* plan = NULL;
  CHECK_GCG(gcg_spmm_plan_create(&plan, n, n, nnz, d_ptr, NULL, 0, 256, 1, st));
  size_t wsb = 0;
  CHECK_GCG(gcg_spmm_plan_workspace_bytes(plan, K, &wsb));
  if (wsb != 0) { printf("ordered plan wants a workspace\n"); return 22; }
  CHECK_GCG(gcg_spmm_csr_f32_planned(plan, d_ptr, d_idx, d_val, d_Z, K, K, d_Y, K, NULL,
                                     GCG_ACT_NONE, NULL, 0, st));
  CHECK_HIP(hipMemcpyAsync(got, d_Y, sizeof(float) * n * K, hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipStreamSynchronize(st));
  host_spmm(n, indptr, idx, val, Z, K, NULL, 0, NULL, ref);
  if (memcmp(got, ref, sizeof(float) * n * K) != 0) { printf("ordered differs\n"); return 23; }
  CHECK_GCG(gcg_spmm_plan_destroy(plan));

  /* 3) fast plan (long rows split into segments + fix-up): 1e-5, bitwise on unsplit rows */
  CHECK_GCG(gcg_spmm_plan_create(&plan, n, n, nnz, d_ptr, NULL, 0, 256, 0, st));
  CHECK_GCG(gcg_spmm_plan_workspace_bytes(plan, K, &wsb));
  void* d_ws = NULL;
  if (wsb == 0) { printf("fast plan split no row\n"); return 24; }
  CHECK_HIP(hipMalloc(&d_ws, wsb));
  CHECK_GCG(gcg_spmm_csr_f32_planned(plan, d_ptr, d_idx, d_val, d_Z, K, K, d_Y, K, NULL,
                                     GCG_ACT_NONE, d_ws, wsb, st));
  CHECK_HIP(hipMemcpyAsync(got, d_Y, sizeof(float) * n * K, hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipStreamSynchronize(st));
  for (int r = 0; r < n; ++r) {
    const int split = indptr[r + 1] - indptr[r] > 256;
    for (int c = 0; c < K; ++c) {
      const float a = got[(size_t)r * K + c], b = ref[(size_t)r * K + c];
      if (split ? fabsf(a - b) > 1e-4f * (1.0f + fabsf(b)) : a != b) {
        printf("fast differs at row %d col %d: %g vs %g\n", r, c, a, b);
        return 25;
      }
    }
  }
  /* too small a workspace is a status, not a fault */
  if (gcg_spmm_csr_f32_planned(plan, d_ptr, d_idx, d_val, d_Z, K, K, d_Y, K, NULL, GCG_ACT_NONE,
                               d_ws, wsb - 16, st) != GCG_ERR_WORKSPACE)
    return 26;
  CHECK_GCG(gcg_spmm_plan_destroy(plan));

  /* 4) row subset with duplicates (target_indices, mlpconv.py:94) + gate, planned ordered */
  CHECK_GCG(gcg_spmm_plan_create(&plan, n, n, nnz, d_ptr, d_rows, n_sub, 256, 1, st));
  CHECK_GCG(gcg_spmm_csr_f32_planned_gate(plan, d_ptr, d_idx, d_val, d_Z, K, K, d_Y, K, d_b,
                                          GCG_ACT_RELU, d_gate, K, NULL, 0, st));
  uint8_t* gate = malloc((size_t)n_sub * K);
  CHECK_HIP(hipMemcpyAsync(got, d_Y, sizeof(float) * n_sub * K, hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipMemcpyAsync(gate, d_gate, (size_t)n_sub * K, hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipStreamSynchronize(st));
  float* pre = malloc(sizeof(float) * n_sub * K);
  host_spmm(n_sub, indptr, idx, val, Z, K, bias, 0, rows, pre);
  host_spmm(n_sub, indptr, idx, val, Z, K, bias, 1, rows, ref);
  if (memcmp(got, ref, sizeof(float) * n_sub * K) != 0) { printf("subset differs\n"); return 27; }
  int zeros = 0;
  for (int i = 0; i < n_sub * K; ++i) {
    const uint8_t want = pre[i] > 0.0f ? 2 : (pre[i] == 0.0f ? 1 : 0);
    zeros += pre[i] == 0.0f;
    if (gate[i] != want) { printf("gate differs at %d\n", i); return 28; }
  }
  /* 4b) the same subset with a gather hint (bit 31 on every other column: non-temporal
   *     gathers of those rows): the cache policy changes, the bytes do not */
  int32_t* hint = malloc(sizeof(int32_t) * nnz);
  for (int i = 0; i < nnz; ++i) hint[i] = (idx[i] & 1) ? (int32_t)((uint32_t)idx[i] | 0x80000000u) : idx[i];
  int32_t* d_hint;
  CHECK_HIP(hipMalloc((void**)&d_hint, sizeof(int32_t) * nnz));
  CHECK_HIP(hipMemcpy(d_hint, hint, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
  CHECK_GCG(gcg_spmm_csr_f32_planned_hint(plan, d_ptr, d_idx, d_val, d_Z, K, K, d_Y, K, d_b,
                                          GCG_ACT_RELU, d_gate, K, NULL, 0, d_hint, st));
  CHECK_HIP(hipMemcpyAsync(got, d_Y, sizeof(float) * n_sub * K, hipMemcpyDeviceToHost, st));
  CHECK_HIP(hipStreamSynchronize(st));
  if (memcmp(got, ref, sizeof(float) * n_sub * K) != 0) { printf("hinted subset differs\n"); return 31; }
  CHECK_GCG(gcg_spmm_plan_destroy(plan));

  /* 5) argument errors come back as status codes with a message */
  if (gcg_spmm_csr_f32(n, n, nnz, d_ptr, d_idx, d_val, d_Z, K, K, d_Y, K - 1, NULL, 0, NULL, 0,
                       st) != GCG_ERR_INVALID_ARG || strlen(gcg_last_error()) == 0)
    return 29;
  if (gcg_spmm_csr_f32_gate(n, n, nnz, d_ptr, d_idx, d_val, d_Z, K, K, d_Y, K, NULL, GCG_ACT_NONE,
                            NULL, 0, d_gate, K, st) != GCG_ERR_INVALID_ARG)
    return 30;

  CHECK_HIP(hipStreamSynchronize(st));
  hipFree(d_ptr); hipFree(d_idx); hipFree(d_val); hipFree(d_Z); hipFree(d_Y); hipFree(d_b);
  hipFree(d_rows); hipFree(d_gate); hipFree(d_ws); hipFree(d_status); hipFree(d_hint);
  CHECK_HIP(hipStreamDestroy(st));
  printf("gpu abi ok: %d rows, %d nnz, K=%d, plan-less/ordered/subset+gate(+hint) bitwise, "
         "fast within 1e-4 (%d exact-zero pre-activations)\n", n, nnz, K, zeros);
  free(indptr); free(idx); free(val); free(Z); free(ref); free(got); free(gate); free(pre);
  free(hint);
  return 0;
}
