/*
 * gcg_spmm.h -- C-ABI of the MI355X (gfx950) graph-convolution hot path.
 *
 * This is the drop-in boundary for the one hot path of afcarl/graphconvgeo:
 * the normalized-adjacency x dense-features product Y = act(H . Z + b) that the
 * reference computes with `theano.sparse.dot` (S.dot) inside its two Lasagne
 * graph-convolution layers. Every entry point names the reference site it replaces.
 *
 *   reference                                   replaced by
 *   ------------------------------------------  -----------------------------------
 *   mlpconv.py:73   S.dot(self.H, activation)   gcg_spmm_csr_f32 / _planned
 *   mlpconv.py:90   S.dot(self.H, activation)   (same; width C instead of K)
 *   mlpconv.py:71   S.dot(input, self.W)        (same kernel: X (CSR N x F) . W1)
 *   mlpconv.py:75-77 + b, rectify               fused epilogue: bias != NULL, act = GCG_ACT_RELU
 *   mlpconv.py:92-94 + b, [target_indices, :]   fused epilogue: bias, out_rows subset
 *   Theano grad of S.dot (x.T . gz)             gcg_spmm_* on CSR(H^T) (= H, H symmetric)
 *                                               and CSR(X^T) from gcg_csr_transpose_f32
 *   Theano grad of Y[target_indices] (inc_subtensor, duplicates add)
 *                                               gcg_scatter_add_rows_f32
 *   data.py:226-250,364-370 graph projection    gcg_project_mention_graph
 *   tensormain.py:170-180 H = D^-1/2 (A+I) D^-1/2  gcg_normalize_adjacency_f32
 *   main.py:530 / tensormain.py:114 X_conv = H * X gcg_spgemm_products + gcg_spgemm
 *
 * Conventions (scipy CSR layout, as `scipy.sparse.csr_matrix` holds it):
 *   indptr  int32[n_rows + 1], indices int32[nnz], vals float32[nnz]; dense operands
 *   are row-major float32 with an explicit leading dimension (elements, >= K), K <= 4,194,240.
 *   All pointers are DEVICE pointers (hipMalloc / torch CUDA tensors) unless the
 *   parameter name ends in `_host`. Nothing in the hot path allocates, synchronizes,
 *   or throws; every function returns a gcg_status (0 = ok). `stream` is a
 *   hipStream_t (NULL = the legacy default stream). Calls are reentrant per stream;
 *   the only global state is the per-thread last-error message.
 *
 * Numerics: per output element the products H[r,j]*Z[j,c] are accumulated in
 * CSR storage order, each product and each sum rounded separately (no FMA).
 * That is exactly scipy's `csr_matvecs` (the executor behind the reference's
 * S.dot), so the plan-less and ordered paths match scipy float32 bit for bit.
 * The planned fast path splits rows longer than its task size across waves and
 * adds the per-segment partials in order: equal to scipy within 1e-5 (abs, on
 * normalized-H inputs), not bitwise, for those rows only.
 */
#ifndef GCG_SPMM_H
#define GCG_SPMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* gcg_stream_t; /* hipStream_t */

typedef enum {
  GCG_OK = 0,
  GCG_ERR_INVALID_ARG = 1,  /* null pointer, negative or inconsistent size   */
  GCG_ERR_MISALIGNED = 2,   /* pointer not 4-byte aligned                     */
  GCG_ERR_HIP = 3,          /* a HIP runtime call or kernel launch failed     */
  GCG_ERR_ALLOC = 4,        /* host or device allocation failed (plan create) */
  GCG_ERR_BAD_CSR = 5,      /* indptr not monotone / out of range, bad index  */
  GCG_ERR_WORKSPACE = 6     /* workspace missing or too small                 */
} gcg_status;

enum { GCG_ACT_NONE = 0, GCG_ACT_RELU = 1 };

/* Library version, "major.minor.patch". */
const char* gcg_version(void);
/* Content hash of the sources the library was built from (graphconvgeo_amd/_build.py
 * source_hash); the Python binding refuses a library whose hash differs from the tree's. */
const char* gcg_source_hash(void);
/* Text of the last error raised on this host thread ("" if none). */
const char* gcg_last_error(void);

/*
 * Plan-less SpMM, one 64-lane wave per output row, storage-order accumulation:
 *   for i in [0, n_out):  r = out_rows ? out_rows[i] : i
 *       Y[i, 0:K] = act( sum_{j in row r, storage order} vals[j] * Z[indices[j], 0:K] + bias )
 * n_out == n_rows when out_rows == NULL. Bitwise equal to scipy float32 `H @ Z`
 * (rows re-indexed by out_rows). Replaces S.dot at mlpconv.py:71,73,90 and the
 * row gather at mlpconv.py:94. The CSR must be valid (see gcg_csr_validate).
 * Vector width: 16-B gathers when ldz % 4 == 0, ldy % 4 == 0 and Z / Y / bias are 16-B
 * aligned. When K % 4 != 0 they still are (round 4): the last vector of a row also READS Z's
 * columns [K, round4(K)) -- inside the row, since ldz % 4 == 0 means ldz >= round4(K), and
 * never used -- so Z's buffer must extend to column round4(K) of its last row (any [n, ldz]
 * allocation does); bias, Y and gate are never touched past column K.
 */
gcg_status gcg_spmm_csr_f32(int64_t n_rows, int64_t n_cols, int64_t nnz,
                            const int32_t* indptr, const int32_t* indices,
                            const float* vals, const float* Z, int64_t ldz, int64_t K,
                            float* Y, int64_t ldy, const float* bias, int act,
                            const int32_t* out_rows, int64_t n_out,
                            gcg_stream_t stream);

/*
 * nnz-balanced launch plan for one CSR (and one optional output-row list).
 * Built once per H (H is shared by both layers and every epoch, mlpconv.py:214,293),
 * reused for every K. Reads indptr (and out_rows) back to the host once and
 * validates indptr; this call synchronizes `stream` -- it is NOT a hot-path call.
 *   task_nnz  : target nonzeros per wave task (0 = default: clamp(nnz / 8192, 32, 512), ordered
 *               plans clamp(nnz / 32768, 32, 128), or up to 256 when rows average >= 256
 *               nonzeros).
 *   ordered   : 1 = never split a row's sum (bitwise scipy order): rows longer than task_nnz
 *                   are scheduled first, those longer than 8 x task_nnz on a whole workgroup
 *                   each (the storage-order sum handed from wave to wave, still bitwise); one
 *                   also longer than 1/768 of the plan's nonzeros is cut into 2 column slices
 *                   on two workgroups when the launch is two 256-float chunks wide (256 < K
 *                   per 512-float panel, round 5): each slice sums all the row's nonzeros for
 *                   its columns, in storage order -- still bitwise;
 *               2 = ordered with every whole-workgroup row unsliced (A/B and tests);
 *               0 = split rows longer than task_nnz into segments (fast).
 */
typedef struct gcg_spmm_plan gcg_spmm_plan;

gcg_status gcg_spmm_plan_create(gcg_spmm_plan** plan, int64_t n_rows, int64_t n_cols,
                                int64_t nnz, const int32_t* indptr,
                                const int32_t* out_rows, int64_t n_out, int64_t task_nnz,
                                int ordered, gcg_stream_t stream);
gcg_status gcg_spmm_plan_destroy(gcg_spmm_plan* plan);
/* Bytes of device workspace gcg_spmm_csr_f32_planned needs for width K (0 if none). */
gcg_status gcg_spmm_plan_workspace_bytes(const gcg_spmm_plan* plan, int64_t K, size_t* bytes);
/* Plan statistics: tasks, long rows (split into segments in a fast plan, run on a whole
 * workgroup in an ordered plan), segments, max task nnz. */
gcg_status gcg_spmm_plan_info(const gcg_spmm_plan* plan, int64_t* n_tasks, int64_t* n_long_rows,
                              int64_t* n_segments, int64_t* max_task_nnz);
/* Whole-workgroup rows of an ordered plan: all of them, those cut into column slices, and the
 * slices per cut row. Ordered plans need no workspace. */
gcg_status gcg_spmm_plan_hub_rows(const gcg_spmm_plan* plan, int64_t* n_coop_rows,
                                  int64_t* n_sliced_rows, int64_t* n_slices);

/* Planned SpMM: same contract as gcg_spmm_csr_f32; out_rows/n_out come from the plan. */
gcg_status gcg_spmm_csr_f32_planned(const gcg_spmm_plan* plan, const int32_t* indptr,
                                    const int32_t* indices, const float* vals,
                                    const float* Z, int64_t ldz, int64_t K, float* Y,
                                    int64_t ldy, const float* bias, int act, void* workspace,
                                    size_t workspace_bytes, gcg_stream_t stream);

/*
 * The same two SpMMs with the rectify gate written beside Y (act must be GCG_ACT_RELU):
 * gate[i][c] (uint8, row stride ldgate >= K, ldgate % 4 == 0, 4-B aligned base) = 2, 1 or 0
 * for a pre-activation > 0, == 0 or < 0 (NaN: 0) -- twice the factor of Theano's rectify
 * gradient 0.5 * (1 + sgn(x)) (relu = 0.5*(x+|x|), mlpconv.py:77). It replaces keeping the
 * output for the backward mask, and unlike the output it tells an exact-zero pre-activation
 * (gradient g/2) from a negative one (gradient 0). Consumed by gcg_relu_backward_gate_f32.
 */
gcg_status gcg_spmm_csr_f32_gate(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                 const int32_t* indptr, const int32_t* indices,
                                 const float* vals, const float* Z, int64_t ldz, int64_t K,
                                 float* Y, int64_t ldy, const float* bias, int act,
                                 const int32_t* out_rows, int64_t n_out, uint8_t* gate,
                                 int64_t ldgate, gcg_stream_t stream);
gcg_status gcg_spmm_csr_f32_planned_gate(const gcg_spmm_plan* plan, const int32_t* indptr,
                                         const int32_t* indices, const float* vals,
                                         const float* Z, int64_t ldz, int64_t K, float* Y,
                                         int64_t ldy, const float* bias, int act, uint8_t* gate,
                                         int64_t ldgate, void* workspace,
                                         size_t workspace_bytes, gcg_stream_t stream);

/*
 * Planned SpMM with a gather hint (round 3): gather_hint (device, nullable, nnz int32) is the
 * column index array with bit 31 set on every "cold" column -- a column whose Z row the caller
 * expects to be gathered rarely. Cold rows are gathered with non-temporal loads, so they do not
 * displace the hot rows (hub nodes of a power-law graph) from the L2 / Infinity Cache; the
 * result is bitwise the one without the hint (only the cache policy of the loads changes).
 * Used by the dwordx4 launches of up to 512 columns per panel (ldz % 4 == 0 and 16-B aligned
 * Z / Y / bias, any K); every other launch reads `indices`. graphconvgeo_amd.sparse builds the
 * hint (DeviceCSR.gather_hint).
 */
gcg_status gcg_spmm_csr_f32_planned_hint(const gcg_spmm_plan* plan, const int32_t* indptr,
                                         const int32_t* indices, const float* vals,
                                         const float* Z, int64_t ldz, int64_t K, float* Y,
                                         int64_t ldy, const float* bias, int act, uint8_t* gate,
                                         int64_t ldgate, void* workspace,
                                         size_t workspace_bytes, const int32_t* gather_hint,
                                         gcg_stream_t stream);

/*
 * Host-only planner (no device memory, no HIP calls): the task list the plan uses,
 * exposed for testing and for host-side tools. `tasks_host` receives n_tasks int32
 * quadruples {a, b, c, d}: c == -4 -> column slice b of d of the row at position a (ordered);
 * otherwise d < 0 -> rows of positions [a, b) (c == -2: one row on a whole workgroup);
 * d >= 0 -> segment of position a covering nonzeros [b, c) into workspace slot d. `long_host` receives
 * n_long quadruples {position, first_slot, n_slots, 0}. Pass NULL buffers to size.
 */
gcg_status gcg_spmm_plan_host(int64_t n_rows, const int32_t* indptr_host,
                              const int32_t* out_rows_host, int64_t n_out, int64_t task_nnz,
                              int ordered, int32_t* tasks_host, int64_t tasks_cap,
                              int64_t* n_tasks, int32_t* long_host, int64_t long_cap,
                              int64_t* n_long, int64_t* n_slots);

/*
 * Device CSR check: indptr[0] == 0, monotone, indptr[n_rows] == nnz, every
 * index in [0, n_cols). Writes 0 (ok) or a gcg_status code to *status_dev
 * (a device int32). Asynchronous on `stream`.
 */
gcg_status gcg_csr_validate(int64_t n_rows, int64_t n_cols, int64_t nnz,
                            const int32_t* indptr, const int32_t* indices,
                            int32_t* status_dev, gcg_stream_t stream);

/*
 * Scatter-add of rows (backward of Y[target_indices] at mlpconv.py:94, where
 * target indices repeat because train indices are drawn with replacement,
 * tensormain.py:226):  for i in [0, n_idx): out[idx[i], 0:K] += src[i, 0:K].
 * Deterministic: duplicates are added in increasing i, via the CSR of idx built
 * by gcg_index_csr (sorted_pos/seg_ptr). `out` is NOT zeroed first.
 */
gcg_status gcg_index_csr(int64_t n_idx, const int32_t* idx, int64_t n_rows, int32_t* seg_ptr,
                         int32_t* sorted_pos, void* workspace, size_t workspace_bytes,
                         size_t* workspace_needed, gcg_stream_t stream);
gcg_status gcg_scatter_add_rows_f32(int64_t n_rows, const int32_t* seg_ptr,
                                    const int32_t* sorted_pos, const float* src, int64_t lds,
                                    int64_t K, float* out, int64_t ldo, gcg_stream_t stream);

/*
 * Rectify backward with the bias gradient in one pass (Theano's grad of
 * rectify(S.dot(H, Z) + b), mlpconv.py:75-77): g = gY where Y > 0 else 0 (g_out may alias gY),
 * bias_grad[c] = sum_r g[r][c] (nullable; deterministic: per-block partials in the workspace,
 * summed in block order). K <= 1024. The workspace (size from _workspace_bytes) is required.
 */
gcg_status gcg_relu_backward_f32_workspace_bytes(int64_t M, int64_t K, size_t* bytes);
gcg_status gcg_relu_backward_f32(int64_t M, int64_t K, const float* gY, int64_t ldg,
                                 const float* Y, int64_t ldy, float* g_out, int64_t ldo,
                                 float* bias_grad /*nullable*/, void* workspace,
                                 size_t workspace_bytes, gcg_stream_t stream);

/*
 * Theano's rectify backward from the gate bytes of gcg_spmm_*_gate, with the bias gradient:
 * g = gY, gY/2 or 0 for gate 2, 1, 0 (the gradient of 0.5*(x+|x|) at x > 0, x == 0, x < 0),
 * bias_grad as gcg_relu_backward_f32 (same workspace size). K <= 1024.
 */
gcg_status gcg_relu_backward_gate_f32(int64_t M, int64_t K, const float* gY, int64_t ldg,
                                      const uint8_t* gate, int64_t ldgate, float* g_out,
                                      int64_t ldo, float* bias_grad /*nullable*/,
                                      void* workspace, size_t workspace_bytes,
                                      gcg_stream_t stream);

/*
 * Column sums out[c] = sum_r X[r][c] (the bias gradient of a dense projection, colsum of the
 * logits gradient; Theano's grad of T.dot(h, W) + b, mlpconv.py:88-93), deterministic, same
 * kernels and workspace (gcg_relu_backward_f32_workspace_bytes) as gcg_relu_backward_f32.
 */
gcg_status gcg_column_sum_f32(int64_t M, int64_t K, const float* X, int64_t ldx, float* out,
                              void* workspace, size_t workspace_bytes, gcg_stream_t stream);

/*
 * lasagne.updates.adam (mlpconv.py:263) for one float32 parameter of n elements, in place:
 *   m = b1*m + (1-b1)*g;  v = b2*v + (1-b2)*g*g;  p -= a_t*m / (sqrt(v) + eps),
 * with a_t = lr*sqrt(1-b2^t)/(1-b1^t) read from the device scalar *step_dev (so the call can
 * sit inside a captured HIP graph and be replayed with a new step size).
 */
gcg_status gcg_adam_step_f32(int64_t n, float* p, const float* g, float* m, float* v,
                             const float* step_dev, float beta1, float beta2, float eps,
                             gcg_stream_t stream);

/*
 * The weight penalty of the MLPCONV loss (mlpconv.py:235-243: lasagne.regularization l1 =
 * sum|W|, l2 = sum W^2, scaled by regul_coef * share) for one float32 weight of n elements:
 *   *out = ((acc_in ? *acc_in : 0) + l1 * sum|W|) + l2 * sum W^2
 * acc_in (nullable, may alias out) chains the weights of one loss in order. Deterministic
 * (fixed grid, partials added in order); workspace >= GCG_L1L2_WORKSPACE_BYTES device bytes.
 * gcg_l1l2_grad_f32 writes its gradient dW = s * (l1 * sgn(W) + 2 * l2 * W), sgn(0) = 0 (Theano's
 * grad of abs), s = *scale_dev (the upstream gradient, a device scalar) or 1 when NULL.
 */
#define GCG_L1L2_WORKSPACE_BYTES 2048
gcg_status gcg_l1l2_penalty_f32(int64_t n, const float* W, float l1, float l2,
                                const float* acc_in, float* out, void* workspace,
                                size_t workspace_bytes, gcg_stream_t stream);
gcg_status gcg_l1l2_grad_f32(int64_t n, const float* W, float l1, float l2,
                             const float* scale_dev, float* dW, gcg_stream_t stream);

/*
 * CSR transpose on the device (CSR(X^T) for the X^T . dZ1 gradient of
 * mlpconv.py:71). Output is sorted by (row, col) with stable order for equal
 * entries. out_indptr int32[n_cols+1], out_indices int32[nnz], out_vals f32[nnz].
 */
gcg_status gcg_csr_transpose_f32(int64_t n_rows, int64_t n_cols, int64_t nnz,
                                 const int32_t* indptr, const int32_t* indices,
                                 const float* vals, int32_t* out_indptr, int32_t* out_indices,
                                 float* out_vals, void* workspace, size_t workspace_bytes,
                                 size_t* workspace_needed, gcg_stream_t stream);

/*
 * Graph operator on the device (tensormain.py:170-180): from an undirected edge list
 * (u[e], v[e]) build H = D^-1/2 (A + I) D^-1/2 as a canonical CSR (rows and columns
 * sorted; duplicate edges collapse to one binary entry, as networkx stores one edge per
 * pair). H_ij = float32(float64(d_i^-1/2) * float64(d_j^-1/2)) with d = row degree incl.
 * the self loop: bitwise the reference's float64 D*adj*D product after .astype(float32)
 * (tensormain.py:221). Capacity: indices/vals hold 2*n_edges + n entries; the actual nnz
 * is written to *nnz_dev (device int64). *status_dev = GCG_ERR_BAD_CSR on an endpoint out
 * of [0, n). Pass all-NULL outputs to size the workspace.
 */
gcg_status gcg_normalize_adjacency_f32(int64_t n, int64_t n_edges, const int32_t* u,
                                       const int32_t* v, int self_loops, int32_t* indptr,
                                       int32_t* indices, float* vals, int64_t* nnz_dev,
                                       void* workspace, size_t workspace_bytes,
                                       size_t* workspace_needed, int32_t* status_dev,
                                       gcg_stream_t stream);

/*
 * SpGEMM C = A . B for the host "input convolution" X_conv = H * X (main.py:530,
 * tensormain.py:114; then .tocsr().astype('float32')). A: m x n CSR (values float32, or
 * float64 when a_is_f64 -- the reference's H is float64 there), B: n x p CSR float32.
 * Every C entry is summed in scipy csr_matmat's traversal order (A row order, then B row
 * order), each product and sum rounded in the accumulation type (accumulate_f64 = 1:
 * float64, the reference's H64 * X32 upcast), exact zero sums dropped (as scipy), then
 * rounded to float32. Output CSR is canonical (sorted columns), as astype() leaves it.
 * Step 1: gcg_spgemm_products -> number of products P (synchronizes). Step 2: gcg_spgemm
 * with c_idx/c_val of capacity P, c_ptr of m+1; actual nnz to *nnz_c_dev (<= INT32_MAX).
 * Not a hot-path call: it allocates stream-ordered temporaries and synchronizes. The
 * row-wise path (p within 8 LDS slabs) uses c_idx/c_val themselves as its products-sized
 * scratch (C rows written at their product offsets, then compacted in place), so it only
 * allocates ~30 B per row of A; the expand-sort-reduce path used for wider p allocates ~40 B
 * per product per 2^29-product row chunk. Entries of c_idx/c_val past nnz(C) are undefined.
 */
gcg_status gcg_spgemm_products(int64_t m, int64_t nnz_a, const int32_t* a_ptr, const int32_t* a_idx,
                               int64_t n, const int32_t* b_ptr, int64_t* n_products,
                               gcg_stream_t stream);
gcg_status gcg_spgemm(int64_t m, int64_t n, int64_t p, int64_t nnz_a, const int32_t* a_ptr,
                      const int32_t* a_idx, const void* a_val, int a_is_f64, int64_t nnz_b,
                      const int32_t* b_ptr, const int32_t* b_idx, const float* b_val,
                      int accumulate_f64, int64_t n_products, int32_t* c_ptr, int32_t* c_idx,
                      float* c_val, int64_t* nnz_c_dev, gcg_stream_t stream);
/* gcg_spgemm with the path forced (tests, measurement; every path gives the same C, bitwise):
 * flags GCG_SPGEMM_EXPAND_SORT = the expand-sort-reduce path at any p, GCG_SPGEMM_DENSE_SLABS =
 * every row on the dense LDS slabs (no short-row radix-sort kernel), GCG_SPGEMM_COMPACT_TEMPORARY
 * = compact C through an nnz(C)-sized temporary instead of in place; chunk_products > 0 caps the
 * products per expand-sort-reduce row chunk (0 = 2^29). gcg_spgemm = flags 0, chunk 0. */
enum { GCG_SPGEMM_EXPAND_SORT = 1, GCG_SPGEMM_DENSE_SLABS = 2, GCG_SPGEMM_COMPACT_TEMPORARY = 4 };
gcg_status gcg_spgemm_ex(int64_t m, int64_t n, int64_t p, int64_t nnz_a, const int32_t* a_ptr,
                         const int32_t* a_idx, const void* a_val, int a_is_f64, int64_t nnz_b,
                         const int32_t* b_ptr, const int32_t* b_idx, const float* b_val,
                         int accumulate_f64, int64_t n_products, int32_t* c_ptr, int32_t* c_idx,
                         float* c_val, int64_t* nnz_c_dev, int32_t flags, int64_t chunk_products,
                         gcg_stream_t stream);

/*
 * Mention-graph projection on the device (DataLoader.get_graph's celebrity filter,
 * data.py:364-370, then efficient_collaboration_weighted_projected_graph2, data.py:226-250).
 * Input: the bipartite user/mention graph as incidences (a[e], b[e]) over n_nodes ids, ids <
 * n_targets are users (their self loops are implicit, as get_graph adds them), ids >= n_targets
 * mention-only names. A mention node survives iff 1 < degree <= celebrity_threshold. Output:
 * every pair of users that share a surviving neighbour (a user node's own self loop makes it a
 * neighbour of itself), deduplicated, u < v, sorted, into caller-owned device arrays out_u /
 * out_v of `capacity` entries; *n_edges = the edge count. Pass out_u = out_v = NULL to size:
 * *n_edges then receives the number of pairs before deduplication, an upper bound. Allocates
 * stream-ordered temporaries and synchronizes `stream`; not a hot-path call.
 */
gcg_status gcg_project_mention_graph(int64_t n_targets, int64_t n_nodes, int64_t n_inc,
                                     const int32_t* a, const int32_t* b, int celebrity_threshold,
                                     int32_t* out_u, int32_t* out_v, int64_t capacity,
                                     int64_t* n_edges, int32_t* status_dev, gcg_stream_t stream);

/*
 * Dense side of the output layer on the matrix cores. Row-major operands; A: M x K (lda),
 * B: K x N (ldb), C: M x N (ldc). A and B need 16-B aligned bases and ld % 4 == 0; B is read at
 * columns < round4(N), so ldb >= round4(N) (pad the weight, as graphconvgeo_amd.dense does).
 *
 * Arithmetic and tile are explicit per call (round 5) -- no environment variable changes what a
 * dense entry computes:
 *   math  GCG_MATH_F32     v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulation; the k
 *                          order inside a 16-deep step is permuted (step s takes k = k0 + 4q + s),
 *                          so results equal a BLAS sgemm within f32 rounding, not bit for bit.
 *         GCG_MATH_BF16X6  f32 on the bf16 matrix cores: every f32 operand split into three bf16
 *                          planes x = x0 + x1 + x2 (round to nearest, 8 significant bits each), the
 *                          six plane products of order <= 2^-16 accumulated in f32
 *                          (v_mfma_f32_16x16x32_bf16), each exact. The planes hold x exactly
 *                          (3 x 8 significant bits), |x1| <= 2^-8 |x|, |x2| <= 2^-17 |x|, so the
 *                          dropped a1b2 + a2b1 + a2b2 are <= (2^-24 + 2^-34) |a||b| per product --
 *                          one f32 rounding of the product (tests/test_bf16x6_numerics.py pins
 *                          these bounds; tests/test_dense_gpu.py the whole product's error against
 *                          float64, <= 1.25 x the f32 kernel's). A last k chunk with <= 16 live
 *                          k carries two plane products per MFMA (the fragments' zero high halves
 *                          hold another plane of the low halves' k): 3 MFMAs instead of 6 there,
 *                          every product still exact, the same in every bf16x6 form.
 *                          f32 semantics at the edges: a tile whose bf16x6 result is not finite
 *                          (an infinite operand, |x| above bf16's largest finite 3.39e38, NaN, or
 *                          overflow) is recomputed on the f32 MFMA in the f32 kernel's k order, so
 *                          +-Inf propagates and Inf * 0 gives NaN exactly as with GCG_MATH_F32.
 *   tile  0 = the default tile, a pure function of (M, N, K); 1..gcg_dense_tile_count(op, math)
 *         = a measured alternative (tests, measurement); the same products except where noted.
 */
enum { GCG_MATH_F32 = 0, GCG_MATH_BF16X6 = 1 };
enum { GCG_DENSE_GEMM = 0, GCG_DENSE_GEMM_NT = 1, GCG_DENSE_FUSED = 2, GCG_DENSE_GEMM_TN = 3 };
/* Alternative tiles of product op (GCG_DENSE_*) in arithmetic math: tile indices 1..n are valid;
 * -1 when that arithmetic is not available for the product. */
int32_t gcg_dense_tile_count(int32_t op, int32_t math);

/*
 * gcg_gemm: C = act(A . B + bias)        T.dot(h, W) (+ b) at mlpconv.py:88 / the propagate-first
 *   form of mlpconv.py:88-93, and Theano's g . W^T (W^T passed as B). GCG_MATH_F32 only; tile 0
 *   stages B through LDS (gemm_bl_kernel), tile 1 reads it straight into registers (gemm_kernel):
 *   the same k order, bitwise equal.
 * gcg_gemm_f32 = gcg_gemm(..., GCG_MATH_F32, 0, ...).
 */
gcg_status gcg_gemm(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* B,
                    int64_t ldb, const float* bias /*nullable*/, int act, float* C, int64_t ldc,
                    int32_t math, int32_t tile, gcg_stream_t stream);
gcg_status gcg_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                        const float* B, int64_t ldb, const float* bias /*nullable*/, int act,
                        float* C, int64_t ldc, gcg_stream_t stream);

/*
 * gcg_gemm_nt: C = act(A . Bt^T + bias) with the second operand stored transposed (Bt: N x K
 * row-major, ldbt >= round4(K), ldbt % 4 == 0, 16-B aligned base; A likewise with lda). The
 * projection T.dot(h, W) (mlpconv.py:88) with Bt = W^T, and Theano's input gradient g . W^T with
 * Bt = W itself. In the k step that reaches past K the fragment elements at k >= K are zeroed in
 * registers, so operand padding may hold anything (NaN included).
 *   GCG_MATH_F32: both operands through the asynchronous LDS-DMA (global_load_lds) into a ring of
 *     k chunks (tile 0: 16-deep chunks, 4 stages); every tile the same k order.
 *   GCG_MATH_BF16X6: ws != NULL (gcg_gemm_nt_workspace(N, K, math) bytes, 16-B aligned): Bt's
 *     three planes split once per call into it by a small kernel on the same stream, A split in
 *     registers (tile 0: A in registers, 128 x 64 G columns with G padding N least, or -- where
 *     that pads less -- 128 x 192 tiles over N's whole 192-column blocks and the narrowest tile
 *     over the rest, as two launches on the stream); ws == NULL: both operands split in the loop
 *     (tile 0 only). Every bf16x6 form accumulates the same six plane products in the same order:
 *     bitwise equal to each other.
 * gcg_gemm_nt_f32 = gcg_gemm_nt(..., GCG_MATH_F32, 0, NULL, 0, ...);
 * gcg_gemm_nt_f32_bf16x6 = gcg_gemm_nt(..., GCG_MATH_BF16X6, 0, ws, ws_bytes, ...).
 */
gcg_status gcg_gemm_nt(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                       const float* Bt, int64_t ldbt, const float* bias /*nullable*/, int act,
                       float* C, int64_t ldc, int32_t math, int32_t tile, void* ws /*nullable*/,
                       int64_t ws_bytes, gcg_stream_t stream);
int64_t gcg_gemm_nt_workspace(int64_t N, int64_t K, int32_t math);
gcg_status gcg_gemm_nt_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                           const float* Bt, int64_t ldbt, const float* bias /*nullable*/,
                           int act, float* C, int64_t ldc, gcg_stream_t stream);
gcg_status gcg_gemm_nt_f32_bf16x6(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                  const float* Bt, int64_t ldbt, const float* bias /*nullable*/,
                                  int act, float* C, int64_t ldc, void* ws /*nullable*/,
                                  int64_t ws_bytes, gcg_stream_t stream);
/* = gcg_gemm_nt_workspace(N, K, GCG_MATH_BF16X6) */
int64_t gcg_gemm_nt_bf16x6_workspace(int64_t N, int64_t K);

/*
 * Fused output layer + loss (N <= 1024; one workgroup owns whole rows):
 *   logits = A . W + bias                                       mlpconv.py:88-93
 *   labels != NULL: out = (softmax(logits) - onehot(labels)) * scale * row_weight[i]  (the logits
 *     gradient of categorical_crossentropy(...).mean() with scale = 1/M, mlpconv.py:229-230),
 *     loss_rows[i] = -log softmax(logits)[i, labels[i]] * row_weight[i],
 *     correct_rows[i] (nullable) = row_weight[i] if the first-index argmax equals labels[i] else 0
 *     (argmax + T.eq accuracy, mlpconv.py:227,252);
 *   labels == NULL: out = softmax(logits) (predict_proba, mlpconv.py:329-335);
 *   out may be NULL when labels are given (evaluation: loss and accuracy only).
 * row_weight (device, nullable = all 1, then bitwise the unweighted result): with the distinct
 * targets as rows and their multiplicities as weights, one call computes the loss and gradient of
 * a target list drawn with replacement (tensormain.py:226) over its distinct rows only.
 * scale_dev (nullable, device): multiplies scale (the upstream gradient of the loss, read on the
 * device so the call can sit inside a captured HIP graph). The logits never reach HBM. out needs
 * ldo % 4 == 0 and a 16-B aligned base; its padding columns [N, round4(N)) are written with zeros
 * (whole dwordx4 row stores). W's padding columns [N, ldw) may hold anything (NaN included): they
 * never reach a logit. A label outside [0, N) gives that row a NaN loss, no hit, no onehot.
 *   GCG_MATH_F32 (gemm_kernel): 32 rows x 4 waves; tiles 1..5 split the weight's register set
 *     into 0 / 2 / 4 / 8 / 16 rotating parts (tile 0: 8 at N > 768, else 4) -- bitwise equal.
 *   GCG_MATH_BF16X6 (gemm_fused6_kernel): ws != NULL (gcg_project_softmax_xent_workspace(N, K,
 *     math) bytes, 16-B aligned): the weight's three bf16 planes split once per call into it;
 *     tile 0 = tile 3 = 64 rows x 8 waves at N > 768 (row sums over 8 column waves), else 32
 *     rows x 4 waves, the A chunk split once per workgroup into LDS planes; tile 1 = 32 rows x 4
 *     waves at any N (bitwise the ws == NULL form); tile 2 = the 64-row form (N > 768 only);
 *     tiles 1 / 2 split A in every wave's registers, bitwise equal to tile 3 of their shape.
 *     ws == NULL: the weight split in every workgroup's registers,
 *     32 rows x 4 waves (tile 0 only). The 64-row form is within f32 rounding of the 32-row one
 *     (another association of the row sums), with the same hits.
 * Legacy entries: gcg_project_softmax_xent_f32 and _weighted_f32 = GCG_MATH_F32, tile 0;
 * _weighted_ws_f32 = GCG_MATH_BF16X6, tile 0 (with ws, or the in-register split when NULL).
 */
gcg_status gcg_project_softmax_xent(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                                    const float* W, int64_t ldw, const float* bias /*nullable*/,
                                    const int32_t* labels /*nullable*/, float scale,
                                    const float* scale_dev /*nullable*/, float* out /*nullable*/,
                                    int64_t ldo, float* loss_rows,
                                    float* correct_rows /*nullable*/,
                                    const float* row_weight /*nullable*/, int32_t math,
                                    int32_t tile, void* ws /*nullable*/, int64_t ws_bytes,
                                    gcg_stream_t stream);
int64_t gcg_project_softmax_xent_workspace(int64_t N, int64_t K, int32_t math);
gcg_status gcg_project_softmax_xent_f32(int64_t M, int64_t N, int64_t K, const float* A,
                                        int64_t lda, const float* W, int64_t ldw,
                                        const float* bias /*nullable*/,
                                        const int32_t* labels /*nullable*/, float scale,
                                        const float* scale_dev /*nullable*/,
                                        float* out /*nullable*/, int64_t ldo, float* loss_rows,
                                        float* correct_rows /*nullable*/, gcg_stream_t stream);
/* = gcg_project_softmax_xent_workspace(N, K, GCG_MATH_BF16X6) */
int64_t gcg_project_softmax_xent_bf16x6_workspace(int64_t N, int64_t K);
gcg_status gcg_project_softmax_xent_weighted_ws_f32(
    int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, const float* W, int64_t ldw,
    const float* bias /*nullable*/, const int32_t* labels /*nullable*/, float scale,
    const float* scale_dev /*nullable*/, float* out /*nullable*/, int64_t ldo, float* loss_rows,
    float* correct_rows /*nullable*/, const float* row_weight /*nullable*/, void* ws /*nullable*/,
    int64_t ws_bytes, gcg_stream_t stream);

/*
 * The same row epilogue for logits that already exist (the reference order, where the
 * logits are the H SpMM's output rows, mlpconv.py:90-94): one wave per row, N <= 4096,
 * out may alias logits; out == NULL computes loss_rows / correct_rows only (the forward
 * half; the gradient pass then runs with out set and scale_dev = the upstream gradient).
 */
gcg_status gcg_softmax_xent_f32(int64_t M, int64_t N, const float* logits, int64_t ldl,
                                const int32_t* labels /*nullable*/, float scale,
                                const float* scale_dev /*nullable*/, float* out /*nullable*/,
                                int64_t ldo, float* loss_rows, float* correct_rows /*nullable*/,
                                gcg_stream_t stream);

/*
 * Weighted forms of the two above: row i's loss, hit and gradient row are multiplied by
 * row_weight[i] (device, nullable = all 1 -- then bitwise the unweighted calls). With the
 * distinct targets as rows and their multiplicities as weights, one call computes the loss
 * and gradient of a target list drawn with replacement (tensormain.py:226) over its distinct
 * rows only: sum_i w_i loss_i = the sum over the full list, and the gradient of a distinct row
 * is the sum of its duplicates' gradients (Theano's inc_subtensor adds them, mlpconv.py:94).
 */
gcg_status gcg_project_softmax_xent_weighted_f32(int64_t M, int64_t N, int64_t K,
                                                 const float* A, int64_t lda, const float* W,
                                                 int64_t ldw, const float* bias /*nullable*/,
                                                 const int32_t* labels /*nullable*/, float scale,
                                                 const float* scale_dev /*nullable*/,
                                                 float* out /*nullable*/, int64_t ldo,
                                                 float* loss_rows,
                                                 float* correct_rows /*nullable*/,
                                                 const float* row_weight /*nullable*/,
                                                 gcg_stream_t stream);
gcg_status gcg_softmax_xent_weighted_f32(int64_t M, int64_t N, const float* logits, int64_t ldl,
                                         const int32_t* labels /*nullable*/, float scale,
                                         const float* scale_dev /*nullable*/,
                                         float* out /*nullable*/, int64_t ldo, float* loss_rows,
                                         float* correct_rows /*nullable*/,
                                         const float* row_weight /*nullable*/,
                                         gcg_stream_t stream);

/*
 * Weight gradient C = scale * A^T . B (Theano's grad of T.dot(h, W) w.r.t. W: h^T . gz,
 * mlpconv.py:88; P^T . G in the propagate-first order), A: R x M, B: R x N, C: M x N, the
 * reduction over R (~10^6 rows) split across waves; the per-split partials (caller-owned
 * workspace, size from gcg_gemm_tn_workspace_bytes for the same math and tile) are summed in
 * split order, so the result is deterministic (equal to a BLAS sgemm within f32 rounding). A and
 * B: 16-B aligned, lda >= round4(M), ldb >= round4(N), ld % 4 == 0. scale_dev: nullable device
 * scalar.
 *   GCG_MATH_F32 (f32 MFMA): tile 0 = per-wave 64 x 64 NG tiles (NG padding N least) or, for
 *     M <= 256 in 64-row bands with N <= 512, waves stacked along M; tiles 1..7 = other wave
 *     layouts and split counts (another summation order: within f32 rounding).
 *   GCG_MATH_BF16X6 (tile 0 only): per-wave 64 x 64 tiles on the bf16 matrix cores, each
 *     32-row chunk's six plane products summed apart and added to the split's running sum once
 *     (error against float64 at or below the f32 form's); non-finite tiles recomputed in f32.
 * gcg_gemm_tn_f32[_workspace_bytes] = the GCG_MATH_F32, tile 0 forms.
 */
gcg_status gcg_gemm_tn_workspace_bytes(int64_t R, int64_t M, int64_t N, int32_t math,
                                       int32_t tile, size_t* bytes);
gcg_status gcg_gemm_tn(int64_t R, int64_t M, int64_t N, const float* A, int64_t lda,
                       const float* B, int64_t ldb, const float* scale_dev /*nullable*/, float* C,
                       int64_t ldc, int32_t math, int32_t tile, void* workspace,
                       size_t workspace_bytes, gcg_stream_t stream);
gcg_status gcg_gemm_tn_f32_workspace_bytes(int64_t R, int64_t M, int64_t N, size_t* bytes);
gcg_status gcg_gemm_tn_f32(int64_t R, int64_t M, int64_t N, const float* A, int64_t lda,
                           const float* B, int64_t ldb, const float* scale_dev /*nullable*/,
                           float* C, int64_t ldc, void* workspace, size_t workspace_bytes,
                           gcg_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* GCG_SPMM_H */
