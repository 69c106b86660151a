/*
 * recsys_hip.h — C-ABI of the MI355X (gfx950) hot-path library `librecsys_hip.so`.
 *
 * Scope: the two-tower retrieval + DCN ranking forward/backward path of
 * OnlyAhad13/Recommendation-System-MAANG-NVIDIA- (`src/models.py` MultiTowerModel /
 * DeepCrossNetwork / MultiTaskModel driven by `src/trainer.py` ProductionTrainer).
 * The reference has no native code of its own: every entry point below replaces a
 * TensorFlow / Keras / TFRS kernel invoked from a reference call site, cited per function.
 *
 * Conventions (all entry points):
 *   - plain pointers + int64 sizes, no framework types; every pointer is a DEVICE pointer
 *     unless stated otherwise; the caller owns every buffer (workspaces are sized by the
 *     matching *_workspace_bytes query) and the library never allocates on the hot path;
 *   - all work is enqueued on `stream` (a hipStream_t; NULL = default stream); no entry point
 *     synchronises, so every one is hipGraph-capturable;
 *   - return RS_OK (0) or a negative status; rs_last_error() describes the last failure of the
 *     calling thread; no C++ exception crosses the ABI;
 *   - fp32 row-major storage; Keras layouts (Dense kernel [in, out], Embedding [V+1, D],
 *     row 0 = OOV) so reference weights load without transposes.
 */
#ifndef RECSYS_HIP_H
#define RECSYS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* rs_stream_t; /* hipStream_t */

enum {
  RS_OK = 0,
  RS_ERR_INVALID_ARG = -1, /* shape / alignment / null-pointer violation */
  RS_ERR_UNSUPPORTED = -2, /* valid but not implemented (e.g. D not in the compiled set) */
  RS_ERR_HIP = -3,         /* a HIP runtime call or launch failed */
  RS_ERR_WORKSPACE = -4    /* workspace smaller than the *_workspace_bytes query */
};

/* ABI revision; bumped whenever a signature below changes. */
int rs_abi_version(void);
/* Text of the last failure on the calling thread ("" if none). Host pointer, static storage. */
const char* rs_last_error(void);

/* ---------------------------------------------------------------------------------------
 * a2 / K2 — embedding row gather.
 * Replaces keras.layers.Embedding.__call__ (src/models.py:71,74; called at :85,:89).
 * out[b, :] = table[ids[b], :]. ids outside [0, num_rows) produce a zero row and add one to
 * *bad_ids (nullable), mirroring Keras' InvalidArgumentError without a host sync.
 * ------------------------------------------------------------------------------------- */
int rs_embedding_gather_f32(const float* table, int64_t num_rows, int64_t dim,
                            const int64_t* ids, int64_t n, float* out, int32_t* bad_ids,
                            rs_stream_t stream);

/* Same update with the clip norm supplied by the caller: *sumsq (device) = ||G||_F^2 over the
 * un-deduplicated rows of every replica (the data-parallel exchange all-reduces the replicas'
 * local sums and hands over locally deduplicated rows: clip_by_norm is linear, so scaling the
 * partial sums equals scaling the raw rows up to rounding). sumsq may be NULL when clipnorm <= 0. */
int rs_sparse_adagrad_sumsq_f32(float* table, float* accum, int64_t num_rows, int64_t dim,
                                const int64_t* ids, const float* grad_rows, int64_t grad_ld, int64_t n,
                                const float* sumsq, const int64_t* iteration, float lr0, float decay_rate,
                                int64_t decay_steps, float clipnorm, float epsilon, void* workspace,
                                size_t workspace_bytes, rs_stream_t stream);
/* The sparse update of up to 32 tables in one launch sequence (one sort of all tables' keys, one
 * clip-norm pass, one fragment pass, one apply pass: ~9 launches instead of ~9 per table). Table k:
 * tables[k] / accums[k] [num_rows[k]][dim], ids[k] [n[k]], grad_rows[k] [n[k]] rows of stride
 * grad_ld[k]; sumsq == NULL: each table clipped by the norm of its own raw rows (as
 * rs_sparse_adagrad_ld_f32), else sumsq[k] = that norm^2 (as rs_sparse_adagrad_sumsq_f32). Each
 * table's result is bitwise that of its single-table update when all n[k] are equal (the same
 * windows and ordered sums), and the same sums up to association otherwise. Replaces the per-table
 * apply_gradients loop of the reference's optimizer over its embedding variables
 * (src/trainer.py:157-163, Keras Adagrad over the models' tables, src/models.py:73,83,112). */
size_t rs_sparse_adagrad_multi_workspace_bytes(int ntables, const int64_t* n, int64_t dim);
int rs_sparse_adagrad_multi_f32(int ntables, float* const* tables, float* const* accums, const int64_t* num_rows,
                                int64_t dim, const int64_t* const* ids, const float* const* grad_rows,
                                const int64_t* grad_ld, const int64_t* n, const float* const* sumsq,
                                const int64_t* iteration, float lr0, float decay_rate, int64_t decay_steps,
                                float clipnorm, float epsilon, void* workspace, size_t workspace_bytes,
                                rs_stream_t stream);
/* rs_sparse_adagrad_multi_f32, then *iteration += 1 once every table is updated (the apply pass's
 * last workgroup does it after every workgroup has read the step: the optimizer's
 * rs_iteration_increment launch folded into the sparse update). */
int rs_sparse_adagrad_multi_step_f32(int ntables, float* const* tables, float* const* accums, const int64_t* num_rows,
                                     int64_t dim, const int64_t* const* ids, const float* const* grad_rows,
                                     const int64_t* grad_ld, const int64_t* n, const float* const* sumsq,
                                     int64_t* iteration, float lr0, float decay_rate, int64_t decay_steps,
                                     float clipnorm, float epsilon, void* workspace, size_t workspace_bytes,
                                     rs_stream_t stream);
/* rs_sparse_adagrad_multi_step_f32 with each table's ids already in sorted order: orders[k] lists
 * table k's positions 0..n[k]-1 by ascending id, equal ids by ascending position, ids outside
 * [0, num_rows[k]) last (a stable sort's result; the in-batch id plan's order entry,
 * rs_inbatch_unique_ids_pair_order_i64, is exactly that for the user and item tables). The
 * update's own sort is skipped; the result is bitwise the unordered entry's. */
int rs_sparse_adagrad_multi_step_ordered_f32(int ntables, float* const* tables, float* const* accums,
                                             const int64_t* num_rows, int64_t dim, const int64_t* const* ids,
                                             const float* const* grad_rows, const int64_t* grad_ld, const int64_t* n,
                                             const float* const* sumsq, int64_t* iteration, float lr0,
                                             float decay_rate, int64_t decay_steps, float clipnorm, float epsilon,
                                             const int32_t* const* orders, void* workspace, size_t workspace_bytes,
                                             rs_stream_t stream);
/* rs_sparse_adagrad_multi_step_ordered_f32 with the plan's run heads as well (HOST arrays of device
 * pointers, one per table): starts[k][p] = the first position of table k's p-th distinct id in
 * orders[k], dids[k][p] = that id (>= num_rows[k]: the out-of-range group, not applied),
 * *nslots[k] = the distinct count (device) — rs_inbatch_unique_ids_plan_i64's u_start / u_did /
 * info[0] for the user table, c_* / info[2] for the item table. The apply pass then runs one lane
 * slice per distinct id (dim 32, 64, 128 or 256; tables 16-byte aligned); bitwise the ordered
 * entry's result. */
int rs_sparse_adagrad_multi_step_planned_f32(int ntables, float* const* tables, float* const* accums,
                                             const int64_t* num_rows, int64_t dim, const int64_t* const* ids,
                                             const float* const* grad_rows, const int64_t* grad_ld, const int64_t* n,
                                             const float* const* sumsq, int64_t* iteration, float lr0,
                                             float decay_rate, int64_t decay_steps, float clipnorm, float epsilon,
                                             const int32_t* const* orders, const int32_t* const* starts,
                                             const int64_t* const* dids, const int64_t* const* nslots,
                                             void* workspace, size_t workspace_bytes, rs_stream_t stream);
/* Local deduplication of an IndexedSlices gradient (the data-parallel exchange sends each replica's
 * unique rows only): out_ids[0..*out_count) = the distinct valid ids ascending, out_rows = the sum
 * of each id's rows in input order (the same ordered sums as the update), ids outside
 * [0, num_rows) dropped; *sumsq (nullable) = sum of squares of the n raw rows. out_ids / out_rows
 * must hold n entries; *out_count is written on the device (no host sync). */
size_t rs_sparse_dedupe_workspace_bytes(int64_t n, int64_t dim, int64_t num_rows);
int rs_sparse_dedupe_f32(const int64_t* ids, const float* grad_rows, int64_t grad_ld, int64_t n, int64_t num_rows,
                         int64_t dim, int64_t* out_ids, float* out_rows, int64_t* out_count, float* sumsq,
                         void* workspace, size_t workspace_bytes, rs_stream_t stream);

/* rs_sparse_dedupe_f32 over an id plan of the same ids (rs_inbatch_unique_ids_plan_i64: order =
 * the ids' stable ascending order, starts / dids / *nslots = its run heads, distinct ids and distinct
 * count; the data-parallel step's local slices are exactly the plan's ids): no sort, flag or scan
 * pass; bitwise rs_sparse_dedupe_f32's outputs. dim 32, 64, 128 or 256; 16-byte rows. */
int rs_sparse_dedupe_planned_f32(const int64_t* ids, const float* grad_rows, int64_t grad_ld, int64_t n,
                                 int64_t num_rows, int64_t dim, const int32_t* order, const int32_t* starts,
                                 const int64_t* dids, const int64_t* nslots, int64_t* out_ids, float* out_rows,
                                 int64_t* out_count, float* sumsq, void* workspace, size_t workspace_bytes,
                                 rs_stream_t stream);
/* The stable ascending order (int32 [n]) of nruns runs of ids concatenated, each run sorted
 * ascending without repeats (the deduplicating exchange's all-gathered ids: each rank's
 * rs_sparse_dedupe output, in rank order): run_off [nruns + 1] (HOST) = the runs' offsets. Equal ids
 * keep run order, so this is the permutation a stable sort gives — what
 * rs_sparse_adagrad_multi_step_ordered_f32 takes in place of its own sort. nruns <= 64. */
int rs_merge_runs_order_i64(const int64_t* ids, const int64_t* run_off, int nruns, int32_t* order,
                            rs_stream_t stream);

/* The gathers of up to 8 tables of the same width in ONE launch (the user and item lookups of
 * a training step, src/models.py:85,89): out_j[b, :] = table_j[ids_j[b], :] for every j, same
 * out-of-range rule (one shared bad_ids counter). `tables`, `num_rows`, `ids`, `n` and `outs` are
 * HOST arrays of ntables entries; the pointers they hold are device pointers. */
int rs_embedding_gather_tables_f32(int ntables, const float* const* tables, const int64_t* num_rows,
                                   const int64_t* const* ids, const int64_t* n, float* const* outs,
                                   int64_t dim, int32_t* bad_ids, rs_stream_t stream);

/* The same gathers with each table's rows copied in a given order: position p of table j copies
 * batch row orders[j][p] (HOST array of nullable device int32 pointers; NULL = batch order). With
 * the rows in ascending-id order (rs_inbatch_unique_ids_pair_order_i64) the lanes of a wave read
 * nearby table rows, so a wave touches few translation pages; the result is the same. */
int rs_embedding_gather_tables_ordered_f32(int ntables, const float* const* tables, const int64_t* num_rows,
                                           const int64_t* const* ids, const int32_t* const* orders,
                                           const int64_t* n, float* const* outs, int64_t dim, int32_t* bad_ids,
                                           rs_stream_t stream);

/* The gathers over a batch's distinct ids (the towers' lookups run once per distinct id, src/models.py:
 * 85,89): position p of table j copies the row of id ids_j[reps[j][p]] into out_j[p] for p below the
 * DEVICE count *counts[j] (reps / counts: HOST arrays of device pointers, e.g. the id plan's rep and
 * distinct count of rs_inbatch_unique_ids_pair_i64); positions from the count to n[j] are not
 * written (a graph sized for n serves any count). dim 32, 64 or 128. */
int rs_embedding_gather_tables_rows_f32(int ntables, const float* const* tables, const int64_t* num_rows,
                                        const int64_t* const* ids, const int32_t* const* reps,
                                        const int64_t* const* counts, const int64_t* n, float* const* outs,
                                        int64_t dim, int32_t* bad_ids, rs_stream_t stream);

/* The distinct-id gathers straight from a plan's distinct ids (rs_inbatch_unique_ids_plan_i64's
 * u_did / c_did): out_j[p] = table_j[dids_j[p]] for p < n[j]; an id >= num_rows gives a zero row
 * (counted in bad_ids), a negative id (a slot past the distinct count) leaves out_j[p] unwritten.
 * One dependent load (the id) before the row stream instead of three (count, representative, id);
 * the rows are read in ascending-id order. dim 32, 64 or 128. */
int rs_embedding_gather_tables_ids_f32(int ntables, const float* const* tables, const int64_t* num_rows,
                                       const int64_t* const* dids, const int64_t* n, float* const* outs,
                                       int64_t dim, int32_t* bad_ids, rs_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * a2 bwd + a13 / K3 + K11 — sparse embedding update.
 * Replaces the IndexedSlices gradient of keras.layers.Embedding + Keras (>=2.11) optimizer
 * apply_gradients with Adagrad(ExponentialDecay(lr0, decay_steps, decay_rate, staircase),
 * clipnorm) (src/trainer.py:157-163):
 *   g_k  <- g_k * clipnorm / max(||G||_F, clipnorm)   (norm over the n un-deduplicated rows)
 *   gs_r  = sum_{k: ids[k]=r} g_k                       (duplicates summed in input order)
 *   acc_r += gs_r^2 ; table_r -= lr_t * gs_r / sqrt(acc_r + epsilon)
 *   lr_t  = lr0 * decay_rate^floor(*iteration / decay_steps)     (*iteration read on device)
 * Deterministic: sort + ordered segment sums, no float atomics. clipnorm <= 0 disables clipping.
 * dim <= 256; above 64 columns dim must be even (a multiple of 4 above 128) and the table /
 * accumulator 16-byte aligned (rows move as 2- / 4-float vectors per lane).
 * ------------------------------------------------------------------------------------- */
size_t rs_sparse_adagrad_workspace_bytes(int64_t n, int64_t dim, int64_t num_rows);
int rs_sparse_adagrad_f32(float* table, float* accum, int64_t num_rows, int64_t dim,
                          const int64_t* ids, const float* grad_rows, int64_t n,
                          const int64_t* iteration, float lr0, float decay_rate,
                          int64_t decay_steps, float clipnorm, float epsilon, void* workspace,
                          size_t workspace_bytes, rs_stream_t stream);
/* Same with a row stride for grad_rows (grad row k at grad_rows + k * grad_ld): the per-feature
 * column slices of dLoss/dx0 in the config-5 multi-feature model. */
int rs_sparse_adagrad_ld_f32(float* table, float* accum, int64_t num_rows, int64_t dim,
                             const int64_t* ids, const float* grad_rows, int64_t grad_ld, int64_t n,
                             const int64_t* iteration, float lr0, float decay_rate,
                             int64_t decay_steps, float clipnorm, float epsilon, void* workspace,
                             size_t workspace_bytes, rs_stream_t stream);

/* Config-5 (Criteo-shaped, extension) feature assembly: nfeat embedding tables (DEVICE arrays of
 * table pointers and row counts), ids [nfeat][B], dense features [B][nd]:
 *   x0[b] = [T_0[ids[0][b]] || ... || T_{nfeat-1}[ids[nfeat-1][b]] || dense[b] || 0 pad]  (ld cols).
 * Every table has at least one row (row 0, the OOV row); an invalid id gives a zero row and is counted. */
int rs_multi_embedding_gather_f32(const float* const* tables, const int64_t* num_rows, int nfeat,
                                  int64_t E, const int64_t* ids, int64_t B, const float* dense,
                                  int64_t nd, float* x0, int64_t ld, int32_t* bad_ids,
                                  rs_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * a3 / a8 / K4 / K7 — fp32 MFMA GEMM (v_mfma_f32_32x32x2_f32) with fused epilogue.
 * Replaces keras.layers.Dense (MatMul + BiasAdd + ReLU) in the towers (src/models.py:76-77)
 * and the DCN deep net (src/models.py:26-29,46-48), and the dX GEMM of their gradients.
 *   C = epilogue(op(A) @ op(B))    op(A): [M,K], op(B): [K,N]
 *   trans_a = 0: A is [M][lda] ; trans_a = 1: A is [K][lda]
 *   trans_b = 0: B is [K][ldb] ; trans_b = 1: B is [N][ldb]
 *   epilogue: v += bias[n] (nullable); activation 1 = relu; v *= (mask[m*ldm+n] > 0)
 *   (mask nullable: relu'(y) of the layer below); v += beta * C_old.
 * Requires 16-byte aligned pointers and leading dimensions that are multiples of 4.
 * ------------------------------------------------------------------------------------- */
enum { RS_ACT_NONE = 0, RS_ACT_RELU = 1 };
/* Contraction precision of the GEMM-shaped kernels (the *_prec_f32 entry points; the plain
 * entries are RS_PREC_F32). fp32 operands, fp32 accumulation in every mode:
 *   RS_PREC_F32        f32 operands on v_mfma_f32_32x32x2_f32;
 *   RS_PREC_F32_SPLIT9 every fp32 operand split exactly into three bf16 terms (x = h + m + l)
 *                      and all nine cross products summed on v_mfma_f32_32x32x16_bf16: the
 *                      fp32 products exactly, only the order of the additions differs;
 *   RS_PREC_F32_SPLIT6 the same without the three products below 2^-23 of |x.y| (m.l, l.m,
 *                      l.l): within one fp32 ulp per product, 2.7x the f32 MFMA product rate. */
enum { RS_PREC_F32 = 0, RS_PREC_F32_SPLIT6 = 6, RS_PREC_F32_SPLIT9 = 9 };
int rs_gemm_prec_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                     int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                     const float* bias, int activation, const float* mask, int64_t ldm, float beta,
                     int precision, rs_stream_t stream);
int rs_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                const float* bias, int activation, const float* mask, int64_t ldm, float beta,
                rs_stream_t stream);

/* Split-reduction GEMM for weight gradients (reduction over the batch, K >> M, N):
 *   C = op(A) @ op(B) + addend_scale * addend      (addend nullable, [M][ldc] layout)
 * computed as ordered partial slabs + a fixed-order reduction (bitwise reproducible).
 * Used with trans_a = 1 for dW = X^T G (Keras Dense kernel gradient) and with the L2
 * regularizer gradient 2*l2*W folded in as the addend (src/models.py:27). */
size_t rs_gemm_splitk_workspace_bytes(int64_t M, int64_t N, int64_t K);
int rs_gemm_splitk_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                       const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                       int64_t ldc, const float* addend, float addend_scale, void* workspace,
                       size_t workspace_bytes, rs_stream_t stream);
int rs_gemm_splitk_prec_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                            const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                            int64_t ldc, const float* addend, float addend_scale, int precision,
                            void* workspace, size_t workspace_bytes, rs_stream_t stream);

/* Dense weight and bias gradients in one split-K GEMM: dWdb[M + 1][N] = [X^T G ; 1^T G], i.e.
 * rows 0..M-1 = dW = X^T G (X [K][ldx] = the layer input, G [K][ldg] = dL/d(pre-activation)) and
 * row M = db = the column sums of G (a synthetic all-ones row of X^T). Replaces the MatMul grad +
 * BiasAddGrad of keras Dense (src/models.py:26-29,76-77). M must be a multiple of 4. W (nullable,
 * [M][N]) adds w_scale * (*w_dscale if non-null) * W to dW: the l2 kernel-regularizer gradient
 * (src/models.py:27) with its upstream gradient read on the device. */
size_t rs_gemm_wgrad_bias_workspace_bytes(int64_t M, int64_t N, int64_t K);
int rs_gemm_wgrad_bias_prec_f32(int64_t M, int64_t N, int64_t K, const float* X, int64_t ldx, const float* G,
                                int64_t ldg, float* dWdb, const float* W, float w_scale, const float* w_dscale,
                                int precision, void* workspace, size_t workspace_bytes, rs_stream_t stream,
                                void* queue);

/* Grouped launches: 1..4 problems of ONE shape (the user and item towers' Dense layers,
 * src/models.py:76-77,86,90, run at identical shapes) in one grid, each problem's results bitwise
 * those of its own single launch (same tiles, same sums). rs_gemm_group_prec_f32: C[g] =
 * act(op(A[g]) op(B[g]) + bias[g]) masked by mask[g] (bias / mask arrays nullable, entries
 * nullable) as rs_gemm_prec_f32. rs_gemm_wgrad_bias_group_prec_f32: dWdb [ngroup][M + 1][N] (one
 * contiguous buffer) = rs_gemm_wgrad_bias_prec_f32 of (X[g], G[g]) without the l2 addend. */
int rs_gemm_group_prec_f32(int ngroup, int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                           const float* const* A, int64_t lda, const float* const* B, int64_t ldb, float* const* C,
                           int64_t ldc, const float* const* bias, int activation, const float* const* mask,
                           int64_t ldm, float beta, int precision, rs_stream_t stream);
/* rs_gemm_group_prec_f32 with each problem's B also given as a fragment image (b_img[g], from
 * rs_mlp_weight_image_f32: the forward image of W for op(B) = W, the chain image of W for op(B) =
 * W^T; NULL array = none). The large-batch skinny kernel at precision 6 then stages the pre-split
 * fragments instead of splitting B in every workgroup (bitwise the same products and sums); every
 * other kernel reads B as usual. */
int rs_gemm_group_img_prec_f32(int ngroup, int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                               const float* const* A, int64_t lda, const float* const* B, int64_t ldb,
                               float* const* C, int64_t ldc, const float* const* bias, int activation,
                               const float* const* mask, int64_t ldm, float beta, int precision,
                               const void* const* b_img, rs_stream_t stream);
size_t rs_gemm_wgrad_bias_group_workspace_bytes(int ngroup, int64_t M, int64_t N, int64_t K);
int rs_gemm_wgrad_bias_group_prec_f32(int ngroup, int64_t M, int64_t N, int64_t K, const float* const* X,
                                      int64_t ldx, const float* const* G, int64_t ldg, float* dWdb, int precision,
                                      void* workspace, size_t workspace_bytes, rs_stream_t stream, void* queue);

/* Distinct-row Dense layers (the towers over a batch's distinct ids, src/models.py:85-90: a tower row
 * is a function of the id alone). rs_gemm_group_rows_prec_f32: the forward or dX of
 * rs_gemm_group_prec_f32 (trans_a = 0, beta = 0) on the weight-stationary kernel, with m_dev[g]
 * (nullable array / entries) = a device int64 holding problem g's row count (<= M; rows past it are
 * neither read nor written, so a graph sized for M serves any count), mask_rows[g] (nullable) =
 * int32 row map: the ReLU mask of output row m is row mask_rows[g][m] of mask[g] (the per-batch-row
 * dX of a layer whose activations are stored once per distinct id), and a_rows[g] (nullable) = int32
 * row map: output row m reads row a_rows[g][m] of A[g] (a per-batch-row layer over distinct rows'
 * inputs: the towers' top layer writes the batch rows directly). Precision 6 / 9, K and N in
 * {64, 128, 256}, >= 32768 rows over all problems; RS_ERR_UNSUPPORTED otherwise.
 * rs_gemm_wgrad_bias_group_rows_prec_f32: rs_gemm_wgrad_bias_group_prec_f32 with X's rows mapped:
 * contraction row k (a batch row) reads row x_rows[g][k] of X[g] (the layer input stored per distinct
 * id); the same split-K tiles and slab order, so the sums are bitwise those over the expanded X.
 * Precision 6 / 9. */
int rs_gemm_group_rows_prec_f32(int ngroup, int trans_b, int64_t M, int64_t N, int64_t K, const float* const* A,
                                int64_t lda, const int32_t* const* a_rows, const float* const* B, int64_t ldb,
                                float* const* C, int64_t ldc, const float* const* bias, int activation,
                                const float* const* mask, int64_t ldm, const int32_t* const* mask_rows,
                                const int64_t* const* m_dev, int precision, rs_stream_t stream);
int rs_gemm_wgrad_bias_group_rows_prec_f32(int ngroup, int64_t M, int64_t N, int64_t K, const float* const* X,
                                           int64_t ldx, const int32_t* const* x_rows, const float* const* G,
                                           int64_t ldg, float* dWdb, int precision, void* workspace,
                                           size_t workspace_bytes, rs_stream_t stream, void* queue);

/* A whole Dense stack's forward in one launch (the towers and the DCN deep net, src/models.py:
 * 26-29,76-77, at small batches where per-layer launches cost more than their math): for G = 1..2
 * stacks of one architecture, L = 1..6 layers, y[s*L + l] = act_l(y[s*L + l - 1] W_l + b[s*L + l])
 * with y_{-1} = x[s]. dims[0..L] are the widths: dims[0] (x's row length) a multiple of 32 in
 * 32..256, dims[l + 1] (layer l's output width) 64, 128 or 256. Row-major, dense leading
 * dimensions; b nullable (or its entries); relu[l] != 0 applies a ReLU. Every layer's output is
 * written (the backward's operands). The weights enter as img[s], stack s's fragment image
 * (rs_mlp_weight_image_f32 of W [dims[l]][dims[l + 1]], the keras kernel layout). precision
 * RS_PREC_F32_SPLIT6 / 9 (the same split products as rs_gemm_prec_f32 at that precision; the k-sum
 * order differs, so results agree to the fp32 rounding of the sums). */
size_t rs_mlp_weight_image_bytes(int L, const int64_t* dims);
/* img[s] (rs_mlp_weight_image_bytes, 16-byte aligned) <- every 16x16x32 MFMA B fragment of each
 * W[s*L + l] (for the forward) and of its transpose (for the chain) as exact three-term bf16
 * splits; widths multiples of 32. Rebuild after every weight update. */
int rs_mlp_weight_image_f32(int G, int L, const int64_t* dims, const float* const* W, void* const* img,
                            rs_stream_t stream);
/* The same images for n layers of any stacks in one launch: layer i (W[i] [K[i]][N[i]]) gets its
 * forward image at dst[i] and its chain image right after it (6 K N bytes each) — so layer l of a
 * stack image sits at the offset rs_mlp_weight_image_f32 gives it (a model builds every stack
 * node's image of a step in one launch). */
int rs_mlp_weight_images_f32(int n, const int64_t* K, const int64_t* N, const float* const* W, void* const* dst,
                             rs_stream_t stream);
int rs_mlp_fwd_prec_f32(int G, int L, const int64_t* dims, int64_t M, const float* const* x, const void* const* img,
                        const float* const* b, const int* relu, float* const* y, int precision, rs_stream_t stream);
/* The backward's input-gradient chain of the same stacks in one launch: from g_top[s] [M][dims[L]]
 * (dL/d of the top layer's pre-activation, its own ReLU already applied), for l = L-1 .. 0:
 * g[s*L + l] [M][dims[l]] = g_{l+1} W_l^T, zeroed where y[s*L + l - 1] <= 0 when relu[l - 1]
 * (TF's ReluGrad; y = the forward outputs as rs_mlp_fwd_prec_f32 wrote them), g_{L} = g_top, W_l
 * from img[s] (the forward's image). g[s*L + 0] = dL/dx; when every stack's is NULL that stage is
 * skipped. Widths dims[1..L] (and dims[0] when dL/dx is wanted) 64, 128 or 256. Each g[s*L + l] is
 * the operand of layer l - 1's weight gradient. */
int rs_mlp_bwd_chain_prec_f32(int G, int L, const int64_t* dims, int64_t M, const float* const* g_top,
                              const void* const* img, const float* const* y, const int* relu, float* const* g,
                              int precision, rs_stream_t stream);
/* The weight gradients of the same stacks in one launch: for every stack s and layer l,
 * dWdb[s*L + l] [dims[l] + 1][dims[l + 1]] = x_l^T g_l in its first dims[l] rows and the column sums
 * of g_l in its last (rs_gemm_wgrad_bias_prec_f32's layout), x_l = x[s*L + l] [M][dims[l]] (layer
 * l's input), g_l = g[s*L + l] [M][dims[l + 1]]; with w_reg (nullable, or its entries) dW +=
 * w_scale * (*w_dscale) * w_reg (the folded l2 term). Widths multiples of 64. M is split into up
 * to 16 slices whose partial images the ordered slab reduction sums (one job per layer, queued on
 * `queue` when given, as rs_gemm_wgrad_bias_prec_f32's). Workspace: rs_mlp_wgrad_workspace_bytes
 * (0 when M needs one slice). M = 0 writes dW = the l2 term (or 0) and db = 0 (x, g may be null). */
size_t rs_mlp_wgrad_workspace_bytes(int G, int L, const int64_t* dims, int64_t M);
int rs_mlp_wgrad_prec_f32(int G, int L, const int64_t* dims, int64_t M, const float* const* x, const float* const* g,
                          float* const* dWdb, const float* const* w_reg, float w_scale, const float* w_dscale,
                          int precision, void* workspace, size_t workspace_bytes, rs_stream_t stream, void* queue);

/* Pre-split operands for the split-precision GEMMs (RS_PREC_F32_SPLIT6 / 9): a plane image holds
 * the three exact bf16 terms (h, m, l) of every element of an fp32 matrix X [rows][cols] (leading
 * dim ldx), in the byte layout the GEMM streams into LDS unchanged. layout 0 (KC) treats the
 * columns as the contraction index (the A of X W, or the B^T of W X^T), layout 1 (KM) the rows
 * (the A^T of X^T Y, or the B of W X). Size: rs_plane_image_bytes(contraction extent, other
 * extent), i.e. (cols, rows) for KC and (rows, cols) for KM. */
size_t rs_plane_image_bytes(int64_t k_extent, int64_t extent);
int rs_plane_image_f32(const float* X, int64_t ldx, int64_t rows, int64_t cols, int layout, void* img,
                       rs_stream_t stream);
/* C = act(op(A) op(B) + bias) + beta C from plane images: A is a KC image of A [M][K] when
 * !trans_a, a KM image of A^T [K][M] when trans_a; B is a KM image of B [K][N] when !trans_b, a KC
 * image of B^T [N][K] when trans_b. Bitwise the sums of rs_gemm_prec_f32 at the same precision
 * (same products, same k order), on 256 x 256 tiles streamed by LDS-DMA. */
int rs_gemm_planes_prec_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const void* Aimg,
                            const void* Bimg, float* C, int64_t ldc, const float* bias, int activation,
                            float beta, int precision, rs_stream_t stream);

/* The same product with the contraction range split over workgroups (weight gradients, K = batch):
 * C [M][N] dense = op(A) op(B) + addend_scale * addend, slabs summed in a fixed order. */
size_t rs_gemm_planes_splitk_workspace_bytes(int64_t M, int64_t N, int64_t K);
int rs_gemm_planes_splitk_prec_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const void* Aimg,
                                   const void* Bimg, float* C, const float* addend, float addend_scale,
                                   int precision, void* workspace, size_t workspace_bytes, rs_stream_t stream);

/* Plane-pair GEMM (precision 6): C[M][N] = epilogue(sum_k A[m][k] B[n][k]) with both operands
 * given as xgemm images (bf16 planes h, m, l of every fp32 element; 8 KB blocks per (plane, 16-k
 * block, 256-row tile)), built by rs_xgemm_image_f32 from an fp32 matrix viewed as [rows][k_extent]
 * (trans = 0: stored [rows][ldx]; trans = 1: stored [k_extent][ldx], i.e. the transpose is taken
 * while splitting). Two cross products per 16x16x32 MFMA, 256 x 256 tiles.
 * Replaces the Dense / DCN-v2 cross MatMuls (src/models.py:26-29,38-44) on the split path. */
size_t rs_xgemm_image_bytes(int64_t rows, int64_t k_extent);
int rs_xgemm_image_f32(const float* X, int64_t ldx, int64_t rows, int64_t k_extent, int trans, void* img,
                       rs_stream_t stream);
/* Both xgemm images from ONE read of X [rows][k_extent] (k_extent % 4 == 0, dense rows): img =
 * rs_xgemm_image_f32(X, trans 0) and img_t = rs_xgemm_image_f32 of X^T (rows k_extent,
 * contraction rows), byte for byte. With relu_y (nullable, [rows][k_extent]) the images are those
 * of X * (relu_y > 0) (TF ReluGrad of a Dense layer's output), and colsum (nullable, [k_extent])
 * receives that matrix's column sums (the bias gradient, ordered). The workspace is needed when
 * relu_y or colsum is given. Used by the DCN-v2 trunk's deep tower (src/models.py:26-29,46-48
 * shape, config 5) on the plane-pair GEMM. */
size_t rs_xgemm_image_dual_workspace_bytes(int64_t rows, int64_t k_extent);
int rs_xgemm_image_dual_f32(const float* X, const float* relu_y, int64_t rows, int64_t k_extent, void* img,
                            void* img_t, float* colsum, void* workspace, size_t workspace_bytes, rs_stream_t stream);
int rs_xgemm_prec_f32(int64_t M, int64_t N, int64_t K, const void* Aimg, const void* Bimg, float* C, int64_t ldc,
                      const float* bias, int activation, float beta, int precision, rs_stream_t stream);
size_t rs_xgemm_splitk_workspace_bytes(int64_t M, int64_t N, int64_t K);
int rs_xgemm_splitk_prec_f32(int64_t M, int64_t N, int64_t K, const void* Aimg, const void* Bimg, float* C,
                             const float* addend, float addend_scale, int precision, void* workspace,
                             size_t workspace_bytes, rs_stream_t stream);

/* ReLU backward + bias gradient: g = dy * (y > 0) (y nullable: identity), colsum[n] = sum_m g.
 * Deterministic ordered column sums. g may alias dy. A float4 pass runs when N % 4 == 0 and
 * dy, y, g and the workspace are all 16-B aligned, else a scalar pass; the two sum the rows in
 * different blocks, so for the same data the colsum bits are fixed per path (always the same
 * for the same alignment), not across paths. */
size_t rs_colsum_workspace_bytes(int64_t M, int64_t N);
int rs_relu_bwd_colsum_f32(const float* dy, const float* y, int64_t M, int64_t N, float* g,
                           float* colsum, void* workspace, size_t workspace_bytes,
                           rs_stream_t stream, void* queue);

/* Sum of squares, out[0] = scale * sum(x^2) (Keras l2 regularizer value, src/models.py:27). */
size_t rs_sum_squares_workspace_bytes(int64_t n);
/* out = scale * sum over 1..8 tensors of sum(x_k^2) (fp64 partials, one partial pass for all):
 * the l2 kernel regularizer of a whole Dense stack (src/models.py:27). x, n: host arrays. */
size_t rs_sum_squares_multi_workspace_bytes(int ntensors, const int64_t* n);
int rs_sum_squares_multi_f32(int ntensors, const float* const* x, const int64_t* n, float scale, float* out,
                             void* workspace, size_t workspace_bytes, rs_stream_t stream);
int rs_sum_squares_f32(const float* x, int64_t n, float scale, float* out, void* workspace,
                       size_t workspace_bytes, rs_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * a5 + a7 / K5 + K6 — DCN (v1, vector weight) cross stack, all L layers in one pass.
 * Replaces tf.concat([u, i], 1) (src/models.py:128) and DeepCrossNetwork.call's cross loop
 * (src/models.py:38-44):  x0 = [u || v] (width d = 2*D);
 *   s_l = x_l . w_l ;  x_{l+1} = x0 * s_l + b_l + x_l          (w, b packed as [L][d])
 * Outputs x0 [B][d], xL [B][d], s [B][L] (saved for the backward).
 * ------------------------------------------------------------------------------------- */
int rs_dcn_cross_vec_fwd_f32(const float* u, const float* v, int64_t B, int64_t D, int L,
                             const float* w, const float* b, float* x0, float* xl, float* s,
                             rs_stream_t stream);
/* Backward: given g_xl = dLoss/dxL and g_x0_extra = dLoss/dx0 from other consumers of x0
 * (the deep net; nullable) produce the two halves of dLoss/dx0, g_u = [:, :D] and
 * g_v = [:, D:] (the concat's backward), and g_w [L][d], g_b [L][d] (ordered sums). */
size_t rs_dcn_cross_vec_bwd_workspace_bytes(int64_t B, int64_t D, int L);
int rs_dcn_cross_vec_bwd_f32(const float* x0, const float* s, const float* w, const float* b,
                             int64_t B, int64_t D, int L, const float* g_xl,
                             const float* g_x0_extra, float* g_u, float* g_v, float* g_w,
                             float* g_b, void* workspace, size_t workspace_bytes,
                             rs_stream_t stream, void* queue);
/* The same, with the gradients of another consumer of u and v (the retrieval task's dU and dC,
 * src/models.py:137, on the same tower outputs as the concat at :128) added last to g_u / g_v in
 * the kernel: g_u = (cross + extra) + add_u, bitwise what a separate accumulation pass produces. */
int rs_dcn_cross_vec_bwd_add_f32(const float* x0, const float* s, const float* w, const float* b, int64_t B,
                                 int64_t D, int L, const float* g_xl, const float* g_x0_extra, const float* add_u,
                                 const float* add_v, float* g_u, float* g_v, float* g_w, float* g_b, void* workspace,
                                 size_t workspace_bytes, rs_stream_t stream, void* queue);

/* ---------------------------------------------------------------------------------------
 * K6 extension (BASELINE config 5; no reference code: the reference cross weight is [d,1]) —
 * DCN-v2 matrix cross stack, u_l = x_l W_l + b_l, x_{l+1} = x0 * u_l + x_l, W packed [L][d][d]
 * (Keras [in][out]), b [L][d]. Forward writes x_1..x_L to xs [L][B][d] (x_L = output) and u_l
 * to us [L][B][d] for the backward. d must be a multiple of 4 (pad x0 with zero columns).
 * ------------------------------------------------------------------------------------- */
int rs_dcn_cross_mat_fwd_f32(const float* x0, int64_t B, int64_t d, int L, const float* W,
                             const float* b, float* xs, float* us, rs_stream_t stream);
size_t rs_dcn_cross_mat_bwd_workspace_bytes(int64_t B, int64_t d, int L);
/* g_x0 = dLoss/dx0 (direct x0 terms + the residual chain + g_x0_extra, nullable), g_W, g_b. */
int rs_dcn_cross_mat_bwd_f32(const float* x0, const float* xs, const float* us, const float* W,
                             int64_t B, int64_t d, int L, const float* g_xl,
                             const float* g_x0_extra, float* g_x0, float* g_W, float* g_b,
                             void* workspace, size_t workspace_bytes, rs_stream_t stream);
/* The same at a contraction precision (RS_PREC_*) for the layer GEMMs. */
int rs_dcn_cross_mat_fwd_prec_f32(const float* x0, int64_t B, int64_t d, int L, const float* W,
                                  const float* b, float* xs, float* us, int precision, rs_stream_t stream);
int rs_dcn_cross_mat_bwd_prec_f32(const float* x0, const float* xs, const float* us, const float* W,
                                  int64_t B, int64_t d, int L, const float* g_xl,
                                  const float* g_x0_extra, float* g_x0, float* g_W, float* g_b, int precision,
                                  void* workspace, size_t workspace_bytes, rs_stream_t stream);
/* Plane-image path of the same stack at precision 6 (the config-5 default): every GEMM operand is
 * split once into an xgemm image (rs_xgemm_image_f32) and the three GEMMs per layer run on the
 * plane-pair kernel (rs_xgemm_*). Same products as rs_dcn_cross_mat_*_prec_f32 at precision 6; the
 * fp32 additions run in another order (within a few fp32 ulps of each other).
 * ximg (rs_dcn_cross_mat_planes_bytes) receives the forward's images of x_0^T..x_{L-1}^T, which
 * the backward reads for dW_l = x_l^T t: keep it alive between the two calls. */
size_t rs_dcn_cross_mat_planes_bytes(int64_t B, int64_t d, int L);
size_t rs_dcn_cross_mat_fwd_planes_workspace_bytes(int64_t B, int64_t d);
int rs_dcn_cross_mat_fwd_planes_f32(const float* x0, int64_t B, int64_t d, int L, const float* W, const float* b,
                                    float* xs, float* us, void* ximg, int precision, void* workspace,
                                    size_t workspace_bytes, rs_stream_t stream);
/* The same with x0's xgemm image (rs_xgemm_image_f32 of x0, trans 0; rs_xgemm_image_bytes(B, d)
 * bytes) also written to x0_img (nullable): the DCN-v2 trunk's deep tower reads x0 from it. */
int rs_dcn_cross_mat_fwd_planes_x0img_f32(const float* x0, int64_t B, int64_t d, int L, const float* W,
                                          const float* b, float* xs, float* us, void* ximg, void* x0_img,
                                          int precision, void* workspace, size_t workspace_bytes,
                                          rs_stream_t stream);
size_t rs_dcn_cross_mat_bwd_planes_workspace_bytes(int64_t B, int64_t d, int L);
int rs_dcn_cross_mat_bwd_planes_f32(const float* x0, const float* xs, const float* us, const float* W,
                                    const void* ximg, int64_t B, int64_t d, int L, const float* g_xl,
                                    const float* g_x0_extra, float* g_x0, float* g_W, float* g_b, int precision,
                                    void* workspace, size_t workspace_bytes, rs_stream_t stream);

/* a12 — compute_loss's task weighting (src/models.py:147): *total = w_ret *ret + w_rat *rating
 * + w_ctr *ctr (ctr nullable = 0), fp32 left to right, one launch; the backward writes
 * grads[0..2] = *g * (w_ret, w_rat, w_ctr). */
int rs_loss_combine_f32(const float* ret, const float* rating, const float* ctr, float w_ret, float w_rat,
                        float w_ctr, float* total, rs_stream_t stream);
int rs_loss_combine_bwd_f32(const float* g, float w_ret, float w_rat, float w_ctr, float* grads,
                            rs_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * a9 / K8 — concat([xL, deep]) + rating head Dense(1) + ctr head Dense(1, sigmoid).
 * Replaces src/models.py:50 and :119-120,131.  z = [xl || h] (width dx + dh);
 *   rating[b] = z . w_r + b_r[0] ;  ctr[b] = sigmoid(z . w_c + b_c[0]).
 * ------------------------------------------------------------------------------------- */
int rs_heads_fwd_f32(const float* xl, int64_t dx, const float* h, int64_t dh, int64_t B,
                     const float* w_r, const float* b_r, const float* w_c, const float* b_c,
                     float* rating, float* ctr, rs_stream_t stream);
/* Backward. Per-row upstream grads: dr_b = g_rating[b] + (*gs_rat) * unit_r[b],
 * dp_b = g_ctr[b] + (*gs_ctr) * unit_c[b] (every term nullable); dlogit = dp * p * (1 - p).
 * Outputs g_xl [B][dx], g_h [B][dh], g_wr/g_wc [dx+dh], g_br/g_bc [1] (ordered sums).
 * Any width: rows wider than 1,024 floats run as column chunks. */
size_t rs_heads_bwd_workspace_bytes(int64_t B, int64_t dx, int64_t dh);
int rs_heads_bwd_f32(const float* xl, int64_t dx, const float* h, int64_t dh, int64_t B,
                     const float* w_r, const float* w_c, const float* ctr,
                     const float* g_rating, const float* g_ctr, const float* unit_r,
                     const float* unit_c, const float* gs_rat, const float* gs_ctr,
                     float* g_xl, float* g_h, float* g_wr, float* g_br, float* g_wc,
                     float* g_bc, void* workspace, size_t workspace_bytes, rs_stream_t stream,
                     void* queue);

/* The heads backward with compute_loss's task weighting folded in (src/models.py:147, the backward
 * of rs_ranking_losses_combine_f32's total): the per-row upstream gradients are dr_b = (*g_total *
 * w_rat) unit_r[b] and dp_b = (*g_total * w_ctr) unit_c[b] (dp_b = 0 without RS_HEADS_USE_CTR), and
 * g_ret[0] = *g_total * w_ret (the retrieval task's gradient). flags: RS_HEADS_USE_CTR, and
 * RS_HEADS_RELU_H when h is the output of a ReLU layer (the DCN deep net, src/models.py:26-29):
 * g_h is then the gradient at that layer's pre-activation, g_h = 0 where h <= 0 (TF's ReluGrad, so
 * the deep net's backward starts from it). Same outputs and queue rule as rs_heads_bwd_f32. */
#define RS_HEADS_USE_CTR 1
#define RS_HEADS_RELU_H 2
int rs_heads_bwd_combine_f32(const float* xl, int64_t dx, const float* h, int64_t dh, int64_t B, const float* w_r,
                             const float* w_c, const float* ctr, const float* unit_r, const float* unit_c,
                             const float* g_total, float w_ret, float w_rat, float w_ctr, int flags, float* g_ret,
                             float* g_xl, float* g_h, float* g_wr, float* g_br, float* g_wc, float* g_bc,
                             void* workspace, size_t workspace_bytes, rs_stream_t stream, void* queue);

/* ---------------------------------------------------------------------------------------
 * a11 / K10 — tfrs.tasks.Ranking(MSE) and Ranking(BCE, sample_weight = class weight of the
 * label) (src/models.py:122-123,138-145).  loss[0] = mean_b (r_b - y_b)^2 ;
 *   ctr_mode 0: loss[1] = (1/B) sum_b sw_b * bce_b        (per-sample weighting)
 *   ctr_mode 1: loss[1] = mean_b(bce_b) * mean_b(sw_b)    (Keras 3 rank-1 broadcasting)
 *   bce_b = -(y log(pc + 1e-7) + (1 - y) log(1 - pc + 1e-7)), pc = clip(p, 1e-7, 1 - 1e-7)
 *   sw_b = use_class_weights ? (y_b == 1 ? cw1 : cw0) : 1.
 * Also writes unit_r[b] = dloss0/dr_b and unit_c[b] = dloss1/dp_b (for rs_heads_bwd_f32).
 * ------------------------------------------------------------------------------------- */
size_t rs_ranking_losses_workspace_bytes(int64_t B);
int rs_ranking_losses_f32(const float* rating_pred, const float* ctr_pred, const float* rating,
                          const float* y_implicit, int64_t B, int use_class_weights, float cw0,
                          float cw1, int ctr_mode, float* loss, float* unit_r, float* unit_c,
                          void* workspace, size_t workspace_bytes, rs_stream_t stream);
/* The same losses with compute_loss's weighting (src/models.py:147) and the train step's
 * regularizer in the same launch sequence: *total = (w_ret *ret + w_rat loss[0]) + w_ctr loss[1]
 * (the ctr term only with use_ctr, :140), *total_reg (nullable) = *total + *reg (reg nullable: + 0).
 * Up to B = 16384 the whole sequence is ONE launch (one workgroup; the same partials and trees). */
int rs_ranking_losses_combine_f32(const float* rating_pred, const float* ctr_pred, const float* rating,
                                  const float* y_implicit, int64_t B, int use_class_weights, float cw0, float cw1,
                                  int ctr_mode, const float* ret, const float* reg, float w_ret, float w_rat,
                                  float w_ctr, int use_ctr, float* loss, float* total, float* total_reg,
                                  float* unit_r, float* unit_c, void* workspace, size_t workspace_bytes,
                                  rs_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * a10 / K9 — tfrs.tasks.Retrieval() in-batch softmax cross-entropy (src/models.py:116,137):
 *   S = U C^T (B x B, never materialised), L = sum_i (logsumexp_j S_ij - S_ii)  (SUM).
 * Forward (flash-style, fp32 MFMA, online row max): row_loss[B], lse[B], loss_sum[0] (fp32;
 * loss_sum64 fp64, nullable; ordered sums). If dU != NULL the forward also produces the
 * unit-upstream gradient dU = weight * (softmax(S) C - C) from the same pass.
 * ------------------------------------------------------------------------------------- */
size_t rs_inbatch_softmax_workspace_bytes(int64_t B, int64_t D);
int rs_inbatch_softmax_xent_fwd_f32(const float* U, const float* C, int64_t B, int64_t D,
                                    float weight, float* row_loss, float* lse,
                                    float* loss_sum, double* loss_sum64, float* dU,
                                    void* workspace, size_t workspace_bytes,
                                    rs_stream_t stream);
/* Backward: dC = g * weight * (softmax(S)^T U - U) using the forward's lse, and
 * dU_out = g * dU_unit (the forward's unit gradient; both nullable), g = *gscale (nullable: 1). */
int rs_inbatch_softmax_xent_bwd_f32(const float* U, const float* C, int64_t B, int64_t D,
                                    float weight, const float* lse, const float* gscale,
                                    const float* dU_unit, float* dU_out, float* dC,
                                    void* workspace, size_t workspace_bytes,
                                    rs_stream_t stream);

/* ---------------------------------------------------------------------------------------
 * a13 / K11 — dense Adagrad over many tensors, one launch sequence.
 * Replaces keras.optimizers.Adagrad(ExponentialDecay(...), clipnorm=1.0) applied to the dense
 * variables (src/trainer.py:157-163): per tensor g <- g * clipnorm / max(||g||, clipnorm),
 * acc += g^2, p -= lr_t * g / sqrt(acc + epsilon). `slots` is a DEVICE array.
 * ------------------------------------------------------------------------------------- */
typedef struct {
  float* param;
  const float* grad;
  float* accum;
  int64_t numel;
} rs_dense_slot;
size_t rs_adagrad_dense_workspace_bytes(int ntensors, int64_t max_numel);
int rs_adagrad_dense_f32(const rs_dense_slot* slots, int ntensors, int64_t max_numel,
                         const int64_t* iteration, float lr0, float decay_rate,
                         int64_t decay_steps, float clipnorm, float epsilon, void* workspace,
                         size_t workspace_bytes, rs_stream_t stream);
/* *iteration += 1 on the device (Keras optimizer.iterations). */
int rs_iteration_increment(int64_t* iteration, rs_stream_t stream);

/* Deferred reductions (launch count of small-batch training steps). The entry points that end in
 * an ordered second-stage reduction of a parameter gradient (rs_gemm_wgrad_bias_prec_f32,
 * rs_gemm_wgrad_bias_group_prec_f32, rs_relu_bwd_colsum_f32, rs_dcn_cross_vec_bwd[_add]_f32,
 * rs_heads_bwd_f32 with one column chunk) take a trailing `queue` (HOST pointer, nullable): NULL
 * launches the reduction at once; a queue initialised by rs_reduction_queue_init receives it
 * instead, and rs_reduction_queue_flush(queue, stream) runs every queued reduction in ONE launch
 * with bitwise the same sums. Until the flush the queued outputs are not written, and the
 * workspaces, addends and outputs handed to those calls must stay allocated. The queue is
 * caller-owned memory of rs_reduction_queue_bytes() bytes (8-byte aligned): the library keeps no
 * state of its own, so two training loops use two queues and never see each other's jobs. A queue
 * is not thread-safe (one backward at a time); its jobs belong to the stream they were queued on
 * (a call on another stream first launches what is queued, on the old stream), and a full queue
 * launches its jobs before taking the next. Replaces nothing in the reference: TF launches one
 * reduction per gradient op (src/trainer.py:163 apply_gradients reads the gradients). */
size_t rs_reduction_queue_bytes(void);
int rs_reduction_queue_init(void* queue, size_t bytes);
int rs_reduction_queue_flush(void* queue, rs_stream_t stream);
/* number of queued reductions (>= 0), or RS_ERR_INVALID_ARG for an uninitialised queue */
int rs_reduction_queue_pending(const void* queue);

/* ---------------------------------------------------------------------------------------
 * a16 / K12 / K13 — exact brute-force inner-product top-K.
 * Replaces np.dot(user_embs, item_embs.T) + np.argpartition(-sim, k) of
 * ProductionTrainer._evaluate (src/trainer.py:204-212) and faiss.IndexFlatIP.search
 * (src/trainer.py:240-243, app/recommendation_service.py:71-72; cosine = L2-normalised rows).
 * out[q][0..k) ordered by (-score, index); index = row + index_base (row-sharded tables pass
 * their first global row). k <= 128, N < 2^31 per call, D in {32, 64, 128}.
 * ------------------------------------------------------------------------------------- */
size_t rs_topk_ip_workspace_bytes(int64_t nq, int64_t N, int64_t D, int k);
int rs_topk_ip_f32(const float* queries, int64_t nq, const float* items, int64_t N, int64_t D,
                   int k, int64_t index_base, float* out_scores, int64_t* out_index,
                   void* workspace, size_t workspace_bytes, rs_stream_t stream);
/* The same with the scan's contraction precision (RS_PREC_*): the split kernels run for more than
 * 64 queries at D = 128 (the MFMA-bound regime); on dyadic-grid data their scores, and so the
 * lists, are bitwise those of RS_PREC_F32. */
int rs_topk_ip_prec_f32(const float* queries, int64_t nq, const float* items, int64_t N, int64_t D,
                        int k, int64_t index_base, float* out_scores, int64_t* out_index, int precision,
                        void* workspace, size_t workspace_bytes, rs_stream_t stream);
/* RS_TOPK_LIST_SCAN, OR'd into that precision argument: the single-pass list scan even where the
 * bound-first scan would run (> 64 queries, >= 2^20 rows, split precision). Same lists, bitwise:
 * both scans score every (query, item) with the same kernel arithmetic and order by (-score, index);
 * it exists to check the one against the other. */
#define RS_TOPK_LIST_SCAN 0x100
/* Merge nlists sorted per-query lists (e.g. all-gathered shard results) [nq][nlists][k] into
 * [nq][k] under the same ordering (the C4 row-sharded top-K exchange step). */
size_t rs_topk_merge_workspace_bytes(int64_t nq, int64_t nlists, int k);
int rs_topk_merge_f32(const float* in_scores, const int64_t* in_index, int64_t nq,
                      int64_t nlists, int k, float* out_scores, int64_t* out_index,
                      void* workspace, size_t workspace_bytes, rs_stream_t stream);

/* Score-storing variant of the in-batch softmax (same reference call site, src/models.py:116,137):
 * the forward also writes the B x B fp32 scores (rs_inbatch_scores_bytes(B) bytes, 32 x 32 tile
 * layout private to the pair) and the backward reads them instead of recomputing U C^T, halving
 * the backward's MFMA work (17.2 GB at B = 65536: sized for 288 GB of HBM). Results are bitwise
 * equal to the recomputing pair. dU is required by the forward. */
size_t rs_inbatch_scores_bytes(int64_t B);
int rs_inbatch_softmax_xent_fwd_store_f32(const float* U, const float* C, int64_t B, int64_t D,
                                          float weight, float* row_loss, float* lse,
                                          float* loss_sum, double* loss_sum64, float* dU,
                                          float* scores, void* workspace, size_t workspace_bytes,
                                          rs_stream_t stream);
int rs_inbatch_softmax_xent_bwd_stored_f32(const float* U, const float* C, int64_t B, int64_t D,
                                           float weight, const float* lse, const float* scores,
                                           const float* gscale, const float* dU_unit,
                                           float* dU_out, float* dC, void* workspace,
                                           size_t workspace_bytes, rs_stream_t stream);
/* RS_INBATCH_FWD_WS, OR'd into the precision argument of a backward entry that reads kept scores
 * (rs_inbatch_softmax_xent_bwd_stored_prec_f32, _bwd_dedup_f32, _bwd_dedup_dev_f32): the workspace
 * is the one the matching storing forward was given (same B, D, precision), untouched since; the
 * forward's split image of U is reused instead of split again (one launch fewer). Without it the
 * backward's workspace may be any buffer of the queried size. */
#define RS_INBATCH_FWD_WS 0x100
/* The same pair with the contraction precision chosen by the caller (RS_PREC_*, declared with
 * the GEMM above; the plain entries are RS_PREC_F32). The split kernels are compiled for
 * D = 128; other widths run the RS_PREC_F32 kernels. */
int rs_inbatch_softmax_xent_fwd_store_prec_f32(const float* U, const float* C, int64_t B, int64_t D,
                                               float weight, float* row_loss, float* lse,
                                               float* loss_sum, double* loss_sum64, float* dU,
                                               float* scores, int precision, void* workspace,
                                               size_t workspace_bytes, rs_stream_t stream);
int rs_inbatch_softmax_xent_bwd_stored_prec_f32(const float* U, const float* C, int64_t B, int64_t D,
                                                float weight, const float* lse, const float* scores,
                                                const float* gscale, const float* dU_unit,
                                                float* dU_out, float* dC, int precision,
                                                void* workspace, size_t workspace_bytes,
                                                rs_stream_t stream);

/* Deduplicated pair (same reference call site, src/models.py:116,137): batches drawn from skewed
 * id distributions repeat tower rows, and a row repeated n times is n identical columns (or rows)
 * of S. rs_inbatch_unique_rows_f32 finds the distinct rows of X [B][D] BY CONTENT (bitwise, via a
 * 64-bit hash, sort and verification): rep[u] = first batch row of distinct row u (u < nu),
 * inv[i] = distinct index of row i, count[u] = its multiplicity (count holds ceil(B/32)*32 floats,
 * zero past nu), info[0] = nu, info[1] = rows whose bits differ from their representative's (a hash
 * collision: the caller must then use the full pair). Device outputs, no host synchronisation.
 * The pair then runs the row pass over Bu distinct users x Bc distinct items (item counts as
 * weights) and the col pass over Bc x Bu (user counts as weights): per batch row the same loss,
 * lse, dU and dC as rs_inbatch_softmax_xent_fwd_store_prec_f32 / _bwd_stored_prec_f32 up to the
 * order of the fp32 sums, for Bu x Bc instead of B x B pair work. A side that is not deduplicated
 * passes NULL rep / inv / count and Bx = B. D = 128, precision RS_PREC_F32_SPLIT6 / 9; `scores`
 * is a buffer of rs_inbatch_scores_bytes(B) (Bu x Bc of it is used); dU is required. */
size_t rs_inbatch_unique_rows_workspace_bytes(int64_t B);
int rs_inbatch_unique_rows_f32(const float* X, int64_t B, int64_t D, int32_t* rep, float* count, int32_t* inv,
                               int64_t* info, void* workspace, size_t workspace_bytes, rs_stream_t stream);
/* Both sides at once (one hash / sort / scan sequence over U and C): u_* and c_* as above,
 * info[0..3] = (distinct users, user collision rows, distinct items, item collision rows). */
size_t rs_inbatch_unique_pair_workspace_bytes(int64_t B);
int rs_inbatch_unique_pair_f32(const float* U, const float* C, int64_t B, int64_t D, int32_t* u_rep,
                               float* u_count, int32_t* u_inv, int32_t* c_rep, float* c_count, int32_t* c_inv,
                               int64_t* info, void* workspace, size_t workspace_bytes, rs_stream_t stream);
/* The same outputs from the rows' integer ids instead of their content, for rows that are a
 * function of the id alone (the reference's towers: Embedding -> Dense stack, src/models.py:85-90):
 * rows with equal ids are grouped (no hash, no verification; info[1] = info[3] = 0); ids outside
 * [0, user_rows) / [0, item_rows) form one group per side (the gather's zero rows). Workspace:
 * rs_inbatch_unique_pair_workspace_bytes(B). */
int rs_inbatch_unique_ids_pair_i64(const int64_t* user_ids, const int64_t* item_ids, int64_t B, int64_t user_rows,
                                   int64_t item_rows, int32_t* u_rep, float* u_count, int32_t* u_inv, int32_t* c_rep,
                                   float* c_count, int32_t* c_inv, int64_t* info, void* workspace,
                                   size_t workspace_bytes, rs_stream_t stream);
/* The same search with each side's batch rows listed in ascending-id order (stable: equal ids in
 * batch order): u_order / c_order [B] int32 — the order rs_embedding_gather_tables_ordered_f32 reads
 * the tables in. */
int rs_inbatch_unique_ids_pair_order_i64(const int64_t* user_ids, const int64_t* item_ids, int64_t B,
                                         int64_t user_rows, int64_t item_rows, int32_t* u_rep, float* u_count,
                                         int32_t* u_inv, int32_t* u_order, int32_t* c_rep, float* c_count,
                                         int32_t* c_inv, int32_t* c_order, int64_t* info, void* workspace,
                                         size_t workspace_bytes, rs_stream_t stream);
/* The id plan with its optional outputs (each pair nullable together): u_order / c_order as in
 * rs_inbatch_unique_ids_pair_order_i64; u_did / c_did [B] int64 = each distinct slot's id (slots
 * are in ascending-id order; the group of out-of-range ids gets user_rows / item_rows, slots from the
 * distinct count on -1) — the ids rs_embedding_gather_tables_ids_f32 reads, with no further lookup;
 * u_start / c_start [B] int32 = each slot's first position in the side's order (slots past the count
 * unset) — the run heads rs_sparse_adagrad_multi_step_planned_f32 applies. With u_did / c_did, info
 * holds 6 entries: info[4] / info[5] = each side's distinct count without the out-of-range group (the
 * count rs_sparse_dedupe of the side's ids keeps). */
int rs_inbatch_unique_ids_plan_i64(const int64_t* user_ids, const int64_t* item_ids, int64_t B, int64_t user_rows,
                                   int64_t item_rows, int32_t* u_rep, float* u_count, int32_t* u_inv,
                                   int32_t* u_order, int64_t* u_did, int32_t* u_start, int32_t* c_rep,
                                   float* c_count, int32_t* c_inv, int32_t* c_order, int64_t* c_did,
                                   int32_t* c_start, int64_t* info, void* workspace, size_t workspace_bytes,
                                   rs_stream_t stream);
size_t rs_inbatch_dedup_workspace_bytes(int64_t B, int64_t D);
int rs_inbatch_softmax_xent_fwd_dedup_f32(const float* U, const float* C, int64_t B, int64_t D, float weight,
                                          const int32_t* u_rep, const int32_t* u_inv, int64_t Bu,
                                          const int32_t* c_rep, const float* c_count, int64_t Bc,
                                          float* row_loss, float* lse, float* loss_sum, double* loss_sum64,
                                          float* dU, float* scores, int precision, void* workspace,
                                          size_t workspace_bytes, rs_stream_t stream);
int rs_inbatch_softmax_xent_bwd_dedup_f32(const float* U, int64_t B, int64_t D, float weight, const float* lse,
                                          const float* scores, const float* gscale, const float* dU_unit,
                                          float* dU_out, float* dC, const int32_t* u_rep, const float* u_count,
                                          int64_t Bu, const int32_t* c_inv, int64_t Bc, int precision,
                                          void* workspace, size_t workspace_bytes, rs_stream_t stream);

/* The same pair with the distinct counts read ON THE DEVICE (no host synchronisation, so a training
 * step that uses it can be captured in a hipGraph): Bu = info[0] and Bc = info[2], the info array of
 * rs_inbatch_unique_ids_pair_i64 / rs_inbatch_unique_pair_f32 (whose collision counts info[1],
 * info[3] must be 0 — always so for the id search). Both sides are deduplicated; every grid is
 * sized for Bu = Bc = B and the stream-K shape is derived on the device by the host rule, so the
 * results are bitwise those of the host-count entries above at the same counts. */
int rs_inbatch_softmax_xent_fwd_dedup_dev_f32(const float* U, const float* C, int64_t B, int64_t D, float weight,
                                              const int32_t* u_rep, const int32_t* u_inv, const int32_t* c_rep,
                                              const float* c_count, const int64_t* info, float* row_loss, float* lse,
                                              float* loss_sum, double* loss_sum64, float* dU, float* scores,
                                              int precision, void* workspace, size_t workspace_bytes,
                                              rs_stream_t stream);
int rs_inbatch_softmax_xent_bwd_dedup_dev_f32(const float* U, int64_t B, int64_t D, float weight, const float* lse,
                                              const float* scores, const float* gscale, const float* dU_unit,
                                              float* dU_out, float* dC, const int32_t* u_rep, const float* u_count,
                                              const int32_t* c_inv, const int64_t* info, int precision,
                                              void* workspace, size_t workspace_bytes, rs_stream_t stream);

/* ---- ranking-metric suite ------------------------------------------------
 * Replaces AdvancedMetrics (src/evaluation.py:22-104) on integer item rows: pred [U][K] (K <= 1024)
 * top-K lists, lens [U] list lengths (nullable = all K; ragged lists are padded rows), truth [U]
 * true item per list, ks = up to 8 cut-offs (host array). out (device,
 * doubles) = for each cut-off k: recall@k, precision@k, ndcg@k, map@k; then mrr (whole list),
 * diversity (mean |set(list)|/len(list)), coverage (distinct listed items in [0, n_items) / n_items).
 * Means over the U lists with an ordered reduction (bit-reproducible). */
size_t rs_rank_metrics_workspace_bytes(int64_t U, int nks, int64_t n_items);
int rs_rank_metrics_i64(const int64_t* pred, int64_t U, int K, const int32_t* lens,
                        const int64_t* truth, const int32_t* ks, int nks, int64_t n_items, double* out,
                        void* workspace, size_t workspace_bytes, rs_stream_t stream);

/* faiss.normalize_L2 (src/trainer.py:241, app/recommendation_service.py:70): out[r] = x[r] /
 * ||x[r]||_2 for rows with a non-zero norm (x * (1/sqrt(sum x^2))), others copied; out may
 * alias x. */
int rs_l2_normalize_rows_f32(const float* x, int64_t n, int64_t D, float* out, rs_stream_t stream);

/* ---- input pipeline -------------------------------------------------------
 * Replaces ds.shuffle(50000) of make_ds (src/trainer.py:115-116): the epoch's element order under
 * tf.data's shuffle-buffer process (a buffer of buffer_size elements; each output is a uniformly
 * drawn slot, refilled with the next input element; the buffer drains once the input is out).
 * Output i is input j with j < i + buffer_size; every index in [0, n) appears once; buffer_size
 * >= n is a full uniform shuffle, 1 the identity. Deterministic in (seed, epoch). HOST memory
 * (order[n]); no GPU work. */
int rs_shuffle_buffer_order_i64(int64_t n, int64_t buffer_size, uint64_t seed, uint64_t epoch, int64_t* order);

#ifdef __cplusplus
}
#endif
#endif /* RECSYS_HIP_H */
