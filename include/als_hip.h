/*
 * als_hip.h — C ABI of libals_hip.so, the MI355X (gfx950) ALS hot path.
 *
 * This is the drop-in boundary for the ALS path of
 * amy-leaf/Recommender-System-using-Apache-Spark-MLlib-.  The reference calls
 * the ALS core through pyspark (RecommenderSystem.py:132 import,
 * :148-149 / :163 / :218 `ALS.train`, :150 / :165 / :222 / :232 `predictAll`);
 * the arithmetic behind those calls lives in Apache Spark
 * (`ml/recommendation/ALS.scala`, not vendored).  Each entry point below
 * replaces one upstream routine on that path; the comment names it and the
 * reference call site that reaches it.
 *
 * Conventions
 *  - Every pointer except the `*_host` ones is DEVICE memory owned by the caller.
 *    The library never allocates on a compute call; scratch comes from a
 *    caller-provided workspace sized by the matching *_workspace_bytes().
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *    All compute calls are asynchronous on that stream.
 *  - Factor matrices are row-major fp32 with leading dimension `ld`
 *    (ld % 4 == 0, ld >= k, base 16-byte aligned).  Output factor rows are
 *    written in full: columns [k, ld) are written as zero, and factor inputs
 *    (Y_src of als_solve_half / als_yty) must carry zeros there too.
 *  - Return value: 0 on success, negative ALS_E* code on argument error;
 *    als_last_error() returns a thread-local message for the last failure.
 *  - Dense indices: ids are mapped to dense row numbers in ascending id order
 *    (als_index_build), the device analogue of Spark's sorted InBlock.srcIds.
 */
#ifndef ALS_HIP_H
#define ALS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ALS_ABI_VERSION 6

#define ALS_OK 0
#define ALS_EINVAL (-1)   /* bad argument (shape, null pointer, rank) */
#define ALS_EWORKSPACE (-2) /* workspace too small */
#define ALS_EDEVICE (-3)  /* HIP runtime error (launch failure, no device) */
#define ALS_EUNSUPPORTED (-4)

/* ---- library ---------------------------------------------------------- */
int als_abi_version(void);
const char* als_last_error(void);
/* Number of HIP devices visible (0 on a host without a GPU); never launches work. */
int als_device_count(void);

/* ---- K1: rating-block construction (replaces Spark partitionRatings /
 *      makeBlocks / InBlock / LocalIndexEncoder, reached from ALS.train at
 *      RecommenderSystem.py:148-149) ------------------------------------ */

/* Dense id map.  ids[n] in [0, id_space).  Writes map_out[id_space]
 * (dense index or -1 if the id does not occur), uniq_out[<=id_space]
 * (ascending distinct ids) and *n_uniq_dev (device int32). */
size_t als_index_workspace_bytes(int64_t n, int32_t id_space);
int als_index_build(const int32_t* ids, int64_t n, int32_t id_space,
                    int32_t* map_out, int32_t* uniq_out, int32_t* n_uniq_dev,
                    void* ws, size_t ws_bytes, void* stream);

/* Stable counting sort of a COO rating list by dense row (row = row_map[row_ids[e]]),
 * producing CSR: row_ptr_out[n_rows+1] (int64), col_out[nnz] = col_map[col_ids[e]]
 * and val_out[nnz] in input order within each row (Spark keeps duplicates:
 * each (u,i) occurrence is its own term, Appendix A.1).  nnz < 2^31. */
size_t als_csr_workspace_bytes(int64_t nnz, int32_t n_rows);
int als_csr_build(const int32_t* row_ids, const int32_t* row_map,
                  const int32_t* col_ids, const int32_t* col_map,
                  const float* vals, int64_t nnz, int32_t n_rows,
                  int64_t* row_ptr_out, int32_t* col_out, float* val_out,
                  void* ws, size_t ws_bytes, void* stream);

/* Work schedule for one CSR side: rows with <= chunk ratings ("light") are
 * solved one wavefront each, longest first; heavier rows are split into
 * chunk-sized tasks whose partial normal equations (fp32 sums within a task,
 * stored as those fp32 values) are summed in fp64 and solved in a second launch.  Two-step: count (device int32[3] = n_light, n_heavy,
 * n_chunks) then build into caller buffers sized from those counts. */
size_t als_schedule_workspace_bytes(int32_t n_rows);
int als_schedule_count(const int64_t* row_ptr, int32_t n_rows, int32_t chunk,
                       int32_t* counts_dev, void* stream);
int als_schedule_build(const int64_t* row_ptr, int32_t n_rows, int32_t chunk,
                       int32_t n_light, int32_t n_heavy, int32_t n_chunks,
                       int32_t* light_rows, int32_t* heavy_rows,
                       int32_t* heavy_slot_begin /* n_heavy+1 */,
                       int32_t* chunk_row, int64_t* chunk_begin, int64_t* chunk_end,
                       void* ws, size_t ws_bytes, void* stream);

/* ---- K2/K3: normal equations + Cholesky (replaces Spark computeFactors,
 *      NormalEquation.add (dspr/daxpy), CholeskySolver.solve (dppsv)) ---- */

/* One half-sweep: for every dst row j (all rows of the schedule)
 *   explicit:  A_j = sum_s y_s y_s^T + reg*n_j*I,          b_j = sum_s r_js y_s
 *   implicit:  A_j = YtY + sum_s c1 y_s y_s^T + reg*n+_j*I, b_j = sum_{r>0} (1+c1) y_s,
 *              c1 = alpha*|r|, n+_j = #{r_js > 0}
 * from fp32 factors.  The Gram runs on the f16 matrix cores with every value
 * split into two f16 halves (hi*hi + hi*lo + lo*hi: ~2^-21 relative per product)
 * after a power-of-two scaling set by max |Y_src| over its n_src rows and
 * max |rating|.  Explicit: Y_src is split once per call into a table in the
 * workspace ((n_src + 1) x k_pad words) and the rhs runs on the matrix cores too;
 * implicit: the split follows the per-rating confidence weight, in registers.
 * fp32 sums within a task (the schedule's chunk: engine.chunk_for picks 4096
 * ratings, 16384 for explicit fits at k > 64), fp64 across a heavy row's tasks;
 * solved by a square-root-free block LDL^T (the solution of Spark's Cholesky
 * dppsv) in fp32, stored fp32 into X_dst[row*ld ..].  k <= 128, n_src < 2^31.
 * Parity bar: 1e-4 relative per row against the fp64 restatement of Spark's
 * dspr + dppsv (oracle/); the measured maxima per configuration (ranks 1-128,
 * explicit/implicit, full-size half-sweeps) are in DESIGN.md section 1 and
 * tests/test_gpu_kernels.py / test_gpu_configs.py.  yty_packed (implicit only): lower-packed
 * fp64 k_pad x k_pad Gram from als_yty.  status_dev: device int32, set to
 * (row+1) of a row whose Cholesky pivot was not positive (0 = all rows ok;
 * Spark raises from dppsv in that case).  ws: 16-byte aligned.
 * phases (ALS_PHASE_* bits below; ALS_PHASE_ALL = the normal call): PREP = Y_src
 * prep (max |Y_src|; explicit: the split table), RSCALE = rating scale (max
 * |rating| of this block), LAUNCH1 = heavy-row chunk partials + fused primal
 * light-row gram/solve, DUAL = the dual-path light rows (see n_light_primal),
 * LAUNCH2 = heavy-row reduce + solve, RESCUE = re-solve of the rows that missed
 * the split window (below).  They run in the order PREP, RSCALE, LAUNCH1, DUAL,
 * LAUNCH2, RESCUE; split across calls, issue them in that order on one stream
 * with the same workspace (PREP starts an empty rescue list; RESCUE empties it
 * again, so every LAUNCH1 ... RESCUE sequence needs its RESCUE).  Blocks that share Y_src (row chunks of one half-sweep) may share
 * one PREP: it sits at a fixed workspace offset (size the workspace for the
 * largest n_chunks and n_rows).
 * Split window (explicit): the Gram/rhs split uses one power-of-two scale per
 * launch, so a row whose own factor rows (or ratings) all sit more than ~2^18
 * below the launch maxima would lose precision in the f16 lo halves.  Such a row
 * is detected in its task (max diagonal of its Gram / max |rating| against the
 * window) and re-solved in the RESCUE launch with a scale of its own (fp32 rows
 * split in registers, fp32 rhs), so the 1e-4 bar holds for any magnitude spread.
 * n_light_primal (0 <= n_light_primal <= n_light): the first n_light_primal light
 * rows are solved on the k x k normal equations above; the remaining light rows
 * (the tail of the longest-first light list) must have <= 96 ratings (64 < k <= 128)
 * or <= 32 ratings (32 < k <= 64) and are solved through the equivalent n x n dual
 * system (push-through identity (Y^T Y + lambda n I)^-1 Y^T r =
 * Y^T (Y Y^T + lambda n I)^-1 r), allowed for explicit feedback, 32 < k <= 128,
 * reg > 0 only (a longer row there is reported through status_dev).
 * n_light_primal = n_light keeps every row on the primal path.
 * Two-segment schedules (ABI 6; the sharded engine's pipelined item half-sweep,
 * distributed.py): chunk task c of this call writes partial slot chunk_slot0 + c,
 * and heavy_slot_begin2 (nullable, n_heavy + 1 entries) gives each heavy row a
 * second slot range, summed with the first in LAUNCH2.  A half-sweep whose source
 * rows arrive in two parts then runs as two calls on one workspace: the early
 * segments' chunk partials (PREP over the arrived prefix of Y_src, LAUNCH1,
 * chunk_slot0 = 0), then the late segments' (chunk_slot0 = number of early slots)
 * with LAUNCH2 and RESCUE over every row; the workspace is sized for all slots
 * (the slot region sits before the split table, so the two calls' different n_src
 * leave the early partials in place).  Normal calls pass NULL and 0. */
#define ALS_PHASE_LAUNCH1 1
#define ALS_PHASE_LAUNCH2 2
#define ALS_PHASE_PREP 4
#define ALS_PHASE_RSCALE 8
#define ALS_PHASE_DUAL 16
#define ALS_PHASE_RESCUE 32
#define ALS_PHASE_ALL 63
/* n_rows: rows of the block (n_light + n_heavy; the largest block when shared). */
size_t als_solve_workspace_bytes(int32_t k, int32_t n_chunks, int64_t n_src, int32_t n_rows);
int als_solve_half(const int64_t* row_ptr, const int32_t* col, const float* val,
                   const int32_t* light_rows, int32_t n_light, int32_t n_light_primal,
                   const int32_t* heavy_rows, const int32_t* heavy_slot_begin, int32_t n_heavy,
                   const int32_t* chunk_row, const int64_t* chunk_begin, const int64_t* chunk_end,
                   int32_t n_chunks, const int32_t* heavy_slot_begin2, int32_t chunk_slot0,
                   const float* Y_src, int64_t n_src, float* X_dst, int32_t ld, int32_t k,
                   float reg, int implicit, float alpha, const double* yty_packed,
                   int32_t* status_dev, void* ws, size_t ws_bytes, int phases, void* stream);

/* K2b: YtY = sum over all n rows of Y of y y^T in fp64 (replaces Spark
 * computeYtY's dspr + treeAggregate).  Output: lower-packed fp64, k_pad(k_pad+1)/2
 * entries, k_pad = als_k_pad(k). */
int32_t als_k_pad(int32_t k);
size_t als_yty_workspace_bytes(int64_t n, int32_t k);
int als_yty(const float* Y, int64_t n, int32_t ld, int32_t k, double* yty_packed_out,
            void* ws, size_t ws_bytes, void* stream);

/* ---- K4: predict / RMSE (replaces MatrixFactorizationModel.predict (ddot)
 *      reached from predictAll at RecommenderSystem.py:150,165,222,232, and the
 *      computeError join+reduce at RecommenderSystem.py:103-129) --------- */

/* pred_out[e] = <U[umap[u[e]]], V[imap[i[e]]]> in fp64 over fp32 factors,
 * NaN when either id is unknown (out of map range or map == -1). */
int als_predict(const int32_t* u, const int32_t* i, int64_t n,
                const int32_t* umap, int32_t umap_size, const int32_t* imap, int32_t imap_size,
                const float* U, const float* V, int32_t ld, int32_t k,
                double* pred_out, void* stream);

/* sse_count_out[0] = sum (r - p)^2 over pairs whose ids are both known,
 * sse_count_out[1] = number of such pairs (inner-join semantics of
 * computeError).  Deterministic (fixed-order fp64 reduction). */
size_t als_rmse_workspace_bytes(int64_t n);
int als_rmse_partial(const int32_t* u, const int32_t* i, const float* r, int64_t n,
                     const int32_t* umap, int32_t umap_size, const int32_t* imap, int32_t imap_size,
                     const float* U, const float* V, int32_t ld, int32_t k,
                     double* sse_count_out, void* ws, size_t ws_bytes, void* stream);

/* ---- K5: recommendForAll (replaces ALSModel.recommendForAll: blockify +
 *      sgemm + bounded priority queue; reference equivalent is the
 *      predictAll + takeOrdered(20) flow at RecommenderSystem.py:229-247) -- */

/* For each of the n_q query rows of Q, the `top` rows of V with the largest
 * score <q, v>, ordered by score descending then index ascending.
 * idx_out[n_q*top] (dense row index of V, -1 when n_v < top), score_out[n_q*top].
 * Scores: fp32-grade products on the f16 matrix cores (q and v split into f16
 * hi + lo after power-of-two scaling, ~2^-21 relative to |q||v|) for every k and
 * top: V is swept with hi.hi alone against the row's k-th score minus a proven
 * bound on the dropped terms, and blocks past it get the full hi.hi + hi.lo + lo.hi
 * score, so every listed pair carries its exact split score.  Lists: registers of
 * one owner lane for top <= 16; for top <= 128 the running top scores in four-lane
 * ("quad") register lists and every key reaching the row's k-th score in a per-row
 * log in the workspace, from which the exact top keys are selected; sorted LDS lists
 * above.  Rows of V holding NaN score NaN and are never listed.
 * k <= 128, top <= 256.  The n_q x n_v score matrix is never materialised.
 * Workspace (16-byte aligned): scale words, the hi and lo f16 planes of V in sweep
 * (decreasing norm) order, the order, bucket counts, the scaled row norms and, for
 * 16 < top <= 128, the key logs (1,024 keys per query row of up to 4,096 x 128 rows). */
size_t als_topk_workspace_bytes(int64_t n_q, int64_t n_v, int32_t k, int32_t top);
int als_topk(const float* Q, int64_t n_q, const float* V, int64_t n_v,
             int32_t ld, int32_t k, int32_t top,
             int32_t* idx_out, float* score_out, void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ALS_HIP_H */
