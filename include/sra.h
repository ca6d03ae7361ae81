/*
 * sra.h — C ABI of the MI355X-native Byzantine-robust gradient-reduction
 * engine ("SRA": secure robust aggregation), libsra.so.
 *
 * Each entry point replaces one aggregator of the reference
 * (wanglun1996/secure-robust-federated-learning @ v1); the reference symbol it
 * replaces is cited per function.  The reference is pure Python, so the
 * "binding a maintainer would add" is the ctypes layer in
 * secure-robust-federated-learning_amd/_lib.py.
 *
 * Conventions (all entry points):
 *  - X is a device pointer to an N x d float32 matrix, client-major: client i's
 *    flattened update is X[i*ldx .. i*ldx+d).  ldx >= d (elements).
 *  - All pointers are device pointers owned by the caller; nothing is
 *    allocated on the hot path (workspace comes from the *_workspace query).
 *  - Calls are asynchronous and ordered on `stream` (a hipStream_t; NULL = the
 *    legacy default stream).
 *  - Return 0 (SRA_OK) or a negative sra_status; sra_last_error() gives a
 *    thread-local message.  No global mutable state.
 */
#ifndef SRA_H_
#define SRA_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  SRA_OK = 0,
  SRA_ERR_ARG = -1,          /* bad pointer / size / parameter       -> ValueError   */
  SRA_ERR_SHAPE = -2,        /* inconsistent N, d, ldx              -> ValueError   */
  SRA_ERR_UNSUPPORTED = -3,  /* N or mode outside what is built     -> NotImplementedError */
  SRA_ERR_EMPTY_BUCKET = -4, /* MoM bucket with no member           -> ValueError   */
  SRA_ERR_THETA = -5,        /* Bulyan theta <= 0                    -> IndexError   */
  SRA_ERR_HIP = -6,          /* HIP runtime error                    -> RuntimeError */
  SRA_ERR_WORKSPACE = -7,    /* workspace too small                  -> ValueError   */
  SRA_ERR_INFEASIBLE = -8    /* no feasible capped-simplex projection-> TypeError    */
} sra_status;

/* Thread-local text of the last error on this thread. */
const char* sra_last_error(void);

/* ABI version (major*10000 + minor*100 + patch). */
int sra_version(void);

/* Largest client count served by the register-resident k-select path
 * (larger N goes through the LDS path). */
int sra_max_register_clients(void);

/* Number of device row indices (Krum / Bulyan selections, row gathers) found
 * outside their matrix since the last reset; each was clamped to the matrix.
 * Non-zero means a bug (the GPU tests assert 0).  Synchronous: waits for the
 * device.  A library built with -DSRA_DEVICE_ASSERT traps instead. */
int sra_row_fault_count(int32_t reset, uint32_t* count);

/* ------------------------------------------------------------------------ */
/* Coordinate-wise aggregators (k1: per-coordinate k-select)                 */
/* ------------------------------------------------------------------------ */

/* out[j] = mean_i X[i, j]: sequential fp32 sum over clients in order, then /N.
 * Replaces the inline `--agg average` of src/simulate.py:235-244
 * (np.average(axis=0)). */
int sra_average_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* out, void* stream);

/* Coordinate-wise median, numpy semantics: even N -> (s[N/2-1]+s[N/2])/2 in
 * fp32, odd N -> s[(N-1)/2]; any NaN in a column -> NaN.
 * Replaces robust_estimator.median (src/robust_estimator.py:220-221). */
int sra_median_f32(const float* X, int64_t n, int64_t d, int64_t ldx, float* out, void* stream);

/* Coordinate-wise trimmed mean: sort each column (NaN last), drop b values at
 * each end, sum the rest sequentially in ascending order in fp32, divide by
 * N-2b.  Bit-exact with robust_estimator.trimmed_mean
 * (src/robust_estimator.py:223-232) for d > 1; b = int(N*beta) is computed by
 * the caller exactly as the reference does. */
int sra_trimmed_mean_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t b, float* out,
                         void* stream);


/* ------------------------------------------------------------------------ */
/* Pairwise L2 / Krum (k2 MFMA Gram + k3 client-space scoring)               */
/* ------------------------------------------------------------------------ */

/* Workspace for sra_gram_f32 (partial-Gram slab), in bytes. */
int sra_gram_workspace_bytes(int64_t n, int64_t d, size_t* bytes);

/* G (n x n, fp64, row-major, symmetric) = centred Gram of the clients:
 * G_ij = sum_k (X[i,k] - mu_k)(X[j,k] - mu_k) with mu a per-coordinate shift,
 * so ||x_i - x_j||^2 = G_ii + G_jj - 2 G_ij.  bf16 MFMA on an exact three-way
 * split of every centred fp32 value (six products per term: fp32-product
 * accuracy), fp32 partials per k-group, fp64 reduction.
 * 1 <= n <= 8192 (n > 256: one launch per pair of 128-client blocks, all
 * centred by the fp32 mean over the n clients).  Feeds krum_
 * (src/robust_estimator.py:234-244). */
int sra_gram_f32(const float* X, int64_t n, int64_t d, int64_t ldx, double* G, void* ws, size_t ws_bytes,
                 void* stream);

/* Workspace for sra_krum_select_f32, in bytes. */
int sra_krum_workspace_bytes(int64_t n, int64_t d, size_t* bytes);

/* `rounds` Krum selections with f fixed over a shrinking set:
 *  round t scores every remaining client by the numpy-pairwise fp32 sum of
 *  its (n_remaining - f - 2) smallest distances (Python slice semantics),
 *  picks the first minimum and removes it; order[t] = its client index.
 *  rounds = 1 is robust_estimator.krum (src/robust_estimator.py:246-249);
 *  rounds = theta is the selection of bulyan(aggsubfunc='krum') (:286-296).
 *  scores (optional, n floats) receive round 0's scores = krum_'s metric.
 *  Distances: from the centred Gram for d > 1024; for d <= 1024, or data with
 *  a NaN / inf, each pair's fp32 difference squared and summed in fp64 (the
 *  reference's np.linalg.norm of the difference, :242).  1 <= n <= 8192
 *  (n > 512: the rounds compact each row through a global scratch). */
int sra_krum_select_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t f, int32_t rounds,
                        int32_t* order, float* scores, void* ws, size_t ws_bytes, void* stream);

/* Workspace for sra_krum_from_gram, in bytes (12*n*n, plus the rounds'
 * scratch for n > 512). */
int sra_krum_from_gram_workspace_bytes(int64_t n, size_t* bytes);

/* Same selection from a precomputed Gram G (e.g. summed over GPUs);
 * ws from sra_krum_from_gram_workspace_bytes. */
int sra_krum_from_gram(const double* G, int64_t n, int32_t f, int32_t rounds, int32_t* order, float* scores,
                       void* ws, size_t ws_bytes, void* stream);

/* Exact per-pair route over a column-sharded layer: the
 * reference's np.linalg.norm(sample - sample_) (src/robust_estimator.py:242)
 * squared is a sum over columns, so each rank's shard contributes
 *   acc[i*nb + j] (i < j) = sum_k fp32(x_ik - x_jk)^2   (fp64)
 * over its columns, class-coded in place: NaN when any term is NaN, else +inf
 * when any is inf (fp64 addition of the ranks' partials keeps that class
 * rule).  Rows are the n clients (bucket_size 1) or the means of consecutive
 * buckets of bucket_size clients (np.mean order, mom_krum's rows); nb =
 * ceil(n / bucket_size) <= 8192.  acc is nb x nb fp64 (only i < j written,
 * the rest zeroed); ws from sra_krum_pair_sq_workspace_bytes. */
int sra_krum_pair_sq_workspace_bytes(int64_t n, int32_t bucket_size, size_t* bytes);
int sra_krum_pair_sq_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t bucket_size, double* acc,
                         void* ws, size_t ws_bytes, void* stream);

/* The selection of sra_krum_from_gram from the summed class-coded pair sums
 * of sra_krum_pair_sq_f32 (distance = sqrt(fp32(acc)), NaN sorted last in
 * each row, first minimum score): the unsharded exact route's scoring. */
int sra_krum_from_pairs_workspace_bytes(int64_t n, size_t* bytes);
int sra_krum_from_pairs(const double* acc, int64_t n, int32_t f, int32_t rounds, int32_t* order, float* scores,
                        void* ws, size_t ws_bytes, void* stream);

/* out[r, :] = X[rows[r], :] for r < nrows (rows is a device int32 array of
 * indices into the n rows of X; an index outside [0, n) is clamped and counted,
 * see sra_row_fault_count). */
int sra_gather_rows_f32(const float* X, int64_t n, int64_t d, int64_t ldx, const int32_t* rows, int32_t nrows,
                        float* out, int64_t ldo, void* stream);

/* ------------------------------------------------------------------------ */
/* Median-of-means bucketing (k5)                                            */
/* ------------------------------------------------------------------------ */

/* out[b, :] = mean of X rows [b*bucket_size, min((b+1)*bucket_size, n)),
 * sequential fp32 sum / count, b < nbuckets.  SRA_ERR_EMPTY_BUCKET if a bucket
 * would be empty (the reference then raises ValueError).
 * Replaces the bucketing of src/robust_estimator.py:135-140, 210-216, 251-256. */
int sra_bucket_mean_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t bucket_size, int32_t nbuckets,
                        float* out, int64_t ldo, void* stream);

/* mom_krum (src/robust_estimator.py:250-256) without the bucket matrix: the
 * Gram of the nb = ceil(n / bucket_size) bucket means is formed straight from
 * the client rows (each read once), Krum picks over the buckets as
 * sra_krum_select_f32 with rounds = 1 (order[0] = the bucket), and out (d
 * floats) receives that bucket's mean, bit for bit sra_bucket_mean_f32's row.
 * 1 <= bucket_size <= 4 and nb <= 192, else SRA_ERR_UNSUPPORTED (the caller
 * then takes sra_bucket_mean_f32 + sra_krum_select_f32). */
/* The centred Gram (nb x nb fp64, nb = ceil(n / bucket_size)) of the bucket
 * means of sra_bucket_mean_f32, formed from the client rows without writing
 * the means (mom_krum's distances; per column shard, summed by all-reduce for
 * a sharded mom_krum).  Workspace: sra_gram_workspace_bytes(nb, d).  1 <=
 * bucket_size <= 4, nb <= 192. */
int sra_gram_buckets_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t bucket_size, double* G,
                         void* ws, size_t ws_bytes, void* stream);
int sra_mom_krum_workspace_bytes(int64_t n, int64_t d, int32_t bucket_size, size_t* bytes);
int sra_mom_krum_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t f, int32_t bucket_size,
                     int32_t* order, float* out, void* ws, size_t ws_bytes, void* stream);


/* ------------------------------------------------------------------------ */
/* Bulyan (k4)                                                               */
/* ------------------------------------------------------------------------ */

/* Workspace for sra_bulyan_f32, in bytes (mode: 0 krum, 1 median, 2 trimmedmean). */
int sra_bulyan_workspace_bytes(int64_t n, int64_t d, int32_t f, int32_t mode, size_t* bytes);

/* robust_estimator.bulyan (src/robust_estimator.py:277-332): theta = n - 2f
 * selection rounds (mode 0: Krum with f fixed, the chosen clients; 1/2: the
 * coordinate-wise median / trimmed mean (beta 0.1) of the remaining clients,
 * whose nearest client is removed), then the per-coordinate Bulyan median
 * with numpy's fp64 pairwise tie-break and the mean of the beta = theta - 2f
 * nearest values.  out: d float64 values.  selected (optional, theta int32):
 * the chosen clients in krum mode.  status (optional, one int32, written
 * stream-ordered): 1 if a median / trimmed-mean round found no strict
 * minimum distance -- every distance NaN / inf, where the reference's
 * `assert min_index != None` (:308, :321) raises -- else 0.  theta <= 0 ->
 * SRA_ERR_THETA.  1 <= n <= 8192 (more than 128 remaining clients: LDS k-select + distance
 * passes per round, the distances in groups of 1024 rows above 512; theta > 128: an
 * LDS-sorted per-coordinate stage, 64 coordinates per tile up to theta = 512, fewer above). */
int sra_bulyan_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t f, int32_t mode, double* out,
                   int32_t* selected, int32_t* status, void* ws, size_t ws_bytes, void* stream);


/* One selection round of Bulyan's median / trimmed-mean modes
 * (src/robust_estimator.py:297-322) over the listed clients rows[0, nr) of an
 * N x d block (a whole layer or a column shard of it): agg (d floats) = the
 * coordinate-wise median (mode 1) or trimmed mean (mode 2; dba != 0: the DBA
 * harness's lower median, src/DBA/helper.py:1025) of the listed rows; dist[r]
 * (nr doubles) = squared L2 distance of listed row r to agg over this block's
 * columns.  Column shards' dist vectors sum to the full distance (up to fp64
 * rounding: the per-tile partials are associated differently).  N <= 8192
 * (rounds with more than 128 listed rows take an LDS k-select + distance pass);
 * workspace from sra_bulyan_round_workspace_bytes (sized by the block's d). */
int sra_bulyan_round_workspace_bytes(int64_t n, int64_t d, size_t* bytes);
int sra_bulyan_round_f32(const float* X, int64_t n, int64_t d, int64_t ldx, const int32_t* rows, int32_t nr,
                         int32_t mode, int32_t dba, float* agg, double* dist, void* ws, size_t ws_bytes,
                         void* stream);
/* The round's pick: the first strict minimum of dist (NaN never chosen; all
 * NaN / inf -> *status = 1, the reference's AssertionError) is removed from
 * rows[0, nr) into rows_next[0, nr - 1), order preserved. */
int sra_bulyan_pick(const double* dist, const int32_t* rows, int32_t nr, int32_t* rows_next, int32_t* status,
                    void* stream);

/* The per-coordinate Bulyan stage alone on theta float32 rows (row i = the
 * i-th selected vector in selection order, row stride lds): out[j] (float64)
 * as sra_bulyan_f32's final stage computes it for robust_estimator.py:324-330
 * (bulyan_one_coordinate over np_grads[:, j], beta = theta - 2f, Python slice
 * semantics for beta < 0).  1 <= theta <= 8192; workspace from
 * sra_bulyan_stage_workspace_bytes (8 d bytes plus a few hundred). */
int sra_bulyan_stage_workspace_bytes(int64_t theta, int64_t d, size_t* bytes);
int sra_bulyan_stage_f32(const float* S, int64_t theta, int64_t d, int64_t lds, int32_t beta, double* out,
                         void* ws, size_t ws_bytes, void* stream);

/* The per-coordinate Bulyan stage on float64 values, any input order:
 * robust_estimator.bulyan_median (src/robust_estimator.py:259-270) and
 * bulyan_one_coordinate (:272-275) for every column of the theta x d matrix A
 * (row i = the i-th selected value, row stride lda).  median_index[j]
 * (optional) = np.argmin of the pairwise-summed distance rows (first NaN if
 * any); median_row (optional, theta x d, row stride ldr) = that distance row;
 * out[j] = mean of arr[argsort(row)[:beta]] (Python slice semantics; equal
 * distances take the smaller value first).  1 <= theta <= 8192. */
int sra_bulyan_coordinate_f64(const double* A, int64_t theta, int64_t d, int64_t lda, int32_t beta, double* out,
                              int64_t* median_index, double* median_row, int64_t ldr, void* stream);

/* ------------------------------------------------------------------------ */
/* Spectral filters (k6)                                                     */
/* ------------------------------------------------------------------------ */

/* Workspace for sra_filter_f32 / sra_filter_debug_f32, in bytes: the n x n
 * (padded 128 x 128) fp64 Gram, weights and flags of up to 8192 chunks at a
 * time (longer layers are processed in batches of 8192 chunks; 256 chunks
 * of n x n for n > 128). */
int sra_filter_workspace_bytes(int64_t n, int64_t d, int32_t itv, size_t* bytes);

/* mode 0: robust_estimator.filterL2 (src/robust_estimator.py:144-208);
 * mode 1: robust_estimator.ex_noregret (src/robust_estimator.py:42-133).
 * The layer (n x d) is cut into itv-wide chunks (last one partial); each chunk
 * is filtered in client space from its centred fp64-MFMA Gram (top eigenpair
 * by Lanczos, fp64).  out: d float64 values.  1 <= n <= 1024 (n > 128: the
 * Gram in global memory, a 1024-thread re-orthogonalising solver per chunk,
 * two threads per client row up to n = 512, one above).
 * status: two device int32, zeroed by the caller.  ex_noregret whose
 * capped-simplex projection has no feasible candidate (projected_c = None,
 * robust_estimator.py:99) continues like the reference: the next iteration
 * uses weights=None; status[0] = 2 when that iteration does not exit early
 * (the reference then fails with TypeError at :75); otherwise -- or when it
 * happens at the last iteration (:101) -- the chunk's result is the plain fp32
 * mean of the kept clients, and status[1] counts such chunks.  ex_noregret with ceil(eps*n) = 0 or fewer than 2 clients left
 * after the Krum pre-filter -> SRA_ERR_ARG (the reference raises ValueError). */
int sra_filter_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv, double eps,
                   double sigma, double expansion, double* out, int32_t* status, void* ws, size_t ws_bytes,
                   void* stream);

/* As sra_filter_f32, and records every chunk's discrete decisions into trace
 * (device int32, nchunks rows of 1 + 2 * H int32, H = max(n, 128), i.e.
 * SRA_FILTER_TRACE_STRIDE for n <= 128; replaces nothing in the
 * reference -- it exposes what robust_estimator.py:163-174 / :49-51, :71-99
 * decide, so tests can pin them):
 *   [0]            iterations completed (< T when the early exit fired)
 *   [1 + it]       filterL2: the client removed at iteration it (argmax tau,
 *                  first index, original numbering); ex_noregret: how many
 *                  weights the kept KL-projection candidate caps
 *   [1 + H + i]    1 if client i is active at the end (filterL2: not removed;
 *                  ex_noregret: kept by the Krum pre-filter), else 0
 * Unused decision slots are left untouched. */
#define SRA_FILTER_TRACE_STRIDE (1 + 2 * 128)
int sra_filter_trace_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv, double eps,
                         double sigma, double expansion, double* out, int32_t* status, int32_t* trace, void* ws,
                         size_t ws_bytes, void* stream);

/* Diagnostics variant: as sra_filter_f32, and additionally writes chunk 0's
 * centred Gram (128 x 128 fp64, row-major, zero-padded) followed by one record
 * of 144 doubles per filter iteration (weights before the update [128], top
 * eigenvalue, Lanczos steps, Ritz residual, tridiagonal checks, active
 * clients, w'Gw, restarts, second Gram-Schmidt passes, cycles) into dbg, which
 * must hold SRA_FILTER_DEBUG_DOUBLES doubles. */
#define SRA_FILTER_DEBUG_DOUBLES (128 * 128 + 256 * 144)
int sra_filter_debug_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv,
                         double eps, double sigma, double expansion, double* out, int32_t* status, double* dbg,
                         void* ws, size_t ws_bytes, void* stream);

/* Workspace for sra_mom_filter_f32, in bytes (nbuckets <= 128). */
int sra_mom_filter_workspace_bytes(int64_t nbuckets, int64_t d, int32_t itv, size_t* bytes);

/* The median-of-means forms in one call: mode 0 robust_estimator.mom_filterL2
 * (src/robust_estimator.py:210-218), mode 1 mom_ex_noregret (:135-142).  X
 * holds the n clients; filtered row r is the np.mean of clients
 * [r * bucket_size, min((r + 1) * bucket_size, n)), formed inside the chunk-Gram
 * loads (a sequential fp32 sum over the bucket's clients / their count, the
 * bits sra_bucket_mean_f32 writes) -- no separate bucket-mean pass, but each
 * batch's bucket rows (nbuckets x min(chunks, 16384) x itv floats) are written
 * once to the workspace for the chunk means: up to d = 1.6e7 at itv 1000 that
 * is the whole bucket matrix (6.4 GB at C5), which
 * sra_mom_filter_workspace_bytes reports.
 * Results equal sra_bucket_mean_f32 followed by sra_filter_f32 bit for bit.
 * nbuckets <= 128 (SRA_ERR_UNSUPPORTED above: run the two calls instead); an
 * empty trailing bucket -> SRA_ERR_EMPTY_BUCKET (the reference's ValueError). */
int sra_mom_filter_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t mode, int32_t itv,
                       int32_t bucket_size, int32_t nbuckets, double eps, double sigma, double expansion,
                       double* out, int32_t* status, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ */
/* Cross-layer-norm clipping (k7): the stateful inline aggregators           */
/* iclr2022_bucketing (src/simulate.py:335-366) and icml2021_history (:367-388) */
/* ------------------------------------------------------------------------ */

/* out[w, :] = mean of X rows [w*stride, min(w*stride + width, n)) for w < nwin:
 * sequential sum over the window's rows in the input precision, divided by the
 * row count (an empty window gives NaN, like np.average of an empty list).
 * stride = 1, width = perround // buckets are the overlapping windows
 * choices[b : b + perround//buckets] of src/simulate.py:344-351. */
int sra_window_mean_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t stride, int32_t width,
                        int32_t nwin, float* out, int64_t ldo, void* stream);
int sra_window_mean_f64(const double* X, int64_t n, int64_t d, int64_t ldx, int32_t stride, int32_t width,
                        int32_t nwin, double* out, int64_t ldo, void* stream);

/* Workspace for sra_clip_scale_*, in bytes (seg: host array of nseg+1 offsets). */
int sra_clip_workspace_bytes(int64_t k, const int64_t* seg, int32_t nseg, size_t* bytes);

/* Per-row clipping factor against prev (d fp64, device) with the norm taken
 * across all layer segments: sq_r = sum_l ||M[r, seg_l] - prev[seg_l]||^2 (each
 * layer norm squared after the sqrt, in layer order), norm_r = sqrt(sq_r),
 * scale[r] = min(1, tau / norm_r) with Python's min (tau/0 -> 1, NaN -> 1).
 * seg is a HOST array of nseg+1 column offsets (seg[0] = 0, seg[nseg] = d).
 * norm (optional, k doubles) receives norm_r.
 * Replaces simulate.py:352-356 (bucketing) and :374-378 (history). */
int sra_clip_scale_f32(const float* M, int64_t k, int64_t d, int64_t ldm, const double* prev, const int64_t* seg,
                       int32_t nseg, double tau, double* scale, double* norm, void* ws, size_t ws_bytes,
                       void* stream);
int sra_clip_scale_f64(const double* M, int64_t k, int64_t d, int64_t ldm, const double* prev, const int64_t* seg,
                       int32_t nseg, double tau, double* scale, double* norm, void* ws, size_t ws_bytes,
                       void* stream);

/* out[j] = (sum_r (M[r,j] - prev[j]) * scale[r]) / k in fp64, summed sequentially
 * over r (np.average(axis=0) of the clipped rows, simulate.py:358-364 / 380-386).
 * clipped (optional, k x d fp64, row stride ldc) receives the clipped rows -- the
 * arrays icml2021_history stores back into local_grads (simulate.py:380). */
int sra_clipped_mean_f32(const float* M, int64_t k, int64_t d, int64_t ldm, const double* prev, const double* scale,
                         double* clipped, int64_t ldc, double* out, void* stream);
int sra_clipped_mean_f64(const double* M, int64_t k, int64_t d, int64_t ldm, const double* prev, const double* scale,
                         double* clipped, int64_t ldc, double* out, void* stream);

/* ---- k8: attack-side callers of the path (src/attack.py) ---- */

/* attack_krum (attack.py:202-262) for one layer: X holds the layer of ALL m
 * clients (row-major, ldx); mal_mask[m] (device, 1 = malicious) and
 * benign_rows[nbenign] (device, ascending) describe mal_index.  Writes the
 * malicious layer value -lambda * sign(sum of benign rows) (fp64, d), lambda
 * (device scalar) and krum's pick at that lambda.  lambda runs 1, 1/2, ... to the
 * first value below lower_bound, like the reference loop (upper_bound is
 * overwritten to 1.0 there, :237). */
int sra_attack_krum_workspace_bytes(int64_t m, int64_t d, double lower_bound, size_t* bytes);
int sra_attack_krum_f32(const float* X, int64_t m, int64_t d, int64_t ldx, const int32_t* mal_mask,
                        const int32_t* benign_rows, int32_t nbenign, double lower_bound, double* mal_row,
                        double* lam_out, int32_t* chosen_out, void* ws, size_t ws_bytes, void* stream);
/* bulyan_attack_krum (src/attack.py:264-308): the same lambda search with the
 * caller's direction dir (d floats; the reference's attack_vec[param_index]:
 * ones for the target layer, zeros elsewhere) in place of the benign sign.
 * Malicious rows = -lambda * dir (float64).  Workspace as sra_attack_krum_f32. */
int sra_attack_krum_dir_f32(const float* X, int64_t m, int64_t d, int64_t ldx, const int32_t* mal_mask,
                            const int32_t* benign_rows, int32_t nbenign, const float* dir, double lower_bound,
                            double* mal_row, double* lam_out, int32_t* chosen_out, void* ws, size_t ws_bytes,
                            void* stream);

/* Python's `random` stream (MT19937, genrand_uint32) on the device: state_in =
 * random.getstate()[1] as 625 uint32 (624 words + position); writes the nwords
 * tempered outputs and the advanced state (random.setstate continues from it).
 * Replaces the per-element random.uniform draws of attack_trimmedmean
 * (attack.py:184-194). */
int sra_mt19937_words(const uint32_t* state_in, int64_t nwords, uint32_t* words, uint32_t* state_out,
                      void* stream);

/* attack_trimmedmean (attack.py:157-198) over all D parameters: X = all
 * clients' updates (row-major, ldx), benign_rows (device), params = the
 * network's current parameters (D, fp32), words = 2*D outputs of
 * sra_mt19937_words.  Writes the malicious clients' update (fp64, D). */
int sra_attack_trimmedmean_f32(const float* X, int64_t D, int64_t ldx, const int32_t* benign_rows, int32_t nbenign,
                               const float* params, const uint32_t* words, double b, double* mal_row, void* stream);

/* attack_xie (attack.py:362-372) for one layer: out = (-weight * sum of rows[])
 * / nchoices in the input precision, rows = the benign chosen clients. */
int sra_attack_xie_f32(const float* X, int64_t d, int64_t ldx, const int32_t* rows, int32_t nrows, double weight,
                       int64_t nchoices, float* out, void* stream);
int sra_attack_xie_f64(const double* X, int64_t d, int64_t ldx, const int32_t* rows, int32_t nrows, double weight,
                       int64_t nchoices, double* out, void* stream);

/* ---- k9: device-resident client-update store ----
 * The step either side of the aggregation in simulate.py's round loop.  A
 * parameter table describes the network: ptrs[nseg] = device addresses of the
 * contiguous float32 parameter tensors (a device array of uint64), seg[nseg+1]
 * = their offsets in the flat index space (device int64, seg[0] = 0,
 * seg[nseg] = D).  One launch covers the whole network. */

/* flat = concat(params): params_copy (simulate.py:146-148). */
int sra_params_flatten_f32(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D, float* flat,
                           void* stream);
/* row = snapshot - params in fp32 (simulate.py:193-194, numpy's float32 minus
 * after the per-layer D2H), then params = snapshot (the restore, :196-199). */
int sra_record_delta_f32(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D, const float* snapshot,
                         float* row, void* stream);
/* Momentum form (simulate.py:190-191, iclr2022_bucketing / icml2021_history):
 * row = (double) fl32(one_minus_beta * fl32(snapshot - params)) + beta * row,
 * one_minus_beta = float32(1 - beta) as numpy casts the Python scalar; then
 * params = snapshot. */
int sra_record_momentum_f64(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D,
                            const float* snapshot, float one_minus_beta, double beta, double* row, void* stream);
/* params -= agg (simulate.py:400-404): float32 minus for an f32 aggregate; an
 * f64 aggregate is subtracted in fp64 and rounded once to fp32 (torch's
 * p.data.sub_(float64 tensor)). */
int sra_apply_update_f32(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D, const float* agg,
                         void* stream);
int sra_apply_update_f64(const uint64_t* ptrs, const int64_t* seg, int32_t nseg, int64_t D, const double* agg,
                         void* stream);

/* ---- k10: the DBA harness's Helper aggregators (src/DBA/helper.py) ---- */

/* out[j] = s_k of column j (ascending, NaN anywhere -> NaN); k = (n-1)/2 is
 * torch.median's lower median (Helper.median, helper.py:529-569).  n <= 16384
 * (n > 128: an LDS bitonic sort per coordinate tile). */
int sra_order_stat_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t k, float* out, void* stream);
/* out = (sequential fp32 sum of the rows) / divisor, correctly rounded:
 * Helper.mom_krum's aliased bucket (helper.py:857-863, divisor count + 1) and
 * Helper.sharding's shard average (helper.py:1155-1164, divisor count). */
int sra_rows_sum_div_f32(const float* X, int64_t rows, int64_t d, int64_t ldx, float divisor, float* out,
                         void* stream);
/* out = sum_r fl32(w[r] * X[r]) accumulated in row order from 0 in fp32, no
 * FMA (Helper.weighted_average_oracle, helper.py:1199-1221); w: device fp32. */
int sra_weighted_sum_f32(const float* X, int64_t rows, int64_t d, int64_t ldx, const float* w, float* out,
                         void* stream);
/* As sra_clip_scale_f32 with the DBA norm rule (Helper.history / bucketing,
 * helper.py:753-759, 803-809): norm = sqrt(norm + ||layer_l - prev_l||^2) after
 * every layer, scale = min(1, tau / norm). */
int sra_clip_scale_running_f32(const float* M, int64_t k, int64_t d, int64_t ldm, const double* prev,
                               const int64_t* seg, int32_t nseg, double tau, double* scale, double* norm, void* ws,
                               size_t ws_bytes, void* stream);
/* Helper.bulyan_krum / bulyan_median / bulyan_trimmed_mean (helper.py:942-1137):
 * as sra_bulyan_f32 (same modes, workspace from sra_bulyan_workspace_bytes)
 * with the DBA selection rules -- Krum rounds count the zero self-distance
 * (= Krum with f + 1 over the others; f = 1 is rejected), median rounds take
 * the lower median.  The per-coordinate stage is shared (fp64). */
int sra_bulyan_dba_f32(const float* X, int64_t n, int64_t d, int64_t ldx, int32_t f, int32_t mode, double* out,
                       int32_t* selected, int32_t* status, void* ws, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SRA_H_ */
