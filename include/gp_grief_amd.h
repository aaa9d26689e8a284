/*
 * gp_grief_amd -- C ABI of the MI355X (gfx950) Kronecker / GRIEF GP hot path.
 *
 * The reference (scwolof/gp_grief) has no native layer: its drop-in surface is
 * the Python API.  Each entry point below names the reference routine whose
 * arithmetic it replaces (paths relative to the reference checkout).  The
 * Python host mirror (the gp_grief_amd package) binds these with ctypes; a C or cgo
 * caller binds them as-is.
 *
 * Conventions
 *   - every function returns an int status: GG_OK (0) or a negative code;
 *     gg_last_error() returns the thread's last message;
 *   - pointers named *_dev are device (HBM) pointers, *_host host pointers;
 *   - vectors are contiguous float64, C-order over the Kronecker factor list
 *     (factor 0 slowest) exactly like the reference's (N,1) column vectors;
 *   - `stream` is a hipStream_t (NULL = default stream); calls only enqueue
 *     work unless documented as synchronising;
 *   - handles are not thread-safe; one handle = one device.
 */
#ifndef GP_GRIEF_AMD_H
#define GP_GRIEF_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GG_ABI_VERSION 1

#define GG_OK 0
#define GG_ERR_VALUE (-1)   /* bad shape / argument      -> ValueError            */
#define GG_ERR_LINALG (-2)  /* not SPD / non-finite       -> numpy.linalg.LinAlgError */
#define GG_ERR_RUNTIME (-3) /* HIP / RCCL / allocation    -> RuntimeError          */
#define GG_ERR_ASSERT (-4)  /* structural precondition    -> AssertionError        */

typedef void* gg_stream; /* hipStream_t */
typedef struct gg_kron gg_kron;
typedef struct gg_cg gg_cg;

/* ------------------------------------------------------------------ runtime */
int gg_abi_version(void);
int gg_last_error(char* buf, size_t len);
/* The library's GG_* environment switches (kernel-variant A/B knobs and
 * diagnostics) are read from a process snapshot, never on a launch path: taken
 * at the first use and again at every gg_kron_create and gg_cg_work_elems (so
 * a handle latches the environment it was made in); gg_knobs_reload re-takes
 * it for the handle-free entry points (dense / GRIEF / eigen).  No reference
 * counterpart (the reference has no native code).                           */
int gg_knobs_reload(void);
int gg_set_device(int device);
int gg_device_synchronize(void);

/* --------------------------------------------------- Kronecker operator (P1)
 * KronMatrix(K, sym)                    gp_grief/tensors/kron_matrix.py:19-42
 * factors_host[k] is a rows[k] x cols[k] row-major float64 matrix.  The handle
 * copies them to HBM in MFMA B-operand fragment order (for K and K^T).      */
int gg_kron_create(int d, const int64_t* rows, const int64_t* cols,
                   const double* const* factors_host, gg_kron** out);
int gg_kron_destroy(gg_kron* K);
/* n_out / n_in: operator shape (transposed if transpose != 0); work_elems:
 * float64 elements of the `work_dev` scratch gg_kron_matvec needs.          */
int gg_kron_shape(const gg_kron* K, int transpose, int64_t* n_out, int64_t* n_in,
                  int64_t* work_elems);
/* Bit k of *mask is set when factor k of the operator (of K^T if transpose)
 * is applied through the centrosymmetric even/odd split: square factors with
 * max |F - J F J| <= 16 eps max |F| (J = index reversal; every stationary
 * kernel on an evenly spaced grid), m >= GG_KRON_FOLD_MIN (default 48),
 * unless GG_KRON_FOLD=0 at gg_kron_create.  Half the MFMA work of the dense
 * factor, same result up to rounding.  No
 * reference counterpart: an execution detail of kron_matrix.py:52-97.     */
int gg_kron_fold_mask(const gg_kron* K, int transpose, int64_t* mask);

/* y = (K_0 (x) ... (x) K_{d-1})^{T?} x + shift * x
 * KronMatrix.kronvec_prod / __mul__ / .T     kron_matrix.py:52-102, 203-213
 * (shift != 0 needs a square operator; x and y must not alias).            */
int gg_kron_matvec(const gg_kron* K, int transpose, const double* x_dev, double* y_dev,
                   double shift, double* work_dev, gg_stream stream);
/* reps back-to-back gg_kron_matvec calls with HIP events around every mode
 * product on the stream (synchronising): launch_ms_host[k] (d entries) is the
 * summed time of position k over the reps, *total_ms_host the event time of
 * all reps.  Measurement entry (bench.py's isolated K*x leg).              */
int gg_kron_matvec_timed(const gg_kron* K, int transpose, const double* x_dev, double* y_dev,
                         double shift, double* work_dev, int reps, double* launch_ms_host,
                         double* total_ms_host, gg_stream stream);

/* The parity-block basis of a centrosymmetric operator: with
 * every factor square, of even order m_k = 2 h_k and centrosymmetric (J F J =
 * F: every stationary kernel on an evenly spaced grid), the orthogonal change
 * of basis P (per axis u_i = (x_i + x_{m-1-i}) / sqrt 2, v_i = (x_i -
 * x_{m-1-i}) / sqrt 2) makes the operator block diagonal over the 2^d parity
 * patterns, each block a Kronecker product of h_k x h_k matrices
 * S = F[j][i] + F[j][m-1-i], T = F[j][i] - F[j][m-1-i].  Block layout: block
 * B = sum_k beta_k 2^{d-1-k} (slowest) of prod h_k elements, C order over the
 * slab index (i_0 .. i_{d-3}) inside; a slab (the innermost two axes, h x h)
 * k-step tiled: element (i, a) at (a / 4) 4 h + 4 i + a % 4 (round 5: each
 * 4-column group contiguous, the unit the pair launch's GEMM 1 contracts).
 * A matvec there is d - 1 launches (the last two axes of a block share one
 * launch): the CG (gg_cg_*) runs in this basis by default when it exists
 * (gg_cg_set_basis), folding b at start and unfolding x at every close.
 * Existence: 2 <= d <= 6, h_{d-2} = h_{d-1} <= 100, every h <= 112
 * (GG_KRON_BLOCK=0 at gg_kron_create disables it).  The two innermost axes
 * of the layout have extent hp = 16 TF + 4 >= h (TF in 1..6: the pair
 * kernels' slab shapes); where h is not of that form (m = 64, 96, 128 ...,
 * round 6) the positions past h are zero padding -- *n, the block layout's
 * length, is then 2^d prod(h_k) (hp / h)^2 > the grid's n.  The CG and the
 * Lanczos probe take the block basis by default on one GPU where it is
 * unpadded (padded slabs measured slower than the grid basis there); the
 * block-sharded CG wherever it exists (no exchange between ranks).  No reference counterpart: an execution detail of
 * kron_matrix.py:52-97.                                                     */
int gg_kron_block_info(const gg_kron* K, int* available, int64_t* n, int* launches);
/* y = P x (inverse: x = P^T y, the unfold); x, y distinct: the grid vector
 * (the operator's n) and the block-layout vector (gg_kron_block_info's n).  */
int gg_kron_block_fold(const gg_kron* K, int inverse, const double* x_dev, double* y_dev,
                       gg_stream stream);
/* y = (P K P^T + shift I) x in the block layout; work_dev: n (the block layout's) doubles (d >= 3).
 * The operator of kron_matrix.py:52-97 in the parity-block basis.           */
int gg_kron_block_matvec(const gg_kron* K, const double* x_dev, double* y_dev, double shift,
                         double* work_dev, gg_stream stream);
/* A block range [blk0, blk0 + nblk) of the block layout (a rank of the
 * block-sharded CG: rank g of G = 2^K ranks owns blocks g 2^d / G ..): the
 * forward fold writes those blocks only (y: nblk * n / 2^d doubles, x the full
 * grid vector); the inverse reads them (y's other blocks count as 0) and
 * writes their contribution to every element of the grid vector y -- summed
 * over the ranks, P^T of the whole block vector.                           */
int gg_kron_block_fold_range(const gg_kron* K, int inverse, const double* x_dev, double* y_dev,
                             int64_t blk0, int64_t nblk, gg_stream stream);
/* y = (P K P^T + shift I) x on blocks [blk0, blk0 + nblk) (x, y hold them). */
int gg_kron_block_matvec_range(const gg_kron* K, const double* x_dev, double* y_dev,
                               double shift, double* work_dev, int64_t blk0, int64_t nblk,
                               gg_stream stream);
/* reps of gg_kron_block_matvec with HIP events around each of its d - 1
 * launches (synchronising; as gg_kron_matvec_timed).                       */
int gg_kron_block_matvec_timed(const gg_kron* K, const double* x_dev, double* y_dev,
                               double shift, double* work_dev, int reps, double* launch_ms_host,
                               double* total_ms_host, gg_stream stream);

/* y = x / (prod_k lam_k[i_k] + shift), the eigenvalue product decoded from
 * the flat index on the fly (never expanded).  solve_schur's divide,
 * kron_matrix.py:349-350.  lam_dev: concatenated per-factor eigenvalues.   */
int gg_kron_diag_scale(int d, const int64_t* m, const double* lam_dev, double shift,
                       int mode, const double* x_dev, double* y_dev, gg_stream stream);
#define GG_DIAG_DIVIDE 0   /* y = x / (t + shift)            */
#define GG_DIAG_POSTVAR 1  /* y = t * shift / (t + shift)    (x unused) */
#define GG_DIAG_MULTIPLY 2 /* y = x * (t + shift)            */

/* sum_i log(prod_k lam_k[i_k] + shift) over the whole grid (synchronising).
 * Shifted generalisation of KronMatrix.log_det, kron_matrix.py:466-474.     */
int gg_kron_logdet_shifted(int d, const int64_t* m, const double* lam_dev, double shift,
                           double* out_host, gg_stream stream);

/* ------------------------------------------------- vector primitives (CG ops) */
int gg_dot(const double* x_dev, const double* y_dev, int64_t n, double* out_host,
           gg_stream stream); /* synchronising */
int gg_axpby(double a, const double* x_dev, double b, double* y_dev, int64_t n,
             gg_stream stream); /* y = a x + b y */
/* A[i][:] *= w[i] (mode 0), /= w[i] (mode 1), or A = A*A elementwise (mode 2). */
int gg_scale_rows(double* A_dev, int64_t rows, int64_t cols, const double* w_dev, int mode,
                  gg_stream stream);
/* y = x / (t + shift) for an explicit eigenvalue vector t (solve_schur with an
 * expanded t, kron_matrix.py:349-350).                                        */
int gg_diag_divide(const double* t_dev, double shift, const double* x_dev, double* y_dev,
                   int64_t n, gg_stream stream);

/* ------------------------------------------------------------- CG (P1 solve)
 * Unpreconditioned CG on (K + shift I) x = b, x0 = 0, the recurrence of
 * scipy.sparse.linalg.cg (the reference's solver_counter, linalg.py:53-71, is
 * its iteration callback).  All scalars stay on the device; the host polls
 * convergence every `check_every` iterations.  work_dev: gg_cg_work_elems.
 * Two recurrences (gg_cg_set_recurrence, before gg_cg_start):
 *   fused (1, the default when d >= 2): every vector update rides on a mode
 *     product; beta from the exact expansion of |r - alpha q|^2 (the true r.r
 *     drives the stopping test and alpha) -- same iterates as scipy's up to
 *     rounding;
 *   textbook (0): scipy's operation order (separate x / r update pass).
 * Either way gg_cg_iterate returns in the textbook state (x_k, r_k, k).     */
int gg_cg_work_elems(const gg_kron* K, int64_t* elems);
int gg_cg_create(const gg_kron* K, double shift, double* work_dev, gg_cg** out);
int gg_cg_destroy(gg_cg* cg);
int gg_cg_start(gg_cg* cg, const double* b_dev, double* x_dev, double rtol, double atol,
                gg_stream stream);
int gg_cg_set_recurrence(gg_cg* cg, int fused);
int gg_cg_get_recurrence(const gg_cg* cg, int* fused);
/* Where the fused recurrence's vector passes ride (any time; same iterates):
 *   0: prologue writes r and p_new (first mode product), x update after the
 *      second mode product, epilogue reads p_new and r;
 *   1: the epilogue (last mode product) recomputes p_new = r + beta p_old and
 *      stores it, so the prologue only writes r;
 *   2: as 1, and the epilogue also applies x += alpha p_old (no side job).
 * Layouts 1 / 2 need the first factor's rows within one launch (<= 256).   */
int gg_cg_set_fusion(gg_cg* cg, int layout);
int gg_cg_get_fusion(const gg_cg* cg, int* layout);
/* Fused recurrence, layouts 0 / 1: x updated every other iteration (default
 * on; GG_CG_XDEFER=0 at gg_cg_create turns it off): the side job applies two
 * deferred steps x += a_{j-1} p_{j-1} + a_j p_j in one pass (three direction
 * buffers in work_dev); gg_cg_iterate still returns the textbook state.
 * set: before gg_cg_start; get: 1 when the deferral is in effect.         */
int gg_cg_set_xdefer(gg_cg* cg, int on);
int gg_cg_get_xdefer(const gg_cg* cg, int* on);
/* The x window of the block-basis CG (x_defer mode 3; GG_CG_XWIN at
 * gg_cg_work_elems / gg_cg_create, default 8, 0 = mode 2's balanced pairs):
 * x is cut into K regions and each iteration's pair launch brings ONE region
 * up to date with the (at most K) steps it has not seen, so x moves once per
 * K iterations and each direction once -- (K + 2) / K passes per iteration
 * instead of 2, with K + 1 direction buffers in work_dev.  Same iterates up to
 * rounding.  *K: the window in effect (once started; before, what gg_cg_start
 * will pick), 0 when x is updated otherwise.                              */
int gg_cg_get_xwin(const gg_cg* cg, int* K);
/* With the window in the block basis the CG keeps no r in memory (round 6,
 * GG_CG_RDERIVE=0 at create keeps it): the prologue takes r_{j-1} = p_{j-1} -
 * beta_{j-1} p_{j-2} from the two directions the window's ring holds, so it
 * reads p_{j-2} instead of r and stores no r -- 5 passes instead of 6; r is
 * materialised by a repair and by every close (the textbook state).  Same
 * iterates up to rounding.  *on: 1 when in effect (or, before start, when
 * gg_cg_start will choose it).                                             */
int gg_cg_get_rderive(const gg_cg* cg, int* on);
/* A reference stream rate for the fused CG prologue launch on this box
 * (bench.py, round 6): the prologue's streams alone over the handle's own
 * buffers -- read p_old, r, q, write r, p_new, q (six passes); with derived r
 * read p_old, p_{j-2}, q, write p_new, q (five) -- values unchanged, the
 * launch's non-temporal mask, a plain grid-stride kernel: two untimed and
 * `reps` timed passes, HIP events on the stream (synchronising).  *ms_host:
 * time per pass; offsets_host (4 entries, may be NULL): the addresses of the
 * second stream (r or p_{j-2}), p_old, p_new, q modulo 2 MiB.  Call after
 * gg_cg_start and before the iterations (it overwrites p_new and the slot
 * p_{j-2} will take, which the first prologues write anyway).              */
int gg_cg_calibrate(gg_cg* cg, int reps, double* ms_host, int64_t* offsets_host,
                    gg_stream stream);
/* Fused recurrence, layout 0: where r_j.q_j (for beta's |r - alpha q|^2
 * expansion) comes from.  1 (default; GG_CG_RQ=0 at gg_cg_create turns it
 * off): the conjugacy identity r_j.q_j = p_j.q_j - beta_j p_j.q_{j-1}, with
 * p_j.q_{j-1} summed by the first mode product's prologue (which reads q_{j-1}
 * anyway), so the last epilogue makes no pass over r; 0: the epilogue reads r.
 * set: before gg_cg_start; get: 1 when the identity is in effect.         */
int gg_cg_set_rq(gg_cg* cg, int mode);
int gg_cg_get_rq(const gg_cg* cg, int* mode);
/* The recurrence's basis (before gg_cg_start): 1 (default where the operator
 * has one, GG_CG_BASIS=0 at gg_cg_create turns it off) runs the fused
 * recurrence (layout 0, x_defer 2, r.q identity) in the parity-block basis of
 * gg_kron_block_info: b folded at start, the iterate kept folded, the
 * caller's x written by the unfold at every close; 0 the original layout.
 * get: 1 when the block basis is (or will be, at start) in effect.
 * gg_cg_launches: kernel launches per matvec (d, or d - 1 in the block
 * basis): the positions of gg_cg_profile_read.                              */
int gg_cg_set_basis(gg_cg* cg, int block);
int gg_cg_get_basis(const gg_cg* cg, int* block);
int gg_cg_launches(const gg_cg* cg, int* launches);
int gg_cg_iterate(gg_cg* cg, int max_iters, int check_every, gg_stream stream);
/* gg_cg_iterate = gg_cg_iterate_open + gg_cg_close.  _open leaves the fused
 * recurrence open (the last iteration's r update and the deferred x steps
 * pending; the next _open continues it seamlessly, the device stopping test
 * and done flag stay exact); gg_cg_close applies them -- the textbook state
 * (x, r, iteration count).  Read x or gg_cg_status's counts after a close. */
int gg_cg_iterate_open(gg_cg* cg, int max_iters, int check_every, gg_stream stream);
int gg_cg_close(gg_cg* cg, gg_stream stream);
int gg_cg_status(gg_cg* cg, int* iters, int* converged, double* resid_norm, double* tol,
                 gg_stream stream); /* synchronising */
/* Cancelled betas of the fused recurrence since start (|r_{j+1}|^2 from the
 * three-term expansion below 1e-6 rho_j): repaired by gg_cg_iterate with a
 * true r.r, restarted (p = r) by a sharded rank's _finish, and by
 * gg_cg_iterate too when GG_CG_RESTART=1 at gg_cg_create (the A/B that
 * measures the restart penalty on one GPU).  Synchronising.  No reference
 * counterpart (scipy's textbook CG has no cancellation test).              */
int gg_cg_cancels(gg_cg* cg, int* cancels, gg_stream stream);
/* A rank of a sharded CG whose operator is block-diagonal across ranks (the
 * parity sharding of gp_grief_amd/distributed.py: this handle's operator is
 * the rank's block, (K + shift I) restricted to it), every dot product
 * summed over ranks by the caller -- ONE all-reduce per iteration.
 * start_partial: r = b, x = 0, local r.r into rr_dev[0]; the caller
 * all-reduces rr_dev; start_finish: tolerances from the global norm.
 * iterate_partial: one fused iteration (layout 0: prologue, x side job,
 * epilogue on the mode products, as gg_cg_iterate) writing the local sums
 * red_dev[5] = [r.r, p.q_old, p.q, r.q, q.q]; the caller all-reduces red_dev;
 * iterate_finish: the scalar step (cg_fused_scalars on the global sums).  A
 * cancelled beta restarts with p = r (no repair pass: it would need a second
 * all-reduce).  close_partial: the deferred x steps and the pending r update,
 * local r.r into rr_dev; after the all-reduce, close_finish -- the textbook
 * state.  Reference: scipy's cg recurrence on kron_matrix.py:52-97's
 * operator (e); no reference counterpart for sharding. */
int gg_cg_start_partial(gg_cg* cg, const double* b_dev, double* x_dev, double* rr_dev,
                        gg_stream stream);
/* A sharded-CG rank over blocks [blk0, blk0 + nblk) of the operator's
 * parity-block layout (d >= 3): the rank's part of the operator is exactly
 * those diagonal blocks, so the _partial / _finish steps above run the block
 * kernels on them (gg_kron_block_matvec_range) with no exchange.  b and x are
 * the rank's blocks (gg_kron_block_fold_range).  work_dev: 16-byte aligned,
 * gg_cg_work_elems_blocks doubles.  gg_cg_start refuses such a handle.      */
int gg_cg_work_elems_blocks(const gg_kron* K, int64_t nblk, int64_t* elems);
int gg_cg_create_blocks(const gg_kron* K, int64_t blk0, int64_t nblk, double shift,
                        double* work_dev, gg_cg** out);
/* The other decompositions' once-per-solve fold / unfold on the device
 * (round 6; gp_grief_amd/distributed.py solve, which before folded on the
 * host and gathered host arrays through object collectives).
 * gg_parity_fold -- world = 2^K ranks, factors 0..K-1 of even order: forward
 * in = the grid vector (C order over m), out = rank's block in the even / odd
 * basis of axes 0..K-1, C order over (m_K .. m_{d-1}, h_0 .. h_{K-1}) (the
 * local factor order of distributed.parity_local_factors); inverse in = that
 * block, out = its contribution P^T to EVERY grid element (summed over the
 * ranks by the caller's all-reduce).
 * gg_shard0_fold -- factor 0's row blocks (the transpose decomposition;
 * layout (m_1 .. m_{d-1}, a), a = i_0 - rank m_0 / world fastest): forward
 * out = the rank's elements of the grid vector in; inverse writes them back
 * into the grid vector out (its other elements untouched).                */
int gg_parity_fold(int d, const int64_t* m, int world, int rank, int inverse,
                   const double* in_dev, double* out_dev, gg_stream stream);
int gg_shard0_fold(int d, const int64_t* m, int world, int rank, int inverse,
                   const double* in_dev, double* out_dev, gg_stream stream);
int gg_cg_start_finish(gg_cg* cg, const double* rr_dev, double rtol, double atol,
                       gg_stream stream);
int gg_cg_iterate_partial(gg_cg* cg, double* red_dev, gg_stream stream);
int gg_cg_iterate_finish(gg_cg* cg, const double* red_dev, gg_stream stream);
int gg_cg_close_partial(gg_cg* cg, double* rr_dev, gg_stream stream);
int gg_cg_close_finish(gg_cg* cg, const double* rr_dev, gg_stream stream);
/* Live timing: while enabled, every gg_cg_iterate matvec records HIP events
 * around each of its d mode products on the CG stream.  profile_read
 * (synchronising) returns the number of profiled matvecs and, per mode
 * product position k, the summed duration in ms.  Enabling resets.        */
int gg_cg_profile(gg_cg* cg, int enable);
int gg_cg_profile_read(gg_cg* cg, int* n_matvecs, double* mode_ms, int mode_ms_len);

/* ----------------------------------------------- Lanczos (SLQ log-det, P1)
 * k steps of three-term Lanczos on (K + shift I) from z / ||z|| where z is the
 * Rademacher probe (seed, probe) (oracle/cg.py probe_signs).  Writes the
 * tridiagonal (alphas[k], betas[k]) to host memory (synchronising).
 * work_dev: 4 * n elements.                                                   */
int gg_lanczos_probe(const gg_kron* K, double shift, uint64_t seed, int probe, int steps,
                     double* work_dev, double* alphas_host, double* betas_host,
                     int* steps_done, gg_stream stream);
/* The same with live per-step timing: step_ms_host[j] (steps entries) is the
 * HIP-event time of step j on the stream (the first event after the probe is
 * drawn); launch_ms_host (d + 1 entries, may be NULL) the summed time of each
 * mode-product position over the steps (d - 1 positions in the parity-block
 * basis, the rest 0), then the closing pass's time: once per probe, after
 * the last step, the streaming pass that forms beta_{steps-1} (T_k itself
 * needs beta_0 .. beta_{k-2}; with the update fused into the next step's
 * first launch, the last step has no next step to carry it).  No reference
 * counterpart (SLQ is absent from the reference).  */
int gg_lanczos_probe_timed(const gg_kron* K, double shift, uint64_t seed, int probe, int steps,
                           double* work_dev, double* alphas_host, double* betas_host,
                           int* steps_done, double* step_ms_host, double* launch_ms_host,
                           gg_stream stream);
/* Where the probe runs (round 6): *block = 1 when the operator has a
 * parity-block basis with d >= 3 (GG_LZ_BASIS=0 at gg_kron_create's snapshot
 * keeps the grid layout) -- the probe is folded once (P z) and every step is
 * the fused block step, d - 1 launches and 10 passes over N (the Lanczos
 * tridiagonal of P K P^T from P z is that of K from z: P is orthogonal);
 * *launches: the launches per step (the positions of launch_ms_host, the rest
 * of its d entries 0).                                                       */
int gg_lanczos_info(const gg_kron* K, int* block, int* launches);
int gg_probe_fill(uint64_t seed, int probe, double* z_dev, int64_t n, gg_stream stream);

/* --------------------------------------- per-factor symmetric eigensolver
 * KronMatrix.schur / svd / eig_vals per factor   kron_matrix.py:161-200, 355-366
 * Householder tridiagonalisation + implicit QL on device, one workgroup per
 * matrix (GG_EIG=jacobi: parallel cyclic Jacobi).  A_dev: `count` row-major
 * m[i] x m[i] symmetric matrices concatenated; on return Q_dev holds the
 * eigenvectors (columns) and lam_dev the eigenvalues, ascending.              */
int gg_sym_eig_batched(int count, const int64_t* m, const double* A_dev, double* Q_dev,
                       double* lam_dev, double* work_dev, int64_t work_elems,
                       int max_sweeps, gg_stream stream);
int gg_sym_eig_work_elems(int count, const int64_t* m, int64_t* elems);
/* Subset path (GRIEF setup, grief_kernel.py:168-190 needs every eigenvalue but
 * only the eigenvectors of the selected indices):
 *   gg_sym_eig_tridiag: Householder tridiagonalisation A = Z T Z^T,
 *     Z = H_0 ... H_{m-3}; R_dev gets the reflectors as rows (m[i] x m[i]
 *     blocks laid out like Q_dev), lam_dev the eigenvalues of T (= of A,
 *     ascending) by bisection; T and the reflector scales stay in work_dev
 *     (gg_sym_eig_work_elems).
 *   gg_sym_eig_tridiag_vectors: for factor i the nsel[i] eigenvalue indices
 *     sel (host, concatenated over factors) -> unit eigenvectors y of T by
 *     inverse iteration, then the reflectors applied (Z y): rows of Y_dev
 *     (concatenated nsel[i] x m[i] blocks) are the eigenvectors of A.  Valid
 *     when every selected eigenvalue is separated from its neighbours (the
 *     caller checks; no cluster reorthogonalisation).                         */
int gg_sym_eig_tridiag(int count, const int64_t* m, const double* A_dev, double* R_dev,
                       double* lam_dev, double* work_dev, int64_t work_elems, gg_stream stream);
int gg_sym_eig_tridiag_vectors(int count, const int64_t* m, const double* R_dev,
                               const double* work_dev, int64_t work_elems,
                               const double* lam_dev, const int* nsel, const int* sel,
                               double* Y_dev, gg_stream stream);
/* Rows of each k[i] x m[i] block of V_dev (concatenated, row-major)
 * orthonormalised in place (classical Gram-Schmidt twice, last row first). */
/* Eigenvector rows of centrosymmetric factors (order 2 h[f]) from their
 * half-order problems: V_dev holds, per factor, the even half's ke[f] rows
 * then the odd half's ko[f] rows (h[f] each); out_dev receives per factor
 * ke[f] + ko[f] rows of 2 h[f]: [y; J y] / sqrt 2 (even), [y; -J y] / sqrt 2
 * (odd).  The GRIEF subset setup's split of grief_kernel.py:168-190.       */
int gg_centro_expand(int nf, const int64_t* h, const int64_t* ke, const int64_t* ko,
                     const double* V_dev, double* out_dev, gg_stream stream);
int gg_rows_orthonormalize(int count, const int64_t* k, const int64_t* m, double* V_dev,
                           gg_stream stream);


/* ------------------------------------------------------- GRIEF basis (P2)
 * Stationary covariance k(x_i, z_j) for x: nx x dims, z: nz x dims row-major
 * (RBF / Exponential / Matern32 / Matern52, gp_grief/kern/stationary.py:108-258).
 * mode: 0 out = k, 1 out *= k, 2 out += k (kernel products / sums,
 * basekernel.py:139-155).                                                   */
#define GG_KERN_RBF 0
#define GG_KERN_EXPONENTIAL 1
#define GG_KERN_MATERN32 2
#define GG_KERN_MATERN52 3
int gg_cov(int kind, double variance, double lengthscale, int dims, const double* x_dev,
           int64_t nx, const double* z_dev, int64_t nz, int mode, double* out_dev,
           gg_stream stream);
/* Per-dimension tables of expand_SKC (gp_grief/tensors/tensors.py:97-128):
 * X[u][a] = sum_k qsel[u][k] k(xg[k], x[a * x_stride]); writes
 * ltab[a*U + col0 + u] = log|X| (0 where X == 0) and stab = sign(X), or with
 * stab_dev == NULL the value table ltab[a*U + col0 + u] = X (half the bytes;
 * what gg_grief_phi needs).                                                  */
int gg_grief_tables(int kind, double variance, double lengthscale, const double* x_dev,
                    int64_t x_stride, int64_t n, const double* xg_dev, int m,
                    const double* qsel_dev, int u, double* ltab_dev, double* stab_dev, int U,
                    int col0, gg_stream stream);
/* The tables of all nf dimensions in one launch (the same values as nf
 * gg_grief_tables calls; GriefKernel.cov's expand_SKC loop over dims,
 * gp_grief/kern/grief_kernel.py:96-104).  Host arrays of nf entries; factor f
 * reads x_dev[a * x_stride + x_offsets[f]].                                  */
int gg_grief_tables_all(int nf, const int* kinds, const double* variances,
                        const double* lengthscales, const double* x_dev, int64_t x_stride,
                        const int64_t* x_offsets, int64_t n, const double* const* xg_devs,
                        const int* ms, const double* const* qsel_devs, const int* us,
                        double* ltab_dev, double* stab_dev, int U, const int* col0s,
                        gg_stream stream);
/* Phi[a][j] = prod_f stab[a][c_jf] * exp(sum_f ltab[a][c_jf] - log_lam[j] / 2)
 * (GriefKernel.cov, gp_grief/kern/grief_kernel.py:96-104); cidx: p x d int32.
 * stab_dev == NULL: ltab is the value table (X itself) and Phi[a][j] =
 * prod_f ltab[a][c_jf] * exp(-log_lam[j] / 2).  transposed != 0 writes Phi^T
 * (p x n).                                                                   */
int gg_grief_phi(const double* ltab_dev, const double* stab_dev, int U, int64_t n,
                 const int* cidx_dev, int d, const double* log_lam_dev, int p, int transposed,
                 double* phi_dev, gg_stream stream);
/* expand_SKC(S, K, C, logged) (gp_grief/tensors/tensors.py:97-128) from the
 * stacked unique rows X (U x n row-major: rows row0_f .. row0_f + u_f - 1 are
 * (K_f)[unique_f] . C_f) and cidx (p x d int32, c_jf = row0_f + inverse_f[j]):
 * logged -> out = sum_f log|X[c_jf]| (0 for X == 0), sign_dev = prod_f sign;
 * else out = prod_f X[c_jf].  out: p x n.                                     */
int gg_expand_skc(const double* x_dev, int U, int64_t n, const int* cidx_dev, int d, int p,
                  int logged, double* out_dev, int* sign_dev, gg_stream stream);

/* ----------------------------------------- dense FP64 (GRIEF p x p system)
 * C = alpha op(A) op(B) + beta C on FP64 MFMA, row-major with leading dims.
 * uplo 1/2 writes only the lower/upper triangle.  splitk_dev (optional,
 * splitk_elems doubles) enables split-K for tall-skinny products such as
 * A = Phi^T Phi (gp_grief_model.py:149).                                      */
int gg_gemm(int trans_a, int trans_b, int M, int N, int K, double alpha, const double* A_dev,
            int64_t lda, const double* B_dev, int64_t ldb, double beta, double* C_dev,
            int64_t ldc, int uplo, double* splitk_dev, int64_t splitk_elems, gg_stream stream);
/* splitk_dev elements gg_gemm uses for this shape with the register-staged
   kernel's rule (0: it will not split K); kept for callers of round 1 --
   gg_gemm_workspace_elems below knows the transposes and uplo (the TN Gram
   kernel's own split) and is the one to use.                                 */
int gg_gemm_splitk_elems(int M, int N, int K, int64_t* elems);
/* The same for the exact call (transposes and uplo known): the TN kernel
   splits K when its tiles quantise badly onto the resident slots.           */
int gg_gemm_workspace_elems(int trans_a, int trans_b, int M, int N, int K, int uplo,
                            int64_t* elems);
/* y = alpha op(A) x + beta y, A: rows x cols row-major (Phi^T y, Phi v).    */
int gg_gemv(int trans, int64_t rows, int cols, double alpha, const double* A_dev, int64_t lda,
            const double* x_dev, double beta, double* y_dev, double* work_dev,
            int64_t work_elems, gg_stream stream);
/* P = A + diag(s / w)  (w NULL -> s), gp_grief_model.py:152                  */
int gg_add_diag(int n, const double* A_dev, int64_t lda, double s, const double* w_dev,
                double* P_dev, int64_t ldp, gg_stream stream);
/* Blocked Cholesky P = L L^T in place (lower), cho_factor, :153.  winv_dev
 * (gg_potrf_work_elems) receives the inverted diagonal blocks used by
 * gg_potrs; logdet_host = log det P.  Non-SPD -> GG_ERR_LINALG (synchronising).
 * The trailing updates run on a second stream of the device (look-ahead);
 * the call returns with all of its work complete. */
int gg_potrf_work_elems(int n, int64_t* elems);
int gg_potrf(int n, double* A_dev, int64_t lda, double* winv_dev, double* logdet_host,
             gg_stream stream);
/* B <- L^-1 B (which=1), L^-T B (2) or P^-1 B (3), B: n x r (cho_solve).
 * tmp_dev: 64 * r doubles.  The chained kernels take their block rows from a
 * ticket counter in arrival order, so progress does not depend on the order
 * the hardware dispatches workgroups; a bounded spin turns a lost flag into
 * GG_ERR_RUNTIME (B is then undefined).  GG_TRSV_CHAIN=0 selects the blocked
 * GEMM substitution instead.                                                 */
int gg_potrs(int n, int r, const double* L_dev, int64_t lda, const double* winv_dev,
             double* B_dev, int64_t ldb, int which, double* tmp_dev, gg_stream stream);
/* X = L^-1 (lower) from gg_potrf's factor and winv_dev, by recursive halving
 * on the MFMA GEMM.  The 64 x 64 diagonal blocks of X are written in full
 * (zeros above their diagonal); X's entries above the diagonal outside those
 * blocks are neither read nor written.  Replaces the
 * reference's cho_solve(P, I) for the adjoint gradient's diag(P^-1)
 * (gp_grief_model.py:228-235).                                               */
int gg_trtri(int n, const double* L_dev, int64_t lda, const double* winv_dev, double* X_dev,
             int64_t ldx, gg_stream stream);
/* out[j] = sum_{i >= j} M[i][j]^2 (diag of P^-1 from M = L^-1).              */
int gg_colsumsq_lower(int n, const double* M_dev, int64_t ld, double* out_dev,
                      gg_stream stream);

/* ------------------------------- Khatri-Rao contraction (off-grid P1 posterior)
 * out[j] = sum_g c[g] prod_f U_f[j][g_f] over the grid g (factor 0 slowest):
 * K(X*, grid) c for the row-partitioned Khatri-Rao cross covariance
 * KhatriRaoMatrix(GridKernel.cov_kr(X*, xg)) (gp_grief/kern/grid_kernel.py:148-179,
 * tensors/khatri_rao_matrix.py:7-50, BlockMatrix.__mul__ block_matrix.py:48-66).
 * ulast_dev: U_{d-1}, M x m_{d-1} row-major.  ut_dev: host array of d-1 device
 * pointers, ut_dev[f] = U_f^T (m_f x M row-major).  work_dev: at least
 * gg_kr_work_elems doubles (more work = fewer GEMM chunks).  1 <= d <= 32.     */
int gg_kr_work_elems(int d, const int64_t* m, int64_t M, int64_t* min_elems);
int gg_kr_contract(int d, const int64_t* m, const double* c_dev, const double* ulast_dev,
                   const double* const* ut_dev, int64_t M, double* out_dev, double* work_dev,
                   int64_t work_elems, gg_stream stream);
/* Row-col Khatri-Rao running product (RowColKhatriRaoMatrix.get_rows,
 * gp_grief/tensors/khatri_rao_matrix.py:117-140) over n elements of one factor
 * block X_i = R_i K_i C_i.  mode 0: P = X (first != 0) or P *= X.  mode 1
 * (logged): S *= sign(X), P += log|X| with X taken as 1 where S == 0 (first:
 * S = 1, P = 0 before the update).                                            */
int gg_kr_hadamard(int64_t n, const double* X_dev, double* P_dev, double* S_dev, int mode,
                   int first, gg_stream stream);

/* --------------------------------------------- P1 sharded over G ranks (RCCL)
 * The Kronecker operator with factor 0 split over `world` ranks (one per GPU).
 * Local vector layout: (m_1, ..., m_{d-1}, a) with a = i_0 - rank * m_0 / G the
 * fastest index.  One matvec = phase1 -> all-to-all(send -> recv, N/G^2 per
 * peer) -> phase2 -> all-to-all(send -> y_local); the exchanges are the
 * caller's (torch.distributed / RCCL).  phase1 can fuse CG's p = r + beta p
 * (cg_r_dev / cg_scalars_dev from gg_cgs, else NULL).  All buffers n_local.  */
typedef struct gg_kron_dist gg_kron_dist;
int gg_kron_dist_create(int d, const int64_t* m, const double* const* factors_host, int world,
                        int rank, gg_kron_dist** out);
int gg_kron_dist_destroy(gg_kron_dist* D);
int gg_kron_dist_sizes(const gg_kron_dist* D, int64_t* n_local, int64_t* work_elems);
/* Bit k set: factor k of the sharded operator runs through the
 * centrosymmetric even/odd split (as gg_kron_fold_mask).                  */
int gg_kron_dist_fold_mask(const gg_kron_dist* D, int64_t* mask);
int gg_kron_dist_phase1(const gg_kron_dist* D, double* x_local_dev, double* send_dev,
                        double* work_dev, const double* cg_r_dev, const void* cg_scalars_dev,
                        gg_stream stream);
int gg_kron_dist_phase2(const gg_kron_dist* D, const double* recv_dev, double* send_dev,
                        gg_stream stream);
/* Push mode: no all-to-all.  Each rank owns one exchange buffer xbuf = [recv |
 * out] (2 n_local doubles, any device allocation); gg_kron_dist_set_peers
 * learns every rank's xbuf, by IPC handle (one process per GPU: gg_ipc_handle
 * gives the 64-byte hipIpcMemHandle of the allocation holding a pointer and
 * the pointer's offset in it) or by plain pointer (ranks in one process).
 * phase1_push's last mode product stores each element straight into its
 * destination rank's recv over xGMI; after a barrier on all ranks,
 * phase2_push reads the own recv and stores into the owners' out, which after
 * a second barrier holds K x in the input layout.  scratch: n_local.       */
int gg_ipc_handle(const void* dev_ptr, void* handle_out, int64_t* offset_out);
int gg_kron_dist_set_peers(gg_kron_dist* D, double* own_xbuf, int use_ipc, const void* handles,
                           const int64_t* offsets, void* const* ptrs);
int gg_kron_dist_phase1_push(const gg_kron_dist* D, double* x_local_dev, double* scratch_dev,
                             double* work_dev, const double* cg_r_dev,
                             const void* cg_scalars_dev, gg_stream stream);
int gg_kron_dist_phase2_push(const gg_kron_dist* D, gg_stream stream);

/* Device CG scalars for a host-driven (sharded) CG: the same recurrence as
 * gg_cg_*, with each global dot product all-reduced by the caller between the
 * kernels that produce the local value (out_dev) and consume it.             */
typedef struct gg_cgs gg_cgs;
int gg_cgs_create(gg_cgs** out);
int gg_cgs_destroy(gg_cgs* c);
int gg_cgs_scalars(gg_cgs* c, void** scalars_dev);
int gg_cgs_local_dot(gg_cgs* c, const double* x_dev, const double* y_dev, int64_t n,
                     double* out_dev, gg_stream stream);
int gg_cgs_init(gg_cgs* c, const double* rr_dev, double rtol, double atol, gg_stream stream);
int gg_cgs_shift_dot(gg_cgs* c, double* q_dev, const double* p_dev, int64_t n, double shift,
                     double* out_dev, gg_stream stream);
int gg_cgs_alpha(gg_cgs* c, const double* pq_dev, gg_stream stream);
int gg_cgs_update(gg_cgs* c, double* x_dev, double* r_dev, const double* p_dev,
                  const double* q_dev, int64_t n, double* out_dev, gg_stream stream);
int gg_cgs_rho(gg_cgs* c, const double* rr_dev, gg_stream stream);
int gg_cgs_status(gg_cgs* c, int* iters, int* done, double* rho, double* tol,
                  gg_stream stream); /* synchronising */

/* Fused sharded CG: the single-GPU fused recurrence (gg_cg_*, recurrence
 * "fused") across ranks, ONE all-reduce of five doubles per iteration.  Per
 * iteration j: gg_kron_dist_phase1_fused (mode product 1 carries the
 * prologue -- with q_old = K p_old (unshifted) and s = shift: r -= alpha
 * (q_old + s p_old) when pending, p_new = r + beta p_old into its own buffer,
 * r.r and p_new.(q_old + s p_old) partials; mode product 2 the balanced
 * deferred x update, half of x per iteration; the last one the all-to-all /
 * push epilogue; push != 0: scratch as in phase1_push), the exchanges and
 * phase 2 as for the textbook CG (K p lands in q), gg_cgs_fused_post (reads
 * only: p.(q + s p) and |q + s p|^2; writes red[5] = [r.r, p_new.q_old',
 * p.q', 0, q'.q'] local, q' = q + s p), the caller's all-reduce of red,
 * gg_cgs_fused_scalars (alpha, beta by the |r - alpha q'|^2 expansion with
 * r.q' = p.q' - beta p.q_old', the x deferral).  Leaving the iterations:
 * gg_cgs_fused_close (deferred x steps, pending r -= alpha (q + s p) with p
 * the last direction, local r.r into rr_dev; half = 2 ceil(n_local / 4)),
 * the caller's all-reduce of rr_dev, gg_cgs_fused_close_rho -- the textbook
 * state, as gg_cg_iterate leaves it (q stays K p, unshifted).  Needs d >= 4, folded factors 1..d-1,
 * 16-byte aligned even-length vectors.  Reference: the CG the reference's
 * GP solves need on the operator of
 * kron_matrix.py:52-97; no reference counterpart for the sharding.         */
int gg_kron_dist_phase1_fused(const gg_kron_dist* D, const double* p_old_dev, double* p_new_dev,
                              double* send_dev, double* work_dev, double* r_dev,
                              const double* q_old_dev, double* x_dev, gg_cgs* cgs,
                              double shift, int push, gg_stream stream);
int gg_cgs_fused_post(gg_cgs* c, const double* q_dev, const double* p_dev, int64_t n,
                      double shift, double* red_dev, gg_stream stream);
int gg_cgs_fused_scalars(gg_cgs* c, const double* red_dev, const double* p_new_dev,
                         gg_stream stream);
int gg_cgs_fused_close(gg_cgs* c, double* x_dev, double* r_dev, const double* q_dev,
                       const double* p_dev, int64_t n, int64_t half, double shift,
                       double* rr_dev, gg_stream stream);
int gg_cgs_fused_close_rho(gg_cgs* c, const double* rr_dev, gg_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* GP_GRIEF_AMD_H */
