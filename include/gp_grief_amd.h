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

/* y = (K_0 (x) ... (x) K_{d-1})^{T?} x + shift * x
 * KronMatrix.kronvec_prod / __mul__ / .T     kron_matrix.py:52-102, 203-213
 * (shift != 0 needs a square operator; x and y must not alias).            */
int gg_kron_matvec(const gg_kron* K, int transpose, const double* x_dev, double* y_dev,
                   double shift, double* work_dev, gg_stream stream);

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
/* y = x / (t + shift) for an explicit eigenvalue vector t (solve_schur with an
 * expanded t, kron_matrix.py:349-350).                                        */
int gg_diag_divide(const double* t_dev, double shift, const double* x_dev, double* y_dev,
                   int64_t n, gg_stream stream);

/* ------------------------------------------------------------- CG (P1 solve)
 * Unpreconditioned CG on (K + shift I) x = b, x0 = 0, the recurrence of
 * scipy.sparse.linalg.cg (the reference's solver_counter, linalg.py:53-71, is
 * its iteration callback).  All scalars stay on the device; the host polls
 * convergence every `check_every` iterations.  work_dev: gg_cg_work_elems. */
int gg_cg_work_elems(const gg_kron* K, int64_t* elems);
int gg_cg_create(const gg_kron* K, double shift, double* work_dev, gg_cg** out);
int gg_cg_destroy(gg_cg* cg);
int gg_cg_start(gg_cg* cg, const double* b_dev, double* x_dev, double rtol, double atol,
                gg_stream stream);
int gg_cg_iterate(gg_cg* cg, int max_iters, int check_every, gg_stream stream);
int gg_cg_status(gg_cg* cg, int* iters, int* converged, double* resid_norm, double* tol,
                 gg_stream stream); /* synchronising */

/* ----------------------------------------------- Lanczos (SLQ log-det, P1)
 * k steps of three-term Lanczos on (K + shift I) from z / ||z|| where z is the
 * Rademacher probe (seed, probe) (oracle/cg.py probe_signs).  Writes the
 * tridiagonal (alphas[k], betas[k]) to host memory (synchronising).
 * work_dev: 4 * n elements.                                                   */
int gg_lanczos_probe(const gg_kron* K, double shift, uint64_t seed, int probe, int steps,
                     double* work_dev, double* alphas_host, double* betas_host,
                     int* steps_done, gg_stream stream);
int gg_probe_fill(uint64_t seed, int probe, double* z_dev, int64_t n, gg_stream stream);

/* --------------------------------------- per-factor symmetric eigensolver
 * KronMatrix.schur / svd / eig_vals per factor   kron_matrix.py:161-200, 355-366
 * Parallel cyclic (two-sided) Jacobi on device, one workgroup per matrix.  A_dev: `count`
 * row-major m[i] x m[i] symmetric matrices concatenated; on return Q_dev holds
 * the eigenvectors (columns) and lam_dev the eigenvalues, ascending.          */
int gg_sym_eig_batched(int count, const int64_t* m, const double* A_dev, double* Q_dev,
                       double* lam_dev, double* work_dev, int64_t work_elems,
                       int max_sweeps, gg_stream stream);
int gg_sym_eig_work_elems(int count, const int64_t* m, int64_t* elems);

#ifdef __cplusplus
}
#endif
#endif /* GP_GRIEF_AMD_H */
