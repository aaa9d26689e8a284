"""CPU oracle for the gp_grief Kronecker / GRIEF hot path -- TEST INFRASTRUCTURE.

This package is a NumPy restatement of the reference algorithms
(scwolof/gp_grief, read-only checkout at /root/reference), written from the
reference's behaviour, not copied from it.  It exists only as the CHECKER:

  * tests/ compare the HIP product path against it,
  * __graft_entry__.smoke() checks one small device call against it,
  * bench.py times it as the `cpu_baseline` leg.

Nothing in gp_grief_amd/ imports, calls or links it; the product path fails
loudly when the HIP library is missing instead of falling back here.

Pinning: every function is checked against the golden fixtures in
tests/golden/*.npz, which tests/golden/make_golden.py produced by importing the
reference itself in the build container (tests/test_oracle_golden.py).  The
CG recurrence restates SciPy 1.15.3 `scipy.sparse.linalg.cg` (a third-party
dependency of the survey's CG restatement; the reference has no CG) and is
pinned by the scipy-cg history stored in grid_gp.npz.  The SLQ Lanczos log-det
has no reference implementation at all: it is pinned only against the exact
eigenvalue log-det (statistical tolerance), i.e. "parity unpinned" for the
Lanczos recurrence itself.
"""
from .kron import (kron_matvec, kron_matvec_T, kron_matvec_dsymm, kron_matvec_entries, kron_expand, log_kron,
                   find_extremum_eigs, factor_eigh, solve_schur, eig_log_det,
                   logdet_shifted, grid_latent_var, kr_contract, grid_offgrid_predict,
                   rowcol_kr_expand)
from .kernels import cov_1d
from .cg import cg_solve, slq_logdet, lanczos_tridiag
from .grief import (grief_inducing, grief_phi, grief_fit, grief_lml,
                    grief_adjoint_grad, grief_predict)
from .web import (web_lml_grad, web_predict, web_transformed_setup,
                  web_transformed_lml_grad, web_transformed_predict)

__all__ = [
    "kron_matvec", "kron_matvec_T", "kron_matvec_dsymm", "kron_matvec_entries", "kron_expand", "log_kron", "find_extremum_eigs",
    "factor_eigh", "solve_schur", "eig_log_det", "logdet_shifted", "grid_latent_var",
    "kr_contract", "grid_offgrid_predict", "rowcol_kr_expand", "cov_1d", "cg_solve", "slq_logdet", "lanczos_tridiag", "grief_inducing", "grief_phi",
    "grief_fit", "grief_lml", "grief_adjoint_grad", "grief_predict",
    "web_lml_grad", "web_predict", "web_transformed_setup", "web_transformed_lml_grad",
    "web_transformed_predict",
]
