"""Krylov solvers -- CPU oracle (test infrastructure only).

The reference has no CG and no Lanczos (gp_grief/linalg.py holds
only the iteration counter `solver_counter`, linalg.py:53-71, whose call
signature the callbacks below keep).

cg_solve restates the recurrence of SciPy 1.15.3 scipy.sparse.linalg.cg
(unpreconditioned, x0 = 0): stop when ||r|| < max(atol, rtol*||b||) is seen
at the top of an iteration; p = beta*p + r; alpha = rho / (p.q).  Pinned by
the scipy history stored in tests/golden/grid_gp.npz.

slq_logdet is stochastic Lanczos quadrature for log det(A); no reference
exists (parity unpinned), it is checked against the exact eigenvalue log-det.
The Rademacher probes come from a counter hash that the HIP library computes
identically (gp_grief_amd/csrc/gg_vec.hip, gg_probe_kernel), so CPU and GPU
Lanczos run on the same probe vectors.
"""
import numpy as np

_M64 = (1 << 64) - 1


def probe_signs(seed, probe, n):
    """Rademacher vector: bit 63 of splitmix64(seed*2^32 + probe*2^40 ... + i)."""
    i = np.arange(n, dtype=np.uint64)
    base = np.uint64(((int(seed) & 0xffffffff) << 32) ^ ((int(probe) & 0xffff) << 16)
                     ^ 0x9E3779B97F4A7C15) & np.uint64(_M64)
    with np.errstate(over="ignore"):
        z = base + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return np.where((z >> np.uint64(63)) == 0, 1.0, -1.0)


def cg_solve(matvec, b, rtol=1e-5, atol=0.0, maxiter=None, callback=None):
    """Returns (x, info, iters): info 0 = converged, else maxiter."""
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    bnorm = np.linalg.norm(b)
    tol = max(float(atol), float(rtol) * float(bnorm))
    x = np.zeros_like(b)
    if bnorm == 0:
        return b.copy(), 0, 0
    if maxiter is None:
        maxiter = b.size * 10
    r = b.copy()
    p = None
    rho_prev = None
    for it in range(maxiter):
        if np.linalg.norm(r) < tol:
            return x, 0, it
        rho = float(np.dot(r, r))
        if it == 0:
            p = r.copy()
        else:
            p *= rho / rho_prev
            p += r
        q = matvec(p)
        alpha = rho / float(np.dot(p, q))
        x += alpha * p
        r -= alpha * q
        rho_prev = rho
        if callback is not None:
            callback(x)
    return x, maxiter, maxiter


def lanczos_tridiag(matvec, z, steps):
    """Plain three-term Lanczos from z/||z||; returns (alphas, betas)."""
    v = np.asarray(z, dtype=np.float64) / np.linalg.norm(z)
    v_prev = np.zeros_like(v)
    beta = 0.0
    alphas, betas = [], []
    for _ in range(steps):
        w = matvec(v) - beta * v_prev
        a = float(np.dot(w, v))
        w -= a * v
        beta = float(np.linalg.norm(w))
        alphas.append(a)
        betas.append(beta)
        if beta <= 1e-300:
            break
        v_prev, v = v, w / beta
    return np.array(alphas), np.array(betas[:len(alphas) - 1])


def quadrature_logdet(alphas, betas, znorm2):
    """z^T log(A) z ~ ||z||^2 sum_j tau_j^2 log(theta_j) from the Lanczos T."""
    T = np.diag(alphas) + np.diag(betas, 1) + np.diag(betas, -1)
    theta, U = np.linalg.eigh(T)
    return znorm2 * float(np.sum(U[0, :] ** 2 * np.log(theta)))


def slq_logdet(matvec, n, probes=8, steps=30, seed=0):
    """Stochastic Lanczos quadrature estimate of log det(A) (mean over probes)."""
    ests = []
    for j in range(probes):
        z = probe_signs(seed, j, n)
        a, b = lanczos_tridiag(matvec, z, steps)
        ests.append(quadrature_logdet(a, b, float(n)))
    return float(np.mean(ests)), np.array(ests)
