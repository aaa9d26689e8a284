"""linalg: the reference's helpers plus the device Krylov solvers.

Host utilities with the reference's behaviour (gp_grief/linalg.py):
  solve_schur, solve_chol :10-50   (dense helpers of the reference's GPRegressionModel)
  solver_counter          :53-71   (iteration callback / best-parameter backup)
  log_kron                :74-89
  uniquetol               :92-104
  LogexpTransformation    :107-125
Device solvers (no reference implementation exists):
  cg            -- scipy.sparse.linalg.cg's recurrence on (K + shift I), every
                   vector op and scalar on the MI355X (gg_cg_*).
  slq_logdet    -- stochastic Lanczos quadrature, Lanczos on the device
                   (gg_lanczos_probe); the k x k tridiagonal eigensolve of the
                   quadrature is host-side (k <= a few hundred).
"""
import ctypes
import logging
import sys

import numpy as np

logger = logging.getLogger(__name__)


class solver_counter:
    """Iteration counter usable as a solver / optimiser callback (linalg.py:53-71)."""

    def __init__(self, disp=True):
        self._disp = disp
        self.niter = 0
        self.backup = None

    def __call__(self, rk=None, msg='', store=None):
        self.niter += 1
        if self._disp:
            logger.info('iter %3i. %s' % (self.niter, msg))
            sys.stdout.flush()
        if store is not None:
            self.backup = store


def solve_schur(Q, t, x, shift=0.0):
    """(K + shift I) y = x for a dense K = Q diag(t) Q^T (linalg.py:10-32);
    the Kronecker form is KronMatrix.solve_schur (device).  Dense host helper
    of the reference's GPRegressionModel, kept for the import surface."""
    if x.shape != (Q.shape[0], 1):
        raise ValueError('x is the wrong shape, must be (%d,1)' % Q.shape[0])
    y = np.dot(Q.T, x)
    y = y / np.reshape(t + shift, y.shape)
    return np.dot(Q, y)


def solve_chol(U, x):
    """y = U \\ (U^T \\ x) for an upper Cholesky factor U (linalg.py:35-50);
    dense host helper (the models use the device gg_potrs)."""
    from scipy.linalg import solve_triangular
    if x.shape != (U.shape[0], 1):
        raise ValueError('x is the wrong shape, must be (%d,1)' % U.shape[0])
    y = solve_triangular(U, x, trans=1, lower=False, check_finite=False)
    return solve_triangular(U, y, trans=0, lower=False, check_finite=False)


def log_kron(a, b, a_logged=False, b_logged=False):
    """log(kron(a, b)) for 1-D a, b without forming the product (linalg.py:74-89)."""
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.ndim == b.ndim == 1, "currenly only working for 1d arrays"
    if not a_logged:
        a = np.log(a)
    if not b_logged:
        b = np.log(b)
    return (a.reshape((-1, 1)) + b.reshape((1, -1))).reshape(-1)


def uniquetol(x, tol=1e-6, relative=False):
    assert x.ndim == 1
    if relative:
        tol = np.float64(tol) * np.ptp(x)
    return x[~(np.triu(np.abs(x[:, None] - x) <= tol, 1)).any(0)]


class LogexpTransformation:
    """Softplus transform for positive parameters (linalg.py:107-125)."""
    _lim_val = 36.
    _log_lim_val = np.log(np.finfo(np.float64).max)

    def inverse_transform(self, x):
        return np.where(x > self._lim_val, x,
                        np.log1p(np.exp(np.clip(x, -self._log_lim_val, self._lim_val))))

    def transform(self, f):
        return np.where(f > self._lim_val, f, np.log(np.expm1(f)))

    def transform_grad(self, f, grad_f):
        return grad_f * np.where(f > self._lim_val, 1., -np.expm1(-f))


# ---------------------------------------------------------------- device CG
class CGResult(object):
    def __init__(self, x, info, iters, resid, tol):
        self.x, self.info, self.iters, self.resid, self.tol = x, info, iters, resid, tol


class KronCG(object):
    """Resident CG state for (K + shift I) x = b on one MI355X.

    The operator and all CG vectors (x, r, three p buffers, q + one matvec
    scratch) live in HBM; no host synchronisation inside an iteration.

    recurrence="fused" (default for d >= 2): an iteration is the d mode
    products plus one scalar kernel -- r -= alpha q, p = r + beta p (and r.r)
    ride on the first mode product, the x update on the second / third, p.q /
    r.q / q.q on the last; beta comes from |r - alpha q|^2 expanded
    (gg_vec.hip).  xdefer (fusion layouts 0 / 1; default 2): x is updated in
    deferred pairs of steps, two steps in one pass -- 2: each pair applied to
    half of x in each of the next two iterations (every side launch carries one
    pass), 1: the whole pair every other iteration, 0: every iteration (True =
    2, False = 0).  rq (layout 0; default 1): beta's r.q from the conjugacy
    identity p.q - beta p.q_prev (the prologue sums p.q_prev; the last
    epilogue does not read r), 0: r.q read in the epilogue.
    recurrence="textbook":
    scipy's operation order, with a separate x / r update pass.  Both leave
    iterate() in the textbook state.
    """

    def __init__(self, K, shift, recurrence="fused", fusion=None, xdefer=None, rq=None,
                 basis=None):
        from . import device as dev
        from . import native
        self.K = K
        self.shift = float(shift)
        self._dk = K._device()
        L = native.lib()
        we = ctypes.c_int64()
        native.check(L.gg_cg_work_elems(self._dk.h, ctypes.byref(we)))
        self.work = dev.empty(we.value)
        h = ctypes.c_void_p()
        native.check(L.gg_cg_create(self._dk.h, self.shift, native.dptr(self.work),
                                    ctypes.byref(h)), "gg_cg_create")
        self.h = h
        if recurrence not in ("fused", "textbook"):
            raise ValueError("recurrence must be 'fused' or 'textbook'")
        if recurrence == "textbook":
            native.check(L.gg_cg_set_recurrence(h, 0), "gg_cg_set_recurrence")
        f = ctypes.c_int()
        native.check(L.gg_cg_get_recurrence(h, ctypes.byref(f)))
        self.recurrence = "fused" if f.value else "textbook"
        if fusion is not None:
            native.check(L.gg_cg_set_fusion(h, int(fusion)), "gg_cg_set_fusion")
        native.check(L.gg_cg_get_fusion(h, ctypes.byref(f)))
        self.fusion = f.value
        if xdefer is not None:
            # True: the library default (2, balanced); an int selects 0 / 1 / 2
            mode = (2 if xdefer else 0) if isinstance(xdefer, bool) else int(xdefer)
            native.check(L.gg_cg_set_xdefer(h, mode), "gg_cg_set_xdefer")
        native.check(L.gg_cg_get_xdefer(h, ctypes.byref(f)))
        self.xdefer = f.value
        if rq is not None:
            native.check(L.gg_cg_set_rq(h, int(bool(rq))), "gg_cg_set_rq")
        native.check(L.gg_cg_get_rq(h, ctypes.byref(f)))
        self.rq = f.value
        if basis is not None:
            # "block": the parity-block basis (default where it exists), "grid": off
            if basis not in ("block", "grid"):
                raise ValueError("basis must be 'block' or 'grid'")
            native.check(L.gg_cg_set_basis(h, int(basis == "block")), "gg_cg_set_basis")
        native.check(L.gg_cg_get_basis(h, ctypes.byref(f)))
        self.basis = "block" if f.value else "grid"
        # the block basis's x window (x_defer mode 3, GG_CG_XWIN; 0: not in effect)
        native.check(L.gg_cg_get_xwin(h, ctypes.byref(f)))
        self.xwin = f.value
        # r derived from the window's directions (no r in memory; GG_CG_RDERIVE)
        native.check(L.gg_cg_get_rderive(h, ctypes.byref(f)))
        self.rderive = bool(f.value)
        self.n = int(K.shape[0])
        self.x = None

    def start(self, b_dev, rtol=1e-5, atol=0.0, x_out=None):
        from . import device as dev
        from . import native
        if b_dev.numel() != self.n:
            raise ValueError("b must have %d entries" % self.n)
        self.b = dev.ensure_aligned(b_dev.reshape(-1))
        self.x = dev.empty(self.n) if x_out is None else x_out
        native.check(native.lib().gg_cg_start(self.h, native.dptr(self.b), native.dptr(self.x),
                                              float(rtol), float(atol), native.stream_ptr()),
                     "gg_cg_start")

    def iterate(self, n_iter, check_every=0, close=True):
        """n_iter iterations; close=False leaves the fused recurrence open
        (its last r update and deferred x steps pending, continued by the next
        call) -- close() (or a later iterate(close=True)) restores the
        textbook state before x or the counts are read."""
        from . import native
        n_iter = min(int(n_iter), 2 ** 31 - 1)
        name = "gg_cg_iterate" if close else "gg_cg_iterate_open"
        native.check(getattr(native.lib(), name)(self.h, n_iter, min(int(check_every), n_iter),
                                                 native.stream_ptr()), name)

    def close(self):
        """Apply the pending r update and deferred x steps (gg_cg_close)."""
        from . import native
        native.check(native.lib().gg_cg_close(self.h, native.stream_ptr()), "gg_cg_close")

    def status(self):
        from . import native
        it, conv = ctypes.c_int(), ctypes.c_int()
        res, tol = ctypes.c_double(), ctypes.c_double()
        native.check(native.lib().gg_cg_status(self.h, ctypes.byref(it), ctypes.byref(conv),
                                               ctypes.byref(res), ctypes.byref(tol),
                                               native.stream_ptr()))
        return it.value, bool(conv.value), res.value, tol.value

    def calibrate(self, reps=5):
        """The fused prologue's six streams alone over this handle's buffers
        (gg_cg_calibrate; after start, before the iterations): (ms per pass,
        [r, p_old, p_new, q addresses mod 2 MiB])."""
        from . import native
        ms = ctypes.c_double()
        off = (ctypes.c_int64 * 4)()
        native.check(native.lib().gg_cg_calibrate(self.h, int(reps), ctypes.byref(ms), off,
                                                  native.stream_ptr()), "gg_cg_calibrate")
        return ms.value, [int(v) for v in off]

    def cancels(self):
        """Cancelled betas since start (gg_cg_cancels; synchronising)."""
        from . import native
        v = ctypes.c_int()
        native.check(native.lib().gg_cg_cancels(self.h, ctypes.byref(v), native.stream_ptr()),
                     "gg_cg_cancels")
        return v.value

    def profile(self, enable=True):
        """Record HIP events around every mode product of later iterations."""
        from . import native
        native.check(native.lib().gg_cg_profile(self.h, int(bool(enable))), "gg_cg_profile")

    def launches(self):
        """Kernel launches per matvec (d; d - 1 in the block basis)."""
        from . import native
        v = ctypes.c_int()
        native.check(native.lib().gg_cg_launches(self.h, ctypes.byref(v)))
        return v.value

    def profile_read(self):
        """(profiled matvecs, [summed ms per launch position]) (synchronising)."""
        from . import native
        d = self.launches()
        nm = ctypes.c_int()
        buf = (ctypes.c_double * 16)()
        native.check(native.lib().gg_cg_profile_read(self.h, ctypes.byref(nm), buf, 16),
                     "gg_cg_profile_read")
        return nm.value, [buf[k] for k in range(d)]

    def __del__(self):
        try:
            from . import native
            if getattr(self, "h", None) is not None and self.h.value:
                native.load().gg_cg_destroy(self.h)
        except Exception:
            pass


def cg(K, b, shift=0.0, rtol=1e-5, atol=0.0, maxiter=None, check_every=None, callback=None,
       recurrence="fused", fusion=None, basis=None, comm=None, decomposition="auto"):
    """Solve (K + shift I) x = b with CG on the device (x0 = 0).

    Same stopping rule and iterates as scipy.sparse.linalg.cg (recurrence:
    see KronCG).  b: numpy
    (N,1)/(N,) or a CUDA tensor; x is returned in the same kind.  `callback`
    (e.g. a solver_counter) is called once per completed iteration, after the
    solve, with no arguments beyond the counter protocol (the iterates stay on
    the device).  Returns (x, info) like scipy: info = 0 converged, else the
    number of iterations run.

    comm (multi-GPU, one process per GPU): a torch.distributed process group,
    True for the default group, or an exchange object -- every rank calls cg
    with the same K and b and gets the whole x; the solve is sharded by
    distributed.solve (decomposition "auto": the parity-block basis's blocks
    over 2^K ranks where it exists, else the even / odd parity blocks, else
    factor 0 sharded).
    """
    from . import device as dev
    n = int(K.shape[0])
    was_dev = dev.is_device_array(b)
    bd = dev.to_device(b)
    if bd.numel() != n:
        raise ValueError('b is the wrong shape, must have %d entries' % n)
    if maxiter is None:
        maxiter = n * 10
    if check_every is None:
        check_every = 10 if n >= 1 << 20 else 50
    if comm is not None:
        from . import distributed
        # the sharded solve runs its own recurrence (fused, layout 0, in the
        # decomposition's basis): a non-default choice cannot be honoured there
        if recurrence != "fused" or fusion not in (None, 0) or basis is not None:
            raise ValueError("comm=: the sharded CG runs the fused recurrence (layout 0) in "
                             "the decomposition's own basis; recurrence / fusion / basis "
                             "cannot be chosen")
        x, info, it, how = distributed.solve(K, bd, shift, comm, rtol, atol, maxiter,
                                             check_every, decomposition)
        if callback is not None:
            for _ in range(it):
                callback()
        out = (x.reshape(tuple(b.shape)) if b.numel() == n else x) if was_dev else \
            dev.to_host(x).reshape(np.shape(b))
        res, tol = getattr(distributed.solve, "last_resid", (None, None))
        cg.last = CGResult(out, info, it, res, tol)
        cg.last.decomposition = how
        return out, info
    solver = KronCG(K, shift, recurrence, fusion=fusion, basis=basis)
    solver.start(bd, rtol, atol)
    # one call: the library polls the device's done flag every check_every
    # iterations and stops issuing work once converged
    solver.iterate(maxiter, check_every=check_every)
    it, conv, res, tol = solver.status()
    if callback is not None:
        for _ in range(it):
            callback()
    info = 0 if conv else it
    x = solver.x
    if was_dev:
        out = x.reshape(tuple(b.shape)) if b.numel() == n else x
    else:
        out = dev.to_host(x).reshape(np.shape(b))
    cg.last = CGResult(out, info, it, res, tol)
    return out, info


def lanczos_info(K):
    """(block, launches): whether gg_lanczos_probe runs the probe in the
    operator's parity-block basis (round 6; GG_LZ_BASIS=0 keeps the grid
    layout) and its launches per step."""
    from . import native
    b, L = ctypes.c_int(), ctypes.c_int()
    native.check(native.lib().gg_lanczos_info(K._device().h, ctypes.byref(b), ctypes.byref(L)),
                 "gg_lanczos_info")
    return bool(b.value), L.value


def lanczos_tridiag(K, shift, steps, seed=0, probe=0, work=None, timed=False):
    """Device Lanczos on (K + shift I) from a Rademacher probe: (alphas, betas).

    work: optional device workspace of >= 4 N elements (allocated here
    otherwise).  timed=True also returns the per-step HIP-event times (ms, one
    per step run) and the summed time of each mode-product position
    (gg_lanczos_probe_timed): (alphas, betas, step_ms, launch_ms); the
    once-per-probe closing pass (the last beta's streaming pass, after the
    last step) is left in lanczos_tridiag.closing_ms."""
    from . import device as dev
    from . import native
    dk = K._device()
    n = int(K.shape[0])
    if work is None:
        work = dev.empty(4 * n)
    elif int(work.numel()) < 4 * n:
        raise ValueError("Lanczos workspace needs %d elements" % (4 * n))
    a = (ctypes.c_double * steps)()
    b = (ctypes.c_double * steps)()
    done = ctypes.c_int()
    if timed:
        d = len(dk._keep)
        sm = (ctypes.c_double * steps)()
        lm = (ctypes.c_double * (d + 1))()
        native.check(native.lib().gg_lanczos_probe_timed(
            dk.h, float(shift), int(seed), int(probe), int(steps), native.dptr(work), a, b,
            ctypes.byref(done), sm, lm, native.stream_ptr()), "gg_lanczos_probe_timed")
    else:
        native.check(native.lib().gg_lanczos_probe(dk.h, float(shift), int(seed), int(probe),
                                                   int(steps), native.dptr(work), a, b,
                                                   ctypes.byref(done), native.stream_ptr()),
                     "gg_lanczos_probe")
    k = done.value
    out = np.array(a[:k]), np.array(b[:max(k - 1, 0)])
    if timed:
        lanczos_tridiag.closing_ms = lm[d]
        return out + ([sm[j] for j in range(steps)], [lm[i] for i in range(d)])
    return out


lanczos_tridiag.closing_ms = None


def slq_logdet(K, shift, probes=8, steps=30, seed=0):
    """Stochastic Lanczos quadrature estimate of log det(K + shift I)."""
    n = int(K.shape[0])
    ests = []
    for j in range(probes):
        a, b = lanczos_tridiag(K, shift, steps, seed=seed, probe=j)
        T = np.diag(a) + np.diag(b, 1) + np.diag(b, -1)
        theta, U = np.linalg.eigh(T)
        ests.append(float(n) * float(np.sum(U[0, :] ** 2 * np.log(theta))))
    return float(np.mean(ests)), np.array(ests)
