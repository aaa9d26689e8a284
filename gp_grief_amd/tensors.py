"""Structured tensors: the drop-in KronMatrix backed by the HIP library.

Mirrors gp_grief/tensors/kron_matrix.py (class KronMatrix, :12-474),
gp_grief/tensors/khatri_rao_matrix.py (row-partitioned KhatriRaoMatrix, :7-50;
RowColKhatriRaoMatrix and its Transposed variant, :53-210) and gp_grief/tensors/selection_matrix.py (SelectionMatrixSparse, :55-107): same
constructor, attributes (n, sshape, shape, ndim, square, sym, read-only K),
method names, return shapes and exception types.

Where the arithmetic lives:
  * every N-sized operation (matvec, transposed matvec, the eigenvalue divide of
    solve_schur, shifted log-det, Kronecker-structured solves) runs on the
    device through the C ABI (gp_grief_amd.native);
  * per-factor eigendecompositions run on the device (Householder
    tridiagonalisation + implicit QL; for the GRIEF setup, bisection + inverse
    iteration for the selected eigenvectors only);
  * factor-sized bookkeeping (diag of factors, expand of small Kronecker
    products, per-factor Cholesky / inverse used to build a device operator,
    the top-p eigen-selection) stays on the host exactly as in the reference,
    where it is O(sum m_i^2) or O(d p m).

Vectors may be numpy (N,1) arrays -- copied over PCIe and the result returned
as numpy, like the reference -- or float64 CUDA tensors of shape (N,1), which
stay resident in HBM and are returned as CUDA tensors.
"""
import ctypes
from logging import getLogger
from warnings import warn

import numpy as np

from . import device as dev
from . import native
from .linalg import log_kron

logger = getLogger(__name__)


class _DeviceKron(object):
    """Owner of a gg_kron handle (factors in HBM, MFMA fragment order)."""

    def __init__(self, factors):
        L = native.lib()
        mats = [np.ascontiguousarray(np.asarray(f, dtype=np.float64)) for f in factors]
        for f in mats:
            if f.ndim != 2:
                raise ValueError("device Kronecker factors must be 2-D matrices")
        self._keep = mats
        rows = native.i64_array([f.shape[0] for f in mats])
        cols = native.i64_array([f.shape[1] for f in mats])
        ptrs = (ctypes.c_void_p * len(mats))(*[f.ctypes.data for f in mats])
        h = ctypes.c_void_p()
        native.check(L.gg_kron_create(len(mats), rows, cols, ptrs, ctypes.byref(h)),
                     "gg_kron_create")
        self.h = h
        self._work = {}
        self.n_rows = int(np.prod([f.shape[0] for f in mats]))
        self.n_cols = int(np.prod([f.shape[1] for f in mats]))

    def shape(self, transpose):
        a, b, w = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        native.check(native.lib().gg_kron_shape(self.h, int(transpose), ctypes.byref(a),
                                                ctypes.byref(b), ctypes.byref(w)))
        return a.value, b.value, w.value

    def fold_mask(self, transpose=False):
        """Bit k set: factor k runs through the centrosymmetric even/odd split
        (gg_kron_fold_mask; half the MFMA work)."""
        v = ctypes.c_int64()
        native.check(native.lib().gg_kron_fold_mask(self.h, int(transpose), ctypes.byref(v)))
        return v.value

    def block_info(self):
        """(available, n, launches per matvec) of the parity-block basis
        (gg_kron_block_info)."""
        a, n, l = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int()
        native.check(native.lib().gg_kron_block_info(self.h, ctypes.byref(a), ctypes.byref(n),
                                                     ctypes.byref(l)))
        return bool(a.value), n.value, l.value

    def block_n(self):
        """The block layout's length: n, or more when the two innermost
        (pair) axes are padded to 16 TF + 4 (round 6)."""
        return self.block_info()[1]

    def block_fold(self, xd, inverse=False, out=None):
        """P x (inverse: P^T x) between the grid and the block layout."""
        y = dev.empty(self.n_rows if inverse else self.block_n()) if out is None else out
        native.check(native.lib().gg_kron_block_fold(self.h, int(bool(inverse)),
                                                     native.dptr(xd), native.dptr(y),
                                                     native.stream_ptr()), "gg_kron_block_fold")
        return y

    def block_fold_range(self, xd, blk0, nblk, inverse=False, out=None):
        """Blocks [blk0, blk0 + nblk) of P x from the grid vector x; inverse:
        their contribution P^T (those blocks) to the grid vector
        (gg_kron_block_fold_range; summed over a sharded CG's ranks)."""
        _, n, _ = self.block_info()
        nl = n // (1 << len(self._keep)) * int(nblk)
        y = dev.empty(self.n_rows if inverse else nl) if out is None else out
        native.check(native.lib().gg_kron_block_fold_range(
            self.h, int(bool(inverse)), native.dptr(xd), native.dptr(y), int(blk0), int(nblk),
            native.stream_ptr()), "gg_kron_block_fold_range")
        return y

    def block_matvec_range(self, xd, blk0, nblk, shift=0.0, out=None):
        """(P K P^T + shift I) on blocks [blk0, blk0 + nblk) of the block
        layout (gg_kron_block_matvec_range)."""
        y = dev.empty(xd.numel()) if out is None else out
        native.check(native.lib().gg_kron_block_matvec_range(
            self.h, native.dptr(xd), native.dptr(y), float(shift),
            native.dptr(self._block_work()), int(blk0), int(nblk), native.stream_ptr()),
            "gg_kron_block_matvec_range")
        return y

    def _block_work(self):
        if "block" not in self._work:
            self._work["block"] = dev.empty(self.block_n())
        return self._work["block"]

    def block_matvec(self, xd, shift=0.0, out=None):
        """(P K P^T + shift I) x in the block layout (gg_kron_block_matvec)."""
        y = dev.empty(self.block_n()) if out is None else out
        native.check(native.lib().gg_kron_block_matvec(self.h, native.dptr(xd), native.dptr(y),
                                                       float(shift),
                                                       native.dptr(self._block_work()),
                                                       native.stream_ptr()),
                     "gg_kron_block_matvec")
        return y

    def block_matvec_timed(self, xd, out, reps, shift=0.0):
        """reps block-basis matvecs with HIP events around every launch
        (gg_kron_block_matvec_timed): (per-launch summed ms, total ms)."""
        _, _, L = self.block_info()
        lm = (ctypes.c_double * max(L, 1))()
        tot = ctypes.c_double()
        native.check(native.lib().gg_kron_block_matvec_timed(
            self.h, native.dptr(xd), native.dptr(out), float(shift),
            native.dptr(self._block_work()), int(reps), lm, ctypes.byref(tot),
            native.stream_ptr()), "gg_kron_block_matvec_timed")
        return [lm[k] for k in range(L)], tot.value

    def work(self, transpose):
        key = bool(transpose)
        if key not in self._work:
            _, _, w = self.shape(transpose)
            self._work[key] = dev.empty(max(w, 1))
        return self._work[key]

    def matvec(self, xd, transpose=False, shift=0.0, out=None):
        n_out, n_in, _ = self.shape(transpose)
        if xd.numel() != n_in:
            raise ValueError("x has %d elements, operator needs %d" % (xd.numel(), n_in))
        y = dev.empty(n_out) if out is None else out
        w = self.work(transpose)
        native.check(native.lib().gg_kron_matvec(self.h, int(transpose), native.dptr(xd),
                                                 native.dptr(y), float(shift), native.dptr(w),
                                                 native.stream_ptr()), "gg_kron_matvec")
        return y

    def matvec_timed(self, xd, out, reps, transpose=False, shift=0.0):
        """reps matvecs x -> out with HIP events around every mode product
        (gg_kron_matvec_timed, synchronising): (per-position summed ms, total ms)."""
        n_out, n_in, _ = self.shape(transpose)
        if xd.numel() != n_in or out.numel() != n_out:
            raise ValueError("x / out have the wrong length")
        w = self.work(transpose)
        d = len(self._keep)
        lm = (ctypes.c_double * d)()
        tot = ctypes.c_double()
        native.check(native.lib().gg_kron_matvec_timed(
            self.h, int(transpose), native.dptr(xd), native.dptr(out), float(shift),
            native.dptr(w), int(reps), lm, ctypes.byref(tot), native.stream_ptr()),
            "gg_kron_matvec_timed")
        return [lm[k] for k in range(d)], tot.value

    def release_work(self):
        self._work = {}

    def __del__(self):
        try:
            if getattr(self, "h", None) is not None and self.h.value:
                native.load().gg_kron_destroy(self.h)
        except Exception:
            pass


def _as_matrix(Ki):
    if isinstance(Ki, np.ndarray):
        return Ki
    if hasattr(Ki, "expand"):
        return np.asarray(Ki.expand())
    return np.asarray(Ki)


def _vector_in(x, n, msg):
    """Shape-check an (n,1) vector and return (device 1-D tensor, was_device)."""
    if tuple(x.shape) != (n, 1):
        raise ValueError(msg)
    return dev.to_device(x), dev.is_device_array(x)


def _vector_out(yd, was_device):
    if was_device:
        return yd.reshape(-1, 1)
    return dev.to_host(yd).reshape((-1, 1))


def _is_symmetric(M):
    return np.allclose(M, M.T, rtol=1e-12, atol=1e-14 * max(1.0, float(np.abs(M).max())))


def device_sym_eig(factors, max_sweeps=40):
    """Eigendecomposition of symmetric factors on the device (ascending)."""
    L = native.lib()
    t = dev.torch()
    mats = [np.asarray(f, dtype=np.float64) for f in factors]
    for f in mats:
        if f.ndim != 2 or f.shape[0] != f.shape[1]:
            raise AssertionError("factor must be square")
        if not np.allclose(f, f.T, rtol=1e-12, atol=1e-14 * max(1.0, np.abs(f).max())):
            raise NotImplementedError("the device eigensolver handles symmetric factors "
                                      "(every grid-kernel factor is symmetric)")
    m = [f.shape[0] for f in mats]
    A = dev.to_device(np.concatenate([f.reshape(-1) for f in mats]))
    Q = dev.empty(A.numel())
    lam = dev.empty(sum(m))
    marr = native.i64_array(m)
    we = ctypes.c_int64()
    native.check(L.gg_sym_eig_work_elems(len(m), marr, ctypes.byref(we)))
    work = dev.empty(max(we.value, 1))
    native.check(L.gg_sym_eig_batched(len(m), marr, native.dptr(A), native.dptr(Q),
                                      native.dptr(lam), native.dptr(work), we.value,
                                      int(max_sweeps), native.stream_ptr()),
                 "gg_sym_eig_batched")
    Qh = dev.to_host(Q)
    lh = dev.to_host(lam)
    del t
    outQ, outL = [], []
    o = lo = 0
    for mi in m:
        outQ.append(np.asfortranarray(Qh[o:o + mi * mi].reshape(mi, mi)))
        outL.append(lh[lo:lo + mi].copy())
        o += mi * mi
        lo += mi
    return outQ, outL


def centro_halves(F):
    """(Ke, Ko) with eig(F) = eig(Ke) u eig(Ko) for a symmetric centrosymmetric
    F of even order m = 2h (J F J = F, J the exchange matrix -- every
    stationary kernel on an evenly spaced grid: the GRIEF inducing factors).
    With F = [[A, B], [B^T, J A J]] the orthogonal Q = [[I, I], [J, -J]] / sqrt 2
    gives Q^T F Q = diag(A + B J, A - B J): the even eigenvectors of F are
    [y; J y] / sqrt 2 (y of Ke), the odd ones [y; -J y] / sqrt 2 (y of Ko).
    Half the order: a quarter of the tridiagonalisation work per half, two
    independent problems.  F a device tensor; None when F is not
    centrosymmetric to 16 eps max|F| (or m is odd or below 16).  The split
    uses the centrosymmetric part (F + J F J) / 2 (a perturbation below the
    eigensolver's own rounding)."""
    t = dev.torch()
    m = int(F.shape[0])
    if m % 2 or m < 16:
        return None
    Fr = t.flip(F, (0, 1))
    scale = float(F.abs().max())
    if float((F - Fr).abs().max()) > 16 * np.finfo(np.float64).eps * max(scale, 1e-300):
        return None
    Fs = 0.5 * (F + Fr)
    h = m // 2
    A = Fs[:h, :h]
    BJ = t.flip(Fs[:h, h:], (1,))
    Ke = A + BJ
    Ko = A - BJ
    return 0.5 * (Ke + Ke.t()), 0.5 * (Ko + Ko.t())


def centro_halves_host(F):
    """centro_halves for a host factor (numpy): the split the GRIEF setup uses
    on its host-built grid factors, whose halves then go to the device in one
    copy."""
    m = F.shape[0]
    if m % 2 or m < 16:
        return None
    Fr = F[::-1, ::-1]
    if np.abs(F - Fr).max() > 16 * np.finfo(np.float64).eps * max(np.abs(F).max(), 1e-300):
        return None
    Fs = 0.5 * (F + Fr)
    h = m // 2
    A = Fs[:h, :h]
    BJ = Fs[:h, h:][:, ::-1]
    Ke, Ko = A + BJ, A - BJ
    return 0.5 * (Ke + Ke.T), 0.5 * (Ko + Ko.T)


def centro_merge(lam_e, lam_o):
    """The ascending spectrum of F from its halves, and for every position the
    half (0 even, 1 odd) and the index within it."""
    lam = np.concatenate([lam_e, lam_o])
    half = np.concatenate([np.zeros(lam_e.size, np.int64), np.ones(lam_o.size, np.int64)])
    idx = np.concatenate([np.arange(lam_e.size), np.arange(lam_o.size)])
    order = np.argsort(lam, kind="stable")
    return lam[order], half[order], idx[order]


def centro_expand(Vh, hs, kes, kos):
    """Eigenvector rows of centrosymmetric factors from their halves' rows
    (gg_centro_expand, one launch): Vh = [V_e0, V_o0, V_e1, V_o1, ...] as
    returned by device_sym_eig_tridiag_vectors (one buffer, in that order);
    factor f gets (ke + ko) x 2h rows, the even ones first: [y; J y] / sqrt 2,
    then [y; -J y] / sqrt 2."""
    L = native.lib()
    nf = len(hs)
    tot = sum((int(ke) + int(ko)) * 2 * int(h) for h, ke, ko in zip(hs, kes, kos))
    out = dev.empty(max(tot, 1))
    native.check(L.gg_centro_expand(nf, native.i64_array(hs), native.i64_array(kes),
                                    native.i64_array(kos), native.dptr(Vh[0]), native.dptr(out),
                                    native.stream_ptr()), "gg_centro_expand")
    res, o = [], 0
    for h, ke, ko in zip(hs, kes, kos):
        k, m = int(ke) + int(ko), 2 * int(h)
        res.append(out[o:o + k * m].view(k, m))
        o += k * m
    return res


def device_sym_eig_tridiag(factors):
    """Eigenvalues of symmetric factors (ascending, host arrays) by Householder
    tridiagonalisation + bisection on the device, plus a handle for
    device_sym_eig_tridiag_vectors (the GRIEF setup needs every eigenvalue but
    only the selected eigenvectors: grief_kernel.py:168-190).  Factors may be
    host arrays or device tensors (no host round trip)."""
    L = native.lib()
    t = dev.torch()
    on_dev = all(dev.is_device_array(f) for f in factors)
    mats = list(factors) if on_dev else [np.asarray(f, dtype=np.float64) for f in factors]
    for f in mats:
        if f.ndim != 2 or f.shape[0] != f.shape[1]:
            raise AssertionError("factor must be square")
    m = [int(f.shape[0]) for f in mats]
    if on_dev:
        A = t.cat([f.to(t.float64).contiguous().reshape(-1) for f in mats])
    else:
        A = dev.to_device(np.concatenate([f.reshape(-1) for f in mats]))
    R = dev.empty(A.numel())
    lam = dev.empty(sum(m))
    marr = native.i64_array(m)
    we = ctypes.c_int64()
    native.check(L.gg_sym_eig_work_elems(len(m), marr, ctypes.byref(we)))
    work = dev.empty(max(we.value, 1))
    native.check(L.gg_sym_eig_tridiag(len(m), marr, native.dptr(A), native.dptr(R),
                                      native.dptr(lam), native.dptr(work), we.value,
                                      native.stream_ptr()), "gg_sym_eig_tridiag")
    lh = dev.to_host(lam)
    out, o = [], 0
    for mi in m:
        out.append(lh[o:o + mi].copy())
        o += mi
    return out, dict(m=m, R=R, lam=lam, work=work, work_elems=we.value)


def device_sym_eig_tridiag_vectors(handle, selections):
    """Unit eigenvectors of the selected (ascending-order) indices per factor as
    device tensors V_f (len(sel_f) x m_f; row k = eigenvector sel_f[k], i.e.
    the rows Q_f^T[sel_f, :]): inverse iteration on the tridiagonal, the
    Householder reflectors applied to each vector in place (Z is never formed),
    then a re-orthonormalisation of the rows (gg_rows_orthonormalize) so they
    are orthonormal to ~eps."""
    L = native.lib()
    m = handle["m"]
    assert len(selections) == len(m)
    sel = [np.asarray(s, dtype=np.int64).reshape(-1) for s in selections]
    nsel = (ctypes.c_int * len(m))(*[int(s.size) for s in sel])
    flat = np.concatenate(sel) if sum(s.size for s in sel) else np.zeros(0, dtype=np.int64)
    carr = (ctypes.c_int * max(flat.size, 1))(*[int(v) for v in flat])
    V = dev.empty(max(sum(int(s.size) * mi for s, mi in zip(sel, m)), 1))
    native.check(L.gg_sym_eig_tridiag_vectors(
        len(m), native.i64_array(m), native.dptr(handle["R"]), native.dptr(handle["work"]),
        handle["work_elems"], native.dptr(handle["lam"]), nsel, carr, native.dptr(V),
        native.stream_ptr()), "gg_sym_eig_tridiag_vectors")
    out, oy = [], 0
    for s, mi in zip(sel, m):
        k = int(s.size)
        out.append(V[oy:oy + k * mi].view(k, mi))
        oy += k * mi
    # inverse iteration leaves neighbours ~eps ||T|| / gap from orthogonal:
    # classical Gram-Schmidt twice, largest eigenvalue (last row) first
    native.check(L.gg_rows_orthonormalize(len(m), native.i64_array([int(s.size) for s in sel]),
                                          native.i64_array(m), native.dptr(V),
                                          native.stream_ptr()), "gg_rows_orthonormalize")
    return out


class KronMatrix(object):
    """Kronecker product of matrices (kron_matrix.py:12-474) on MI355X."""

    def __init__(self, K, sym=False):
        self._K = K
        self.n = len(self.K)
        self.sshape = np.vstack([np.shape(Ki) for Ki in self.K])
        self.shape = np.atleast_1d(np.prod(np.float64(self.sshape), axis=0))
        if np.all(self.shape < np.iinfo(np.uint64).max):
            self.shape = np.uint64(self.shape)
        self.ndim = self.shape.size
        assert self.ndim <= 2, "kron matrix cannot be more than 2d"
        self.square = self.ndim == 2 and self.shape[0] == self.shape[1]
        self.sym = sym
        self._dev = None
        self._dev_key = None
        if sym:
            assert np.array_equal(self.sshape[:, 0], self.sshape[:, 1]), \
                'this matrix cannot be symmetric: it is not square'
            self.ensure_fortran()

    @property
    def K(self):
        return self._K

    @K.setter
    def K(self, K):
        raise AttributeError("Attribute is Read only.")

    # ------------------------------------------------------------- device
    def _device(self):
        key = tuple(id(Ki) for Ki in self._K)
        if self._dev is None or self._dev_key != key:
            assert self.ndim == 2, "device operator needs 2-D factors"
            self._dev = _DeviceKron([_as_matrix(Ki) for Ki in self._K])
            self._dev_key = key
        return self._dev

    def matvec_device(self, xd, transpose=False, shift=0.0, out=None):
        """y = (K^{T?} + shift I) x for a resident 1-D float64 CUDA tensor."""
        return self._device().matvec(dev.ensure_aligned(xd), transpose, shift, out)

    # ------------------------------------------------------------- products
    def kronvec_prod(self, x):
        """K*x (kron_matrix.py:52-97) on the device; x is (N,1)."""
        n_in = int(self.shape[1])
        xd, was_dev = _vector_in(x, n_in, 'x is the wrong shape, must be (%d,1), not %s'
                                 % (n_in, repr(tuple(np.shape(x)))))
        return _vector_out(self.matvec_device(xd), was_dev)

    def __mul__(self, x):
        return self.kronvec_prod(x)

    def kronkron_prod(self, X):
        """K*X for KronMatrix X (kron_matrix.py:105-116): per-factor products."""
        if not isinstance(X, KronMatrix):
            raise TypeError("X is not a KronMatrix")
        elif X.n != self.n:
            raise TypeError('inconsistent kron structure')
        elif not np.array_equal(X.sshape[1], self.sshape[0]):
            raise TypeError("Dimensions of X submatricies are not consistent")
        return KronMatrix([np.dot(_as_matrix(self.K[i]), _as_matrix(X.K[i]))
                           for i in range(self.n)])

    def kronvec_div(self, x):
        """K \\ x (kron_matrix.py:119-142) = (K_0^-1 (x) ...) x, applied on the device."""
        assert self.ndim == 2
        if tuple(x.shape) != (int(self.shape[0]), 1):
            raise ValueError('x wrong shape, must be (%d,1)' % self.shape[0])
        inv = [np.linalg.inv(_as_matrix(Ki)) for Ki in self.K]
        return KronMatrix(inv) * x

    def chol(self):
        """Upper Cholesky factor per sub-matrix (kron_matrix.py:145-158)."""
        assert self.square
        C = np.empty(self.n, dtype=object)
        for i, Ki in enumerate(self.K):
            if hasattr(Ki, "chol"):
                C[i] = Ki.chol()
            else:
                C[i] = np.linalg.cholesky(Ki).T
        return KronMatrix(C)

    def _split_symmetric(self):
        """Indices of the factors that are numerically symmetric (the device
        eigensolver's domain) and the factor matrices."""
        mats = [_as_matrix(Ki) for Ki in self.K]
        sym = [i for i, M in enumerate(mats)
               if M.ndim == 2 and M.shape[0] == M.shape[1] and _is_symmetric(M)]
        return sym, mats

    def schur(self):
        """(Q, T) per factor (kron_matrix.py:161-171): symmetric factors by the
        device eigensolver (T diagonal), other factors by the real Schur form
        (scipy.linalg.schur, factor-sized host LAPACK, as the reference)."""
        assert self.square
        import scipy.linalg as sla
        Q = [None] * self.n
        T = [None] * self.n
        todo = []
        for i, Ki in enumerate(self.K):
            if hasattr(Ki, "schur"):
                T[i], Q[i] = Ki.schur()
            else:
                todo.append(i)
        sym, mats = self._split_symmetric()
        dev_idx = [i for i in todo if i in sym]
        if dev_idx:
            Qd, lam = device_sym_eig([mats[i] for i in dev_idx])
            for i, q, l in zip(dev_idx, Qd, lam):
                Q[i], T[i] = q, np.diag(l)
        for i in todo:
            if i not in dev_idx:
                T[i], Q[i] = sla.schur(mats[i])
        return KronMatrix(Q), KronMatrix(T)

    def svd(self):
        """(Q, eig_vals) of a PSD KronMatrix (kron_matrix.py:174-200), descending:
        symmetric factors by the device eigensolver, others by the factor-sized
        host SVD (np.linalg.svd, as the reference)."""
        assert self.square, "matrix must be square for current implementation"
        sym, mats = self._split_symmetric()
        Q = [None] * self.n
        lam = [None] * self.n
        dev_idx = [i for i in range(self.n) if i in sym and not hasattr(self.K[i], "svd")]
        try:
            if dev_idx:
                Qd, ld = device_sym_eig([mats[i] for i in dev_idx])
                for i, q, l in zip(dev_idx, Qd, ld):
                    Q[i] = np.asfortranarray(q[:, ::-1])
                    lam[i] = l[::-1].copy()
            for i, Ki in enumerate(self.K):
                if i in dev_idx:
                    continue
                if hasattr(Ki, "svd"):
                    Q[i], lam[i] = Ki.svd()
                else:
                    Q[i], lam[i] = np.linalg.svd(mats[i], full_matrices=0, compute_uv=1)[:2]
        except np.linalg.LinAlgError:
            logger.error('SVD failed on a dimension.')
            raise
        return KronMatrix(Q), KronMatrix(lam)

    def transpose(self):
        assert self.ndim == 2
        if self.sym:
            return self
        return KronMatrix([Ki.T for Ki in self.K])
    T = property(transpose)

    def expand(self, log_expansion=False):
        """Dense expansion (kron_matrix.py:215-239) -- host, for small operators."""
        if log_expansion:
            Kb = np.array([0.])
            for Ki in self.K:
                Kb = log_kron(a=Kb, b=_as_matrix(Ki), a_logged=True)
        else:
            Kb = 1.
            if self.ndim == 1 and self.n > 10:
                warn('consider using numerically more stable log_expansion')
            for Ki in self.K:
                Kb = np.kron(Kb, _as_matrix(Ki))
        return Kb.reshape(np.int64(self.shape))

    def inv(self):
        assert self.square
        return KronMatrix([Ki.inv() if hasattr(Ki, "inv") else np.linalg.inv(Ki)
                           for Ki in self.K])

    def diag(self):
        """Diagonal as a 1-D KronMatrix (kron_matrix.py:254-265)."""
        assert self.ndim == 2
        D = np.empty(self.n, dtype=object)
        for i, Ki in enumerate(self.K):
            D[i] = Ki.diag() if hasattr(Ki, "diag") else np.diag(Ki)
        return KronMatrix(D)

    def sub_cond(self):
        assert self.square
        return [np.linalg.cond(Ki) for Ki in self.K]

    def sub_shift(self, shift=1e-6):
        """K_i += shift I in place (kron_matrix.py:276-286)."""
        if not np.array_equal(self.sshape[:, 0], self.sshape[:, 1]):
            raise RuntimeError('can only apply sub_shift for square matricies')
        for i, Ki in enumerate(self.K):
            self.K[i] = Ki + shift * np.identity(self.sshape[i, 0])
        if self.sym:
            self.ensure_fortran()
        self._dev = None
        return self

    def ensure_fortran(self):
        for i, Ki in enumerate(self.K):
            if isinstance(Ki, np.ndarray):
                self.K[i] = np.asarray(Ki, order='F')
        return self

    def solve_chol(U, x):
        """U \\ (U' \\ x) (kron_matrix.py:297-325) as one device Kron matvec."""
        if tuple(x.shape) != (int(U.shape[0]), 1):
            raise ValueError('x wrong shape, must be (%d,1)' % U.shape[0])
        F = []
        for Ui in U.K:
            Ui = _as_matrix(Ui)
            Uinv = np.linalg.inv(Ui)
            F.append(Uinv.dot(Uinv.T))
        return KronMatrix(F) * x

    def solve_schur(Q, t, x, shift=0.0):
        """(K + shift I) y = x via Q ((Q^T x) / (t + shift)) (kron_matrix.py:328-352).

        t: expanded eigenvalue vector (N,), the T KronMatrix from schur, or a
        1-D eigenvalue KronMatrix; in the Kronecker cases the eigenvalue
        product is decoded on the device per element and never expanded.
        """
        n = int(Q.shape[0])
        xd, was_dev = _vector_in(x, n, 'x wrong shape, must be (%d,1)' % n)
        L = native.lib()
        y = Q.matvec_device(xd, transpose=True)
        if isinstance(t, KronMatrix):
            eig = t.diag() if t.ndim == 2 else t
            lam = [np.asarray(e, dtype=np.float64).reshape(-1) for e in eig.K]
            lamd = dev.to_device(np.concatenate(lam))
            native.check(L.gg_kron_diag_scale(len(lam), native.i64_array([l.size for l in lam]),
                                              native.dptr(lamd), float(shift),
                                              native.GG_DIAG_DIVIDE, native.dptr(y),
                                              native.dptr(y), native.stream_ptr()),
                         "gg_kron_diag_scale")
        else:
            td = dev.to_device(t)
            if td.numel() != n:
                raise ValueError("t must have %d entries" % n)
            native.check(L.gg_diag_divide(native.dptr(td), float(shift), native.dptr(y),
                                          native.dptr(y), n, native.stream_ptr()),
                         "gg_diag_divide")
        out = Q.matvec_device(y)
        return _vector_out(out, was_dev)

    def eig_vals(self):
        """Eigenvalues per factor as a 1-D KronMatrix (kron_matrix.py:355-366):
        symmetric factors (sym=True or numerically symmetric) by the device
        eigensolver, others by np.linalg.eigvals on the host (factor-sized;
        complex for a non-normal factor, as in the reference)."""
        assert self.ndim == 2
        sym, mats = self._split_symmetric()
        if self.sym:
            sym = list(range(self.n))
        eigs = [None] * self.n
        dev_idx = [i for i in range(self.n) if i in sym and not hasattr(self.K[i], "eig_vals")]
        if dev_idx:
            _, lam = device_sym_eig([mats[i] for i in dev_idx])
            for i, l in zip(dev_idx, lam):
                eigs[i] = l
        for i, Ki in enumerate(self.K):
            if eigs[i] is None:
                eigs[i] = Ki.eig_vals() if hasattr(Ki, "eig_vals") else np.linalg.eigvals(mats[i])
        return KronMatrix(eigs)

    def find_extremum_eigs(eigs, n_eigs, mode='largest', log_expand=False, sort=True,
                           compute_global_loc=False):
        """Positions of the n_eigs extreme Kronecker eigenvalues (kron_matrix.py:369-446).

        Host logic, O((d-1) p m), with the reference's numpy primitives so that
        ties resolve identically (np.argpartition / np.argsort).
        """
        assert eigs.ndim == 1, "eigs must be a 1D KronMatrix"
        assert isinstance(n_eigs, (int, np.integer)), \
            "n_eigs=%s must be an integer" % repr(n_eigs)
        assert n_eigs >= 1, "must use at least 1 eigenvalue"
        assert n_eigs <= eigs.shape[0], "n_eigs > number of eigenvalues"
        assert mode == 'largest' or mode == 'smallest'
        if not log_expand and eigs.n > 10:
            warn('should use log option which will be more numerically stable')
        p = int(n_eigs)

        def extreme(vec):
            if vec.size <= p:
                return np.arange(vec.size), vec
            if mode == 'largest':
                ind = np.argpartition(vec, -p)[-p:]
            else:
                ind = np.argpartition(vec, p)[:p]
            return ind, vec[ind]

        loc, vals = extreme(np.asarray(eigs.K[0]))
        loc = loc.reshape((-1, 1))
        if log_expand:
            vals = np.log(vals)
        for i in range(1, eigs.n):
            Ki = np.asarray(eigs.K[i])
            if log_expand:
                cand = log_kron(a=vals, b=Ki, a_logged=True)
            else:
                cand = np.kron(vals, Ki)
            ind, vals = extreme(cand)
            prev = loc[np.floor_divide(ind, Ki.size), :]
            loc = np.hstack([prev.reshape((ind.size, -1)),
                             np.mod(ind, Ki.size).astype(prev.dtype).reshape((-1, 1))])
        gloc = None
        if compute_global_loc:
            gloc = np.zeros(loc.shape[0], dtype=int)
            stride = 1
            for i in reversed(range(eigs.n)):
                gloc = stride * loc[:, i] + gloc
                stride *= np.size(eigs.K[i])
        if sort:
            order = np.argsort(vals)[::-1]
            vals = vals[order]
            loc = loc[order]
            if gloc is not None:
                gloc = gloc[order]
        return loc, vals, gloc

    def get_col(self, pos):
        assert len(pos) == self.n
        assert np.size(pos[0]) == 1
        assert isinstance(pos[0], int)
        assert self.ndim == 2
        return KronMatrix([self.K[i][:, j].reshape((-1, 1)) for i, j in enumerate(pos)])

    def log_det(eig_vals):
        """log det from per-factor eigenvalues (kron_matrix.py:466-474)."""
        assert eig_vals.ndim == 1
        ldet = 0
        for i, eigs in enumerate(eig_vals.K):
            repetition = np.prod(np.delete(eig_vals.sshape, i))
            ldet += repetition * np.sum(np.log(eigs))
        return ldet

    def log_det_shifted(eig_vals, shift):
        """log det(K + shift I) = sum_grid log(prod lambda + shift), on the device.

        Extension of log_det (the reference covers only shift = 0); the grid
        sum is streamed on the device with the index decoded per element.
        """
        assert eig_vals.ndim == 1
        lam = [np.asarray(e, dtype=np.float64).reshape(-1) for e in eig_vals.K]
        lamd = dev.to_device(np.concatenate(lam))
        out = ctypes.c_double()
        native.check(native.lib().gg_kron_logdet_shifted(
            len(lam), native.i64_array([l.size for l in lam]), native.dptr(lamd), float(shift),
            ctypes.byref(out), native.stream_ptr()), "gg_kron_logdet_shifted")
        return out.value


class SelectionMatrixSparse(object):
    """Row selection with unique / inverse index (selection_matrix.py:55-107)."""
    ndim = 2

    def __init__(self, indicies):
        assert isinstance(indicies, tuple)
        assert len(indicies) == 2
        assert indicies[0].ndim == 1
        self.shape = [indicies[0].size, indicies[1]]
        self.indicies = indicies[0]
        self.unique, self.unique_inverse = np.unique(self.indicies, return_inverse=True)

    def mul(self, x):
        assert x.ndim == 2
        return x[self.indicies, :]
    dot = __mul__ = mul

    def mul_unique(self, x):
        assert x.ndim == 2
        return x[self.unique, :]

    def mul_T(self, x):
        raise NotImplementedError('Not finished')

    def __getitem__(self, key):
        if isinstance(key, tuple):
            key = key[0]
        return SelectionMatrixSparse(indicies=(np.atleast_1d(self.indicies[key]), self.shape[1]))


def _dev_rows(A):
    """(M, m) row-major float64 device matrix from numpy or a tensor."""
    t = dev.torch()
    if isinstance(A, t.Tensor):
        Ad = A.detach().to(t.float64)
        return (Ad if Ad.is_cuda else Ad.to(dev.device())).contiguous()
    return t.from_numpy(np.ascontiguousarray(np.asarray(A, dtype=np.float64))).to(dev.device())


class KhatriRaoMatrix(object):
    """Row-partitioned Khatri-Rao matrix (khatri_rao_matrix.py:7-50, partition
    0): row j is kron(A_0[j], ..., A_{d-1}[j]), A_f of shape (M, m_f), factor 0
    slowest -- the form GridKernel.cov_kr returns for K(X*, grid).  The product
    with an N-vector (BlockMatrix.__mul__, block_matrix.py:48-66) is the device
    contraction gg_kr_contract: one FP64 MFMA GEMM against the fastest factor
    plus a coalesced weighted column sum; the N-vector is read once per chunk.
    Column partitioning (partition=1) is off the grid-prediction path."""

    def __init__(self, A, partition=None):
        if partition != 0:
            raise NotImplementedError("only the row-partitioned (partition=0) form is provided")
        A = list(A)
        assert len(A) >= 1
        M = int(A[0].shape[0])
        for Ai in A:
            assert Ai.ndim == 2 and int(Ai.shape[0]) == M, "blocks must share the row count"
        self.A = A
        self.d = len(A)
        self.partition = 0
        self.block_shape = (M, 1)
        self.shape = (M, int(np.prod([int(Ai.shape[1]) for Ai in A])))
        self._tabs = None

    def _tables(self):
        if self._tabs is None:
            ulast = _dev_rows(self.A[-1])
            uts = [_dev_rows(Ai).t().contiguous() for Ai in self.A[:-1]]   # U_f^T (m_f x M)
            self._tabs = (ulast, uts)
        return self._tabs

    def contract(self, cd, out=None, work_elems=None):
        """out (M,) device = self . cd for a 1-D float64 device vector of length N.
        work_elems (optional) caps the scratch size (smaller = more GEMM chunks)."""
        L = native.lib()
        M, N = self.shape
        if int(cd.numel()) != N:
            raise ValueError('x is the wrong shape, must be (%d,1)' % N)
        ulast, uts = self._tables()
        m = [int(Ai.shape[1]) for Ai in self.A]
        marr = native.i64_array(m)
        need = ctypes.c_int64()
        native.check(L.gg_kr_work_elems(self.d, marr, M, ctypes.byref(need)))
        outer = N // m[-1]
        # d <= 8 runs the fused kernel (partials only); the two-pass path gets
        # up to ~1 GiB of GEMM chunk beyond the minimum: few chunks, modest HBM
        extra = 0 if self.d <= 8 else min(outer * M, max(0, (1 << 27) - need.value))
        if work_elems is not None:
            extra = max(0, int(work_elems) - need.value)
        work = dev.empty(need.value + extra)
        if out is None:
            out = dev.empty(M)
        ptrs = (ctypes.c_void_p * max(1, len(uts)))(*[native.dptr(u) for u in uts])
        native.check(L.gg_kr_contract(self.d, marr, native.dptr(dev.ensure_aligned(cd)),
                                      native.dptr(ulast), ptrs, M, native.dptr(out),
                                      native.dptr(work), int(work.numel()),
                                      native.stream_ptr()), "gg_kr_contract")
        return out

    def __mul__(self, x):
        M, N = self.shape
        if tuple(x.shape) != (N, 1):
            raise ValueError('x is the wrong shape, must be (%d,1), not %s' % (N, repr(x.shape)))
        xd, was_dev = _vector_in(x, N, 'x is the wrong shape')
        return _vector_out(self.contract(xd), was_dev)


class RowColKhatriRaoMatrix(object):
    """A = R K C with A[a, b] = prod_i (R_i K_i C_i)[a, b]
    (khatri_rao_matrix.py:53-178): R row-partitioned, C column-partitioned
    Khatri-Rao factors, K a Kronecker product (merged into C at construction,
    C_i <- K_i C_i, as the reference does).  The matrix is never formed whole:
    products and get_rows work on chunks of n_rows_at_once rows (the
    reference's nGb memory cap), each chunk = d FP64 MFMA GEMMs R_i[rows] C_i
    combined elementwise on the device (gg_kr_hadamard), then one GEMV."""

    def __init__(self, R, K, C, nGb=1.):
        R = list(R)
        C = list(C)
        self.d = len(R)
        if K is not None:
            K = list(K)
            assert len(K) == len(C) == self.d, "number of dims inconsistent"
        self._init_blocks([_dev_rows(Ri) for Ri in R],
                          [self._merge(K[i] if K is not None else None, C[i], R[i])
                           for i in range(self.d)], nGb)

    @staticmethod
    def _merge(Ki, Ci, Ri):
        from . import dense
        Cd = _dev_rows(Ci)
        if Ki is None:
            return Cd
        assert Ki.shape[0] == Ki.shape[1] == Ri.shape[1], \
            "K must be a square Kronecker product matrix, and must be consistent with R"
        return dense.matmul(_dev_rows(Ki), Cd)

    def _init_blocks(self, Rd, Cd, nGb):
        self._R, self._C = Rd, Cd
        for Ri, Ci in zip(Rd, Cd):
            assert int(Ri.shape[1]) == int(Ci.shape[0]), "inner dimensions differ"
            assert int(Ri.shape[0]) == int(Rd[0].shape[0])
            assert int(Ci.shape[1]) == int(Cd[0].shape[1])
        self.shape = (int(Rd[0].shape[0]), int(Cd[0].shape[1]))
        self.nGb = nGb
        self.n_rows_at_once = 1
        if nGb is not None:
            self.n_rows_at_once = max(1, int(np.floor(nGb * 1e9 / (8 * self.shape[1]))))

    @classmethod
    def _from_blocks(cls, Rd, Cd, nGb):
        obj = cls.__new__(cls)
        obj.d = len(Rd)
        RowColKhatriRaoMatrix._init_blocks(obj, Rd, Cd, nGb)
        return obj

    @property
    def T(self):
        """A^T = C^T K^T R^T: the same structure with R_i <- C_i^T, C_i <- R_i^T."""
        return RowColKhatriRaoMatrix._from_blocks([c.t().contiguous() for c in self._C],
                                                  [r.t().contiguous() for r in self._R],
                                                  self.nGb)

    def _rows_dev(self, Rsel, logged):
        """Device rows for the row blocks Rsel[i] (k x m_i): product or (log, sign)."""
        from . import dense
        L = native.lib()
        t = dev.torch()
        k, n = int(Rsel[0].shape[0]), self.shape[1]
        P = t.empty((k, n), dtype=t.float64, device=self._C[0].device)
        S = t.empty((k, n), dtype=t.float64, device=P.device) if logged else None
        X = t.empty((k, n), dtype=t.float64, device=P.device) if self.d > 1 or logged else P
        for i in range(self.d):
            Xi = dense.matmul(Rsel[i], self._C[i], C=X if (self.d > 1 or logged) else P)
            if self.d > 1 or logged:
                native.check(L.gg_kr_hadamard(k * n, native.dptr(Xi), native.dptr(P),
                                              native.dptr(S) if logged else None,
                                              int(logged), int(i == 0), native.stream_ptr()),
                             "gg_kr_hadamard")
        return (P, S) if logged else P

    def get_rows(self, i_rows, logged=False):
        """Rows i_rows (index array or slice) of A, as host arrays (:110-140)."""
        idx = np.arange(self.shape[0])[i_rows]
        idx = np.atleast_1d(idx)
        t = dev.torch()
        it = t.from_numpy(np.ascontiguousarray(idx, dtype=np.int64)).to(self._R[0].device)
        Rsel = [Ri.index_select(0, it).contiguous() for Ri in self._R]
        out = self._rows_dev(Rsel, logged)
        if logged:
            return dev.to_host(out[0]), dev.to_host(out[1])
        return dev.to_host(out)

    def expand(self, logged=False):
        return self.get_rows(slice(None), logged=logged)

    def __mul__(self, x):
        """y = A x chunk by chunk of rows (:143-158)."""
        from . import dense
        if tuple(x.shape) != (self.shape[1], 1):
            raise AssertionError("x must be (%d,1)" % self.shape[1])
        xd, was_dev = _vector_in(x, self.shape[1], 'x is the wrong shape')
        y = dev.empty(self.shape[0])
        step = self.n_rows_at_once
        for i0 in range(0, self.shape[0], step):
            i1 = min(self.shape[0], i0 + step)
            P = self._rows_dev([Ri[i0:i1] for Ri in self._R], False)
            dense.matvec(P, xd, y=y[i0:i1])
        return _vector_out(y, was_dev)


class RowColKhatriRaoMatrixTransposed(RowColKhatriRaoMatrix):
    """(R K C)^T handled as rows of the transpose (khatri_rao_matrix.py:181-210):
    shape (N, p), products A^T x; .T returns the untransposed matrix."""

    def __init__(self, R, K, C, nGb=1.):
        base = RowColKhatriRaoMatrix(R, K, C, nGb=None)
        self.d = base.d
        self._untransposed = (base._R, base._C)
        RowColKhatriRaoMatrix._init_blocks(self, [c.t().contiguous() for c in base._C],
                                           [r.t().contiguous() for r in base._R], nGb)

    @property
    def T(self):
        R, C = self._untransposed
        return RowColKhatriRaoMatrix._from_blocks(R, C, self.nGb)


# ------------------------------------------------------------ structure helpers
# The reference's small composition classes (selection_matrix.py:6-52,
# tensors.py:6-94, block_matrix.py:4-96).  They hold no arithmetic of their own:
# every product is delegated to the operands (KronMatrix / KhatriRaoMatrix
# products run on the device), so they are kept as host bookkeeping for the
# drop-in import surface.

class SelectionMatrix(object):
    """One nonzero per row: (S x)[r] = x[idx[r]] (selection_matrix.py:6-52).
    `indicies`: a bool mask (its True positions, in order) or (int_idx, size)."""
    ndim = 2

    def __init__(self, indicies):
        if isinstance(indicies, tuple):
            assert len(indicies) == 2
            assert indicies[0].ndim == 1
            self.shape = [indicies[0].size, indicies[1]]
            self.idx = np.asarray(indicies[0], dtype=np.int64)
        else:
            assert indicies.ndim == 1
            assert indicies.dtype == bool
            self.shape = [int(np.count_nonzero(indicies)), indicies.size]
            self.idx = np.nonzero(indicies)[0]

    def mul(self, x):
        return x[self.idx]

    def mul_T(self, x):
        """S^T x: scatter-add of the rows of x into a zero (size, ...) array."""
        if dev.is_device_array(x):
            t = dev.torch()
            out = t.zeros((self.shape[1],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
            return out.index_add_(0, t.as_tensor(self.idx, device=x.device), x)
        out = np.zeros((self.shape[1],) + np.shape(x)[1:], dtype=np.result_type(x))
        np.add.at(out, self.idx, x)
        return out


class Array(object):
    """Wraps a plain matrix so it composes with the tensor classes (tensors.py:77-94)."""

    def __init__(self, A):
        self.A = A
        self.shape = A.shape

    def __mul__(self, x):
        return self.A.dot(x)

    @property
    def T(self):
        return Array(self.A.T)

    def expand(self):
        return self.A


class TensorProduct(object):
    """(T_0 T_1 ... T_{k-1}) x applied right to left, never expanded (tensors.py:6-38)."""

    def __init__(self, tensor_list):
        self.tensors = tensor_list
        self.n_tensors = len(tensor_list)
        self.shape = (self.tensors[0].shape[0], self.tensors[-1].shape[1])
        for a, b in zip(self.tensors[:-1], self.tensors[1:]):
            assert a.shape[1] == b.shape[0]

    @property
    def T(self):
        raise NotImplementedError('easy to do this')

    def __mul__(self, x):
        assert x.shape == (self.shape[1], 1), "vector is wrong shape"
        for T in reversed(self.tensors):
            x = T * x
        return x


class TensorSum(object):
    """(T_0 + ... + T_{k-1}) x without expansion (tensors.py:41-74)."""

    def __init__(self, tensor_list):
        self.tensors = tensor_list
        self.n_tensors = len(tensor_list)
        self.shape = self.tensors[0].shape
        for a in self.tensors[1:]:
            assert np.array_equal(np.asarray(a.shape), np.asarray(self.shape))

    @property
    def T(self):
        raise NotImplementedError('easy to do this')

    def __mul__(self, x):
        assert x.shape == (self.shape[1], 1), "vector is wrong shape"
        y = None
        for T in self.tensors:
            v = T * x
            y = v if y is None else y + v
        return y


class BlockMatrix(object):
    """Matrix of blocks; products block row by block row (block_matrix.py:4-96).
    A: 2-D object array of blocks with shape, __mul__, T and expand."""

    def __init__(self, A):
        assert A.ndim == 2, 'A must be 2d'
        self.A = A
        self.block_shape = A.shape
        self._partition_shape = ([int(b.shape[0]) for b in A[:, 0]],
                                 [int(b.shape[1]) for b in A[0, :]])
        self.shape = tuple(int(np.sum(s)) for s in self._partition_shape)
        for i in range(self.block_shape[0]):
            for j in range(self.block_shape[1]):
                assert tuple(A[i, j].shape) == self.partition_shape(i, j), \
                    "A[%d,%d].shape should be %s, not %s" % (
                        i, j, repr(self.partition_shape(i, j)), repr(A[i, j].shape))
        self.vec_split = np.cumsum([0] + self._partition_shape[1], dtype='i')

    def partition_shape(self, i, j):
        return (self._partition_shape[0][i], self._partition_shape[1][j])

    def __mul__(self, x):
        assert x.shape == (self.shape[1], 1)
        cut = self.vec_split
        xs = [x[cut[j]:cut[j + 1]] for j in range(self.block_shape[1])]
        rows = []
        for i in range(self.block_shape[0]):
            acc = None
            for j in range(self.block_shape[1]):
                v = self.A[i, j] * xs[j]
                acc = v if acc is None else acc + v
            rows.append(acc)
        if dev.is_device_array(rows[0]):
            return dev.torch().cat(rows, 0)
        return np.concatenate(rows, axis=0)

    def transpose(self):
        At = np.empty(self.block_shape[::-1], dtype=object)
        for i in range(self.block_shape[0]):
            for j in range(self.block_shape[1]):
                At[j, i] = self.A[i, j].T
        return self.__class__(A=At)
    T = property(transpose)

    def expand(self):
        out = np.zeros(self.shape)
        rs = np.cumsum([0] + self._partition_shape[0])
        cs = np.cumsum([0] + self._partition_shape[1])
        for i in range(self.block_shape[0]):
            for j in range(self.block_shape[1]):
                out[rs[i]:rs[i + 1], cs[j]:cs[j + 1]] = self.A[i, j].expand()
        return out


def expand_SKC(S, K, C, logged=True):
    """Rows of (selection Khatri-Rao) x (Kronecker) x (column Khatri-Rao), the
    GRIEF eigenfunction core (tensors.py:97-128).

    S: list of SelectionMatrixSparse (p rows each); K: list of m_i x m_i (the
    grid eigenvector factors transposed); C: list of m_i x n cross covariances.
    Per factor only the unique selected rows are formed, X_i = K_i[unique_i] C_i
    (FP64 MFMA GEMM), then one device pass gathers them through the inverse
    indices into the p x n result: (sum log|X|, prod sign) with the sign taken
    before zeros are replaced (logged), or prod X.  numpy in -> numpy out;
    CUDA tensors stay on the device.
    """
    from . import dense
    assert isinstance(S, (list, np.ndarray))
    assert isinstance(S[0], SelectionMatrixSparse)
    assert isinstance(K, (list, np.ndarray))
    assert isinstance(C, (list, np.ndarray))
    t = dev.torch()
    on_dev = dev.is_device_array(C[0])
    rows, cols, row0 = [], [], 0
    for s, k, c in zip(S, K, C):
        kd = _dev_rows(k)[t.as_tensor(s.unique, device=dev.device())]
        rows.append(dense.matmul(kd, _dev_rows(c)))               # u_i x n
        cols.append(row0 + np.asarray(s.unique_inverse, dtype=np.int64).reshape(-1))
        row0 += int(np.size(s.unique))
    X = t.cat(rows, 0).contiguous()
    n = int(X.shape[1])
    p = int(np.size(cols[0]))
    d = len(cols)
    cidx = t.as_tensor(np.stack(cols, axis=1).astype(np.int32), device=X.device).contiguous()
    out = dev.empty(p * n)
    sign = t.empty(p * n, dtype=t.int32, device=X.device) if logged else None
    native.check(native.lib().gg_expand_skc(
        native.dptr(X), row0, n, native.dptr(cidx), d, p, int(bool(logged)), native.dptr(out),
        native.dptr(sign) if logged else None, native.stream_ptr()), "gg_expand_skc")
    out = out.reshape(p, n)
    if logged:
        sign = sign.reshape(p, n)
        return (out, sign) if on_dev else (dev.to_host(out), dev.to_host(sign))
    return out if on_dev else dev.to_host(out)
