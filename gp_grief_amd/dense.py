"""Thin device wrappers over the dense FP64 C ABI (gg_gemm / gg_gemv / gg_potrf /
gg_potrs) used by the GRIEF models.  All operands are row-major float64 CUDA
tensors; nothing here computes on the host."""
import ctypes

import numpy as np

from . import device as dev
from . import native


def _lib():
    return native.lib()


def matmul(A, B, ta=False, tb=False, alpha=1.0, beta=0.0, C=None, uplo=0, splitk=True):
    """C = alpha op(A) op(B) + beta C on FP64 MFMA (2-D tensors, row-major)."""
    t = dev.torch()
    A = A.contiguous()
    B = B.contiguous()
    M = A.shape[1] if ta else A.shape[0]
    K = A.shape[0] if ta else A.shape[1]
    Kb = B.shape[1] if tb else B.shape[0]
    N = B.shape[0] if tb else B.shape[1]
    if K != Kb:
        raise ValueError("inner dimensions differ: %d vs %d" % (K, Kb))
    if C is None:
        C = t.empty((M, N), dtype=t.float64, device=A.device)
        beta = 0.0
    work = None
    welems = 0
    if splitk and K >= 4096:
        # exactly the slabs gg_gemm will use for this call (none when the tile
        # grid alone fills the GPU evenly): no oversized, never-touched workspace
        need = ctypes.c_int64()
        native.check(_lib().gg_gemm_workspace_elems(int(ta), int(tb), int(M), int(N), int(K),
                                                    int(uplo), ctypes.byref(need)))
        welems = need.value
        work = dev.empty(welems) if welems > 0 else None
    native.check(_lib().gg_gemm(int(ta), int(tb), int(M), int(N), int(K), float(alpha),
                                native.dptr(A), A.shape[1], native.dptr(B), B.shape[1],
                                float(beta), native.dptr(C), C.shape[1], int(uplo),
                                native.dptr(work) if work is not None else None, int(welems),
                                native.stream_ptr()), "gg_gemm")
    return C


def matvec(A, x, trans=False, alpha=1.0, beta=0.0, y=None):
    """y = alpha op(A) x + beta y for a 2-D A and 1-D x (HBM-bound GEMV kernels)."""
    A = A.contiguous()
    R, Cn = A.shape
    n_out = Cn if trans else R
    if y is None:
        y = dev.empty(n_out)
        beta = 0.0
    work = dev.empty(2048 * Cn) if trans else None
    native.check(_lib().gg_gemv(int(trans), int(R), int(Cn), float(alpha), native.dptr(A),
                                int(Cn), native.dptr(x.contiguous()), float(beta),
                                native.dptr(y), native.dptr(work) if work is not None else None,
                                int(work.numel()) if work is not None else 0,
                                native.stream_ptr()), "gg_gemv")
    return y


def dot(x, y):
    out = ctypes.c_double()
    native.check(_lib().gg_dot(native.dptr(x), native.dptr(y), int(x.numel()),
                               ctypes.byref(out), native.stream_ptr()), "gg_dot")
    return out.value


class Cholesky(object):
    """P = L L^T on the device (lower, in place on a copy of P)."""

    def __init__(self, P):
        n = int(P.shape[0])
        self.n = n
        self.L = P.contiguous().clone()
        we = ctypes.c_int64()
        native.check(_lib().gg_potrf_work_elems(n, ctypes.byref(we)))
        self.winv = dev.empty(we.value)
        ld = ctypes.c_double()
        native.check(_lib().gg_potrf(n, native.dptr(self.L), n, native.dptr(self.winv),
                                     ctypes.byref(ld), native.stream_ptr()), "gg_potrf")
        self.logdet = ld.value

    def solve(self, B, which=3):
        """P^-1 B (which 3), L^-1 B (1) or L^-T B (2); B is (n,) or (n, r); returns new.
        which | 4: B is lower triangular (forward only; L^-1 of the identity)."""
        t = dev.torch()
        X = B.contiguous().clone()
        r = 1 if X.dim() == 1 else int(X.shape[1])
        tmp = dev.empty(64 * max(r, 1))
        native.check(_lib().gg_potrs(self.n, r, native.dptr(self.L), self.n,
                                     native.dptr(self.winv), native.dptr(X), r, int(which),
                                     native.dptr(tmp), native.stream_ptr()), "gg_potrs")
        del t
        return X

    def inverse(self):
        """L^-1 (lower; the strict upper triangle is zero), gg_trtri."""
        t = dev.torch()
        X = t.zeros((self.n, self.n), dtype=t.float64, device=self.L.device)
        native.check(_lib().gg_trtri(self.n, native.dptr(self.L), self.n, native.dptr(self.winv),
                                     native.dptr(X), self.n, native.stream_ptr()), "gg_trtri")
        return X

    def inverse_diag(self):
        """diag(P^-1) = column sums of squares of L^-1."""
        Linv = self.inverse()
        out = dev.empty(self.n)
        native.check(_lib().gg_colsumsq_lower(self.n, native.dptr(Linv), self.n,
                                              native.dptr(out), native.stream_ptr()))
        return out


def add_diag(A, s, w=None):
    """P = A + diag(s / w) (w a device vector or None)."""
    n = int(A.shape[0])
    P = dev.torch().empty_like(A)
    native.check(_lib().gg_add_diag(n, native.dptr(A.contiguous()), n, float(s),
                                    native.dptr(w) if w is not None else None, native.dptr(P),
                                    n, native.stream_ptr()), "gg_add_diag")
    return P


def axpby(a, x, b, y):
    native.check(_lib().gg_axpby(float(a), native.dptr(x), float(b), native.dptr(y),
                                 int(x.numel()), native.stream_ptr()), "gg_axpby")
    return y


def scale_rows(A, w, mode=0):
    """In place: rows of A (2-D, or a 1-D vector) times w (mode 0) / over w (1); 2 = square."""
    rows = int(A.shape[0])
    cols = 1 if A.dim() == 1 else int(A.shape[1])
    native.check(_lib().gg_scale_rows(native.dptr(A), rows, cols,
                                      native.dptr(w) if w is not None else None, int(mode),
                                      native.stream_ptr()), "gg_scale_rows")
    return A


def host(x):
    return np.asarray(dev.to_host(x))
