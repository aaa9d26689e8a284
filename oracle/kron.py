"""Kronecker-structured linear algebra -- CPU oracle (test infrastructure only).

Each function restates one reference routine of
/root/reference/gp_grief/tensors/kron_matrix.py or gp_grief/linalg.py; the
citation is in its docstring.  Index convention (kron_matrix.py:19-42, np.kron):
the flattened vector is a C-order tensor over the factor list, factor 0 the
slowest axis.  (GridKernel.cov_grid reverses the input dimensions,
grid_kernel.py:109, so input dimension 0 ends up fastest.)
"""
import numpy as np


def kron_matvec(factors, x):
    """y = (K_0 (x) K_1 (x) ... (x) K_{d-1}) x.

    Restates KronMatrix.kronvec_prod (kron_matrix.py:52-97): one GEMM per
    factor.  Each step contracts the slowest remaining axis against K_k and
    appends the new axis as the fastest one, so after d steps the axes are back
    in order (the reference gets the same rotation from its F-order reshapes
    and transposes).  BLAS3 via numpy.matmul, threads from OpenBLAS.
    """
    y = np.ascontiguousarray(x, dtype=np.float64).reshape(-1)
    ncols = int(np.prod([np.shape(k)[1] for k in factors]))
    if y.size != ncols:
        raise ValueError('x is the wrong shape, must be (%d,1), not %s'
                         % (ncols, repr(np.shape(x))))
    for K in factors:
        K = np.asarray(K, dtype=np.float64)
        p, q = K.shape
        Y = y.reshape(q, -1)
        y = np.matmul(Y.T, K.T).reshape(-1)
    return y


def kron_matvec_dsymm(factors, x):
    """y = (K_0 (x) ... (x) K_{d-1}) x for symmetric factors, in the reference's
    own BLAS call sequence -- the CPU baseline of bench.py.

    Restates the `sym` branch of KronMatrix.kronvec_prod
    (kron_matrix.py:74-96): factors are visited last to first; each step views
    the running vector as (m_i, N/m_i) in Fortran order (a copy whenever the
    previous transpose left it C-ordered), applies BLAS3 dsymm with the factor
    on the left (side=0) or, for a C-ordered operand, on the right (side=1),
    and keeps the transposed product.  Same arithmetic as kron_matvec; the
    point is the cost profile (F-order copies + dsymm) of the reference.
    """
    from scipy.linalg import blas
    y = np.asarray(x, dtype=np.float64).reshape(-1, 1)
    for K in reversed(list(factors)):
        K = np.asarray(K, dtype=np.float64)
        a = K if np.isfortran(K) else K.T     # symmetric: either is K
        y = np.reshape(y, (K.shape[1], -1), order='F')
        if np.isfortran(y):
            y = blas.dsymm(1.0, a, y, side=0).T
        else:
            y = blas.dsymm(1.0, a, y.T, side=1)
    return y.reshape(-1, order='F')


def kron_matvec_entries(factors, x, idx):
    """Selected entries (K x)[idx] of a Kronecker matvec without forming K x.

    Entry i of (K_0 (x) ... (x) K_{d-1}) x is x (as the C-order tensor over the
    factors, factor 0 slowest) contracted with row i_k of every K_k -- the
    definition of the Kronecker product (np.kron order, kron_matrix.py:19-42).
    Entries sharing i_0 share the first (N-flop) contraction, so a handful of
    entries of a 200^4 product cost a few GEMVs over x.  For spot checks of a
    full-size device matvec against the reference arithmetic.
    """
    F = [np.asarray(K, dtype=np.float64) for K in factors]
    shape = [K.shape[1] for K in F]
    X = np.asarray(x, dtype=np.float64).reshape(shape)
    rows = [np.unravel_index(int(i), [K.shape[0] for K in F]) for i in np.ravel(idx)]
    out = np.empty(len(rows))
    cache = {}
    for n, r in enumerate(rows):
        if r[0] not in cache:
            cache[r[0]] = np.tensordot(F[0][r[0]], X, axes=(0, 0))
        t = cache[r[0]]
        for k in range(1, len(F)):
            t = np.tensordot(F[k][r[k]], t, axes=(0, 0))
        out[n] = float(t)
    return out


def kron_matvec_T(factors, x):
    """(K_0 (x) ... )^T x -- KronMatrix.transpose (kron_matrix.py:203-213) then *."""
    return kron_matvec([np.asarray(k).T for k in factors], x)


def kron_expand(factors):
    """Dense expansion, KronMatrix.expand (kron_matrix.py:215-239), 1-D or 2-D."""
    out = np.ones((1,) * np.ndim(factors[0]))
    for K in factors:
        out = np.kron(out, np.asarray(K))
    return out.reshape(-1) if np.ndim(factors[0]) == 1 else out


def log_kron(a, b, a_logged=False, b_logged=False):
    """log(kron(a, b)) for 1-D a, b -- linalg.log_kron (linalg.py:74-89)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.ndim != 1 or b.ndim != 1:
        raise AssertionError("currenly only working for 1d arrays")
    la = a if a_logged else np.log(a)
    lb = b if b_logged else np.log(b)
    return np.add.outer(la, lb).reshape(-1)


def find_extremum_eigs(eig_factors, n_eigs, mode='largest', log_expand=False,
                       sort=True, compute_global_loc=False):
    """Top/bottom-p entries of a 1-D Kronecker vector by sequential pruning.

    Restates KronMatrix.find_extremum_eigs (kron_matrix.py:369-446): after each
    factor only the n_eigs extreme partial products survive (np.argpartition,
    the same primitive, so ties break identically), positions are tracked per
    factor, and the survivors are finally sorted descending with np.argsort.
    Returns (eig_loc [p x d] int, eig_vals [p], global_loc or None).
    """
    if mode not in ('largest', 'smallest'):
        raise AssertionError("mode must be largest or smallest")
    p = int(n_eigs)

    def extreme(vec):
        if vec.size <= p:
            return np.arange(vec.size), vec
        if mode == 'largest':
            ind = np.argpartition(vec, -p)[-p:]
        else:
            ind = np.argpartition(vec, p)[:p]
        return ind, vec[ind]

    f0 = np.asarray(eig_factors[0], dtype=np.float64)
    loc, vals = extreme(f0)
    loc = loc.reshape((-1, 1))
    if log_expand:
        vals = np.log(vals)
    for f in eig_factors[1:]:
        f = np.asarray(f, dtype=np.float64)
        if log_expand:
            cand = np.add.outer(vals, np.log(f)).reshape(-1)
        else:
            cand = np.multiply.outer(vals, f).reshape(-1)
        ind, vals = extreme(cand)
        prev = loc[ind // f.size, :]
        loc = np.hstack([prev.reshape((ind.size, -1)),
                         (ind % f.size).astype(prev.dtype).reshape((-1, 1))])
    gloc = None
    if compute_global_loc:
        gloc = np.zeros(loc.shape[0], dtype=np.int64)
        stride = 1
        for i in range(len(eig_factors) - 1, -1, -1):
            gloc = gloc + stride * loc[:, i]
            stride *= np.size(eig_factors[i])
    if sort:
        order = np.argsort(vals)[::-1]
        vals = vals[order]
        loc = loc[order]
        if gloc is not None:
            gloc = gloc[order]
    return loc, vals, gloc


def factor_eigh(factors):
    """Per-factor symmetric eigendecomposition (Q_i, lambda_i).

    The reference uses a real Schur form per factor (KronMatrix.schur,
    kron_matrix.py:161-171; LAPACK gees), whose T is diagonal for symmetric
    factors; numpy.linalg.eigh gives the same pairs up to ordering, column
    sign and rounding.  Every quantity the tests compare is invariant to those.
    """
    Q, lam = [], []
    for K in factors:
        w, v = np.linalg.eigh(np.asarray(K, dtype=np.float64))
        Q.append(v)
        lam.append(w)
    return Q, lam


def solve_schur(Q, t, x, shift=0.0):
    """(K + shift I)^{-1} x = Q ((Q^T x) / (t + shift)) -- kron_matrix.py:328-352."""
    y = kron_matvec_T(Q, x)
    y = y / (np.asarray(t).reshape(-1) + shift)
    return kron_matvec(Q, y)


def eig_log_det(eig_factors):
    """log det of K from per-factor eigenvalues -- KronMatrix.log_det (:466-474)."""
    sizes = np.array([np.size(e) for e in eig_factors], dtype=np.float64)
    total = np.prod(sizes)
    return float(sum((total / sizes[i]) * np.sum(np.log(e))
                     for i, e in enumerate(eig_factors)))


def _partial_products(eig_factors):
    out = np.ones(1)
    for e in eig_factors:
        out = np.multiply.outer(out, np.asarray(e, dtype=np.float64)).reshape(-1)
    return out


def logdet_shifted(eig_factors, shift, chunk_last=True):
    """log det(K + shift I) = sum_N log(prod_i lambda_i + shift).

    The reference offers only the unshifted log det (kron_matrix.py:466-474);
    the survey's verified recipe is sum(log(T.diag().expand()+s)).
    Streamed over the last factor so that N-sized arrays are never formed.
    """
    head = _partial_products(eig_factors[:-1])
    acc = 0.0
    for lam in np.asarray(eig_factors[-1], dtype=np.float64):
        acc += float(np.sum(np.log(head * lam + shift)))
    return acc


def grid_latent_var(Q, eig_factors, shift):
    """diag(K - K (K + s I)^{-1} K) on the grid = (Q o Q)-Kron * (t s / (t + s)).

    Composed from reference primitives (KronMatrix([Q_i**2]) times
    the expanded eigenvalue vector); the reference has no single routine.
    """
    t = _partial_products(eig_factors)
    return kron_matvec([np.asarray(q) ** 2 for q in Q], t * shift / (t + shift))


def kr_contract(blocks, c):
    """out[j] = kron(A_0[j], ..., A_{d-1}[j]) . c for a row-partitioned
    Khatri-Rao matrix (khatri_rao_matrix.py:7-50; BlockMatrix.__mul__
    block_matrix.py:48-66 applies it one KronMatrix row at a time).  Here each
    row is contracted factor by factor: the slowest axis first, as a small GEMV."""
    M = blocks[0].shape[0]
    shape = [b.shape[1] for b in blocks]
    C = np.asarray(c, dtype=np.float64).reshape(shape)
    out = np.empty(M)
    for j in range(M):
        t = C
        for b in blocks:
            t = np.tensordot(b[j], t, axes=(0, 0))
        out[j] = float(t)
    return out


def grid_offgrid_predict(factors, cross_blocks, kss, alpha, shift):
    """Off-grid posterior of a full-grid GP (the f8 fixture's recipe,
    grid_kernel.py:148-179 + kron_matrix.py:328-352): mean = K(X*, grid) alpha;
    latent var = k** - sum_g (prod_f (Q_f^T k_f(x*))[g_f])^2 / (prod_f t_f[g_f] + s)."""
    Q, t = factor_eigh(factors)
    mean = kr_contract(cross_blocks, alpha)
    lam = t[0]
    for ti in t[1:]:
        lam = np.multiply.outer(lam, ti).reshape(-1)
    cinv = 1.0 / (lam + shift)
    V2 = [(b.dot(q)) ** 2 for b, q in zip(cross_blocks, Q)]
    return mean, kss - kr_contract(V2, cinv)


def rowcol_kr_expand(R, K, C, logged=False):
    """A[a, b] = prod_i X_i[a, b], X_i = R_i (K_i C_i) -- RowColKhatriRaoMatrix
    (khatri_rao_matrix.py:53-158: C_i <- K_i C_i at construction, get_rows /
    expand).  logged: (log|A| accumulated until the running sign hits 0, sign)
    with the reference's running-sign rule (:127-133)."""
    if logged:
        log, sign = 0., 1.
    else:
        prod = 1.
    for Ri, Ki, Ci in zip(R, K, C):
        X = Ri.dot(Ki.dot(Ci) if Ki is not None else Ci)
        if logged:
            sign = sign * np.int32(np.sign(X))
            X = X.copy()
            X[sign == 0] = 1.
            log = log + np.log(np.abs(X))
        else:
            prod = prod * X
    return (log, sign) if logged else prod


# ---------------------------------------------------------- parity-block basis
# No reference routine: the build's change of basis for centrosymmetric
# factors.  Restated here (test infrastructure) so the
# device fold / block operator can be checked against the dense product of
# kron_matvec (kron_matrix.py:52-97), which itself is reference-pinned.

def _slab_perm(hr, hc):
    """pos[i hc + a] = (a // 4) 4 hr + w i + a % 4, w = min(4, hc - 4 (a // 4))
    (the last column group narrower when hc % 4 != 0: host-only shapes)."""
    i, a = np.meshgrid(np.arange(hr), np.arange(hc), indexing="ij")
    q = a // 4
    w = np.minimum(4, hc - 4 * q)
    return (q * 4 * hr + w * i + a % 4).reshape(-1)


def slab_tile(xb, hs, inverse=False):
    """The block layout's k-step tiling of each slab (gg_kronb.hip header): the
    two innermost axes (hr x hc) of every block, C-order element (i, a) at
    position (a // 4) 4 hr + 4 i + a % 4 (whole 4-column groups; the device
    block basis has hc = 16 TF + 4).  inverse=True undoes it."""
    hr, hc = int(hs[-2]), int(hs[-1])
    pos = _slab_perm(hr, hc)
    t = np.asarray(xb, dtype=np.float64).reshape(-1, hr * hc)
    out = np.empty_like(t)
    if inverse:
        out[:, :] = t[:, pos]
    else:
        out[:, pos] = t
    return out.reshape(-1)


def block_pad(h):
    """The device's slab extent for pair axes of half order h (gg_kronb.hip
    block_create, round 6): the smallest 16 TF + 4 >= h, TF >= 1 -- the pair
    kernels' shape; the rows / columns past h are zero."""
    h = int(h)
    return 16 * max(1, -(-(h - 4) // 16)) + 4


def block_extents(ms, pad=False):
    """The block layout's per-axis extents: h_k = m_k / 2, the two innermost
    padded to block_pad when pad (the device layout)."""
    hs = [int(m) // 2 for m in ms]
    if pad:
        hs[-2], hs[-1] = block_pad(hs[-2]), block_pad(hs[-1])
    return hs


def block_fold(x, ms, inverse=False, pad=False):
    """P x for the orthogonal per-axis butterfly u_i = (x_i + x_{m-1-i}) / sqrt 2,
    v_i = (x_i - x_{m-1-i}) / sqrt 2 (i < m/2) on every axis (C order, factor 0
    slowest).  Block layout: parity pattern beta (bit d-1-k for axis k) slowest,
    then (i'_0 .. i'_{d-3}) C order, each slab (i'_{d-2}, i'_{d-1}) k-step tiled
    (slab_tile).  inverse=True applies P^T (block -> grid).  pad: the two
    innermost axes zero-padded to block_pad(h) (the device layout for pair
    orders that are not 16 TF + 4; a no-op for those that are).
    """
    ms = [int(m) for m in ms]
    d = len(ms)
    hs = [m // 2 for m in ms]
    es = block_extents(ms, pad)
    s = 1.0 / np.sqrt(2.0)
    if pad and es != hs:
        if not inverse:
            nb = int(np.prod(hs))
            y = slab_tile(block_fold(x, ms), hs, inverse=True)
            out = np.zeros((2 ** d,) + tuple(es))
            out[(slice(None),) + tuple(slice(0, h) for h in hs)] = y.reshape((2 ** d,) + tuple(hs))
            return slab_tile(out.reshape(-1), es)
        y = slab_tile(np.asarray(x, dtype=np.float64), es, inverse=True)
        y = y.reshape((2 ** d,) + tuple(es))[(slice(None),) + tuple(slice(0, h) for h in hs)]
        return block_fold(slab_tile(np.ascontiguousarray(y).reshape(-1), hs), ms, inverse=True)
    if not inverse:
        t = np.asarray(x, dtype=np.float64).reshape(ms)
        # per axis: [lo half ; reversed hi half] -> (even, odd) stacked on a new
        # leading parity axis; the parity axes collect in front in axis order
        parts = [t]
        for k in range(d):
            nxt = []
            for a in parts:
                lo = np.take(a, np.arange(hs[k]), axis=k)
                hi = np.take(a, np.arange(ms[k] - 1, hs[k] - 1, -1), axis=k)
                nxt.append((lo + hi) * s)
                nxt.append((lo - hi) * s)
            parts = nxt
        return slab_tile(np.concatenate([p.reshape(-1) for p in parts]), hs)
    nb = int(np.prod(hs))
    y = slab_tile(x, hs, inverse=True)
    parts = [y[b * nb:(b + 1) * nb].reshape(hs) for b in range(2 ** d)]
    for k in reversed(range(d)):
        nxt = []
        for j in range(0, len(parts), 2):
            e, o = parts[j], parts[j + 1]
            lo = (e + o) * s
            hi = (e - o) * s
            nxt.append(np.concatenate([lo, np.flip(hi, axis=k)], axis=k))
        parts = nxt
    return parts[0].reshape(-1)


def block_factors(F):
    """(S, T) of a centrosymmetric factor of even order: S[j][i] = F[j][i] +
    F[j][m-1-i], T[j][i] = F[j][i] - F[j][m-1-i] (j, i < m/2)."""
    F = np.asarray(F, dtype=np.float64)
    m = F.shape[0]
    h = m // 2
    Fr = F[:h, ::-1][:, :h]          # F[j][m-1-i]
    return F[:h, :h] + Fr, F[:h, :h] - Fr


def block_matvec(factors, xb, pad=False):
    """(P K P^T) x_b in the block layout: block beta is the Kronecker product of
    S_k (beta_k = 0) / T_k (beta_k = 1) (kron_matvec on each block).  pad: the
    device layout (block_fold's pad; the factors zero-padded alike)."""
    d = len(factors)
    hs = block_extents([np.shape(F)[0] for F in factors], pad)
    st = []
    for F, e in zip(factors, hs):
        S, T = block_factors(F)
        if S.shape[0] != e:
            Sp, Tp = np.zeros((e, e)), np.zeros((e, e))
            Sp[:S.shape[0], :S.shape[0]], Tp[:S.shape[0], :S.shape[0]] = S, T
            S, T = Sp, Tp
        st.append((S, T))
    nb = int(np.prod(hs))
    xb = slab_tile(xb, hs, inverse=True)
    out = np.empty_like(xb)
    for b in range(2 ** d):
        fs = [st[k][(b >> (d - 1 - k)) & 1] for k in range(d)]
        out[b * nb:(b + 1) * nb] = kron_matvec(fs, xb[b * nb:(b + 1) * nb])
    return slab_tile(out, hs)
