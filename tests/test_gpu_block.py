"""The Kronecker operator in its parity-block basis on the MI355X (gg_kronb.hip).

Every factor F of a stationary kernel on an evenly spaced grid is
centrosymmetric (J F J = F); in the orthogonal basis P of per-axis
even / odd butterflies the operator is block diagonal over the 2^d parity
patterns.  The device computes P x (the fold), the
block operator P K P^T (d - 1 launches: in-place mode products on axes
0..d-3 and one launch for the two innermost axes of every block), and runs
the fused CG there.  Parity is against the reference's product
KronMatrix.kronvec_prod (gp_grief/tensors/kron_matrix.py:52-97) through the
oracle: unfold(block_matvec(fold x)) vs oracle.kron_matvec at 1e-13
relative, the device fold vs the oracle's restatement at 1e-15, and CG
solves vs the oracle CG (iterations within 2 %, x to 1e-8).
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def gg(gpu):
    import gp_grief_amd
    return gp_grief_amd


def grid_factor(m, ell=0.15, kind="RBF"):
    g = np.linspace(0.0, 1.0, m)
    return oracle.cov_1d(kind, g, g, 1.0, ell) + 1e-12 * np.eye(m)


def factors(ms, seed=0):
    kinds = ["RBF", "Matern52", "RBF", "Matern32", "RBF", "Exponential"]
    return [grid_factor(m, 0.1 + 0.03 * k + 0.01 * seed, kinds[k % len(kinds)])
            for k, m in enumerate(ms)]


def dev(gg, x):
    return gg.device.to_device(np.ascontiguousarray(x, dtype=np.float64).reshape(-1))


def host(gg, xd):
    return gg.device.to_host(xd).reshape(-1)


# shapes: d = 2 .. 6; the pair orders 40 / 72 / 200 (h = 20 / 36 / 100) and
# leading orders with h = 1..100 (full tiles, 4-row tails, padded tiles)
SHAPES = [
    (200, 200),
    (40, 40),
    (8, 72, 72),
    (12, 40, 40),
    (10, 200, 200),
    (6, 14, 40, 40),
    (2, 34, 40, 40),
    (40, 8, 72, 72),
    (4, 6, 8, 40, 40),
    (200, 6, 40, 40),
    (6, 104, 104),        # pair TF 3 .. 5 (h = 52, 68, 84: round 5)
    (4, 136, 136),
    (2, 168, 168),
    (104, 8, 136, 136),   # a fast mode kernel of order 104 (axis 0): JT 4
    (2, 4, 2, 6, 40, 40),  # d = 6: four mode launches before the pair
]


@pytest.mark.parametrize("ms", SHAPES)
def test_block_info(gg, ms):
    K = gg.tensors.KronMatrix(factors(ms), sym=True)
    ok, n, L = K._device().block_info()
    assert ok and n == int(np.prod(ms)) and L == len(ms) - 1


@pytest.mark.parametrize("ms,why", [
    ((9, 40, 40), "odd order"),
    ((8, 40, 72), "unequal pair orders"),
    ((8, 208, 208), "pair h = 104 > 100 (no 16 TF + 4 slab kernel)"),
    ((8, 240, 40, 40), "h > 112"),
])
def test_block_unavailable(gg, ms, why):
    K = gg.tensors.KronMatrix(factors(ms), sym=True)
    assert not K._device().block_info()[0], why


def test_block_unavailable_not_centrosymmetric(gg):
    F = factors((8, 40, 40))
    F[0] = F[0] + np.diag(np.linspace(0.0, 0.1, 8))   # breaks J F J = F
    K = gg.tensors.KronMatrix(F, sym=True)
    assert not K._device().block_info()[0]


@pytest.mark.parametrize("ms", SHAPES)
def test_block_fold_vs_oracle(gg, ms):
    K = gg.tensors.KronMatrix(factors(ms), sym=True)
    dk = K._device()
    x = np.random.default_rng(1).standard_normal(int(np.prod(ms)))
    xb = host(gg, dk.block_fold(dev(gg, x)))
    ref = oracle.kron.block_fold(x, ms)
    assert rel(xb, ref) < 1e-15
    back = host(gg, dk.block_fold(dev(gg, xb), inverse=True))
    assert rel(back, x) < 1e-15
    assert abs(np.linalg.norm(xb) - np.linalg.norm(x)) < 1e-13 * np.linalg.norm(x)


@pytest.mark.parametrize("ms", SHAPES)
@pytest.mark.parametrize("shift", [0.0, 0.05])
def test_block_matvec_vs_oracle(gg, ms, shift):
    F = factors(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    dk = K._device()
    n = int(np.prod(ms))
    x = np.random.default_rng(2).standard_normal(n)
    xb = oracle.kron.block_fold(x, ms)
    yb = host(gg, dk.block_matvec(dev(gg, xb), shift=shift))
    refb = oracle.kron.block_matvec(F, xb) + shift * xb
    assert rel(yb, refb) < 1e-13
    # through the fold: the reference's product
    y = oracle.kron.block_fold(yb, ms, inverse=True)
    assert rel(y, oracle.kron_matvec(F, x) + shift * x) < 1e-13


@pytest.mark.parametrize("ms", [(40, 40, 40, 40), (200, 6, 40, 40), (40, 8, 72, 72),
                                (72, 36, 72, 72), (104, 8, 72, 72), (136, 4, 40, 40),
                                (168, 4, 40, 40)])
def test_block_fast_kernels_match_generic(gg, monkeypatch, ms):
    """The fixed-count mode kernels (h = 16 TF + 4: blk_mode_fast_kernel) and
    the generic ones compute the same k-step sums in the same order: the block
    matvec is bitwise equal; a fused CG (prologue and side-job launches) over
    a few iterations agrees to 1e-12 (the fused launches run 8-wave
    workgroups, so the r.r partials group differently)."""
    F = factors(ms)
    n = int(np.prod(ms))
    x = np.random.default_rng(8).standard_normal(n)
    out = []
    for fast in ("1", "0"):
        monkeypatch.setenv("GG_BLK_MODE_FAST", fast)
        K = gg.tensors.KronMatrix(F, sym=True)
        y = host(gg, K._device().block_matvec(dev(gg, x), shift=0.03))
        s = gg.linalg.KronCG(K, 0.03)
        s.start(dev(gg, x), rtol=1e-14)
        s.iterate(9)
        out.append((y, host(gg, s.x), s.status()))
    assert np.array_equal(out[0][0], out[1][0])
    assert rel(out[0][1], out[1][1]) < 1e-12
    assert out[0][2][0] == out[1][2][0] == 9


@pytest.mark.parametrize("ms", [(40, 8, 72, 72), (10, 200, 200), (6, 14, 40, 40),
                                (6, 104, 104), (4, 136, 136), (2, 168, 168)])
def test_block_pair_lds_kernel_matches_register_kernel(gg, monkeypatch, ms):
    """blk_pair_lds_kernel (GEMM 1's operands through the LDS-DMA ring; one
    or two slabs per workgroup) and blk_pair_kernel run the same MFMA chains
    in the same k order: the block matvec is bitwise equal (pair orders 72
    and 200; order 40 has no LDS variant and must fall back; (10, 200, 200)
    has an odd slab count per block, so SPW 2 falls back to 1); a fused CG
    agrees to 1e-12 (the p.q / q.q partials group over different
    workgroups)."""
    F = factors(ms)
    n = int(np.prod(ms))
    x = np.random.default_rng(9).standard_normal(n)
    out = []
    for lds, spw in (("1", "2"), ("1", "1"), ("0", "2")):
        monkeypatch.setenv("GG_BLK_PAIR_LDS", lds)
        monkeypatch.setenv("GG_BLK_PAIR_SPW", spw)
        K = gg.tensors.KronMatrix(F, sym=True)
        y = host(gg, K._device().block_matvec(dev(gg, x), shift=0.02))
        s = gg.linalg.KronCG(K, 0.02)
        s.start(dev(gg, x), rtol=1e-14)
        s.iterate(7)
        out.append((y, host(gg, s.x), s.status()))
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0])
        assert rel(out[0][1], o[1]) < 1e-12
        assert o[2][0] == 7
    assert out[0][2][0] == 7


@pytest.mark.parametrize("ms", [(40, 40, 40, 40), (8, 200, 200)])
def test_block_prologue_nontemporal_bitwise(gg, monkeypatch, ms):
    """The CG prologue with non-temporal streams (GG_BLK_PRO_NT, fast kernel
    KIND 3) and the pair launch's non-temporal p loads / q stores
    (GG_BLK_EPI_NT), both the default, run the same arithmetic: a fused CG
    agrees bitwise with either off."""
    F = factors(ms)
    x = np.random.default_rng(10).standard_normal(int(np.prod(ms)))
    out = []
    for pro, epi in (("0", "0"), ("1", "0"), ("1", "1"), ("0", "1")):
        monkeypatch.setenv("GG_BLK_PRO_NT", pro)
        monkeypatch.setenv("GG_BLK_EPI_NT", epi)
        K = gg.tensors.KronMatrix(F, sym=True)
        s = gg.linalg.KronCG(K, 0.03)
        s.start(dev(gg, x), rtol=1e-14)
        s.iterate(8)
        out.append((host(gg, s.x), s.status()))
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0])
        assert out[0][1] == o[1]


def test_block_matvec_repeatable(gg):
    """Bitwise repeatable (no atomics; fixed slab / strip assignment)."""
    ms = (12, 72, 72)
    K = gg.tensors.KronMatrix(factors(ms), sym=True)
    dk = K._device()
    xd = dev(gg, np.random.default_rng(3).standard_normal(int(np.prod(ms))))
    a = host(gg, dk.block_matvec(xd, shift=0.01))
    b = host(gg, dk.block_matvec(xd, shift=0.01))
    assert np.array_equal(a, b)


def oracle_cg(F, b, shift, rtol, maxiter):
    return oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, b, rtol=rtol,
                           maxiter=maxiter)


@pytest.mark.parametrize("ms,shift", [((10, 40, 40), 0.05), ((6, 12, 40, 40), 0.05),
                                      ((4, 8, 72, 72), 0.2), ((8, 6, 8, 40, 40), 0.1),
                                      ((40, 40, 40, 40), 0.5), ((40, 72, 72), 0.2),
                                      ((6, 104, 104), 0.1), ((4, 6, 136, 136), 0.1),
                                      ((8, 6, 168, 168), 0.2), ((2, 4, 2, 6, 40, 40), 0.1)])
def test_block_cg_vs_oracle(gg, ms, shift):
    F = factors(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    n = int(np.prod(ms))
    b = np.random.default_rng(4).standard_normal((n, 1))
    solver = gg.linalg.KronCG(K, shift)
    assert solver.basis == "block" and solver.launches() == len(ms) - 1
    x, info = gg.linalg.cg(K, b, shift=shift, rtol=1e-10, maxiter=20000)
    it = gg.linalg.cg.last.iters
    xs, _, its = oracle_cg(F, b[:, 0], shift, 1e-10, 20000)
    assert info == 0
    assert abs(it - its) <= max(2, 0.02 * its), (it, its)
    assert rel(x, xs) < 1e-8
    r = oracle.kron_matvec(F, x[:, 0]) + shift * x[:, 0] - b[:, 0]
    assert np.linalg.norm(r) <= 1.5e-10 * np.linalg.norm(b)


def test_block_cg_matches_grid_basis(gg):
    ms, shift = (6, 14, 40, 40), 0.05
    K = gg.tensors.KronMatrix(factors(ms, 1), sym=True)
    b = np.random.default_rng(5).standard_normal((int(np.prod(ms)), 1))
    xb, ib = gg.linalg.cg(K, b, shift=shift, rtol=1e-10, basis="block")
    itb = gg.linalg.cg.last.iters
    xg, ig = gg.linalg.cg(K, b, shift=shift, rtol=1e-10, basis="grid")
    itg = gg.linalg.cg.last.iters
    assert ib == 0 and ig == 0
    assert abs(itb - itg) <= max(2, 0.02 * itg)
    assert rel(xb, xg) < 1e-8


def test_block_cg_open_chain_bitwise(gg):
    """Open iterations chain into one closed call bitwise (the recurrence's
    pending update and deferred x steps carry across calls), as in the grid
    basis (test_gpu_fold.py test_cg_open_iterations_chain_bitwise)."""
    ms, shift = (6, 12, 40, 40), 0.05
    K = gg.tensors.KronMatrix(factors(ms, 2), sym=True)
    bd = dev(gg, np.random.default_rng(6).standard_normal(int(np.prod(ms))))
    a = gg.linalg.KronCG(K, shift)
    a.start(bd, rtol=1e-14)
    a.iterate(37)
    xa = host(gg, a.x)
    c = gg.linalg.KronCG(K, shift)
    c.start(bd, rtol=1e-14)
    for k in (5, 11, 1, 20):
        c.iterate(k, close=False)
    c.close()
    assert np.array_equal(host(gg, c.x), xa)
    assert a.status()[0] == c.status()[0] == 37


def test_block_cg_state_textbook_after_close(gg):
    """After a close the caller's x is P^T x_b: the true residual of x
    matches the recurrence's |r| (the textbook state)."""
    ms, shift = (8, 72, 72), 0.05
    F = factors(ms, 3)
    K = gg.tensors.KronMatrix(F, sym=True)
    b = np.random.default_rng(7).standard_normal(int(np.prod(ms)))
    s = gg.linalg.KronCG(K, shift)
    s.start(dev(gg, b), rtol=1e-14)
    s.iterate(30)
    it, conv, res, tol = s.status()
    x = host(gg, s.x)
    r = b - (oracle.kron_matvec(F, x) + shift * x)
    assert it == 30 and not conv
    assert abs(np.linalg.norm(r) - res) <= 1e-6 * np.linalg.norm(b)


# ---- x_defer mode 3: the x window (gg_cg_get_xwin, GG_CG_XWIN) -------------
@pytest.mark.parametrize("K", [0, 2, 3, 4, 6, 8])
@pytest.mark.parametrize("ms,shift", [((6, 12, 72, 72), 0.05), ((8, 6, 104, 104), 0.1)])
def test_block_cg_window_vs_oracle(gg, monkeypatch, K, ms, shift):
    """Every window K (0: mode 2's balanced pairs) solves to the oracle CG's
    answer: iterations within 2 %, x to 1e-8, true residual at the tolerance."""
    monkeypatch.setenv("GG_CG_XWIN", str(K))
    F = factors(ms, 4)
    Km = gg.tensors.KronMatrix(F, sym=True)
    n = int(np.prod(ms))
    b = np.random.default_rng(11).standard_normal((n, 1))
    s = gg.linalg.KronCG(Km, shift)
    assert s.basis == "block" and s.xwin == (K if K >= 2 else 0)
    x, info = gg.linalg.cg(Km, b, shift=shift, rtol=1e-10, maxiter=20000)
    it = gg.linalg.cg.last.iters
    xs, _, its = oracle_cg(F, b[:, 0], shift, 1e-10, 20000)
    assert info == 0
    assert abs(it - its) <= max(2, 0.02 * its), (it, its)
    assert rel(x, xs) < 1e-8
    r = oracle.kron_matvec(F, x[:, 0]) + shift * x[:, 0] - b[:, 0]
    assert np.linalg.norm(r) <= 1.5e-10 * np.linalg.norm(b)


@pytest.mark.parametrize("K", [4, 8])
def test_block_cg_window_open_chain_bitwise(gg, monkeypatch, K):
    """Open calls chain into one closed call bitwise with the window too (the
    armed region and the ring of directions carry across calls)."""
    monkeypatch.setenv("GG_CG_XWIN", str(K))
    ms, shift = (6, 12, 72, 72), 0.05   # the LDS pair launch (h >= 36) carries the window
    Km = gg.tensors.KronMatrix(factors(ms, 2), sym=True)
    bd = dev(gg, np.random.default_rng(6).standard_normal(int(np.prod(ms))))
    a = gg.linalg.KronCG(Km, shift)
    assert a.xwin == K
    a.start(bd, rtol=1e-14)
    a.iterate(37)
    xa = host(gg, a.x)
    c = gg.linalg.KronCG(Km, shift)
    c.start(bd, rtol=1e-14)
    for k in (5, 11, 1, 20):
        c.iterate(k, close=False)
    c.close()
    assert np.array_equal(host(gg, c.x), xa)
    assert a.status()[0] == c.status()[0] == 37


@pytest.mark.parametrize("K", [2, 3, 4, 6, 8])
def test_block_cg_window_matches_pairs(gg, monkeypatch, K):
    """x never feeds back into the recurrence (r, p, q and the scalars are the
    same kernels whatever the x schedule), so a window K run and a mode-2
    (pairs) run have bitwise the same residual history and x equal up to the
    order of x's sums -- one 37-iteration call, and closed chunks of 1, 7, 3
    and 26 iterations (every close flushes all regions; the recurrence then
    continues), each chunk's x with the true residual |r_k| of its status."""
    ms, shift = (8, 72, 72), 0.05
    F = factors(ms, 3)
    b = np.random.default_rng(7).standard_normal(int(np.prod(ms)))
    runs = {}
    monkeypatch.setenv("GG_CG_RDERIVE", "0")   # the same r recurrence in both
    for w in (str(K), "0"):
        monkeypatch.setenv("GG_CG_XWIN", w)
        Km = gg.tensors.KronMatrix(F, sym=True)
        a = gg.linalg.KronCG(Km, shift)
        assert a.xwin == (K if w != "0" else 0)
        a.start(dev(gg, b), rtol=1e-14)
        a.iterate(37)
        c = gg.linalg.KronCG(Km, shift)
        c.start(dev(gg, b), rtol=1e-14)
        chunks = []
        for k in (1, 7, 3, 26):
            c.iterate(k)
            it, conv, res, tol = c.status()
            x = host(gg, c.x)
            r = b - (oracle.kron_matvec(F, x) + shift * x)
            assert abs(np.linalg.norm(r) - res) <= 1e-6 * np.linalg.norm(b), (w, k)
            chunks.append((x, (it, conv, res)))
        runs[w] = (host(gg, a.x), a.status(), chunks)
    (xw, sw, cw), (xp, sp, cp) = runs[str(K)], runs["0"]
    assert sw == sp and sw[0] == 37
    assert rel(xw, xp) < 1e-11
    for (x1, s1), (x2, s2) in zip(cw, cp):
        assert s1 == s2
        assert rel(x1, x2) < 1e-11


def test_block_cg_window_converges_inside_first_window(gg, monkeypatch):
    """A solve that converges before the ring has filled (fewer iterations
    than the window) still returns the full x."""
    monkeypatch.setenv("GG_CG_XWIN", "8")
    ms, shift = (4, 8, 72, 72), 1e7   # (K + s I) ~ s I: a few iterations
    F = factors(ms, 5)
    Km = gg.tensors.KronMatrix(F, sym=True)
    b = np.random.default_rng(8).standard_normal((int(np.prod(ms)), 1))
    assert gg.linalg.KronCG(Km, shift).xwin == 8
    x, info = gg.linalg.cg(Km, b, shift=shift, rtol=1e-8, maxiter=1000)
    it = gg.linalg.cg.last.iters
    xs, _, its = oracle_cg(F, b[:, 0], shift, 1e-8, 1000)
    assert its < 8, its
    assert info == 0 and it < 8 and abs(it - its) <= 1
    assert rel(x, xs) < 1e-9


# ---- the fused Lanczos step in the block basis (gg_lanczos_info) -----------
@pytest.mark.parametrize("ms", [(40, 40, 40, 40), (72, 72, 72, 72), (8, 6, 104, 104),
                                (12, 72, 72), (4, 6, 8, 40, 40), (2, 4, 2, 6, 40, 40)])
def test_block_lanczos_matches_grid_and_oracle(gg, monkeypatch, ms):
    """The probe folded once and every step in the parity-block basis gives the
    grid-basis tridiagonal (P is orthogonal: same Krylov space) to 1e-10 over
    the first 12 steps, and the oracle's (oracle.lanczos_tridiag on the
    reference operator kron_matrix.py:52-97 from the same probe) to 1e-8."""
    F = factors(ms, 6)
    n = int(np.prod(ms))
    s = 0.03
    out = {}
    for basis in ("1", "0"):
        monkeypatch.setenv("GG_LZ_BASIS", basis)
        K = gg.tensors.KronMatrix(F, sym=True)
        blk, L = gg.linalg.lanczos_info(K)
        assert blk == (basis == "1") and L == (len(ms) - 1 if blk else len(ms))
        out[basis] = gg.linalg.lanczos_tridiag(K, s, 20, seed=7, probe=2)
    (ab, bb), (ag, bg) = out["1"], out["0"]
    k = min(ab.size, ag.size, 12)
    np.testing.assert_allclose(ab[:k], ag[:k], rtol=1e-10)
    np.testing.assert_allclose(bb[:k - 1], bg[:k - 1], rtol=1e-10)
    zp = oracle.cg.probe_signs(7, 2, n)
    ao, bo = oracle.lanczos_tridiag(lambda v: oracle.kron_matvec(F, v) + s * v, zp, 20)
    np.testing.assert_allclose(ab[:k], ao[:k], rtol=1e-8)
    np.testing.assert_allclose(bb[:k - 1], bo[:k - 1], rtol=1e-7)


def test_block_lanczos_timed_and_slq(gg):
    """The timed probe (bench.py's Lanczos leg) runs the same steps: identical
    tridiagonal, a time per step and per launch (d - 1 positions, the d-th
    entry 0); SLQ in the block basis against the exact shifted log det."""
    ms = (8, 12, 72, 72)
    F = factors(ms, 7)
    K = gg.tensors.KronMatrix(F, sym=True)
    assert gg.linalg.lanczos_info(K) == (True, 3)
    a0, b0 = gg.linalg.lanczos_tridiag(K, 0.05, 12, seed=3, probe=1)
    a1, b1, step_ms, launch_ms = gg.linalg.lanczos_tridiag(K, 0.05, 12, seed=3, probe=1,
                                                           timed=True)
    assert np.array_equal(a0, a1) and np.array_equal(b0, b1)
    assert len(step_ms) == 12 and all(t > 0 for t in step_ms)
    assert all(t > 0 for t in launch_ms[:3]) and launch_ms[3] == 0.0
    # the closing pass (beta_{k-1}) is timed apart from the 12 steps
    assert gg.linalg.lanczos_tridiag.closing_ms > 0
    Q, lam = oracle.factor_eigh(F)
    exact = float(np.sum(np.log(oracle.kron_expand(lam) + 0.05)))
    est, _ = gg.linalg.slq_logdet(K, 0.05, probes=8, steps=60, seed=1)
    assert abs(est - exact) < 0.02 * abs(exact), (est, exact)


# ---- padded pair axes (round 6): h not of the form 16 TF + 4 --------------
# the layout pads the two innermost axes to hp = 16 TF + 4 >= h (zeros in the
# vectors and the factors), so 64^d / 96^d / 128^d grids (h = 32 / 48 / 64)
# have the block basis (the block-sharded CG, no exchange); one GPU keeps the
# grid basis by default there (measured faster, gg_kronb.hip block_efficient)
PADDED = [((6, 64, 64), False), ((4, 96, 96), False), ((2, 8, 128, 128), False),
          ((4, 6, 100, 100), False), ((8, 48, 48), False), ((12, 32, 32), False),
          ((10, 64, 64), False), ((6, 72, 72), True)]


@pytest.mark.parametrize("ms,efficient", PADDED)
def test_block_padded_info_fold_matvec(gg, ms, efficient):
    F = factors(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    dk = K._device()
    ok, nb, L = dk.block_info()
    es = oracle.kron.block_extents(ms, pad=True)
    assert ok and L == len(ms) - 1 and nb == int(np.prod(es)) << len(ms)
    n = int(np.prod(ms))
    x = np.random.default_rng(12).standard_normal(n)
    xb = host(gg, dk.block_fold(dev(gg, x)))
    assert rel(xb, oracle.kron.block_fold(x, ms, pad=True)) < 1e-15
    assert rel(host(gg, dk.block_fold(dev(gg, xb), inverse=True)), x) < 1e-15
    for shift in (0.0, 0.05):
        yb = host(gg, dk.block_matvec(dev(gg, xb), shift=shift))
        assert rel(yb, oracle.kron.block_matvec(F, xb, pad=True) + shift * xb) < 1e-13
        y = oracle.kron.block_fold(yb, ms, inverse=True, pad=True)
        assert rel(y, oracle.kron_matvec(F, x) + shift * x) < 1e-13
        # the padding (exact zeros of the folded random vector) stays zero
        assert np.all(yb[oracle.kron.block_fold(x, ms, pad=True) == 0.0] == 0.0)
    assert gg.linalg.KronCG(K, 0.05).basis == ("block" if efficient else "grid")


@pytest.mark.parametrize("ms,shift", [((6, 64, 64), 0.05), ((4, 8, 96, 96), 0.1),
                                      ((8, 48, 48), 0.05)])
def test_block_padded_cg_vs_oracle(gg, ms, shift):
    """The CG in the padded block basis (forced where the default keeps the
    grid) against the oracle CG: iterations within 2 %, x to 1e-8."""
    F = factors(ms, 8)
    K = gg.tensors.KronMatrix(F, sym=True)
    b = np.random.default_rng(13).standard_normal((int(np.prod(ms)), 1))
    x, info = gg.linalg.cg(K, b, shift=shift, rtol=1e-10, maxiter=20000, basis="block")
    it = gg.linalg.cg.last.iters
    xs, _, its = oracle_cg(F, b[:, 0], shift, 1e-10, 20000)
    assert info == 0
    assert abs(it - its) <= max(2, 0.02 * its), (it, its)
    assert rel(x, xs) < 1e-8


def test_cg_create_refuses_workspace_sized_under_another_snapshot(gg, monkeypatch):
    """gg_cg_create reads its layout from the current GG_* snapshot: a
    workspace gg_cg_work_elems sized under a smaller window is refused (a
    clean GG_ERR_VALUE instead of buffers past its end)."""
    import ctypes
    from gp_grief_amd import native
    monkeypatch.setenv("GG_CG_XWIN", "2")
    K = gg.tensors.KronMatrix(factors((6, 12, 72, 72)), sym=True)
    dk = K._device()
    L = native.lib()
    we = ctypes.c_int64()
    native.check(L.gg_cg_work_elems(dk.h, ctypes.byref(we)))
    work = gg.device.empty(we.value)
    monkeypatch.setenv("GG_CG_XWIN", "8")
    native.check(L.gg_knobs_reload())
    h = ctypes.c_void_p()
    st = L.gg_cg_create(dk.h, 0.05, native.dptr(work), ctypes.byref(h))
    assert st == -1 and not h.value
    # sized again under the current snapshot: accepted
    native.check(L.gg_cg_work_elems(dk.h, ctypes.byref(we)))
    work = gg.device.empty(we.value)
    native.check(L.gg_cg_create(dk.h, 0.05, native.dptr(work), ctypes.byref(h)))
    native.check(L.gg_cg_destroy(h))


# ---- derived r (gg_cg_get_rderive): no r in memory with the window ---------
# (derived r needs the fast prologue kernel on axis 0: an order 16 TF + 4 >= 40)
@pytest.mark.parametrize("ms,shift", [((40, 6, 72, 72), 0.05), ((104, 2, 72, 72), 0.1),
                                      ((40, 72, 72), 0.2)])
def test_block_cg_rderive_vs_stored_and_oracle(gg, monkeypatch, ms, shift):
    """The prologue taking r_{j-1} = p_{j-1} - beta_{j-1} p_{j-2} (5 passes)
    solves to the oracle CG's answer, within 2 % of its iterations, like the
    stored-r recurrence (GG_CG_RDERIVE=0); after 37 open iterations + close
    the materialised r is the true residual of the unfolded x.  (Mid-solve
    the two recurrences' iterates differ by CG's amplification of their
    different rounding -- 5e-5 relative at iteration 37 here -- so they are
    compared where it is defined: at convergence, against the oracle.)"""
    F = factors(ms, 9)
    n = int(np.prod(ms))
    b = np.random.default_rng(14).standard_normal(n)
    xs, _, its = oracle_cg(F, b, shift, 1e-10, 20000)
    out = {}
    for rd in ("1", "0"):
        monkeypatch.setenv("GG_CG_RDERIVE", rd)
        K = gg.tensors.KronMatrix(F, sym=True)
        s = gg.linalg.KronCG(K, shift)
        assert s.rderive == (rd == "1") and s.xwin == 8
        x, info = gg.linalg.cg(K, b.reshape(-1, 1), shift=shift, rtol=1e-10, maxiter=20000)
        it = gg.linalg.cg.last.iters
        assert info == 0 and abs(it - its) <= max(2, 0.02 * its), (rd, it, its)
        assert rel(x, xs) < 1e-8
        s.start(dev(gg, b), rtol=1e-14)
        for k in (5, 11, 21):
            s.iterate(k, close=False)
        s.close()
        itc, conv, res, tol = s.status()
        xc = host(gg, s.x)
        r = b - (oracle.kron_matvec(F, xc) + shift * xc)
        assert itc == 37 and abs(np.linalg.norm(r) - res) <= 1e-8 * np.linalg.norm(b)
        out[rd] = (xc, res)


def test_block_cg_rderive_repairs(gg, monkeypatch):
    """Forced cancellations (GG_CG_CANCEL_TOL = 0.3 counts beta < 0.3 as
    cancelled) exercise the repair with derived r: it materialises r_j from
    the directions, takes the true r.r, and the solve still lands on the
    oracle's x."""
    monkeypatch.setenv("GG_CG_CANCEL_TOL", "0.3")
    ms, shift = (40, 6, 72, 72), 0.05
    F = factors(ms, 10)
    K = gg.tensors.KronMatrix(F, sym=True)
    s = gg.linalg.KronCG(K, shift)
    assert s.rderive
    b = np.random.default_rng(15).standard_normal(int(np.prod(ms)))
    s.start(dev(gg, b), rtol=1e-10)
    s.iterate(20000, check_every=25)
    it, conv, res, tol = s.status()
    assert conv and s.cancels() > 0
    xs, _, its = oracle_cg(F, b, shift, 1e-10, 20000)
    assert rel(host(gg, s.x), xs) < 1e-8
