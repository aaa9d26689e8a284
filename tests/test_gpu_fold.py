"""The centrosymmetric even/odd split of the Kronecker mode product on the MI355X.

Every stationary kernel on an evenly spaced grid gives a factor F with
J F J = F (J reverses the index order); gg_kron_create then packs the two
half-size blocks Es / Ea and the mode product runs as two h x h GEMMs
(mode_product_fold_kernel).  The product it computes is
the reference's KronMatrix.kronvec_prod (gp_grief/tensors/kron_matrix.py:52-97)
up to rounding: these tests hold it to the oracle's dense product at 1e-13
relative (one GEMM chain) and to the unfolded device kernel, for every launch
kind the CG / Lanczos drivers use (plain, textbook / fused / Lanczos
prologues, side job, fused epilogue), even and odd m, the 4x4x4 tails, and
partial row strips.  GG_KRON_FOLD_MIN=8 lets small factors take the split.
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


@pytest.fixture
def fold_small(monkeypatch):
    monkeypatch.setenv("GG_KRON_FOLD_MIN", "8")
    monkeypatch.delenv("GG_KRON_FOLD", raising=False)


def grid_factor(m, ell=0.15, kind="RBF"):
    g = np.linspace(0.0, 1.0, m)
    return oracle.cov_1d(kind, g, g, 1.0, ell) + 1e-12 * np.eye(m)


def kron(gg, F):
    return gg.tensors.KronMatrix(F, sym=True)


def fold_mask(K, transpose=False):
    return K._device().fold_mask(transpose)


# m: even / odd, below / at / above a 16-column tile, the 4x4x4 tails (even m
# with a last half-tile of 1..8 columns: 200, 230, 100), the 256 limit
MS = [8, 9, 16, 17, 31, 32, 33, 47, 64, 65, 97, 100, 127, 128, 129, 199, 200, 201, 230, 255,
      256]


@pytest.mark.parametrize("m", MS)
def test_fold_matvec_vs_oracle(gg, fold_small, m):
    """[F_m, B_7, F_m]: the split on the first and the last mode product
    (7 < 8 stays dense), forward and transposed, vs the dense oracle and
    vs the unfolded kernel."""
    F = [grid_factor(m, 0.12), grid_factor(7, 0.3), grid_factor(m, 0.2, "Matern52")]
    K = kron(gg, F)
    assert fold_mask(K) == 0b101 and fold_mask(K, True) == 0b101
    n = 7 * m * m
    x = np.random.default_rng(m).standard_normal((n, 1))
    y = K * x
    ref = oracle.kron_matvec(F, x[:, 0])
    assert rel(y, ref) < 1e-13
    assert rel(K.T * x, ref) < 1e-13   # symmetric factors: K^T = K


def test_fold_matches_unfolded_kernel(gg, monkeypatch):
    F = [grid_factor(200, 0.1), grid_factor(64, 0.11), grid_factor(49, 0.3)]
    x = np.random.default_rng(0).standard_normal((200 * 64 * 49, 1))
    monkeypatch.setenv("GG_KRON_FOLD", "0")
    K0 = kron(gg, F)
    assert fold_mask(K0) == 0
    y0 = K0 * x
    monkeypatch.delenv("GG_KRON_FOLD")
    K1 = kron(gg, F)
    assert fold_mask(K1) == 0b111   # default GG_KRON_FOLD_MIN = 48
    y1 = K1 * x
    assert rel(y1, y0) < 1e-14
    assert rel(y1, oracle.kron_matvec(F, x[:, 0])) < 1e-13


@pytest.mark.parametrize("m0", [199, 200])
def test_fold_lean_matches_clamped(gg, monkeypatch, m0):
    """The kLean kernels (SGPR row base + 32-bit lane offsets; default for the
    m = 199 / 200 shape) and the clamped ones (GG_FOLD_LEAN=0) run the same
    arithmetic: the plain matvec and a fused CG (prologue, side and epilogue
    launches) agree bitwise."""
    F = [grid_factor(m0, 0.1), grid_factor(200, 0.13), grid_factor(200, 0.2, "Matern52")]
    n = m0 * 200 * 200
    x = np.random.default_rng(m0).standard_normal((n, 1))
    out = {}
    for lean in ("1", "0"):
        monkeypatch.setenv("GG_FOLD_LEAN", lean)
        K = kron(gg, F)
        assert fold_mask(K) == 0b111
        y = K * x
        xs, info = gg.linalg.cg(K, x, shift=0.05, rtol=0.0, maxiter=6, recurrence="fused")
        out[lean] = (np.asarray(y), np.asarray(xs))
    monkeypatch.delenv("GG_FOLD_LEAN")
    assert np.array_equal(out["1"][0], out["0"][0])
    assert np.array_equal(out["1"][1], out["0"][1])
    assert rel(out["1"][0], oracle.kron_matvec(F, x[:, 0])) < 1e-13


def test_cg_open_iterations_chain_bitwise(gg):
    """iterate(close=False) calls continue one open fused recurrence: open(5)
    + open(7) + close() is the same launch sequence as iterate(12), bitwise;
    the counts and x are the textbook state after the close."""
    import torch
    F = [grid_factor(200, 0.1), grid_factor(200, 0.13), grid_factor(200, 0.2, "Matern52")]
    K = kron(gg, F)
    b = torch.from_numpy(np.random.default_rng(8).standard_normal(200 ** 3)).cuda()
    out = []
    for chain in ([12], [5, 7]):
        cg = gg.linalg.KronCG(K, 0.05)
        cg.start(b, rtol=0.0, atol=0.0)
        for k in chain:
            cg.iterate(k, close=False)
        cg.close()
        out.append((cg.x.cpu().numpy().copy(), cg.status()))
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1][0] == out[1][1][0] == 12 and out[0][1][2] == out[1][1][2]


def test_fold_centrosymmetric_nonsymmetric_and_transpose(gg, fold_small):
    """A centrosymmetric but non-symmetric factor: the transposed operator's
    split is packed from F^T."""
    rng = np.random.default_rng(4)
    C = rng.standard_normal((37, 37))
    Fc = C + C[::-1, ::-1]
    F = [Fc, grid_factor(12)]
    K = gg.tensors.KronMatrix(F)
    assert fold_mask(K) == 0b11 and fold_mask(K, True) == 0b11
    x = rng.standard_normal((37 * 12, 1))
    assert rel(K * x, oracle.kron_matvec(F, x[:, 0])) < 1e-13
    FT = [f.T for f in F]
    assert rel(K.T * x, oracle.kron_matvec(FT, x[:, 0])) < 1e-13


def test_fold_not_taken(gg, fold_small):
    """Random SPD factors, a grid factor perturbed above the 16 eps test, and
    non-square factors stay on the dense kernel."""
    rng = np.random.default_rng(2)
    A = rng.standard_normal((40, 40))
    G = grid_factor(40)
    Gp = G.copy()
    Gp[3, 5] += 1e-13
    Gp[5, 3] += 1e-13
    F = [A.dot(A.T) / 40 + np.eye(40), Gp, rng.standard_normal((30, 20))]
    K = gg.tensors.KronMatrix(F)
    assert fold_mask(K) == 0
    x = rng.standard_normal((40 * 40 * 20, 1))
    assert rel(K * x, oracle.kron_matvec(F, x[:, 0])) < 1e-13


@pytest.mark.parametrize("ms", [(24, 20, 16, 18), (200, 24), (24, 200), (40, 36, 10)])
def test_fold_cg_fused_and_textbook(gg, fold_small, ms):
    """Every CG launch kind on folded factors (prologue, side job, fused
    epilogue; textbook prologue + shift / p.q epilogue) vs the exact solve."""
    F = [grid_factor(m, 0.15 * (1 + 0.05 * k)) for k, m in enumerate(ms)]
    K = kron(gg, F)
    assert fold_mask(K) == sum(1 << k for k, m in enumerate(ms) if m >= 8)
    n = int(np.prod(ms))
    b = np.random.default_rng(3).standard_normal((n, 1))
    s = 0.05
    xf, inf = gg.linalg.cg(K, b, shift=s, rtol=1e-10, recurrence="fused")
    itf = gg.linalg.cg.last.iters
    xt, intb = gg.linalg.cg(K, b, shift=s, rtol=1e-10, recurrence="textbook")
    assert inf == 0 and intb == 0
    xo, _, ito = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + s * v, b[:, 0], rtol=1e-10)
    assert abs(itf - ito) <= max(3, 0.05 * ito), (itf, ito)
    Q, lam = oracle.factor_eigh(F)
    ex = oracle.solve_schur(Q, oracle.kron_expand(lam), b[:, 0], s)
    assert rel(xf, ex) < 1e-8 and rel(xt, ex) < 1e-8
    res = b[:, 0] - (oracle.kron_matvec(F, xf[:, 0]) + s * xf[:, 0])
    assert np.linalg.norm(res) < 2e-10 * np.linalg.norm(b)


def test_fold_cg_odd_n_textbook(gg, fold_small):
    F = [grid_factor(m) for m in (17, 13, 9)]
    K = kron(gg, F)
    assert fold_mask(K) == 0b111
    b = np.random.default_rng(8).standard_normal((17 * 13 * 9, 1))
    x, info = gg.linalg.cg(K, b, shift=0.1, rtol=1e-10)
    assert info == 0 and gg.linalg.KronCG(K, 0.1).recurrence == "textbook"
    Q, lam = oracle.factor_eigh(F)
    assert rel(x, oracle.solve_schur(Q, oracle.kron_expand(lam), b[:, 0], 0.1)) < 1e-8


@pytest.mark.parametrize("ms", [(20, 18, 16, 12), (200, 30), (9, 8, 7)])
def test_fold_lanczos_vs_oracle(gg, fold_small, ms):
    """Fused Lanczos on folded factors: the CGP 3 prologue (even d) and the
    separate update pass (odd d)."""
    F = [grid_factor(m, 0.15 * (1 + 0.05 * k)) for k, m in enumerate(ms)]
    K = kron(gg, F)
    n = int(np.prod(ms))
    s = 0.03
    a, b = gg.linalg.lanczos_tridiag(K, s, 20, seed=7, probe=2)
    zp = oracle.cg.probe_signs(7, 2, n)
    ao, bo = oracle.lanczos_tridiag(lambda v: oracle.kron_matvec(F, v) + s * v, zp, 20)
    k = min(a.size, ao.size, 12)
    np.testing.assert_allclose(a[:k], ao[:k], rtol=1e-8)
    np.testing.assert_allclose(b[:k - 1], bo[:k - 1], rtol=1e-7)


def test_fold_partial_strips(gg, fold_small):
    """Row counts M that are not multiples of the 64-row workgroup or the
    16-row wave strip, on every position."""
    F = [grid_factor(33), grid_factor(11), grid_factor(9)]
    K = kron(gg, F)
    assert fold_mask(K) == 0b111
    x = np.random.default_rng(1).standard_normal((33 * 11 * 9, 1))
    assert rel(K * x, oracle.kron_matvec(F, x[:, 0])) < 1e-13
    y = K._device().matvec(gg.device.to_device(x[:, 0]), shift=0.7)
    assert rel(y.cpu().numpy(), oracle.kron_matvec(F, x[:, 0]) + 0.7 * x[:, 0]) < 1e-13


@pytest.mark.parametrize("fusion", [0, 1, 2])
@pytest.mark.parametrize("xdefer", ["2", "1", "0"])
def test_fold_cg_fusion_layouts_and_deferred_x(gg, fold_small, monkeypatch, fusion, xdefer):
    """Fused CG on folded factors with each fusion layout (1: p_new recomputed
    in the folded epilogue; 2: the dense epilogue kernel with the x update) and
    the x update deferred in pairs (2: half a pair per iteration, 1: a whole
    pair every other iteration) or not: same solution as the exact solve, and
    iterate() chunks of odd length (deferred steps pending across calls) reach
    the same iterate as one call."""
    import torch
    monkeypatch.setenv("GG_CG_XDEFER", xdefer)
    F = [grid_factor(m, 0.15 * (1 + 0.05 * k)) for k, m in enumerate((24, 20, 16, 18))]
    K = kron(gg, F)
    n = 24 * 20 * 16 * 18
    s = 0.05
    b = np.random.default_rng(12).standard_normal((n, 1))
    x, info = gg.linalg.cg(K, b, shift=s, rtol=1e-10, fusion=fusion)
    assert info == 0
    Q, lam = oracle.factor_eigh(F)
    ex = oracle.solve_schur(Q, oracle.kron_expand(lam), b[:, 0], s)
    assert rel(x, ex) < 1e-8
    one = gg.linalg.KronCG(K, s, fusion=fusion)
    assert one.xdefer == (int(xdefer) if fusion != 2 else 0)
    bt = torch.tensor(b[:, 0], device="cuda")
    one.start(bt, rtol=0.0)
    one.iterate(23)
    chunks = gg.linalg.KronCG(K, s, fusion=fusion)
    chunks.start(bt, rtol=0.0)
    for k in (3, 1, 7, 5, 7):
        chunks.iterate(k)
    torch.cuda.synchronize()
    assert one.status()[0] == chunks.status()[0] == 23
    # a chunk boundary closes with the textbook update (true r.r for beta
    # instead of the expansion, deferred x steps flushed): rounding-level
    assert rel(chunks.x.cpu().numpy(), one.x.cpu().numpy()) < 1e-9


@pytest.mark.parametrize("dims", [(24, 20, 16, 18), (30, 22, 14)])
def test_fold_cg_xdefer_modes_agree(gg, fold_small, dims):
    """The three x-update schedules (immediate, a pair every other iteration,
    half a pair per iteration) give the same iterate after the same number of
    iterations, for every count (pairs open, half applied, complete at the
    exit), d = 4 (two side launches per half) and d = 3 (one)."""
    import torch
    F = [grid_factor(m, 0.15 * (1 + 0.05 * k)) for k, m in enumerate(dims)]
    K = kron(gg, F)
    n = int(np.prod(dims))
    b = torch.tensor(np.random.default_rng(5).standard_normal(n), device="cuda")
    for its in (1, 2, 3, 4, 5, 9):
        xs = []
        for mode in (0, 1, 2):
            cg = gg.linalg.KronCG(K, 0.05, xdefer=mode)
            assert cg.xdefer == mode
            cg.start(b, rtol=0.0)
            cg.iterate(its)
            assert cg.status()[0] == its
            xs.append(cg.x.cpu().numpy())
        assert rel(xs[1], xs[0]) < 1e-12
        assert rel(xs[2], xs[0]) < 1e-12


@pytest.mark.parametrize("dims,centro", [((24, 20, 16, 18), True), ((30, 22, 14), True),
                                         ((26, 18, 20, 12), False)])
def test_cg_rq_identity_matches_epilogue_rq(gg, fold_small, dims, centro):
    """beta's r.q from the conjugacy identity (p.q - beta p.q_prev, the
    prologue summing p.q_prev; gg_cg_set_rq 1) against r.q read in the
    epilogue (0): the same iterate at every iteration count, single calls and
    chunked calls (each re-entry starts with a non-pending prologue), on the
    folded kernels and on mode_product_kernel (non-centrosymmetric factors);
    and the same convergence to a tolerance."""
    import torch
    rng = np.random.default_rng(11)
    F = []
    for k, m in enumerate(dims):
        if centro:
            F.append(grid_factor(m, 0.15 * (1 + 0.05 * k)))
        else:
            g = np.sort(rng.uniform(0.0, 1.0, m))
            F.append(oracle.cov_1d("RBF", g, g, 1.0, 0.2) + 1e-10 * np.eye(m))
    K = kron(gg, F)
    assert (fold_mask(K) != 0) == centro
    n = int(np.prod(dims))
    b = torch.tensor(rng.standard_normal(n), device="cuda")
    s = 0.05
    # at s = 0.05 the system is ill-conditioned enough that any rounding
    # change grows by ~1e8 over 25 iterations (the textbook and the fused
    # recurrence differ by 5e-8 there): the identity must stay as close to the
    # textbook iterate as the epilogue r.q does
    for its in (1, 2, 3, 7, 25):
        xs = []
        for kw in (dict(recurrence="textbook"), dict(rq=0), dict(rq=1)):
            cg = gg.linalg.KronCG(K, s, **kw)
            if "rq" in kw:
                assert cg.rq == kw["rq"]
            cg.start(b, rtol=0.0)
            cg.iterate(its)
            assert cg.status()[0] == its
            xs.append(cg.x.cpu().numpy())
        base = max(rel(xs[1], xs[0]), 1e-13)
        assert rel(xs[2], xs[0]) < 4 * base, (its, rel(xs[2], xs[0]), base)
    chunks = gg.linalg.KronCG(K, s, rq=1)
    chunks.start(b, rtol=0.0)
    for k in (3, 1, 7, 5, 9):
        chunks.iterate(k)
    assert rel(chunks.x.cpu().numpy(), xs[0]) < 4 * base
    counts = []
    s = 2.0   # a conditioning that converges in a few hundred iterations
    for rq in (0, 1):
        cg = gg.linalg.KronCG(K, s, rq=rq)
        cg.start(b, rtol=1e-10)
        cg.iterate(4000, check_every=10)
        it, conv, res, tol = cg.status()
        assert conv, (rq, it, res, tol)
        counts.append(it)
        x = cg.x.cpu().numpy()
        bh = b.cpu().numpy()
        r_true = bh - (oracle.kron_matvec(F, x) + s * x)
        assert np.linalg.norm(r_true) <= 1e-8 * np.linalg.norm(bh)
    assert abs(counts[0] - counts[1]) <= 1, counts


@pytest.mark.parametrize("ms", [(20, 18, 16, 12), (9, 8, 7)])
def test_lanczos_timed_matches_untimed(gg, fold_small, ms):
    """gg_lanczos_probe_timed (bench.py's Lanczos leg) runs the same steps as
    gg_lanczos_probe: identical tridiagonal, one positive time per step, and a
    per-position mode-product time for every factor."""
    F = [grid_factor(m, 0.15 * (1 + 0.05 * k)) for k, m in enumerate(ms)]
    K = kron(gg, F)
    a0, b0 = gg.linalg.lanczos_tridiag(K, 0.03, 12, seed=3, probe=1)
    a1, b1, step_ms, launch_ms = gg.linalg.lanczos_tridiag(K, 0.03, 12, seed=3, probe=1,
                                                           timed=True)
    assert np.array_equal(a0, a1) and np.array_equal(b0, b1)
    assert len(step_ms) == 12 and all(t > 0 for t in step_ms)
    assert len(launch_ms) == len(ms) and all(t > 0 for t in launch_ms)
    # the closing pass (the last beta) is timed apart from the steps: a pass
    # of its own with the update fused (even d), none otherwise
    cl = gg.linalg.lanczos_tridiag.closing_ms
    assert cl is not None and (cl > 0 if len(ms) % 2 == 0 else cl >= 0)


def test_matvec_timed_matches_matvec(gg, fold_small):
    """gg_kron_matvec_timed (bench.py's isolated K*x leg) computes the plain
    matvec, reps times, with a time for every mode-product position."""
    import torch
    F = [grid_factor(200, 0.1), grid_factor(40, 0.13), grid_factor(36, 0.2, "Matern52")]
    K = kron(gg, F)
    n = 200 * 40 * 36
    x = torch.from_numpy(np.random.default_rng(5).standard_normal(n)).cuda()
    dk = K._device()
    y0 = dk.matvec(x).clone()
    y1 = torch.empty_like(x)
    per, tot = dk.matvec_timed(x, y1, 3)
    assert torch.equal(y0, y1)
    assert len(per) == 3 and all(t > 0 for t in per) and tot >= 0.99 * sum(per)
    assert rel(y1.cpu().numpy(), oracle.kron_matvec(F, x.cpu().numpy())) < 1e-13


def test_cg_prologue_shape_change_on_live_handle(gg, monkeypatch):
    """the prologue's workgroup shape is chosen per launch from env
    knobs (GG_FOLD_PRO_W), while its r.r / p.q_old partial arrays are sized at
    gg_cg_create.  Switching 12 -> 4 -> 12 waves between iterate calls on one
    handle must sum exactly the partials each launch wrote (no stale tail, no
    overrun): the iterate agrees with an unswitched run to rounding."""
    F = [grid_factor(200, 0.1), grid_factor(48, 0.13), grid_factor(40, 0.2, "Matern52")]
    K = kron(gg, F)
    n = 200 * 48 * 40
    import torch
    b = torch.from_numpy(np.random.default_rng(11).standard_normal(n)).cuda()
    monkeypatch.setenv("GG_FOLD_PRO_W", "12")
    ref = gg.linalg.KronCG(K, 0.05)
    ref.start(b, rtol=0.0)
    ref.iterate(9)
    sw = gg.linalg.KronCG(K, 0.05)
    sw.start(b, rtol=0.0)
    for w in ("12", "4", "12"):
        monkeypatch.setenv("GG_FOLD_PRO_W", w)
        sw.iterate(3)
    it0, _, r0, _ = ref.status()
    it1, _, r1, _ = sw.status()
    assert it0 == it1 == 9
    assert abs(r1 - r0) <= 1e-8 * abs(r0)
    assert rel(sw.x.cpu().numpy(), ref.x.cpu().numpy()) < 1e-10

