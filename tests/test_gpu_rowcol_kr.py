"""RowColKhatriRaoMatrix / RowColKhatriRaoMatrixTransposed on the MI355X
against the reference-generated fixture rowcol_kr.npz (tests/golden/
make_golden.py f9_rowcol_kr, the test_RowColKhatriRaoMatrix.py setting plus
a 300 x 800 case) and the oracle (oracle.rowcol_kr_expand)."""
import numpy as np
import pytest

import oracle
from conftest import golden

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def tensors(gpu):
    import gp_grief_amd.tensors
    return gp_grief_amd.tensors


def _blocks(z, tag):
    d = int(z[tag + "_d"])
    return ([z["%s_R%d" % (tag, i)] for i in range(d)], [z["%s_K%d" % (tag, i)] for i in range(d)],
            [z["%s_C%d" % (tag, i)] for i in range(d)])


@pytest.mark.parametrize("tag", ["t", "b"])
@pytest.mark.parametrize("nGb", [1., 1e-5])
def test_rowcol_kr_fixture(tensors, tag, nGb):
    z = golden("rowcol_kr.npz")
    R, K, C = _blocks(z, tag)
    A = tensors.RowColKhatriRaoMatrix(R=R, K=K, C=C, nGb=nGb)
    AT = tensors.RowColKhatriRaoMatrixTransposed(R=R, K=K, C=C, nGb=nGb)
    assert A.shape == (R[0].shape[0], C[0].shape[1]) and AT.shape == A.shape[::-1]
    assert rel(A * z[tag + "_vec"], z[tag + "_Avec"]) < 1e-12
    assert rel(A.T * z[tag + "_vecT"], z[tag + "_ATvecT"]) < 1e-12
    assert rel(AT * z[tag + "_vecT"], z[tag + "_ATT_vecT"]) < 1e-12
    assert rel(AT.T * z[tag + "_vec"], z[tag + "_Avec"]) < 1e-12
    assert rel(A.get_rows(np.arange(min(24, A.shape[0]))), z[tag + "_expand"]) < 1e-13
    log, sign = A.get_rows(slice(0, 24), logged=True)
    assert np.array_equal(sign, z[tag + "_sign"])
    assert np.max(np.abs(log - z[tag + "_log"])) < 1e-11
    full = A.expand()
    assert full.shape == A.shape
    assert rel(full, oracle.rowcol_kr_expand(R, K, C)) < 1e-13
    ls, ss = A.expand(logged=True)
    assert rel(ss * np.exp(ls), full) < 1e-12


def test_rowcol_kr_without_k_and_wrong_shape(tensors):
    rng = np.random.default_rng(3)
    R = [rng.random((40, m)) - 0.5 for m in (5, 7)]
    C = [rng.random((m, 90)) - 0.5 for m in (5, 7)]
    A = tensors.RowColKhatriRaoMatrix(R=R, K=None, C=C)
    x = rng.random((90, 1))
    assert rel(A * x, oracle.rowcol_kr_expand(R, [None, None], C).dot(x)) < 1e-13
    with pytest.raises(AssertionError):
        A * np.ones((89, 1))
