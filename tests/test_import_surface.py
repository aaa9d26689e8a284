"""The drop-in import path: every name the reference's package __init__ files
export (gp_grief/tensors/__init__.py:2-9, kern/__init__.py:2-9,
models/__init__.py:2-6, gp_grief/__init__.py:1-7) resolves through the
`gp_grief` package to the MI355X implementation, including file-level deep
imports.  CPU-only: imports and host-side construction, no device calls."""
import importlib
import logging

import numpy as np
import pytest

EXPORTS = {
    "gp_grief.tensors": ["KronMatrix", "SelectionMatrix", "SelectionMatrixSparse", "BlockMatrix",
                         "TensorProduct", "TensorSum", "Array", "expand_SKC",
                         "KhatriRaoMatrix", "RowColKhatriRaoMatrix",
                         "RowColKhatriRaoMatrixTransposed"],
    "gp_grief.kern": ["BaseKernel", "GPyKernel", "Stationary", "RBF", "Exponential", "Matern32",
                      "Matern52", "GridKernel", "GriefKernel", "WEBKernel", "RBF_RFF"],
    "gp_grief.models": ["BaseModel", "GPRegressionModel", "GPGriefModel", "GPwebModel",
                        "GPwebTransformedModel"],
    "gp_grief.grid": ["InducingGrid"],
    "gp_grief.linalg": ["solve_schur", "solve_chol", "solver_counter", "log_kron", "uniquetol",
                        "LogexpTransformation"],
}
DEEP = {
    "gp_grief.tensors.kron_matrix": "KronMatrix",
    "gp_grief.tensors.selection_matrix": "SelectionMatrixSparse",
    "gp_grief.tensors.tensors": "expand_SKC",
    "gp_grief.tensors.khatri_rao_matrix": "RowColKhatriRaoMatrix",
    "gp_grief.tensors.block_matrix": "BlockMatrix",
    "gp_grief.kern.grief_kernel": "GriefKernel",
    "gp_grief.kern.grid_kernel": "GridKernel",
    "gp_grief.kern.stationary": "Matern52",
    "gp_grief.models.gp_grief_model": "GPGriefModel",
    "gp_grief.models.basemodel": "BaseModel",
}


@pytest.mark.parametrize("mod", sorted(EXPORTS))
def test_reference_exports_resolve(mod):
    m = importlib.import_module(mod)
    impl = importlib.import_module(mod.replace("gp_grief.", "gp_grief_amd."))
    for name in EXPORTS[mod]:
        assert getattr(m, name) is getattr(impl, name), (mod, name)


@pytest.mark.parametrize("mod", sorted(DEEP))
def test_deep_imports(mod):
    m = importlib.import_module(mod)
    assert getattr(m, DEEP[mod]) is getattr(importlib.import_module(
        mod.rsplit(".", 1)[0].replace("gp_grief.", "gp_grief_amd.")), DEEP[mod])


def test_package_level_behaviour():
    import gp_grief
    for sub in ("kern", "models", "tensors", "linalg", "grid"):
        assert hasattr(gp_grief, sub)
    assert callable(gp_grief.debug)
    assert logging.getLogger().handlers   # reference configures root logging on import


def test_host_structure_helpers():
    from gp_grief.tensors import (Array, TensorProduct, TensorSum, BlockMatrix,
                                  SelectionMatrix, SelectionMatrixSparse)
    rng = np.random.default_rng(0)
    A, B = rng.standard_normal((4, 3)), rng.standard_normal((3, 5))
    x = rng.standard_normal((5, 1))
    np.testing.assert_allclose(TensorProduct([Array(A), Array(B)]) * x, A.dot(B).dot(x))
    C = rng.standard_normal((4, 5))
    np.testing.assert_allclose(TensorSum([Array(A.dot(B)), Array(C)]) * x,
                               (A.dot(B) + C).dot(x))
    blocks = np.empty((2, 2), dtype=object)
    Ms = [[rng.standard_normal((2, 3)), rng.standard_normal((2, 2))],
          [rng.standard_normal((1, 3)), rng.standard_normal((1, 2))]]
    for i in range(2):
        for j in range(2):
            blocks[i, j] = Array(Ms[i][j])
    bm = BlockMatrix(blocks)
    dense = np.block(Ms)
    np.testing.assert_allclose(bm.expand(), dense)
    np.testing.assert_allclose(bm * x, dense.dot(x))
    np.testing.assert_allclose(bm.T.expand(), dense.T)
    mask = np.array([True, False, True, True, False])
    S = SelectionMatrix(mask)
    v = rng.standard_normal((5, 2))
    np.testing.assert_array_equal(S.mul(v), v[mask])
    back = S.mul_T(S.mul(v))
    np.testing.assert_array_equal(back[mask], v[mask])
    assert np.all(back[~mask] == 0)
    Ss = SelectionMatrixSparse((np.array([3, 1, 3, 0]), 5))
    np.testing.assert_array_equal(Ss.mul_unique(v), v[[0, 1, 3]])
    np.testing.assert_array_equal(Ss.unique[Ss.unique_inverse], [3, 1, 3, 0])


def test_gpy_kernel_without_gpy_raises():
    from gp_grief.kern import GPyKernel
    try:
        import GPy  # noqa: F401
        pytest.skip("GPy importable")
    except ImportError:
        pass
    with pytest.raises(ImportError):
        GPyKernel(1, kernel="RBF")
