"""gp_grief.tensors -> gp_grief_amd.tensors (reference: gp_grief/tensors/__init__.py:2-9)."""
import sys as _sys

from gp_grief_amd.tensors import (KronMatrix, SelectionMatrix, SelectionMatrixSparse,  # noqa: F401
                                  BlockMatrix, TensorProduct, TensorSum, Array, expand_SKC,
                                  KhatriRaoMatrix, RowColKhatriRaoMatrix,
                                  RowColKhatriRaoMatrixTransposed)
from .._alias import register as _register

_register(_sys.modules[__name__], {
    "kron_matrix": ["KronMatrix"],
    "selection_matrix": ["SelectionMatrix", "SelectionMatrixSparse"],
    "block_matrix": ["BlockMatrix"],
    "tensors": ["TensorProduct", "TensorSum", "Array", "expand_SKC"],
    "khatri_rao_matrix": ["KhatriRaoMatrix", "RowColKhatriRaoMatrix",
                          "RowColKhatriRaoMatrixTransposed"],
})
