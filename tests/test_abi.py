"""CPU-side checks of the C-ABI library: it loads, exports every declared
symbol, and maps status codes to the reference's exception types.  No compute
call is made (there is no GPU in the build container)."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def declared():
    src = open(os.path.join(ROOT, "include", "gp_grief_amd.h")).read()
    return re.findall(r"^int (gg_\w+)\(", src, re.M)


def test_header_declares_entry_points():
    names = declared()
    assert len(names) >= 20
    assert "gg_kron_matvec" in names and "gg_cg_iterate" in names


def test_library_exports_every_declared_symbol():
    from gp_grief_amd import native
    lib = native.load()
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared()) == set(native.SIGNATURES), "ctypes table out of sync with header"
    assert lib.gg_abi_version() == 1


def test_status_code_mapping():
    from gp_grief_amd import native
    native.load()
    with pytest.raises(ValueError):
        native.check(native.GG_ERR_VALUE)
    with pytest.raises(np.linalg.LinAlgError):
        native.check(native.GG_ERR_LINALG)
    with pytest.raises(AssertionError):
        native.check(native.GG_ERR_ASSERT)
    with pytest.raises(RuntimeError):
        native.check(native.GG_ERR_RUNTIME)
    native.check(native.GG_OK)


def test_library_is_gfx950_only():
    so = os.path.join(ROOT, "gp_grief_amd", "libgpgrief.so")
    blob = open(so, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets
