"""Register the reference's file-level submodules (e.g. gp_grief.tensors.kron_matrix)
as views of the package namespace, so deep imports resolve too."""
import sys
import types


def register(package, names_by_module):
    for mod, names in names_by_module.items():
        full = package.__name__ + "." + mod
        m = types.ModuleType(full, "gp_grief alias of %s (served by gp_grief_amd)" % full)
        for n in names:
            setattr(m, n, getattr(package, n))
        sys.modules[full] = m
        setattr(package, mod, m)
