"""Device-memory plumbing (PyTorch-ROCm tensors as HBM buffers) for the C ABI."""
import numpy as np

from . import native


def torch():
    import torch as _t
    return _t


def device():
    t = torch()
    native.lib()  # raises if no MI355X / library
    return t.device("cuda", t.cuda.current_device())


def is_device_array(x):
    t = torch()
    return isinstance(x, t.Tensor) and x.is_cuda


def empty(n):
    t = torch()
    return t.empty(int(n), dtype=t.float64, device=device())


def zeros(n):
    t = torch()
    return t.zeros(int(n), dtype=t.float64, device=device())


def to_device(x):
    """1-D contiguous float64 device tensor holding x (numpy, matrix or tensor)."""
    t = torch()
    if isinstance(x, t.Tensor):
        xd = x.detach()
        if xd.dtype != t.float64:
            xd = xd.to(t.float64)
        if not xd.is_cuda:
            xd = xd.to(device())
        return xd.reshape(-1).contiguous()
    arr = np.ascontiguousarray(np.asarray(x, dtype=np.float64)).reshape(-1)
    return t.from_numpy(arr).to(device())


def to_host(xd):
    return xd.detach().cpu().numpy()


def ensure_aligned(xd):
    """The vector kernels use 16-byte loads: realign a view that is not."""
    if xd.data_ptr() % 16 != 0:
        return xd.clone()
    return xd
