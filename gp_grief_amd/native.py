"""ctypes binding of libgpgrief.so (the C ABI declared in include/gp_grief_amd.h).

The product path has exactly one implementation: the HIP library.  If the
shared object is missing, or no MI355X is visible, every compute call raises;
there is no CPU fallback (the CPU restatement in oracle/ is test-only).
Device memory and streams come from PyTorch-ROCm (plumbing only): buffers are
torch.float64 CUDA tensors whose data_ptr() is handed to the C ABI together
with torch's current HIP stream.
"""
import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgpgrief.so")

GG_OK = 0
GG_ERR_VALUE = -1
GG_ERR_LINALG = -2
GG_ERR_RUNTIME = -3
GG_ERR_ASSERT = -4

GG_DIAG_DIVIDE = 0
GG_DIAG_POSTVAR = 1
GG_DIAG_MULTIPLY = 2

_c_i64p = ctypes.POINTER(ctypes.c_int64)
_c_dp = ctypes.c_void_p  # device or host double* (passed as raw addresses)
_vp = ctypes.c_void_p

# name -> argtypes (every function returns c_int status)
SIGNATURES = {
    "gg_abi_version": [],
    "gg_last_error": [ctypes.c_char_p, ctypes.c_size_t],
    "gg_set_device": [ctypes.c_int],
    "gg_device_synchronize": [],
    "gg_kron_create": [ctypes.c_int, _c_i64p, _c_i64p, ctypes.POINTER(ctypes.c_void_p),
                       ctypes.POINTER(ctypes.c_void_p)],
    "gg_kron_destroy": [_vp],
    "gg_kron_shape": [_vp, ctypes.c_int, _c_i64p, _c_i64p, _c_i64p],
    "gg_kron_fold_mask": [_vp, ctypes.c_int, _c_i64p],
    "gg_kron_matvec": [_vp, ctypes.c_int, _c_dp, _c_dp, ctypes.c_double, _c_dp, _vp],
    "gg_kron_matvec_timed": [_vp, ctypes.c_int, _c_dp, _c_dp, ctypes.c_double, _c_dp,
                             ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_double), _vp],
    "gg_kron_block_info": [_vp, ctypes.POINTER(ctypes.c_int), _c_i64p,
                           ctypes.POINTER(ctypes.c_int)],
    "gg_kron_block_fold": [_vp, ctypes.c_int, _c_dp, _c_dp, _vp],
    "gg_kron_block_matvec": [_vp, _c_dp, _c_dp, ctypes.c_double, _c_dp, _vp],
    "gg_kron_block_fold_range": [_vp, ctypes.c_int, _c_dp, _c_dp, ctypes.c_int64, ctypes.c_int64,
                                 _vp],
    "gg_kron_block_matvec_range": [_vp, _c_dp, _c_dp, ctypes.c_double, _c_dp, ctypes.c_int64,
                                   ctypes.c_int64, _vp],
    "gg_kron_block_matvec_timed": [_vp, _c_dp, _c_dp, ctypes.c_double, _c_dp, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double), _vp],
    "gg_kron_diag_scale": [ctypes.c_int, _c_i64p, _c_dp, ctypes.c_double, ctypes.c_int, _c_dp,
                           _c_dp, _vp],
    "gg_kron_logdet_shifted": [ctypes.c_int, _c_i64p, _c_dp, ctypes.c_double,
                               ctypes.POINTER(ctypes.c_double), _vp],
    "gg_dot": [_c_dp, _c_dp, ctypes.c_int64, ctypes.POINTER(ctypes.c_double), _vp],
    "gg_axpby": [ctypes.c_double, _c_dp, ctypes.c_double, _c_dp, ctypes.c_int64, _vp],
    "gg_scale_rows": [_c_dp, ctypes.c_int64, ctypes.c_int64, _c_dp, ctypes.c_int, _vp],
    "gg_diag_divide": [_c_dp, ctypes.c_double, _c_dp, _c_dp, ctypes.c_int64, _vp],
    "gg_cg_work_elems": [_vp, _c_i64p],
    "gg_knobs_reload": [],
    "gg_cg_create": [_vp, ctypes.c_double, _c_dp, ctypes.POINTER(ctypes.c_void_p)],
    "gg_cg_work_elems_blocks": [_vp, ctypes.c_int64, _c_i64p],
    "gg_cg_create_blocks": [_vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_double, _c_dp,
                            ctypes.POINTER(ctypes.c_void_p)],
    "gg_cg_destroy": [_vp],
    "gg_cg_start": [_vp, _c_dp, _c_dp, ctypes.c_double, ctypes.c_double, _vp],
    "gg_cg_iterate": [_vp, ctypes.c_int, ctypes.c_int, _vp],
    "gg_cg_iterate_open": [_vp, ctypes.c_int, ctypes.c_int, _vp],
    "gg_cg_close": [_vp, _vp],
    "gg_cg_set_recurrence": [_vp, ctypes.c_int],
    "gg_cg_get_recurrence": [_vp, ctypes.POINTER(ctypes.c_int)],
    "gg_cg_set_fusion": [_vp, ctypes.c_int],
    "gg_cg_get_fusion": [_vp, ctypes.POINTER(ctypes.c_int)],
    "gg_cg_set_xdefer": [_vp, ctypes.c_int],
    "gg_cg_get_xdefer": [_vp, ctypes.POINTER(ctypes.c_int)],
    "gg_cg_get_xwin": [_vp, ctypes.POINTER(ctypes.c_int)],
    "gg_cg_get_rderive": [_vp, ctypes.POINTER(ctypes.c_int)],
    "gg_cg_calibrate": [_vp, ctypes.c_int, _c_dp, _c_i64p, _vp],
    "gg_cg_set_rq": [_vp, ctypes.c_int],
    "gg_cg_get_rq": [_vp, ctypes.POINTER(ctypes.c_int)],
    "gg_cg_set_basis": [_vp, ctypes.c_int],
    "gg_cg_get_basis": [_vp, ctypes.POINTER(ctypes.c_int)],
    "gg_cg_launches": [_vp, ctypes.POINTER(ctypes.c_int)],
    "gg_cg_start_partial": [_vp, _c_dp, _c_dp, _c_dp, _vp],
    "gg_parity_fold": [ctypes.c_int, _c_i64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp,
                       _c_dp, _vp],
    "gg_shard0_fold": [ctypes.c_int, _c_i64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp,
                       _c_dp, _vp],
    "gg_cg_start_finish": [_vp, _c_dp, ctypes.c_double, ctypes.c_double, _vp],
    "gg_cg_iterate_partial": [_vp, _c_dp, _vp],
    "gg_cg_iterate_finish": [_vp, _c_dp, _vp],
    "gg_cg_close_partial": [_vp, _c_dp, _vp],
    "gg_cg_close_finish": [_vp, _c_dp, _vp],
    "gg_cg_cancels": [_vp, ctypes.POINTER(ctypes.c_int), _vp],
    "gg_cg_status": [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), _vp],
    "gg_cg_profile": [_vp, ctypes.c_int],
    "gg_cg_profile_read": [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double),
                           ctypes.c_int],
    "gg_lanczos_probe": [_vp, ctypes.c_double, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                         _c_dp, ctypes.POINTER(ctypes.c_double),
                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int), _vp],
    "gg_lanczos_probe_timed": [_vp, ctypes.c_double, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                               _c_dp, ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                               _vp],
    "gg_lanczos_info": [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
    "gg_probe_fill": [ctypes.c_uint64, ctypes.c_int, _c_dp, ctypes.c_int64, _vp],
    "gg_sym_eig_batched": [ctypes.c_int, _c_i64p, _c_dp, _c_dp, _c_dp, _c_dp, ctypes.c_int64,
                           ctypes.c_int, _vp],
    "gg_sym_eig_work_elems": [ctypes.c_int, _c_i64p, _c_i64p],
    "gg_sym_eig_tridiag": [ctypes.c_int, _c_i64p, _c_dp, _c_dp, _c_dp, _c_dp, ctypes.c_int64,
                           _vp],
    "gg_sym_eig_tridiag_vectors": [ctypes.c_int, _c_i64p, _c_dp, _c_dp, ctypes.c_int64, _c_dp,
                                   ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                   _c_dp, _vp],
    "gg_rows_orthonormalize": [ctypes.c_int, _c_i64p, _c_i64p, _c_dp, _vp],
    "gg_centro_expand": [ctypes.c_int, _c_i64p, _c_i64p, _c_i64p, _c_dp, _c_dp, _vp],
    "gg_cov": [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int, _c_dp,
               ctypes.c_int64, _c_dp, ctypes.c_int64, ctypes.c_int, _c_dp, _vp],
    "gg_grief_tables": [ctypes.c_int, ctypes.c_double, ctypes.c_double, _c_dp, ctypes.c_int64,
                        ctypes.c_int64, _c_dp, ctypes.c_int, _c_dp, ctypes.c_int, _c_dp, _c_dp,
                        ctypes.c_int, ctypes.c_int, _vp],
    "gg_grief_tables_all": [ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                            _c_dp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.c_int64,
                            ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int),
                            ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int),
                            _c_dp, _c_dp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), _vp],
    "gg_grief_phi": [_c_dp, _c_dp, ctypes.c_int, ctypes.c_int64, _c_dp, ctypes.c_int, _c_dp,
                     ctypes.c_int, ctypes.c_int, _c_dp, _vp],
    "gg_kr_work_elems": [ctypes.c_int, _c_i64p, ctypes.c_int64, _c_i64p],
    "gg_kr_contract": [ctypes.c_int, _c_i64p, _c_dp, _c_dp, ctypes.POINTER(ctypes.c_void_p),
                       ctypes.c_int64, _c_dp, _c_dp, ctypes.c_int64, _vp],
    "gg_kr_hadamard": [ctypes.c_int64, _c_dp, _c_dp, _c_dp, ctypes.c_int, ctypes.c_int, _vp],
    "gg_gemm": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                ctypes.c_double, _c_dp, ctypes.c_int64, _c_dp, ctypes.c_int64, ctypes.c_double,
                _c_dp, ctypes.c_int64, ctypes.c_int, _c_dp, ctypes.c_int64, _vp],
    "gg_gemm_splitk_elems": [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_i64p],
    "gg_gemm_workspace_elems": [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int, _c_i64p],
    "gg_expand_skc": [_c_dp, ctypes.c_int, ctypes.c_int64, _c_dp, ctypes.c_int, ctypes.c_int,
                      ctypes.c_int, _c_dp, _c_dp, _vp],
    "gg_gemv": [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_double, _c_dp,
                ctypes.c_int64, _c_dp, ctypes.c_double, _c_dp, _c_dp, ctypes.c_int64, _vp],
    "gg_add_diag": [ctypes.c_int, _c_dp, ctypes.c_int64, ctypes.c_double, _c_dp, _c_dp,
                    ctypes.c_int64, _vp],
    "gg_potrf_work_elems": [ctypes.c_int, _c_i64p],
    "gg_potrf": [ctypes.c_int, _c_dp, ctypes.c_int64, _c_dp, ctypes.POINTER(ctypes.c_double),
                 _vp],
    "gg_potrs": [ctypes.c_int, ctypes.c_int, _c_dp, ctypes.c_int64, _c_dp, _c_dp,
                 ctypes.c_int64, ctypes.c_int, _c_dp, _vp],
    "gg_trtri": [ctypes.c_int, _c_dp, ctypes.c_int64, _c_dp, _c_dp, ctypes.c_int64, _vp],
    "gg_colsumsq_lower": [ctypes.c_int, _c_dp, ctypes.c_int64, _c_dp, _vp],
    "gg_kron_dist_create": [ctypes.c_int, _c_i64p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                            ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)],
    "gg_kron_dist_destroy": [_vp],
    "gg_kron_dist_sizes": [_vp, _c_i64p, _c_i64p],
    "gg_kron_dist_fold_mask": [_vp, _c_i64p],
    "gg_kron_dist_phase1": [_vp, _c_dp, _c_dp, _c_dp, _c_dp, _vp, _vp],
    "gg_kron_dist_phase2": [_vp, _c_dp, _c_dp, _vp],
    "gg_ipc_handle": [_c_dp, ctypes.c_void_p, _c_i64p],
    "gg_kron_dist_set_peers": [_vp, _c_dp, ctypes.c_int, ctypes.c_void_p, _c_i64p,
                               ctypes.POINTER(ctypes.c_void_p)],
    "gg_kron_dist_phase1_push": [_vp, _c_dp, _c_dp, _c_dp, _c_dp, _vp, _vp],
    "gg_kron_dist_phase2_push": [_vp, _vp],
    "gg_cgs_create": [ctypes.POINTER(ctypes.c_void_p)],
    "gg_cgs_destroy": [_vp],
    "gg_cgs_scalars": [_vp, ctypes.POINTER(ctypes.c_void_p)],
    "gg_cgs_local_dot": [_vp, _c_dp, _c_dp, ctypes.c_int64, _c_dp, _vp],
    "gg_cgs_init": [_vp, _c_dp, ctypes.c_double, ctypes.c_double, _vp],
    "gg_cgs_shift_dot": [_vp, _c_dp, _c_dp, ctypes.c_int64, ctypes.c_double, _c_dp, _vp],
    "gg_cgs_alpha": [_vp, _c_dp, _vp],
    "gg_cgs_update": [_vp, _c_dp, _c_dp, _c_dp, _c_dp, ctypes.c_int64, _c_dp, _vp],
    "gg_cgs_rho": [_vp, _c_dp, _vp],
    "gg_kron_dist_phase1_fused": [_vp, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp, _vp,
                                  ctypes.c_double, ctypes.c_int, _vp],
    "gg_cgs_fused_post": [_vp, _c_dp, _c_dp, ctypes.c_int64, ctypes.c_double, _c_dp, _vp],
    "gg_cgs_fused_scalars": [_vp, _c_dp, _c_dp, _vp],
    "gg_cgs_fused_close": [_vp, _c_dp, _c_dp, _c_dp, _c_dp, ctypes.c_int64, ctypes.c_int64,
                           ctypes.c_double, _c_dp, _vp],
    "gg_cgs_fused_close_rho": [_vp, _c_dp, _vp],
    "gg_cgs_status": [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), _vp],
}

GG_KERN = {"RBF": 0, "Exponential": 1, "Matern32": 2, "Matern52": 3}

_lock = threading.Lock()
_lib = None


class NativeUnavailable(RuntimeError):
    """libgpgrief.so is not built / cannot be loaded, or no GPU is visible."""


def load():
    """Load the shared object (no GPU needed just to load and inspect it)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # PyTorch-ROCm bundles its own libamdhip64; load it FIRST so that the
        # library resolves its HIP dependency to that same runtime instead of
        # bringing a second runtime into the process.
        import torch  # noqa: F401
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                "%s is not built; run `python -c 'import __graft_entry__ as g; g.build()'`"
                % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        _lib = lib
        return lib


def last_error():
    buf = ctypes.create_string_buffer(4096)
    load().gg_last_error(buf, 4096)
    return buf.value.decode(errors="replace")


def check(status, what=""):
    if status == GG_OK:
        return
    msg = last_error()
    if what:
        msg = "%s: %s" % (what, msg)
    if status == GG_ERR_VALUE:
        raise ValueError(msg)
    if status == GG_ERR_LINALG:
        raise np.linalg.LinAlgError(msg)
    if status == GG_ERR_ASSERT:
        raise AssertionError(msg)
    raise RuntimeError(msg)


_ready = False


def lib():
    """The library, with cuda:0 (or the current torch device) verified usable."""
    global _ready
    L = load()
    if not _ready:
        import torch
        if not torch.cuda.is_available():
            raise NativeUnavailable("no ROCm GPU visible: the gp_grief_amd product path runs "
                                    "only on MI355X (gfx950)")
        name = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
        if not str(name).startswith("gfx950"):
            raise NativeUnavailable("libgpgrief.so is built for gfx950, device is %s" % name)
        check(L.gg_set_device(torch.cuda.current_device()), "gg_set_device")
        _ready = True
    return L


def knobs_reload():
    """Re-read the library's GG_* environment switches (gg_knobs_reload): the
    handle-free entry points (dense, GRIEF, eigen) see the environment as of
    this call; Kronecker / CG handles latch it when they are made."""
    check(lib().gg_knobs_reload(), "gg_knobs_reload")


def stream_ptr():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def i64_array(values):
    arr = (ctypes.c_int64 * len(values))(*[int(v) for v in values])
    return arr


def dptr(t):
    """Raw device address of a contiguous float64 torch tensor."""
    return ctypes.c_void_p(t.data_ptr())
