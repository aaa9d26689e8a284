"""P1 across GPUs: the Kronecker CG with factor 0 sharded over ranks.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Vectors are sharded along factor 0 (the slowest axis of the reference's
flattening); every rank holds N/G elements in the local layout
(m_1, ..., m_{d-1}, a), a = i_0 - rank * m_0/G fastest.  A matvec is two
local MFMA phases with one exchange after each (include/gp_grief_amd.h,
gg_kron_dist_*).  Two CG recurrences (DistKronCG(recurrence=...)):
  "fused" (default where the engine supports it: d >= 4 with factors 1..d-1
         on the centrosymmetric split): the single-GPU fused recurrence
         (gg_cg_iterate) -- the CG prologue (r -= alpha q_old, p = r + beta p,
         partial r.r and p.q_old) rides on phase 1's first mode product, the
         deferred x update on its second, and the four dot products of an
         iteration are ONE all-reduce of five doubles;
  "textbook": scipy's order, two scalar all-reduces per iteration.
Both stop on scipy's rule; a sharded solve takes the single-GPU iteration
count up to rounding.  One difference from gg_cg_iterate: where the fused
beta cancels (|r_{j+1}|^2 < 1e-6 rho_j from the three-term expansion), the
single-GPU path repairs it with the true r.r; the sharded one restarts
(beta = 0, p = r) instead of paying a second all-reduce every iteration.

Two exchange modes (DistKronCG(mode=...)):
  "push" (opt-in; needs engine.supports_push): the last mode product of each
         phase stores its output straight into the destination ranks' buffers
         in peer memory over xGMI (IPC-mapped), so the exchange overlaps the
         MFMA work instead of following it; a system-scope release ends each
         storing kernel and a stream-ordered barrier (an RCCL all-reduce of
         one double) separates the phases;
  "a2a" (default): the phases write a send buffer and RCCL all_to_all_single
         moves it.

The arithmetic lives in the "engine" (HipEngine: the C ABI on this rank's
GPU).  The exchange is injected: `TorchExchange` (RCCL / gloo collectives) in
production; the tests also drive the same orchestration with virtual ranks.
"""
import ctypes
import os

import numpy as np

from . import device as dev
from . import native


def local_index_map(m, world, rank):
    """Global flat indices (C order over the factors) of this rank's local
    elements, in local order.  Host helper for scatter / gather and tests."""
    m = [int(v) for v in m]
    s0 = m[0] // world
    rest = int(np.prod(m[1:]))
    a = np.arange(s0)
    r = np.arange(rest)
    # local (r, a) -> global (i0 = rank*s0 + a, r)
    return ((rank * s0 + a)[None, :] * rest + r[:, None]).reshape(-1)


def scatter_global(vec, m, world, rank):
    return np.asarray(vec).reshape(-1)[local_index_map(m, world, rank)]


def gather_global(locals_, m):
    world = len(locals_)
    n = int(np.prod(m))
    out = np.empty(n)
    for g, loc in enumerate(locals_):
        out[local_index_map(m, world, g)] = np.asarray(loc).reshape(-1)
    return out


class TorchExchange(object):
    """All-to-all, all-reduce, barrier and handle exchange over a
    torch.distributed process group (nccl = RCCL; gloo for CPU-side tests,
    where device tensors are reduced through a host copy)."""

    in_process = False

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.group = group
        self.backend = str(dist.get_backend(group))
        self._tok = None

    def all_to_all(self, out, inp):
        self.dist.all_to_all_single(out, inp, group=self.group)

    def all_reduce(self, t):
        if t.is_cuda and self.backend == "gloo":
            h = t.cpu()
            self.dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            self.dist.all_reduce(t, group=self.group)

    def barrier(self):
        """Stream-ordered barrier: every rank's earlier kernels have finished
        (their peer stores landed) before any rank's later kernels start."""
        if self.backend == "nccl":
            if self._tok is None:
                self._tok = self.torch.zeros(1, dtype=self.torch.float64, device="cuda")
            self.dist.all_reduce(self._tok, group=self.group)  # RCCL, stream-ordered
        else:
            self.torch.cuda.synchronize()
            self.dist.barrier(group=self.group)

    def all_gather_object(self, obj):
        out = [None] * self.dist.get_world_size(self.group)
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def all_gather(self, t):
        """The ranks' equal-length 1-D tensors concatenated in rank order (one
        RCCL all-gather into a device tensor; under gloo through host copies)."""
        world = self.dist.get_world_size(self.group)
        if self.backend == "nccl":
            out = self.torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
            self.dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
            return out
        h = t.detach().cpu().contiguous()
        parts = [self.torch.empty_like(h) for _ in range(world)]
        self.dist.all_gather(parts, h, group=self.group)
        return self.torch.cat(parts).to(t.device)

    def size(self):
        return self.dist.get_world_size(self.group)

    def rank(self):
        return self.dist.get_rank(self.group)


class HipEngine(object):
    """This rank's share of the sharded operator and CG scalars on its GPU."""

    supports_push = True

    def __init__(self, factors, world, rank):
        L = native.lib()
        mats = [np.ascontiguousarray(np.asarray(f, dtype=np.float64)) for f in factors]
        for f in mats:
            if f.ndim != 2 or f.shape[0] != f.shape[1]:
                raise ValueError("the sharded operator needs square factors")
        self._keep = mats
        self.m = [f.shape[0] for f in mats]
        self.world, self.rank = int(world), int(rank)
        ptrs = (ctypes.c_void_p * len(mats))(*[f.ctypes.data for f in mats])
        h = ctypes.c_void_p()
        native.check(L.gg_kron_dist_create(len(mats), native.i64_array(self.m), ptrs, int(world),
                                           int(rank), ctypes.byref(h)), "gg_kron_dist_create")
        self.h = h
        nl, we = ctypes.c_int64(), ctypes.c_int64()
        native.check(L.gg_kron_dist_sizes(self.h, ctypes.byref(nl), ctypes.byref(we)))
        self.n_local = nl.value
        fm = ctypes.c_int64()
        native.check(L.gg_kron_dist_fold_mask(self.h, ctypes.byref(fm)))
        self.fold_mask = fm.value   # factors on the centrosymmetric split
        self.work = dev.empty(we.value)
        c = ctypes.c_void_p()
        native.check(L.gg_cgs_create(ctypes.byref(c)), "gg_cgs_create")
        self.cgs = c
        sc = ctypes.c_void_p()
        native.check(L.gg_cgs_scalars(self.cgs, ctypes.byref(sc)))
        self.sc = sc
        self.red = dev.zeros(2)  # [0]: the scalar being all-reduced
        self.red5 = dev.zeros(5)  # fused recurrence: [r.r, p.q_old, p.q, 0, q.q]
        self.xbuf = None         # push mode: [recv | out], 2 n_local

    def empty(self):
        return dev.empty(self.n_local)

    def zeros(self):
        return dev.zeros(self.n_local)

    # ---- push-mode exchange setup
    def setup_push(self, exchange):
        """Allocate this rank's exchange buffer and learn every peer's: by IPC
        handle across processes, by pointer for ranks sharing a process.
        Returns the view where K x lands (the "out" half)."""
        L = native.lib()
        self.xbuf = dev.zeros(2 * self.n_local)
        ptr = self.xbuf.data_ptr()
        if getattr(exchange, "in_process", False):
            ptrs = exchange.all_gather_object(ptr)
            arr = (ctypes.c_void_p * self.world)(*ptrs)
            native.check(L.gg_kron_dist_set_peers(self.h, ctypes.c_void_p(ptr), 0, None, None,
                                                  arr), "gg_kron_dist_set_peers")
        else:
            hbuf = ctypes.create_string_buffer(64)
            off = ctypes.c_int64()
            native.check(L.gg_ipc_handle(ctypes.c_void_p(ptr), hbuf, ctypes.byref(off)),
                         "gg_ipc_handle")
            allh = exchange.all_gather_object((hbuf.raw, off.value))
            blob = ctypes.create_string_buffer(b"".join(h for h, _ in allh), 64 * self.world)
            offs = native.i64_array([o for _, o in allh])
            native.check(L.gg_kron_dist_set_peers(self.h, ctypes.c_void_p(ptr), 1, blob, offs,
                                                  None), "gg_kron_dist_set_peers")
        return self.xbuf[self.n_local:]

    def phase1(self, x, send, r=None):
        native.check(native.lib().gg_kron_dist_phase1(
            self.h, native.dptr(x), native.dptr(send), native.dptr(self.work),
            native.dptr(r) if r is not None else None, self.sc if r is not None else None,
            native.stream_ptr()), "gg_kron_dist_phase1")

    def phase2(self, recv, send):
        native.check(native.lib().gg_kron_dist_phase2(self.h, native.dptr(recv),
                                                      native.dptr(send), native.stream_ptr()),
                     "gg_kron_dist_phase2")

    def phase1_push(self, x, scratch, r=None):
        native.check(native.lib().gg_kron_dist_phase1_push(
            self.h, native.dptr(x), native.dptr(scratch), native.dptr(self.work),
            native.dptr(r) if r is not None else None, self.sc if r is not None else None,
            native.stream_ptr()), "gg_kron_dist_phase1_push")

    def phase2_push(self):
        native.check(native.lib().gg_kron_dist_phase2_push(self.h, native.stream_ptr()),
                     "gg_kron_dist_phase2_push")

    # ---- fused recurrence (gg_kron_dist_phase1_fused / gg_cgs_fused_*)
    @property
    def supports_fused(self):
        d = len(self.m)
        return d >= 4 and (self.fold_mask >> 1) == (1 << (d - 1)) - 1 and self.n_local % 2 == 0

    def phase1_fused(self, p_old, p_new, send, r, q_old, x, shift, push):
        native.check(native.lib().gg_kron_dist_phase1_fused(
            self.h, native.dptr(p_old), native.dptr(p_new), native.dptr(send),
            native.dptr(self.work), native.dptr(r), native.dptr(q_old), native.dptr(x), self.cgs,
            float(shift), int(bool(push)), native.stream_ptr()), "gg_kron_dist_phase1_fused")

    def fused_post(self, q, p, shift):
        native.check(native.lib().gg_cgs_fused_post(
            self.cgs, native.dptr(q), native.dptr(p), self.n_local, float(shift),
            native.dptr(self.red5), native.stream_ptr()), "gg_cgs_fused_post")

    def fused_scalars(self, p_new):
        native.check(native.lib().gg_cgs_fused_scalars(
            self.cgs, native.dptr(self.red5), native.dptr(p_new), native.stream_ptr()),
            "gg_cgs_fused_scalars")

    def fused_close(self, x, r, q, p, shift):
        half = 2 * ((self.n_local + 3) // 4)
        native.check(native.lib().gg_cgs_fused_close(
            self.cgs, native.dptr(x), native.dptr(r), native.dptr(q), native.dptr(p),
            self.n_local, half, float(shift), native.dptr(self.red), native.stream_ptr()),
            "gg_cgs_fused_close")

    def fused_close_rho(self):
        native.check(native.lib().gg_cgs_fused_close_rho(self.cgs, native.dptr(self.red),
                                                         native.stream_ptr()),
                     "gg_cgs_fused_close_rho")

    def fused_reduce_buffer(self):
        return self.red5

    # ---- CG scalar steps; each writes / reads self.red[0]
    def local_dot(self, x, y):
        native.check(native.lib().gg_cgs_local_dot(self.cgs, native.dptr(x), native.dptr(y),
                                                   self.n_local, native.dptr(self.red),
                                                   native.stream_ptr()))

    def cg_init(self, rtol, atol):
        native.check(native.lib().gg_cgs_init(self.cgs, native.dptr(self.red), float(rtol),
                                              float(atol), native.stream_ptr()))

    def shift_dot(self, q, p, shift):
        native.check(native.lib().gg_cgs_shift_dot(self.cgs, native.dptr(q), native.dptr(p),
                                                   self.n_local, float(shift),
                                                   native.dptr(self.red), native.stream_ptr()))

    def cg_alpha(self):
        native.check(native.lib().gg_cgs_alpha(self.cgs, native.dptr(self.red),
                                               native.stream_ptr()))

    def cg_update(self, x, r, p, q):
        native.check(native.lib().gg_cgs_update(self.cgs, native.dptr(x), native.dptr(r),
                                                native.dptr(p), native.dptr(q), self.n_local,
                                                native.dptr(self.red), native.stream_ptr()))

    def cg_rho(self):
        native.check(native.lib().gg_cgs_rho(self.cgs, native.dptr(self.red),
                                             native.stream_ptr()))

    def cg_status(self):
        it, done = ctypes.c_int(), ctypes.c_int()
        rho, tol = ctypes.c_double(), ctypes.c_double()
        native.check(native.lib().gg_cgs_status(self.cgs, ctypes.byref(it), ctypes.byref(done),
                                                ctypes.byref(rho), ctypes.byref(tol),
                                                native.stream_ptr()))
        return it.value, bool(done.value), rho.value, tol.value

    def reduce_buffer(self):
        return self.red[:1]

    def copy(self, dst, src):
        dst.copy_(src)

    def zero(self, x):
        x.zero_()

    def __del__(self):
        try:
            L = native.load()
            if getattr(self, "h", None) is not None and self.h.value:
                L.gg_kron_dist_destroy(self.h)
            if getattr(self, "cgs", None) is not None and self.cgs.value:
                L.gg_cgs_destroy(self.cgs)
        except Exception:
            pass


class DistKronCG(object):
    """CG on (K + shift I) x = b with K sharded over the ranks of `exchange`.

    engine: HipEngine (or a test engine with the same methods); all vectors
    are this rank's local shards.  mode: "push" (peer-memory exchange inside
    the mode products, needs engine.supports_push) or "a2a" (RCCL all-to-all);
    "auto" = "a2a".
    """

    def __init__(self, engine, exchange, shift, mode="auto", recurrence="auto"):
        self.e = engine
        self.x_ex = exchange
        self.shift = float(shift)
        n = engine.n_local
        self.n_local = n
        # recurrence: "fused" (the single-GPU fused recurrence, one 5-double
        # all-reduce per iteration; engines with supports_fused: d >= 4,
        # folded factors 1..d-1), "textbook" (scipy's order, two scalar
        # all-reduces), "auto" = fused where supported
        if recurrence not in ("auto", "fused", "textbook"):
            raise ValueError("recurrence must be 'auto', 'fused' or 'textbook'")
        can_fuse = bool(getattr(engine, "supports_fused", False))
        if recurrence == "fused" and not can_fuse:
            raise ValueError("this engine / operator cannot run the fused recurrence")
        self.recurrence = "fused" if (recurrence == "fused" or
                                      (recurrence == "auto" and can_fuse)) else "textbook"
        if mode == "auto":
            # all-to-all unless asked: push mode's peer stores are validated
            # against it per run (bench.py) but not yet by a one-GPU-per-rank test
            mode = "a2a"
        if mode not in ("push", "a2a"):
            raise ValueError("mode must be 'push', 'a2a' or 'auto'")
        self.mode = mode
        self.r, self.p = engine.empty(), engine.zeros()
        if self.recurrence == "fused":
            # direction buffers (current, free, the deferred pair) as in
            # gg_cg_iterate's balanced x deferral
            self.pbuf = [self.p, engine.zeros(), engine.zeros(), engine.zeros()]
        self.send = engine.empty()
        if mode == "push":
            self.q = engine.setup_push(exchange)   # K p lands in the peer-visible buffer
            self.recv = None
        else:
            self.q, self.recv = engine.empty(), engine.empty()
        self.x = None
        self._prof = None

    # ---- per-phase timing (GPU engines): HIP events on the compute stream;
    # a collective's time is what the compute stream waits for it
    def profile(self, enable, iterations=64):
        """Start (or stop) per-phase timing.  The events for `iterations`
        profiled iterations are created here, outside the timed loop, and
        reused by later sessions; more are made only if a session runs
        longer."""
        self._prof = [] if enable else None
        if enable:
            import torch
            pool = getattr(self, "_ev_pool", [])
            while len(pool) < 8 * max(1, int(iterations)) + 1:
                pool.append(torch.cuda.Event(enable_timing=True))
            self._ev_pool = pool

    def _mark(self, name):
        if self._prof is not None:
            import torch
            k = len(self._prof)
            if k < len(self._ev_pool):
                e = self._ev_pool[k]
            else:
                e = torch.cuda.Event(enable_timing=True)
                self._ev_pool.append(e)
            e.record()
            self._prof.append((name, e))

    def profile_read(self):
        """ms per phase name summed over the profiled iterations (the interval
        ending at each mark is charged to that mark's phase)."""
        import torch
        torch.cuda.synchronize()
        out = {}
        ev = self._prof or []
        for (_, e0), (n1, e1) in zip(ev[:-1], ev[1:]):
            if n1 == "start":
                continue
            out[n1] = out.get(n1, 0.0) + e0.elapsed_time(e1)
        return out

    def _allreduce(self):
        self.x_ex.all_reduce(self.e.reduce_buffer())
        self._mark("allreduce")

    def _matvec_into_q(self, x, fuse_cg):
        if self.mode == "push":
            self.e.phase1_push(x, self.send, r=self.r if fuse_cg else None)
            self._mark("phase1")
            self.x_ex.barrier()   # every rank's chunks have landed in every recv
            self._mark("exchange1")
            self.e.phase2_push()
            self._mark("phase2")
            self.x_ex.barrier()   # every rank's q is complete
            self._mark("exchange2")
        else:
            self.e.phase1(x, self.send, r=self.r if fuse_cg else None)
            self._mark("phase1")
            self.x_ex.all_to_all(self.recv, self.send)
            self._mark("exchange1")
            self.e.phase2(self.recv, self.send)
            self._mark("phase2")
            self.x_ex.all_to_all(self.q, self.send)
            self._mark("exchange2")

    def apply(self, x, y, fuse_cg=False):
        """y = K x (no shift) for local shards; fuse_cg: x <- beta x + r first."""
        self._matvec_into_q(x, fuse_cg)
        if y is not self.q:
            self.e.copy(y, self.q)

    def start(self, b, rtol=1e-5, atol=0.0, x_out=None):
        self.x = self.e.zeros() if x_out is None else x_out
        self.e.zero(self.x)
        self.e.copy(self.r, b)
        self.e.local_dot(self.r, self.r)
        self._allreduce()
        self.e.cg_init(rtol, atol)
        if self.recurrence == "fused":
            self.e.zero(self.q)   # q_old of the first prologue (not pending)

    def _iterate_fused(self, n_iter, close=True):
        """The fused recurrence: per iteration phase 1 (prologue, x side job),
        the exchanges and phase 2 (K p_new lands in q, kept unshifted), a
        read-only pass for p.q' and q'.q' (q' = q + shift p_new), ONE
        all-reduce of five doubles, the scalars; leaving, the deferred x and
        pending r update and one all-reduce of r.r -- the textbook state
        (gg_cg_iterate's contract), with q = K p."""
        push = self.mode == "push"
        pb = self.pbuf
        for _ in range(int(n_iter)):
            self._mark("start")
            p_old, p_new = pb[0], pb[1]
            self.e.phase1_fused(p_old, p_new, self.send, self.r, self.q, self.x, self.shift, push)
            self._mark("phase1")
            if push:
                self.x_ex.barrier()
                self._mark("exchange1")
                self.e.phase2_push()
                self._mark("phase2")
                self.x_ex.barrier()
                self._mark("exchange2")
            else:
                self.x_ex.all_to_all(self.recv, self.send)
                self._mark("exchange1")
                self.e.phase2(self.recv, self.send)
                self._mark("phase2")
                self.x_ex.all_to_all(self.q, self.send)
                self._mark("exchange2")
            self.e.fused_post(self.q, p_new, self.shift)
            self._mark("vector")
            self.x_ex.all_reduce(self.e.fused_reduce_buffer())
            self._mark("allreduce")
            self.e.fused_scalars(p_new)
            self._mark("scalars")
            # (cur, free, p_{j-2}, p_{j-3}) <- (free, p_{j-3}, cur, p_{j-2})
            pb[0], pb[1], pb[2], pb[3] = p_new, pb[3], p_old, pb[2]
        self.p = pb[0]
        if close:
            self.close()

    def close(self):
        """Leave the fused recurrence (deferred x steps, pending r update):
        the textbook state; a no-op for the textbook recurrence."""
        if self.recurrence != "fused":
            return
        self.e.fused_close(self.x, self.r, self.q, self.p, self.shift)
        self._allreduce()
        self.e.fused_close_rho()

    def iterate(self, n_iter, close=True):
        """close=False (fused recurrence) leaves it open for the next call."""
        if self.recurrence == "fused":
            return self._iterate_fused(n_iter, close)
        for _ in range(int(n_iter)):
            self._mark("start")
            self._matvec_into_q(self.p, fuse_cg=True)        # p = r + beta p ; q = K p
            self.e.shift_dot(self.q, self.p, self.shift)     # q += s p ; local p.q
            self._mark("vector")
            self._allreduce()
            self.e.cg_alpha()
            self.e.cg_update(self.x, self.r, self.p, self.q)  # x, r ; local r.r
            self._mark("vector")
            self._allreduce()
            self.e.cg_rho()
            self._mark("scalars")

    def status(self):
        return self.e.cg_status()

    def solve(self, b, rtol=1e-5, atol=0.0, maxiter=None, check_every=20):
        self.start(b, rtol, atol)
        n_global = self.n_local  # caller may pass maxiter; default like scipy uses n
        maxiter = 10 * n_global if maxiter is None else maxiter
        done_iters = 0
        while done_iters < maxiter:
            k = min(check_every, maxiter - done_iters)
            self.iterate(k)
            done_iters += k
            it, done, rho, tol = self.status()
            if done:
                break
        it, done, rho, tol = self.status()
        return self.x, (0 if done and np.sqrt(max(rho, 0.0)) < tol else it)


# ------------------------------------------------------------ parity sharding
# A centrosymmetric factor F (J F J = F, J the index reversal; every
# stationary kernel on an evenly spaced grid) of even order m = 2h is
# block-diagonal in the even / odd basis: with u_i = (x_i + x_{m-1-i}) / sqrt 2
# and v_i = (x_i - x_{m-1-i}) / sqrt 2 (an orthogonal change of basis P),
# P F P^T = diag(S, T), S[j, i] = F[j, i] + F[j, m-1-i], T[j, i] = F[j, i] -
# F[j, m-1-i] (i, j < h; both symmetric when F is).  Taking the grid vector to
# that basis along factors 0..K-1 makes K = F_0 x ... x F_{d-1} block-diagonal
# with 2^K blocks X_0 x ... x X_{K-1} x F_K x ... x F_{d-1}, X_k in {S_k, T_k}:
# with one block per rank (G = 2^K), the matvec needs no exchange at all and
# the CG's dot products are the only collective -- ONE all-reduce of five
# doubles per iteration (the north star's "single RCCL all-reduce for the CG
# dot product").  P is orthogonal, so the CG on the transformed system takes
# the same iterates (x~ = P x) up to rounding; the per-iteration work is the
# single-GPU fused CG's (the folded kernel applies S and T to u and v; here the
# folding of factors 0..K-1 happens once, in the right-hand side and the
# solution).

def centro_split(F, rtol=16.0):
    """(S, T) of a square, even-order, centrosymmetric factor; None when F is
    not one (max |F - J F J| > rtol eps max |F|, the test gg_kron_create
    applies before folding)."""
    F = np.asarray(F, dtype=np.float64)
    if F.ndim != 2 or F.shape[0] != F.shape[1] or F.shape[0] % 2:
        return None
    m = F.shape[0]
    scale = float(np.abs(F).max()) if F.size else 0.0
    if np.abs(F - F[::-1, ::-1]).max() > rtol * np.finfo(np.float64).eps * max(scale, 1e-300):
        return None
    C = 0.5 * (F + F[::-1, ::-1])      # the centrosymmetric part
    h = m // 2
    A, B = C[:h, :h], C[:h, m - 1:h - 1:-1]   # B[j, i] = C[j, m-1-i]
    return np.ascontiguousarray(A + B), np.ascontiguousarray(A - B)


def parity_ok(factors, world):
    """world = 2^K with K <= d and factors 0..K-1 centrosymmetric of even order."""
    world = int(world)
    if world < 1 or world & (world - 1):
        return False
    K = world.bit_length() - 1
    if K > len(factors):
        return False
    return all(centro_split(factors[k]) is not None for k in range(K))


def parity_local_factors(factors, world, rank):
    """Rank g's block as the factor list of its local operator: the
    unsharded factors F_K .. F_{d-1} first, then X_k = S_k (bit k of g clear,
    bit 0 = the most significant of K) or T_k for k < K.  The order is the
    local vector layout (C order over m_K .. m_{d-1}, h_0 .. h_{K-1}): the
    first mode product, which carries the CG prologue (six streams), then runs
    on a centrosymmetric factor's tuned folded kernel -- per-rank iteration at
    G = 8 5.55-5.70 -> 5.27-5.28 ms against the sharded factors first
    (profiles/r04/y_parity_order.jsonl)."""
    K = int(world).bit_length() - 1
    head, tail = [], []
    for k, F in enumerate(factors):
        if k < K:
            S, T = centro_split(F)
            tail.append(T if (int(rank) >> (K - 1 - k)) & 1 else S)
        else:
            head.append(np.ascontiguousarray(np.asarray(F, dtype=np.float64)))
    return head + tail


def parity_local_axes(d, world):
    """Global axis of each local axis (the local layout of
    parity_local_factors)."""
    K = int(world).bit_length() - 1
    return list(range(K, d)) + list(range(K))


def _parity_transform(X, K, inverse=False):
    """Apply (or undo) the even / odd basis change along axes 0..K-1 of the
    d-dimensional array X (host)."""
    r2 = np.sqrt(0.5)
    for k in range(K):
        X = np.moveaxis(X, k, 0)
        m = X.shape[0]
        h = m // 2
        if not inverse:
            lo, hi = X[:h], X[m - 1:h - 1:-1]
            X = np.concatenate([(lo + hi) * r2, (lo - hi) * r2], axis=0)
        else:
            u, v = X[:h], X[h:]
            lo, hi = (u + v) * r2, (u - v) * r2
            X = np.concatenate([lo, hi[::-1]], axis=0)
        X = np.moveaxis(X, 0, k)
    return X


def device_parity_fold(x, m, world, rank, inverse=False, out=None):
    """gg_parity_fold on the device: the grid vector -> this rank's block in
    the even / odd basis of factors 0..K-1 (the layout of parity_fold's
    entries); inverse: the block -> its contribution to the grid vector
    (summed over the ranks by an all-reduce, as parity_unfold's result)."""
    m = [int(v) for v in m]
    n = int(np.prod(m))
    y = dev.empty(n if inverse else n // int(world)) if out is None else out
    native.check(native.lib().gg_parity_fold(len(m), native.i64_array(m), int(world), int(rank),
                                             int(bool(inverse)), native.dptr(x), native.dptr(y),
                                             native.stream_ptr()), "gg_parity_fold")
    return y


def device_shard0_fold(x, m, world, rank, inverse=False, out=None):
    """gg_shard0_fold on the device: this rank's factor-0 row block of the
    grid vector (the scatter_global layout); inverse: written back into the
    grid vector `out` (zeroed here when not given: this rank's contribution)."""
    m = [int(v) for v in m]
    n = int(np.prod(m))
    if out is None:
        out = dev.zeros(n) if inverse else dev.empty(n // int(world))
    native.check(native.lib().gg_shard0_fold(len(m), native.i64_array(m), int(world), int(rank),
                                             int(bool(inverse)), native.dptr(x),
                                             native.dptr(out), native.stream_ptr()),
                 "gg_shard0_fold")
    return out


def parity_fold(vec, m, world):
    """Host: the global vector (C order over factors of sizes m) -> every
    rank's local block in the even / odd basis (flattened, C order over the
    local factor sizes)."""
    m = [int(v) for v in m]
    K = int(world).bit_length() - 1
    X = _parity_transform(np.asarray(vec, dtype=np.float64).reshape(m), K)
    axes = parity_local_axes(len(m), world)
    out = []
    for g in range(int(world)):
        sl = tuple(slice(((g >> (K - 1 - k)) & 1) * (m[k] // 2),
                         (((g >> (K - 1 - k)) & 1) + 1) * (m[k] // 2)) if k < K else slice(None)
                   for k in range(len(m)))
        out.append(np.ascontiguousarray(np.transpose(X[sl], axes)).reshape(-1))
    return out


def parity_unfold(locals_, m):
    """Host: every rank's local block -> the global vector."""
    m = [int(v) for v in m]
    world = len(locals_)
    K = world.bit_length() - 1
    X = np.empty(m)
    axes = parity_local_axes(len(m), world)
    lshape = [m[a] // 2 if a < K else m[a] for a in axes]
    inv = np.argsort(axes)
    for g, loc in enumerate(locals_):
        sl = tuple(slice(((g >> (K - 1 - k)) & 1) * (m[k] // 2),
                         (((g >> (K - 1 - k)) & 1) + 1) * (m[k] // 2)) if k < K else slice(None)
                   for k in range(len(m)))
        X[sl] = np.transpose(np.asarray(loc).reshape(lshape), inv)
    return _parity_transform(X, K, inverse=True).reshape(-1)


class ParityHipEngine(object):
    """This rank's block of the parity-sharded operator as a resident fused CG
    (linalg.KronCG on the local factors) driven through the C ABI's
    gg_cg_*_partial / _finish split."""

    def __init__(self, factors, world, rank, shift):
        from . import linalg, tensors
        self.local_factors = parity_local_factors(factors, world, rank)
        self.K = tensors.KronMatrix(self.local_factors)
        self.cg = linalg.KronCG(self.K, shift, recurrence="fused")
        if self.cg.recurrence != "fused" or self.cg.fusion != 0:
            raise ValueError("the parity-sharded rank needs the fused recurrence (layout 0)")
        self.n_local = int(self.cg.n)
        self.red5 = dev.zeros(5)
        self.red1 = dev.zeros(1)

    def empty(self):
        return dev.empty(self.n_local)

    def zeros(self):
        return dev.zeros(self.n_local)

    def apply(self, x, y):
        self.K._device().matvec(x, out=y)

    def _c(self, name, *args):
        native.check(getattr(native.lib(), name)(self.cg.h, *args, native.stream_ptr()), name)

    def start_partial(self, b, x):
        self._c("gg_cg_start_partial", native.dptr(b), native.dptr(x), native.dptr(self.red1))
        return self.red1

    def start_finish(self, rtol, atol):
        self._c("gg_cg_start_finish", native.dptr(self.red1), float(rtol), float(atol))

    def iterate_partial(self):
        self._c("gg_cg_iterate_partial", native.dptr(self.red5))
        return self.red5

    def iterate_finish(self):
        self._c("gg_cg_iterate_finish", native.dptr(self.red5))

    def close_partial(self):
        self._c("gg_cg_close_partial", native.dptr(self.red1))
        return self.red1

    def close_finish(self):
        self._c("gg_cg_close_finish", native.dptr(self.red1))

    def status(self):
        return self.cg.status()

    def cancels(self):
        return self.cg.cancels()

    def profile(self, enable):
        self.cg.profile(enable)

    def profile_read(self):
        return self.cg.profile_read()


class ParityShardCG(object):
    """CG on (K + shift I) x = b with K's factors 0..K-1 parity-sharded over
    2^K ranks (module notes above): no exchange in the matvec, one all-reduce
    of five doubles per iteration (+ one scalar each at start and when
    leaving iterate()).  Vectors are this rank's block in the even / odd
    basis (parity_fold / parity_unfold; bench.py builds it on the device).
    engine: ParityHipEngine (default) or a test engine with its methods."""

    def __init__(self, factors, world, rank, exchange, shift, engine=None):
        if not parity_ok(factors, world):
            raise ValueError("parity sharding needs 2^K ranks and factors 0..K-1 "
                             "centrosymmetric of even order")
        self.world, self.rank = int(world), int(rank)
        self.x_ex = exchange
        self.shift = float(shift)
        self.e = engine if engine is not None else ParityHipEngine(factors, world, rank, shift)
        self.n_local = self.e.n_local
        self.x = None
        self._prof = None
        self.mode = getattr(self.e, "mode", "parity")
        self.recurrence = "fused"

    # per-phase timing on the compute stream (as DistKronCG.profile); host
    # timestamps when there is no GPU (the CPU rehearsal's test engines)
    def profile(self, enable, iterations=64):
        import torch
        self._prof = [] if enable else None
        self._host_timer = not torch.cuda.is_available()
        self.e.profile(enable)
        if enable and not self._host_timer:
            pool = getattr(self, "_ev_pool", [])
            while len(pool) < 4 * max(1, int(iterations)) + 1:
                pool.append(torch.cuda.Event(enable_timing=True))
            self._ev_pool = pool

    def _mark(self, name):
        if self._prof is not None:
            if self._host_timer:
                import time
                self._prof.append((name, time.perf_counter()))
                return
            import torch
            k = len(self._prof)
            if k < len(self._ev_pool):
                e = self._ev_pool[k]
            else:
                e = torch.cuda.Event(enable_timing=True)
                self._ev_pool.append(e)
            e.record()
            self._prof.append((name, e))

    def profile_read(self):
        out = {}
        ev = self._prof or []
        if not getattr(self, "_host_timer", False):
            import torch
            torch.cuda.synchronize()
        for (_, e0), (n1, e1) in zip(ev[:-1], ev[1:]):
            if n1 == "start":
                continue
            dt = 1e3 * (e1 - e0) if self._host_timer else e0.elapsed_time(e1)
            out[n1] = out.get(n1, 0.0) + dt
        return out

    def apply(self, x, y):
        """y = (this rank's block of K) x (no shift)."""
        self.e.apply(x, y)

    def start(self, b, rtol=1e-5, atol=0.0, x_out=None):
        self.x = self.e.zeros() if x_out is None else x_out
        self.x_ex.all_reduce(self.e.start_partial(b, self.x))
        self.e.start_finish(rtol, atol)

    def iterate(self, n_iter, close=True):
        """close=False leaves the recurrence open (the next call continues
        it); close() applies the pending updates before x or counts are read."""
        for _ in range(int(n_iter)):
            self._mark("start")
            red = self.e.iterate_partial()
            self._mark("launches")
            self.x_ex.all_reduce(red)
            self._mark("allreduce")
            self.e.iterate_finish()
            self._mark("scalars")
        if close:
            self.close()

    def close(self):
        self.x_ex.all_reduce(self.e.close_partial())
        self.e.close_finish()

    def status(self):
        """(iterations, converged, residual norm, tolerance) -- gg_cg_status."""
        return self.e.status()

    def cancels(self):
        """Cancelled betas this solve (each restarted the recurrence; the
        engine's gg_cg_cancels, or 0 for an engine without the count)."""
        return self.e.cancels() if hasattr(self.e, "cancels") else 0

    def solve(self, b, rtol=1e-5, atol=0.0, maxiter=None, check_every=20):
        self.start(b, rtol, atol)
        maxiter = 10 * self.n_local * self.world if maxiter is None else maxiter
        done_iters = 0
        while done_iters < maxiter:
            k = min(check_every, maxiter - done_iters)
            self.iterate(k)
            done_iters += k
            it, conv, res, tol = self.status()
            if conv or not np.isfinite(res):
                break
        it, conv, res, tol = self.status()
        return self.x, (0 if conv else it)


# ---------------------------------------------------------------- block sharding
# The operator in its parity-block basis (gg_kronb.hip)
# is block diagonal over the 2^d parity patterns beta (block index B =
# sum_k beta_k 2^{d-1-k}, factor 0 the most significant bit).  With G = 2^K
# ranks, rank g owns blocks [g 2^d / G, (g + 1) 2^d / G) -- the blocks whose
# top K bits are g, i.e. the parity sharding of factors 0..K-1 above -- and
# runs the single-GPU block kernels on them (gg_cg_create_blocks: d - 1
# launches per iteration, no exchange, one all-reduce of five doubles).  The
# right-hand side is folded on the device straight from the grid vector into
# the rank's blocks (gg_kron_block_fold_range); the solution's unfold writes
# each rank's contribution to the grid vector, summed by one all-reduce.

def block_range(d, world, rank):
    """(first block, block count) of rank `rank` of `world` = 2^K <= 2^d."""
    nb = (1 << int(d)) // int(world)
    return int(rank) * nb, nb


def block_shard_ok(K, world):
    """world = 2^K <= 2^d and K (a KronMatrix) has a device parity-block
    basis with d >= 3 (every factor square, even-order, centrosymmetric; the
    last two of equal order m = 2h with h = 16 TF + 4, TF in 1..6: m in {40,
    72, 104, 136, 168, 200} -- include/gp_grief_amd.h gg_kron_block_info).
    Decided on this rank alone: solve() takes the decomposition only when
    every rank agrees (a rank whose device operator failed must not pick
    another collective pattern than its peers)."""
    world = int(world)
    if world < 1 or world & (world - 1):
        return False
    d = len(K.K)
    if d < 3 or world > (1 << d):
        return False
    try:
        return bool(K._device().block_info()[0])
    except Exception:  # noqa: BLE001 -- no device library / no GPU
        return False


class BlockHipEngine(object):
    """Rank `rank`'s blocks of the operator's parity-block basis as a resident
    fused CG driven through gg_cg_*_partial / _finish (the engine interface
    of ParityHipEngine); vectors are the rank's blocks, C order inside each."""

    mode = "block"

    def __init__(self, K, world, rank, shift):
        if not block_shard_ok(K, world):
            raise ValueError("block sharding needs 2^K <= 2^d ranks and a parity-block basis")
        self.K = K
        self.dk = K._device()
        self.d = len(K.K)
        self.blk0, self.nblk = block_range(self.d, world, rank)
        L = native.lib()
        we = ctypes.c_int64()
        native.check(L.gg_cg_work_elems_blocks(self.dk.h, self.nblk, ctypes.byref(we)),
                     "gg_cg_work_elems_blocks")
        self.work = dev.empty(we.value)
        h = ctypes.c_void_p()
        native.check(L.gg_cg_create_blocks(self.dk.h, self.blk0, self.nblk, float(shift),
                                           native.dptr(self.work), ctypes.byref(h)),
                     "gg_cg_create_blocks")
        self.h = h
        self.shift = float(shift)
        xw = ctypes.c_int()
        native.check(L.gg_cg_get_xwin(self.h, ctypes.byref(xw)), "gg_cg_get_xwin")
        self.xwin = xw.value   # x_defer mode 3's window on this rank (0: pairs)
        native.check(L.gg_cg_get_rderive(self.h, ctypes.byref(xw)), "gg_cg_get_rderive")
        self.rderive = bool(xw.value)   # no r in memory on this rank
        _, n, self.launches = self.dk.block_info()
        self.n = n
        self.n_local = n // (1 << self.d) * self.nblk
        self.local_factors = None
        self.red5 = dev.zeros(5)
        self.red1 = dev.zeros(1)

    def empty(self):
        return dev.empty(self.n_local)

    def zeros(self):
        return dev.zeros(self.n_local)

    def fold(self, b_grid, out=None):
        """This rank's blocks of P b (b: the grid vector, on the device)."""
        return self.dk.block_fold_range(b_grid, self.blk0, self.nblk, out=out)

    def unfold(self, x_local, out=None):
        """This rank's contribution to P^T x (a grid vector; the sum over
        the ranks is the solution)."""
        return self.dk.block_fold_range(x_local, self.blk0, self.nblk, inverse=True, out=out)

    def unfold_all(self, x_blocks, out=None):
        """P^T x of the whole block vector (every rank's blocks in rank
        order, as an all-gather leaves them): the solution on the grid."""
        return self.dk.block_fold_range(x_blocks, 0, 1 << self.d, inverse=True, out=out)

    def apply(self, x, y):
        self.dk.block_matvec_range(x, self.blk0, self.nblk, out=y)

    def _c(self, name, *args):
        native.check(getattr(native.lib(), name)(self.h, *args, native.stream_ptr()), name)

    def start_partial(self, b, x):
        self._c("gg_cg_start_partial", native.dptr(b), native.dptr(x), native.dptr(self.red1))
        return self.red1

    def start_finish(self, rtol, atol):
        self._c("gg_cg_start_finish", native.dptr(self.red1), float(rtol), float(atol))

    def iterate_partial(self):
        self._c("gg_cg_iterate_partial", native.dptr(self.red5))
        return self.red5

    def iterate_finish(self):
        self._c("gg_cg_iterate_finish", native.dptr(self.red5))

    def close_partial(self):
        self._c("gg_cg_close_partial", native.dptr(self.red1))
        return self.red1

    def close_finish(self):
        self._c("gg_cg_close_finish", native.dptr(self.red1))

    def status(self):
        it, conv = ctypes.c_int(), ctypes.c_int()
        res, tol = ctypes.c_double(), ctypes.c_double()
        native.check(native.lib().gg_cg_status(self.h, ctypes.byref(it), ctypes.byref(conv),
                                               ctypes.byref(res), ctypes.byref(tol),
                                               native.stream_ptr()))
        return it.value, bool(conv.value), res.value, tol.value

    def cancels(self):
        v = ctypes.c_int()
        self._c("gg_cg_cancels", ctypes.byref(v))
        return v.value

    def profile(self, enable):
        native.check(native.lib().gg_cg_profile(self.h, int(bool(enable))), "gg_cg_profile")

    def profile_read(self):
        """(profiled iterations, [summed ms per launch position])."""
        nm = ctypes.c_int()
        buf = (ctypes.c_double * 16)()
        native.check(native.lib().gg_cg_profile_read(self.h, ctypes.byref(nm), buf, 16),
                     "gg_cg_profile_read")
        return nm.value, [buf[k] for k in range(self.launches)]

    def __del__(self):
        try:
            if getattr(self, "h", None) is not None and self.h.value:
                native.load().gg_cg_destroy(self.h)
        except Exception:  # noqa: BLE001
            pass


def comm_exchange(comm):
    """(exchange, world, rank) of a `comm` argument: an exchange object
    (TorchExchange, or the tests' virtual-rank exchange) with size() / rank();
    a torch.distributed process group; or True / "world" for the default
    group."""
    if hasattr(comm, "all_reduce") and hasattr(comm, "size"):
        return comm, int(comm.size()), int(comm.rank())
    ex = TorchExchange(None if comm is True or comm == "world" else comm)
    return ex, ex.size(), ex.rank()


def block_solution(eng, ex, xl):
    """The grid solution on every rank from the ranks' block shares.  Default
    (GG_DIST_SOLUTION=gather): one all-gather of the N / G shares (each rank
    receives (G - 1) N / G doubles) and the whole unfold on every rank;
    "reduce": each rank unfolds its own blocks into a zero grid vector (every
    element: each grid point mixes all 2^d blocks) and one all-reduce of N
    doubles sums them (a ring moves 2 (G - 1) N / G per rank).  Exchanges or
    engines without all_gather / unfold_all take the all-reduce."""
    how = os.environ.get("GG_DIST_SOLUTION", "gather")
    if how not in ("gather", "reduce"):
        raise ValueError("GG_DIST_SOLUTION must be 'gather' or 'reduce'")
    if how == "gather" and hasattr(ex, "all_gather") and hasattr(eng, "unfold_all"):
        return eng.unfold_all(ex.all_gather(xl))
    x = eng.unfold(xl)
    ex.all_reduce(x)
    return x


def solve(K, b, shift=0.0, comm=True, rtol=1e-5, atol=0.0, maxiter=None, check_every=20,
          decomposition="auto", engine=None):
    """CG on (K + shift I) x = b across the ranks of `comm` (every rank passes
    the same K and b, numpy or a device tensor; every rank gets the whole x
    back, as a device tensor).  decomposition: "block" (the parity-block
    basis, blocks over 2^K ranks, no exchange), "parity" (factors 0..K-1 in
    the even / odd basis, host-folded blocks), "transpose" (factor 0 sharded,
    two exchanges per matvec) or "auto" (the first that applies, in that
    order).  Returns (x, info, iterations, decomposition).  engine (tests):
    a factory (K, world, rank, shift) -> engine for the block decomposition
    in place of BlockHipEngine (its fold / unfold take host arrays).
    solve.last_cancels: the calling rank's cancelled-beta restarts (block /
    parity; the transpose decomposition's CG has no cancellation test)."""
    import torch
    ex, world, rank = comm_exchange(comm)
    F = [np.asarray(f, dtype=np.float64) for f in K.K]
    m = [f.shape[0] for f in F]
    n = int(np.prod(m))
    maxiter = 10 * n if maxiter is None else int(maxiter)
    if decomposition == "auto":
        # every rank takes the same decomposition: the block basis only where
        # all ranks built it (parity_ok is host arithmetic on identical factors)
        ok = engine is not None or block_shard_ok(K, world)
        if world > 1:
            ok = all(ex.all_gather_object(bool(ok)))
        decomposition = ("block" if ok else
                         "parity" if parity_ok(F, world) else "transpose")
    if decomposition == "block":
        if engine is not None:
            eng = engine(K, world, rank, shift)
            bg = b
        else:
            eng = BlockHipEngine(K, world, rank, shift)
            bg = dev.to_device(b).reshape(-1)
        cg = ParityShardCG(F, world, rank, ex, shift, engine=eng)
        xl, info = cg.solve(eng.fold(bg), rtol, atol, maxiter, check_every)
        x = block_solution(eng, ex, xl)
        it, _, res, tol = cg.status()
        solve.last_cancels = cg.cancels()
    elif decomposition == "parity":
        # device fold of the rank's block, device unfold of its contribution,
        # one all-reduce of the grid vector (round 6: no host arrays)
        bd = dev.to_device(b).reshape(-1)
        cg = ParityShardCG(F, world, rank, ex, shift)
        bl = device_parity_fold(bd, m, world, rank)
        xl, info = cg.solve(bl, rtol, atol, maxiter, check_every)
        solve.last_cancels = cg.cancels()
        x = device_parity_fold(xl, m, world, rank, inverse=True)
        ex.all_reduce(x)
        it, _, res, tol = cg.status()
    elif decomposition == "transpose":
        bd = dev.to_device(b).reshape(-1)
        eng = HipEngine(F, world, rank)
        cg = DistKronCG(eng, ex, shift)
        xl, info = cg.solve(device_shard0_fold(bd, m, world, rank), rtol, atol, maxiter,
                            check_every)
        x = device_shard0_fold(xl, m, world, rank, inverse=True)
        ex.all_reduce(x)
        it, _, rho, tol = cg.status()
        res = float(np.sqrt(max(rho, 0.0)))
        solve.last_cancels = None
    else:
        raise ValueError("decomposition must be 'auto', 'block', 'parity' or 'transpose'")
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    # the global residual norm and tolerance of the finished solve (linalg.cg.last)
    solve.last_resid = (float(res), float(tol))
    return x, info, it, decomposition
