"""Test-only helpers for the sharded Kronecker CG (gp_grief_amd/distributed.py).

NumpyEngine: the engine interface of distributed.HipEngine restated with NumPy
on torch CPU tensors (so gloo collectives work on them).  Its layout logic is
written independently of the HIP kernels' address maps (reshape / transpose
here, integer address arithmetic there), so agreement checks both.

ThreadExchange: all-to-all / all-reduce between virtual ranks that run as
Python threads in one process (used to drive G HipEngines on one GPU).
"""
import threading

import numpy as np
import torch

import oracle


class NumpyEngine(object):
    def __init__(self, factors, world, rank):
        self.F = [np.asarray(f, dtype=np.float64) for f in factors]
        self.m = [f.shape[0] for f in self.F]
        self.G, self.rank = world, rank
        self.s0 = self.m[0] // world
        self.n_local = int(np.prod(self.m)) // world
        self.red = torch.zeros(2, dtype=torch.float64)
        self.sc = dict(rho=0.0, rho_prev=0.0, alpha=0.0, beta=0.0, tol=0.0, iters=0, done=False,
                       first=True)

    def empty(self):
        return torch.empty(self.n_local, dtype=torch.float64)

    def zeros(self):
        return torch.zeros(self.n_local, dtype=torch.float64)

    def phase1(self, x, send, r=None):
        xv = x.numpy()
        if r is not None and not self.sc["done"]:
            xv[:] = r.numpy() if self.sc["first"] else self.sc["beta"] * xv + r.numpy()
        d, G, s0 = len(self.m), self.G, self.s0
        X = xv.reshape(self.m[1:] + [s0])
        X = np.moveaxis(X, -1, 0)                      # (s0, m1, ..., m_{d-1})
        for k in range(1, d):
            X = np.moveaxis(np.tensordot(self.F[k], X, axes=([1], [k])), 0, k)
        p1 = self.m[1]
        Y = X.reshape(s0, G, p1 // G, -1).transpose(1, 0, 2, 3)
        send.numpy()[:] = Y.reshape(-1)

    def phase2(self, recv, send):
        m0 = self.m[0]
        Z = self.F[0].dot(recv.numpy().reshape(m0, -1))   # (p0, C)
        C = Z.shape[1]
        send.numpy()[:] = Z.T.reshape(C, self.G, self.s0).transpose(1, 0, 2).reshape(-1)

    # ---- the fused recurrence (HipEngine.phase1_fused / fused_*), restated
    # from cg_fused_scalars_kernel (xmode 2, conjugacy r.q) and the balanced
    # x deferral; partial sums are plain local dot products here
    supports_fused = True

    def phase1_fused(self, p_old, p_new, send, r, q_old, x, shift, push):
        sc = self.sc
        if sc["done"]:
            return
        rv, pn = r.numpy(), p_new.numpy()
        qe = q_old.numpy() + shift * p_old.numpy()     # q_old = K p_old, unshifted
        if sc["pending"]:
            rv -= sc["alpha"] * qe
        self.rr_local = float(np.dot(rv, rv))
        pn[:] = rv + sc["beta"] * p_old.numpy()
        self.pqo_local = float(np.dot(pn, qe))
        h = sc["xh"]
        if h < 2:   # the side job: half h of the active pair
            H = self.half()
            lo, hi = (0, H) if h == 0 else (H, self.n_local)
            xv = x.numpy()
            xv[lo:hi] += sc["xc"][0] * sc["xp"][0].numpy()[lo:hi] + \
                sc["xc"][1] * sc["xp"][1].numpy()[lo:hi]
        self.phase1(p_new, send)

    def half(self):
        return min(2 * ((self.n_local + 3) // 4), self.n_local)

    def fused_post(self, q, p, shift):
        self.red5 = getattr(self, "red5", torch.zeros(5, dtype=torch.float64))
        if self.sc["done"]:
            return
        qv = q.numpy() + shift * p.numpy()   # q itself stays K p
        self.red5[:] = torch.tensor([self.rr_local, self.pqo_local, float(np.dot(p.numpy(), qv)),
                                     0.0, float(np.dot(qv, qv))], dtype=torch.float64)

    def fused_reduce_buffer(self):
        self.red5 = getattr(self, "red5", torch.zeros(5, dtype=torch.float64))
        return self.red5

    def fused_scalars(self, p_new):
        sc = self.sc
        if sc["done"]:
            return
        rr, pqo, pq, _, qq = [float(v) for v in self.red5]
        if sc["pending"]:
            sc.update(rho_prev=sc["rho"], rho=rr, iters=sc["iters"] + 1)
            if not np.sqrt(rr) >= sc["tol"]:
                sc.update(done=True, pending=False)
                if sc["xh"] < 2:
                    sc["xh"] += 1
                return
        rho = sc["rho"]
        alpha = rho / pq
        rq = pq - sc["beta"] * pqo
        rt = rho - 2.0 * alpha * rq + alpha * alpha * qq
        repair = rt < 1e-6 * rho
        sc.update(alpha=alpha, beta=0.0 if repair else rt / rho, first=False, pending=True)
        if sc["xh"] < 2:
            sc["xh"] += 1
        if not sc["xs"]:
            sc.update(xs=True, xsc=alpha, xsp=p_new)
        else:
            sc.update(xc=[sc["xsc"], alpha], xp=[sc["xsp"], p_new], xh=0, xs=False)

    def fused_close(self, x, r, q, p, shift):
        sc = self.sc
        xv = x.numpy()
        if sc["xs"]:
            xv += sc["xsc"] * sc["xsp"].numpy()
        if sc["xh"] < 2:
            lo = 0 if sc["xh"] == 0 else self.half()
            xv[lo:] += sc["xc"][0] * sc["xp"][0].numpy()[lo:] + \
                sc["xc"][1] * sc["xp"][1].numpy()[lo:]
        sc.update(xh=2, xs=False)
        self.red[0] = 0.0
        if not sc["done"] and sc["pending"]:
            rv = r.numpy()
            rv -= sc["alpha"] * (q.numpy() + shift * p.numpy())
            self.red[0] = float(np.dot(rv, rv))

    def fused_close_rho(self):
        sc = self.sc
        if sc["done"] or not sc["pending"]:
            return
        s = float(self.red[0])
        sc.update(rho_prev=sc["rho"], rho=s, iters=sc["iters"] + 1, first=False, pending=False)
        sc["beta"] = s / sc["rho_prev"]
        if not np.sqrt(s) >= sc["tol"]:
            sc["done"] = True

    def local_dot(self, x, y):
        self.red[0] = float(np.dot(x.numpy(), y.numpy()))

    def cg_init(self, rtol, atol):
        s = float(self.red[0])
        self.sc.update(rho=s, tol=max(atol, rtol * np.sqrt(s)), iters=0, first=True,
                       pending=False, alpha=0.0, beta=0.0, xh=2, xs=False)
        self.sc["done"] = s == 0.0 or not np.sqrt(s) >= self.sc["tol"]

    def shift_dot(self, q, p, shift):
        if self.sc["done"]:
            return
        qv = q.numpy()
        qv += shift * p.numpy()
        self.red[0] = float(np.dot(p.numpy(), qv))

    def cg_alpha(self):
        if not self.sc["done"]:
            self.sc["alpha"] = self.sc["rho"] / float(self.red[0])

    def cg_update(self, x, r, p, q):
        if self.sc["done"]:
            return
        a = self.sc["alpha"]
        x.numpy()[:] += a * p.numpy()
        r.numpy()[:] -= a * q.numpy()
        self.red[0] = float(np.dot(r.numpy(), r.numpy()))

    def cg_rho(self):
        if self.sc["done"]:
            return
        s = float(self.red[0])
        self.sc.update(rho_prev=self.sc["rho"], rho=s, iters=self.sc["iters"] + 1, first=False)
        self.sc["beta"] = s / self.sc["rho_prev"]
        if not np.sqrt(s) >= self.sc["tol"]:
            self.sc["done"] = True

    def cg_status(self):
        return self.sc["iters"], self.sc["done"], self.sc["rho"], self.sc["tol"]

    def reduce_buffer(self):
        return self.red[:1]

    def copy(self, dst, src):
        dst.copy_(src)

    def zero(self, x):
        x.zero_()


class ThreadExchange(object):
    """Collectives between `world` threads of one process (virtual ranks)."""

    def __init__(self, world):
        self.G = world
        self.bar = threading.Barrier(world)
        self.slots = [None] * world
        self.local = threading.local()

    def bind(self, rank):
        self.local.rank = rank

    def all_to_all(self, out, inp):
        g = self.local.rank
        self.slots[g] = inp
        self.bar.wait()
        c = out.numel() // self.G
        for h in range(self.G):
            out[h * c:(h + 1) * c].copy_(self.slots[h][g * c:(g + 1) * c])
        self.bar.wait()

    in_process = True  # peers' device buffers are plain pointers

    def size(self):
        return self.G

    def rank(self):
        return self.local.rank

    def barrier(self):
        torch.cuda.synchronize()
        self.bar.wait()

    def all_gather_object(self, obj):
        g = self.local.rank
        self.slots[g] = obj
        self.bar.wait()
        out = list(self.slots)
        self.bar.wait()
        return out

    def all_gather(self, t):
        g = self.local.rank
        self.slots[g] = t.clone()
        self.bar.wait()
        out = torch.cat(list(self.slots))
        self.bar.wait()
        return out

    def all_reduce(self, t):
        g = self.local.rank
        self.slots[g] = t.clone()
        self.bar.wait()
        acc = self.slots[0].clone()
        for h in range(1, self.G):
            acc += self.slots[h]
        self.bar.wait()
        t.copy_(acc)
        self.bar.wait()


def bind_device(rank):
    """One GPU per rank when the box has several (rank % device count), so
    the process tests run cross-device -- peer stores and RCCL over xGMI --
    on any multi-GPU node; on one GPU every rank shares cuda:0."""
    n = torch.cuda.device_count()
    if n > 0:
        torch.cuda.set_device(rank % n)
    return rank % n if n > 0 else None


def run_threads(world, fn):
    """Run fn(rank) in `world` threads; re-raise the first failure."""
    errs = [None] * world
    out = [None] * world

    def body(g):
        try:
            out[g] = fn(g)
        except BaseException as e:  # pragma: no cover - surfaced below
            errs[g] = e

    ts = [threading.Thread(target=body, args=(g,)) for g in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    return out


def reference_factors(m, d, seed=0):
    g = np.linspace(0, 1, m)
    return [oracle.cov_1d("RBF", g, g, 1.0, 0.15 * (1 + 0.1 * k)) + 1e-12 * np.eye(m)
            for k in range(d)]


def make_factors(m, d):
    """bench.py's GG_BENCH_ENGINE hook: the factors of the CPU rehearsal."""
    return reference_factors(m, d)


class ParityNumpyEngine(object):
    """distributed.ParityHipEngine restated with NumPy on torch CPU tensors:
    this rank's block of the parity-sharded operator (oracle.kron_matvec on
    the local factors) and the fused CG recurrence split at its one
    reduction (gg_cg_iterate_partial / _finish: r -= alpha q_old and r.r,
    p = r + beta p and p.q_old, q = A p + s p with p.q and q.q; the scalars
    from the global sums with beta from the |r - alpha q|^2 expansion and
    r.q from the conjugacy identity; a cancelled beta restarts with p = r).
    x is updated one step late (no deferred pairs)."""

    def __init__(self, factors, world, rank, shift):
        from gp_grief_amd.distributed import parity_local_factors
        self.F = parity_local_factors(factors, world, rank)
        self.shift = float(shift)
        self.n_local = int(np.prod([f.shape[0] for f in self.F]))
        self.red5 = torch.zeros(5, dtype=torch.float64)
        self.red1 = torch.zeros(1, dtype=torch.float64)
        self.sc = {}

    def empty(self):
        return torch.empty(self.n_local, dtype=torch.float64)

    def zeros(self):
        return torch.zeros(self.n_local, dtype=torch.float64)

    def apply(self, x, y):
        y.numpy()[:] = oracle.kron_matvec(self.F, x.numpy())

    def _A(self, v):
        return oracle.kron_matvec(self.F, v) + self.shift * v

    def start_partial(self, b, x):
        self.x = x
        self.r = b.numpy().copy()
        x.numpy()[:] = 0.0
        self.p = np.zeros(self.n_local)
        self.q = np.zeros(self.n_local)
        self.red1[0] = float(self.r @ self.r)
        return self.red1

    def start_finish(self, rtol, atol):
        s = float(self.red1[0])
        tol = max(atol, rtol * np.sqrt(s))
        self.sc = dict(rho=s, tol=tol, iters=0, pending=False, alpha=0.0, beta=0.0,
                       done=(s == 0.0 or not np.sqrt(s) >= tol))

    def iterate_partial(self):
        sc = self.sc
        if sc["done"]:
            return self.red5
        if sc["pending"]:
            self.x.numpy()[:] += sc["alpha"] * self.p
            self.r -= sc["alpha"] * self.q
        pn = self.r + sc["beta"] * self.p
        pqo = float(pn @ self.q)
        qn = self._A(pn)
        self.red5[:] = torch.tensor([float(self.r @ self.r), pqo, float(pn @ qn), 0.0,
                                     float(qn @ qn)], dtype=torch.float64)
        self.p, self.q = pn, qn
        return self.red5

    def iterate_finish(self):
        sc = self.sc
        if sc["done"]:
            return
        rr, pqo, pq, _, qq = [float(v) for v in self.red5]
        if sc["pending"]:
            sc.update(rho=rr, iters=sc["iters"] + 1)
            if not np.sqrt(rr) >= sc["tol"]:
                sc.update(done=True, pending=False)
                return
        rho = sc["rho"]
        alpha = rho / pq
        rq = pq - sc["beta"] * pqo
        rt = rho - 2.0 * alpha * rq + alpha * alpha * qq
        sc.update(alpha=alpha, beta=0.0 if rt < 1e-6 * rho else rt / rho, pending=True)

    def close_partial(self):
        sc = self.sc
        self.red1[0] = 0.0
        if sc["pending"] and not sc["done"]:
            self.x.numpy()[:] += sc["alpha"] * self.p
            self.r -= sc["alpha"] * self.q
            self.red1[0] = float(self.r @ self.r)
        return self.red1

    def close_finish(self):
        sc = self.sc
        if sc["done"] or not sc["pending"]:
            return
        s = float(self.red1[0])
        sc.update(beta=s / sc["rho"], rho=s, iters=sc["iters"] + 1, pending=False)
        if not np.sqrt(s) >= sc["tol"]:
            sc["done"] = True

    def status(self):
        sc = self.sc
        res = np.sqrt(max(sc["rho"], 0.0))
        return sc["iters"], bool(sc["done"] and res < sc["tol"]), res, sc["tol"]

    def profile(self, enable):
        pass


class BlockNumpyEngine(ParityNumpyEngine):
    """distributed.BlockHipEngine restated with NumPy on torch CPU tensors:
    rank g's blocks [g 2^d / G, (g + 1) 2^d / G) of the operator in its
    parity-block basis (oracle.kron.block_factors per block, kron_matvec
    inside each), with ParityNumpyEngine's fused recurrence; fold / unfold
    through oracle.kron.block_fold (the unfold is this rank's contribution,
    the rest of the block vector zero)."""

    mode = "block"

    def __init__(self, K, world, rank, shift):
        from gp_grief_amd.distributed import block_range
        F = [np.asarray(f, dtype=np.float64) for f in K.K]
        self.ms = [f.shape[0] for f in F]
        self.d = len(F)
        self.blk0, self.nblk = block_range(self.d, world, rank)
        st = [oracle.kron.block_factors(f) for f in F]
        self.nb = int(np.prod([m // 2 for m in self.ms]))
        self.blocks = [[st[k][(b >> (self.d - 1 - k)) & 1] for k in range(self.d)]
                       for b in range(self.blk0, self.blk0 + self.nblk)]
        self.shift = float(shift)
        self.n_local = self.nb * self.nblk
        self.red5 = torch.zeros(5, dtype=torch.float64)
        self.red1 = torch.zeros(1, dtype=torch.float64)
        self.sc = {}

    def profile(self, enable):
        self._prof_on = bool(enable)
        self._prof_n, self._prof_s = 0, 0.0

    def profile_read(self):
        """(iterations, [ms per launch position]): the host time of the
        block products split evenly over the d - 1 launch positions."""
        L = self.d - 1
        return self._prof_n, [1e3 * self._prof_s / L] * L

    def _A(self, v):
        import time
        t0 = time.perf_counter()
        out = self._Kb(v) + self.shift * v
        if getattr(self, "_prof_on", False):
            self._prof_n += 1
            self._prof_s += time.perf_counter() - t0
        return out

    def _Kb(self, v):
        hs = [m // 2 for m in self.ms]
        v = oracle.kron.slab_tile(v, hs, inverse=True)   # the block layout's slab tiling
        out = np.empty_like(v)
        for j, fs in enumerate(self.blocks):
            out[j * self.nb:(j + 1) * self.nb] = oracle.kron_matvec(
                fs, v[j * self.nb:(j + 1) * self.nb])
        return oracle.kron.slab_tile(out, hs)

    def apply(self, x, y):
        y.numpy()[:] = self._Kb(x.numpy())

    def fold(self, b):
        bb = oracle.kron.block_fold(np.asarray(b, dtype=np.float64).reshape(-1), self.ms)
        return torch.from_numpy(bb[self.blk0 * self.nb:(self.blk0 + self.nblk) * self.nb].copy())

    def unfold(self, xl):
        full = np.zeros(self.nb << self.d)
        full[self.blk0 * self.nb:(self.blk0 + self.nblk) * self.nb] = np.asarray(xl)
        return torch.from_numpy(oracle.kron.block_fold(full, self.ms, inverse=True))

    def unfold_all(self, xall):
        """P^T of the whole block vector (the ranks' shares in rank order)."""
        return torch.from_numpy(oracle.kron.block_fold(np.asarray(xall, dtype=np.float64),
                                                       self.ms, inverse=True))
