"""Gram A = Phi^T Phi (lower, n x p Phi) timed with the rows of Phi padded to
a leading dimension lda >= p: does the row stride of the DMA'd k-rows set the
small-p Gram's rate?  One JSON line per (p, lda).  Tuning aid."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gp_grief_amd import native
    lib = native.lib()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    shapes = [(1000, [1000, 1008, 1016, 1024, 1040, 1064, 1096, 1152, 1280]),
              (2000, [2000, 2016, 2048, 2064])]
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0)
    for p, ldas in shapes:
        ref = None
        for lda in ldas:
            full = torch.randn((n, lda), dtype=torch.float64, device="cuda", generator=gen)
            full[:, :p] = torch.randn((n, p), dtype=torch.float64, device="cuda",
                                      generator=torch.Generator(device="cuda").manual_seed(1))
            C = torch.zeros((p, p), dtype=torch.float64, device="cuda")
            need = ctypes.c_int64()
            native.check(lib.gg_gemm_workspace_elems(1, 0, p, p, n, 1, ctypes.byref(need)))
            work = torch.empty(max(1, need.value), dtype=torch.float64, device="cuda")

            def f():
                native.check(lib.gg_gemm(1, 0, p, p, n, 1.0, native.dptr(full), lda,
                                         native.dptr(full), lda, 0.0, native.dptr(C), p, 1,
                                         native.dptr(work), int(need.value),
                                         native.stream_ptr()), "gg_gemm")
            f()
            torch.cuda.synchronize()
            best = None
            for _ in range(5):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
            L = torch.tril(C)
            if ref is None:
                ref = L.clone()
            print(json.dumps({"p": p, "lda": lda, "ms": best, "tflops": n * p * p / best / 1e9,
                              "same_as_unpadded": bool(torch.equal(L, ref))}), flush=True)
            del full, C, work
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
