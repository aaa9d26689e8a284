"""Diagnostic: is the prologue launch's slow / fast mode a property of the
process or of the allocation?  Re-creates the CG state (fresh work buffer)
several times in one process, shifting the allocator with small keep-alive
tensors, and prints the mode-product times of each instance."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench
import gp_grief_amd as gg

m, d, s = 200, 4, 0.1
K, F = bench.grid_factors(m, d)
dev = torch.device("cuda", 0)
y = bench.grid_rhs_device(m, d, torch, dev)
keep = []
for trial in range(6):
    solver = gg.linalg.KronCG(K, s)
    solver.start(y, rtol=0.0, atol=0.0)
    solver.iterate(2, check_every=0)
    solver.profile(True)
    solver.iterate(8, check_every=0)
    torch.cuda.synchronize()
    n_mv, mode_ms = solver.profile_read()
    solver.profile(False)
    print(trial, "work ptr 0x%x" % solver.work.data_ptr(),
          [round(t / n_mv, 2) for t in mode_ms], flush=True)
    del solver
    torch.cuda.empty_cache()
    keep.append(torch.empty((trial + 1) * 3 * 2 ** 20 + 12345, dtype=torch.float64, device=dev))
