"""bench.py's roofline bookkeeping on the host (no GPU): pass counts per
launch position, the kernel each position runs, and the choice of the
rocprof-dominant kernel (largest total time per iteration)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import numpy as np  # noqa: E402
import pytest  # noqa: E402


def test_launch_passes_fused_layout0_d4():
    # prologue 6, x side job split over positions 1 and 2, epilogue 4: 17 passes
    assert bench.launch_passes(4, "fused", 0) == [6, 3.5, 3.5, 4]
    assert sum(bench.launch_passes(4, "fused", 0)) == 17


def test_launch_kernels_groups_side_job_positions():
    assert bench.launch_kernels(4, "fused", 0) == ["prologue", "side", "side", "epilogue"]
    assert bench.launch_kernels(3, "fused", 0) == ["prologue", "side", "epilogue"]
    assert bench.launch_kernels(4, "textbook", 0) == ["prologue", "plain", "plain", "epilogue"]


def test_dominant_group_is_largest_total_not_largest_launch():
    per = [17.3, 12.3, 12.2, 13.9]          # ms by position (fused, d = 4)
    kinds = bench.launch_kernels(4, "fused", 0)
    group, kind = bench.dominant_group(per, kinds)
    assert kind == "side" and group == [1, 2]
    roof, extra = bench.roofline_report(per, 200 ** 4, 200, 4, "fused", 56.5, 0)
    assert roof["positions"] == [1, 2]
    assert abs(roof["launch_ms"] - 12.25) < 1e-9
    assert roof["bound"] == "mfma"          # 8.1 ms of MFMA > 5.6 ms of HBM at 3.5 passes
    assert extra["largest_launch"]["position"] == 0
    assert 0 < roof["frac"] < 1


def test_roofline_folded_launches_are_hbm_bound():
    """With every factor on the centrosymmetric split the side-job launch
    executes n m FLOP (4.1 ms of MFMA at 200^4) against 3.5 passes of HBM
    (5.6 ms): priced against HBM."""
    per = [15.5, 9.2, 9.3, 11.7]
    roof, extra = bench.roofline_report(per, 200 ** 4, 200, 4, "fused", 46.5, 0, 0b1111)
    assert roof["positions"] == [1, 2] and roof["bound"] == "hbm"
    assert abs(roof["flop_per_launch"] - 200 ** 4 * 200) < 1
    assert abs(roof["achieved"] - 3.5 * 8 * 200 ** 4 / 9.25e-3 / 1e9) < 1e-6
    # x deferred to every other iteration: 1 pass per side launch on average
    assert bench.launch_passes(4, "fused", 0, True) == [6, 3, 3, 4]
    assert bench.launch_passes(4, "fused", 1, True) == [5, 3, 3, 5]
    # conjugacy r.q: the epilogue reads p only
    assert bench.launch_passes(4, "fused", 0, 2, True) == [6, 3, 3, 3]
    assert extra["fold_mask"] == 0b1111
    assert abs(extra["matvec_dense_equivalent_tflops"] - 2 * extra["matvec_tflops"]) < 1e-9


def test_rhs_identical_in_every_shard_layout():
    """bench.py's right-hand side is a function of the global index, so the
    sharded layouts of every N hold the single-GPU vector."""
    import torch
    from gp_grief_amd.distributed import scatter_global
    m, d = 8, 3
    dev = torch.device("cpu")
    y = bench.grid_rhs_device(m, d, torch, dev).numpy()
    assert y.shape == (m ** d,) and abs(y).max() < 3.2
    for world in (1, 2, 4, 8):
        for rank in range(world):
            loc = bench.local_rhs(m, d, world, rank, torch, dev).numpy()
            ref = scatter_global(y, [m] * d, world, rank)
            assert (loc == ref).all()


def test_pmc_traffic_requires_matching_sources(tmp_path, monkeypatch):
    import json
    rec = {"recurrence": "fused", "fusion_layout": 0, "fold_mask": 15, "x_deferred": True,
           "source_sha256": bench.kernel_source_hash(), "calibrated_on_own_pattern": True,
           "per_position": [{"position": k, "traffic_bytes": 1e10 * (k + 1)} for k in range(4)]}
    os.makedirs(os.path.dirname(tmp_path / bench.PMC_JSON))
    path = tmp_path / bench.PMC_JSON
    json.dump(rec, open(path, "w"))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    for rel in bench.KERNEL_SOURCES:      # the same sources under the fake root
        os.makedirs(os.path.dirname(tmp_path / rel), exist_ok=True)
        with open(os.path.join(ROOT, rel), "rb") as f, open(tmp_path / rel, "wb") as g:
            g.write(f.read())
    t, src = bench.pmc_traffic(200, 4, [1, 2], "fused", 0, 15)
    assert t == 2.5e10 and src == bench.PMC_JSON
    t, why = bench.pmc_traffic(200, 4, [1, 2], "fused", 0, 0)
    assert t is None and "fold" in why
    with open(tmp_path / bench.KERNEL_SOURCES[0], "ab") as g:
        g.write(b"// changed\n")
    t, why = bench.pmc_traffic(200, 4, [1, 2], "fused", 0, 15)
    assert t is None and why.startswith("stale")


def test_cpu_share_reports_its_limit():
    threads, share = bench.cpu_share()
    assert threads >= 1 and share["limited_by"] in ("affinity_mask", "cgroup_cpu_quota",
                                                    "OMP_NUM_THREADS")
    assert threads <= share["affinity_cpus"]


@pytest.mark.parametrize("world,m,d", [(2, 8, 3), (4, 6, 3), (8, 4, 4)])
def test_parity_local_rhs_matches_host_fold(world, m, d):
    """bench.parity_local_rhs (device formula of every rank's even / odd block
    of the right-hand side) equals distributed.parity_fold of the global one."""
    import torch
    from gp_grief_amd.distributed import parity_fold
    yg = bench.rhs_at(torch.arange(m ** d, dtype=torch.int64), m, d, torch).numpy()
    ref = parity_fold(yg, [m] * d, world)
    for g in range(world):
        loc = bench.parity_local_rhs(m, d, world, g, torch, torch.device("cpu")).numpy()
        assert np.abs(loc - ref[g]).max() < 1e-13 * np.abs(yg).max()
