"""bench.py's roofline bookkeeping on the host (no GPU): pass counts per
launch position, the kernel each position runs, and the choice of the
rocprof-dominant kernel (largest total time per iteration)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


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
