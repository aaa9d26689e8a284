"""bench.py --gpus N starts one rank per device itself (torch.distributed.run
as a child process) and reports the world size it ran at.  Rehearsed on CPU:
gloo backend, the NumPy test engine (GG_BENCH_ENGINE), 2 ranks."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run_bench(world, shard, block_engine=False):
    env = dict(os.environ)
    env.update(GG_BENCH_BACKEND="gloo", GG_BENCH_ENGINE="dist_helpers:NumpyEngine",
               GG_BENCH_PARITY_ENGINE="dist_helpers:ParityNumpyEngine",
               PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "tests"), ROOT,
                                           env.get("PYTHONPATH", "")]),
               OMP_NUM_THREADS="1")
    if block_engine:
        env["GG_BENCH_BLOCK_ENGINE"] = "dist_helpers:BlockNumpyEngine"
    else:
        env.pop("GG_BENCH_BLOCK_ENGINE", None)
    env.pop("WORLD_SIZE", None)
    env.pop("GG_DIST_SHARD", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                          "--grid", "8", "--dims", "3", "--steps", "3", "--warmup", "1",
                          "--shard", shard],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world,shard", [(2, "transpose"), (2, "auto"), (4, "parity")])
def test_bench_gpus_flag_spawns_ranks(world, shard):
    """transpose: factor 0 sharded, two all-to-alls per matvec (NumpyEngine);
    auto / parity: the parity blocks, no exchange (ParityNumpyEngine).  On
    CPU (gloo, no GPU) the line says it is a rehearsal, not a scaling run."""
    rec = _run_bench(world, shard)
    assert rec["n_gpus"] == world
    assert rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["scaling"] == "rehearsal" and rec["value"] > 0
    assert rec["backend"] == "gloo" and rec["physical_gpus"] == 0
    assert "RCCL" not in rec["config"]["parallelism"]
    assert rec["config"]["exchange"] == ("a2a" if shard == "transpose" else "none")


@pytest.mark.parametrize("world,shard", [(2, "block"), (4, "auto"), (8, "block")])
def test_bench_block_sharded_line(world, shard):
    """The block decomposition's N > 1 line (BlockNumpyEngine standing in for
    BlockHipEngine): the per-rank roofline dict of the dominant launch, the
    all-reduce's share of the iteration, the N = 1 cpu_baseline reference."""
    rec = _run_bench(world, shard, block_engine=True)
    assert rec["n_gpus"] == world and rec["value"] > 0
    cfg = rec["config"]
    assert cfg["cg_basis"] == "block" and cfg["exchange"] == "none"
    assert cfg["blocks_per_rank"] == 8 // world and cfg["n_per_rank"] == 8 ** 3 // world
    assert cfg["launches_per_iteration"] == 2
    roof = rec["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "scope"):
        assert k in roof
    assert roof["bound"] in ("hbm", "mfma") and roof["achieved"] > 0
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-9 * max(1.0, roof["frac"])
    ar = rec["allreduce"]
    assert ar["doubles_per_iteration"] == 5 and 0.0 <= ar["share_of_iteration"] <= 1.0
    assert rec["cpu_baseline"]["value"] is None and "n_gpus = 1" in \
        rec["cpu_baseline"]["reference"]
    assert rec["scaling"] == "rehearsal" and rec["backend"] == "gloo"
    assert len(rec["local_launch_ms"]) == 2


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr
