"""bench.py --gpus N starts one rank per device itself (torch.distributed.run
as a child process) and reports the world size it ran at.  Rehearsed on CPU:
gloo backend, the NumPy test engine (GG_BENCH_ENGINE), 2 ranks."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.parametrize("world,shard", [(2, "transpose"), (2, "auto"), (4, "parity")])
def test_bench_gpus_flag_spawns_ranks(world, shard):
    """transpose: factor 0 sharded, two all-to-alls per matvec (NumpyEngine);
    auto / parity: the parity blocks, no exchange (ParityNumpyEngine)."""
    env = dict(os.environ)
    env.update(GG_BENCH_BACKEND="gloo", GG_BENCH_ENGINE="dist_helpers:NumpyEngine",
               GG_BENCH_PARITY_ENGINE="dist_helpers:ParityNumpyEngine",
               PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "tests"), ROOT,
                                           env.get("PYTHONPATH", "")]),
               OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("GG_DIST_SHARD", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                          "--grid", "8", "--dims", "3", "--steps", "3", "--warmup", "1",
                          "--shard", shard],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == world
    assert rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["scaling"] == "strong" and rec["value"] > 0
    assert rec["config"]["exchange"] == ("a2a" if shard == "transpose" else "none")


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr
