"""bench.py's multi-GPU launch contract on CPU: `bench.py --gpus N` without a
torch.distributed environment starts N rank processes itself (torch.distributed.run
as a child, before any GPU call).  Default workloads: C3 at N = 1 (the north-star
config), C4 strong-scaled at N > 1 (BASELINE config 4, "vertex-partitioned across
2/4/8 MI355X"); --weak gives the R-MAT 24 + log2 N series for power-of-two N."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--launch-check"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]


def test_single_gpu_default_is_c3():
    (row,) = _launch()
    assert row["world"] == 1 and row["config_id"] == "C3" and row["cfg"]["scale"] == 24


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_spawns_ranks_on_c4(n):
    rows = _launch("--gpus", str(n))
    assert sorted(r["rank"] for r in rows) == list(range(n))
    assert all(r["world"] == n and r["local_rank"] == r["rank"] for r in rows)
    assert all(r["config_id"] == "C4" and r["cfg"]["scale"] == 26 and r["scaling"] == "strong" for r in rows)


@pytest.mark.parametrize("n,scale,cid", [(2, 25, "R-MAT-25"), (4, 26, "C4")])
def test_weak_series(n, scale, cid):
    rows = _launch("--gpus", str(n), "--weak")
    assert len(rows) == n
    assert all(r["config_id"] == cid and r["cfg"]["scale"] == scale and r["scaling"] == "weak" for r in rows)


def test_weak_refuses_non_power_of_two():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--weak", "--launch-check"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "power-of-two" in r.stderr


def test_explicit_config_is_strong_scaling():
    rows = _launch("--gpus", "2", "--config", "C5")
    assert len(rows) == 2 and all(r["config_id"] == "C5" and r["scaling"] == "strong" for r in rows)
