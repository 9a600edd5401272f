"""bench.py's multi-rank plumbing on the CPU (no GPU): `--gpus N` without a
launcher spawns N ranks under torch.distributed.run before any GPU call,
shards the channels with fmx_dist.shard, and carries the collectives
(gather of the scan levels, summed channel count) over gloo (--dry-run)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=240, env=env)
    return r


@pytest.mark.parametrize("workload,n,total,rank0", [("cfg3", 2, 8192, 4096), ("cfg4", 2, 16384, 8192),
                                                     ("cfg4", 3, 16384, 5462)])
def test_spawned_ranks_shard_and_gather(workload, n, total, rank0):
    r = _run(["--gpus", str(n), "--workload", workload, "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == n and d["world_reported"] == n
    assert d["total_channels"] == total and d["channels_summed"] == total
    assert d["channels_rank0"] == rank0
    assert d["gathered"] == total
    assert d["scaling"] == ("weak" if workload == "cfg3" else "strong")


def test_single_rank_dry_run():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["channels_summed"] == 4096 and d["scaling"] == "weak"


def test_driver_scaling_invocation_defaults_to_cfg4():
    """The driver's N>1 command names no workload: it gets BASELINE's Cfg4
    curve (16384 channels sharded, 2048 per GPU at N=8)."""
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["total_channels"] == 16384 and d["channels_rank0"] == 8192 and d["scaling"] == "strong"


def test_launcher_world_mismatch_fails():
    r = _run(["--gpus", "4", "--dry-run"], env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
