"""Multi-GPU sharding logic, exercised with world_size 2 on
the CPU gloo backend: contiguous channel shards, max-over-ranks timing,
counter sums and the scan-line gather of per-channel levels."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fmtuner-sdr_amd"))
    import fmx_dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = fmx_dist.shard(total, world, rank)
    levels = torch.arange(b, e, dtype=torch.float32) * 0.5
    allv = fmx_dist.gather_levels(levels)
    tmax = fmx_dist.max_over_ranks(1.0 + rank)
    sums = fmx_dist.sum_counters([e - b, 1.0])
    q.put((rank, b, e, allv.tolist(), tmax, sums.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_covers_all_channels_balanced():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "fmtuner-sdr_amd"))
    import fmx_dist
    for total in (1, 7, 4096, 16384, 10_000):
        for world in (1, 2, 4, 8):
            spans = [fmx_dist.shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("world,total", [(2, 16), (2, 17), (3, 10)])
def test_gloo_gather_and_reduce(world, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, b, e, allv, tmax, sums in res:
        assert allv == [0.5 * i for i in range(total)]
        assert tmax == float(world)
        assert sums == [total, float(world)]
