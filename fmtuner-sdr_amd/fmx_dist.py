"""fmx_dist -- channel sharding across the GPUs of one node.

Channels are independent, so the data path needs no collective: GPU g owns
the contiguous channel range shard(C, G, g).  RCCL (torch.distributed
"nccl") is used only off the data path:
  * max_over_ranks()      the bench's max-over-ranks step time;
  * sum_counters()        per-GPU counters (samples, groups, errors);
  * gather_levels()       the multi-channel scan line: every rank's
                          per-channel RF levels gathered to all ranks
                          (4 B/channel/block, the GPU replacement of the
                          reference's sequential retune scan, main.cpp:1064-1121).
"""
import torch
import torch.distributed as dist


def shard(total, world, rank):
    """[begin, end) of the channels owned by `rank` (contiguous, balanced)."""
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def _ready():
    return dist.is_available() and dist.is_initialized()


def max_over_ranks(value, device="cpu"):
    if not _ready():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_counters(values, device="cpu"):
    t = torch.as_tensor(values, dtype=torch.float64, device=device).clone()
    if _ready():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def gather_levels(levels):
    """levels: this rank's per-channel float tensor (shard lengths may differ
    by one when C % world != 0).  Returns the concatenation over ranks in rank
    order: lengths are exchanged first, shards padded to the longest for the
    all_gather, and the padding dropped."""
    if not _ready():
        return levels
    world = dist.get_world_size()
    n = torch.tensor([levels.numel()], dtype=torch.int64, device=levels.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    lens = [int(x.item()) for x in ns]
    width = max(lens)
    padded = torch.zeros(width, dtype=levels.dtype, device=levels.device)
    padded[:levels.numel()] = levels.reshape(-1)
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded)
    return torch.cat([p[:k] for p, k in zip(parts, lens)])
