"""Multi-GPU: one process per GPU, the header stream sharded contiguously,
tables replicated (every rank loads the same maps), and one SUM all-reduce
of the u64 counter block over RCCL (xGMI) per reporting interval — the only
collective on this path.  Verdicts need no exchange: each
header's verdict is a pure function of the header and the tables."""
from __future__ import annotations

import os


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous slice [start, end) of an n_total-header stream for rank."""
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def allreduce_block(t, group=None):
    """SUM all-reduce of an int64 counter block in place (two's-complement
    int64 addition is u64 addition mod 2^64, so the sums are exact)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def allreduce_counters(dp, group=None, stream=None):
    """Export this rank's device counters, all-reduce them over the group and
    fold the global totals into this rank's host maps (policy entry
    packets/bytes, cilium_metrics)."""
    import torch
    _, n = dp.counters_device()
    t = torch.empty(n, dtype=torch.int64,
                    device=f"cuda:{torch.cuda.current_device()}")
    dp.counters_export(t, stream)
    allreduce_block(t, group)
    dp.counters_import(t, stream)
    dp.counters_sync(stream)
    return t
