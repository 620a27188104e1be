"""Image-parallel sharding across GPUs (one process per GPU).

Frames are independent: rank r of N decodes its own frames
with its own context, streams and host Huffman workers.  Nothing crosses the
GPUs on the data path -- no RCCL collective; torch.distributed is used only
for the launch barrier and the host-side aggregation of counters/timers
(gloo or nccl, whichever the process group runs).
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Balanced contiguous [begin, end) of n_items for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, r = divmod(n_items, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def shard_round_robin(n_items: int, rank: int, world: int) -> List[int]:
    """Frames i with i % world == rank (stream order interleaved over GPUs)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return list(range(rank, n_items, world))


def aggregate(stats: Dict[str, float], reduce_max=("seconds",)) -> Dict[str, float]:
    """Host-side aggregation over the process group: sums counters, takes the
    max of the keys in `reduce_max` (wall time of the slowest rank)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dict(stats)
    return allreduce_stats(stats, reduce_max)


def allreduce_stats(stats: Dict[str, float], reduce_max=("seconds",)) -> Dict[str, float]:
    """aggregate's collective part: one SUM and one MAX all-reduce of float64
    vectors (on the device for RCCL, on the host for gloo).  Split out so a
    one-rank RCCL group on a single GPU can run the exact calls an N-GPU run
    makes (tests/test_gpu_rccl.py)."""
    import torch
    import torch.distributed as dist
    keys = sorted(stats)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    sums = torch.tensor([0.0 if k in reduce_max else float(stats[k]) for k in keys], dtype=torch.float64,
                        device=dev)
    maxs = torch.tensor([float(stats[k]) if k in reduce_max else 0.0 for k in keys], dtype=torch.float64,
                        device=dev)
    dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    dist.all_reduce(maxs, op=dist.ReduceOp.MAX)
    return {k: (maxs[i].item() if k in reduce_max else sums[i].item()) for i, k in enumerate(keys)}
