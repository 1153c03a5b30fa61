"""Frame sharding and timing across ranks (one process per GPU).

Stylisation of a frame stream is embarrassingly parallel: CIN normalises per frame
(``styleTransfer.py:65``) and BatchNorm uses moving statistics at inference, so frame i's output does
not depend on any other frame. Rank r of W takes frame batches ``r, r+W, r+2W, ...``; nothing crosses
ranks on the data path. The only collectives are host-side bookkeeping (a barrier around the timed
region and a MAX of the elapsed time), which run over whatever process group is initialised
(RCCL on the GPU box, gloo in the CPU tests).
"""
from __future__ import annotations

import time
from typing import Callable, List, Sequence

import torch
import torch.distributed as dist


def rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_batches(n_frames: int, batch: int, rank: int, world: int) -> List[range]:
    """Frame index ranges (batches of <= ``batch``) owned by ``rank``: batch k goes to rank k % world."""
    batches = [range(s, min(s + batch, n_frames)) for s in range(0, n_frames, batch)]
    return batches[rank::world]


def max_over_ranks(value: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_region(fn: Callable[[], None], steps: int, sync: Callable[[], None], device=None) -> float:
    """barrier + sync, run ``steps`` x fn, sync + barrier; returns the MAX elapsed over ranks."""
    distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if distributed:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    if distributed:
        dist.barrier()
    return max_over_ranks(time.perf_counter() - t0, device)


def gather_frames(local: Sequence[torch.Tensor], local_ids: Sequence[int], n_frames: int):
    """Reassemble a sharded stream on every rank (only for small outputs / tests)."""
    rank, world = rank_world()
    payload = list(zip(local_ids, [t.cpu() for t in local]))
    if world == 1:
        gathered = [payload]
    else:
        gathered = [None] * world
        dist.all_gather_object(gathered, payload)
    out = [None] * n_frames
    for part in gathered:
        for i, t in part:
            out[i] = t
    return out
