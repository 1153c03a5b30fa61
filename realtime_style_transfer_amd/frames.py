"""Frame sharding, rank setup and timing across ranks (one process per GPU).

Stylisation of a frame stream is embarrassingly parallel: CIN normalises per frame
(``styleTransfer.py:65``) and BatchNorm uses moving statistics at inference, so frame i's output does
not depend on any other frame. Rank r of W takes frame batches ``r, r+W, r+2W, ...``; nothing crosses
ranks on the data path. The only collectives are host-side bookkeeping (a barrier around the timed
region, a MAX of the elapsed time and a SUM of the frames processed), which run over whatever process
group is initialised (RCCL on the GPU box, gloo in the CPU tests). ``bench.py`` drives its timed regions
through this module, and ``launch_ranks`` is how ``bench.py --gpus N`` starts its N ranks.

The reference has no multi-GPU code (``train_network.py:14-23`` pins one GPU); this is SURVEY §8e.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

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


def _distributed() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _reduce_device(device=None):
    """Where a bookkeeping tensor for a collective lives: the GPU for RCCL, the host for gloo."""
    if _distributed() and dist.get_backend() == "nccl":
        return device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def max_over_ranks(value: float, device=None) -> float:
    if not _distributed():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_reduce_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, device=None) -> float:
    if not _distributed():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_reduce_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def timed_region(fn: Callable[[], None], steps: int, sync: Callable[[], None], device=None) -> float:
    """barrier + sync, run ``steps`` x fn, sync + barrier; returns the MAX elapsed over ranks."""
    distributed = _distributed()
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


# ---------------------------------------------------------------------------------------- rank setup
@dataclass
class RankContext:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: Optional[str]

    def sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def timed(self, fn: Callable[[], None], steps: int) -> float:
        return timed_region(fn, steps, self.sync, self.device if self.device.type == "cuda" else None)

    def close(self):
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(nproc: int, script: str, argv: Sequence[str], env: Optional[dict] = None) -> int:
    """Start ``nproc`` ranks of ``script`` (one process per GPU) under torch.distributed.run on this node and
    wait for them: a CHILD process — the caller has not touched the GPU and is not replaced (no exec).
    Returns the launcher's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", script, *argv]
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=e).returncode


def init_ranks(backend: Optional[str] = None, device_type: str = "cuda") -> RankContext:
    """Read RANK/LOCAL_RANK/WORLD_SIZE (torch.distributed.run) and join the process group.

    ``backend`` None picks RCCL ("nccl") for GPU ranks and gloo for CPU ranks. With gloo, GPU ranks may
    share a device (rank r on cuda:(local_rank % device_count)) — how the multi-rank path is rehearsed on a
    one-GPU box; RCCL needs one GPU per rank."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type == "cuda":
        n = torch.cuda.device_count()
        if n == 0:
            raise RuntimeError("no GPU visible (use device_type='cpu' for the plumbing check)")
        if backend is None:
            backend = "nccl"
        if backend == "nccl" and local_rank >= n:
            raise RuntimeError(f"local rank {local_rank} but only {n} GPU(s): RCCL needs one GPU per rank")
        device = torch.device("cuda", local_rank % n)
        torch.cuda.set_device(device)
    else:
        backend = backend or "gloo"
        device = torch.device("cpu")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    else:
        backend = None
    return RankContext(rank, world, local_rank, device, backend)
