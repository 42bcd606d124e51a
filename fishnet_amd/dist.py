"""Multi-GPU plumbing (one process per GPU, torch.distributed; backend "nccl"
is RCCL over xGMI on MI355X, "gloo" is used for the CPU tests).

The evaluation path shards without any data-path exchange: every rank
evaluates its own positions.  The only collectives are:
  * one broadcast of the packed net image from rank 0 (47 MB at HD = 1024),
    which each rank then adopts with ``Evaluator(None, image_ptr=...)``;
  * a max-reduction of the timed-region length (bench contract);
  * an optional gather of per-rank results to rank 0 for a caller that wants
    the whole batch in one place.
"""
from __future__ import annotations

import os

import numpy as np


def env_rank() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def shard_seed(seed: int, rank: int) -> int:
    """Per-rank playout seed (weak scaling: every rank gets its own positions)."""
    return seed + 1_000_003 * rank


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [begin, end) share of `total` independent units (strong scaling)."""
    return total * rank // world, total * (rank + 1) // world


def broadcast_image(image: np.ndarray | None, device, src: int = 0):
    """Broadcast rank `src`'s packed net image (uint8) to every rank.

    Returns a uint8 tensor on `device` holding the image on every rank.
    """
    import torch
    import torch.distributed as dist

    rank = dist.get_rank()
    if rank == src:
        assert image is not None
        buf = torch.from_numpy(np.ascontiguousarray(image, dtype=np.uint8)).to(device)
        size = torch.tensor([buf.numel()], dtype=torch.int64, device=device)
    else:
        size = torch.zeros(1, dtype=torch.int64, device=device)
    dist.broadcast(size, src)
    if rank != src:
        buf = torch.empty(int(size.item()), dtype=torch.uint8, device=device)
    dist.broadcast(buf, src)
    return buf


def max_over_ranks(value: float, device) -> float:
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_to_rank0(local, device):
    """Every rank's 1-D int32 results concatenated on rank 0 (None elsewhere).

    One dist.gather to rank 0 (RCCL over xGMI for "nccl"): each rank sends its
    shard once, padded to the largest shard; nothing goes to the other ranks.
    `local` is a numpy array or a tensor already on `device`."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    t = local if isinstance(local, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(local, dtype=np.int32))
    t = t.to(device=device, dtype=torch.int32).reshape(-1)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n)  # world x 8 bytes
    sizes = [int(x.item()) for x in sizes]
    cap = max(sizes)
    if t.numel() < cap:
        t = torch.cat([t, torch.zeros(cap - t.numel(), dtype=torch.int32, device=device)])
    parts = [torch.empty(cap, dtype=torch.int32, device=device) for _ in range(world)] if rank == 0 else None
    dist.gather(t, parts, dst=0)
    if rank != 0:
        return None
    return np.concatenate([p[:k].cpu().numpy() for p, k in zip(parts, sizes)])


def shard_groups(off: np.ndarray, rank: int, world: int) -> tuple[int, int]:
    """This rank's contiguous run of whole groups [g0, g1), balanced by position
    count (fnnue_partition_groups; a game or a parent with its children is
    never split across ranks)."""
    from .nnue import partition_groups

    cut = partition_groups(off, world)
    return int(cut[rank]), int(cut[rank + 1])
