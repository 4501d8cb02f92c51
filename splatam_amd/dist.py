"""Frame sharding across GPUs: one process per GPU, every rank
tracks / renders its own frames against the same Gaussian map.

The only exchange steps are the ones the path really has:
  * broadcast of the canonical Gaussian map from rank 0 after a map update
    (56 B per Gaussian; RCCL over xGMI with backend "nccl");
  * all-reduce (sum) of per-Gaussian accumulators when results are merged
    (e.g. the Fisher / Hessian diagonals of ros_handler.py:807-829);
  * max over ranks of wall times (bench.py).
All functions are no-ops for a single process, and work with the "gloo"
backend on CPU for tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

MAP_KEYS = ("means3D", "rgb_colors", "unnorm_rotations", "logit_opacities", "log_scales")


def world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def frames_for_rank(num_frames: int, rank: int | None = None, world_size: int | None = None) -> list[int]:
    """Rank r handles frames r, r+W, r+2W, ..."""
    r, w = world()
    r = r if rank is None else rank
    w = w if world_size is None else world_size
    return list(range(r, num_frames, w))


def broadcast_map(params: dict, keys=MAP_KEYS, src: int = 0) -> int:
    """In-place broadcast of the Gaussian map tensors; returns the bytes sent per rank."""
    _, w = world()
    nbytes = 0
    for k in keys:
        t = params[k]
        nbytes += t.numel() * t.element_size()
        if w > 1:
            with torch.no_grad():
                dist.broadcast(t.data, src=src)
    return nbytes


def all_reduce_sum_(t: torch.Tensor) -> torch.Tensor:
    if world()[1] > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def max_over_ranks(x: float, device=None) -> float:
    if world()[1] == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
