"""Frame sharding across GPUs: one process per GPU, every rank
tracks / renders its own frames against the same Gaussian map.

The only exchange steps are the ones the path really has:
  * broadcast of the canonical Gaussian map from rank 0 after a map update
    (56 B per Gaussian; RCCL over xGMI with backend "nccl"): FlatMap lays the map's
    tensors out as views of one contiguous buffer, so the whole map is ONE collective
    (no per-tensor launch and protocol overhead), and MapBroadcaster double-buffers it:
    the broadcast of the next map version runs on a side stream into a back buffer while
    the ranks keep tracking against the current one, and is copied into the live map
    (one device copy) at the next frame boundary;
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


class FlatMap:
    """The map tensors params[k] (k in `keys`) re-seated as views of one contiguous float32 buffer `flat`
    (their .data is replaced in place: the tensor objects, their requires_grad and any reference held to
    them stay valid; HIP graphs must be captured after this, as they bake the addresses in)."""

    def __init__(self, params: dict, keys=MAP_KEYS):
        self.keys = tuple(keys)
        ref = params[self.keys[0]]
        for k in self.keys:
            if params[k].dtype != torch.float32 or params[k].device != ref.device:
                raise RuntimeError("FlatMap: every map tensor must be float32 on one device")
        total = sum(params[k].numel() for k in self.keys)
        self.flat = torch.empty(total, dtype=torch.float32, device=ref.device)
        self.spans = {}
        off = 0
        with torch.no_grad():
            for k in self.keys:
                t = params[k]
                n = t.numel()
                view = self.flat[off:off + n].view(t.shape)
                view.copy_(t)
                t.data = view
                self.spans[k] = (off, n)
                off += n
        self.params = params

    @property
    def nbytes(self) -> int:
        return self.flat.numel() * self.flat.element_size()

    def check(self) -> bool:
        """True while every map tensor is still the view FlatMap seated (no one replaced its storage)."""
        base = self.flat.data_ptr()
        return all(self.params[k].data_ptr() == base + 4 * self.spans[k][0] and self.params[k].is_contiguous()
                   for k in self.keys)


def broadcast_flat(fm: FlatMap, src: int = 0) -> int:
    """Blocking broadcast of the whole map from `src` in one collective; returns the bytes sent per rank."""
    if world()[1] > 1:
        if not fm.check():
            raise RuntimeError("FlatMap: a map tensor no longer views the flat buffer")
        dist.broadcast(fm.flat, src=src)
    return fm.nbytes


class MapBroadcaster:
    """Double-buffered map broadcast overlapped with the next frame's work.

    start(): the source rank snapshots the live map into the back buffer (one device copy on the caller's
    stream), then every rank issues ONE broadcast of the back buffer, on a side stream (nccl) that waits only
    for that snapshot -- the caller's stream goes on with the frame's HIP-graph replays against the live map.
    finish(): the caller's stream waits for the collective and the receiving ranks copy the back buffer into
    the live map (one device copy), so the map version broadcast at one frame boundary is the one the frame
    after the next boundary tracks against -- one frame of staleness, the price of the overlap.  Without a
    process group both are no-ops."""

    def __init__(self, fm: FlatMap, src: int = 0):
        self.fm, self.src = fm, src
        self.back = torch.empty_like(fm.flat)
        self.work = None
        dev = fm.flat.device
        self.stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None

    def start(self):
        rank, w = world()
        if w == 1:
            return
        if self.work is not None:
            raise RuntimeError("MapBroadcaster.start: the previous broadcast was not finished")
        if not self.fm.check():
            raise RuntimeError("FlatMap: a map tensor no longer views the flat buffer")
        if rank == self.src:
            with torch.no_grad():
                self.back.copy_(self.fm.flat)
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream(self.fm.flat.device))
            with torch.cuda.stream(self.stream):
                self.work = dist.broadcast(self.back, src=self.src, async_op=True)
        else:
            self.work = dist.broadcast(self.back, src=self.src, async_op=True)

    def finish(self):
        if self.work is None:
            return
        self.work.wait()  # nccl: the caller's current stream waits for the collective; gloo: the host waits
        if world()[0] != self.src:
            with torch.no_grad():
                self.fm.flat.copy_(self.back)
        self.work = None


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
