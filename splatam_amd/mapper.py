"""SplaTAM's per-frame mapping loop replayed as one HIP graph.

scripts/splatam.py:842-905 maps every frame with `num_iters` iterations
(configs/replica/splatam.py:16: 60) of get_loss(mapping=True) + backward + Adam
over the Gaussian parameters, with a freshly initialised optimizer per frame
(initialize_optimizer, splatam.py:166-172) and, per iteration, a keyframe drawn
uniformly from the mapping window (np.random.randint, splatam.py:851).

GraphMapper captures one frame's mapping -- the optimizer-state reset plus all
`iters_per_graph` iterations -- into a torch.cuda.CUDAGraph: the Adam step runs
inside the transform backward (gsr_map_transform_bwd_adam, step numbers 1..N
baked into the captured launches), the rasterization uses the static-capacity
dual forward, and the keyframe sequence is drawn once at construction from
numpy's global random stream (np.random.randint, the reference's own draw) or,
with `seed`, from a seeded np.random.RandomState; a replay repeats it, so build
one mapper per frame for fresh draws.
Each replay is one frame's mapping.  An iteration whose forward overflows the
binning capacity skips its Adam step on the device (its status row, sticky
across replays, reports it).  Densification / pruning (which change P)
are outside the graph, as they are outside the reference's inner loop body.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _C
from .glue import MapAdam, map_transform
from .layout import views
from .slam import MappingConfig, _get_loss_mapping_fused, color_key, fused_mapping_eligible

TILE_SORT_CAP = 4096  # longest tile list the static mode handles (render_fwd's per-tile sort)
GAUSS_KEYS = ("means3D", "unnorm_rotations", "logit_opacities", "log_scales")


def probe_num_rendered(params, curr_data, time_idx) -> tuple[int, int]:
    """(num_rendered, longest tile list) of a keyframe at its current pose (eager, synchronous)."""
    cam = curr_data["cam"]
    key = color_key(params)
    with torch.no_grad():
        means, rots, dcol, opac, scales, col = map_transform(params, time_idx, curr_data["w2c"], key)
        sh, colors = (col, torch.Tensor([])) if key == "shs" else (torch.Tensor([]), col)
        out = _C.rasterize_gaussians_dual(cam.bg, means, colors, dcol, opac, scales, rots, cam.scale_modifier,
                                          torch.Tensor([]), cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy,
                                          cam.image_height, cam.image_width, sh, cam.sh_degree, cam.campos,
                                          cam.prefiltered)
        n, img, binning = out[0], out[6], out[5]
        r = views(img, binning, cam.image_width, cam.image_height, n)["ranges"]
        longest = int((r[:, 1] - r[:, 0]).max().item()) if r.numel() else 0
    return int(n), longest


class GraphMapper:
    def __init__(self, params: dict, keyframes: list, iters_per_graph: int = 60, cfg: MappingConfig = MappingConfig(),
                 headroom: float = 1.5, min_extra: int = 65536, seed: int | None = None, timing: bool = False):
        if not keyframes:
            raise RuntimeError("GraphMapper needs at least one keyframe")
        for kf in keyframes:
            if not fused_mapping_eligible(params, kf, cfg):
                raise RuntimeError("GraphMapper needs the fused mapping configuration (camera fixed, L1 + SSIM)")
        key = color_key(params)
        for k in GAUSS_KEYS + (key,):
            p = params[k]
            if not (p.is_leaf and p.requires_grad):
                raise RuntimeError(f"params[{k!r}] must be a leaf tensor requiring grad")
        self.params, self.keyframes, self.cfg = params, keyframes, cfg
        dev = params["means3D"].device
        probes = [probe_num_rendered(params, kf, kf["id"]) for kf in keyframes]
        longest = max(p[1] for p in probes)
        if longest > TILE_SORT_CAP:
            raise RuntimeError(f"a tile list of {longest} > {TILE_SORT_CAP}: use the eager (synchronous) path")
        self.capacity = max(1, int(headroom * max(p[0] for p in probes)) + int(min_extra))
        self.iters = int(iters_per_graph)
        rng = np.random if seed is None else np.random.RandomState(seed)
        self.sequence = [int(rng.randint(0, len(keyframes))) for _ in range(self.iters)]  # splatam.py:851
        self.status = torch.zeros(self.iters, 4, dtype=torch.int32, device=dev)
        self.adam = MapAdam(params, cfg.lrs, color_key=key)
        self.adam.capacity = self.capacity
        self.seed = torch.ones((), dtype=torch.float32, device=dev)           # static loss-gradient seed
        self.means2D = torch.zeros(params["means3D"].shape[0], 3, device=dev)  # no grad (no densification stats)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        snapshot = {k: params[k].detach().clone() for k in GAUSS_KEYS + (key,)}
        with torch.cuda.stream(side):  # warm-up iterations outside the capture, then the state is restored
            for k in range(min(2, self.iters)):
                self._iteration(k)
            with torch.no_grad():
                for k, v in snapshot.items():
                    params[k].copy_(v)
            self.status.zero_()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        del snapshot
        if timing:
            from . import profiling
            profiling.enable_timing(clock_stages=("render_bwd", "render_fwd"))
        self.graph = torch.cuda.CUDAGraph()
        self.stream = side
        with torch.cuda.graph(self.graph, stream=side):
            self.adam.reset()          # initialize_optimizer per frame: zero moments, step 0
            for k in range(self.iters):
                self.loss = self._iteration(k)

    def _iteration(self, k: int):
        kf = self.keyframes[self.sequence[k]]
        self.adam.status = self.status[k]  # this iteration's forward guards its Adam step
        loss, _, _ = _get_loss_mapping_fused(self.params, kf, kf["id"], self.cfg, adam=self.adam,
                                             capacity=self.capacity, status=self.status[k], means2D=self.means2D)
        torch.autograd.backward(loss, self.seed)
        return loss.detach()

    def run(self, check: bool = False):
        """Enqueue one frame's mapping (one graph launch, no host sync).  An iteration whose forward
        overflowed skips its own Adam step (the steps guard on that forward's counters), but the bias
        corrections of the later steps still count it; with `check` the replay ends with one host sync
        and raises on any overflow, so the caller can rebuild with more headroom and re-map the frame."""
        if check:
            self.reset_status()
        self.graph.replay()
        if check and self.overflowed():
            raise RuntimeError(f"binning capacity {self.capacity} exceeded during mapping: rebuild the mapper "
                               "with more headroom and re-run the frame")

    def reset_status(self):
        self.status.zero_()

    def overflowed(self) -> bool:
        """True if any iteration since the last reset_status() exceeded the binning capacity (one host sync)."""
        st = self.status.cpu()
        return bool((st[:, 0] > self.capacity).any() or (st[:, 2] > TILE_SORT_CAP).any() or (st[:, 1] != 0).any())

    def num_rendered(self) -> list[int]:
        return [int(x) for x in self.status[:, 0].cpu()]
