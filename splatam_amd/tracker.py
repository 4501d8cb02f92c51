"""SplaTAM tracking iterations replayed as one HIP graph.

scripts/splatam.py tracks every frame with a fixed number of iterations
(configs/replica/splatam.py:59: 40) of get_loss(tracking=True) + backward +
Adam on the camera pose.  Each iteration is ~15 kernel launches whose host
cost (Python, autograd, ctypes) exceeds their GPU time once the rasterizer is
fast, so the iterations are captured once into a torch.cuda.CUDAGraph
(hipGraph) and replayed: the host issues one launch per `iters_per_graph`
iterations.

The pose optimizer (torch.optim.Adam semantics) runs inside the transform
backward (gsr_track_transform_bwd_adam), so an iteration is the loss forward
and backward only.  Capture requires a forward that never waits on the host: the dual forward runs
in its static mode (gsr_forward_dual_static) with a binning capacity taken
from an eager probe of the same frame times `headroom`.  Every captured
iteration merges its binning counters into its own row of `status` (sticky
across replays, include/gsr.h); `overflowed()` reads them (one host sync) and
reports whether any iteration since the last `reset_status()` exceeded the
capacity.  An overflowing iteration leaves the pose and the optimizer state
untouched (its Adam step is skipped on the device), so the frame can be re-run
from `begin_frame()` after rebuilding the tracker with more headroom.

A frame (scripts/splatam.py:700-763) is `begin_frame()` (fresh optimizer,
best candidate = the current pose with loss 1e20), `num_iters / iters_per_graph`
replays, and `end_frame()`, which writes the best candidate pose back -- the
pose after the step of the lowest-loss iteration (:726-731, :760-763), tracked
on the device inside the captured backward.  `track_frame(num_iters)` does all
three.  The warm-up iterations run at construction are undone (pose restored,
optimizer reset).
"""
from __future__ import annotations

import torch

from . import _C
from .layout import views
from .rasterizer import GaussianRasterizationSettings
from .slam import TrackingConfig, _get_loss_tracking_fused, fused_eligible

TILE_SORT_CAP = 4096  # longest tile list the static mode handles (render_fwd's per-tile sort)


def probe_num_rendered(params, curr_data, time_idx) -> tuple[int, int]:
    """(num_rendered, longest tile list) of the frame at the current pose (eager, synchronous)."""
    from .glue import track_transform
    cam: GaussianRasterizationSettings = curr_data["cam"]
    with torch.no_grad():
        means, rots, dcol, opac, scales = track_transform(params, time_idx, curr_data["w2c"])
        out = _C.rasterize_gaussians_dual(cam.bg, means, params["rgb_colors"], dcol, opac, scales, rots,
                                          cam.scale_modifier, torch.Tensor([]), cam.viewmatrix, cam.projmatrix,
                                          cam.tanfovx, cam.tanfovy, cam.image_height, cam.image_width,
                                          torch.Tensor([]), cam.sh_degree, cam.campos, cam.prefiltered)
        n, img, binning = out[0], out[6], out[5]
        r = views(img, binning, cam.image_width, cam.image_height, n)["ranges"]
        longest = int((r[:, 1] - r[:, 0]).max().item()) if r.numel() else 0
    return int(n), longest


class GraphTracker:
    def __init__(self, params: dict, curr_data: dict, time_idx: int, iters_per_graph: int = 20,
                 cfg: TrackingConfig = TrackingConfig(), lrs=(0.0004, 0.002), headroom: float = 1.5,
                 warmup_iters: int = 3, min_extra: int = 65536, timing: bool = False, fuse_pose: bool = False,
                 prime: bool = False, prime_ms: float = 0.0, clock_stages=None, alive=None,
                 capacity: int | None = None):
        if not fused_eligible(params, curr_data, cfg):
            raise RuntimeError("GraphTracker needs the fused tracking configuration (only the pose requires grad)")
        self.params, self.curr, self.t, self.cfg = params, curr_data, time_idx, cfg
        self.fuse_pose = fuse_pose  # pose chain + Adam inside the rasterizer's per-Gaussian backward
        # alive: uint8 [P] mask of a capacity-padded map (splatam_amd.sequence), read by every replay
        if alive is not None and not fuse_pose:
            raise RuntimeError("GraphTracker: an alive mask needs fuse_pose=True")
        self.alive = alive
        dev = params["means3D"].device
        if capacity is None:  # (capacity: the binning capacity given, e.g. for a map that grows between frames)
            n, longest = probe_num_rendered(params, curr_data, time_idx)
            if longest > TILE_SORT_CAP:
                raise RuntimeError(f"a tile list of {longest} > {TILE_SORT_CAP}: use the eager (synchronous) path")
            capacity = max(1, int(headroom * n) + int(min_extra))
        self.capacity = int(capacity)
        self.iters = int(iters_per_graph)
        self.status = torch.zeros(self.iters, 4, dtype=torch.int32, device=dev)
        rots, trans = params["cam_unnorm_rots"], params["cam_trans"]
        if not (rots.is_leaf and trans.is_leaf and rots.requires_grad and trans.requires_grad):
            raise RuntimeError("cam_unnorm_rots / cam_trans must be leaf tensors requiring grad")
        # Adam on the pose fused into the transform backward (gsr_track_transform_bwd_adam): the
        # iteration is loss forward + backward only -- no .grad, zero_grad or optimizer kernels
        from .glue import PoseAdam
        self.adam = PoseAdam(dev, lr_q=lrs[0], lr_t=lrs[1], track_best=True)
        self.adam.capacity = self.capacity
        self.seed = torch.ones((), dtype=torch.float32, device=dev)          # static loss-gradient seed
        self.means2D = torch.zeros(params["means3D"].shape[0], 3, device=dev)  # no grad: tracking ignores it
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        q0, t0 = rots[..., time_idx].detach().clone(), trans[..., time_idx].detach().clone()
        with torch.cuda.stream(side):  # warm-up iterations (real tracking iterations) outside the capture
            for _ in range(max(1, warmup_iters)):
                self._iteration(0)
            with torch.no_grad():  # ... undone: the frame starts from its pose with a fresh optimizer
                rots[..., time_idx] = q0
                trans[..., time_idx] = t0
            self.adam.reset()
            self.status.zero_()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        from . import profiling
        self.clock_stages = tuple(clock_stages) if clock_stages is not None else profiling.CLOCK_STAGES
        if timing:  # in-kernel device-clock stamps of the captured stages (accumulate over replays)
            torch.cuda.synchronize(dev)
            profiling.enable_timing(clock_stages=self.clock_stages)
        self.graph = torch.cuda.CUDAGraph()
        self.stream = side
        with torch.cuda.graph(self.graph, stream=side):  # capture on the warm-up stream (autograd nodes live there)
            for k in range(self.iters):
                self.loss = self._iteration(k)
        self.prime_replays, self.prime_ms = 0, 0.0
        if prime:  # one replay (graph upload, first-launch costs), undone like the warm-up iterations
            # prime_ms: further replays until that much wall time has passed since the first one -- the
            # GPU's clock ramps up over the first ~25 ms of sustained work (GRBM_COUNT per microsecond of the
            # fused render rises ~9 % over its first ~50 launches, profiles/r7c_clk.txt), so a short timed
            # region right behind a short warm-up would time the ramp, not the kernel
            import time
            t0p = time.perf_counter()
            while True:
                self.graph.replay()
                self.prime_replays += 1
                torch.cuda.synchronize(dev)
                self.prime_ms = 1000.0 * (time.perf_counter() - t0p)
                if self.prime_ms >= prime_ms:
                    break
            with torch.no_grad():
                rots[..., time_idx] = q0
                trans[..., time_idx] = t0
            self.adam.reset()
            self.status.zero_()
            torch.cuda.synchronize(dev)
            if timing:
                profiling.enable_timing(clock_stages=self.clock_stages)

    def _iteration(self, k: int):
        self.adam.status = self.status[k]  # this iteration's forward guards its Adam step
        if self.fuse_pose:
            from .glue import tracking_iteration
            # (images=False: the replays keep the rendered images in registers -- the loss and the render
            # backward run in the same launch and the tracker reads neither image)
            loss, _ = tracking_iteration(self.params, self.curr, self.t, self.cfg, pose_adam=self.adam,
                                         capacity=self.capacity, status=self.status[k], seed=self.seed,
                                         images=False, alive=self.alive)
            torch.autograd.backward(loss, self.seed)
            return loss.detach()
        loss, _, _ = _get_loss_tracking_fused(self.params, self.curr, self.t, self.cfg, dual=True,
                                              capacity=self.capacity, status=self.status[k], pose_adam=self.adam,
                                              means2D=self.means2D, seed=self.seed)
        self.adam.loss = loss  # best-candidate selection in the transform backward
        torch.autograd.backward(loss, self.seed)
        self.adam.loss = None
        return loss.detach()

    def begin_frame(self):
        """initialize_optimizer + candidate = the current pose, current_min_loss = 1e20 (splatam.py:700-705)."""
        with torch.no_grad():
            self.adam.state.zero_()
            self.adam.best[0] = 1e20
            self.adam.best[1:5] = self.params["cam_unnorm_rots"][0, :, self.t]
            self.adam.best[5:8] = self.params["cam_trans"][0, :, self.t]

    def end_frame(self):
        """Copy the best candidate pose back into the frame's column (splatam.py:760-763)."""
        with torch.no_grad():
            self.params["cam_unnorm_rots"][0, :, self.t] = self.adam.best[1:5]
            self.params["cam_trans"][0, :, self.t] = self.adam.best[5:8]

    def track_frame(self, num_iters: int, check: bool = True):
        """One frame's tracking: begin_frame, num_iters iterations (a multiple of iters_per_graph), end_frame.

        An iteration whose forward overflowed skips its own pose step (the fused steps guard on that
        forward's counters, not on the sticky status rows; the pose optimizer's step count lives on the
        device, so later iterations are consistent).  `check` (the default) ends the frame with one host
        sync and raises if any iteration of it overflowed -- the frozen pose is never returned silently;
        check=False (timing loops) skips the sync: read overflowed() afterwards."""
        if num_iters % self.iters:
            raise ValueError(f"num_iters {num_iters} is not a multiple of iters_per_graph {self.iters}")
        if check:
            self.reset_status()
        self.begin_frame()
        for _ in range(num_iters // self.iters):
            self.run()
        self.end_frame()
        if check and self.overflowed():
            raise RuntimeError(f"binning capacity {self.capacity} exceeded while tracking frame {self.t}: "
                               "rebuild the tracker with more headroom and re-run the frame")

    def reset_status(self):
        self.status.zero_()

    def run(self):
        """Enqueue `iters_per_graph` tracking iterations (one graph launch, no host sync)."""
        self.graph.replay()

    def overflowed(self) -> bool:
        """True if any iteration since the last reset_status() exceeded the binning capacity (one host sync)."""
        st = self.status.cpu()
        return bool((st[:, 0] > self.capacity).any() or (st[:, 2] > TILE_SORT_CAP).any() or (st[:, 1] != 0).any())

    def num_rendered(self) -> list[int]:
        """Per captured iteration: the largest num_rendered since the last reset_status()."""
        return [int(x) for x in self.status[:, 0].cpu()]
