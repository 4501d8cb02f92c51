"""Fisher-information view scoring on the backward_power=2 path.

The fork's active-mapping node scores candidate camera poses by the expected
information gain of a view (scripts/ros_handler.py:807-902):

  * compute_Hessian(w2c) (:847-902): the Gaussians moved into the candidate
    camera frame (means only; rotations / opacities / scales / colours as
    rendervars), one RGB render with GaussianRasterizer(backward_power=2), and a
    backward seeded with 1e-3 everywhere; H = [dL/dmeans_cam (P,3), dL/dopacity
    (P,1)] -- per-pair gradients squared before summation, i.e. the diagonal of
    the Gauss-Newton / Fisher matrix;
  * compute_H_visited_inv (:807-829): H_train = sum of H over the visited poses,
    H_train_inv = 1 / (H_train + 0.1);
  * compute_eig_score (:832-836): sum(H(candidate) * H_train_inv).

FisherScorer restates these over a *batch* of poses and shards the batch over
ranks (one process per GPU): H_train is the all-reduce (sum) of the per-rank
partial sums (RCCL over xGMI, 16 B per Gaussian), candidate scores are formed on
the device and exchanged once with an all-gather.  Each pose's render +
power-2 backward runs through the HIP rasterizer (gsr_forward / gsr_backward
with power = 2) and only the two gradients H needs are requested, which selects
the Fisher kernels (gauss_mpack, render_bwd_fisher, gauss_bwd_fisher: 4 powered
values per pixel-Gaussian pair instead of the full path's 22).

BatchedFisher renders a batch of K poses per host launch: the K transforms, static-
capacity forwards (gsr_forward_static), power-2 backwards and the per-pose reductions
(H accumulation for the visited poses, or the EIG score of each candidate) are captured
once into a HIP graph and replayed with the poses written into a device [K,4,4] tensor.
Every pose's Hessian is bitwise the per-pose FisherScorer.hessian's.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import dist as sd
from .rasterizer import GaussianRasterizer

SEED = 1e-3      # im.backward(gradient=torch.ones_like(im) * 1e-3)  (ros_handler.py:888)
# the gradients H reads (ros_handler.py:884-889): dmeans3D and dopacity -- the Fisher-selective
# backward_power kernel (gsr_backward_power.hip render_bwd_fisher_kernel), 4 values per pair
FISHER_NEEDS = (False, False, True, True, False, False, False, False)
H_EPS = 0.1      # torch.reciprocal(H_train + 0.1)                   (ros_handler.py:829)


def camera_points(means: torch.Tensor, w2c: torch.Tensor) -> torch.Tensor:
    """(rel_w2c @ pts4.T).T[:, :3] (ros_handler.py:863-866) in one launch (gsr_points_to_camera: each
    coordinate summed left to right; a [P,3] x [3,3] addmm took a 22 us hipBLASLt kernel); shared by the
    per-pose and the batched paths, so both see bitwise the same camera-frame points."""
    from ._lib import lib
    if means.device.type != "cuda":
        raise RuntimeError("Fisher scoring runs on ROCm devices only (no CPU fallback)")
    means = means.detach().float().contiguous()
    w2c = w2c.detach().to(means.device).float().contiguous()
    pts = torch.empty_like(means)
    rc = lib.gsr_points_to_camera(means.shape[0], means.data_ptr(), w2c.data_ptr(), pts.data_ptr(),
                                  torch.cuda.current_stream(means.device).cuda_stream)
    if rc != 0:
        raise RuntimeError(f"gsr_points_to_camera: {lib.gsr_last_error().decode(errors='replace')}")
    return pts


class FisherScorer:
    def __init__(self, params: dict, cam, hessian_fn=None):
        """params: SplaTAM parameter dict (means3D, rgb_colors, unnorm_rotations, logit_opacities,
        log_scales); cam: GaussianRasterizationSettings of the scoring camera.  hessian_fn(w2c) -> H
        overrides the per-pose Hessian (tests of the sharding on CPU)."""
        self.params, self.cam = params, cam
        self._hessian_fn = hessian_fn
        self.H_train_inv = None
        if hessian_fn is None:
            with torch.no_grad():  # ros_handler.py:868-874
                self.rotations = F.normalize(params["unnorm_rotations"])
                self.opacities = torch.sigmoid(params["logit_opacities"])
                scales = torch.exp(params["log_scales"])
                self.scales = torch.tile(scales, (1, 3)) if scales.shape[-1] == 1 else scales
                self.colors = params["rgb_colors"]

    def hessian(self, w2c: torch.Tensor) -> torch.Tensor:
        """compute_Hessian(rel_w2c, return_points=True): H [P,4] for one camera (w2c [4,4])."""
        if self._hessian_fn is not None:
            return self._hessian_fn(w2c)
        means = self.params["means3D"].detach()
        w2c = w2c.to(means.device).float()
        with torch.no_grad():
            pts = camera_points(means, w2c)
        pts.requires_grad_(True)
        opac = self.opacities.detach().clone().requires_grad_(True)
        means2D = torch.zeros_like(pts)
        im, _, _ = GaussianRasterizer(self.cam, backward_power=2)(
            means3D=pts, means2D=means2D, opacities=opac, colors_precomp=self.colors.detach(),
            scales=self.scales.detach(), rotations=self.rotations.detach())
        im.backward(gradient=torch.full_like(im, SEED))
        return torch.cat([pts.grad.reshape(pts.shape[0], -1), opac.grad.reshape(pts.shape[0], -1)], dim=1)

    def fit_visited(self, w2cs, batch: "BatchedFisher | None" = None) -> torch.Tensor:
        """compute_H_visited_inv over all visited poses: each rank sums the Hessians of its shard
        (poses r, r+W, ...), one all-reduce merges them.  Returns (and keeps) H_train_inv.
        batch: a BatchedFisher(mode="sum") -- the shard is rendered K poses per graph launch."""
        r, w = sd.world()
        H = None
        mine = [w2cs[j] for j in range(r, len(w2cs), w)]
        if batch is not None:
            for c in range(0, len(mine), batch.K):
                chunk = mine[c:c + batch.K]
                h = batch.hessian_sum(chunk)
                if h is None:  # a pose exceeded the graph's binning capacity: the eager path re-sizes
                    h = sum(self.hessian(w2c) for w2c in chunk)
                H = h.clone() if H is None else H + h
        for w2c in ([] if batch is not None else mine):
            h = self.hessian(w2c)
            H = h if H is None else H + h
        if H is None:  # this rank has no pose: contribute zeros of the right shape
            P = self.params["means3D"].shape[0]
            H = torch.zeros(P, 4, device=self.params["means3D"].device)
        sd.all_reduce_sum_(H)
        self.H_train_inv = torch.reciprocal(H + H_EPS)
        return self.H_train_inv

    def eig_scores(self, w2cs, batch: "BatchedFisher | None" = None) -> torch.Tensor:
        """compute_eig_score for every candidate pose: sum(H(pose) * H_train_inv).  The batch is
        sharded over ranks; returns all scores (float64, in pose order) on every rank.
        batch: a BatchedFisher(mode="scores") -- K candidate poses per graph launch."""
        if self.H_train_inv is None:
            raise RuntimeError("fit_visited() first (H_train_inv)")
        r, w = sd.world()
        n = len(w2cs)
        per = -(-n // w) if n else 0
        dev = self.H_train_inv.device
        local = torch.zeros(max(per, 1), dtype=torch.float64, device=dev)
        mine = list(range(r, n, w))
        if batch is not None:
            for c in range(0, len(mine), batch.K):
                idx = mine[c:c + batch.K]
                sc = batch.scores([w2cs[j] for j in idx], self.H_train_inv)
                if sc is None:  # capacity overflow in the graph: score this chunk on the eager path
                    sc = torch.stack([(self.hessian(w2cs[j]) * self.H_train_inv).sum().double() for j in idx])
                local[c:c + len(idx)] = sc
        for k, j in enumerate([] if batch is not None else mine):
            local[k] = (self.hessian(w2cs[j]) * self.H_train_inv).sum().double()
        if w == 1:
            return local[:n]
        gathered = [torch.zeros_like(local) for _ in range(w)]
        dist.all_gather(gathered, local)
        out = torch.zeros(n, dtype=torch.float64, device=dev)
        for rr in range(w):
            idx = list(range(rr, n, w))
            out[idx] = gathered[rr][:len(idx)]
        return out


class BatchedFisher:
    """K poses of FisherScorer's Hessian per HIP-graph launch.

    mode "sum": `hessian_sum(w2cs)` returns sum_k H(w2c_k) (compute_H_visited_inv's H_train before the
    all-reduce); mode "scores": `scores(w2cs, H_inv)` returns [sum(H(w2c_k) * H_inv) for k] (float64 like
    FisherScorer.eig_scores).  Fewer than K poses pad the batch with weight-0 slots.  The binning capacity
    comes from eager probes of `probe_w2cs` times `headroom`; `overflowed()` reports (sticky) whether a
    replay exceeded it (results then invalid: rebuild with more headroom)."""

    def __init__(self, scorer: FisherScorer, K: int, mode: str = "sum", probe_w2cs=None, headroom: float = 1.5,
                 min_extra: int = 65536):
        from . import _C
        if scorer._hessian_fn is not None:
            raise RuntimeError("BatchedFisher renders through the rasterizer (no hessian_fn override)")
        if mode not in ("sum", "scores"):
            raise ValueError("mode is 'sum' or 'scores'")
        self.sc, self.K, self.mode = scorer, int(K), mode
        cam = scorer.cam
        means = scorer.params["means3D"].detach().contiguous()
        dev = means.device
        self.means = means
        P = means.shape[0]
        self.w2c = torch.eye(4, device=dev).repeat(self.K, 1, 1).contiguous()
        self.weight = torch.zeros(self.K, device=dev)
        self.H_inv = torch.zeros(P, 4, device=dev)
        self.status = torch.zeros(self.K, 4, dtype=torch.int32, device=dev)
        self.seed = torch.full((3, cam.image_height, cam.image_width), SEED, device=dev)  # ros_handler.py:888
        self.e = torch.Tensor([])
        probes = list(probe_w2cs) if probe_w2cs is not None else [torch.eye(4, device=dev)]
        n = 0
        with torch.no_grad():
            for w in probes:
                pts = camera_points(means, w.to(dev).float())
                n = max(n, self._forward(_C, pts, 0)[0])
        self.capacity = max(1, int(headroom * n) + int(min_extra))
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self._body(_C)  # warm-up (allocator pools, kernels) outside the capture
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.status.zero_()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=side):
            self._body(_C)

    def _forward(self, _C, pts, capacity):
        sc, cam = self.sc, self.sc.cam
        return _C.rasterize_gaussians(cam.bg, pts, sc.colors.detach(), sc.opacities.detach(), sc.scales.detach(),
                                      sc.rotations.detach(), cam.scale_modifier, self.e, cam.viewmatrix,
                                      cam.projmatrix, cam.tanfovx, cam.tanfovy, cam.image_height, cam.image_width,
                                      self.e, cam.sh_degree, cam.campos, cam.prefiltered, capacity=capacity,
                                      status=self.status[self._k] if capacity else None)

    def _grads(self, _C, k):
        """(dL/dmeans_cam [P,3], dL/dopacity [P,1]) of pose slot k (power-2 backward, Fisher kernels)."""
        sc, cam = self.sc, self.sc.cam
        self._k = k
        pts = camera_points(self.means, self.w2c[k])
        n, color, radii, geom, binning, img, depth = self._forward(_C, pts, self.capacity)
        g = _C.rasterize_gaussians_backward(cam.bg, pts, radii, sc.colors.detach(), sc.scales.detach(),
                                            sc.rotations.detach(), cam.scale_modifier, self.e, cam.viewmatrix,
                                            cam.projmatrix, cam.tanfovx, cam.tanfovy, self.seed, self.e,
                                            cam.sh_degree, cam.campos, geom, n, binning, img, 2,
                                            needs=FISHER_NEEDS)
        return g[3], g[2]

    def _body(self, _C):
        from ._lib import lib
        self._k = 0
        with torch.no_grad():
            if self.mode == "sum":
                self.out = torch.zeros_like(self.H_inv)
                P = self.out.shape[0]
                stream = torch.cuda.current_stream(self.out.device).cuda_stream
                for k in range(self.K):
                    dm, dop = self._grads(_C, k)
                    # out += [dm, dop] * weight[k] in one launch (bitwise torch's add_(cat(...) * w))
                    rc = lib.gsr_fisher_accumulate(P, dm.data_ptr(), dop.data_ptr(),
                                                   self.weight.data_ptr() + 4 * k, self.out.data_ptr(), stream)
                    if rc != 0:
                        raise RuntimeError(f"gsr_fisher_accumulate: {lib.gsr_last_error().decode(errors='replace')}")
            else:
                self.out = torch.zeros(self.K, dtype=torch.float32, device=self.H_inv.device)
                for k in range(self.K):
                    dm, dop = self._grads(_C, k)
                    self.out[k] = (torch.cat([dm, dop.reshape(-1, 1)], dim=1) * self.H_inv).sum()

    def _load(self, w2cs):
        if len(w2cs) > self.K:
            raise ValueError(f"at most {self.K} poses per launch")
        with torch.no_grad():
            self.weight.zero_()
            for k, w in enumerate(w2cs):
                self.w2c[k].copy_(w)
                self.weight[k] = 1.0

    def hessian_sum(self, w2cs, check: bool = True) -> torch.Tensor | None:
        """sum over the (<= K) poses of H(w2c) [P,4] (one graph launch).  With `check` (one host sync)
        returns None when a pose of this launch exceeded the binning capacity (its Hessian would be
        missing from the sum): the caller re-renders the chunk eagerly or rebuilds with more headroom."""
        if self.mode != "sum":
            raise RuntimeError("built for mode='scores'")
        self._load(w2cs)
        if check:
            self.status.zero_()
        self.graph.replay()
        if check and self.overflowed(len(w2cs)):
            return None
        return self.out

    def scores(self, w2cs, H_inv, check: bool = True) -> torch.Tensor | None:
        """sum(H(w2c_k) * H_inv) for each of the (<= K) poses, float64 (one graph launch); None on a
        capacity overflow of any of them (see hessian_sum)."""
        if self.mode != "scores":
            raise RuntimeError("built for mode='sum'")
        self._load(w2cs)
        with torch.no_grad():
            self.H_inv.copy_(H_inv)
        if check:
            self.status.zero_()
        self.graph.replay()
        if check and self.overflowed(len(w2cs)):
            return None
        return self.out[:len(w2cs)].double()

    def overflowed(self, n: int | None = None) -> bool:
        """True if a replay since the last status reset exceeded the capacity in one of the first `n`
        slots (default: all K; padded slots render the previous poses and are not results)."""
        st = self.status[: self.K if n is None else n].cpu()
        return bool((st[:, 0] > self.capacity).any() or (st[:, 2] > st[:, 3]).any() or (st[:, 1] != 0).any())
