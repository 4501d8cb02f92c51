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
with power = 2: gauss_jac, render_bwd_power, gauss_bwd_power) and only the two
gradients H needs are requested.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import dist as sd
from .rasterizer import GaussianRasterizer

SEED = 1e-3      # im.backward(gradient=torch.ones_like(im) * 1e-3)  (ros_handler.py:888)
H_EPS = 0.1      # torch.reciprocal(H_train + 0.1)                   (ros_handler.py:829)


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
        with torch.no_grad():  # (rel_w2c @ pts4.T).T[:, :3]
            pts4 = torch.cat((means, torch.ones(means.shape[0], 1, device=means.device)), dim=1)
            pts = (w2c @ pts4.T).T[:, :3].contiguous()
        pts.requires_grad_(True)
        opac = self.opacities.detach().clone().requires_grad_(True)
        means2D = torch.zeros_like(pts)
        im, _, _ = GaussianRasterizer(self.cam, backward_power=2)(
            means3D=pts, means2D=means2D, opacities=opac, colors_precomp=self.colors.detach(),
            scales=self.scales.detach(), rotations=self.rotations.detach())
        im.backward(gradient=torch.full_like(im, SEED))
        return torch.cat([pts.grad.reshape(pts.shape[0], -1), opac.grad.reshape(pts.shape[0], -1)], dim=1)

    def fit_visited(self, w2cs) -> torch.Tensor:
        """compute_H_visited_inv over all visited poses: each rank sums the Hessians of its shard
        (poses r, r+W, ...), one all-reduce merges them.  Returns (and keeps) H_train_inv."""
        r, w = sd.world()
        H = None
        for j in range(r, len(w2cs), w):
            h = self.hessian(w2cs[j])
            H = h if H is None else H + h
        if H is None:  # this rank has no pose: contribute zeros of the right shape
            P = self.params["means3D"].shape[0]
            H = torch.zeros(P, 4, device=self.params["means3D"].device)
        sd.all_reduce_sum_(H)
        self.H_train_inv = torch.reciprocal(H + H_EPS)
        return self.H_train_inv

    def eig_scores(self, w2cs) -> torch.Tensor:
        """compute_eig_score for every candidate pose: sum(H(pose) * H_train_inv).  The batch is
        sharded over ranks; returns all scores (float64, in pose order) on every rank."""
        if self.H_train_inv is None:
            raise RuntimeError("fit_visited() first (H_train_inv)")
        r, w = sd.world()
        n = len(w2cs)
        per = -(-n // w) if n else 0
        dev = self.H_train_inv.device
        local = torch.zeros(max(per, 1), dtype=torch.float64, device=dev)
        for k, j in enumerate(range(r, n, w)):
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
