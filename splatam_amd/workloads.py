"""The benchmark workloads (BASELINE.json configs 3 and 4) as functions, so that bench.py times exactly what
the GPU parity tests pin (tests/test_gpu_pinned.py) -- the same map, pose perturbation and targets.

* tracking_frame: config 3's SplaTAM tracking frame -- the map of init_tracking_params (scripts/splatam.py:
  103-160, Gaussians in the first camera's frame, pose perturbed by a seeded 0.5 deg / 1 cm), its target
  image and depth rendered at the unperturbed pose (the synthetic stand-in for a dataset frame).
* mapping_workload: config 4's mapping window -- init_mapping_params (anisotropic, SH degree 3) and K
  keyframe targets rendered from a colour-perturbed copy of the map at each keyframe's pose; `prunable`
  Gaussians get opacities under prune_gaussians' removal threshold (configs/replica/splatam.py:101-111:
  0.005), so the mapping frame's pruning iterations (0 and 20) remove Gaussians the way a real sequence's
  faded Gaussians are removed.
* sequence_workload: a synthetic capture (frames along a trajectory, a map with a hole to densify) for the
  SLAM sequence leg (splatam_amd.sequence).
"""
from __future__ import annotations

import torch

from .rasterizer import GaussianRasterizer
from .scenes import Scene
from .slam import _rendervar_colors, camera_settings, color_key, init_mapping_params, init_tracking_params, \
    transform_to_frame, transformed_params2depthplussilhouette, transformed_params2rendervar


def render_targets(params, cam, w2c, t, perturb=None):
    """Target image and depth (im [3,H,W], depth [1,H,W]) of pose column t of `params` rendered with the
    unchanged two-call loop (scripts/splatam.py:255,259); `perturb` replaces params before rendering."""
    truth = dict(params) if perturb is None else perturb
    with torch.no_grad():
        tg = transform_to_frame(truth, t, False, False)
        im, _, _ = GaussianRasterizer(cam)(**_rendervar_colors(truth, transformed_params2rendervar(truth, tg)))
        ds, _, _ = GaussianRasterizer(cam)(**transformed_params2depthplussilhouette(truth, w2c, tg))
    return im, ds[0:1].clone()


def tracking_frame(scene: Scene, dev, num_frames: int = 1, frame: int = 0):
    """(params, curr): init_tracking_params with `num_frames` pose columns and the target of `frame`
    rendered at the unperturbed (identity) pose."""
    params = init_tracking_params(scene, num_frames=max(1, num_frames), device=dev)
    cam = camera_settings(scene.cam, dev)
    w2c = torch.eye(4, device=dev)
    gt = dict(params)
    gt["cam_unnorm_rots"] = torch.zeros_like(params["cam_unnorm_rots"])
    gt["cam_unnorm_rots"][0, 0] = 1.0
    gt["cam_trans"] = torch.zeros_like(params["cam_trans"])
    im, depth = render_targets(params, cam, w2c, frame, perturb=gt)
    return params, {"cam": cam, "w2c": w2c, "im": im.clone(), "depth": depth}


def mapping_keyframes(params, cam, K: int, rank: int, dev, depth_noise: float = 0.01):
    """K keyframe targets (cam / im / depth / w2c / id): the map with perturbed colours rendered at each
    keyframe's pose (the synthetic stand-in for the dataset frames the reference maps against), the depth with
    seeded multiplicative noise (sensor depth is not the map's own render: with the exact render as target every
    depth residual is 0, where the L1 gradient is discontinuous -- torch's |x| has gradient 0 there -- and an ulp
    of difference in the transform turns it into +-1 per pixel)."""
    key = color_key(params)
    w2c = torch.eye(4, device=dev)
    g = torch.Generator().manual_seed(1234)
    kfs = []
    truth = dict(params)
    with torch.no_grad():
        truth[key] = params[key] * 0.9 + 0.05 * torch.rand(params[key].shape, generator=g).to(dev)
    for j in range(K):
        t = rank * K + j
        im, depth = render_targets(params, cam, w2c, t, perturb=truth)
        if depth_noise > 0:
            depth = depth * (1.0 + depth_noise * torch.randn(depth.shape, generator=g).to(dev))
        kfs.append({"cam": cam, "w2c": w2c, "im": im.clamp(0, 1), "depth": depth, "id": t})
    return kfs


def make_prunable(params, fraction: float, seed: int = 4321, opacity: float = 0.002):
    """Sets the logit opacity of a seeded `fraction` of the Gaussians to logit(`opacity`) (< the 0.005
    removal threshold of prune_gaussians): those are removed at the frame's first pruning iteration."""
    P = params["means3D"].shape[0]
    n = int(round(fraction * P))
    if n <= 0:
        return torch.zeros(0, dtype=torch.long)
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(P, generator=g)[:n]
    lo = float(torch.logit(torch.tensor(opacity, dtype=torch.float64)))
    with torch.no_grad():
        params["logit_opacities"][idx.to(params["logit_opacities"].device)] = lo
    return idx


def mapping_workload(scene: Scene, K: int, dev, rank: int = 0, world: int = 1, prunable: float = 0.0):
    """(params, cam, kfs): config 4's mapping window of K keyframes (pose columns rank*K .. rank*K + K - 1 of
    K * world), the Gaussian parameters left as plain tensors (callers set requires_grad)."""
    params = init_mapping_params(scene, num_frames=K * max(world, 1), device=dev)
    cam = camera_settings(scene.cam, dev, sh_degree=scene.sh_degree)
    kfs = mapping_keyframes(params, cam, K, rank, dev)  # targets from the map before the low opacities
    if prunable > 0:
        make_prunable(params, prunable)
    return params, cam, kfs


def sequence_workload(scene: Scene, num_frames: int, dev, hole: float = 0.2, step=(0.02, 0.3),
                      prunable: float = 0.0):
    """(params, frames, cam, w2c, intrinsics, gt_poses): a synthetic capture for splatam_amd.sequence.

    The scene (camera frame of frame 0) is the truth; frame t's camera has moved by t * step = (metres along
    x, degrees about y) and its target image / depth are the truth rendered there (the depth as a sensor
    reports it -- rendered depth / silhouette where the silhouette exceeds 0.5, else 0 -- with 1 % seeded
    noise, as mapping_keyframes).  The map SplaTAM starts from is the truth without the Gaussians whose
    projection in frame 0 falls in the left `hole` fraction of the image (the part the first frames must add
    by densification) and with pose columns t > 0 left at init_tracking_params' perturbed values (the
    sequence overwrites them from the constant-velocity model); `prunable` as make_prunable."""
    truth = init_tracking_params(scene, num_frames=max(1, num_frames), device=dev)
    cam = camera_settings(scene.cam, dev)
    w2c = torch.eye(4, device=dev)
    gt = dict(truth)
    q = torch.zeros(1, 4, num_frames, device=dev)
    tr = torch.zeros(1, 3, num_frames, device=dev)
    for t in range(num_frames):
        a = torch.deg2rad(torch.tensor(step[1] * t, dtype=torch.float64))
        q[0, 0, t], q[0, 2, t] = float(torch.cos(a / 2)), float(torch.sin(a / 2))
        tr[0, 0, t] = step[0] * t
    gt["cam_unnorm_rots"], gt["cam_trans"] = q, tr
    g = torch.Generator().manual_seed(99)
    frames = []
    for t in range(num_frames):
        im, _ = render_targets(truth, cam, w2c, t, perturb=gt)
        with torch.no_grad():  # sensor-like depth: the surface depth (rendered depth / silhouette), 0 where uncovered
            tg = transform_to_frame(gt, t, False, False)
            ds, _, _ = GaussianRasterizer(cam)(**transformed_params2depthplussilhouette(gt, w2c, tg))
            sil = ds[1:2]
            depth = torch.where(sil > 0.5, ds[0:1] / sil.clamp_min(1e-6), torch.zeros_like(sil))
        depth = depth * (1.0 + 0.01 * torch.randn(depth.shape, generator=g).to(dev))
        frames.append({"im": im.clamp(0, 1).contiguous(), "depth": depth.contiguous()})
    c = scene.cam
    u = truth["means3D"][:, 0] / truth["means3D"][:, 2] * c.fx + c.cx
    keep = u >= hole * c.W
    params = {k: (v[keep].contiguous() if v.shape[0] == keep.shape[0] and k not in ("cam_unnorm_rots", "cam_trans")
                  else v.clone()) for k, v in truth.items()}
    params["cam_unnorm_rots"][..., 0] = q[..., 0]
    params["cam_trans"][..., 0] = tr[..., 0]
    if prunable > 0:
        make_prunable(params, prunable)
    return params, frames, cam, w2c, (c.fx, c.fy, c.cx, c.cy), (q, tr)
