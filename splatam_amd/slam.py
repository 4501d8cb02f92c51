"""SplaTAM's caller glue around the rasterizer: the unchanged callers of the
drop-in API, restated so the tracking / mapping iteration can be run and
benchmarked without SplaTAM's dataset / wandb / cv2 dependencies.

Follows utils/slam_helpers.py (transform_to_frame 252-304, rendervar builders
124-139 / 234-249, get_depth_and_silhouette 196-213), utils/slam_external.py
(build_rotation 25-42, calc_ssim 66-97) and scripts/splatam.py get_loss
(220-353) with the Replica tracking config (configs/replica/splatam.py:59-70).
Everything here is plain torch on the rasterizer's device; the rasterizer
itself is splatam_amd.rasterizer (HIP).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .rasterizer import GaussianRasterizationSettings, GaussianRasterizer, rasterize_gaussians_dual
from .scenes import Scene


def build_rotation(q):
    """slam_external.py:25-42 (normalises q first)."""
    q = q / torch.sqrt((q * q).sum(dim=1, keepdim=True))
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], dim=1)
    return R.reshape(-1, 3, 3)


def quat_mult(q1, q2):
    """slam_helpers.py quat_mult (Hamilton product, w first)."""
    w1, x1, y1, z1 = q1.T
    w2, x2, y2, z2 = q2.T
    return torch.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2]).T


def _affine(pts, R, t):
    """pts @ R^T + t written elementwise: mathematically the reference's
    (rel_w2c @ pts4.T).T[:, :3], but its backward w.r.t. (R, t) is a plain
    reduction over the P points instead of a K=P GEMM (250 us on hipBLASLt)."""
    return (pts.unsqueeze(1) * R.unsqueeze(0)).sum(-1) + t


def transform_to_frame(params, time_idx, gaussians_grad, camera_grad, fast=True):
    """slam_helpers.py:252-304 (fast=False: the literal matmul formulation)."""
    rots = params["cam_unnorm_rots"][..., time_idx]
    trans = params["cam_trans"][..., time_idx]
    if not camera_grad:
        rots, trans = rots.detach(), trans.detach()
    cam_rot = F.normalize(rots)
    dev = params["means3D"].device
    rel_w2c = torch.eye(4, device=dev, dtype=torch.float32)
    rel_w2c[:3, :3] = build_rotation(cam_rot)[0]
    rel_w2c[:3, 3] = trans[0]
    pts = params["means3D"] if gaussians_grad else params["means3D"].detach()
    unnorm = params["unnorm_rotations"] if gaussians_grad else params["unnorm_rotations"].detach()
    if fast:
        out = {"means3D": _affine(pts, rel_w2c[:3, :3], rel_w2c[:3, 3])}
    else:
        pts4 = torch.cat((pts, torch.ones(pts.shape[0], 1, device=dev)), dim=1)
        out = {"means3D": (rel_w2c @ pts4.T).T[:, :3]}
    if params["log_scales"].shape[1] == 1:
        out["unnorm_rotations"] = unnorm
    else:
        out["unnorm_rotations"] = quat_mult(cam_rot, F.normalize(unnorm))
    return out


def _scales(params):
    ls = params["log_scales"]
    return torch.exp(torch.tile(ls, (1, 3)) if ls.shape[1] == 1 else ls)


def get_depth_and_silhouette(pts_3D, w2c, fast=True):
    """slam_helpers.py:196-213: per-Gaussian colours [z, 1, z^2] for the depth/silhouette render."""
    if fast:
        z = (pts_3D * w2c[2, :3]).sum(-1, keepdim=True) + w2c[2, 3]
    else:
        pts4 = torch.cat((pts_3D, torch.ones_like(pts_3D[:, :1])), dim=-1)
        z = (w2c @ pts4.transpose(0, 1)).transpose(0, 1)[:, 2:3]
    return torch.cat([z, torch.ones_like(z), z * z], dim=1)


def transformed_params2rendervar(params, tg):
    """slam_helpers.py:124-139."""
    return {"means3D": tg["means3D"], "colors_precomp": params["rgb_colors"],
            "rotations": F.normalize(tg["unnorm_rotations"]), "opacities": torch.sigmoid(params["logit_opacities"]),
            "scales": _scales(params),
            "means2D": torch.zeros_like(params["means3D"], requires_grad=True) + 0}


def transformed_params2depthplussilhouette(params, w2c, tg, fast=True):
    """slam_helpers.py:234-249."""
    return {"means3D": tg["means3D"], "colors_precomp": get_depth_and_silhouette(tg["means3D"], w2c, fast),
            "rotations": F.normalize(tg["unnorm_rotations"]), "opacities": torch.sigmoid(params["logit_opacities"]),
            "scales": _scales(params),
            "means2D": torch.zeros_like(params["means3D"], requires_grad=True) + 0}


def camera_settings(cam, device) -> GaussianRasterizationSettings:
    """setup_camera (recon_helpers.py:4-27) moved to `device`."""
    return GaussianRasterizationSettings(
        image_height=cam.H, image_width=cam.W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.zeros(3, dtype=torch.float32, device=device), scale_modifier=1.0,
        viewmatrix=cam.viewmatrix.to(device).contiguous(), projmatrix=cam.projmatrix.to(device).contiguous(),
        sh_degree=0, campos=cam.campos.to(device).contiguous(), prefiltered=False)  # contiguous: no per-call copy


@dataclass
class TrackingConfig:
    """configs/replica/splatam.py:59-70 (tracking block)."""
    use_sil_for_loss: bool = True
    sil_thres: float = 0.99
    use_l1: bool = True
    ignore_outlier_depth_loss: bool = False
    w_im: float = 0.5
    w_depth: float = 1.0


def fused_eligible(params, curr_data, cfg: TrackingConfig) -> bool:
    """The fused HIP glue covers SplaTAM's tracking configuration: only the camera
    pose needs gradients, L1 with the silhouette mask, no outlier-depth rejection."""
    gauss_keys = ("means3D", "rgb_colors", "unnorm_rotations", "logit_opacities", "log_scales")
    return (cfg.use_l1 and cfg.use_sil_for_loss and not cfg.ignore_outlier_depth_loss
            and params["means3D"].is_cuda and not any(params[k].requires_grad for k in gauss_keys)
            and curr_data["im"].dim() == 3 and curr_data["depth"].dim() == 3)


def _get_loss_tracking_fused(params, curr_data, iter_time_idx, cfg: TrackingConfig, dual=True, capacity=0,
                             status=None, pose_adam=None, means2D=None, seed=None):
    """means2D: optional caller-owned [P,3] tensor (the tracker passes a static one without grad).
    seed: the static loss seed the caller will backward with (loss gradient formed in the forward)."""
    from .glue import track_transform, tracking_l1
    means, rots, dcol, opac, scales = track_transform(params, iter_time_idx, curr_data["w2c"], pose_adam)
    P = means.shape[0]
    if means2D is None:
        means2D = torch.zeros(P, 3, device=means.device, requires_grad=True)
    if dual:  # both renders in one rasterization (means2D.grad then holds the sum over both images)
        im, depth_sil, radius, _ = rasterize_gaussians_dual(means, means2D, None, params["rgb_colors"], dcol, opac,
                                                            scales, rots, None, curr_data["cam"], capacity, status,
                                                            grad2_channels=1)  # the L1 loss reads depth only
    else:
        means2D_ds = torch.zeros(P, 3, device=means.device, requires_grad=True)
        ras = GaussianRasterizer(raster_settings=curr_data["cam"])
        im, radius, _ = ras(means3D=means, means2D=means2D, colors_precomp=params["rgb_colors"], opacities=opac,
                            scales=scales, rotations=rots)
        depth_sil, _, _ = ras(means3D=means, means2D=means2D_ds, colors_precomp=dcol, opacities=opac, scales=scales,
                              rotations=rots)
    loss = tracking_l1(im, depth_sil, curr_data["im"], curr_data["depth"], cfg.sil_thres, cfg.w_im, cfg.w_depth,
                       seed=seed)
    return loss, radius, means2D


def get_loss_tracking(params, curr_data, iter_time_idx, cfg: TrackingConfig = TrackingConfig(), fast=True,
                      fused=True, dual=True):
    """scripts/splatam.py:220-353 with tracking=True: two renders (RGB, [z,1,z^2]), masked L1 sums.

    fused=True (and fused_eligible): the pose transform / rendervar builders and
    the masked L1 loss run as the HIP glue kernels of include/gsr_glue.h, and with
    dual=True the two renders share one rasterization (gsr_forward_dual).
    fast=True evaluates the same loss without host synchronisation: boolean-mask
    indexing `x[mask].sum()` becomes `where(mask, x, 0).sum()` (same value and
    gradient, NaNs outside the mask excluded exactly as indexing excludes them),
    and the pose transform avoids the K=P GEMM (see _affine).  fast=False is the
    literal statement of the reference code."""
    if fused and fast and fused_eligible(params, curr_data, cfg):
        return _get_loss_tracking_fused(params, curr_data, iter_time_idx, cfg, dual=dual)
    tg = transform_to_frame(params, iter_time_idx, gaussians_grad=False, camera_grad=True, fast=fast)
    rendervar = transformed_params2rendervar(params, tg)
    depth_sil_rendervar = transformed_params2depthplussilhouette(params, curr_data["w2c"], tg, fast=fast)
    rendervar["means2D"].retain_grad()
    im, radius, _ = GaussianRasterizer(raster_settings=curr_data["cam"])(**rendervar)
    depth_sil, _, _ = GaussianRasterizer(raster_settings=curr_data["cam"])(**depth_sil_rendervar)
    depth = depth_sil[0, :, :].unsqueeze(0)
    silhouette = depth_sil[1, :, :]
    presence_sil_mask = silhouette > cfg.sil_thres
    depth_sq = depth_sil[2, :, :].unsqueeze(0)
    uncertainty = (depth_sq - depth ** 2).detach()
    nan_mask = (~torch.isnan(depth)) & (~torch.isnan(uncertainty))
    mask = (curr_data["depth"] > 0) & nan_mask
    if cfg.use_sil_for_loss:
        mask = mask & presence_sil_mask
    mask = mask.detach()
    color_mask = torch.tile(mask, (3, 1, 1)).detach()
    if fast:
        zero = torch.zeros((), device=depth.device, dtype=depth.dtype)
        loss_depth = torch.where(mask, torch.abs(curr_data["depth"] - depth), zero).sum()
        loss_im = torch.where(color_mask, torch.abs(curr_data["im"] - im), zero).sum()
    else:
        loss_depth = torch.abs(curr_data["depth"] - depth)[mask].sum()
        loss_im = torch.abs(curr_data["im"] - im)[color_mask].sum()
    loss = cfg.w_im * loss_im + cfg.w_depth * loss_depth
    return loss, radius, rendervar["means2D"]


def init_tracking_params(scene: Scene, num_frames: int, device, pose_noise=(0.5, 0.01), seed=0):
    """SplaTAM parameter dict (scripts/splatam.py:103-172 layout) with iso log_scales [P,1],
    plus per-frame camera poses perturbed from identity by `pose_noise` = (deg, m)."""
    g = torch.Generator().manual_seed(seed + 1000)
    P = scene.P
    params = {
        "means3D": scene.means3D.clone(),
        "rgb_colors": scene.colors.clone(),
        "unnorm_rotations": scene.rotations.clone(),
        "logit_opacities": torch.logit(scene.opacities.clamp(1e-6, 1 - 1e-6)),
        "log_scales": torch.log(scene.scales[:, :1]).clone(),
    }
    rots = torch.zeros(1, 4, num_frames)
    rots[0, 0] = 1.0
    trans = torch.zeros(1, 3, num_frames)
    ang = torch.deg2rad(torch.tensor(pose_noise[0]))
    for t in range(num_frames):
        axis = torch.randn(3, generator=g)
        axis = axis / axis.norm()
        rots[0, 0, t] = torch.cos(ang / 2)
        rots[0, 1:, t] = axis * torch.sin(ang / 2)
        d = torch.randn(3, generator=g)
        trans[0, :, t] = pose_noise[1] * d / d.norm()
    params["cam_unnorm_rots"] = rots
    params["cam_trans"] = trans
    out = {k: v.to(device).float().contiguous() for k, v in params.items()}
    assert out["means3D"].shape[0] == P
    return out
