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

import math
import os
from dataclasses import dataclass, field

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
    dev, dt = params["means3D"].device, params["means3D"].dtype
    rel_w2c = torch.eye(4, device=dev, dtype=dt)
    rel_w2c[:3, :3] = build_rotation(cam_rot)[0]
    rel_w2c[:3, 3] = trans[0]
    pts = params["means3D"] if gaussians_grad else params["means3D"].detach()
    unnorm = params["unnorm_rotations"] if gaussians_grad else params["unnorm_rotations"].detach()
    if fast:
        out = {"means3D": _affine(pts, rel_w2c[:3, :3], rel_w2c[:3, 3])}
    else:
        pts4 = torch.cat((pts, torch.ones(pts.shape[0], 1, device=dev, dtype=dt)), dim=1)
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
    return {"means3D": tg["means3D"], "colors_precomp": params.get("rgb_colors"),
            "rotations": F.normalize(tg["unnorm_rotations"]), "opacities": torch.sigmoid(params["logit_opacities"]),
            "scales": _scales(params),
            "means2D": torch.zeros_like(params["means3D"], requires_grad=True) + 0}


def transformed_params2depthplussilhouette(params, w2c, tg, fast=True):
    """slam_helpers.py:234-249."""
    return {"means3D": tg["means3D"], "colors_precomp": get_depth_and_silhouette(tg["means3D"], w2c, fast),
            "rotations": F.normalize(tg["unnorm_rotations"]), "opacities": torch.sigmoid(params["logit_opacities"]),
            "scales": _scales(params),
            "means2D": torch.zeros_like(params["means3D"], requires_grad=True) + 0}


def camera_settings(cam, device, sh_degree: int = 0) -> GaussianRasterizationSettings:
    """setup_camera (recon_helpers.py:4-27) moved to `device` (sh_degree > 0: SH colour renders)."""
    return GaussianRasterizationSettings(
        image_height=cam.H, image_width=cam.W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
        bg=torch.zeros(3, dtype=torch.float32, device=device), scale_modifier=1.0,
        viewmatrix=cam.viewmatrix.to(device).contiguous(), projmatrix=cam.projmatrix.to(device).contiguous(),
        sh_degree=sh_degree, campos=cam.campos.to(device).contiguous(), prefiltered=False)  # contiguous: no per-call copy


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
    from .glue import dual_render_tracking_l1, track_transform, tracking_l1
    means, rots, dcol, opac, scales = track_transform(params, iter_time_idx, curr_data["w2c"], pose_adam)
    P = means.shape[0]
    if means2D is None:
        means2D = torch.zeros(P, 3, device=means.device, requires_grad=True)
    if dual and capacity > 0 and seed is not None:  # static mode with a static seed: loss in the render epilogue
        loss, radius = dual_render_tracking_l1(means, params["rgb_colors"], dcol, opac, scales, rots, curr_data["cam"],
                                               capacity, status, curr_data["im"], curr_data["depth"], cfg, seed)
        return loss, radius, means2D
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
                      fused=True, dual=True, fuse_pose=False, variables=None, renderer=None):
    """scripts/splatam.py:220-353 with tracking=True: two renders (RGB, [z,1,z^2]), masked L1 sums.

    fused=True (and fused_eligible): the pose transform / rendervar builders and
    the masked L1 loss run as the HIP glue kernels of include/gsr_glue.h, and with
    dual=True the two renders share one rasterization (gsr_forward_dual).
    fast=True evaluates the same loss without host synchronisation: boolean-mask
    indexing `x[mask].sum()` becomes `where(mask, x, 0).sum()` (same value and
    gradient, NaNs outside the mask excluded exactly as indexing excludes them),
    and the pose transform avoids the K=P GEMM (see _affine).  fast=False is the
    literal statement of the reference code.  fuse_pose=True (with fused, dual): one autograd node for the
    whole iteration whose backward fuses the pose chain into the rasterizer's per-Gaussian backward
    (glue.tracking_iteration, gsr_track_backward_dual).  variables: SplaTAM's densification statistics,
    updated like splatam.py:257,349-351 (literal path only)."""
    if fused and fast and fused_eligible(params, curr_data, cfg):
        if fuse_pose and dual:
            from .glue import tracking_iteration
            loss, radius = tracking_iteration(params, curr_data, iter_time_idx, cfg)
            return loss, radius, None
        return _get_loss_tracking_fused(params, curr_data, iter_time_idx, cfg, dual=dual)
    tg = transform_to_frame(params, iter_time_idx, gaussians_grad=False, camera_grad=True, fast=fast)
    rendervar = transformed_params2rendervar(params, tg)
    depth_sil_rendervar = transformed_params2depthplussilhouette(params, curr_data["w2c"], tg, fast=fast)
    Renderer = GaussianRasterizer if renderer is None else renderer
    rendervar["means2D"].retain_grad()
    im, radius, _ = Renderer(raster_settings=curr_data["cam"])(**rendervar)
    depth_sil, _, _ = Renderer(raster_settings=curr_data["cam"])(**depth_sil_rendervar)
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
    if variables is not None:  # splatam.py:257,349-351
        variables["means2D"] = rendervar["means2D"]
        seen = radius > 0
        variables["max_2D_radius"][seen] = torch.max(radius[seen], variables["max_2D_radius"][seen])
        variables["seen"] = seen
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


# ------------------------------------------------------------------ mapping --
@dataclass
class MappingConfig:
    """configs/replica/splatam.py:82-103 (mapping block); `shs` is this build's lr for the
    SH colour parameters of config 4 (SplaTAM itself renders precomputed rgb_colors)."""
    use_sil_for_loss: bool = False
    use_l1: bool = True
    ignore_outlier_depth_loss: bool = False
    w_im: float = 0.5
    w_depth: float = 1.0
    lrs: dict = field(default_factory=lambda: dict(means3D=0.0001, rgb_colors=0.0025, shs=0.0025,
                                                   unnorm_rotations=0.001, logit_opacities=0.05, log_scales=0.001,
                                                   cam_unnorm_rots=0.0, cam_trans=0.0))
    # configs/replica/splatam.py:112 (True in the gaussian_splatting / post_splatam_opt configs): the
    # densification statistics read means2D.grad of the RGB render alone (splatam.py:256,
    # slam_external.py:100-104), which one dual rasterization does not provide
    use_gaussian_splatting_densification: bool = False
    # configs/replica/splatam.py:101-111: prune_gaussians (utils/slam_external.py:167-188) between
    # loss.backward() and optimizer.step() of every mapping iteration (scripts/splatam.py:876-878)
    prune_gaussians: bool = True
    pruning_dict: dict = field(default_factory=lambda: dict(start_after=0, remove_big_after=0, stop_after=20,
                                                           prune_every=20, removal_opacity_threshold=0.005,
                                                           final_removal_opacity_threshold=0.005,
                                                           reset_opacities=False, reset_opacities_every=500))
    # configs/replica/splatam.py:113-123 (used when use_gaussian_splatting_densification)
    densify_dict: dict = field(default_factory=lambda: dict(start_after=500, remove_big_after=3000, stop_after=5000,
                                                           densify_every=100, grad_thresh=0.0002,
                                                           num_to_split_into=2, removal_opacity_threshold=0.005,
                                                           final_removal_opacity_threshold=0.005,
                                                           reset_opacities_every=3000))


def _gaussian(window_size, sigma):
    """slam_external.py:49-51."""
    gauss = torch.Tensor([math.exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)])
    return gauss / gauss.sum()


def create_window(window_size, channel):
    """slam_external.py:54-58."""
    w1 = _gaussian(window_size, 1.5).unsqueeze(1)
    w2 = w1.mm(w1.t()).float().unsqueeze(0).unsqueeze(0)
    return w2.expand(channel, 1, window_size, window_size).contiguous()


def calc_ssim(img1, img2, window_size=11, size_average=True):
    """slam_external.py:61-97 (literal torch: five depthwise 11x11 convolutions)."""
    channel = img1.size(-3)
    window = create_window(window_size, channel).to(img1.device).type_as(img1)
    pad = window_size // 2
    mu1 = F.conv2d(img1, window, padding=pad, groups=channel)
    mu2 = F.conv2d(img2, window, padding=pad, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    sigma1_sq = F.conv2d(img1 * img1, window, padding=pad, groups=channel) - mu1_sq
    sigma2_sq = F.conv2d(img2 * img2, window, padding=pad, groups=channel) - mu2_sq
    sigma12 = F.conv2d(img1 * img2, window, padding=pad, groups=channel) - mu1_mu2
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    ssim_map = ((2 * mu1_mu2 + c1) * (2 * sigma12 + c2)) / ((mu1_sq + mu2_sq + c1) * (sigma1_sq + sigma2_sq + c2))
    return ssim_map.mean() if size_average else ssim_map.mean(1).mean(1).mean(1)


def l1_loss_v1(x, y):
    """utils/gs_helpers.py:18-19."""
    return torch.abs(x - y).mean()


def color_key(params) -> str:
    return "shs" if "shs" in params else "rgb_colors"


def _rendervar_colors(params, rv):
    if "shs" in params:  # SH colours (config 4): the rasterizer evaluates them (forward.cu:20-73)
        rv.pop("colors_precomp")
        rv["shs"] = params["shs"]
    return rv


def fused_mapping_eligible(params, curr_data, cfg: MappingConfig) -> bool:
    """The fused HIP glue covers SplaTAM's mapping configuration: Gaussians optimised, camera
    fixed (do_ba=False), L1 + SSIM image loss, no silhouette mask, no outlier-depth rejection, and
    no Gaussian-splatting densification (it needs the RGB render's own means2D gradient; the two
    renders then run as two rasterizer calls, the literal path)."""
    return (cfg.use_l1 and not cfg.use_sil_for_loss and not cfg.ignore_outlier_depth_loss
            and not cfg.use_gaussian_splatting_densification
            and params["means3D"].is_cuda and not params["cam_unnorm_rots"].requires_grad
            and not params["cam_trans"].requires_grad
            and curr_data["im"].dim() == 3 and curr_data["depth"].dim() == 3)


_SH_ADAM_FUSED = True  # False: the colour step in gsr_map_transform_bwd_adam (A/B, parity tests)
# the static mapping forward with precomputed colours forms the transform inside its preprocess
# (gsr_forward_dual_static_xf); GSR_MAP_XF_FUSED=0 / False: the transform as its own launch (A/B, parity tests)
_MAP_XF_FUSED = os.environ.get("GSR_MAP_XF_FUSED", "1") != "0"


def _get_loss_mapping_fused(params, curr_data, iter_time_idx, cfg: MappingConfig, adam=None, capacity=0, status=None,
                            means2D=None, alive=None):
    """The fused mapping iteration; capacity > 0: static-capacity rasterization (HIP-graph capturable),
    means2D: optional caller-owned [P,3] tensor (the mapper passes a static one without grad), alive: the
    static forward's pruning mask (GraphMapper's in-frame prune_gaussians)."""
    from .glue import map_transform, mapping_loss
    key = color_key(params)
    defer = [] if (_MAP_XF_FUSED and capacity > 0 and key != "shs") else None
    means, rots, dcol, opac, scales, col = map_transform(params, iter_time_idx, curr_data["w2c"], key, adam, defer)
    if means2D is None:
        means2D = torch.zeros(means.shape[0], 3, device=means.device, requires_grad=True)
    sh, colors = (col, None) if key == "shs" else (None, col)
    # SH colours: the mapping optimizer's colour step runs inside the rasterizer's SH backward stage
    # (gsr_backward_dual_sh_adam) instead of after a round trip of the gradient through HBM
    sh_adam = adam if (adam is not None and sh is not None and _SH_ADAM_FUSED) else None
    im, depth_sil, radius, _ = rasterize_gaussians_dual(means, means2D, sh, colors, dcol, opac, scales, rots, None,
                                                        curr_data["cam"], capacity, status, grad2_channels=1,
                                                        sh_adam=sh_adam, guard_sink=adam, alive=alive,
                                                        xform=defer[0] if defer else None)
    loss = mapping_loss(im, depth_sil, curr_data["im"], curr_data["depth"], cfg.w_im, cfg.w_depth)
    return loss, radius, means2D


def get_loss_mapping(params, curr_data, iter_time_idx, cfg: MappingConfig = MappingConfig(), fused=True,
                     adam=None, loss_dtype=None, variables=None, renderer=None):
    """scripts/splatam.py:220-353 with mapping=True, do_ba=False: two renders (RGB or SH colours, and
    [z,1,z^2]), masked mean depth L1 and 0.8 L1 + 0.2 (1 - SSIM) on the image.

    fused=True (and fused_mapping_eligible): the transform / rendervar builders run as
    gsr_track_transform_fwd + gsr_map_transform_bwd, both renders share one rasterization, and the
    loss is the fused SSIM/L1 kernel pair; `adam` (glue.MapAdam) then applies the mapping optimizer's
    step inside the transform backward.  fused=False is the literal statement of the reference
    (loss_dtype=torch.float64 evaluates its loss terms in double: a tighter test reference; renderer: the
    GaussianRasterizer class the caller imports; variables: the densification statistics, updated like
    splatam.py:257,349-351)."""
    if fused and fused_mapping_eligible(params, curr_data, cfg):
        return _get_loss_mapping_fused(params, curr_data, iter_time_idx, cfg, adam)
    if adam is not None:
        raise RuntimeError("get_loss_mapping: the fused optimizer step needs the fused glue")
    tg = transform_to_frame(params, iter_time_idx, gaussians_grad=True, camera_grad=False, fast=False)
    rendervar = _rendervar_colors(params, transformed_params2rendervar(params, tg))
    depth_sil_rendervar = transformed_params2depthplussilhouette(params, curr_data["w2c"], tg, fast=False)
    rendervar["means2D"].retain_grad()
    Renderer = GaussianRasterizer if renderer is None else renderer
    im, radius, _ = Renderer(raster_settings=curr_data["cam"])(**rendervar)
    depth_sil, _, _ = Renderer(raster_settings=curr_data["cam"])(**depth_sil_rendervar)
    gt_im, gt_depth = curr_data["im"], curr_data["depth"]
    if loss_dtype is not None:
        im, depth_sil, gt_im, gt_depth = (t.to(loss_dtype) for t in (im, depth_sil, gt_im, gt_depth))
    depth = depth_sil[0, :, :].unsqueeze(0)
    depth_sq = depth_sil[2, :, :].unsqueeze(0)
    uncertainty = (depth_sq - depth ** 2).detach()
    nan_mask = (~torch.isnan(depth)) & (~torch.isnan(uncertainty))
    mask = ((gt_depth > 0) & nan_mask).detach()
    loss_depth = torch.abs(gt_depth - depth)[mask].mean()
    loss_im = 0.8 * l1_loss_v1(im, gt_im) + 0.2 * (1.0 - calc_ssim(im, gt_im))
    loss = cfg.w_im * loss_im + cfg.w_depth * loss_depth
    if variables is not None:  # splatam.py:257,349-351
        variables["means2D"] = rendervar["means2D"]
        seen = radius > 0
        variables["max_2D_radius"][seen] = torch.max(radius[seen], variables["max_2D_radius"][seen])
        variables["seen"] = seen
    return loss, radius, rendervar["means2D"]


def map_frame_literal(params, variables, keyframes, num_iters, cfg: MappingConfig = MappingConfig(), optimizer=None,
                      renderer=None, rng=None, losses_out=None, loss_dtype=None):
    """The unchanged mapping loop body of scripts/splatam.py:841-905 for one frame (no progress reports): a
    fresh torch Adam over every parameter group (initialize_optimizer, :842), then per iteration a keyframe
    drawn with np.random.randint (:851), get_loss(mapping=True) through two GaussianRasterizer calls,
    loss.backward(), then (:876-884) prune_gaussians when cfg.prune_gaussians and densify when
    cfg.use_gaussian_splatting_densification (surgery.py restatements; both replace tensors of `params` and
    need variables["scene_radius"]), optimizer.step(), zero_grad.  keyframes: dicts with cam / im / depth /
    w2c / id.  `params` is updated in place (entries replaced when P changes).  loss_dtype: the loss terms in
    that precision (torch.float64: a tighter test reference).  Returns the optimizer."""
    import numpy as np
    from . import surgery
    rng = np.random if rng is None else rng
    if optimizer is None:
        optimizer = mapping_optimizer(params, cfg, fused=False)
    for it in range(num_iters):
        kf = keyframes[int(rng.randint(0, len(keyframes)))]
        loss, _radius, _m2d = get_loss_mapping(params, kf, kf["id"], cfg, fused=False, variables=variables,
                                               renderer=renderer, loss_dtype=loss_dtype)
        loss.backward()
        with torch.no_grad():
            if cfg.prune_gaussians:
                surgery.prune_gaussians(params, variables, optimizer, it, cfg.pruning_dict)
            if cfg.use_gaussian_splatting_densification:
                surgery.densify(params, variables, optimizer, it, cfg.densify_dict)
            optimizer.step()
            optimizer.zero_grad(set_to_none=True)
        if losses_out is not None:
            losses_out.append(loss.detach())
    return optimizer


def init_mapping_params(scene: Scene, num_frames: int, device, pose_noise=(0.5, 0.01), seed=0):
    """Mapping parameter dict: init_tracking_params plus anisotropic log_scales [P,3] when the scene
    is anisotropic, and SH colours `shs` [P,M,3] when it carries them (config 4)."""
    params = init_tracking_params(scene, num_frames, device, pose_noise, seed)
    if not torch.allclose(scene.scales, scene.scales[:, :1].expand_as(scene.scales)):
        params["log_scales"] = torch.log(scene.scales).to(device).float().contiguous()
    if scene.shs is not None:
        params["shs"] = scene.shs.to(device).float().contiguous()
        del params["rgb_colors"]
    return params


def mapping_optimizer(params: dict, cfg: MappingConfig = MappingConfig(), fused=True):
    """initialize_optimizer (scripts/splatam.py:166-172): one Adam group per parameter, eps 1e-15;
    fused=True returns glue.FusedAdam (one HIP launch per step), else torch.optim.Adam."""
    groups = [{"params": [v], "name": k, "lr": cfg.lrs[k]} for k, v in params.items()]
    if fused:
        from .glue import FusedAdam
        return FusedAdam(groups, lr=0.0, eps=1e-15)
    return torch.optim.Adam(groups, lr=0.0, eps=1e-15)


# ------------------------------------------------ literal per-frame tracking --
TRACKING_LRS = dict(means3D=0.0, rgb_colors=0.0, unnorm_rotations=0.0, logit_opacities=0.0, log_scales=0.0,
                    cam_unnorm_rots=0.0004, cam_trans=0.002)  # configs/replica/splatam.py:71-79


def as_parameters(params: dict) -> dict:
    """initialize_params (scripts/splatam.py:150-155): every entry an nn.Parameter requiring grad."""
    return {k: torch.nn.Parameter(v.detach().clone().float().contiguous().requires_grad_(True))
            for k, v in params.items()}


def tracking_variables(P: int, device) -> dict:
    """scripts/splatam.py:157-160."""
    z = lambda: torch.zeros(P, device=device, dtype=torch.float32)  # noqa: E731
    return {"max_2D_radius": z(), "means2D_gradient_accum": z(), "denom": z(), "timestep": z()}


def tracking_optimizer(params: dict, lrs: dict = TRACKING_LRS):
    """initialize_optimizer(params, lrs, tracking=True) (scripts/splatam.py:166-172): torch Adam, one group
    per parameter, default eps."""
    return torch.optim.Adam([{"params": [v], "name": k, "lr": lrs[k]} for k, v in params.items()])


def track_frame_literal(params, variables, curr_data, time_idx, num_iters, cfg: TrackingConfig = TrackingConfig(),
                        optimizer=None, losses_out=None, renderer=None):
    """The unchanged tracking loop body of scripts/splatam.py:700-763 for one frame (use_gt_poses=False,
    no depth-loss-threshold extension): get_loss(tracking=True) through two GaussianRasterizer calls,
    loss.backward(), Adam over every parameter group, zero_grad, the best-candidate pose kept by loss
    (:726-731) and written back after the last iteration (:760-763).  renderer: the GaussianRasterizer class
    the caller imports (default splatam_amd's; diff_gaussian_rasterization's is the same drop-in).
    Returns the optimizer."""
    if optimizer is None:
        optimizer = tracking_optimizer(params)
    cand_rot = params["cam_unnorm_rots"][..., time_idx].detach().clone()
    cand_tran = params["cam_trans"][..., time_idx].detach().clone()
    current_min_loss = float(1e20)
    for _ in range(num_iters):
        loss, _radius, _m2d = get_loss_tracking(params, curr_data, time_idx, cfg, fast=False, fused=False,
                                                variables=variables, renderer=renderer)
        loss.backward()
        optimizer.step()
        optimizer.zero_grad(set_to_none=True)
        with torch.no_grad():
            if losses_out is not None:
                losses_out.append(loss.detach())
            if loss < current_min_loss:
                current_min_loss = loss
                cand_rot = params["cam_unnorm_rots"][..., time_idx].detach().clone()
                cand_tran = params["cam_trans"][..., time_idx].detach().clone()
    with torch.no_grad():
        params["cam_unnorm_rots"][..., time_idx] = cand_rot
        params["cam_trans"][..., time_idx] = cand_tran
    return optimizer
