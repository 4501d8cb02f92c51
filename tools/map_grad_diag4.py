"""Hybrid mapping pipelines (transform / rasterization / loss, each literal or fused) against the literal one."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from splatam_amd import glue
from splatam_amd.rasterizer import GaussianRasterizer, rasterize_gaussians_dual
from splatam_amd.scenes import make_scene
from splatam_amd.slam import MappingConfig, _scales, calc_ssim, color_key, get_depth_and_silhouette, l1_loss_v1, \
    transform_to_frame
from splatam_amd.workloads import mapping_workload

dev = torch.device("cuda:0")
scene = make_scene(20000, 320, 240, seed=7, anisotropic=True, sh_degree=3)
params, cam, kfs = mapping_workload(scene, 4, dev)
key = color_key(params)
kf = kfs[1]
t = kf["id"]
cfg = MappingConfig()
GK = ("means3D", "unnorm_rotations", "logit_opacities", "log_scales", key)


def leaves():
    return {k: (v.detach().clone().requires_grad_(True) if k in GK else v.detach().clone()) for k, v in params.items()}


def xf_lit(p):
    tg = transform_to_frame(p, t, gaussians_grad=True, camera_grad=False, fast=False)
    return (tg["means3D"], F.normalize(tg["unnorm_rotations"]), get_depth_and_silhouette(tg["means3D"], kf["w2c"], False),
            torch.sigmoid(p["logit_opacities"]), _scales(p), p[key])


def xf_fused(p):
    return glue.map_transform(p, t, kf["w2c"], key)


def ras_two(m, r, dc, o, s, col):
    rv = dict(means3D=m, rotations=r, opacities=o, scales=s, means2D=torch.zeros_like(m, requires_grad=True) + 0)
    if key == "shs":
        rv["shs"] = col
    else:
        rv["colors_precomp"] = col
    im, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**rv)
    ds, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(means3D=m, rotations=r, opacities=o, scales=s,
                                                             colors_precomp=dc,
                                                             means2D=torch.zeros_like(m, requires_grad=True) + 0)
    return im, ds


def ras_dual(m, r, dc, o, s, col):
    sh, colors = (col, None) if key == "shs" else (None, col)
    im, ds, _, _ = rasterize_gaussians_dual(m, torch.zeros_like(m), sh, colors, dc, o, s, r, None, kf["cam"], 0,
                                            None, grad2_channels=1)
    return im, ds


def loss_lit(im, ds):
    depth, depth_sq = ds[0:1], ds[2:3]
    unc = (depth_sq - depth ** 2).detach()
    mask = ((kf["depth"] > 0) & (~torch.isnan(depth)) & (~torch.isnan(unc))).detach()
    return cfg.w_im * (0.8 * l1_loss_v1(im, kf["im"]) + 0.2 * (1.0 - calc_ssim(im, kf["im"]))) + \
        cfg.w_depth * torch.abs(kf["depth"] - depth)[mask].mean()


def loss_fused(im, ds):
    return glue.mapping_loss(im, ds, kf["im"], kf["depth"], cfg.w_im, cfg.w_depth)


def run(xf, ras, lo):
    p = leaves()
    outs = xf(p)
    im, ds = ras(*outs[:6]) if len(outs) >= 6 else None
    loss = lo(im, ds)
    loss.backward()
    return float(loss.detach()), {k: p[k].grad.detach().double() for k in GK}


ref_l, ref = run(xf_lit, ras_two, loss_lit)
for name, combo in (("F--", (xf_fused, ras_two, loss_lit)), ("-F-", (xf_lit, ras_dual, loss_lit)),
                    ("--F", (xf_lit, ras_two, loss_fused)), ("FF-", (xf_fused, ras_dual, loss_lit)),
                    ("F-F", (xf_fused, ras_two, loss_fused)), ("-FF", (xf_lit, ras_dual, loss_fused)),
                    ("FFF", (xf_fused, ras_dual, loss_fused))):
    l, g = run(*combo)
    print(name, f"loss rel {abs(l - ref_l) / ref_l:.2e}", " ".join(
        f"{k[:6]} {float((g[k] - ref[k]).norm() / ref[k].norm()):.2e}" for k in GK))


# sensitivity of the literal pipeline itself: the literal transform's outputs perturbed by ~1 ulp
def xf_lit_ulp(p, seed=[0]):
    outs = list(xf_lit(p))
    gg = torch.Generator(device=dev).manual_seed(100 + seed[0])
    seed[0] += 1
    for j in (0, 1, 2):
        outs[j] = outs[j] * (1.0 + 6e-8 * torch.randn(outs[j].shape, device=dev, generator=gg))
    return tuple(outs)


for rep in range(2):
    l, g = run(xf_lit_ulp, ras_two, loss_lit)
    print("L~- ulp", f"loss rel {abs(l - ref_l) / ref_l:.2e}", " ".join(
        f"{k[:6]} {float((g[k] - ref[k]).norm() / ref[k].norm()):.2e}" for k in GK))
