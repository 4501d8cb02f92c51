"""Isolate the fused-vs-literal mapping gradient difference: loss gradient images, the dual rasterizer
backward, the transform backward (config 4 map or a small SH-3 scene)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from splatam_amd import glue
from splatam_amd.rasterizer import GaussianRasterizer, rasterize_gaussians_dual
from splatam_amd.scenes import config_scene, make_scene
from splatam_amd.slam import MappingConfig, calc_ssim, color_key, l1_loss_v1, transform_to_frame, \
    transformed_params2depthplussilhouette, transformed_params2rendervar, _rendervar_colors
from splatam_amd.workloads import mapping_workload

cfg_id = int(sys.argv[1]) if len(sys.argv) > 1 else 1
dev = torch.device("cuda:0")
scene = config_scene(4) if cfg_id == 4 else make_scene(20000, 320, 240, seed=7, anisotropic=True, sh_degree=3)
params, cam, kfs = mapping_workload(scene, 4, dev)
kf = kfs[1]
cfg = MappingConfig()
key = color_key(params)


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


# 1. loss gradient images: literal loss vs fused loss on the same images
tg = transform_to_frame(params, kf["id"], gaussians_grad=False, camera_grad=False, fast=False)
with torch.no_grad():
    rv = _rendervar_colors(params, transformed_params2rendervar(params, tg))
    dv = transformed_params2depthplussilhouette(params, kf["w2c"], tg, fast=False)
    im, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**rv)
    ds, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**dv)
im1, ds1 = im.clone().requires_grad_(True), ds.clone().requires_grad_(True)
depth = ds1[0:1]
depth_sq = ds1[2:3]
unc = (depth_sq - depth ** 2).detach()
nan_mask = (~torch.isnan(depth)) & (~torch.isnan(unc))
mask = ((kf["depth"] > 0) & nan_mask).detach()
loss_l = cfg.w_im * (0.8 * l1_loss_v1(im1, kf["im"]) + 0.2 * (1.0 - calc_ssim(im1, kf["im"]))) + \
    cfg.w_depth * torch.abs(kf["depth"] - depth)[mask].mean()
gi_l, gd_l = torch.autograd.grad(loss_l, (im1, ds1))
im2, ds2 = im.clone().requires_grad_(True), ds.clone().requires_grad_(True)
loss_f = glue.mapping_loss(im2, ds2, kf["im"], kf["depth"], cfg.w_im, cfg.w_depth)
gi_f, gd_f = torch.autograd.grad(loss_f, (im2, ds2))
print(f"loss literal {float(loss_l):.8f} fused {float(loss_f):.8f}")
print(f"dL/dim rel {rel(gi_f, gi_l):.3e} (|g| {float(gi_l.norm()):.3e}); dL/ddepth_sil ch0 rel "
      f"{rel(gd_f[0], gd_l[0]):.3e} (|g| {float(gd_l[0].norm()):.3e}); ch1 |f| {float(gd_f[1].norm()):.3e} |l| "
      f"{float(gd_l[1].norm()):.3e}; ch2 |f| {float(gd_f[2].norm()):.3e} |l| {float(gd_l[2].norm()):.3e}")

# 2. rasterizer: two single calls (literal autograd) vs the dual call, same upstream gradient images
def leaves():
    return {k: v.detach().clone().requires_grad_(True) for k, v in
            dict(m=tg["means3D"], r=torch.nn.functional.normalize(tg["unnorm_rotations"]),
                 o=torch.sigmoid(params["logit_opacities"]), s=torch.exp(params["log_scales"])
                 if params["log_scales"].shape[1] == 3 else torch.exp(params["log_scales"]).repeat(1, 3),
                 c=params[key]).items()}


a = leaves()
zc = transformed_params2depthplussilhouette(params, kf["w2c"], tg, fast=False)["colors_precomp"].detach()
dcol = zc.clone().requires_grad_(True)
rv_a = dict(means3D=a["m"], opacities=a["o"], scales=a["s"], rotations=a["r"],
            means2D=torch.zeros_like(a["m"], requires_grad=True))
if key == "shs":
    rv_a["shs"] = a["c"]
else:
    rv_a["colors_precomp"] = a["c"]
i_a, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**rv_a)
dv_a = dict(means3D=a["m"], opacities=a["o"], scales=a["s"], rotations=a["r"], colors_precomp=dcol,
            means2D=torch.zeros_like(a["m"], requires_grad=True))
d_a, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**dv_a)
torch.autograd.backward([i_a, d_a], [gi_l, gd_l])
b = leaves()
dcol_b = zc.clone().requires_grad_(True)
sh, colors = (b["c"], None) if key == "shs" else (None, b["c"])
i_b, d_b, _, _ = rasterize_gaussians_dual(b["m"], torch.zeros_like(b["m"]), sh, colors, dcol_b, b["o"], b["s"],
                                          b["r"], None, kf["cam"], 0, None, grad2_channels=1)
print(f"images: rgb rel {rel(i_b, i_a):.3e} depth_sil rel {rel(d_b, d_a):.3e}")
gd_l1 = gd_l.clone()
gd_l1[1:] = 0.0
torch.autograd.backward([i_b, d_b], [gi_l, gd_l1])
# (literal with channels 1, 2 of the depth gradient zeroed too, for the like-for-like comparison)
c = leaves()
dcol_c = zc.clone().requires_grad_(True)
rv_c = dict(rv_a, means3D=c["m"], opacities=c["o"], scales=c["s"], rotations=c["r"],
            means2D=torch.zeros_like(c["m"], requires_grad=True))
if key == "shs":
    rv_c["shs"] = c["c"]
else:
    rv_c["colors_precomp"] = c["c"]
i_c, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**rv_c)
d_c, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**dict(dv_a, means3D=c["m"], opacities=c["o"],
                                                                   scales=c["s"], rotations=c["r"],
                                                                   colors_precomp=dcol_c,
                                                                   means2D=torch.zeros_like(c["m"],
                                                                                            requires_grad=True)))
torch.autograd.backward([i_c, d_c], [gi_l, gd_l1])
for k in ("m", "r", "o", "s", "c"):
    print(f"  d{k}: dual vs two calls (ch0 only) rel {rel(b[k].grad, c[k].grad):.3e}; two calls ch0-only vs "
          f"all-channel rel {rel(c[k].grad, a[k].grad):.3e}; |g| {float(a[k].grad.norm()):.3e}")
print(f"  dcolors2 ch0: {rel(dcol_b.grad[:, 0], dcol_c.grad[:, 0]):.3e}")
