"""Diagnostic: isolates which stage of the fused mapping iteration departs from the
literal restatement (GPU).  python tools/diag_mapping.py [aniso]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from splatam_amd import slam  # noqa: E402
from splatam_amd.glue import map_transform, mapping_loss  # noqa: E402
from splatam_amd.rasterizer import GaussianRasterizer, rasterize_gaussians_dual  # noqa: E402
from tests.test_gpu_mapping import GAUSS_KEYS, _map_params, _rel, _scene_targets  # noqa: E402

cuda = torch.device("cuda:0")
aniso = "aniso" in sys.argv
_, params, cam = _map_params(cuda, aniso, False)
curr = _scene_targets(params, cam, cuda)
keys = GAUSS_KEYS + ("rgb_colors",)


def leaves():
    p = dict(params)
    for k in keys:
        p[k] = params[k].detach().clone().requires_grad_(True)
    return p


def run(variant):
    p = leaves()
    if variant == "literal64":
        loss, _, _ = slam.get_loss_mapping(p, curr, 1, fused=False, loss_dtype=torch.float64)
    elif variant == "fused":
        loss, _, _ = slam.get_loss_mapping(p, curr, 1, fused=True)
    else:
        means, rots, dcol, opac, scales, col = map_transform(p, 1, curr["w2c"])
        P = means.shape[0]
        if variant == "two_calls":
            m2a = torch.zeros(P, 3, device=cuda, requires_grad=True)
            m2b = torch.zeros(P, 3, device=cuda, requires_grad=True)
            ras = GaussianRasterizer(cam)
            im, _, _ = ras(means3D=means, means2D=m2a, colors_precomp=col, opacities=opac, scales=scales,
                           rotations=rots)
            ds, _, _ = ras(means3D=means, means2D=m2b, colors_precomp=dcol, opacities=opac, scales=scales,
                           rotations=rots)
        else:
            m2 = torch.zeros(P, 3, device=cuda, requires_grad=True)
            g2c = 3 if variant == "dual3" else 1
            im, ds, _, _ = rasterize_gaussians_dual(means, m2, None, col, dcol, opac, scales, rots, None, cam,
                                                    grad2_channels=g2c)
        loss = mapping_loss(im, ds, curr["im"], curr["depth"])
    loss.backward()
    return {k: p[k].grad for k in keys}


ref = run("literal64")
for v in ("two_calls", "dual3", "dual1", "fused"):
    g = run(v)
    print(v, {k: f"{_rel(g[k], ref[k]):.2e}" for k in keys})

# per-pixel check of the loss kernel on this scene's images
with torch.no_grad():
    p = dict(params)
    tg = slam.transform_to_frame(p, 1, True, False, fast=False)
    rv = slam.transformed_params2rendervar(p, tg)
    im, _, _ = GaussianRasterizer(cam)(**rv)
    ds, _, _ = GaussianRasterizer(cam)(**slam.transformed_params2depthplussilhouette(p, curr["w2c"], tg, fast=False))
a_im, a_ds = im.clone().requires_grad_(True), ds.clone().requires_grad_(True)
mapping_loss(a_im, a_ds, curr["im"], curr["depth"]).backward()
r_im, r_ds = im.double().requires_grad_(True), ds.double().requires_grad_(True)
from tests.test_gpu_mapping import _literal_loss  # noqa: E402
_literal_loss(r_im, r_ds, curr["im"].double(), curr["depth"].double()).backward()
d = (a_im.grad.double() - r_im.grad).abs()
print("im grad rel", _rel(a_im.grad, r_im.grad), "depth grad rel", _rel(a_ds.grad, torch.nan_to_num(r_ds.grad)))
idx = torch.nonzero(d == d.max())[0].tolist()
c, y, x = idx
print("max err at", idx, "err", float(d.max()), "ref", float(r_im.grad[c, y, x]), "im", float(im[c, y, x]),
      "gt", float(curr["im"][c, y, x]), "ref grad norm max", float(r_im.grad.abs().max()))
print("fraction of pixels with im == gt:", float((im == curr["im"]).float().mean()),
      "im==0:", float((im == 0).float().mean()))

# transform forward: literal vs HIP, and the images each produces
with torch.no_grad():
    outs = map_transform(dict(params), 1, curr["w2c"])
    ref_out = (rv["means3D"], rv["rotations"], slam.transformed_params2depthplussilhouette(
        p, curr["w2c"], tg, fast=False)["colors_precomp"], rv["opacities"], rv["scales"])
    for name, o, r in zip(("means", "rot", "dcol", "opac", "scales"), outs, ref_out):
        print(name, "max abs diff", float((o - r).abs().max()), "rel", _rel(o, r))
    im2, _, _ = GaussianRasterizer(cam)(means3D=outs[0], means2D=torch.zeros_like(outs[0]), colors_precomp=outs[5],
                                        opacities=outs[3], scales=outs[4], rotations=outs[1])
    print("image max abs diff (HIP transform vs literal)", float((im2 - im).abs().max()))

gl = run("two_calls")
for k in keys:
    a, r = gl[k].double().reshape(gl[k].shape[0], -1), ref[k].double().reshape(ref[k].shape[0], -1)
    row = (a - r).norm(dim=1) / (r.norm(dim=1) + 1e-3 * r.norm(dim=1).mean() + 1e-30)
    print(k, "rows > 1e-4:", int((row > 1e-4).sum()), "of", row.numel(), "rows > 1e-2:", int((row > 1e-2).sum()),
          "rel L2 excluding them:", _rel(a[row <= 1e-4], r[row <= 1e-4]))
