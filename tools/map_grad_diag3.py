"""The mapping transform backward (gsr_map_transform_bwd) against autograd of the literal transform_to_frame
+ rendervar builders, with random upstream gradients; then the whole fused mapping loss vs the literal one."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from splatam_amd import glue
from splatam_amd.scenes import make_scene
from splatam_amd.slam import MappingConfig, _scales, color_key, get_depth_and_silhouette, get_loss_mapping, \
    transform_to_frame
from splatam_amd.workloads import mapping_workload

dev = torch.device("cuda:0")
scene = make_scene(20000, 320, 240, seed=7, anisotropic=True, sh_degree=3)
params, cam, kfs = mapping_workload(scene, 4, dev)
key = color_key(params)
kf = kfs[1]
t = kf["id"]


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def leaves():
    return {k: (v.detach().clone().requires_grad_(True) if k in ("means3D", "unnorm_rotations", "logit_opacities",
                                                                 "log_scales", key) else v.detach().clone())
            for k, v in params.items()}


g = torch.Generator(device=dev).manual_seed(3)
P = params["means3D"].shape[0]
up = [torch.randn(P, 3, device=dev, generator=g), torch.randn(P, 4, device=dev, generator=g),
      torch.randn(P, 3, device=dev, generator=g), torch.randn(P, 1, device=dev, generator=g),
      torch.randn(P, 3, device=dev, generator=g)]
up[2][:, 1:] = 0.0
a = leaves()
tg = transform_to_frame(a, t, gaussians_grad=True, camera_grad=False, fast=False)
outs = [tg["means3D"], torch.nn.functional.normalize(tg["unnorm_rotations"]),
        get_depth_and_silhouette(tg["means3D"], kf["w2c"], fast=False), torch.sigmoid(a["logit_opacities"]),
        _scales(a)]
torch.autograd.backward(outs, up)
b = leaves()
o = glue.map_transform(b, t, kf["w2c"], key)
torch.autograd.backward(list(o[:5]), up)
for k in ("means3D", "unnorm_rotations", "logit_opacities", "log_scales"):
    print(f"transform d{k}: rel {rel(b[k].grad, a[k].grad):.3e} |g| {float(a[k].grad.norm()):.3e}")
for j, name in enumerate(("means_cam", "rot", "dcol", "opac", "scales")):
    print(f"  forward {name}: rel {rel(o[j], outs[j]):.3e}")
# whole loss
cfg = MappingConfig()
c = leaves()
d = leaves()
ll, _, _ = get_loss_mapping(c, kf, t, cfg, fused=False)
ll.backward()
lf, _, _ = get_loss_mapping(d, kf, t, cfg, fused=True)
lf.backward()
print(f"loss {float(ll):.8f} {float(lf):.8f}")
for k in ("means3D", "unnorm_rotations", "logit_opacities", "log_scales", key):
    print(f"full d{k}: rel {rel(d[k].grad, c[k].grad):.3e}; ratio <f,l>/<l,l> "
          f"{float((d[k].grad.double() * c[k].grad.double()).sum() / (c[k].grad.double() ** 2).sum()):.4f}")
