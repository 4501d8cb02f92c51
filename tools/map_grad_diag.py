"""Config-4 mapping gradient diagnostics: the literal get_loss(mapping=True) gradients against the eager fused
iteration (get_loss_mapping fused=True, autograd .grad) and the captured frame's first-step Adam moments."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from splatam_amd.mapper import GAUSS_KEYS, GraphMapper
from splatam_amd.scenes import config_scene, make_scene
from splatam_amd.slam import MappingConfig, as_parameters, color_key, get_loss_mapping, map_frame_literal, \
    tracking_variables
from splatam_amd.workloads import mapping_workload

cfg_id = int(sys.argv[1]) if len(sys.argv) > 1 else 4
prune = sys.argv[2] == "1" if len(sys.argv) > 2 else True
dev = torch.device("cuda:0")
scene = config_scene(4) if cfg_id == 4 else make_scene(20000, 320, 240, seed=7, anisotropic=True, sh_degree=3)
params, cam, kfs = mapping_workload(scene, 4, dev, prunable=0.02 if prune else 0.0)
key = color_key(params)
P0 = params["means3D"].shape[0]
r = torch.max(kfs[0]["depth"]) / 3.0
cfg = MappingConfig(prune_gaussians=prune)
kf = kfs[1]

# literal, no pruning involved: iteration on the unpruned map
lit = as_parameters(params)
loss_l, _, _ = get_loss_mapping(lit, kf, kf["id"], cfg, fused=False)
loss_l.backward()
# eager fused (autograd)
fz = {k: (v.clone().requires_grad_(True) if k in GAUSS_KEYS + (key,) else v.clone()) for k, v in params.items()}
loss_f, _, _ = get_loss_mapping(fz, kf, kf["id"], cfg, fused=True)
loss_f.backward()
print(f"P {P0} loss literal {float(loss_l):.7f} fused {float(loss_f):.7f}")
for k in GAUSS_KEYS + (key,):
    gl, gf = lit[k].grad.double(), fz[k].grad.double()
    d = (gf - gl)
    rows = d.reshape(d.shape[0], -1).norm(dim=1)
    top = torch.topk(rows, 5)
    print(f"  d{k}: fused vs literal rel L2 {float(d.norm() / gl.norm()):.3e}; |g| {float(gl.norm()):.3e}; "
          f"worst rows {top.indices.tolist()} err {[round(float(x), 6) for x in top.values]} "
          f"|g_row| {[round(float(gl.reshape(gl.shape[0], -1)[i].norm()), 6) for i in top.indices]}")
