"""Per-iteration tracking losses / poses at config 3: the literal loop (track_frame_literal), the eager fused
loop (get_loss_tracking default + torch Adam) and GraphTracker replayed one iteration at a time (diagnostics)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from splatam_amd.scenes import config_scene
from splatam_amd.slam import TrackingConfig, as_parameters, get_loss_tracking, track_frame_literal, tracking_variables
from splatam_amd.tracker import GraphTracker
from splatam_amd.workloads import tracking_frame

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda:0")
params, curr = tracking_frame(config_scene(3), dev)


def pose_leaves(p0):
    p = dict(p0)
    p["cam_unnorm_rots"] = p0["cam_unnorm_rots"].detach().clone().requires_grad_(True)
    p["cam_trans"] = p0["cam_trans"].detach().clone().requires_grad_(True)
    return p


lit = as_parameters(params)
ll = []
track_frame_literal(lit, tracking_variables(params["means3D"].shape[0], dev), curr, 0, N, losses_out=ll)
ll = [float(x) for x in ll]

pe = pose_leaves(params)
opt = torch.optim.Adam([{"params": [pe["cam_unnorm_rots"]], "lr": 0.0004}, {"params": [pe["cam_trans"]], "lr": 0.002}])
le, pose_e = [], []
for _ in range(N):
    opt.zero_grad(set_to_none=True)
    loss, _, _ = get_loss_tracking(pe, curr, 0)
    loss.backward()
    opt.step()
    le.append(float(loss))
    pose_e.append(torch.cat([pe["cam_unnorm_rots"][0, :, 0], pe["cam_trans"][0, :, 0]]).detach().clone())

pg = pose_leaves(params)
tr = GraphTracker(pg, curr, 0, iters_per_graph=1, warmup_iters=1, fuse_pose=True)
tr.begin_frame()
lg, pose_g = [], []
for _ in range(N):
    tr.run()
    torch.cuda.synchronize()
    lg.append(float(tr.loss))
    pose_g.append(torch.cat([pg["cam_unnorm_rots"][0, :, 0], pg["cam_trans"][0, :, 0]]).detach().clone())
for k in range(N):
    print(f"{k:3d} literal {ll[k]:14.4f} eager_fused {le[k]:14.4f} ({(le[k]-ll[k])/ll[k]:+.2e}) graph {lg[k]:14.4f} "
          f"({(lg[k]-ll[k])/ll[k]:+.2e})  |pose_g - pose_e| {float((pose_g[k]-pose_e[k]).abs().max()):.2e}")
print("best", min(ll), min(le), min(lg))
