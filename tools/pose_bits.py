"""Bitwise A/B of the pose-fused tracking path between two libgsr builds (GPU box).

Runs one config-3 GraphTracker frame (graph replays of the fused iteration, pose Adam and best candidate
on the device) and one eager tracking_iteration frame on the library GSR_LIB names, and writes the final
pose, Adam state, best candidate and per-iteration losses to OUT (.npz).  Run it once per library, then
`python tools/pose_bits.py --compare A.npz B.npz` reports whether every array is bitwise equal.

usage: GSR_LIB_AB=1 GSR_LIB=... python tools/pose_bits.py OUT.npz
       python tools/pose_bits.py --compare A.npz B.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out):
    import torch
    from splatam_amd.glue import PoseAdam, tracking_iteration
    from splatam_amd.rasterizer import GaussianRasterizer
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import camera_settings, init_tracking_params, transform_to_frame, \
        transformed_params2depthplussilhouette, transformed_params2rendervar
    from splatam_amd.tracker import GraphTracker
    dev = torch.device("cuda", 0)
    scene = config_scene(3)
    params = init_tracking_params(scene, num_frames=2, device=dev, pose_noise=(0.5, 0.01))
    cam = camera_settings(scene.cam, dev)
    w2c = torch.eye(4, device=dev)
    with torch.no_grad():
        gt = dict(params)
        gt["cam_unnorm_rots"] = torch.zeros_like(params["cam_unnorm_rots"])
        gt["cam_unnorm_rots"][0, 0] = 1.0
        gt["cam_trans"] = torch.zeros_like(params["cam_trans"])
        tg = transform_to_frame(gt, 1, False, False)
        im, _, _ = GaussianRasterizer(cam)(**transformed_params2rendervar(gt, tg))
        ds, _, _ = GaussianRasterizer(cam)(**transformed_params2depthplussilhouette(gt, w2c, tg))
    curr = {"cam": cam, "w2c": w2c, "im": im.clone(), "depth": ds[0:1].clone()}
    res = {}

    def leaves():
        p = dict(params)
        p["cam_unnorm_rots"] = params["cam_unnorm_rots"].detach().clone().requires_grad_(True)
        p["cam_trans"] = params["cam_trans"].detach().clone().requires_grad_(True)
        return p

    p = leaves()
    tr = GraphTracker(p, curr, 1, iters_per_graph=10, warmup_iters=1, fuse_pose=True)
    tr.track_frame(40)
    torch.cuda.synchronize()
    res["graph_q"] = p["cam_unnorm_rots"].detach().cpu().numpy()
    res["graph_t"] = p["cam_trans"].detach().cpu().numpy()
    res["graph_best"] = tr.adam.best.detach().cpu().numpy()
    res["graph_state"] = tr.adam.state.detach().cpu().numpy()
    p = leaves()
    adam = PoseAdam(dev)
    losses = []
    for _ in range(10):
        loss, _ = tracking_iteration(p, curr, 1, tr.cfg, pose_adam=adam)
        loss.backward()
        losses.append(float(loss))
    torch.cuda.synchronize()
    res["eager_q"] = p["cam_unnorm_rots"].detach().cpu().numpy()
    res["eager_t"] = p["cam_trans"].detach().cpu().numpy()
    res["eager_losses"] = np.array(losses, dtype=np.float32)
    np.savez(out, **res)
    print("pose_bits", out, {k: float(np.abs(v).sum()) for k, v in res.items()})


def compare(a, b):
    A, B = np.load(a), np.load(b)
    ok = True
    for k in sorted(A.files):
        eq = A[k].shape == B[k].shape and A[k].tobytes() == B[k].tobytes()
        ok &= eq
        print(f"{k}: {'bitwise equal' if eq else 'DIFFERENT'}")
    print("pose_bits compare:", "all bitwise equal" if ok else "differences")
    return ok


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])
