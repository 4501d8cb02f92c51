"""Per-workgroup timelines of the render kernels (diagnostics): loads the -DGSR_WGTIME=1 build
(splatam_amd/_build_diag/libgsr_diag.so, `python -c "from splatam_amd import build; build.build_diag()"`),
runs the headline tracking iteration (config 3) through the HIP-graph tracker, and reports for
render_fwd / render_bwd of the last iteration: the kernel span, the distribution of workgroup
durations and start times, and the per-CU sum of workgroup durations (load balance).
Usage: python tools/wgtime.py [--config 3] [--out file.json]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSR_LIB"] = os.environ.get("GSR_LIB") or os.path.join(ROOT, "splatam_amd", "_build_diag", "libgsr_diag.so")
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def table(lib, name, n):
    buf = (ctypes.c_ulonglong * (4 * n))()
    fn = getattr(lib, name)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(buf, n) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).copy()


def summarize(t, khz):
    start, end, hwid, xcc = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64), t[:, 2], t[:, 3] & 0xFFFFFFFF
    t0 = start.min()
    us = lambda x: x / khz * 1e3  # noqa: E731
    dur = us(end - start)
    cu = ((xcc & 0xF) << 8) | (((hwid >> 13) & 0x7) << 5) | (((hwid >> 12) & 1) << 4) | ((hwid >> 8) & 0xF)
    per_cu = {}
    for c, d in zip(cu.tolist(), dur.tolist()):
        per_cu.setdefault(c, []).append(d)
    cu_sum = np.array([sum(v) for v in per_cu.values()])
    cu_cnt = np.array([len(v) for v in per_cu.values()])
    return {"span_us": float(us(end.max() - t0)), "n_workgroups": int(len(t)),
            "dur_us": {q: float(np.quantile(dur, q / 100)) for q in (0, 10, 50, 90, 99, 100)},
            "dur_mean_us": float(dur.mean()),
            "start_us": {q: float(np.quantile(us(start - t0), q / 100)) for q in (0, 50, 90, 100)},
            "end_us": {q: float(np.quantile(us(end - t0), q / 100)) for q in (0, 10, 50, 90, 100)},
            "n_cu": len(per_cu), "wg_per_cu": {int(k): int((cu_cnt == k).sum()) for k in np.unique(cu_cnt)},
            "cu_sum_dur_us": {q: float(np.quantile(cu_sum, q / 100)) for q in (0, 50, 100)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from splatam_amd._lib import lib
    from splatam_amd.rasterizer import GaussianRasterizer
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import camera_settings, init_tracking_params, transform_to_frame, \
        transformed_params2depthplussilhouette, transformed_params2rendervar
    from splatam_amd.tracker import GraphTracker
    dev = torch.device("cuda", 0)
    scene = config_scene(a.config)
    params = init_tracking_params(scene, num_frames=1, device=dev)
    cam = camera_settings(scene.cam, dev)
    w2c = torch.eye(4, device=dev)
    with torch.no_grad():
        gt = dict(params)
        gt["cam_unnorm_rots"] = torch.zeros_like(params["cam_unnorm_rots"])
        gt["cam_unnorm_rots"][0, 0] = 1.0
        gt["cam_trans"] = torch.zeros_like(params["cam_trans"])
        tg = transform_to_frame(gt, 0, False, False)
        im, _, _ = GaussianRasterizer(cam)(**transformed_params2rendervar(gt, tg))
        ds, _, _ = GaussianRasterizer(cam)(**transformed_params2depthplussilhouette(gt, w2c, tg))
    curr = {"cam": cam, "w2c": w2c, "im": im.clone(), "depth": ds[0:1].clone()}
    params["cam_unnorm_rots"].requires_grad_(True)
    params["cam_trans"].requires_grad_(True)
    tr = GraphTracker(params, curr, 0, iters_per_graph=4, fuse_pose=True)
    for _ in range(3):
        tr.run()
    torch.cuda.synchronize()
    n = ((scene.cam.W + 15) // 16) * ((scene.cam.H + 15) // 16)
    khz = 100000  # wall_clock64: 100 MHz on MI300/MI355 (hipDeviceAttributeWallClockRate)
    res = {"config": a.config, "tiles": n}
    raw = {}
    for k, name in (("render_fwd", "gsr_diag_wgtime_fwd"), ("render_bwd", "gsr_diag_wgtime_bwd")):
        raw[k] = table(lib, name, n)
        res[k] = summarize(raw[k], khz)
    if a.out:  # per-tile work measures beside the raw timelines (offline analysis)
        from splatam_amd import _C
        from splatam_amd.glue import track_transform
        from splatam_amd.layout import views
        with torch.no_grad():
            means, rots, dcol, opac, scales = track_transform(params, 0, w2c)
            e = torch.Tensor([])
            out = _C.rasterize_gaussians_dual(cam.bg, means, params["rgb_colors"], dcol, opac, scales, rots, 1.0, e,
                                              cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy,
                                              cam.image_height, cam.image_width, e, 0, cam.campos, False)
            v = views(out[6], out[5], cam.image_width, cam.image_height, out[0])
        np.savez(a.out.replace(".json", ".npz"), fwd=raw["render_fwd"], bwd=raw["render_bwd"],
                 ranges=v["ranges"].cpu().numpy(), n_contrib=v["n_contrib"].cpu().numpy(),
                 masks=v["block_masks"].cpu().numpy(), W=cam.image_width, H=cam.image_height)
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
