"""Rasterizer-only microbenchmark (no SplaTAM glue): K x (RGB fwd+bwd, depth/silhouette
fwd+bwd) on one synthetic config; prints per-stage hipEvent timings as JSON.
Used for kernel iteration and for rocprofv3 PMC passes."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from splatam_amd import profiling  # noqa: E402
from splatam_amd.rasterizer import GaussianRasterizer, rasterize_gaussians, rasterize_gaussians_dual  # noqa: E402
from splatam_amd.scenes import config_scene  # noqa: E402
from splatam_amd.slam import camera_settings  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=("dual_lean", "dual", "single", "power"), default="dual_lean",
                    help="dual_lean: one dual rasterization, grads for means3D + depth colours only, depth "
                         "channel of the second image differentiated (tracking)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    s = config_scene(a.config)
    cam = camera_settings(s.cam, dev)
    m3 = s.means3D.to(dev).requires_grad_(True)
    sc = s.scales.to(dev)
    ro = s.rotations.to(dev)
    op = s.opacities.to(dev)
    col = s.colors.to(dev)
    ds = torch.cat([m3.detach()[:, 2:3], torch.ones_like(m3[:, :1]), m3.detach()[:, 2:3] ** 2], 1)
    g = torch.randn(3, s.cam.H, s.cam.W, device=dev)
    g2 = g.clone()
    lean = a.mode == "dual_lean"
    if lean:
        g2[1:] = 0
    ras = GaussianRasterizer(cam)

    full = a.mode != "dual_lean"
    op.requires_grad_(full)
    col.requires_grad_(full)
    ds.requires_grad_(True)

    def it():
        if a.mode == "power":  # drop-in backward_power=2 (hessian_diff_gaussian_rasterization_w_depth)
            m2 = torch.zeros_like(m3, requires_grad=True)
            im, _, _ = rasterize_gaussians(m3, m2, torch.Tensor([]), col, op, sc, ro, torch.Tensor([]), cam, 2)
            im.backward(g)
        elif a.mode == "single":
            for c in (col, ds):
                m2 = torch.zeros_like(m3, requires_grad=True)
                im, _, _ = ras(means3D=m3, means2D=m2, opacities=op, colors_precomp=c, scales=sc, rotations=ro)
                im.backward(g)
        else:
            m2 = torch.zeros_like(m3, requires_grad=full)
            im, im2, _, _ = rasterize_gaussians_dual(m3, m2, None, col, ds, op, sc, ro, None, cam,
                                                     grad2_channels=1 if lean else 3)
            torch.autograd.backward([im, im2], [g, g2])

    for _ in range(a.warmup):
        it()
    torch.cuda.synchronize()
    profiling.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(a.iters):
        it()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    st = profiling.read_timing()
    print(json.dumps({"frames_per_s": a.iters / t, "ms_per_frame": 1000 * t / a.iters,
                      "stages_us": {k: round(v["avg_us"], 2) for k, v in st.items()}}))


if __name__ == "__main__":
    main()
