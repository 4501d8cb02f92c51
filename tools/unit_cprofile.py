"""Python-level host profile (cProfile) of SURVEY 8(d)'s unit through the unchanged-caller API (bench.py
dropin.raster_unit): where the host time of 2 x GaussianRasterizer + backward goes.
Usage: python tools/unit_cprofile.py [--n 300]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--no-profile", action="store_true")
    a = ap.parse_args()
    import diff_gaussian_rasterization as dgr
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import camera_settings, init_tracking_params, transform_to_frame, \
        transformed_params2depthplussilhouette, transformed_params2rendervar
    dev = torch.device("cuda", 0)
    scene = config_scene(3)
    params = init_tracking_params(scene, num_frames=1, device=dev)
    cam = camera_settings(scene.cam, dev)
    w2c = torch.eye(4, device=dev)
    with torch.no_grad():
        tg = transform_to_frame(params, 0, False, False)
        rv1 = transformed_params2rendervar(params, tg)
        rv2 = transformed_params2depthplussilhouette(params, w2c, tg)
    leaf = lambda d: {k: v.detach().clone().requires_grad_(True) for k, v in d.items()}  # noqa: E731
    rv1, rv2 = leaf(rv1), leaf(rv2)
    rv2["means3D"] = rv1["means3D"]
    g1 = torch.randn(3, scene.cam.H, scene.cam.W, device=dev)
    g2 = torch.randn(3, scene.cam.H, scene.cam.W, device=dev)
    R = dgr.GaussianRasterizer

    def unit():
        for d in (rv1, rv2):
            for v in d.values():
                v.grad = None
        im_, _, _ = R(cam)(**rv1)
        ds_, _, _ = R(cam)(**rv2)
        ((im_ * g1).sum() + (ds_ * g2).sum()).backward()

    for _ in range(10):
        unit()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.n):
        unit()
    torch.cuda.synchronize()
    print(f"unit {1e3 * (time.perf_counter() - t0) / a.n:.4f} ms (no profiler)")
    if a.no_profile:
        return
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.n):
        unit()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
