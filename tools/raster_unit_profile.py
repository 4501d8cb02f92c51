"""Host / device split of SURVEY 8(d)'s unit through the unchanged-caller API (bench.py's
`dropin.raster_unit`): 2 x diff_gaussian_rasterization.GaussianRasterizer (RGB, depth/silhouette)
+ backward from Python, eager, every input a leaf requiring grad.

Prints, per unit: wall time; host time spent in each phase (first forward incl. its host sync,
second forward incl. the geometry-reuse comparison, loss, backward); the device time of every kernel
(torch.profiler) and the device-idle remainder; the wall time of the same unit over a 1000-Gaussian scene at
the same image size (the host floor: the same Python, marshalling, allocations and launches with almost no
device work); and the top Python functions of that tiny-scene unit (cProfile, tottime).
Usage: python tools/raster_unit_profile.py [--n 200] [--config 3] [--out file.txt]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import diff_gaussian_rasterization as dgr
    from splatam_amd import _C
    from splatam_amd.scenes import config_scene, make_scene
    from splatam_amd.slam import camera_settings, init_tracking_params, transform_to_frame, \
        transformed_params2depthplussilhouette, transformed_params2rendervar
    dev = torch.device("cuda", 0)
    scene = config_scene(a.config)
    W, H = scene.cam.W, scene.cam.H
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
    g1 = torch.randn(3, H, W, device=dev)
    g2 = torch.randn(3, H, W, device=dev)
    R = dgr.GaussianRasterizer
    acc = {}

    def tick(k, t0):
        t = time.perf_counter()
        acc[k] = acc.get(k, 0.0) + (t - t0)
        return t

    def unit(timed=False):
        t = time.perf_counter()
        for d in (rv1, rv2):
            for v in d.values():
                v.grad = None
        t = tick("zero_grads", t) if timed else t
        im_, _, _ = R(cam)(**rv1)
        t = tick("forward_rgb", t) if timed else t
        ds_, _, _ = R(cam)(**rv2)
        t = tick("forward_depth", t) if timed else t
        loss = (im_ * g1).sum() + (ds_ * g2).sum()
        t = tick("loss", t) if timed else t
        loss.backward()
        tick("backward", t) if timed else t

    for _ in range(10):
        unit()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.n):
        unit(True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(20):
            unit()
        torch.cuda.synchronize()
    kern = {}
    for e in prof.key_averages():
        if e.self_device_time_total > 0:
            kern[e.key] = (e.self_device_time_total / 20, e.count / 20)
    dev_us = sum(v[0] for v in kern.values())
    lines = [f"config {a.config}: unit wall {1e6 * (t2 - t0) / a.n:.1f} us, host (loop, no final sync) "
             f"{1e6 * (t1 - t0) / a.n:.1f} us, device busy {dev_us:.1f} us per unit",
             "host per phase (us/unit): " + ", ".join(f"{k} {1e6 * v / a.n:.1f}" for k, v in acc.items()),
             f"geometry reuse: {_C.reuse_stats()}",
             "device per unit (us, launches):"]
    for k, (us, c) in sorted(kern.items(), key=lambda kv: -kv[1][0]):
        lines.append(f"  {us:8.1f}  x{c:4.1f}  {k[:110]}")
    lines.append(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30))
    # host floor: the same unit over 1000 Gaussians (same image size, same calls and allocations)
    tiny = make_scene(1000, W, H, seed=3)
    tp = init_tracking_params(tiny, num_frames=1, device=dev)
    with torch.no_grad():
        ttg = transform_to_frame(tp, 0, False, False)
        trv1 = leaf(transformed_params2rendervar(tp, ttg))
        trv2 = leaf(transformed_params2depthplussilhouette(tp, w2c, ttg))
    trv2["means3D"] = trv1["means3D"]
    rv1, rv2 = trv1, trv2  # unit() reads these names
    for _ in range(10):
        unit()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    for _ in range(a.n):
        unit()
    torch.cuda.synchronize()
    floor_us = 1e6 * (time.perf_counter() - t3) / a.n
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(100):
        unit()
    torch.cuda.synchronize()
    pr.disable()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
    lines.append(f"host floor (1000 Gaussians, {W}x{H}): unit wall {floor_us:.1f} us; cProfile of 100 such units:")
    lines.append(buf.getvalue())
    # host cost per call (tiny scene): the binding's backward without the autograd engine, the bare C call
    # with pre-built arguments, and the forward (which waits for num_rendered like the reference)
    from splatam_amd._lib import ALLOC_FN, GsrGrads, lib  # noqa: F401
    s_ = cam
    with torch.no_grad():
        args = (s_.bg, trv1["means3D"], trv1["colors_precomp"], trv1["opacities"], trv1["scales"],
                trv1["rotations"], s_.scale_modifier, torch.Tensor([]), s_.viewmatrix, s_.projmatrix, s_.tanfovx,
                s_.tanfovy, s_.image_height, s_.image_width, torch.Tensor([]), s_.sh_degree, s_.campos,
                s_.prefiltered)
        nr, color, radii, gb, bb, ib, depth = _C.rasterize_gaussians(*args)
        torch.cuda.synchronize()
        k = 500
        t = time.perf_counter()
        for _ in range(k):
            _C.rasterize_gaussians(*args)
        fwd_us = 1e6 * (time.perf_counter() - t) / k
        torch.cuda.synchronize()
        bargs = (s_.bg, trv1["means3D"], radii, trv1["colors_precomp"], trv1["scales"], trv1["rotations"],
                 s_.scale_modifier, torch.Tensor([]), s_.viewmatrix, s_.projmatrix, s_.tanfovx, s_.tanfovy, g1,
                 torch.Tensor([]), s_.sh_degree, s_.campos, gb, nr, bb, ib)
        t = time.perf_counter()
        for _ in range(k):
            _C.rasterize_gaussians_backward(*bargs)
        bwd_host_us = 1e6 * (time.perf_counter() - t) / k
        torch.cuda.synchronize()
        t = time.perf_counter()
        torch.cuda.synchronize()
        sync_us = 1e6 * (time.perf_counter() - t)
    lines.append(f"host cost per call (1000 Gaussians): forward {fwd_us:.1f} us (incl. its wait for num_rendered), "
                 f"backward binding {bwd_host_us:.1f} us (host only, no sync), idle synchronize {sync_us:.1f} us")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
