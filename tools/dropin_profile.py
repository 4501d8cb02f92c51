"""Host/device profile of the unchanged-caller tracking iteration (bench.py's `dropin` leg):
torch.profiler over a few iterations of scripts/splatam.py's loop body through
diff_gaussian_rasterization.GaussianRasterizer, printing the top host-side ops and the wall time
per iteration.  Usage: python tools/dropin_profile.py [--iters 20] [--out file.txt]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import diff_gaussian_rasterization as dgr
    from splatam_amd.rasterizer import GaussianRasterizer
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import as_parameters, camera_settings, init_tracking_params, track_frame_literal, \
        tracking_variables, transform_to_frame, transformed_params2depthplussilhouette, transformed_params2rendervar
    dev = torch.device("cuda", 0)
    scene = config_scene(a.config)
    base = init_tracking_params(scene, num_frames=2, device=dev)
    cam = camera_settings(scene.cam, dev)
    w2c = torch.eye(4, device=dev)
    with torch.no_grad():
        tg = transform_to_frame(base, 0, False, False)
        im, _, _ = GaussianRasterizer(cam)(**transformed_params2rendervar(base, tg))
        ds, _, _ = GaussianRasterizer(cam)(**transformed_params2depthplussilhouette(base, w2c, tg))
    curr = {"cam": cam, "w2c": w2c, "im": im.clone(), "depth": ds[0:1].clone()}
    params = as_parameters(base)
    variables = tracking_variables(scene.P, dev)
    R = dgr.GaussianRasterizer
    track_frame_literal(params, variables, curr, 1, 5, renderer=R)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    track_frame_literal(params, variables, curr, 1, a.iters, renderer=R)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.iters
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        track_frame_literal(params, variables, curr, 1, a.iters, renderer=R)
        torch.cuda.synchronize()
    dev_us = sum(e.self_device_time_total for e in prof.key_averages()) / a.iters
    ours = sum(e.self_device_time_total for e in prof.key_averages() if "gsr::" in e.key or "rocclr_copy" in e.key)
    lines = [f"wall per iteration (no profiler): {wall * 1e3:.3f} ms  (GSR_GEOM_CACHE={os.environ.get('GSR_GEOM_CACHE', '0')})",
             f"device time per iteration: {dev_us:.1f} us (all kernels), {ours / a.iters:.1f} us (libgsr kernels + copies)",
             prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40),
             prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=25)]
    from splatam_amd import _C
    lines.insert(2, f"geometry reuse: {_C.REUSE_STATS}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
