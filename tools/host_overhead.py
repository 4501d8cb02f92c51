"""Host-side cost of one tracking step (no device sync inside the step): if the
CPU time per step approaches the wall time per step, the loop is launch-bound."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from splatam_amd.glue import track_transform, tracking_l1  # noqa: E402
from splatam_amd.rasterizer import rasterize_gaussians_dual  # noqa: E402
from splatam_amd.scenes import config_scene  # noqa: E402
from splatam_amd.slam import camera_settings, get_loss_tracking, init_tracking_params  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    s = config_scene(3)
    params = init_tracking_params(s, 1, dev)
    cam = camera_settings(s.cam, dev)
    w2c = torch.eye(4, device=dev)
    curr = {"cam": cam, "w2c": w2c, "im": torch.rand(3, s.cam.H, s.cam.W, device=dev),
            "depth": torch.rand(1, s.cam.H, s.cam.W, device=dev) + 1}
    params["cam_unnorm_rots"].requires_grad_(True)
    params["cam_trans"].requires_grad_(True)
    opt = torch.optim.Adam([params["cam_unnorm_rots"], params["cam_trans"]], lr=1e-3, fused=True)
    acc = {}

    def tick(k, t0):
        t = time.perf_counter()
        acc[k] = acc.get(k, 0.0) + (t - t0)
        return t

    def step(timed):
        t = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        t = tick("zero_grad", t) if timed else t
        means, rots, dcol, opac, scales = track_transform(params, 0, w2c)
        t = tick("transform", t) if timed else t
        m2 = torch.zeros(means.shape[0], 3, device=dev, requires_grad=True)
        im, ds, radius, _ = rasterize_gaussians_dual(means, m2, None, params["rgb_colors"], dcol, opac, scales, rots,
                                                     None, cam)
        t = tick("raster_fwd", t) if timed else t
        loss = tracking_l1(im, ds, curr["im"], curr["depth"])
        t = tick("loss_fwd", t) if timed else t
        loss.backward()
        t = tick("backward", t) if timed else t
        opt.step()
        t = tick("adam", t) if timed else t

    for _ in range(20):
        step(False)
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        step(True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print({k: round(1e6 * v / n, 1) for k, v in acc.items()}, "host us/step", round(1e6 * (t1 - t0) / n, 1),
          "wall us/step", round(1e6 * (t2 - t0) / n, 1))
    # baseline python+torch dispatch cost of trivial ops
    x = torch.zeros(4, device=dev)
    t0 = time.perf_counter()
    for _ in range(1000):
        x.add_(1)
    t1 = time.perf_counter()
    print("torch add_ host us", round((t1 - t0) * 1e3, 2))


if __name__ == "__main__":
    main()
