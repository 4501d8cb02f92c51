"""Diagnostic: how much of each tile list lies behind every pixel's last contributor (the instances
render_bwd zeroes in its prologue: a gather of the instance's render record to find its slot, and one
record store each), per config, with the default tile culling.

usage: python tools/dead_tail.py [config ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from splatam_amd import _C  # noqa: E402
from splatam_amd.layout import views  # noqa: E402
from splatam_amd.scenes import config_scene  # noqa: E402
from splatam_amd.slam import camera_settings, init_tracking_params, transform_to_frame, \
    transformed_params2rendervar  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for cfg in [int(a) for a in sys.argv[1:]] or [3, 4]:
        s = config_scene(cfg)
        params = init_tracking_params(s, 1, dev)
        cam = camera_settings(s.cam, dev)
        with torch.no_grad():
            tg = transform_to_frame(params, 0, False, False)
            rv = transformed_params2rendervar(params, tg)
            W, H = s.cam.W, s.cam.H
            out = _C.rasterize_gaussians(cam.bg, rv["means3D"], rv["colors_precomp"], rv["opacities"], rv["scales"],
                                         rv["rotations"], cam.scale_modifier, torch.Tensor([]), cam.viewmatrix,
                                         cam.projmatrix, cam.tanfovx, cam.tanfovy, H, W, torch.Tensor([]),
                                         cam.sh_degree, cam.campos, cam.prefiltered)
            R, img, bin_ = out[0], out[5], out[4]
            v = views(img, bin_, W, H, R)
            torch.cuda.synchronize()
            rng = v["ranges"].cpu().numpy().astype(np.int64)
            nc = v["n_contrib"].cpu().numpy().reshape(H, W).astype(np.int64)
        gx, gy = (W + 15) // 16, (H + 15) // 16
        ncp = np.zeros((gy * 16, gx * 16), np.int64)
        ncp[:H, :W] = nc
        bmax = ncp.reshape(gy, 16, gx, 16).transpose(0, 2, 1, 3).reshape(gx * gy, 256).max(1)
        length = rng[:, 1] - rng[:, 0]
        dead = np.maximum(length - bmax, 0)
        print(f"config {cfg}: {W}x{H}, P {s.P}, listed instances {int(length.sum())}, behind every pixel's last "
              f"contributor {int(dead.sum())} ({dead.sum() / max(length.sum(), 1):.3f}); tiles with a dead tail "
              f"{int((dead > 0).sum())} of {gx * gy}; longest dead tail {int(dead.max())}", flush=True)


if __name__ == "__main__":
    main()
