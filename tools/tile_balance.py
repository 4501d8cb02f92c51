"""Diagnostic: per-tile work distribution of the bench frame (config 3).

Prints list length per tile and the backward's per-tile trip count
(max n_contrib over the tile's pixels), to judge how far the slowest tile
sets the render kernels' duration when every tile is resident at once."""
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


def stats(name, a):
    q = np.percentile(a, [50, 90, 99])
    print(f"{name:10s} mean {a.mean():8.1f} p50 {q[0]:8.1f} p90 {q[1]:8.1f} p99 {q[2]:8.1f} max {a.max():8d} "
          f"max/mean {a.max() / max(a.mean(), 1e-9):5.2f}")


def main():
    dev = torch.device("cuda:0")
    s = config_scene(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
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
    tiles = ncp.reshape(gy, 16, gx, 16).transpose(0, 2, 1, 3).reshape(gx * gy, 256)
    length = rng[:, 1] - rng[:, 0]
    bmax = tiles.max(1)
    print(f"num_rendered {R} tiles {gx * gy} gaussians {s.P}")
    stats("list_len", length)
    stats("bwd_trip", bmax)
    stats("px_contrib", nc.reshape(-1))
    order = np.sort(bmax)[::-1]
    print("top-16 bwd trip counts", order[:16].tolist())
    print("trip/list ratio mean", float((bmax / np.maximum(length, 1)).mean()))


if __name__ == "__main__":
    main()
