"""Diagnostic: lockstep padding of render_bwd's per-row lists (config 3 bench frame).

Each wave of render_bwd walks the lists of its four 4x4-pixel blocks (one per
16-lane row) in lockstep, 4 entries per step, per 64-entry batch, so a wave pays
max over its rows of ceil(n_row / 4) steps per batch.  This tool reads the exact
block masks render_fwd writes into point_list and the per-pixel last contributor
(n_contrib), applies the same trimming as the kernel (entries behind a block's
last contributor are dropped), and reports the step count for
  * the fixed assignment (wave w owns the 8x8 quadrant w: blocks 4w..4w+3),
  * blocks dealt to waves by their whole-tile list length (sorted, 4 per wave),
  * no lockstep at all (each row alone; the lower bound).
"""
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


def tid_block():
    tid = np.arange(256)
    px = 8 * ((tid >> 6) & 1) + 4 * ((tid >> 4) & 1) + (tid & 3)
    py = 8 * (tid >> 7) + 4 * ((tid >> 5) & 1) + ((tid >> 2) & 3)
    return px, py, (tid >> 4)  # block = 4 * wave + row


def main():
    dev = torch.device("cuda:0")
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    BB = int(sys.argv[2]) if len(sys.argv) > 2 else 64
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
        masks = v["block_masks"].cpu().numpy().astype(np.int64) & 0xFFFF
    gx, gy = (W + 15) // 16, (H + 15) // 16
    px, py, blk = tid_block()
    tot = {"fixed": 0, "sorted": 0, "alone": 0, "sorted_batch": 0}
    entries = 0
    for t in range(gx * gy):
        tx, ty = t % gx, t // gx
        a, b = rng[t]
        if b <= a:
            continue
        X, Y = tx * 16 + px, ty * 16 + py
        inside = (X < W) & (Y < H)
        last = np.where(inside, nc[np.minimum(Y, H - 1), np.minimum(X, W - 1)], 0)
        rm = np.zeros(16, np.int64)
        np.maximum.at(rm, blk, last)
        bmax = int(rm.max())
        m = masks[a:b]
        bits = ((m[:, None] >> np.arange(16)[None]) & 1).astype(bool)  # [pos, block]
        pos = np.arange(b - a)
        bits &= pos[:, None] < rm[None]
        per_block_total = bits.sum(0)
        order = np.argsort(-per_block_total, kind="stable")
        for hi in range(bmax, 0, -BB):
            lo = max(0, hi - BB)
            n = bits[lo:hi].sum(0)  # [16]
            g = (n + 3) // 4
            entries += int(n.sum())
            tot["fixed"] += int(sum(g[4 * w:4 * w + 4].max() for w in range(4)))
            tot["sorted"] += int(sum(g[order[4 * w:4 * w + 4]].max() for w in range(4)))
            gs = np.sort(g)[::-1]
            tot["sorted_batch"] += int(sum(gs[4 * w:4 * w + 4].max() for w in range(4)))
            tot["alone"] += float(g.sum()) / 4
    print(f"config {cfg}: num_rendered {R}, batch {BB}, block-entries {entries} "
          f"({entries * 16 / max(R, 1):.1f} px-evals/instance)")
    for k, val in tot.items():
        print(f"  wave steps {k:13s} {val:12.0f}  ({val / tot['alone']:.3f} x no-lockstep)")


if __name__ == "__main__":
    main()
