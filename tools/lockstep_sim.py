"""CPU estimate of render_bwd's row-list lockstep padding (no GPU needed; the GPU-side counterpart reading the
kernel's own masks is tools/lockstep_stats.py).

From the float32 oracle's binning of a BASELINE config (sorted tile lists, 2D means / conics / opacities,
per-pixel last contributors) each (tile, Gaussian) entry gets the set of 4x4-pixel blocks holding a pixel
with alpha >= 1/255 (the exact per-pixel test, a subset of the kernel's conservative ellipse mask); the
lists are trimmed at each block's last contributor like render_bwd's.  Reported, in wave-steps of four
entries per row, for batches of B entries:
  fixed        wave w walks the four blocks of its 8x8 quadrant (the kernel's assignment)
  tile_sorted  blocks dealt to waves by their whole-tile list length, four per wave (one assignment per tile)
  batch_sorted the same per batch (the bound of re-dealing every batch)
  alone        no lockstep (each row its own steps: the lower bound)
usage: python tools/lockstep_sim.py [config] [batch]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import oracle as orc  # noqa: E402
from splatam_amd.scenes import config_scene  # noqa: E402


def block_of_pixel():
    tid = np.arange(256)
    px = 8 * ((tid >> 6) & 1) + 4 * ((tid >> 4) & 1) + (tid & 3)
    py = 8 * (tid >> 7) + 4 * ((tid >> 5) & 1) + ((tid >> 2) & 3)
    return px, py, tid >> 4  # block b = 4 * wave + row


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    s = config_scene(cfg)
    c = s.cam
    fr = orc.forward(s.means3D.numpy(), s.opacities.numpy(), colors=s.colors.numpy(), scales=s.scales.numpy(),
                     rotations=s.rotations.numpy(), view=c.viewmatrix.numpy(), proj=c.projmatrix.numpy(),
                     campos=c.campos.numpy(), tanfovx=c.tanfovx, tanfovy=c.tanfovy, H=c.H, W=c.W)
    W, H = c.W, c.H
    gx, gy = (W + 15) // 16, (H + 15) // 16
    px, py, blk = block_of_pixel()
    m2, co, pl = fr.means2D.astype(np.float64), fr.conic_opacity.astype(np.float64), fr.point_list
    tot = dict(fixed=0, tile_sorted=0, batch_sorted=0, alone=0.0)
    entries = 0
    for t in range(gx * gy):
        a, b = fr.ranges[t]
        if b <= a:
            continue
        tx, ty = t % gx, t // gx
        X, Y = tx * 16 + px, ty * 16 + py
        inside = (X < W) & (Y < H)
        last = np.where(inside, fr.n_contrib[np.minimum(Y, H - 1), np.minimum(X, W - 1)], 0)
        rm = np.zeros(16, np.int64)
        np.maximum.at(rm, blk, last)
        ids = pl[a:b]
        dx = m2[ids, 0][:, None] - X[None, :]
        dy = m2[ids, 1][:, None] - Y[None, :]
        A, Bc, C, o = co[ids, 0][:, None], co[ids, 1][:, None], co[ids, 2][:, None], co[ids, 3][:, None]
        power = -0.5 * (A * dx * dx + C * dy * dy) - Bc * dx * dy
        alpha = np.minimum(0.99, o * np.exp(np.minimum(power, 0.0)))
        hit = (power <= 0) & (alpha >= 1.0 / 255.0) & inside[None, :]
        bits = np.zeros((b - a, 16), bool)
        for k in range(16):
            bits[:, k] = hit[:, blk == k].any(axis=1)
        pos = np.arange(b - a)
        bits &= pos[:, None] < rm[None, :]
        order = np.argsort(-bits.sum(0), kind="stable")
        bmax = int(rm.max())
        for hi in range(bmax, 0, -B):
            lo = max(0, hi - B)
            n = bits[lo:hi].sum(0)
            g = (n + 3) // 4
            entries += int(n.sum())
            tot["fixed"] += int(sum(g[4 * w:4 * w + 4].max() for w in range(4)))
            tot["tile_sorted"] += int(sum(g[order[4 * w:4 * w + 4]].max() for w in range(4)))
            gs = np.sort(g)[::-1]
            tot["batch_sorted"] += int(sum(gs[4 * w:4 * w + 4].max() for w in range(4)))
            tot["alone"] += float(g.sum()) / 4
    print(f"config {cfg}: num_rendered {fr.num_rendered}, batch {B}, listed (block, entry) items {entries} "
          f"({entries * 16 / max(fr.num_rendered, 1):.1f} pixel-pair evaluations per instance)")
    for k, v in tot.items():
        print(f"  wave-steps {k:13s} {v:12.0f}  ({v / tot['alone']:.3f} x no lockstep)")


if __name__ == "__main__":
    main()
