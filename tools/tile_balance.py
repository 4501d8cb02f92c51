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


def instance_culling(geom, v, W, H, R, P):
    """Per (tile, Gaussian) instance: does any pixel of the tile (of each 4-row
    strip) reach alpha >= 1/255 inside power <= 0?  Same math as the render
    kernels (exp of the conic power, min(0.99, o * G))."""
    rr = geom[:16 * 4 * P].view(torch.float32).reshape(P, 16)
    # render-record form (gsr_common.h): q0 = (x, y, K_AC A, K_AC C), q1 = (K_B B, o, ...)
    k_ac, k_b = -0.5 * 1.4426950408889634, -1.4426950408889634
    x, y, A, C, B, o = rr[:, 0], rr[:, 1], rr[:, 2] / k_ac, rr[:, 3] / k_ac, rr[:, 4] / k_b, rr[:, 5]
    rng = v["ranges"].long()
    T = rng.shape[0]
    gx = (W + 15) // 16
    tile_of = torch.repeat_interleave(torch.arange(T, device=rng.device), (rng[:, 1] - rng[:, 0]).clamp(min=0))
    gid = v["point_list"].long()[:R]
    assert tile_of.numel() == R
    ty, tx = tile_of // gx, tile_of % gx
    ly, lx = torch.meshgrid(torch.arange(16, device=rng.device), torch.arange(16, device=rng.device), indexing="ij")
    any_tile = torch.zeros(R, dtype=torch.bool, device=rng.device)
    blocks_exact, px_ok = [0.0], [0.0]
    strips = torch.zeros(R, 4, dtype=torch.bool, device=rng.device)
    for c0 in range(0, R, 65536):
        sl = slice(c0, min(R, c0 + 65536))
        g = gid[sl]
        px = (tx[sl] * 16)[:, None, None] + lx[None]
        py = (ty[sl] * 16)[:, None, None] + ly[None]
        dx = x[g][:, None, None] - px
        dy = y[g][:, None, None] - py
        pw = -0.5 * (A[g][:, None, None] * dx * dx + C[g][:, None, None] * dy * dy) - B[g][:, None, None] * dx * dy
        al = torch.clamp(o[g][:, None, None] * torch.exp(pw), max=0.99)
        ok = (pw <= 0) & (al >= 1.0 / 255.0) & (px < W) & (py < H)
        strips[sl] = ok.reshape(-1, 4, 64).any(2)
        okb = ok.reshape(-1, 4, 4, 4, 4).permute(0, 1, 3, 2, 4).reshape(-1, 16, 16)  # [inst, block, px]
        blocks_exact[0] += float(okb.any(2).sum())
        px_ok[0] += float(ok.sum())
        any_tile[sl] = strips[sl].any(1)
    # strip_mask (gsr_common.h): the alpha ellipse's axis-aligned box against each strip
    det = A * C - B * B
    kappa = A * C / det
    tau = torch.log(torch.clamp(255.0 * o, min=1.0)) * (1.001 + 4e-6 * kappa) + 1e-3
    hx = torch.sqrt(2 * tau * C / det) * 1.001 + 0.01
    hy = torch.sqrt(2 * tau * A / det) * 1.001 + 0.01
    g = gid
    x0 = (tx * 16).float()
    y0 = (ty * 16).float()
    inx = (x[g] + hx[g] >= x0) & (x[g] - hx[g] <= x0 + 15) & (255.0 * o[g] >= 0.999)
    aabb = torch.stack([inx & (y[g] + hy[g] >= y0 + 4 * w) & (y[g] - hy[g] <= y0 + 4 * w + 3) for w in range(4)], 1)
    # intra-tile wave imbalance of render_bwd: per 128-entry batch the workgroup waits for the
    # wave with the longest strip list (groups of 4), so cost ~ sum over batches of max_w
    lens = (rng[:, 1] - rng[:, 0]).clamp(min=0)
    pos = torch.arange(R, device=rng.device) - rng[tile_of, 0]
    from_back = lens[tile_of] - 1 - pos
    batch = from_back // 128
    nb = int(batch.max()) + 1 if R else 1
    key = tile_of * nb + batch
    cnt = torch.zeros(T * nb, 4, device=rng.device)
    cnt.index_add_(0, key, aabb.float())
    grp = torch.ceil(cnt / 4)
    max_sum, mean_sum = float(grp.max(1).values.sum()), float(grp.mean(1).sum())
    res = {}
    for (sw, sh) in ((16, 4), (8, 8), (16, 8), (8, 16), (16, 16), (8, 4), (4, 4)):
        hits = []
        for oy in range(0, 16, sh):
            for ox in range(0, 16, sw):
                hits.append(inx.new_ones(()) & (x[g] + hx[g] >= x0 + ox) & (x[g] - hx[g] <= x0 + ox + sw - 1) &
                            (y[g] + hy[g] >= y0 + oy) & (y[g] - hy[g] <= y0 + oy + sh - 1) &
                            (255.0 * o[g] >= 0.999))
        hits = torch.stack(hits, 1).float()
        res[f"AABB pass, {sw}x{sh} sub-rects: px-evals/instance"] = float(hits.sum(1).mean() * sw * sh)
    res["bwd wave groups: sum max_w / sum mean_w"] = max_sum / max(mean_sum, 1)
    # per-step cost models: lists per 4x4 block (one 16-lane row each), per 8x4 half-wave,
    # per 8x8 wave; a wave steps max over its sub-lists, 4 entries per step, per 128-batch
    def blocks(bw, bh):
        out = []
        for oy in range(0, 16, bh):
            for ox in range(0, 16, bw):
                out.append((x[g] + hx[g] >= x0 + ox) & (x[g] - hx[g] <= x0 + ox + bw - 1) &
                           (y[g] + hy[g] >= y0 + oy) & (y[g] - hy[g] <= y0 + oy + bh - 1) & (255.0 * o[g] >= 0.999))
        return torch.stack(out, 1).float()
    def steps(bw, bh):
        m = blocks(bw, bh)                                   # [R, nblocks] row-major over the tile
        c = torch.zeros(T * nb, m.shape[1], device=rng.device)
        c.index_add_(0, key, m)
        nbx = 16 // bw
        c = c.reshape(T * nb, 16 // bh, nbx)
        # group sub-blocks into 8x8 waves
        wy, wx = 8 // bh, 8 // bw
        c = c.reshape(T * nb, 2, wy, 2, wx).permute(0, 1, 3, 2, 4).reshape(T * nb, 4, wy * wx)
        return float(torch.ceil(c.max(2).values / 4).sum()), float(torch.ceil(c / 4).sum() / (wy * wx))
    for bw, bh in ((8, 8), (8, 4), (4, 4)):
        st, ideal = steps(bw, bh)
        res[f"wave steps, lists per {bw}x{bh}: total (balanced)"] = st
        res[f"wave steps, lists per {bw}x{bh}: balanced"] = ideal
    res["4x4 blocks with a contributing pixel: px-evals/instance"] = 16 * blocks_exact[0] / R
    res["contributing pixel-pairs/instance"] = px_ok[0] / R
    return {**res,
            "instances contributing (any pixel)": float(any_tile.float().mean()),
            "instances passing strip AABB": float(aabb.any(1).float().mean()),
            "strip pairs passing AABB / all strips": float(aabb.float().mean()),
            "strip pairs contributing / all strips": float(strips.float().mean()),
            "strip pairs / contributing instance": float(strips.float().sum() / any_tile.float().sum().clamp(min=1))}


def main():
    dev = torch.device("cuda:0")
    s = config_scene(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
    params = init_tracking_params(s, 1, dev)
    cam = camera_settings(s.cam, dev)
    with torch.no_grad(), _C.reference_binning():  # every rect instance listed (the statistic is about them)
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
        cull = instance_culling(out[3], v, W, H, R, s.P)
        # gauss_bwd: a lane sums its Gaussian's instance records, RU = 4 per memory round trip;
        # a wave of 64 consecutive Gaussians waits for its longest lane
        per_g = torch.bincount(v["point_list"].long()[:R], minlength=s.P).cpu().numpy()
        pad = (-s.P) % 64
        wv = np.concatenate([per_g, np.zeros(pad, np.int64)]).reshape(-1, 64)
        wave_trips = np.ceil(wv.max(1) / 4.0)
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
    stats("inst/gauss", per_g)
    stats("wave_max", wv.max(1))
    print(f"gauss_bwd record round trips per wave: mean {wave_trips.mean():.2f} "
          f"(balanced {np.ceil(wv.sum(1) / 64 / 4).mean():.2f})")
    for k, val in cull.items():
        print(f"{k:34s} {val:.4f}")


if __name__ == "__main__":
    main()
