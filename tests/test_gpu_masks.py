"""The 4x4-block masks render_fwd writes into the sorted tile lists (render_bwd and the Fisher kernel walk
only the blocks a mask names): conservative and tight.

* conservative: every block holding a pixel where the Gaussian blends (alpha >= 1/255 and power <= 0,
  forward.cu:341-351, evaluated in float64 on the oracle's 2D means / conics with a 1 % alpha margin) has
  its bit set -- a missing bit would silently drop gradient terms;
* tight: the masks name at most 1 % more (instance, block) pairs than the exact ellipse-vs-block test
  restated here in float64 (the kernel's float32 evaluation adds small margins) -- a looser mask costs
  walk steps without changing a result, so the parity tests cannot see it (a shift bug once set garbage
  bits and made render_bwd 11 % slower with every parity test green)."""
import numpy as np
import pytest
import torch

from oracle import oracle as orc
from splatam_amd.scenes import config_scene, make_scene

pytestmark = pytest.mark.gpu


def _block_of_pixel():
    tid = np.arange(256)
    px = 8 * ((tid >> 6) & 1) + 4 * ((tid >> 4) & 1) + (tid & 3)
    py = 8 * (tid >> 7) + 4 * ((tid >> 5) & 1) + ((tid >> 2) & 3)
    return px, py, tid >> 4


def _exact_masks(m2, co, W, H, tx, ty):
    """float64 ellipse-vs-block masks (the kernel's construction without its margins): the alpha >= 1/255
    ellipse's x-extent over each block row's y-span against the block columns' pixel-centre spans."""
    ax, ay = m2[:, 0], m2[:, 1]
    A, B, C, o = co[:, 0], co[:, 1], co[:, 2], co[:, 3]
    det = A * C - B * B
    tau = np.log(np.maximum(255.0 * o, 1e-30))
    out = np.zeros(len(ax), np.int64)
    ok = (det > 0) & (A > 0) & (tau > 0)
    x0, y0 = 16.0 * tx, 16.0 * ty
    with np.errstate(invalid="ignore", divide="ignore"):
        hy = np.sqrt(2 * tau * A / det)
        us = B * np.sqrt(2 * tau / (det * C))
        for r in range(4):
            lo = np.maximum(y0 + 4 * r - ay, -hy)
            hi = np.minimum(y0 + 4 * r + 3 - ay, hy)
            row = lo <= hi
            ul = np.clip(us, lo, hi)
            ur = np.clip(-us, lo, hi)
            wl = np.sqrt(np.maximum(2 * tau * A - det * ul * ul, 0))
            wr = np.sqrt(np.maximum(2 * tau * A - det * ur * ur, 0))
            xmin = ax + (-B * ul - wl) / A
            xmax = ax + (-B * ur + wr) / A
            for c in range(4):
                hit = ok & row & (xmax >= x0 + 4 * c) & (xmin <= x0 + 4 * c + 3)
                bit = 4 * (2 * (r >> 1) + (c >> 1)) + 2 * (r & 1) + (c & 1)
                out |= hit.astype(np.int64) << bit
    return out


@pytest.mark.parametrize("which", ["config1", "aniso"])
def test_block_masks_conservative_and_tight(cuda, which):
    from splatam_amd import _C
    from splatam_amd.layout import views
    s = config_scene(1) if which == "config1" else make_scene(6000, 192, 144, seed=5, anisotropic=True)
    c = s.cam
    e = torch.Tensor([])
    with _C.reference_binning():  # the oracle's lists, entry for entry
        out = _C.rasterize_gaussians(torch.zeros(3, device=cuda), s.means3D.to(cuda), s.colors.to(cuda),
                                     s.opacities.to(cuda), s.scales.to(cuda), s.rotations.to(cuda), 1.0, e,
                                     c.viewmatrix.to(cuda), c.projmatrix.to(cuda), c.tanfovx, c.tanfovy, c.H, c.W,
                                     e, 0, c.campos.to(cuda), False)
    n, img, binning = out[0], out[5], out[4]
    v = views(img, binning, c.W, c.H, n)
    torch.cuda.synchronize()
    masks = v["block_masks"].cpu().numpy().astype(np.int64) & 0xFFFF
    fr = orc.forward(s.means3D.numpy(), s.opacities.numpy(), colors=s.colors.numpy(), scales=s.scales.numpy(),
                     rotations=s.rotations.numpy(), view=c.viewmatrix.numpy(), proj=c.projmatrix.numpy(),
                     campos=c.campos.numpy(), tanfovx=c.tanfovx, tanfovy=c.tanfovy, H=c.H, W=c.W)
    assert n == fr.num_rendered
    np.testing.assert_array_equal(v["point_list"].cpu().numpy().astype(np.int64) & 0xFFFFFFFF, fr.point_list)
    gx = (c.W + 15) // 16
    px, py, blk = _block_of_pixel()
    m2, co = fr.means2D.astype(np.float64), fr.conic_opacity.astype(np.float64)
    # the forward stages (and masks) every entry of a tile only until all its pixels terminate: compare the
    # entries up to each tile's longest n_contrib (the rest may be unmasked)
    missing = listed = exact_bits = 0
    for t in range(len(fr.ranges)):
        a, b = fr.ranges[t]
        if b <= a:
            continue
        tx, ty = t % gx, t // gx
        X, Y = tx * 16 + px, ty * 16 + py
        inside = (X < c.W) & (Y < c.H)
        last = int(np.where(inside, fr.n_contrib[np.minimum(Y, c.H - 1), np.minimum(X, c.W - 1)], 0).max())
        if last == 0:
            continue
        ids = fr.point_list[a:a + last]
        got = masks[a:a + last]
        dx = m2[ids, 0][:, None] - X[None, :]
        dy = m2[ids, 1][:, None] - Y[None, :]
        A, B, C, o = (co[ids, k][:, None] for k in range(4))
        power = -0.5 * (A * dx * dx + C * dy * dy) - B * dx * dy
        alpha = o * np.exp(np.minimum(power, 0.0))
        hit = (power <= 0) & (alpha >= 1.01 / 255.0) & inside[None, :]
        need = np.zeros(len(ids), np.int64)
        for k in range(16):
            need |= hit[:, blk == k].any(axis=1).astype(np.int64) << k
        missing += int(np.count_nonzero(need & ~got))
        listed += int(sum(bin(int(x)).count("1") for x in got))
        exact_bits += int(sum(bin(int(x)).count("1") for x in _exact_masks(m2[ids], co[ids], c.W, c.H, tx, ty)))
    print(f"{which}: {listed} listed (instance, block) pairs, exact float64 ellipse masks {exact_bits} "
          f"(ratio {listed / max(exact_bits, 1):.4f}), blocks with a blending pixel missing: {missing}")
    assert missing == 0
    assert listed <= 1.01 * exact_bits, (listed, exact_bits)
