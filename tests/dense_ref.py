"""Dense, differentiable torch formulation of the reference rasterizer.

Test infrastructure: an independent statement of the forward maths
(forward.cu:20-256, 261-393) whose gradients come from torch.autograd rather
than from hand-written backward formulas.  It reproduces the reference's
gradient conventions where the reference deliberately deviates from exact
autograd:

* alpha = min(0.99, o*G): the backward never zeroes the gradient at the 0.99
  clamp (backward.cu:974-1038) -> straight-through estimator here;
* the +-1.3 tanfov clamp of t.x / t.y: backward.cu:175-176,262-264 zeroes the
  x/y gradient and treats the clamped value as a constant in dJ/dt_z;
* dL/dscale is taken w.r.t. (scale_modifier * scale) (backward.cu:457-459).

The per-tile candidate lists, depth order and the discrete decisions (skip,
early termination) come from the float64 oracle run on the same inputs.
"""
from __future__ import annotations

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]


def eval_sh(deg, sh, dirs):
    x, y, z = dirs[:, 0:1], dirs[:, 1:2], dirs[:, 2:3]
    res = SH_C0 * sh[:, 0]
    if deg > 0:
        res = res - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = res + (SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
                         + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                res = res + (SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
                             + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11]
                             + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
                             + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
                             + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return res + 0.5


def quat_to_rot(q):
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
        2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
        2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], dim=1)
    return R.reshape(-1, 3, 3)


def render_dense(fr, *, means3D, means2D, opacities, view, proj, campos, tanfovx, tanfovy, H, W, bg,
                 colors=None, shs=None, sh_degree=0, scales=None, rotations=None, cov3D=None,
                 scale_modifier=1.0):
    """Differentiable image [3,H,W] following the oracle's binning ``fr``."""
    dt = means3D.dtype
    view = view.reshape(4, 4).to(dt)
    proj = proj.reshape(4, 4).to(dt)
    P = means3D.shape[0]
    ones = torch.ones(P, 1, dtype=dt)
    ph = torch.cat([means3D, ones], 1)
    hom = ph @ proj                      # m[4c+r] layout == row-vector times the [4,4] tensor
    pw = 1.0 / (hom[:, 3] + 1e-7)
    p_proj = hom[:, :2] * pw[:, None] + means2D[:, :2]
    pix_x = ((p_proj[:, 0] + 1.0) * W - 1.0) * 0.5
    pix_y = ((p_proj[:, 1] + 1.0) * H - 1.0) * 0.5
    if cov3D is None:
        R = quat_to_rot(rotations)
        s = scale_modifier * scales
        Sig = R @ torch.diag_embed(s * s) @ R.transpose(1, 2)
    else:
        c = cov3D
        Sig = torch.stack([c[:, 0], c[:, 1], c[:, 2], c[:, 1], c[:, 3], c[:, 4], c[:, 2], c[:, 4], c[:, 5]], 1).reshape(-1, 3, 3)
    t = ph @ view
    tx, ty, tz = t[:, 0], t[:, 1], t[:, 2]
    fx = W / (2 * tanfovx)
    fy = H / (2 * tanfovy)
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    txtz, tytz = tx / tz, ty / tz
    inx = (txtz >= -limx) & (txtz <= limx)
    iny = (tytz >= -limy) & (tytz <= limy)
    txc = torch.where(inx, tx, (txtz.clamp(-limx, limx) * tz).detach())
    tyc = torch.where(iny, ty, (tytz.clamp(-limy, limy) * tz).detach())
    zeros = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zeros, -(fx * txc) / (tz * tz)], 1),
                     torch.stack([zeros, fy / tz, -(fy * tyc) / (tz * tz)], 1)], 1)   # [P,2,3]
    V3 = view[:3, :3].T                                                                 # V3[r][k] = m[4k+r]
    Mx = J @ V3
    cov2 = Mx @ Sig @ Mx.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c2 = cov2[:, 1, 1] + 0.3
    det = a * c2 - b * b
    A, B, C = c2 / det, -b / det, a / det
    if colors is None:
        dirs = means3D - campos.reshape(1, 3).to(dt)
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        colors = torch.clamp_min(eval_sh(sh_degree, shs, dirs), 0.0)
    opac = opacities.reshape(-1)
    gx = (W + 15) // 16
    out = torch.zeros(3, H, W, dtype=dt)
    ranges = fr.ranges
    pl = torch.as_tensor(fr.point_list.astype(np.int64))
    bgv = bg.reshape(3).to(dt)
    for t_id in range(ranges.shape[0]):
        s0, e0 = int(ranges[t_id, 0]), int(ranges[t_id, 1])
        tyi, txi = divmod(t_id, gx)
        ys = torch.arange(tyi * 16, min(tyi * 16 + 16, H))
        xs = torch.arange(txi * 16, min(txi * 16 + 16, W))
        if len(ys) == 0 or len(xs) == 0:
            continue
        yy, xx = torch.meshgrid(ys, xs, indexing="ij")
        pxf = xx.reshape(-1).to(dt)
        pyf = yy.reshape(-1).to(dt)
        if e0 <= s0:
            for ch in range(3):
                out[ch, yy, xx] = bgv[ch]
            continue
        ids = pl[s0:e0]
        dx = pix_x[ids][None, :] - pxf[:, None]
        dy = pix_y[ids][None, :] - pyf[:, None]
        power = -0.5 * (A[ids][None] * dx * dx + C[ids][None] * dy * dy) - B[ids][None] * dx * dy
        G = torch.exp(power)
        araw = opac[ids][None] * G
        alpha = torch.where(araw > 0.99, 0.99 + (araw - araw.detach()), araw)
        with torch.no_grad():
            m = (power <= 0) & (alpha >= 1.0 / 255.0)
            am = torch.where(m, alpha, torch.zeros_like(alpha))
            Tex = torch.cumprod(torch.cat([torch.ones_like(am[:, :1]), 1 - am[:, :-1]], 1), 1)
            stop = m & (Tex * (1 - am) < 1e-4)
            first = torch.where(stop.any(1), stop.float().argmax(1), torch.full((stop.shape[0],), stop.shape[1]))
            keep = m & (torch.arange(m.shape[1])[None, :] < first[:, None])
        ak = torch.where(keep, alpha, torch.zeros_like(alpha))
        T = torch.cumprod(torch.cat([torch.ones_like(ak[:, :1]), 1 - ak[:, :-1]], 1), 1)
        Tfin = T[:, -1] * (1 - ak[:, -1])
        w = ak * T
        col = w @ colors[ids]                                   # [pix,3]
        col = col + Tfin[:, None] * bgv[None, :]
        for ch in range(3):
            out[ch, yy, xx] = col[:, ch].reshape(yy.shape)
    return out
