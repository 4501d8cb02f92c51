"""Bitwise A/B of the render-backward variants between two libgsr builds (GPU box), the companion of
tools/pose_bits.py for the paths that do not step a pose: the single-image full gradient with three
incoming colour channels (bwd_tile C1 = 3) and with only channel 0 (C1 = 1, the depth/silhouette call),
backward_power = 2 (the moment variant), SH colours, and the dual mapping backward (both colour sets,
three channels each).  Writes every output of each case to OUT (.npz); run it once per library, then
`python tools/grad_bits.py --compare A.npz B.npz` reports whether every array is bitwise equal.

usage: GSR_LIB_AB=1 GSR_LIB=... python tools/grad_bits.py OUT.npz
       python tools/grad_bits.py --compare A.npz B.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out):
    import torch
    from oracle import harness
    from splatam_amd import _C
    from splatam_amd.scenes import make_scene
    res = {}
    scene = make_scene(30000, 320, 240, seed=5, anisotropic=True)
    rs = np.random.RandomState(2)
    H, W = scene.cam.H, scene.cam.W
    dpix = rs.randn(3, H, W).astype(np.float32)
    d1 = dpix.copy()
    d1[1:] = 0.0
    cases = {"c3": dict(dL_dcolor=dpix), "c1": dict(dL_dcolor=d1), "pow2": dict(dL_dcolor=dpix, power=2),
             "bg": dict(dL_dcolor=dpix, bg=(0.2, 0.1, 0.3))}
    for name, kw in cases.items():
        r = harness.run_gpu(scene, **kw)
        for k in ("color", "depth", "radii"):
            res[f"{name}/{k}"] = r[k]
        for k, v in r["grads"].items():
            res[f"{name}/d{k}"] = v
    sh = make_scene(20000, 320, 240, seed=6, anisotropic=True, sh_degree=2)
    r = harness.run_gpu(sh, dL_dcolor=dpix, use_sh=True)
    for k, v in r["grads"].items():
        res[f"sh/d{k}"] = v
    # the dual (mapping) backward: both colour sets, three channels each
    dev = torch.device("cuda", 0)
    c = scene.cam
    bg = torch.zeros(3, device=dev)
    args = dict(viewmatrix=c.viewmatrix.to(dev), projmatrix=c.projmatrix.to(dev), tan_fovx=c.tanfovx,
                tan_fovy=c.tanfovy, campos=c.campos.to(dev))
    m = scene.means3D.to(dev)
    col = scene.colors.to(dev)
    col2 = torch.rand(m.shape[0], 3, generator=torch.Generator().manual_seed(9)).to(dev)
    op = scene.opacities.to(dev)
    sc = scene.scales.to(dev)
    rot = scene.rotations.to(dev)
    e = torch.Tensor([])
    n, im, im2, radii, geom, binning, img, depth = _C.rasterize_gaussians_dual(
        bg, m, col, col2, op, sc, rot, 1.0, e, args["viewmatrix"], args["projmatrix"], args["tan_fovx"],
        args["tan_fovy"], H, W, e, 0, args["campos"], False)
    dp2 = torch.from_numpy(rs.randn(3, H, W).astype(np.float32)).to(dev)
    outs = _C.rasterize_gaussians_dual_backward(
        bg, m, radii, col, col2, sc, rot, 1.0, e, args["viewmatrix"], args["projmatrix"], args["tan_fovx"],
        args["tan_fovy"], torch.from_numpy(dpix).to(dev), dp2, e, 0, args["campos"], geom, n, binning, img)
    torch.cuda.synchronize()
    res["dual/color"] = im.cpu().numpy()
    res["dual/color2"] = im2.cpu().numpy()
    for i, o in enumerate(outs):
        if o is not None and o.numel():
            res[f"dual/out{i}"] = o.cpu().numpy()
    np.savez(out, **res)
    print(f"wrote {len(res)} arrays to {out}")


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if k not in B.files or A[k].shape != B[k].shape
           or not np.array_equal(A[k].view(np.uint8), B[k].view(np.uint8))]
    bad += [k for k in B.files if k not in A.files]
    print(f"{len(A.files)} arrays; bitwise equal: {not bad}" + (f"; differ: {bad}" if bad else ""))
    return 0 if not bad else 1


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
