"""Host floor of the unchanged-caller unit (2 x GaussianRasterizer forward + backward) per binding:
a 1000-Gaussian scene at 640x480, so device time is small and the loop measures the host path (autograd, the
binding, launches).  Interleaved rounds of GSR_NATIVE_BINDING 0 / 1 in one process (splatam_amd._C._NATIVE_ON).

usage: python tools/binding_floor.py [units] [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from splatam_amd import _C  # noqa: E402
from splatam_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from splatam_amd.scenes import make_scene  # noqa: E402


def main():
    units = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    s = make_scene(1000, 640, 480, seed=0)
    c = s.cam
    st = GaussianRasterizationSettings(image_height=c.H, image_width=c.W, tanfovx=c.tanfovx, tanfovy=c.tanfovy,
                                       bg=torch.zeros(3, device=dev), scale_modifier=1.0,
                                       viewmatrix=c.viewmatrix.to(dev), projmatrix=c.projmatrix.to(dev), sh_degree=0,
                                       campos=c.campos.to(dev), prefiltered=False)
    m = s.means3D.to(dev).requires_grad_(True)
    col = s.colors.to(dev).requires_grad_(True)
    op = s.opacities.to(dev).requires_grad_(True)
    sc = s.scales.to(dev).requires_grad_(True)
    rot = s.rotations.to(dev).requires_grad_(True)

    def unit():
        m2 = torch.zeros_like(m, requires_grad=True)
        im, _, _ = GaussianRasterizer(st)(means3D=m, means2D=m2, opacities=op, colors_precomp=col, scales=sc,
                                          rotations=rot)
        m2b = torch.zeros_like(m, requires_grad=True)
        ds, _, _ = GaussianRasterizer(st)(means3D=m, means2D=m2b, opacities=op, colors_precomp=col, scales=sc,
                                          rotations=rot)
        (im.sum() + ds.sum()).backward()

    res = {0: [], 1: []}
    for r in range(rounds):
        for nat in (0, 1):
            _C._NATIVE_ON = bool(nat)
            for _ in range(20):
                unit()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(units):
                unit()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / units * 1e6
            res[nat].append(us)
            print(f"round {r} native {nat}: {us:.1f} us per unit (2 forward + 2 backward, 1000 Gaussians)", flush=True)
    for nat in (0, 1):
        v = sorted(res[nat])
        print(f"native {nat}: median {v[len(v) // 2]:.1f} us per unit")


if __name__ == "__main__":
    main()
