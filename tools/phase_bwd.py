"""render_bwd phase breakdown (diagnostics): loads the -DGSR_PHASE=1 build
(python -c "from splatam_amd import build; build.build_variant('phase', ['GSR_PHASE=1'])"),
runs the tracking-style dual rasterization backward (config 3, grads for means3D + the depth colour)
and reports the share of per-wave shader-clock cycles in each phase of render_bwd_kernel
(gsr_backward.hip GSR_PHASE).  Usage: python tools/phase_bwd.py [config] [reps]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSR_LIB"] = os.path.join(ROOT, "splatam_amd", "_diag", "libgsr_phase.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from splatam_amd._lib import lib  # noqa: E402
from splatam_amd.rasterizer import rasterize_gaussians_dual  # noqa: E402
from splatam_amd.scenes import config_scene  # noqa: E402
from splatam_amd.slam import camera_settings  # noqa: E402

NAMES = ["prologue", "staging+barrier", "list_build", "row_walk", "barrier_after_walk", "entry_totals+stores",
         "barrier_after_totals"]


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    s = config_scene(cfg)
    cam = camera_settings(s.cam, dev)
    m3 = s.means3D.to(dev).requires_grad_(True)
    ds = torch.cat([m3.detach()[:, 2:3], torch.ones_like(m3[:, :1]), m3.detach()[:, 2:3] ** 2], 1).requires_grad_(True)
    g = torch.randn(3, s.cam.H, s.cam.W, device=dev)
    g2 = g.clone()
    g2[1:] = 0
    fn = lib.gsr_diag_phase_bwd
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 8)()
    m2 = torch.zeros_like(m3)
    tot = [0] * 8
    for r in range(reps + 1):
        im, im2, _, _ = rasterize_gaussians_dual(m3, m2, None, s.colors.to(dev), ds, s.opacities.to(dev),
                                                 s.scales.to(dev), s.rotations.to(dev), None, cam, grad2_channels=1)
        torch.cuda.synchronize()
        fn(buf)
        torch.autograd.backward([im, im2], [g, g2])
        torch.cuda.synchronize()
        assert fn(buf) == 0
        if r:  # the first repetition warms up
            for k in range(8):
                tot[k] += int(buf[k])
    cyc = sum(tot[:7])
    out = {"config": cfg, "reps": reps, "wave_batches_per_launch": tot[7] / reps,
           "cycles_per_wave_batch": cyc / max(tot[7], 1),
           "share": {n: round(tot[k] / cyc, 4) for k, n in enumerate(NAMES)},
           "cycles_per_launch_all_waves": cyc / reps}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
