"""Render-kernel phase breakdown (diagnostics): loads the -DGSR_PHASE=1 build
(python -c "from splatam_amd import build; build.build_variant('phase', ['GSR_PHASE=1'])"), runs the
tracking-style dual rasterization (config 3; grads for means3D + the depth colour) and reports the share of
per-wave shader-clock cycles in each phase of render_fwd_kernel and render_bwd_kernel (gsr_diag.h).  The
s_memtime stamps wait for outstanding LDS operations, so the shares are indicative, not exact.  With `full`
every Gaussian input requires grad (the mapping-style variant: opacity and colour sums as well).
Usage: python tools/phase.py [config] [reps] [full]"""
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

NAMES = {"bwd": ["prologue", "staging+barrier", "list_build", "row_walk", "barrier_after_walk", "entry_totals+stores",
                 "barrier_after_totals"],
         "fwd": ["prologue+sort", "staging+barrier", "list_build", "row_walk", "barrier_after_walk", "epilogue"]}


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    full = len(sys.argv) > 3 and sys.argv[3] == "full"
    dev = torch.device("cuda:0")
    s = config_scene(cfg)
    cam = camera_settings(s.cam, dev)
    m3 = s.means3D.to(dev).requires_grad_(True)
    ds = torch.cat([m3.detach()[:, 2:3], torch.ones_like(m3[:, :1]), m3.detach()[:, 2:3] ** 2], 1).requires_grad_(True)
    g = torch.randn(3, s.cam.H, s.cam.W, device=dev)
    g2 = g.clone()
    g2[1:] = 0
    fns = {}
    for k in ("fwd", "bwd"):
        f = getattr(lib, f"gsr_diag_phase_{k}")
        f.argtypes = [ctypes.c_void_p]
        fns[k] = f
    buf = (ctypes.c_ulonglong * 8)()
    m2 = torch.zeros_like(m3)
    tot = {k: [0] * 8 for k in fns}
    for r in range(reps + 1):
        for f in fns.values():
            f(buf)  # clear
        leaf = (lambda t: t.to(dev).requires_grad_(True)) if full else (lambda t: t.to(dev))  # noqa: E731
        im, im2, _, _ = rasterize_gaussians_dual(m3, m2, None, leaf(s.colors), ds, leaf(s.opacities),
                                                 leaf(s.scales), leaf(s.rotations), None, cam, grad2_channels=1)
        torch.autograd.backward([im, im2], [g, g2])
        torch.cuda.synchronize()
        for k, f in fns.items():
            assert f(buf) == 0
            if r:  # the first repetition warms up
                for q in range(8):
                    tot[k][q] += int(buf[q])
    out = {"config": cfg, "reps": reps, "full": full}
    for k, t in tot.items():
        n = len(NAMES[k])
        cyc = sum(t[:n])
        out[k] = {"wave_batches_per_launch": t[7] / reps, "cycles_per_launch_all_waves": cyc / reps,
                  "share": {name: round(t[q] / max(cyc, 1), 4) for q, name in enumerate(NAMES[k])}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
