"""render_bwd step statistics (diagnostics): loads the -DGSR_STEPSTAT=1 build
(python -c "from splatam_amd import build; build.build_variant('stepstat', ['GSR_STEPSTAT=1'])"),
runs one tracking-style dual rasterization (config 3, grads for means3D + depth colours) and
reports wave-steps, the share with a contributing pair, contributing pairs per step and the
pad share of the padded row lists.  Usage: python tools/stepstat.py [config]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSR_LIB"] = os.environ.get("GSR_LIB") or os.path.join(ROOT, "splatam_amd", "_diag", "libgsr_stepstat.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from splatam_amd._lib import lib  # noqa: E402
from splatam_amd.rasterizer import rasterize_gaussians_dual  # noqa: E402
from splatam_amd.scenes import config_scene  # noqa: E402
from splatam_amd.slam import camera_settings  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    s = config_scene(cfg)
    cam = camera_settings(s.cam, dev)
    m3 = s.means3D.to(dev).requires_grad_(True)
    ds = torch.cat([m3.detach()[:, 2:3], torch.ones_like(m3[:, :1]), m3.detach()[:, 2:3] ** 2], 1).requires_grad_(True)
    g = torch.randn(3, s.cam.H, s.cam.W, device=dev)
    g2 = g.clone()
    g2[1:] = 0
    fn = lib.gsr_diag_stepstat_bwd
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 8)()
    m2 = torch.zeros_like(m3)
    im, im2, _, _ = rasterize_gaussians_dual(m3, m2, None, s.colors.to(dev), ds, s.opacities.to(dev),
                                             s.scales.to(dev), s.rotations.to(dev), None, cam, grad2_channels=1)
    torch.cuda.synchronize()
    fn(buf)
    torch.autograd.backward([im, im2], [g, g2])
    torch.cuda.synchronize()
    assert fn(buf) == 0
    steps, csteps, ok, pads, batches, items, dead = (int(buf[i]) for i in range(7))
    out = {"config": cfg, "wave_steps": steps, "contributing_step_share": csteps / max(steps, 1),
           "contributing_pairs": ok, "contributing_pairs_per_step": ok / max(steps, 1),
           "pair_slots": 256 * steps, "pad_share": pads / max(256 * steps, 1), "wave_batches": batches,
           "row_items": items, "row_items_without_contribution": dead, "dead_item_share": dead / max(items, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
