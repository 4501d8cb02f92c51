"""Column scan of the [workgroup x tile] count matrix above 512 rows (> 512 * 1024 Gaussians):
tile_colscan_kernel's 32-tile shape, in the bucketed form (scans in duplicate) and in the launch-tail
form of the radix fallback (GSR_FORCE_RADIX=1, read once per process, hence one subprocess per form).
Both binnings order every tile by (depth, id), so image, depth, radii and num_rendered agree bitwise."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[2])
from splatam_amd import _C
from splatam_amd.scenes import make_scene
from splatam_amd.slam import camera_settings, init_tracking_params, transform_to_frame, transformed_params2rendervar
dev = torch.device("cuda:0")
s = make_scene(600000, 160, 120, seed=3)
params = init_tracking_params(s, 1, dev)
cam = camera_settings(s.cam, dev)
with torch.no_grad():
    rv = transformed_params2rendervar(params, transform_to_frame(params, 0, False, False))
    out = _C.rasterize_gaussians(cam.bg, rv["means3D"], rv["colors_precomp"], rv["opacities"], rv["scales"],
                                 rv["rotations"], cam.scale_modifier, torch.Tensor([]), cam.viewmatrix,
                                 cam.projmatrix, cam.tanfovx, cam.tanfovy, s.cam.H, s.cam.W, torch.Tensor([]),
                                 cam.sh_degree, cam.campos, cam.prefiltered)
    torch.cuda.synchronize()
np.savez(sys.argv[1], n=np.array(out[0]), color=out[1].cpu().numpy(), radii=out[2].cpu().numpy(),
         depth=out[6].cpu().numpy())
"""


def _render(tmp_path, radix):
    f = str(tmp_path / f"out_{radix}.npz")
    env = dict(os.environ, GSR_FORCE_RADIX=str(radix))
    r = subprocess.run([sys.executable, "-c", SCRIPT, f, ROOT], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(f)


@pytest.mark.gpu
def test_colscan_32_tile_shape_bucketed_vs_radix(tmp_path):
    a = _render(tmp_path, 0)
    b = _render(tmp_path, 1)
    assert int(a["n"]) > 0 and int(a["n"]) == int(b["n"])
    assert (a["radii"] > 0).sum() > 512 * 1024 // 4  # a large visible set (count matrix of > 512 rows)
    for k in ("color", "depth", "radii"):
        assert np.array_equal(a[k], b[k]), k
