"""Fisher / EIG view scoring (splatam_amd.fisher, ros_handler.py:807-902) on the GPU:
the per-pose Hessian H = [dL/dmeans_cam, dL/dopacity] of the backward_power=2 render
seeded with 1e-3 against the float32 C oracle's fused-mode (per-pair powf) backward."""
import math

import numpy as np
import pytest
import torch

from oracle import harness, oracle
from splatam_amd.fisher import FisherScorer
from splatam_amd.scenes import Scene, make_scene
from splatam_amd.slam import camera_settings, init_tracking_params

pytestmark = pytest.mark.gpu


def _pose(deg, t):
    a = math.radians(deg)
    w2c = torch.eye(4)
    w2c[:3, :3] = torch.tensor([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    w2c[:3, 3] = torch.tensor(t)
    return w2c


@pytest.mark.parametrize("aniso", [False, True])
def test_fisher_hessian_matches_oracle(cuda, aniso):
    scene = make_scene(2500, 96, 72, seed=21, anisotropic=aniso)
    params = init_tracking_params(scene, num_frames=1, device=cuda)
    if aniso:
        params["log_scales"] = torch.log(scene.scales).to(cuda)
    cam = camera_settings(scene.cam, cuda)
    sc = FisherScorer(params, cam)
    w2c = _pose(3.0, [0.02, -0.01, 0.05])
    H = sc.hessian(w2c.to(cuda)).cpu().numpy()
    # the oracle on the same transformed rendervars (ros_handler.py:863-882)
    pts4 = torch.cat([scene.means3D, torch.ones(scene.P, 1)], 1)
    pts = (w2c @ pts4.T).T[:, :3].contiguous()
    rv = Scene(means3D=pts, scales=sc.scales.cpu(), rotations=sc.rotations.cpu(), opacities=sc.opacities.cpu(),
               colors=sc.colors.cpu(), shs=None, sh_degree=0, cam=scene.cam)
    dpix = np.full((3, scene.cam.H, scene.cam.W), 1e-3, np.float32)
    _, ref = harness.run_oracle(rv, dpix, power=2, mode=oracle.FUSED)
    assert harness.rel_l2(H[:, :3], ref["dmeans3D"].reshape(-1, 3)) <= 1e-4
    assert harness.rel_l2(H[:, 3], ref["dopacity"].reshape(-1)) <= 1e-4
    assert (H >= 0).all()  # squared per-pair gradients
    # visited-pose fit and candidate score (single process)
    hinv = sc.fit_visited([w2c.to(cuda), torch.eye(4, device=cuda)])
    s = sc.eig_scores([w2c.to(cuda)])
    torch.testing.assert_close(s[0], (torch.tensor(H, device=cuda) * hinv).sum().double(), rtol=1e-6, atol=0)
