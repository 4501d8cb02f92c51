"""SplaTAM tracking iteration on the GPU: the sync-free harness formulation
(slam.get_loss_tracking(fast=True)) equals the literal restatement of
scripts/splatam.py:220-353 (fast=False) in loss and pose gradients."""
import pytest
import torch

from splatam_amd.scenes import make_scene
from splatam_amd.slam import camera_settings, get_loss_tracking, init_tracking_params, transform_to_frame, \
    transformed_params2depthplussilhouette, transformed_params2rendervar
from splatam_amd.rasterizer import GaussianRasterizer

pytestmark = pytest.mark.gpu


def _setup(cuda, aniso):
    scene = make_scene(5000, 160, 120, seed=3, anisotropic=aniso)
    params = init_tracking_params(scene, num_frames=2, device=cuda)
    cam = camera_settings(scene.cam, cuda)
    w2c = torch.eye(4, device=cuda)
    with torch.no_grad():
        gt = dict(params)
        gt["cam_unnorm_rots"] = torch.zeros_like(params["cam_unnorm_rots"])
        gt["cam_unnorm_rots"][0, 0] = 1.0
        gt["cam_trans"] = torch.zeros_like(params["cam_trans"])
        tg = transform_to_frame(gt, 1, False, False)
        im, _, _ = GaussianRasterizer(cam)(**transformed_params2rendervar(gt, tg))
        ds, _, _ = GaussianRasterizer(cam)(**transformed_params2depthplussilhouette(gt, w2c, tg))
    return params, {"cam": cam, "w2c": w2c, "im": im, "depth": ds[0:1]}


@pytest.mark.parametrize("aniso", [False, True])
def test_fast_glue_equals_literal(cuda, aniso):
    params, curr = _setup(cuda, aniso)
    out = []
    for fast in (False, True):
        rots = params["cam_unnorm_rots"].detach().clone().requires_grad_(True)
        trans = params["cam_trans"].detach().clone().requires_grad_(True)
        p = dict(params, cam_unnorm_rots=rots, cam_trans=trans)
        loss, radius, _ = get_loss_tracking(p, curr, 1, fast=fast)
        loss.backward()
        out.append((loss.item(), rots.grad.clone(), trans.grad.clone(), radius))
    (l0, r0, t0, rad0), (l1, r1, t1, rad1) = out
    assert abs(l0 - l1) <= 1e-5 * abs(l0)
    torch.testing.assert_close(r1, r0, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(t1, t0, rtol=1e-4, atol=1e-6)
    assert torch.equal(rad0, rad1)
    assert float(l0) > 0.0 and float(r0.abs().sum()) > 0.0
