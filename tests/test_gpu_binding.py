"""The native torch binding (splatam_amd/csrc/gsr_torch.cpp) of the drop-in path's per-iteration calls
against the ctypes binding of the same library entry points (splatam_amd/_C.py): identical results, bit for
bit, and the same argument errors (rasterize_points.cu:35-196 semantics)."""
import numpy as np
import pytest
import torch

from oracle import harness
from splatam_amd import _C
from splatam_amd.scenes import make_scene

pytestmark = pytest.mark.gpu


def _run(scene, dpix, native, monkeypatch, **kw):
    monkeypatch.setattr(_C, "_NATIVE_ON", native)
    return harness.run_gpu(scene, dpix, **kw)


@pytest.mark.parametrize("case", ["iso", "aniso_sh", "cov"])
def test_native_binding_matches_ctypes(cuda, case, monkeypatch):
    scene = make_scene(4000, 160, 120, seed=31, anisotropic=case != "iso")
    use_sh = case == "aniso_sh"
    if use_sh:
        scene = make_scene(4000, 160, 120, seed=31, anisotropic=True, sh_degree=2)
    dpix = np.random.RandomState(4).randn(3, scene.cam.H, scene.cam.W).astype(np.float32)
    kw = dict(use_sh=use_sh, use_cov=case == "cov", bg=(0.1, 0.2, 0.3))
    a = _run(scene, dpix, False, monkeypatch, **kw)
    b = _run(scene, dpix, True, monkeypatch, **kw)
    for k in ("color", "depth", "radii"):
        assert np.array_equal(a[k], b[k]), k
    assert set(a["grads"]) == set(b["grads"])
    for k in a["grads"]:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


def test_native_binding_power2_and_selective(cuda, monkeypatch):
    """backward_power = 2 (hessian_diff_gaussian_rasterization_w_depth) and the Fisher-selective request
    (dmeans3D + dopacity only) through both bindings."""
    scene = make_scene(2000, 96, 72, seed=8)
    dpix = np.full((3, scene.cam.H, scene.cam.W), 1e-3, np.float32)
    for grads_for in (None, ("means3D", "opacities")):
        a = _run(scene, dpix, False, monkeypatch, power=2, grads_for=grads_for)
        b = _run(scene, dpix, True, monkeypatch, power=2, grads_for=grads_for)
        assert set(a["grads"]) == set(b["grads"])
        for k in a["grads"]:
            assert np.array_equal(a["grads"][k], b["grads"][k]), (grads_for, k)


def test_native_binding_errors_and_empty(cuda):
    nat = _C._native()
    dev = torch.device(cuda)
    e = torch.Tensor([])
    cam = make_scene(10, 32, 32, seed=1).cam
    args = lambda m, col: (torch.zeros(3, device=dev), m, col, torch.ones(m.shape[0], 1, device=dev),  # noqa: E731
                           torch.ones(m.shape[0], 3, device=dev) * 0.1, torch.tensor([[1., 0, 0, 0]], device=dev)
                           .repeat(m.shape[0], 1), 1.0, e, cam.viewmatrix.to(dev), cam.projmatrix.to(dev), cam.tanfovx,
                           cam.tanfovy, 32, 32, e, 0, cam.campos.to(dev), False)
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        nat.rasterize_gaussians(*args(torch.zeros(4, 2, device=dev), torch.zeros(4, 3, device=dev)))
    with pytest.raises(RuntimeError, match="colors: expected scalar type Float but found torch.float64"):
        nat.rasterize_gaussians(*args(torch.rand(4, 3, device=dev) + 1, torch.zeros(4, 3, dtype=torch.float64,
                                                                                  device=dev)))
    n, color, radii, geom, binning, img, depth = nat.rasterize_gaussians(
        *args(torch.zeros(0, 3, device=dev), torch.zeros(0, 3, device=dev)))
    assert n == 0 and color.shape == (3, 32, 32) and float(color.abs().sum()) == 0 and radii.numel() == 0


def test_dropin_depth_only_loss(cuda):
    """The drop-in Function does not materialise the ignored radii / depth gradients; a loss that reads only
    the depth output (whose gradient the reference ignores, __init__.py:92) still back-propagates, with the
    gradients a zero colour gradient gives, and depth keeps requires_grad as in the reference."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    dev = torch.device(cuda)
    scene = make_scene(3000, 96, 72, seed=12)
    c = scene.cam
    st = GaussianRasterizationSettings(image_height=c.H, image_width=c.W, tanfovx=c.tanfovx, tanfovy=c.tanfovy,
                                       bg=torch.zeros(3, device=dev), scale_modifier=1.0,
                                       viewmatrix=c.viewmatrix.to(dev), projmatrix=c.projmatrix.to(dev), sh_degree=0,
                                       campos=c.campos.to(dev), prefiltered=False)

    def run(depth_only):
        leaf = {k: getattr(scene, k).to(dev).requires_grad_(True)
                for k in ("means3D", "colors", "opacities", "scales", "rotations")}
        m2 = torch.zeros_like(leaf["means3D"], requires_grad=True)
        im, radii, depth = GaussianRasterizer(st)(means3D=leaf["means3D"], means2D=m2, colors_precomp=leaf["colors"],
                                                  opacities=leaf["opacities"], scales=leaf["scales"],
                                                  rotations=leaf["rotations"])
        assert depth.requires_grad and not radii.requires_grad
        (depth.sum() if depth_only else im.sum() * 0.0 + depth.sum()).backward()
        return {k: v.grad for k, v in leaf.items()} | {"means2D": m2.grad}

    a, b = run(True), run(False)
    for k in a:
        assert a[k] is not None and torch.equal(a[k], b[k]), k
        assert float(a[k].abs().sum()) == 0.0, k
