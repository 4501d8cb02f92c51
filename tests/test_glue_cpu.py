"""SplaTAM caller glue (splatam_amd.scenes / splatam_amd.slam) against golden
outputs of the reference's own utils/*.py (tests/golden/make_goldens.py)."""
import os

import numpy as np
import torch

from splatam_amd import scenes, slam

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_setup_camera_matches_reference():
    g = np.load(os.path.join(GOLD, "glue_setup_camera.npz"))
    K = g["K"]
    cam = scenes.setup_camera(int(g["W"]), int(g["H"]), K[0, 0], K[1, 1], K[0, 2], K[1, 2], w2c=g["w2c"])
    np.testing.assert_allclose(cam.viewmatrix.numpy(), g["viewmatrix"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(cam.projmatrix.numpy(), g["projmatrix"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(cam.campos.numpy(), g["campos"], rtol=1e-6, atol=1e-7)
    assert abs(cam.tanfovx - float(g["tanfovx"])) < 1e-12 and abs(cam.tanfovy - float(g["tanfovy"])) < 1e-12
    st = slam.camera_settings(cam, "cpu")
    assert st.sh_degree == int(g["sh_degree"]) and st.prefiltered == bool(g["prefiltered"])
    assert st.scale_modifier == float(g["scale_modifier"]) and float(st.bg.abs().sum()) == 0.0


def _params(g):
    return {k[len("param_"):]: torch.tensor(v) for k, v in g.items() if k.startswith("param_")}


def test_transform_and_rendervars_match_reference():
    for name in ("iso", "aniso"):
        g = np.load(os.path.join(GOLD, f"glue_transform_{name}.npz"))
        params = _params(g)
        tg = slam.transform_to_frame(params, int(g["time_idx"]), gaussians_grad=True, camera_grad=True)
        np.testing.assert_allclose(tg["means3D"].detach().numpy(), g["tg_means3D"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(tg["unnorm_rotations"].detach().numpy(), g["tg_unnorm_rotations"], rtol=1e-5,
                                   atol=1e-6)
        rv = slam.transformed_params2rendervar(params, tg)
        dv = slam.transformed_params2depthplussilhouette(params, torch.tensor(g["w2c"]), tg)
        for key, ref in (("rotations", "rv_rotations"), ("opacities", "rv_opacities"), ("scales", "rv_scales"),
                         ("colors_precomp", "rv_colors")):
            np.testing.assert_allclose(rv[key].detach().numpy(), g[ref], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(dv["colors_precomp"].detach().numpy(), g["dv_colors"], rtol=1e-5, atol=1e-6)
        assert float(rv["means2D"].abs().sum()) == 0.0 and rv["means2D"].requires_grad


def test_build_rotation_matches_reference():
    g = np.load(os.path.join(GOLD, "glue_build_rotation.npz"))
    np.testing.assert_allclose(slam.build_rotation(torch.tensor(g["q"])).numpy(), g["R"], rtol=1e-5, atol=1e-6)


def test_synthetic_scene_is_seeded_and_in_frustum():
    a = scenes.config_scene(1)
    b = scenes.config_scene(1)
    assert torch.equal(a.means3D, b.means3D) and a.P == 10_000
    c = a.cam
    z = a.means3D[:, 2]
    u = a.means3D[:, 0] / z * c.fx + c.cx
    assert float(z.min()) >= 0.5 and float(u.min()) > -1 and float(u.max()) < c.W + 1
