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


# ------------------------------------------------------------------ mapping --
def test_calc_ssim_matches_reference():
    g = np.load(os.path.join(GOLD, "glue_ssim.npz"))
    img1 = torch.tensor(g["img1"], requires_grad=True)
    s = slam.calc_ssim(img1, torch.tensor(g["img2"]))
    s.backward()
    np.testing.assert_allclose(float(s), float(g["ssim"]), rtol=1e-6)
    np.testing.assert_allclose(img1.grad.numpy(), g["grad_img1"], rtol=1e-4, atol=1e-10)


def _ssim_grad_by_partial_maps(x, y, win):
    """The HIP map_loss kernels' factorisation (csrc/gsr_mapping.hip): per-pixel partials
    dS/dmu1, dS/dE[x^2], dS/dE[xy], blurred back with the same zero-padded window."""
    C = x.shape[0]
    k2 = (win[:, None] * win[None, :]).to(x.dtype)  # float32 outer product, like create_window
    w = k2.expand(C, 1, 11, 11)
    conv = lambda t: torch.nn.functional.conv2d(t, w, padding=5, groups=C)  # noqa: E731
    mu1, mu2, e11, e22, e12 = conv(x), conv(y), conv(x * x), conv(y * y), conv(x * y)
    s11, s22, s12 = e11 - mu1 * mu1, e22 - mu2 * mu2, e12 - mu1 * mu2
    A, B = 2 * mu1 * mu2 + 1e-4, 2 * s12 + 9e-4
    Cc, D = mu1 * mu1 + mu2 * mu2 + 1e-4, s11 + s22 + 9e-4
    s = A * B / (Cc * D)
    g0 = 2 * mu2 * (B - A) / (Cc * D) - 2 * mu1 * s * (1 / Cc - 1 / D)
    g1 = -s / D
    g2 = 2 * A / (Cc * D)
    n = s.numel()
    return s.mean(), (conv(g0) + 2 * x * conv(g1) + y * conv(g2)) / n


def test_ssim_partial_map_factorisation_equals_autograd():
    gen = torch.Generator().manual_seed(5)
    x = torch.rand(3, 29, 41, generator=gen, dtype=torch.float64, requires_grad=True)
    y = torch.rand(3, 29, 41, generator=gen, dtype=torch.float64)
    win = slam._gaussian(11, 1.5)
    ref = slam.calc_ssim(x, y)
    ref.backward()
    s, grad = _ssim_grad_by_partial_maps(x.detach(), y, win)
    assert abs(float(s) - float(ref)) < 1e-12
    np.testing.assert_allclose(grad.numpy(), x.grad.numpy(), rtol=1e-9, atol=1e-13)


def test_mapping_transform_gradients_match_reference():
    for name in ("iso", "aniso"):
        g = np.load(os.path.join(GOLD, f"glue_map_transform_{name}.npz"))
        params = _params(g)
        for k in ("means3D", "rgb_colors", "unnorm_rotations", "logit_opacities", "log_scales"):
            params[k].requires_grad_(True)
        tg = slam.transform_to_frame(params, int(g["time_idx"]), gaussians_grad=True, camera_grad=False, fast=False)
        rv = slam.transformed_params2rendervar(params, tg)
        dv = slam.transformed_params2depthplussilhouette(params, torch.tensor(g["w2c"]), tg, fast=False)
        total = sum((rv[k] * torch.tensor(g[u])).sum() for k, u in (("means3D", "g_means"), ("rotations", "g_rot"),
                                                                     ("opacities", "g_opac"), ("scales", "g_scales")))
        total = total + (dv["colors_precomp"] * torch.tensor(g["g_dcol"])).sum()
        total.backward()
        for k in ("means3D", "unnorm_rotations", "logit_opacities", "log_scales"):
            np.testing.assert_allclose(params[k].grad.numpy(), g[f"grad_{k}"], rtol=1e-4, atol=1e-6, err_msg=k)


def test_checkpoint_roundtrip_matches_reference_writer(tmp_path):
    """A params.npz written by the reference's save_params loads without unpickling, and
    ours writes the same keys and arrays back (utils/common_utils.py:35-52)."""
    from splatam_amd import checkpoint
    ref = os.path.join(GOLD, "ref_params.npz")
    p = checkpoint.load_params(ref, device="cpu")
    with np.load(ref, allow_pickle=False) as z:
        keys = sorted(z.files)
        for k in keys:
            np.testing.assert_array_equal(p[k].detach().numpy(), z[k].astype(np.float32))
    assert p["means3D"].requires_grad and p["means3D"].dtype == torch.float32
    out = checkpoint.save_params_ckpt({k: v for k, v in p.items()}, str(tmp_path), 7)
    assert out.endswith("params7.npz")
    with np.load(out, allow_pickle=False) as z2, np.load(ref, allow_pickle=False) as z:
        assert sorted(z2.files) == keys
        for k in keys:
            np.testing.assert_array_equal(z2[k], z[k].astype(np.float32))


def test_prune_and_surgery_keep_optimizer_state_aligned():
    """remove_points / cat_params_to_optimizer / prune_gaussians (slam_external.py:107-192)
    on torch.optim.Adam: moments follow their Gaussians."""
    from splatam_amd import surgery
    g = torch.Generator().manual_seed(0)
    P = 50
    params = {"means3D": torch.randn(P, 3, generator=g), "logit_opacities": torch.randn(P, 1, generator=g) * 3,
              "log_scales": torch.randn(P, 1, generator=g) - 3, "cam_unnorm_rots": torch.randn(1, 4, 2),
              "cam_trans": torch.randn(1, 3, 2)}
    params = {k: torch.nn.Parameter(v) for k, v in params.items()}
    opt = torch.optim.Adam([{"params": [v], "name": k, "lr": 0.01} for k, v in params.items()], lr=0.0, eps=1e-15)
    loss = sum((v ** 2).sum() for v in params.values())
    loss.backward()
    opt.step()
    m_before = opt.state[params["means3D"]]["exp_avg"].clone()
    keep_ref = torch.sigmoid(params["logit_opacities"].detach()).squeeze() >= 0.1
    variables = {"scene_radius": 100.0, "means2D_gradient_accum": torch.arange(P).float(), "denom": torch.ones(P),
                 "max_2D_radius": torch.zeros(P), "timestep": torch.zeros(P)}
    pd = dict(start_after=0, remove_big_after=0, stop_after=20, prune_every=20, removal_opacity_threshold=0.1,
              final_removal_opacity_threshold=0.1, reset_opacities=False, reset_opacities_every=500)
    params, variables = surgery.prune_gaussians(params, variables, opt, 0, pd)
    n = int(keep_ref.sum())
    assert 0 < n < P and params["means3D"].shape[0] == n and params["cam_trans"].shape == (1, 3, 2)
    torch.testing.assert_close(opt.state[params["means3D"]]["exp_avg"], m_before[keep_ref])
    assert torch.equal(variables["means2D_gradient_accum"], torch.arange(P).float()[keep_ref])
    new = {k: params[k].detach()[:3].clone() for k in ("means3D", "logit_opacities", "log_scales")}
    params = surgery.cat_params_to_optimizer(new, params, opt)
    assert params["means3D"].shape[0] == n + 3
    assert float(opt.state[params["means3D"]]["exp_avg"][n:].abs().sum()) == 0.0
