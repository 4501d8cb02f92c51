"""SplaTAM mapping iteration on the GPU (include/gsr_glue.h mapping entry points):
the fused SSIM/L1 loss kernels, the mapping transform backward, the fused Adam
step and the whole fused iteration against the literal restatement of
scripts/splatam.py:220-353 (mapping=True) in splatam_amd.slam, whose torch glue
is itself pinned to the reference's utils/*.py by tests/test_glue_cpu.py."""
import contextlib
import numpy as np
import pytest
import torch

from splatam_amd import slam
from splatam_amd.glue import FusedAdam, MapAdam, map_transform, mapping_loss
from splatam_amd.rasterizer import GaussianRasterizer
from splatam_amd.scenes import make_scene

pytestmark = pytest.mark.gpu

GAUSS_KEYS = ("means3D", "unnorm_rotations", "logit_opacities", "log_scales")


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _images(cuda, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    im = torch.rand(3, H, W, generator=g)
    gt = (im + 0.2 * torch.randn(3, H, W, generator=g)).clamp(0, 1)
    ds = torch.stack([0.5 + 4 * torch.rand(H, W, generator=g), torch.rand(H, W, generator=g),
                      torch.zeros(H, W)])
    ds[2] = ds[0] * ds[0] + 0.01 * torch.rand(H, W, generator=g)
    gd = (ds[0:1] + 0.3 * torch.randn(1, H, W, generator=g)).clamp_min(0)
    gd[:, :, : W // 7] = 0.0                       # invalid depth stripe
    ds[0, 3, 5] = float("nan")                     # a NaN depth pixel is masked out
    return [t.to(cuda) for t in (im, ds, gt, gd)]


def _literal_loss(im, ds, gt, gd, w_im=0.5, w_depth=1.0):
    depth, dsq = ds[0:1], ds[2:3]
    unc = (dsq - depth ** 2).detach()
    mask = ((gd > 0) & ~torch.isnan(depth) & ~torch.isnan(unc)).detach()
    l_d = torch.abs(gd - depth)[mask].mean()
    l_im = 0.8 * slam.l1_loss_v1(im, gt) + 0.2 * (1.0 - slam.calc_ssim(im, gt))
    return w_im * l_im + w_depth * l_d


@pytest.mark.parametrize("hw", [(70, 150), (16, 64), (5, 7), (480, 640)])
def test_mapping_loss_kernel_matches_literal(cuda, hw):
    """Loss and both image gradients vs the literal torch expression in float64
    (float32 kernel: loss within 1e-5 relative, gradients within 1e-5 relative L2)."""
    H, W = hw
    im, ds, gt, gd = _images(cuda, H, W)
    a_im, a_ds = im.clone().requires_grad_(True), ds.clone().requires_grad_(True)
    loss = mapping_loss(a_im, a_ds, gt, gd)
    loss.backward()
    r_im, r_ds = im.double().requires_grad_(True), ds.double().requires_grad_(True)
    ref = _literal_loss(r_im, r_ds, gt.double(), gd.double())
    ref.backward()
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref)), (float(loss), float(ref))
    assert _rel(a_im.grad, r_im.grad) <= 1e-5
    g_ds = torch.nan_to_num(r_ds.grad, nan=0.0)
    assert _rel(a_ds.grad, g_ds) <= 1e-6
    assert float(a_ds.grad[1:].abs().sum()) == 0.0


def test_mapping_loss_empty_depth_mask(cuda):
    """No valid depth: the masked mean is NaN (torch's mean of an empty selection) and
    the depth gradient is zero; the image gradient stays finite."""
    im, ds, gt, gd = _images(cuda, 40, 70)
    gd.zero_()
    a_im, a_ds = im.clone().requires_grad_(True), ds.clone().requires_grad_(True)
    loss = mapping_loss(a_im, a_ds, gt, gd)
    loss.backward()
    assert torch.isnan(loss)
    assert float(a_ds.grad.abs().sum()) == 0.0 and bool(torch.isfinite(a_im.grad).all())


def test_mapping_loss_deterministic(cuda):
    im, ds, gt, gd = _images(cuda, 480, 640, seed=3)
    outs = []
    for _ in range(2):
        a = im.clone().requires_grad_(True)
        loss = mapping_loss(a, ds, gt, gd)
        loss.backward()
        outs.append((loss.item(), a.grad.clone()))
    assert outs[0][0] == outs[1][0] and torch.equal(outs[0][1], outs[1][1])


def _map_params(cuda, aniso, sh, P=3000, W=150, H=110, seed=3):
    scene = make_scene(P, W, H, seed=seed, anisotropic=aniso, sh_degree=3 if sh else 0)
    params = slam.init_mapping_params(scene, num_frames=3, device=cuda)
    cam = slam.camera_settings(scene.cam, cuda, sh_degree=scene.sh_degree)
    return scene, params, cam


@pytest.mark.parametrize("aniso", [False, True])
def test_map_transform_bwd_matches_autograd(cuda, aniso):
    """gsr_map_transform_bwd vs autograd through the literal transform_to_frame + builders (float64)."""
    _, params, _ = _map_params(cuda, aniso, False)
    w2c = torch.eye(4, device=cuda)
    w2c[:3, 3] = torch.tensor([0.05, -0.02, 0.1], device=cuda)
    P = params["means3D"].shape[0]
    g = torch.Generator().manual_seed(9)
    ups = [torch.randn(P, n, generator=g).to(cuda) for n in (3, 4, 3, 1, 3)]
    leaves = {k: params[k].clone().requires_grad_(True) for k in GAUSS_KEYS + ("rgb_colors",)}
    p = dict(params, **leaves)
    outs = map_transform(p, 2, w2c)
    total = sum((o * u).sum() for o, u in zip(outs[:5], ups))
    total.backward()
    ref = {k: v.detach().double().requires_grad_(True) for k, v in params.items() if k in leaves}
    pr = dict({k: v.double() for k, v in params.items()}, **ref)
    tg = slam.transform_to_frame(pr, 2, gaussians_grad=True, camera_grad=False, fast=False)
    rv = slam.transformed_params2rendervar(pr, tg)
    dv = slam.transformed_params2depthplussilhouette(pr, w2c.double(), tg, fast=False)
    outs_ref = (rv["means3D"], rv["rotations"], dv["colors_precomp"], rv["opacities"], rv["scales"])
    for o, r in zip(outs, outs_ref):
        assert _rel(o.detach(), r.detach()) <= 1e-6
    sum((o * u.double()).sum() for o, u in zip(outs_ref, ups)).backward()
    for k in GAUSS_KEYS:
        assert _rel(leaves[k].grad, ref[k].grad) <= 1e-5, k


def _scene_targets(params, cam, cuda):
    """Targets rendered at the unperturbed pose with perturbed colours (so the loss is not ~0)."""
    with torch.no_grad():
        gt = dict(params)
        gt["cam_unnorm_rots"] = torch.zeros_like(params["cam_unnorm_rots"])
        gt["cam_unnorm_rots"][0, 0] = 1.0
        gt["cam_trans"] = torch.zeros_like(params["cam_trans"])
        key = slam.color_key(params)
        gt[key] = params[key] * 0.8 + 0.05
        tg = slam.transform_to_frame(gt, 1, False, False)
        rv = slam._rendervar_colors(gt, slam.transformed_params2rendervar(gt, tg))
        w2c = torch.eye(4, device=cuda)
        im, _, _ = GaussianRasterizer(cam)(**rv)
        ds, _, _ = GaussianRasterizer(cam)(**slam.transformed_params2depthplussilhouette(gt, w2c, tg))
        gd = ds[0:1].clone()
        gd[:, :, :7] = 0.0
    return {"cam": cam, "w2c": w2c, "im": im.clamp(0, 1), "depth": gd}


def _loss_and_grads(params, curr, fused, loss_dtype=None):
    p = dict(params)
    key = slam.color_key(params)
    for k in GAUSS_KEYS + (key,):
        p[k] = params[k].detach().clone().requires_grad_(True)
    loss, radius, _ = slam.get_loss_mapping(p, curr, 1, fused=fused, loss_dtype=loss_dtype)
    loss.backward()
    return loss.item(), {k: p[k].grad for k in GAUSS_KEYS + (key,)}, radius


def _rows_close(a, r, tol=1e-4):
    """Per-Gaussian relative error of the gradient rows (per-element checks on
    Gaussians away from thresholds) -> (fraction of rows within tol, rel L2 over those rows)."""
    a, r = a.double().reshape(a.shape[0], -1), r.double().reshape(r.shape[0], -1)
    rn = r.norm(dim=1)
    row = (a - r).norm(dim=1) / (rn + 1e-3 * rn.mean() + 1e-30)
    ok = row <= tol
    return float(ok.float().mean()), _rel(a[ok], r[ok])


@pytest.mark.parametrize("aniso,sh", [(False, False), (True, False), (True, True)])
def test_get_loss_mapping_fused_equals_literal(cuda, aniso, sh):
    """Fused mapping iteration (HIP transform, dual render, fused SSIM/L1) vs the
    literal one (torch glue, two GaussianRasterizer calls, conv2d SSIM with its loss
    terms in float64, so the reference carries no float32 convolution error).

    Loss within 1e-5 relative.  Gradients: the HIP transform's camera-frame means
    differ from the matmul formulation by an ulp, which flips alpha / transmittance
    thresholds for a few (pixel, Gaussian) pairs, and the gradient of a Gaussian in
    such a pair jumps; so >= 98 % of Gaussians must agree per row within 1e-4, and
    those rows within 1e-5 relative L2.  Isotropic maps: the rotation gradient is
    zero in exact arithmetic (both sides hold rounding noise), so only its size is
    checked."""
    _, params, cam = _map_params(cuda, aniso, sh)
    curr = _scene_targets(params, cam, cuda)
    assert slam.fused_mapping_eligible(params, curr, slam.MappingConfig())
    l0, g0, r0 = _loss_and_grads(params, curr, fused=False, loss_dtype=torch.float64)
    l1, g1, r1 = _loss_and_grads(params, curr, fused=True)
    assert abs(l0 - l1) <= 1e-5 * abs(l0), (l0, l1)
    assert float((r0 == r1).float().mean()) >= 0.999
    for k in g0:
        if k == "unnorm_rotations" and not aniso:
            scale = float(g0["means3D"].abs().max())
            assert float(g1[k].abs().max()) <= 1e-4 * scale and float(g0[k].abs().max()) <= 1e-4 * scale
            continue
        assert float(g0[k].abs().sum()) > 0.0, k
        frac, rel = _rows_close(g1[k], g0[k])
        assert frac >= 0.98 and rel <= 1e-5, (k, frac, rel)


def test_fused_adam_matches_torch(cuda):
    """FusedAdam (gsr_adam_step) vs torch.optim.Adam over 5 steps: several groups, sizes
    that are not multiples of 4, a 16-byte-misaligned tensor (scalar path), eps 1e-15."""
    g = torch.Generator().manual_seed(1)
    base = torch.randn(10001, generator=g).to(cuda)
    shapes = {"a": (1000, 3), "b": (777,), "c": (33, 16, 3), "d": None}
    ps = {k: torch.randn(*s, generator=g).to(cuda) for k, s in shapes.items() if s}
    ps["d"] = base[1:5001]
    lrs = {"a": 1e-4, "b": 0.05, "c": 0.0025, "d": 0.001}
    mine = {k: v.clone() for k, v in ps.items()}
    mine["d"] = base.clone()[1:5001]  # 4-byte offset view: contiguous, not 16-byte aligned (scalar path)
    assert mine["d"].data_ptr() % 16 != 0
    ref = {k: v.clone() for k, v in ps.items()}
    opt_m = FusedAdam([{"params": [mine[k]], "lr": lrs[k]} for k in ps], lr=0.0, eps=1e-15)
    opt_r = torch.optim.Adam([{"params": [ref[k]], "lr": lrs[k]} for k in ps], lr=0.0, eps=1e-15)
    for s in range(5):
        for k in ps:
            gr = torch.randn(ps[k].shape, generator=g).to(cuda) * (10.0 ** (s - 2))
            mine[k].grad, ref[k].grad = gr.clone(), gr.clone()
        opt_m.step()
        opt_r.step()
    for k in ps:
        torch.testing.assert_close(mine[k], ref[k], rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(opt_m.state[mine[k]]["exp_avg_sq"], opt_r.state[ref[k]]["exp_avg_sq"],
                                   rtol=1e-6, atol=1e-12)
        assert float(opt_m.state[mine[k]]["step"]) == 5.0


@pytest.mark.parametrize("sh", [False, True])
def test_fused_map_adam_follows_eager_optimizer(cuda, sh):
    """Three fused mapping iterations with the Adam step inside the transform backward
    (MapAdam) follow three fused iterations whose .grad is stepped by torch.optim.Adam
    (mapping lrs, eps 1e-15).  The first step sees bitwise-equal gradients; later steps
    start from parameters one rounding apart, and with eps = 1e-15 an element whose
    gradient is pure rounding noise may step with the other sign (2 lr apart)."""
    _, params, cam = _map_params(cuda, True, sh)
    curr = _scene_targets(params, cam, cuda)
    cfg = slam.MappingConfig()
    key = slam.color_key(params)
    keys = GAUSS_KEYS + (key,)
    fused_p = {k: v.clone() for k, v in params.items()}
    for k in keys:  # the fused step runs in the transform's backward: autograd must reach it
        fused_p[k].requires_grad_(True)
    adam = MapAdam(fused_p, cfg.lrs, color_key=key)
    eager_p = {k: v.clone() for k, v in params.items()}
    for k in keys:
        eager_p[k].requires_grad_(True)
    opt = torch.optim.Adam([{"params": [eager_p[k]], "lr": cfg.lrs[k]} for k in keys], lr=0.0, eps=1e-15)
    for it in range(3):
        loss, _, _ = slam.get_loss_mapping(fused_p, curr, 1, cfg, fused=True, adam=adam)
        loss.backward()
        opt.zero_grad(set_to_none=True)
        loss_e, _, _ = slam.get_loss_mapping(eager_p, curr, 1, cfg, fused=True)
        loss_e.backward()
        opt.step()
        if it == 0:
            for k in keys:
                torch.testing.assert_close(fused_p[k], eager_p[k].detach(), rtol=1e-6, atol=1e-7)
    assert adam.step == 3
    for k in keys:
        moved = (eager_p[k].detach() - params[k]).abs()
        assert float(moved.max()) > 0.0, k
        err = (fused_p[k] - eager_p[k].detach()).abs()
        close = err <= 1e-6 * params[k].abs() + 1e-7
        assert float(close.float().mean()) >= 0.999, (k, float(close.float().mean()))
        assert float(err.max()) <= 6.0 * cfg.lrs[k] + 1e-6, k


def _keyframes(params, cam, cuda, K=3):
    kfs = []
    with torch.no_grad():
        key = slam.color_key(params)
        truth = dict(params)
        truth[key] = params[key] * 0.8 + 0.05
        w2c = torch.eye(4, device=cuda)
        for t in range(K):
            tg = slam.transform_to_frame(truth, t, False, False)
            im, _, _ = GaussianRasterizer(cam)(**slam._rendervar_colors(truth, slam.transformed_params2rendervar(
                truth, tg)))
            ds, _, _ = GaussianRasterizer(cam)(**slam.transformed_params2depthplussilhouette(truth, w2c, tg))
            kfs.append({"cam": cam, "w2c": w2c, "im": im.clamp(0, 1), "depth": ds[0:1].clone(), "id": t})
    return kfs


@pytest.mark.parametrize("sh", [False, True])
def test_graph_mapper_matches_eager_iterations(cuda, sh):
    """Two replays of a 6-iteration mapping graph (fresh optimizer per replay, keyframes drawn per
    replay and gathered into the captured iterations' slots) follow the same 2 x 6 eager fused
    iterations with MapAdam over the drawn keyframes."""
    from splatam_amd.mapper import GraphMapper
    _, params, cam = _map_params(cuda, True, sh)
    kfs = _keyframes(params, cam, cuda)
    key = slam.color_key(params)
    keys = GAUSS_KEYS + (key,)
    g_p = {k: v.clone() for k, v in params.items()}
    e_p = {k: v.clone() for k, v in params.items()}
    for k in keys:
        g_p[k].requires_grad_(True)
        e_p[k].requires_grad_(True)
    mapper = GraphMapper(g_p, kfs, iters_per_graph=6, seed=7, prune=False)
    assert mapper.redraw
    for k in keys:  # construction (warm-up) leaves the parameters untouched
        assert torch.equal(g_p[k].detach(), params[k]), k
    seqs = []
    for _ in range(2):
        mapper.run()
        seqs.append(list(mapper.sequence))
    torch.cuda.synchronize()
    assert not mapper.overflowed()
    rs = np.random.RandomState(7)  # the reference's per-iteration draws (splatam.py:851)
    assert seqs == [[int(rs.randint(0, len(kfs))) for _ in range(6)] for _ in range(2)]
    assert seqs[0] != seqs[1] and len(set(seqs[0] + seqs[1])) > 1
    adam = MapAdam(e_p, slam.MappingConfig().lrs, color_key=key)
    for seq in seqs:
        adam.reset()
        for j in seq:
            kf = kfs[j]
            loss, _, _ = slam.get_loss_mapping(e_p, kf, kf["id"], fused=True, adam=adam)
            loss.backward()
    for k in keys:
        moved = (e_p[k].detach() - params[k]).abs()
        assert float(moved.max()) > 0.0, k
        err = (g_p[k].detach() - e_p[k].detach()).abs()
        close = err <= 1e-6 * params[k].abs() + 1e-7
        assert float(close.float().mean()) >= 0.995, (k, float(close.float().mean()))


def test_graph_mapper_overflow_halts_and_raises(cuda):
    """An overflowing mapping forward skips its Adam step and halts every later step of the frame
    (MapAdam.halted_word, sticky on the device), so the parameters stay those of the last good
    iteration; run() checks by default and raises, run(check=False) leaves overflowed() to report it."""
    from splatam_amd.mapper import GraphMapper
    _, params, cam = _map_params(cuda, True, False)
    kfs = _keyframes(params, cam, cuda)
    key = slam.color_key(params)
    keys = GAUSS_KEYS + (key,)
    p = {k: v.clone() for k, v in params.items()}
    for k in keys:
        p[k].requires_grad_(True)
    mapper = GraphMapper(p, kfs, iters_per_graph=4, seed=3, headroom=1.0, min_extra=0, prune=False)
    with torch.no_grad():
        p["log_scales"].add_(1.0)  # 2.7x larger footprints: far more tile instances than the capacity
    before = {k: p[k].detach().clone() for k in keys}
    with pytest.raises(RuntimeError, match="capacity"):
        mapper.run()
    for k in keys:
        assert torch.equal(p[k].detach(), before[k]), k
    assert mapper.adam.halted()
    mapper.run(check=False)
    torch.cuda.synchronize()
    assert mapper.overflowed()


def test_map_adam_halted_skips_later_steps(cuda):
    """A set halted word (an earlier skipped step of the frame) makes the fused steps of a valid
    iteration skip too: nothing moves until reset()."""
    _, params, cam = _map_params(cuda, True, False)
    kfs = _keyframes(params, cam, cuda, K=1)
    key = slam.color_key(params)
    keys = GAUSS_KEYS + (key,)
    p = {k: v.clone() for k, v in params.items()}
    for k in keys:
        p[k].requires_grad_(True)
    adam = MapAdam(p, slam.MappingConfig().lrs, color_key=key)
    adam.halted_word.fill_(1)
    loss, _, _ = slam.get_loss_mapping(p, kfs[0], 0, fused=True, adam=adam)
    loss.backward()
    for k in keys:
        assert torch.equal(p[k].detach(), params[k]), k
    adam.reset()
    assert not adam.halted()
    loss, _, _ = slam.get_loss_mapping(p, kfs[0], 0, fused=True, adam=adam)
    loss.backward()
    assert not torch.equal(p["means3D"].detach(), params["means3D"])


def test_fused_adam_through_gaussian_surgery(cuda):
    """FusedAdam keeps torch's state layout, so SplaTAM's optimizer surgery (remove_points /
    cat_params_to_optimizer, slam_external.py:122-163) works on it: after pruning and
    appending Gaussians, further steps match torch.optim.Adam put through the same surgery."""
    from splatam_amd import surgery
    g = torch.Generator().manual_seed(4)
    base = {"means3D": torch.randn(300, 3, generator=g), "logit_opacities": torch.randn(300, 1, generator=g),
            "log_scales": torch.randn(300, 3, generator=g) - 3}
    lrs = {"means3D": 1e-4, "logit_opacities": 0.05, "log_scales": 1e-3}
    runs = []
    for cls in (FusedAdam, torch.optim.Adam):
        params = {k: torch.nn.Parameter(v.clone().to(cuda)) for k, v in base.items()}
        opt = cls([{"params": [v], "name": k, "lr": lrs[k]} for k, v in params.items()], lr=0.0, eps=1e-15)
        gg = torch.Generator().manual_seed(5)
        for s in range(4):
            for k, v in params.items():
                v.grad = torch.randn(v.shape, generator=gg).to(cuda)
            opt.step()
            if s == 1:
                keep = torch.arange(params["means3D"].shape[0], device=cuda) % 3 != 0
                params, _ = surgery.remove_points(~keep, params, {}, opt)
                new = {k: v.detach()[:10] * 1.5 for k, v in params.items()}
                params = surgery.cat_params_to_optimizer(new, params, opt)
        runs.append(params)
    for k in base:
        assert runs[0][k].shape == runs[1][k].shape
        torch.testing.assert_close(runs[0][k].detach(), runs[1][k].detach(), rtol=1e-6, atol=1e-7)


def test_sh_colour_adam_fused_bitwise(cuda, monkeypatch):
    """The colour group's Adam step inside the rasterizer's SH backward stage
    (gsr_backward_dual_sh_adam) against the same step in gsr_map_transform_bwd_adam after the
    gradient's HBM round trip: parameters and optimizer moments bitwise equal after three
    iterations (same element update, same gradients)."""
    _, params, cam = _map_params(cuda, True, True)
    curr = _scene_targets(params, cam, cuda)
    cfg = slam.MappingConfig()
    key = slam.color_key(params)
    assert key == "shs"
    keys = GAUSS_KEYS + (key,)
    out = []
    for fused in (False, True):
        monkeypatch.setattr(slam, "_SH_ADAM_FUSED", fused)
        p = {k: v.clone() for k, v in params.items()}
        for k in keys:
            p[k].requires_grad_(True)
        adam = MapAdam(p, cfg.lrs, color_key=key)
        for _ in range(3):
            loss, _, _ = slam.get_loss_mapping(p, curr, 1, cfg, fused=True, adam=adam)
            loss.backward()
        assert adam.step == 3
        out.append(({k: p[k].detach().clone() for k in keys}, [t.clone() for t in adam.exp_avg + adam.exp_avg_sq]))
    (p0, s0), (p1, s1) = out
    for k in keys:
        assert torch.equal(p0[k], p1[k]), k
        assert float((p1[k] - params[k]).abs().max()) > 0.0, k
    for a, b in zip(s0, s1):
        assert torch.equal(a, b)


@pytest.mark.parametrize("sh", [False, True])
def test_graph_mapper_tile_cull_bitwise(cuda, sh):
    """Tile culling (gsr_settings.binning, culled by default) in the captured mapping frame: parameters after
    two 6-iteration replays are bitwise those of the same frame with culling off (static dual forward, SH or
    RGB colours, the 10-sum render backward, gauss_bwd skipping the culled record slots)."""
    from splatam_amd import _C
    from splatam_amd.mapper import GraphMapper
    _, params, cam = _map_params(cuda, True, sh)
    kfs = _keyframes(params, cam, cuda)
    key = slam.color_key(params)
    keys = GAUSS_KEYS + (key,)
    res = {}
    for mode in (0, 3):  # 0: the reference's lists (reference_binning), 3: culled (the default)
        with (_C.reference_binning() if mode == 0 else contextlib.nullcontext()):
            p = {k: v.clone() for k, v in params.items()}
            for k in keys:
                p[k].requires_grad_(True)
            mapper = GraphMapper(p, kfs, iters_per_graph=6, seed=7, prune=False)
        for _ in range(2):
            mapper.run()
        torch.cuda.synchronize()
        assert not mapper.overflowed()
        res[mode] = {k: p[k].detach().clone() for k in keys}
    for k in keys:
        assert float((res[3][k] - params[k]).abs().max()) > 0.0, k
        assert torch.equal(res[0][k], res[3][k]), k


@pytest.mark.parametrize("prune", [False, True])
def test_graph_mapper_transform_in_preprocess_bitwise(cuda, monkeypatch, prune):
    """The mapping transform formed inside the static forward's preprocess (gsr_forward_dual_static_xf, RGB
    colours) against its own launch (gsr_track_transform_fwd) ahead of gsr_forward_dual_static(_alive): after two
    6-iteration replays (with in-frame pruning: the alive mask culls inside the fused preprocess too) the
    parameters are bitwise equal."""
    from splatam_amd.mapper import GraphMapper
    _, params, cam = _map_params(cuda, True, False)
    kfs = _keyframes(params, cam, cuda)
    key = slam.color_key(params)
    assert key != "shs"
    keys = GAUSS_KEYS + (key,)
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(slam, "_MAP_XF_FUSED", fused)
        p = {k: v.clone() for k, v in params.items()}
        for k in keys:
            p[k].requires_grad_(True)
        mapper = GraphMapper(p, kfs, iters_per_graph=6, seed=7, prune=prune, scene_radius=2.0)
        for _ in range(2):
            mapper.run()
        torch.cuda.synchronize()
        assert not mapper.overflowed()
        res[fused] = ({k: p[k].detach().clone() for k in keys}, mapper.alive.clone())
    for k in keys:
        assert float((res[True][0][k] - params[k]).abs().max()) > 0.0, k
        assert torch.equal(res[False][0][k], res[True][0][k]), k
    assert torch.equal(res[False][1], res[True][1])
