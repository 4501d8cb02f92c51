"""Pruning inside the captured mapping frame and Gaussian-Splatting densification through the drop-in path.

scripts/splatam.py:876-884 runs prune_gaussians (utils/slam_external.py:167-188) and, when enabled,
densify (:191-243) between loss.backward() and optimizer.step() of every mapping iteration.  GraphMapper
keeps P fixed inside its HIP graph: a pruning iteration clears a device alive mask (gsr_map_prune) and
every later forward culls the cleared Gaussians (gsr_forward_dual_static_alive).  These tests check

  * gsr_map_prune's decision against torch's own (sigmoid < threshold, max exp(log_scales) > 0.1 r), on
    values straddling both thresholds;
  * the masked frame against the same fused iterations run eagerly with the Gaussians removed for real
    (remove_points on the parameters and the Adam moments, the optimizer's step count carried over, no
    Adam step at a pruning iteration -- what torch.optim.Adam does after remove_points drops every .grad):
    surviving set, parameters and Adam moments bitwise equal;
  * the surviving set against the literal reference frame (map_frame_literal: torch glue, two
    GaussianRasterizer calls, surgery.prune_gaussians + remove_points, torch.optim.Adam), and its
    parameters within the fused-vs-literal tolerance of tests/test_gpu_mapping.py;
  * densify with the RGB render's own means2D.grad (accumulate_mean2d_gradient) on glue.FusedAdam against
    torch.optim.Adam: the same clone / split / prune set, parameters and moments after the step."""
import numpy as np
import pytest
import torch

from splatam_amd import slam
from splatam_amd.glue import FusedAdam, MapAdam, map_prune, prune_step
from splatam_amd.rasterizer import GaussianRasterizer
from splatam_amd.scenes import make_scene

pytestmark = pytest.mark.gpu

GAUSS_KEYS = ("means3D", "unnorm_rotations", "logit_opacities", "log_scales")
PRUNE6 = dict(start_after=0, remove_big_after=0, stop_after=3, prune_every=3, removal_opacity_threshold=0.005,
              final_removal_opacity_threshold=0.005, reset_opacities=False, reset_opacities_every=500)


def _prunable_params(cuda, sh, P=3000, W=150, H=110, seed=3, anisotropic=True):
    """A mapping map where some Gaussians fall under the opacity threshold now, some after a few
    Adam steps (logit just above it), and some are too big for the scene radius."""
    scene = make_scene(P, W, H, seed=seed, anisotropic=anisotropic, sh_degree=3 if sh else 0)
    params = slam.init_mapping_params(scene, num_frames=3, device=cuda)
    cam = slam.camera_settings(scene.cam, cuda, sh_degree=scene.sh_degree)
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(P, generator=g)
    lo = params["logit_opacities"]
    lo[idx[:150].to(cuda)] = -6.0                                                     # sigmoid 0.0025 < 0.005
    lo[idx[150:300].to(cuda)] = -5.25 + 0.04 * torch.rand(150, 1, generator=g).to(cuda)  # just above it
    params["log_scales"][idx[300:360].to(cuda), -1] = 1.5                               # big Gaussians
    return scene, params, cam


def _keyframes(params, cam, cuda, K=3):
    kfs = []
    with torch.no_grad():
        key = slam.color_key(params)
        truth = dict(params)
        truth[key] = params[key] * 0.8 + 0.05
        truth["logit_opacities"] = params["logit_opacities"] - 0.5  # targets pull the opacities down
        w2c = torch.eye(4, device=cuda)
        for t in range(K):
            tg = slam.transform_to_frame(truth, t, False, False)
            im, _, _ = GaussianRasterizer(cam)(**slam._rendervar_colors(truth, slam.transformed_params2rendervar(
                truth, tg)))
            ds, _, _ = GaussianRasterizer(cam)(**slam.transformed_params2depthplussilhouette(truth, w2c, tg))
            kfs.append({"cam": cam, "w2c": w2c, "im": im.clamp(0, 1), "depth": ds[0:1].clone(), "id": t})
    return kfs


def test_map_prune_decision_matches_torch(cuda):
    """gsr_map_prune clears exactly what slam_external.py:174-181 removes (values at and around both
    thresholds, isotropic and anisotropic scales), and never revives a cleared entry."""
    g = torch.Generator().manual_seed(0)
    P = 200_000
    thr, r = 0.005, torch.tensor(2.7182817, device=cuda)
    lo = (torch.logit(torch.tensor(thr, dtype=torch.float64)).float() + 1e-6 * torch.randn(P, 1, generator=g)).to(cuda)
    lo[:1000] = torch.randn(1000, 1, generator=g).to(cuda) * 4
    big = float((0.1 * r).item())
    for cols in (1, 3):
        ls = (torch.log(torch.tensor(big)) + 1e-6 * torch.randn(P, cols, generator=g)).to(cuda)
        ls[:1000] = torch.randn(1000, cols, generator=g).to(cuda) - 2
        params = {"logit_opacities": lo, "log_scales": ls}
        for use_big in (False, True):
            alive = torch.ones(P, dtype=torch.uint8, device=cuda)
            alive[7] = 0
            map_prune(params, alive, thr, big if use_big else None)
            ref = (torch.sigmoid(lo) < thr).squeeze()
            if use_big:
                ref = torch.logical_or(ref, torch.exp(ls).max(dim=1).values > 0.1 * r)
            ref[7] = True
            assert torch.equal(alive == 0, ref), (cols, use_big, int(((alive == 0) != ref).sum()))
            assert 0 < int(ref.sum()) < P


def _eager_compacted_frame(params, kfs, seq, cfg, big_thr):
    """The fused iterations of one frame with the Gaussians removed for real at the pruning iterations:
    remove_points on the parameters and on MapAdam's moments, the step count carried over, and no
    backward / Adam step at a pruning iteration.  Returns (params, adam, keep mask over the input P)."""
    key = slam.color_key(params)
    keys = GAUSS_KEYS + (key,)
    p = {k: v.detach().clone() for k, v in params.items()}
    for k in keys:
        p[k].requires_grad_(True)
    adam = MapAdam(p, cfg.lrs, color_key=key)
    keep_all = torch.ones(params["means3D"].shape[0], dtype=torch.bool, device=params["means3D"].device)
    for it, j in enumerate(seq):
        kf = kfs[j]
        remove, thr, big, _ = prune_step(it, cfg.pruning_dict)
        loss, _, _ = slam.get_loss_mapping(p, kf, kf["id"], cfg, fused=True, adam=adam)
        if not remove:
            loss.backward()
            continue
        with torch.no_grad():
            to_remove = (torch.sigmoid(p["logit_opacities"]) < thr).squeeze()
            if big:
                to_remove = torch.logical_or(to_remove, torch.exp(p["log_scales"]).max(dim=1).values > big_thr)
            keep = ~to_remove
            for n, k in enumerate(adam.keys):
                p[k] = p[k].detach()[keep].clone().requires_grad_(True)
                adam.exp_avg[n] = adam.exp_avg[n][keep].contiguous()
                adam.exp_avg_sq[n] = adam.exp_avg_sq[n][keep].contiguous()
            idx = keep_all.nonzero().squeeze(1)
            keep_all[idx[~keep]] = False
    return p, adam, keep_all


@pytest.mark.parametrize("sh", [False, True])
def test_graph_mapper_pruning_equals_compacted_frame(cuda, sh):
    """A 6-iteration captured frame pruning at iterations 0 and 3 (the alive mask) against the same fused
    iterations with the pruned Gaussians removed for real: surviving set, parameters and Adam moments
    bitwise equal, and some Gaussians pruned at each pruning iteration."""
    from splatam_amd.mapper import GraphMapper
    _, params, cam = _prunable_params(cuda, sh)
    kfs = _keyframes(params, cam, cuda)
    cfg = slam.MappingConfig(pruning_dict=dict(PRUNE6))
    key = slam.color_key(params)
    g_p = {k: v.clone() for k, v in params.items()}
    for k in GAUSS_KEYS + (key,):
        g_p[k].requires_grad_(True)
    r = torch.max(kfs[0]["depth"]) / 3.0
    mapper = GraphMapper(g_p, kfs, iters_per_graph=6, cfg=cfg, seed=11, scene_radius=r)
    assert sorted(mapper.prune_at) == [0, 3]
    mapper.run()
    torch.cuda.synchronize()
    assert not mapper.overflowed()
    seq = list(mapper.sequence)
    e_p, e_adam, e_keep = _eager_compacted_frame(params, kfs, seq, cfg, mapper.big_thr)
    assert e_adam.step == 4 and mapper.adam.step == 4  # six iterations, two of them pruning ones
    keep = mapper.survivors()
    P0 = params["means3D"].shape[0]
    assert torch.equal(keep, e_keep) and 0 < int(keep.sum()) < P0 - 150
    c_p, c_m, c_v = mapper.compact()
    for n, k in enumerate(e_adam.keys):
        assert torch.equal(c_p[k].detach(), e_p[k].detach()), k
        assert torch.equal(c_m[k], e_adam.exp_avg[n]), k
        assert torch.equal(c_v[k], e_adam.exp_avg_sq[n]), k
    with pytest.raises(RuntimeError):
        mapper.run()


def test_graph_mapper_pruning_follows_literal_frame(cuda):
    """The captured frame against the literal reference frame (map_frame_literal: torch glue, two
    GaussianRasterizer calls, prune_gaussians + remove_points, torch.optim.Adam) over the same keyframe
    sequence: the same Gaussians survive, and their parameters agree within the fused-vs-literal mapping
    tolerance (tests/test_gpu_mapping.py: ulp-level transform differences flip a few alpha / T decisions)."""
    from splatam_amd.mapper import GraphMapper
    _, params, cam = _prunable_params(cuda, False)
    kfs = _keyframes(params, cam, cuda)
    cfg = slam.MappingConfig(pruning_dict=dict(PRUNE6))
    key = slam.color_key(params)
    g_p = {k: v.clone() for k, v in params.items()}
    for k in GAUSS_KEYS + (key,):
        g_p[k].requires_grad_(True)
    r = torch.max(kfs[0]["depth"]) / 3.0
    mapper = GraphMapper(g_p, kfs, iters_per_graph=6, cfg=cfg, seed=5, scene_radius=r)
    mapper.run()
    torch.cuda.synchronize()
    seq = list(mapper.sequence)
    P0 = params["means3D"].shape[0]
    g_vars = slam.tracking_variables(P0, cuda)
    g_vars["max_2D_radius"] += torch.arange(P0, device=cuda, dtype=torch.float32)  # row identity
    keep = mapper.survivors()
    c_p, _, _ = mapper.compact(g_vars)
    # remove_points compacts the per-Gaussian variables too (slam_external.py:155-159): they line up with
    # the compacted map, and the reference's eager get_loss updates max_2D_radius[seen] on them
    Pk = c_p["means3D"].shape[0]
    for k in ("max_2D_radius", "means2D_gradient_accum", "denom", "timestep"):
        assert g_vars[k].shape[0] == Pk, k
    assert torch.equal(g_vars["max_2D_radius"], torch.arange(P0, device=cuda, dtype=torch.float32)[keep])
    loss_after, radius_after, _ = slam.get_loss_mapping(c_p, kfs[0], kfs[0]["id"], cfg, fused=False,
                                                        variables=g_vars)
    assert torch.isfinite(loss_after) and radius_after.shape[0] == Pk
    assert bool(g_vars["seen"].any())
    lit = slam.as_parameters(params)
    variables = slam.tracking_variables(params["means3D"].shape[0], cuda)
    variables["scene_radius"] = r

    class _Seq:  # replays the mapper's draws through the literal loop's rng.randint
        def __init__(self, s):
            self.s = list(s)

        def randint(self, lo, hi):
            return self.s.pop(0)

    slam.map_frame_literal(lit, variables, kfs, 6, cfg, rng=_Seq(seq))
    assert lit["means3D"].shape[0] == c_p["means3D"].shape[0] == int(mapper.survivors().sum())
    for k in GAUSS_KEYS + (key,):
        a, b = c_p[k].detach().double(), lit[k].detach().double()
        err = (a - b).abs()
        close = err <= 1e-5 * b.abs() + 2e-6
        assert float(close.float().mean()) >= 0.99, (k, float(close.float().mean()))


def test_densify_fused_adam_matches_torch_adam(cuda):
    """Gaussian-Splatting densification (slam_external.py:191-243, surgery.densify) fed by the RGB render's
    own means2D.grad through the drop-in GaussianRasterizer, on glue.FusedAdam against torch.optim.Adam:
    statistics accumulated over iterations 0-2, one clone / split / prune step at iteration 2 (after two
    Adam steps, so the moments go through cat_params_to_optimizer / remove_points), then the step: the
    same Gaussians, parameters and moments within Adam's float32 rounding, the same step counts."""
    # isotropic: the reference's split draws exp(log_scales).repeat(n, 3) as [n S, 3] stds (slam_external.py:
    # 214), which holds for SplaTAM's isotropic maps (log_scales [P, 1]) only
    _, params, cam = _prunable_params(cuda, False, seed=5, anisotropic=False)
    kfs = _keyframes(params, cam, cuda)
    dd = dict(start_after=2, remove_big_after=0, stop_after=2, densify_every=2, grad_thresh=2e-4,
              num_to_split_into=2, removal_opacity_threshold=0.005, final_removal_opacity_threshold=0.005,
              reset_opacities_every=3000)
    cfg = slam.MappingConfig(prune_gaussians=False, use_gaussian_splatting_densification=True, densify_dict=dd)
    r = torch.max(kfs[0]["depth"]) / 3.0
    runs = []
    for fused in (True, False):
        p = slam.as_parameters(params)
        variables = slam.tracking_variables(params["means3D"].shape[0], cuda)
        variables["scene_radius"] = r
        # (the reference's densify resizes means2D_gradient_accum / denom / max_2D_radius after its clones and
        # splits but not `timestep`, which its remove_points then indexes with the longer mask -- an IndexError
        # in the reference as in this restatement; SplaTAM's GS densification runs without it)
        del variables["timestep"]
        opt = slam.mapping_optimizer(p, cfg, fused=fused)
        assert isinstance(opt, FusedAdam) == fused
        P0 = p["means3D"].shape[0]
        torch.cuda.manual_seed(1234)  # densify's split samples (torch.normal on the CUDA generator)
        slam.map_frame_literal(p, variables, kfs, 3, cfg, optimizer=opt, rng=np.random.RandomState(2))
        runs.append((p, opt, P0))
    (pf, of, P0), (pt, ot, _) = runs
    assert pf["means3D"].shape[0] == pt["means3D"].shape[0] != P0  # clones / splits / removals happened
    lrs = cfg.lrs
    for k in pf:
        if k in ("cam_unnorm_rots", "cam_trans"):
            continue
        # the surgery happened on bitwise-equal parameters and moments (it follows two steps whose
        # parameters differ by Adam's rounding only, which never moved a clone / split / prune decision:
        # the shapes agree); after the third step an element whose gradient is rounding noise may step
        # with the other sign under eps = 1e-15 (test_gpu_mapping.py::test_fused_map_adam_follows_eager_optimizer)
        # (an isotropic map's rotation gradient is zero in exact arithmetic: both sides step on rounding
        # noise, so only the step bound applies to it)
        a, b = pf[k].detach(), pt[k].detach()
        err = (a - b).abs()
        close = err <= 1e-5 * b.abs() + 1e-6
        assert float(err.max()) <= 6.0 * lrs[k] + 1e-6, (k, float(err.max()))
        if k != "unnorm_rotations":
            assert float(close.float().mean()) >= 0.99, (k, float(close.float().mean()))
        sf, st = of.state[pf[k]], ot.state[pt[k]]
        assert sf["exp_avg"].shape == st["exp_avg"].shape == pf[k].shape
        assert float(sf["step"]) == float(st["step"])
        for m in (("exp_avg", "exp_avg_sq") if k != "unnorm_rotations" else ()):
            e = (sf[m] - st[m]).abs()
            ok = e <= 1e-4 * st[m].abs() + 1e-12
            assert float(ok.float().mean()) >= 0.99, (k, m, float(ok.float().mean()))
