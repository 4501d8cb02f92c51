"""The timed workloads against the literal path at the size they are timed.

bench.py times config 3's tracking iteration through GraphTracker (render_track_kernel, the pose-fused
gauss_bwd) and config 4's mapping frame through GraphMapper (SH-Adam backward, SSIM kernels).  Those fused
paths are checked bitwise against other fused forms elsewhere; here they are compared with the LITERAL
path -- scripts/splatam.py:220-353's get_loss through two GaussianRasterizer calls (the drop-in kernels,
pinned to the C oracle in test_gpu_parity / test_gpu_configs) and torch glue pinned to reference-generated
goldens (test_glue_cpu), with torch.optim.Adam -- on the exact maps, poses and targets the bench times
(splatam_amd.workloads).  Statistics are printed (pytest -s) and kept under profiles/.

* config 3, one iteration: loss within 1e-5 relative, pose gradients within 1e-4 (relative L2
  of the gradient vector; the per-component check uses the same bound against the gradient's norm);
* config 3, the tracker's first captured iteration: its loss and the gradient read back from its Adam state
  (m = (1 - beta1) g after the first step) under the same bounds;
* config 3, a 40-iteration frame (configs/replica/splatam.py:59): every iteration of the contracting phase
  (0-9) within 1e-3 in loss and 1e-5 in pose; over the frame the best loss within 2 % (float32 ulps grow
  along the trajectory once the pose oscillates around the minimum; the eager fused loop with torch's Adam
  drifts from the literal one as much: profiles/r9d_track_traj.txt);
* config 4, the mapping transform: outputs and gradients within 1e-6 of autograd through transform_to_frame;
* config 4, the captured frame's first stepping iteration (after a pruning one): loss within 1e-5, every
  parameter gradient (read back from the fused Adam's first moments) within 1e-4 relative L2 of the literal
  iteration's, with the camera-frame rendervars pinned to the same values (an ulp of difference there moves
  the literal gradients by ~2e-2 on this map: alpha / T decisions, profiles/r9f_map_sensitivity.txt);
* config 4, one 60-iteration mapping frame (configs/replica/splatam.py:16) pruning at iterations 0 and 20:
  the same survivors, and per parameter a distance to the literal frame (L2, relative to the frame's step)
  within 2.5x of the distance between two roundings of the literal frame (float32 / float64 loss terms).
"""
import numpy as np
import pytest
import torch

from splatam_amd.scenes import config_scene
from splatam_amd.slam import TrackingConfig, get_loss_tracking
from splatam_amd.workloads import tracking_frame

pytestmark = pytest.mark.gpu


def _pose_leaves(params):
    p = dict(params)
    p["cam_unnorm_rots"] = params["cam_unnorm_rots"].detach().clone().requires_grad_(True)
    p["cam_trans"] = params["cam_trans"].detach().clone().requires_grad_(True)
    return p


def _grads(params, curr, **mode):
    p = _pose_leaves(params)
    loss, _, _ = get_loss_tracking(p, curr, 0, TrackingConfig(), **mode)
    loss.backward()
    return float(loss), p["cam_unnorm_rots"].grad[..., 0].clone(), p["cam_trans"].grad[..., 0].clone()


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


@pytest.fixture(scope="module")
def config3(cuda):
    return tracking_frame(config_scene(3), torch.device(cuda))


def test_config3_fused_iteration_equals_literal(cuda, config3):
    params, curr = config3
    l0, q0, t0 = _grads(params, curr, fast=False)                                   # literal get_loss
    l1, q1, t1 = _grads(params, curr, fast=True, fused=True, dual=True, fuse_pose=True)  # the timed form
    rl, rq, rt = abs(l1 - l0) / abs(l0), _rel(q1, q0), _rel(t1, t0)
    print(f"config3 iteration: loss {l0:.6f} vs {l1:.6f} (rel {rl:.2e}); dq rel {rq:.2e}, dt rel {rt:.2e}")
    assert l0 > 0 and float(q0.abs().sum()) > 0 and float(t0.abs().sum()) > 0
    assert rl <= 1e-5
    assert rq <= 1e-4 and rt <= 1e-4
    assert float((q1 - q0).abs().max()) <= 1e-4 * float(q0.norm())
    assert float((t1 - t0).abs().max()) <= 1e-4 * float(t0.norm())


def test_config3_graph_tracker_first_iteration_equals_literal(cuda, config3):
    from splatam_amd.tracker import GraphTracker
    params, curr = config3
    l0, q0, t0 = _grads(params, curr, fast=False)
    p = _pose_leaves(params)
    tr = GraphTracker(p, curr, 0, iters_per_graph=1, warmup_iters=1, fuse_pose=True)  # bench.py's form
    tr.begin_frame()
    tr.run()
    torch.cuda.synchronize()
    assert not tr.overflowed()
    st = tr.adam.state
    b1 = tr.adam.betas[0]
    gq, gt = st[0:4] / (1.0 - b1), st[8:11] / (1.0 - b1)  # first step: m = (1 - beta1) g
    l1 = float(tr.loss)
    rl, rq, rt = abs(l1 - l0) / abs(l0), _rel(gq, q0), _rel(gt, t0)
    print(f"config3 GraphTracker iteration 1: loss rel {rl:.2e}; dq rel {rq:.2e}, dt rel {rt:.2e}")
    assert int(st[14]) == 1
    assert rl <= 1e-5
    assert rq <= 1e-4 and rt <= 1e-4


def test_config3_tracked_frame_follows_literal(cuda, config3):
    """One whole 40-iteration tracking frame (configs/replica/splatam.py:59): GraphTracker (one iteration per
    replay here, so every iteration's loss and pose can be read) against track_frame_literal (the unchanged
    loop body of scripts/splatam.py:700-763: two GaussianRasterizer calls, torch.optim.Adam over every group,
    the best candidate by loss).

    Float32 summation-order differences (~1e-7 in the first loss) grow along the trajectory once the pose
    oscillates around the minimum (Adam's lr 0.002 on the translation): the eager fused loop with torch's
    Adam drifts from the literal one exactly as much (profiles/r9d_track_traj.txt).  So: every iteration of the
    contracting phase (0-9) within 1e-3 in loss and 1e-5 in pose, over the frame the same best loss within
    2 %, and the written-back pose the post-step pose of the graph's lowest-loss iteration."""
    from splatam_amd.slam import as_parameters, track_frame_literal, tracking_variables
    from splatam_amd.tracker import GraphTracker
    params, curr = config3
    N, NC = 40, 10
    lit = as_parameters(params)
    ll, lit_pose = [], []
    opt = None
    for k in range(N):  # track_frame_literal one iteration at a time, the optimizer kept across them
        lk = []
        opt = track_frame_literal(lit, tracking_variables(params["means3D"].shape[0], cuda), curr, 0, 1,
                                  optimizer=opt, losses_out=lk)
        ll.append(float(lk[0]))
        # (one-iteration frames write back the post-step pose: it is the only candidate)
        lit_pose.append(torch.cat([lit["cam_unnorm_rots"][0, :, 0], lit["cam_trans"][0, :, 0]]).detach().clone())
    kb = min(range(N), key=lambda k: ll[k])
    p = _pose_leaves(params)
    tr = GraphTracker(p, curr, 0, iters_per_graph=1, warmup_iters=1, fuse_pose=True)
    tr.begin_frame()
    lg, g_pose = [], []
    for _ in range(N):
        tr.run()
        torch.cuda.synchronize()
        lg.append(float(tr.loss))
        g_pose.append(torch.cat([p["cam_unnorm_rots"][0, :, 0], p["cam_trans"][0, :, 0]]).detach().clone())
    tr.end_frame()
    assert not tr.overflowed()
    rl = [abs(lg[k] - ll[k]) / ll[k] for k in range(N)]
    dp = [float((g_pose[k] - lit_pose[k]).abs().max()) for k in range(N)]
    for k in range(N):
        print(f"  iteration {k:2d}: literal {ll[k]:12.4f} graph {lg[k]:12.4f} rel {rl[k]:.2e}  |dpose| {dp[k]:.2e}")
    gbest = float(tr.adam.best[0])
    assert gbest == min(lg)
    # the written-back pose is the post-step pose of the lowest-loss iteration (scripts/splatam.py:726-731,
    # 760-763), as the literal loop's is (scoring the two poses would compare the losses of the iterations after
    # two different minima of an oscillating sequence, not the selection)
    kg = lg.index(gbest)
    wb = torch.cat([p["cam_unnorm_rots"][0, :, 0], p["cam_trans"][0, :, 0]]).detach()
    assert torch.equal(wb, g_pose[kg])
    print(f"config3 40-iteration frame: best loss literal {ll[kb]:.4f} (iteration {kb}) graph {gbest:.4f} "
          f"(iteration {kg}); contracting phase max rel {max(rl[:NC]):.2e}, max |dpose| "
          f"{max(dp[:NC]):.2e}")
    assert ll[kb] < 0.1 * ll[0]  # the frame converges
    assert max(rl[:NC]) <= 1e-3 and max(dp[:NC]) <= 1e-5
    assert abs(gbest - ll[kb]) <= 0.02 * ll[kb]


@pytest.fixture(scope="module")
def config4(cuda):
    from splatam_amd.workloads import mapping_workload
    return mapping_workload(config_scene(4), 4, torch.device(cuda), prunable=0.02)


def test_config4_mapping_transform_equals_literal(cuda, config4):
    """The fused mapping transform (gsr_track_transform_fwd / gsr_map_transform_bwd: transform_to_frame +
    the rendervar builders, slam_helpers.py:124-139,234-304) at config 4 against autograd of the literal
    restatement, seeded random upstream gradients: outputs and every parameter gradient within 1e-6 relative."""
    from splatam_amd import glue
    from splatam_amd.mapper import GAUSS_KEYS
    from splatam_amd.slam import _scales, color_key, get_depth_and_silhouette, transform_to_frame
    params, cam, kfs = config4
    key = color_key(params)
    kf = kfs[1]
    P = params["means3D"].shape[0]
    g = torch.Generator(device=cuda).manual_seed(3)
    up = [torch.randn(P, n, device=cuda, generator=g) for n in (3, 4, 3, 1, 3)]
    up[2][:, 1:] = 0.0  # (mapping differentiates the depth channel of [z, 1, z^2] only)

    def leaves():
        return {k: (v.detach().clone().requires_grad_(True) if k in GAUSS_KEYS + (key,) else v.detach().clone())
                for k, v in params.items()}
    a = leaves()
    tg = transform_to_frame(a, kf["id"], gaussians_grad=True, camera_grad=False, fast=False)
    outs = [tg["means3D"], torch.nn.functional.normalize(tg["unnorm_rotations"]),
            get_depth_and_silhouette(tg["means3D"], kf["w2c"], fast=False), torch.sigmoid(a["logit_opacities"]),
            _scales(a)]
    torch.autograd.backward(outs, up)
    b = leaves()
    o = glue.map_transform(b, kf["id"], kf["w2c"], key)
    torch.autograd.backward(list(o[:5]), up)
    for j, name in enumerate(("means3D", "rotations", "depth colours", "opacities", "scales")):
        e = _rel(o[j].detach(), outs[j].detach())
        print(f"  {name}: rel {e:.2e}")
        assert e <= 1e-6, name
    for k in GAUSS_KEYS:
        e = _rel(b[k].grad, a[k].grad)
        print(f"  d{k}: rel {e:.2e}")
        assert e <= 1e-6, k


def test_config4_mapping_gradients_equal_literal(cuda, config4):
    """The timed mapping iteration's loss and gradients at config 4 (1 M anisotropic SH-3 Gaussians,
    1200x680): a captured two-iteration frame -- iteration 0 prunes (its loss forward only), iteration 1 steps --
    whose every gradient is read back from the fused Adam's first moments (m = (1 - beta1) g), against the
    literal loop's iteration 1 (prune_gaussians + remove_points at iteration 0, then get_loss(mapping=True)
    through two GaussianRasterizer calls and loss.backward()).  SURVEY 8(c): relative L2 <= 1e-4 per tensor."""
    from splatam_amd.mapper import GAUSS_KEYS, GraphMapper
    from splatam_amd.slam import MappingConfig, as_parameters, color_key, get_loss_mapping, map_frame_literal, \
        tracking_variables
    params, cam, kfs = config4
    key = color_key(params)
    P0 = params["means3D"].shape[0]
    r = torch.max(kfs[0]["depth"]) / 3.0
    g_p = {k: v.clone() for k, v in params.items()}
    for k in GAUSS_KEYS + (key,):
        g_p[k].requires_grad_(True)
    mapper = GraphMapper(g_p, kfs, iters_per_graph=2, cfg=MappingConfig(), seed=3, scene_radius=r)
    assert sorted(mapper.prune_at) == [0]
    mapper.run()
    torch.cuda.synchronize()
    seq = list(mapper.sequence)
    keep = mapper.survivors()
    assert mapper.adam.step == 1
    lit = as_parameters(params)
    variables = tracking_variables(P0, cuda)
    variables["scene_radius"] = r

    class _Seq:
        def __init__(self, s):
            self.s = list(s)

        def randint(self, lo, hi):
            return self.s.pop(0)

    map_frame_literal(lit, variables, kfs, 1, MappingConfig(), rng=_Seq(seq[:1]))  # the pruning iteration
    assert lit["means3D"].shape[0] == int(keep.sum()) < P0
    kf = kfs[seq[1]]
    # The literal iteration with the camera-frame rendervars taking the fused transform's values (the gradient
    # still flows through the literal transform_to_frame): an ulp of difference in those inputs moves the
    # literal gradients by ~2e-2 relative on this map (alpha / T thresholds: tools/map_grad_diag4.py,
    # profiles/r9f_map_sensitivity.txt), so without this the comparison would measure that, not the kernels.
    # The fused transform itself is compared with transform_to_frame below (test_config4_mapping_transform...).
    from splatam_amd import glue
    from splatam_amd.slam import _rendervar_colors, transformed_params2depthplussilhouette, \
        transformed_params2rendervar, transform_to_frame
    with torch.no_grad():
        fm, fr, fd, _, _, _ = glue.map_transform({k: v.detach() for k, v in lit.items()}, kf["id"], kf["w2c"], key)
    tg = transform_to_frame(lit, kf["id"], gaussians_grad=True, camera_grad=False, fast=False)
    rv = _rendervar_colors(lit, transformed_params2rendervar(lit, tg))
    dv = transformed_params2depthplussilhouette(lit, kf["w2c"], tg, fast=False)
    pin = lambda x, v: x + (v - x).detach()  # noqa: E731  (value v, gradient of x)
    rv["means3D"] = dv["means3D"] = pin(tg["means3D"], fm)
    rv["rotations"] = dv["rotations"] = pin(rv["rotations"], fr)
    dv["colors_precomp"] = pin(dv["colors_precomp"], fd)
    from splatam_amd.rasterizer import GaussianRasterizer
    im, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**rv)
    ds, _, _ = GaussianRasterizer(raster_settings=kf["cam"])(**dv)
    cfg = MappingConfig()
    depth, depth_sq = ds[0:1], ds[2:3]
    unc = (depth_sq - depth ** 2).detach()
    mask = ((kf["depth"] > 0) & (~torch.isnan(depth)) & (~torch.isnan(unc))).detach()
    from splatam_amd.slam import calc_ssim, l1_loss_v1
    loss = cfg.w_im * (0.8 * l1_loss_v1(im, kf["im"]) + 0.2 * (1.0 - calc_ssim(im, kf["im"]))) + \
        cfg.w_depth * torch.abs(kf["depth"] - depth)[mask].mean()
    loss.backward()
    rl = abs(float(mapper.loss) - float(loss)) / float(loss)
    print(f"config4 mapping iteration 1: loss {float(loss):.6f} (literal) vs {float(mapper.loss):.6f} (graph), "
          f"rel {rl:.2e}")
    assert rl <= 1e-5
    b1 = mapper.adam.betas[0]
    for k, m in zip(mapper.adam.keys, mapper.adam.exp_avg):
        g_graph = (m[keep] / (1.0 - b1)).double()
        g_lit = lit[k].grad.double()
        e = float((g_graph - g_lit).norm() / g_lit.norm())
        print(f"  d{k}: rel L2 {e:.2e} (|g| {float(g_lit.norm()):.3e})")
        assert float(g_lit.norm()) > 0.0, k
        assert e <= 1e-4, (k, e)


def test_config4_mapping_frame_follows_literal(cuda, config4):
    """One 60-iteration mapping frame at config 4 (1 M anisotropic SH-3 Gaussians, 1200x680, 4 keyframes,
    2 % of the map faded under the 0.005 pruning threshold): GraphMapper (bench.py's form) against
    map_frame_literal (scripts/splatam.py:841-905: two GaussianRasterizer calls, torch L1 + calc_ssim,
    prune_gaussians + remove_points, torch.optim.Adam) over the same keyframe draws."""
    from splatam_amd.mapper import GAUSS_KEYS, GraphMapper
    from splatam_amd.slam import MappingConfig, as_parameters, color_key, map_frame_literal, tracking_variables
    params, cam, kfs = config4
    key = color_key(params)
    P0 = params["means3D"].shape[0]
    r = torch.max(kfs[0]["depth"]) / 3.0
    g_p = {k: v.clone() for k, v in params.items()}
    for k in GAUSS_KEYS + (key,):
        g_p[k].requires_grad_(True)
    mapper = GraphMapper(g_p, kfs, iters_per_graph=60, cfg=MappingConfig(), seed=3, scene_radius=r)
    assert sorted(mapper.prune_at) == [0, 20]
    mapper.run()
    torch.cuda.synchronize()
    seq = list(mapper.sequence)
    keep = mapper.survivors()
    c_p, _, _ = mapper.compact()
    lit = as_parameters(params)
    variables = tracking_variables(P0, cuda)
    variables["scene_radius"] = r

    class _Seq:  # the mapper's draws through the literal loop's rng.randint
        def __init__(self, s):
            self.s = list(s)

        def randint(self, lo, hi):
            return self.s.pop(0)

    map_frame_literal(lit, variables, kfs, 60, MappingConfig(), rng=_Seq(seq))
    # the spread of the literal frame itself: the same loop with its loss terms in float64 (another, more exact
    # rounding of the same arithmetic).  Over 60 Adam steps rounding-level gradient differences grow (Adam
    # normalises each element's step, so an element whose gradient is rounding noise steps +-lr either way)
    lit64 = as_parameters(params)
    v64 = tracking_variables(P0, cuda)
    v64["scene_radius"] = r
    map_frame_literal(lit64, v64, kfs, 60, MappingConfig(), rng=_Seq(seq), loss_dtype=torch.float64)
    nk = int(keep.sum())
    print(f"config4 mapping frame: {P0 - nk} of {P0} pruned (graph), {P0 - lit['means3D'].shape[0]} (literal)")
    assert lit["means3D"].shape[0] == c_p["means3D"].shape[0] == lit64["means3D"].shape[0] == nk
    assert P0 - nk >= int(0.02 * P0) - 1
    for k in GAUSS_KEYS + (key,):
        b = lit[k].detach().double()
        step = b - params[k][keep].double()
        spread = {}
        for name, x in (("graph", c_p[k]), ("literal64", lit64[k])):
            a = x.detach().double()
            err = (a - b).abs()
            close = err <= 1e-5 * b.abs() + 2e-6
            spread[name] = float(err.norm() / step.norm())
            print(f"  {k} {name:9s}: {100 * float(close.float().mean()):.3f} % within 1e-5 rel + 2e-6; max err "
                  f"{float(err.max()):.3e}; |err| / |step| (L2) {spread[name]:.3e}; 99.9 % of "
                  f"|err| <= {float(torch.quantile(err.flatten()[::97].float(), 0.999)):.3e}")
        assert float(step.abs().max()) > 0.0, k
        # over 60 Adam steps rounding differences grow (Adam normalises each element's step; alpha / T decisions
        # flip): the captured frame stays within 2.5x of the spread between two roundings of the literal frame
        assert spread["graph"] <= 2.5 * spread["literal64"], (k, spread)
