"""SplaTAM tracking iteration on the GPU: the sync-free torch formulation
(get_loss_tracking(fast=True, fused=False)) and the fused HIP glue
(include/gsr_glue.h, fused=True) equal the literal restatement of
scripts/splatam.py:220-353 (fast=False) in loss and pose gradients."""
import contextlib
import pytest
import torch

from splatam_amd.scenes import make_scene
from splatam_amd.slam import camera_settings, get_loss_tracking, init_tracking_params, transform_to_frame, \
    transformed_params2depthplussilhouette, transformed_params2rendervar
from splatam_amd.rasterizer import GaussianRasterizer

pytestmark = pytest.mark.gpu


def _setup(cuda, aniso, scene=None):
    scene = scene if scene is not None else make_scene(5000, 160, 120, seed=3, anisotropic=aniso)
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


MODES = {"literal": dict(fast=False), "torch_fast": dict(fast=True, fused=False),
         "fused": dict(fast=True, fused=True, dual=False), "fused_dual": dict(fast=True, fused=True, dual=True),
         "fused_pose": dict(fast=True, fused=True, dual=True, fuse_pose=True)}


def _run(params, curr, mode):
    rots = params["cam_unnorm_rots"].detach().clone().requires_grad_(True)
    trans = params["cam_trans"].detach().clone().requires_grad_(True)
    p = dict(params, cam_unnorm_rots=rots, cam_trans=trans)
    loss, radius, means2D = get_loss_tracking(p, curr, 1, **MODES[mode])
    loss.backward()
    return loss.item(), rots.grad.clone(), trans.grad.clone(), radius, (means2D.grad if means2D is not None else None)


@pytest.mark.parametrize("aniso", [False, True])
@pytest.mark.parametrize("mode", ["torch_fast", "fused", "fused_dual", "fused_pose"])
def test_glue_equals_literal(cuda, aniso, mode):
    """Loss within 1e-5 relative; pose gradients within 1e-4 (float32 reduction
    order differs; the L1 gradient is sign-based, so a pixel whose residual or
    silhouette sits on a threshold may flip)."""
    params, curr = _setup(cuda, aniso)
    if mode.startswith("fused"):
        from splatam_amd.slam import TrackingConfig, fused_eligible
        assert fused_eligible(params, curr, TrackingConfig())
    l0, r0, t0, rad0, m0 = _run(params, curr, "literal")
    l1, r1, t1, rad1, m1 = _run(params, curr, mode)
    assert abs(l0 - l1) <= 1e-5 * abs(l0), (l0, l1)
    torch.testing.assert_close(r1, r0, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(t1, t0, rtol=1e-4, atol=1e-6)
    assert float((rad0 == rad1).float().mean()) >= 0.999
    assert float(l0) > 0.0 and float(r0.abs().sum()) > 0.0
    # means2D gradient of the RGB render (retained by the reference for densification stats);
    # the dual rasterization gives means2D no gradient unless asked for the sum (documented)
    if mode not in ("fused_dual", "fused_pose"):
        assert m1 is not None and float((m1 - m0).norm() / m0.norm()) <= 1e-3


@pytest.mark.parametrize("mode", ["fused_dual", "fused_pose"])
def test_fused_glue_deterministic(cuda, mode):
    params, curr = _setup(cuda, True)
    a = _run(params, curr, mode)
    b = _run(params, curr, mode)
    assert a[0] == b[0] and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])


@pytest.mark.parametrize("mode", ["fused_dual", "fused_pose"])
@pytest.mark.parametrize("aniso", [False, True])
def test_fused_glue_time_index_and_w2c(cuda, mode, aniso):
    """Strided pose column (t = 1 of T = 2) and a non-identity w2c for the depth colours."""
    params, curr = _setup(cuda, aniso)
    w2c = torch.eye(4, device=cuda)
    w2c[:3, 3] = torch.tensor([0.05, -0.02, 0.1], device=cuda)
    curr = dict(curr, w2c=w2c)
    l0, r0, t0, _, _ = _run(params, curr, "literal")
    l1, r1, t1, _, _ = _run(params, curr, mode)
    assert abs(l0 - l1) <= 1e-5 * abs(l0)
    torch.testing.assert_close(r1, r0, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(t1, t0, rtol=1e-4, atol=1e-6)
    assert float(r1[..., 0].abs().sum()) == 0.0 and float(t1[..., 0].abs().sum()) == 0.0


def _pose_leaves(params):
    p = dict(params)
    p["cam_unnorm_rots"] = params["cam_unnorm_rots"].detach().clone().requires_grad_(True)
    p["cam_trans"] = params["cam_trans"].detach().clone().requires_grad_(True)
    return p


@pytest.mark.parametrize("fuse_pose", [False, True])
def test_graph_tracker_matches_eager_iterations(cuda, fuse_pose):
    """HIP-graph replay (static-capacity forward, pose Adam fused into the transform
    backward) follows the pose trajectory of the same number of eager iterations
    with torch.optim.Adam (float rounding of the Adam update differs: 1e-6 abs).
    The construction's warm-up iterations are undone (pose restored, optimizer reset)."""
    from splatam_amd.tracker import GraphTracker
    params, curr = _setup(cuda, False)
    S, W = 6, 2
    pe = _pose_leaves(params)
    opt = torch.optim.Adam([{"params": [pe["cam_unnorm_rots"]], "lr": 0.0004},
                            {"params": [pe["cam_trans"]], "lr": 0.002}], fused=True)
    for _ in range(S):
        opt.zero_grad(set_to_none=True)
        loss, _, _ = get_loss_tracking(pe, curr, 1)
        loss.backward()
        opt.step()
    pg = _pose_leaves(params)
    tr = GraphTracker(pg, curr, 1, iters_per_graph=S, warmup_iters=W, fuse_pose=fuse_pose)
    assert torch.equal(pg["cam_unnorm_rots"].detach(), params["cam_unnorm_rots"])  # warm-up undone
    assert torch.equal(pg["cam_trans"].detach(), params["cam_trans"])
    tr.run()
    torch.cuda.synchronize()
    assert not tr.overflowed()
    assert min(tr.num_rendered()) > 0
    torch.testing.assert_close(pg["cam_unnorm_rots"].detach(), pe["cam_unnorm_rots"].detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(pg["cam_trans"].detach(), pe["cam_trans"].detach(), rtol=1e-5, atol=1e-6)
    assert float(tr.loss) > 0.0


@pytest.mark.parametrize("fuse_pose", [False, True])
def test_graph_tracker_reports_overflow(cuda, fuse_pose):
    from splatam_amd.tracker import GraphTracker
    params, curr = _setup(cuda, False)
    p = _pose_leaves(params)
    tr = GraphTracker(p, curr, 1, iters_per_graph=2, warmup_iters=1, headroom=0.5, min_extra=0,
                      fuse_pose=fuse_pose)
    tr.run()
    torch.cuda.synchronize()
    assert tr.overflowed()
    # every iteration overflowed: its Adam step was skipped on the device (pose and state untouched)
    assert torch.equal(p["cam_unnorm_rots"].detach(), params["cam_unnorm_rots"])
    assert torch.equal(p["cam_trans"].detach(), params["cam_trans"])
    assert float(tr.adam.state.abs().sum()) == 0.0


@pytest.mark.parametrize("scale_cols", [1, 3])
def test_track_transform_marks_gaussian_outputs_non_differentiable(cuda, scale_cols):
    """Only the pose is differentiated in tracking: opacities and scales (and the
    rotations of an isotropic map) carry no gradient, so the rasterizer backward
    picks its lean variant (no dL/dopacity sums, depth-channel-only colours2)."""
    from splatam_amd.glue import track_transform
    params, curr = _setup(cuda, False)
    p = dict(params)
    if scale_cols == 3:
        p["log_scales"] = params["log_scales"].repeat(1, 3).contiguous()
    p["cam_unnorm_rots"] = params["cam_unnorm_rots"].detach().clone().requires_grad_(True)
    p["cam_trans"] = params["cam_trans"].detach().clone().requires_grad_(True)
    means, rots, dcol, opac, scales = track_transform(p, 1, curr["w2c"])
    assert means.requires_grad and dcol.requires_grad
    assert not opac.requires_grad and not scales.requires_grad
    assert rots.requires_grad == (scale_cols == 3)


def test_tracking_l1_seeded_forward_gradient(cuda):
    """tracking_l1(seed=s) forms the loss gradient in the forward launch (one kernel);
    backward(s) returns it, and equals the separate backward kernel bitwise; a backward
    with another seed still computes its own gradient.  Repeated calls reuse the
    self-resetting scratch."""
    from splatam_amd.glue import tracking_l1
    g = torch.Generator(device="cpu").manual_seed(5)
    H, W = 48, 64
    im = torch.rand(3, H, W, generator=g).to(cuda)
    ds = torch.rand(3, H, W, generator=g).to(cuda)
    ds[1] = 1.0
    ds[2] = ds[0] ** 2
    gt_im, gt_d = torch.rand(3, H, W, generator=g).to(cuda), torch.rand(1, H, W, generator=g).to(cuda)
    ref = None
    for _ in range(3):
        a, b = im.clone().requires_grad_(True), ds.clone().requires_grad_(True)
        loss = tracking_l1(a, b, gt_im, gt_d)
        loss.backward(torch.full((), 2.0, device=cuda))
        seed = torch.full((), 2.0, device=cuda)
        a2, b2 = im.clone().requires_grad_(True), ds.clone().requires_grad_(True)
        loss2 = tracking_l1(a2, b2, gt_im, gt_d, seed=seed)
        loss2.backward(seed)
        assert torch.equal(loss, loss2)
        assert torch.equal(a.grad, a2.grad) and torch.equal(b.grad, b2.grad)
        if ref is None:
            ref = (loss.detach().clone(), a.grad.clone())
        assert torch.equal(ref[0], loss2.detach()) and torch.equal(ref[1], a2.grad)
    a3 = im.clone().requires_grad_(True)
    loss3 = tracking_l1(a3, ds, gt_im, gt_d, seed=torch.ones((), device=cuda))
    loss3.backward(torch.full((), 2.0, device=cuda))  # not the seed: computed in backward
    assert torch.equal(a3.grad, ref[1])


@pytest.mark.parametrize("aniso", [False, True])
def test_render_epilogue_l1_matches_separate_kernel(cuda, aniso):
    """gsr_track_forward_dual_static (loss + gradient images in the render epilogue) against the static
    dual forward followed by gsr_track_l1_fwd_bwd: images and gradient images bitwise equal, loss equal
    up to the summation order, and the same backward gradients."""
    from splatam_amd.glue import dual_render_tracking_l1, track_transform, tracking_l1
    from splatam_amd.rasterizer import rasterize_gaussians_dual
    from splatam_amd.slam import TrackingConfig
    params, curr = _setup(cuda, aniso)
    cfg = TrackingConfig()
    seed = torch.ones((), device=cuda)
    outs = []
    for fused in (False, True):
        p = _pose_leaves(params)
        means, rots, dcol, opac, scales = track_transform(p, 1, curr["w2c"])
        status = torch.zeros(4, dtype=torch.int32, device=cuda)
        if fused:
            loss, radii = dual_render_tracking_l1(means, p["rgb_colors"], dcol, opac, scales, rots, curr["cam"],
                                                  400000, status, curr["im"], curr["depth"], cfg, seed)
        else:
            m2 = torch.zeros(means.shape[0], 3, device=cuda)
            im, ds, radii, _ = rasterize_gaussians_dual(means, m2, None, p["rgb_colors"], dcol, opac, scales, rots,
                                                        None, curr["cam"], 400000, status, grad2_channels=1)
            loss = tracking_l1(im, ds, curr["im"], curr["depth"], cfg.sil_thres, cfg.w_im, cfg.w_depth, seed=seed)
        torch.autograd.backward(loss, seed)
        outs.append((float(loss), p["cam_unnorm_rots"].grad.clone(), p["cam_trans"].grad.clone(), radii.clone()))
        assert int(status[0]) <= 400000 and int(status[1]) == 0
    (l0, q0, t0, r0), (l1, q1, t1, r1) = outs
    assert abs(l0 - l1) <= 1e-6 * abs(l0)
    assert torch.equal(r0, r1)
    torch.testing.assert_close(q1, q0, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(t1, t0, rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("aniso", [False, True])
@pytest.mark.parametrize("store", [True, False])
def test_transform_fused_preprocess_bitwise(cuda, aniso, store, monkeypatch):
    """gsr_track_forward_dual_static_xf (the tracking transform inside preprocess)
    against gsr_track_transform_fwd + gsr_track_forward_dual_static: loss, radii and the pose gradients
    bitwise equal, with the camera-frame rendervars stored by the forward (then also bitwise equal to
    the separate transform's) or recomputed by the backward (store_rendervars = 0); on a strided pose
    column (t = 1 of T = 2) with a non-identity w2c."""
    from splatam_amd import glue
    from splatam_amd.slam import TrackingConfig
    params, curr = _setup(cuda, aniso)
    w2c = torch.eye(4, device=cuda)
    w2c[:3, 3] = torch.tensor([0.05, -0.02, 0.1], device=cuda)
    curr = dict(curr, w2c=w2c)
    seed = torch.ones((), device=cuda)
    monkeypatch.setattr(glue, "_XF_STORE", store)
    outs = []
    for fused in (False, True):
        monkeypatch.setattr(glue, "_XF_FUSED", fused)
        p = _pose_leaves(params)
        status = torch.zeros(4, dtype=torch.int32, device=cuda)
        loss, radii = glue.tracking_iteration(p, curr, 1, TrackingConfig(), capacity=400000, status=status, seed=seed)
        saved = loss.grad_fn.saved_tensors  # (.., means, rot, dcol, scales, ..)
        rv = [saved[k].clone() for k in (4, 5, 6, 7)]
        torch.autograd.backward(loss, seed)
        outs.append((loss.detach().clone(), radii.clone(), rv, p["cam_unnorm_rots"].grad.clone(),
                     p["cam_trans"].grad.clone()))
        assert int(status[1]) == 0 and 0 < int(status[0]) <= 400000
    (l0, r0, v0, q0, t0), (l1, r1, v1, q1, t1) = outs
    assert torch.equal(l0, l1) and torch.equal(r0, r1)
    if store:
        for a, b in zip(v0, v1):
            assert torch.equal(a, b)
    assert torch.equal(q0, q1) and torch.equal(t0, t1)
    assert float(q1[..., 1].abs().sum()) > 0.0


@pytest.mark.parametrize("case", ["aniso", "config3"])
def test_track_tile_cull_bitwise(cuda, case, monkeypatch):
    """Tile culling (gsr_settings.binning, culled by default): instances whose alpha >= 1/255 ellipse reaches
    no 4x4 block of their tile are left out of the tile lists.  Against the same static iterations with
    culling off: loss, radii and pose gradients bitwise equal (transform fused or not, render backward fused
    or not), num_rendered (the record count) equal, the longest tile list shorter at config 3."""
    from splatam_amd import glue
    from splatam_amd import _C
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import TrackingConfig
    params, curr = _setup(cuda, case == "aniso", config_scene(3) if case == "config3" else None)
    seed = torch.ones((), device=cuda)
    outs = {}
    for mode in (0, 2):  # 0: the reference's lists (reference_binning), 2: culled (the default)
        with (_C.reference_binning() if mode == 0 else contextlib.nullcontext()):
            for fused, rfused in ((False, False), (True, False), (True, True)):
                monkeypatch.setattr(glue, "_XF_FUSED", fused)
                monkeypatch.setattr(glue, "_RENDER_FUSED", rfused)
                p = _pose_leaves(params)
                status = torch.zeros(4, dtype=torch.int32, device=cuda)
                loss, radii = glue.tracking_iteration(p, curr, 1, TrackingConfig(), capacity=1200000, status=status,
                                                      seed=seed)
                torch.autograd.backward(loss, seed)
                outs[mode, fused, rfused] = (loss.detach().clone(), radii.clone(), p["cam_unnorm_rots"].grad.clone(),
                                             p["cam_trans"].grad.clone(), status.clone())
                assert int(status[1]) == 0
    l0, r0, q0, t0, s0 = outs[0, False, False]
    for (mode, fused, rfused), (l1, r1, q1, t1, s1) in outs.items():
        assert torch.equal(l0, l1) and torch.equal(r0, r1), (mode, fused, rfused)
        assert torch.equal(q0, q1) and torch.equal(t0, t1), (mode, fused, rfused)
        assert int(s1[0]) == int(s0[0])
        assert int(s1[2]) == int(outs[mode, False, False][4][2])
    longest = {m: int(outs[m, True, True][4][2]) for m in (0, 2)}
    print("longest tile list unculled / culled:", longest[0], longest[2])
    assert longest[2] <= longest[0]
    if case == "config3":
        assert longest[2] < 0.85 * longest[0]


@pytest.mark.parametrize("case", ["iso", "aniso", "config3"])
def test_track_render_fused_bitwise(cuda, case, monkeypatch):
    """gsr_track_forward_backward_dual_static_xf (render_track_kernel: a tile's forward + L1 loss and its
    render backward in one workgroup) + gsr_track_backward_dual_records against the separate render_fwd /
    render_bwd launches: loss, radii, images and the pose gradients bitwise equal -- on small scenes and at
    BASELINE config 3 (300 k Gaussians, 640x480: multi-batch tiles, 512- and 1024-key sorts).  The fused
    launch without image stores (images=False, GraphTracker's form) gives the same loss, radii and pose
    gradients."""
    from splatam_amd import glue
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import TrackingConfig
    params, curr = _setup(cuda, case == "aniso", config_scene(3) if case == "config3" else None)
    seed = torch.ones((), device=cuda)
    outs = []
    for fused, images in ((False, True), (True, True), (True, False)):
        monkeypatch.setattr(glue, "_RENDER_FUSED", fused)
        p = _pose_leaves(params)
        status = torch.zeros(4, dtype=torch.int32, device=cuda)
        loss, radii = glue.tracking_iteration(p, curr, 1, TrackingConfig(), capacity=1200000, status=status,
                                              seed=seed, images=images)
        saved = loss.grad_fn.saved_tensors  # (.., im, ds at 13, 14)
        ims = [saved[13].clone(), saved[14].clone()] if images else None
        if not images:
            assert saved[13] is None and saved[14] is None
        assert (getattr(loss.grad_fn, "records", None) is not None) == fused
        torch.autograd.backward(loss, seed)
        outs.append((loss.detach().clone(), radii.clone(), ims, p["cam_unnorm_rots"].grad.clone(),
                     p["cam_trans"].grad.clone()))
        assert int(status[1]) == 0 and 0 < int(status[0]) <= 1200000
    (l0, r0, i0, q0, t0), (l1, r1, i1, q1, t1), (l2, r2, _, q2, t2) = outs
    assert torch.equal(l0, l1) and torch.equal(r0, r1)
    assert torch.equal(i0[0], i1[0]) and torch.equal(i0[1], i1[1])
    assert torch.equal(q0, q1) and torch.equal(t0, t1)
    assert torch.equal(l1, l2) and torch.equal(r1, r2) and torch.equal(q1, q2) and torch.equal(t1, t2)
    assert float(q1[..., 1].abs().sum()) > 0.0


def test_track_render_no_images_needs_its_seed(cuda):
    """tracking_iteration(images=False) stores no images: a backward from another loss seed (which would
    recompute the gradient images from them) raises instead of reading unwritten memory."""
    from splatam_amd import glue
    from splatam_amd.slam import TrackingConfig
    if not glue._RENDER_FUSED:
        pytest.skip("fused tracking render disabled (GSR_TRACK_RENDER_FUSED=0)")
    params, curr = _setup(cuda, False, None)
    seed = torch.ones((), device=cuda)
    p = _pose_leaves(params)
    status = torch.zeros(4, dtype=torch.int32, device=cuda)
    loss, _ = glue.tracking_iteration(p, curr, 1, TrackingConfig(), capacity=400000, status=status, seed=seed,
                                      images=False)
    with pytest.raises(RuntimeError, match="images=False"):
        torch.autograd.backward(loss, 2.0 * seed)
