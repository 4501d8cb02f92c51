"""Fused SplaTAM tracking glue (include/gsr_glue.h, csrc/gsr_glue.hip).

Autograd wrappers around the HIP glue kernels that replace, for the tracking
iteration, the ~300 small torch kernels of

* transform_to_frame(params, t, gaussians_grad=False, camera_grad=True)
  (utils/slam_helpers.py:252-304) and the rendervar builders
  (slam_helpers.py:124-139, 234-249) incl. get_depth_and_silhouette
  (slam_helpers.py:196-213)  ->  ``track_transform``;
* the tracking L1 terms of get_loss (scripts/splatam.py:262-296)  ->  ``tracking_l1``.

Only the camera pose receives gradients from ``track_transform`` (the
Gaussians are detached in tracking).  Like the rasterizer there is no CPU
path: these raise on non-ROCm tensors.
"""
from __future__ import annotations

import ctypes
import os

import torch

from ._lib import lib

# tracking transform fused into the rasterizer's preprocess in the static tracking iteration
# (gsr_track_forward_dual_static_xf); GSR_XF_FUSED=0 runs it as its own launch (A/B, parity tests)
_XF_FUSED = os.environ.get("GSR_XF_FUSED", "1") != "0"
# ... and with it the tracking render backward inside the forward's launch (render_track_kernel,
# gsr_track_forward_backward_dual_static_xf); GSR_TRACK_RENDER_FUSED=0 keeps render_bwd a launch of its own
_RENDER_FUSED = (os.environ.get("GSR_TRACK_RENDER_FUSED", "1") != "0" and
                 hasattr(lib, "gsr_track_forward_backward_dual_static_xf"))
# ... without storing the camera-frame rendervars (the backward recomputes them from the world-frame
# map: gsr_track_backward_dual log_scales); True stores them (tests compare them with the separate transform)
_XF_STORE = False


def _check(rc: int, what: str):
    if rc < 0:
        raise RuntimeError(f"{what}: {lib.gsr_last_error().decode(errors='replace')}")


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _byref(s):
    return ctypes.byref(s) if s is not None else None


def _f32c(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: the fused glue runs on ROCm devices only (no CPU fallback)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name}: expected float32, got {t.dtype}")
    return t.contiguous()


class PoseAdam:
    """torch.optim.Adam (no weight decay / amsgrad) state for one frame's pose,
    stepped inside the transform backward (gsr_track_transform_bwd_adam).

    Optional per-iteration bookkeeping (gsr_pose_track): `status` / `capacity` -- the
    static-mode status row of the iteration's forward (an overflow there skips the step);
    `best` (device [8]: min loss, quaternion, translation) with the iteration's `loss` --
    scripts/splatam.py:726-731's best-candidate selection, done on the device."""

    def __init__(self, device, lr_q=0.0004, lr_t=0.002, betas=(0.9, 0.999), eps=1e-8, track_best=False):
        self.lr_q, self.lr_t, self.betas, self.eps = float(lr_q), float(lr_t), betas, float(eps)
        self.state = torch.zeros(15, dtype=torch.float32, device=device)
        self.best = torch.full((8,), 1e20, dtype=torch.float32, device=device) if track_best else None
        self.loss = None      # the current iteration's loss tensor (set before backward)
        self.status = None    # the current iteration's status row
        self.capacity = 0

    def reset(self):
        """A fresh optimizer (SplaTAM re-creates it per frame) and candidate (current_min_loss = 1e20)."""
        self.state.zero_()
        if self.best is not None:
            self.best.fill_(1e20)

    def track(self, loss_ptr=None):
        """The gsr_pose_track of the current iteration, or None."""
        from ._lib import GsrPoseTrack
        if loss_ptr is None and self.loss is not None:
            loss_ptr = self.loss.data_ptr()
        if self.best is None and self.status is None:
            return None
        return GsrPoseTrack(status=self.status.data_ptr() if self.status is not None else None,
                            capacity=int(self.capacity), loss=loss_ptr if self.best is not None else None,
                            best=self.best.data_ptr() if self.best is not None else None)


_SCRATCH: dict = {}


def _scratch(t: torch.Tensor, n: int) -> torch.Tensor:
    """Zero-filled scratch for the glue reductions (gsr_track_scratch_floats): the kernels
    leave it zero-filled, so one persistent buffer per (device, stream, size) serves every
    call issued on that stream (calls on one stream never overlap)."""
    dev = t.device
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream, int(n))
    buf = _SCRATCH.get(key)
    if buf is None:
        buf = torch.zeros(int(n), dtype=torch.float32, device=dev)
        _SCRATCH[key] = buf
    return buf


class _TrackTransform(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cam_rots, cam_trans, means_world, unnorm_rot, logit_opac, log_scales, w2c, time_idx,
                pose_adam=None):
        cam_rots, cam_trans = _f32c(cam_rots, "cam_unnorm_rots"), _f32c(cam_trans, "cam_trans")
        means_world, unnorm_rot = _f32c(means_world, "means3D"), _f32c(unnorm_rot, "unnorm_rotations")
        logit_opac, log_scales, w2c = _f32c(logit_opac, "logit_opacities"), _f32c(log_scales, "log_scales"), \
            _f32c(w2c, "w2c")
        T = cam_rots.shape[-1]
        if cam_rots.shape != (1, 4, T) or cam_trans.shape != (1, 3, T):
            raise RuntimeError("cam_unnorm_rots / cam_trans must be (1,4,T) / (1,3,T)")
        t = int(time_idx)
        P = means_world.shape[0]
        scols = log_scales.shape[1]
        dev = means_world.device
        f32 = dict(dtype=torch.float32, device=dev)
        means_cam = torch.empty(P, 3, **f32)
        rot = torch.empty(P, 4, **f32)
        dcol = torch.empty(P, 3, **f32)
        opac = torch.empty(P, 1, **f32)
        scales = torch.empty(P, 3, **f32)
        rc = lib.gsr_track_transform_fwd(P, means_world.data_ptr(), unnorm_rot.data_ptr(), logit_opac.data_ptr(),
                                         log_scales.data_ptr(), scols, cam_rots.data_ptr() + 4 * t,
                                         cam_trans.data_ptr() + 4 * t, T, w2c.data_ptr(), means_cam.data_ptr(),
                                         rot.data_ptr(), dcol.data_ptr(), opac.data_ptr(), scales.data_ptr(),
                                         _stream(means_world))
        _check(rc, "track_transform_fwd")
        ctx.set_materialize_grads(False)  # no zero-filled grads for unused outputs
        # one call: a second mark_non_differentiable replaces the first set
        if scols == 1:  # isotropic maps: rotations do not depend on the pose either
            ctx.mark_non_differentiable(opac, scales, rot)
        else:
            ctx.mark_non_differentiable(opac, scales)
        ctx.save_for_backward(cam_rots, cam_trans, means_world, unnorm_rot, means_cam, w2c)
        ctx.meta = (t, T, scols)
        ctx.pose_adam = pose_adam
        return means_cam, rot, dcol, opac, scales

    @staticmethod
    def backward(ctx, g_means, g_rot, g_dcol, _g_opac, _g_scales):
        cam_rots, cam_trans, means_world, unnorm_rot, means_cam, w2c = ctx.saved_tensors
        t, T, scols = ctx.meta
        P = means_world.shape[0]
        none = (None,) * 9
        if g_means is None and g_dcol is None and g_rot is None:
            return none
        if g_means is None:
            g_means = torch.zeros_like(means_cam)
        g_means = g_means.contiguous()
        g_rot = g_rot.contiguous() if (g_rot is not None and scols != 1) else None
        g_dcol = g_dcol.contiguous() if g_dcol is not None else None
        opt = ctx.pose_adam
        if opt is not None:  # optimizer step fused into the backward: the pose is updated in place
            scratch = _scratch(means_world, lib.gsr_track_scratch_floats(P))
            rc = lib.gsr_track_transform_bwd_adam(
                P, means_world.data_ptr(), unnorm_rot.data_ptr(), scols, cam_rots.data_ptr() + 4 * t,
                cam_trans.data_ptr() + 4 * t, T, means_cam.data_ptr(), w2c.data_ptr(), g_means.data_ptr(),
                g_rot.data_ptr() if g_rot is not None else None, g_dcol.data_ptr() if g_dcol is not None else None,
                opt.lr_q, opt.lr_t, float(opt.betas[0]), float(opt.betas[1]), opt.eps, opt.state.data_ptr(),
                scratch.data_ptr(), _byref(opt.track()), _stream(means_world))
            _check(rc, "track_transform_bwd_adam")
            return none
        dq = torch.zeros_like(cam_rots)
        dt = torch.zeros_like(cam_trans)
        scratch = _scratch(means_world, lib.gsr_track_scratch_floats(P))
        rc = lib.gsr_track_transform_bwd(P, means_world.data_ptr(), unnorm_rot.data_ptr(), scols,
                                         cam_rots.data_ptr() + 4 * t, means_cam.data_ptr(), w2c.data_ptr(),
                                         g_means.data_ptr(), g_rot.data_ptr() if g_rot is not None else None,
                                         g_dcol.data_ptr() if g_dcol is not None else None,
                                         dq.data_ptr() + 4 * t, dt.data_ptr() + 4 * t, T, scratch.data_ptr(),
                                         _stream(means_world))
        _check(rc, "track_transform_bwd")
        return dq, dt, None, None, None, None, None, None, None


def track_transform(params: dict, time_idx: int, w2c: torch.Tensor, pose_adam: PoseAdam | None = None):
    """Returns (means3D_cam, rotations, depth_colors [z,1,z^2], opacities, scales) for the tracking
    iteration; differentiable w.r.t. params['cam_unnorm_rots'] / params['cam_trans'] only.  With
    pose_adam, the backward applies the Adam step to the frame's pose in place instead of
    returning its gradient (no .grad, no optimizer kernels)."""
    return _TrackTransform.apply(params["cam_unnorm_rots"], params["cam_trans"], params["means3D"].detach(),
                                 params["unnorm_rotations"].detach(), params["logit_opacities"].detach(),
                                 params["log_scales"].detach(), w2c, int(time_idx), pose_adam)


class _TrackingL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, im, depth_sil, gt_im, gt_depth, sil_thres, w_im, w_depth, seed=None):
        im, depth_sil = _f32c(im, "im"), _f32c(depth_sil, "depth_sil")
        gt_im, gt_depth = _f32c(gt_im, "gt_im"), _f32c(gt_depth, "gt_depth")
        _, H, W = im.shape
        if depth_sil.shape != (3, H, W) or gt_im.shape != (3, H, W) or gt_depth.shape != (1, H, W):
            raise RuntimeError("tracking_l1: expected im/depth_sil/gt_im [3,H,W] and gt_depth [1,H,W]")
        loss = torch.empty((), dtype=torch.float32, device=im.device)
        scratch = _scratch(im, lib.gsr_track_scratch_floats(H * W))
        ctx.pre = None
        if seed is not None:  # the caller's static loss seed: gradient images in the same pass
            seed = _f32c(seed, "seed")
            dim, dds = torch.empty_like(im), torch.empty_like(depth_sil)
            rc = lib.gsr_track_l1_fwd_bwd(H, W, im.data_ptr(), depth_sil.data_ptr(), gt_im.data_ptr(),
                                          gt_depth.data_ptr(), float(sil_thres), float(w_im), float(w_depth),
                                          seed.data_ptr(), loss.data_ptr(), dim.data_ptr(), dds.data_ptr(),
                                          scratch.data_ptr(), _stream(im))
            _check(rc, "track_l1_fwd_bwd")
            ctx.pre = (dim, dds, seed)  # the seed stays referenced: its address cannot be reused
        else:
            rc = lib.gsr_track_l1_fwd(H, W, im.data_ptr(), depth_sil.data_ptr(), gt_im.data_ptr(),
                                      gt_depth.data_ptr(), float(sil_thres), float(w_im), float(w_depth),
                                      loss.data_ptr(), scratch.data_ptr(), _stream(im))
            _check(rc, "track_l1_fwd")
        ctx.save_for_backward(im, depth_sil, gt_im, gt_depth)
        ctx.meta = (float(sil_thres), float(w_im), float(w_depth))
        return loss

    @staticmethod
    def backward(ctx, g):
        if ctx.pre is not None and g.data_ptr() == ctx.pre[2].data_ptr():  # seeded with the forward's seed
            return ctx.pre[0], ctx.pre[1], None, None, None, None, None, None
        im, depth_sil, gt_im, gt_depth = ctx.saved_tensors
        sil_thres, w_im, w_depth = ctx.meta
        _, H, W = im.shape
        g = g.contiguous()
        dim = torch.empty_like(im)
        dds = torch.empty_like(depth_sil)
        rc = lib.gsr_track_l1_bwd(H, W, im.data_ptr(), depth_sil.data_ptr(), gt_im.data_ptr(), gt_depth.data_ptr(),
                                  sil_thres, w_im, w_depth, g.data_ptr(), dim.data_ptr(), dds.data_ptr(), _stream(im))
        _check(rc, "track_l1_bwd")
        return dim, dds, None, None, None, None, None, None


def tracking_l1(im, depth_sil, gt_im, gt_depth, sil_thres=0.99, w_im=0.5, w_depth=1.0, seed=None):
    """w_im * sum(mask*|gt_im - im|) + w_depth * sum(mask*|gt_depth - depth|) with SplaTAM's tracking mask.

    seed: optional device scalar that the caller will pass to backward() (a static
    seed, e.g. GraphTracker's ones): the gradient images are then computed in the
    forward pass, from the seed's value at that time; a backward seeded with any
    other tensor computes them itself."""
    return _TrackingL1.apply(im, depth_sil, gt_im, gt_depth, sil_thres, w_im, w_depth, seed)


# ------------------------------------------------------------------ mapping --
class MapAdam:
    """torch.optim.Adam state of SplaTAM's mapping optimizer (scripts/splatam.py:166-172:
    one group per parameter, eps 1e-15) for the five Gaussian tensors, stepped inside the
    mapping transform backward (gsr_map_transform_bwd_adam).  `step` counts like torch's
    per-parameter state["step"]; SplaTAM re-creates the optimizer for every frame (reset())."""

    def __init__(self, params: dict, lrs: dict, color_key: str = "rgb_colors", betas=(0.9, 0.999), eps=1e-15):
        self.keys = ("means3D", "unnorm_rotations", "logit_opacities", "log_scales", color_key)
        self.exp_avg = [torch.zeros_like(params[k]) for k in self.keys]
        self.exp_avg_sq = [torch.zeros_like(params[k]) for k in self.keys]
        self.lr = [float(lrs[k]) for k in self.keys]
        self.betas, self.eps = (float(betas[0]), float(betas[1])), float(eps)
        self.step = 0
        self.status = None  # the current iteration's static-mode status row (reporting; see `guard`)
        self.capacity = 0
        # (geom_buffer, counters offset, capacity) of the current iteration's static forward, set by
        # rasterize_gaussians_dual(guard_sink=...): the fused steps guard on that call's own counters.
        self.guard = None
        # gsr_map_adam.halted: set on the device when a step is skipped because its forward overflowed;
        # every later fused step of the frame is then skipped too (the host `step` keeps counting, so a
        # later step would otherwise apply bias corrections for a step count the state never reached).
        # reset() clears it; halted() reads it (one host sync).
        self.halted_word = torch.zeros(1, dtype=torch.int32, device=params[self.keys[0]].device)

    def reset(self):
        for t in self.exp_avg + self.exp_avg_sq:
            t.zero_()
        self.step = 0
        self.guard = None
        self.halted_word.zero_()

    def halted(self) -> bool:
        """True if a fused step of this frame was skipped (forward overflow): the frame must be re-run
        from reset() with more binning capacity.  One host sync."""
        return bool(self.halted_word.item() != 0)

    def struct(self):
        from ._lib import GsrMapAdam
        s = GsrMapAdam()
        for k in range(5):
            s.exp_avg[k] = self.exp_avg[k].data_ptr()
            s.exp_avg_sq[k] = self.exp_avg_sq[k].data_ptr()
            s.lr[k] = self.lr[k]
        s.step, s.beta1, s.beta2, s.eps = self.step, self.betas[0], self.betas[1], self.eps
        if self.guard is not None:
            geom, off, cap = self.guard
            s.status, s.capacity = geom.data_ptr() + off, cap
        else:
            s.status = self.status.data_ptr() if self.status is not None else None
            s.capacity = int(self.capacity)
        s.halted = self.halted_word.data_ptr()
        return s


class _MapTransform(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means_world, unnorm_rot, logit_opac, log_scales, colors, cam_rots, cam_trans, w2c, time_idx,
                adam=None, defer=None):
        cam_rots, cam_trans = _f32c(cam_rots, "cam_unnorm_rots"), _f32c(cam_trans, "cam_trans")
        means_world, unnorm_rot = _f32c(means_world, "means3D"), _f32c(unnorm_rot, "unnorm_rotations")
        logit_opac, log_scales = _f32c(logit_opac, "logit_opacities"), _f32c(log_scales, "log_scales")
        colors, w2c = _f32c(colors, "colors"), _f32c(w2c, "w2c")
        T = cam_rots.shape[-1]
        if cam_rots.shape != (1, 4, T) or cam_trans.shape != (1, 3, T):
            raise RuntimeError("cam_unnorm_rots / cam_trans must be (1,4,T) / (1,3,T)")
        t = int(time_idx)
        P = means_world.shape[0]
        scols = log_scales.shape[1]
        if colors.shape[0] != P:
            raise RuntimeError("colour parameters must have one row per Gaussian")
        f32 = dict(dtype=torch.float32, device=means_world.device)
        means_cam, rot, dcol = torch.empty(P, 3, **f32), torch.empty(P, 4, **f32), torch.empty(P, 3, **f32)
        opac, scales = torch.empty(P, 1, **f32), torch.empty(P, 3, **f32)
        if defer is None:
            rc = lib.gsr_track_transform_fwd(P, means_world.data_ptr(), unnorm_rot.data_ptr(), logit_opac.data_ptr(),
                                             log_scales.data_ptr(), scols, cam_rots.data_ptr() + 4 * t,
                                             cam_trans.data_ptr() + 4 * t, T, w2c.data_ptr(), means_cam.data_ptr(),
                                             rot.data_ptr(), dcol.data_ptr(), opac.data_ptr(), scales.data_ptr(),
                                             _stream(means_world))
            _check(rc, "map_transform_fwd")
        else:  # the next forward (rasterize_gaussians_dual(xform=...)) forms and writes the five outputs
            defer.append((means_world, unnorm_rot, logit_opac, log_scales, scols, cam_rots.data_ptr() + 4 * t,
                          cam_trans.data_ptr() + 4 * t, T, w2c, (cam_rots, cam_trans)))
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(means_world, unnorm_rot, logit_opac, log_scales, colors, cam_rots, means_cam, w2c)
        ctx.meta = (t, T, scols)
        ctx.adam = adam
        return means_cam, rot, dcol, opac, scales, colors.view_as(colors)

    @staticmethod
    def backward(ctx, g_means, g_rot, g_dcol, g_opac, g_scales, g_col):
        means_world, unnorm_rot, logit_opac, log_scales, colors, cam_rots, means_cam, w2c = ctx.saved_tensors
        t, T, scols = ctx.meta
        P = means_world.shape[0]
        c = lambda x: x.contiguous() if x is not None else None  # noqa: E731
        p = lambda x: x.data_ptr() if x is not None else None  # noqa: E731
        g_means, g_rot, g_dcol, g_opac, g_scales, g_col = map(c, (g_means, g_rot, g_dcol, g_opac, g_scales, g_col))
        if g_means is None:
            g_means = torch.zeros_like(means_cam)
        adam = ctx.adam
        if adam is not None:  # optimizer step fused into the backward: parameters updated in place
            adam.step += 1
            st = adam.struct()
            ccols = colors.numel() // max(P, 1)
            rc = lib.gsr_map_transform_bwd_adam(
                P, means_world.data_ptr(), unnorm_rot.data_ptr(), logit_opac.data_ptr(), log_scales.data_ptr(), scols,
                colors.data_ptr(), ccols, cam_rots.data_ptr() + 4 * t, T, means_cam.data_ptr(), w2c.data_ptr(),
                g_means.data_ptr(), p(g_rot), p(g_dcol), p(g_opac), p(g_scales), p(g_col), ctypes.byref(st),
                _stream(means_world))
            _check(rc, "map_transform_bwd_adam")
            return (None,) * 11
        need = ctx.needs_input_grad
        dm = torch.empty_like(means_world)
        du = torch.empty_like(unnorm_rot) if need[1] else None
        dl = torch.empty_like(logit_opac) if need[2] else None
        ds = torch.empty_like(log_scales) if need[3] else None
        rc = lib.gsr_map_transform_bwd(P, unnorm_rot.data_ptr(), logit_opac.data_ptr(), log_scales.data_ptr(), scols,
                                       cam_rots.data_ptr() + 4 * t, T, means_cam.data_ptr(), w2c.data_ptr(),
                                       g_means.data_ptr(), p(g_rot), p(g_dcol), p(g_opac), p(g_scales), dm.data_ptr(),
                                       p(du), p(dl), p(ds), _stream(means_world))
        _check(rc, "map_transform_bwd")
        return (dm if need[0] else None), du, dl, ds, (g_col if need[4] else None), None, None, None, None, None, None


def prune_step(it: int, prune_dict: dict):
    """What prune_gaussians (utils/slam_external.py:167-188) does at mapping iteration `it`:
    (remove, opacity threshold, remove_big, reset_opacities)."""
    pd = prune_dict
    remove = it <= pd["stop_after"] and it >= pd["start_after"] and it % pd["prune_every"] == 0
    thr = pd["final_removal_opacity_threshold"] if it == pd["stop_after"] else pd["removal_opacity_threshold"]
    big = remove and it >= pd["remove_big_after"]
    reset = it <= pd["stop_after"] and it > 0 and it % pd["reset_opacities_every"] == 0 and bool(pd["reset_opacities"])
    return remove, float(thr), big, reset


def map_prune(params: dict, alive: torch.Tensor, opac_thr: float, big_thr: float | None):
    """gsr_map_prune: clear alive[i] where remove_points would drop Gaussian i (slam_external.py:174-181):
    sigmoid(logit_opacities) < opac_thr, or (big_thr given) max exp(log_scales) > big_thr -- big_thr the
    float32 value of 0.1 * variables['scene_radius'].  In place, no host sync (capturable)."""
    lo, ls = _f32c(params["logit_opacities"], "logit_opacities"), _f32c(params["log_scales"], "log_scales")
    P = lo.shape[0]
    if alive.dtype != torch.uint8 or alive.numel() != P or alive.device != lo.device or not alive.is_contiguous():
        raise RuntimeError("alive must be a contiguous uint8 tensor of P entries on the parameters' device")
    rc = lib.gsr_map_prune(P, lo.data_ptr(), ls.data_ptr(), ls.shape[1], float(opac_thr),
                           float(big_thr) if big_thr is not None else 0.0, 1 if big_thr is not None else 0,
                           alive.data_ptr(), _stream(lo))
    _check(rc, "map_prune")


def map_transform(params: dict, time_idx: int, w2c: torch.Tensor, color_key: str = "rgb_colors",
                  adam: MapAdam | None = None, defer: list | None = None):
    """transform_to_frame(params, t, gaussians_grad=True, camera_grad=False) (slam_helpers.py:252-304)
    + the rendervar builders (slam_helpers.py:124-139, 196-213, 234-249) for the mapping iteration.
    Returns (means3D_cam, rotations, depth_colors [z,1,z^2], opacities, scales, colours); differentiable
    w.r.t. the Gaussian parameters.  With `adam` the backward applies the mapping optimizer's step in
    place (no .grad is produced); the parameters must then require grad, or autograd never calls it.
    defer (a list): no launch -- the transform's inputs are appended to it and the next
    rasterize_gaussians_dual(xform=defer[0]) forms the five outputs inside its preprocess (static mode,
    precomputed colours); nothing may read them before that forward."""
    if adam is not None and not params["means3D"].requires_grad:
        raise RuntimeError("map_transform: the fused optimizer step runs in the backward; the Gaussian "
                           "parameters must require grad")
    return _MapTransform.apply(params["means3D"], params["unnorm_rotations"], params["logit_opacities"],
                               params["log_scales"], params[color_key], params["cam_unnorm_rots"].detach(),
                               params["cam_trans"].detach(), w2c, int(time_idx), adam, defer)


class _MappingLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, im, depth_sil, gt_im, gt_depth, w_im, w_depth):
        im, depth_sil = _f32c(im, "im"), _f32c(depth_sil, "depth_sil")
        gt_im, gt_depth = _f32c(gt_im, "gt_im"), _f32c(gt_depth, "gt_depth")
        _, H, W = im.shape
        if depth_sil.shape != (3, H, W) or gt_im.shape != (3, H, W) or gt_depth.shape != (1, H, W):
            raise RuntimeError("mapping_loss: expected im/depth_sil/gt_im [3,H,W] and gt_depth [1,H,W]")
        loss = torch.empty((), dtype=torch.float32, device=im.device)
        state = torch.empty(lib.gsr_map_loss_state_floats(H, W), dtype=torch.float32, device=im.device)
        scratch = _scratch(im, lib.gsr_map_loss_scratch_floats(H, W))
        rc = lib.gsr_map_loss_fwd(H, W, im.data_ptr(), depth_sil.data_ptr(), gt_im.data_ptr(), gt_depth.data_ptr(),
                                  float(w_im), float(w_depth), loss.data_ptr(), state.data_ptr(), scratch.data_ptr(),
                                  _stream(im))
        _check(rc, "map_loss_fwd")
        ctx.save_for_backward(im, depth_sil, gt_im, gt_depth, state)
        ctx.meta = (float(w_im), float(w_depth))
        return loss

    @staticmethod
    def backward(ctx, g):
        im, depth_sil, gt_im, gt_depth, state = ctx.saved_tensors
        w_im, w_depth = ctx.meta
        _, H, W = im.shape
        g = g.contiguous()
        dim, dds = torch.empty_like(im), torch.empty_like(depth_sil)
        rc = lib.gsr_map_loss_bwd(H, W, im.data_ptr(), depth_sil.data_ptr(), gt_im.data_ptr(), gt_depth.data_ptr(),
                                  w_im, w_depth, g.data_ptr(), state.data_ptr(), dim.data_ptr(), dds.data_ptr(),
                                  _stream(im))
        _check(rc, "map_loss_bwd")
        return dim, dds, None, None, None, None


def mapping_loss(im, depth_sil, gt_im, gt_depth, w_im=0.5, w_depth=1.0):
    """w_im * (0.8 * l1_loss_v1(im, gt_im) + 0.2 * (1 - calc_ssim(im, gt_im))) + w_depth * masked mean depth L1
    (get_loss with mapping=True, scripts/splatam.py:262-296), one fused SSIM/L1 launch each way."""
    return _MappingLoss.apply(im, depth_sil, gt_im, gt_depth, w_im, w_depth)


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (no weight decay / amsgrad / maximize) whose step is one HIP
    launch per 16 tensors (gsr_adam_step).  State keys and shapes are torch's
    ("step", "exp_avg", "exp_avg_sq"), so SplaTAM's optimizer surgery
    (utils/slam_external.py update_params_and_optimizer / cat_params_to_optimizer /
    remove_points) works on it unchanged."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        from ._lib import GsrAdamTensor
        loss = closure() if closure is not None else None
        batches = {}
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.device.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError("FusedAdam: contiguous float32 ROCm tensors only (no CPU fallback)")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                key = (int(st["step"].item()), group["betas"], group["eps"], p.device)
                batches.setdefault(key, []).append((p, p.grad.contiguous(), st, group["lr"]))
        for (step, betas, eps, dev), items in batches.items():
            for k in range(0, len(items), 16):
                chunk = items[k:k + 16]
                arr = (GsrAdamTensor * len(chunk))()
                for j, (p, g, st, lr) in enumerate(chunk):
                    arr[j].param, arr[j].grad = p.data_ptr(), g.data_ptr()
                    arr[j].exp_avg, arr[j].exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                    arr[j].n, arr[j].lr = p.numel(), float(lr)
                with torch.cuda.device(dev):
                    rc = lib.gsr_adam_step(len(chunk), arr, step, float(betas[0]), float(betas[1]), float(eps),
                                           torch.cuda.current_stream(dev).cuda_stream)
                _check(rc, "adam_step")
        return loss


# ------------------------------------------------- fused tracking iteration --
class _TrackIteration(torch.autograd.Function):
    """One SplaTAM tracking iteration (get_loss(tracking=True), scripts/splatam.py:220-353) whose backward
    is gsr_track_backward_dual: render backward, then the per-Gaussian backward with the pose chain (and
    the pose Adam step) fused in.  Differentiable w.r.t. the pose only, like track_transform."""

    @staticmethod
    def forward(ctx, cam_rots, cam_trans, params, curr, t, cfg, pose_adam, capacity, status, means2D, seed,
                images=True, alive=None):
        from . import _C
        cam = curr["cam"]
        cam_rots, cam_trans = _f32c(cam_rots, "cam_unnorm_rots"), _f32c(cam_trans, "cam_trans")
        mw = _f32c(params["means3D"].detach(), "means3D")
        ur = _f32c(params["unnorm_rotations"].detach(), "unnorm_rotations")
        lo = _f32c(params["logit_opacities"].detach(), "logit_opacities")
        ls = _f32c(params["log_scales"].detach(), "log_scales")
        w2c = _f32c(curr["w2c"], "w2c")
        T = cam_rots.shape[-1]
        P, scols = mw.shape[0], ls.shape[1]
        dev = mw.device
        f32 = dict(dtype=torch.float32, device=dev)
        means, rot, dcol = torch.empty(P, 3, **f32), torch.empty(P, 4, **f32), torch.empty(P, 3, **f32)
        opac, scales = torch.empty(P, 1, **f32), torch.empty(P, 3, **f32)
        rgb = _f32c(params["rgb_colors"].detach(), "rgb_colors")
        gt_im, gt_d = _f32c(curr["im"], "gt_im"), _f32c(curr["depth"], "gt_depth")
        H, W = cam.image_height, cam.image_width
        ctx.pre = None
        if alive is not None and not (seed is not None and capacity > 0 and _XF_FUSED):
            raise RuntimeError("tracking_iteration: an alive mask needs the static, transform-fused form "
                               "(capacity > 0, a static seed)")
        if seed is not None and capacity > 0 and _XF_FUSED:
            # static mode, static seed: the transform inside preprocess (gsr_track_forward_dual_static_xf),
            # loss + gradient images in the render epilogue
            seed = _f32c(seed, "seed")
            scratch = _scratch(mw, lib.gsr_track_forward_scratch_floats(W, H))
            xform = (mw, ur, lo, ls, scols, cam_rots.data_ptr() + 4 * t, cam_trans.data_ptr() + 4 * t, T, w2c,
                     _XF_STORE, alive)
            records = None
            if _RENDER_FUSED:  # (a static seed promises the backward): the render backward in the forward's launch
                records = torch.empty(lib.gsr_track_records_floats(capacity), **f32)
            # images=False (fused render only): the rendered images stay in registers -- the loss and the
            # render backward are in the same launch; nothing reads them afterwards unless the backward is
            # taken from another seed, which then raises
            (n, im, ds, radii, geom, binning, img, _, loss, dim, dds) = _C.track_forward_dual_static(
                cam, means, rgb, dcol, opac, scales, rot, capacity, status, gt_im, gt_d, cfg.sil_thres, cfg.w_im,
                cfg.w_depth, seed, scratch, xform=xform, records=records, images=images or records is None)
            ctx.pre = (dim, dds, seed)
            ctx.records = records
            ctx.save_for_backward(cam_rots, cam_trans, mw, ur, means, rot, dcol, scales, rgb, radii, geom, binning,
                                  img, im, ds, gt_im, gt_d, w2c)
            ctx.meta = (t, T, scols, int(n), cam, cfg)
            ctx.pose_adam = pose_adam
            ctx.loss_ptr = loss.data_ptr()
            ctx.log_scales = None if _XF_STORE else ls  # rendervars not stored: the backward recomputes them
            ctx.mark_non_differentiable(radii)
            ctx.set_materialize_grads(False)
            return loss, radii
        rc = lib.gsr_track_transform_fwd(P, mw.data_ptr(), ur.data_ptr(), lo.data_ptr(), ls.data_ptr(), scols,
                                         cam_rots.data_ptr() + 4 * t, cam_trans.data_ptr() + 4 * t, T, w2c.data_ptr(),
                                         means.data_ptr(), rot.data_ptr(), dcol.data_ptr(), opac.data_ptr(),
                                         scales.data_ptr(), _stream(mw))
        _check(rc, "track_transform_fwd")
        empty = torch.Tensor([])
        if seed is not None and capacity > 0:  # static mode, static seed: loss + gradient images in the render epilogue
            seed = _f32c(seed, "seed")
            scratch = _scratch(mw, lib.gsr_track_forward_scratch_floats(W, H))
            (n, im, ds, radii, geom, binning, img, _, loss, dim, dds) = _C.track_forward_dual_static(
                cam, means, rgb, dcol, opac, scales, rot, capacity, status, gt_im, gt_d, cfg.sil_thres, cfg.w_im,
                cfg.w_depth, seed, scratch)
            ctx.pre = (dim, dds, seed)
            ctx.save_for_backward(cam_rots, cam_trans, mw, ur, means, rot, dcol, scales, rgb, radii, geom, binning,
                                  img, im, ds, gt_im, gt_d, w2c)
            ctx.meta = (t, T, scols, int(n), cam, cfg)
            ctx.pose_adam = pose_adam
            ctx.loss_ptr = loss.data_ptr()  # best-candidate selection reads this iteration's loss
            ctx.log_scales = None
            ctx.mark_non_differentiable(radii)
            ctx.set_materialize_grads(False)
            return loss, radii
        n, im, ds, radii, geom, binning, img, _ = _C.rasterize_gaussians_dual(
            cam.bg, means, rgb, dcol, opac, scales, rot, cam.scale_modifier, empty, cam.viewmatrix, cam.projmatrix,
            cam.tanfovx, cam.tanfovy, cam.image_height, cam.image_width, empty, cam.sh_degree, cam.campos,
            cam.prefiltered, capacity=capacity, status=status)
        loss = torch.empty((), **f32)
        scratch = _scratch(mw, lib.gsr_track_scratch_floats(H * W))
        if seed is not None:  # static loss seed: the loss gradient images in the same pass
            seed = _f32c(seed, "seed")
            dim, dds = torch.empty_like(im), torch.empty_like(ds)
            rc = lib.gsr_track_l1_fwd_bwd(H, W, im.data_ptr(), ds.data_ptr(), gt_im.data_ptr(), gt_d.data_ptr(),
                                          float(cfg.sil_thres), float(cfg.w_im), float(cfg.w_depth), seed.data_ptr(),
                                          loss.data_ptr(), dim.data_ptr(), dds.data_ptr(), scratch.data_ptr(),
                                          _stream(mw))
            ctx.pre = (dim, dds, seed)
        else:
            rc = lib.gsr_track_l1_fwd(H, W, im.data_ptr(), ds.data_ptr(), gt_im.data_ptr(), gt_d.data_ptr(),
                                      float(cfg.sil_thres), float(cfg.w_im), float(cfg.w_depth), loss.data_ptr(),
                                      scratch.data_ptr(), _stream(mw))
        _check(rc, "track_l1")
        ctx.save_for_backward(cam_rots, cam_trans, mw, ur, means, rot, dcol, scales, rgb, radii, geom, binning, img,
                              im, ds, gt_im, gt_d, w2c)
        ctx.meta = (t, T, scols, int(n), cam, cfg)
        ctx.pose_adam = pose_adam
        ctx.loss_ptr = loss.data_ptr()
        ctx.log_scales = None
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)
        return loss, radii

    @staticmethod
    def backward(ctx, g, _g_radii):
        from . import _C
        (cam_rots, cam_trans, mw, ur, means, rot, dcol, scales, rgb, radii, geom, binning, img, im, ds, gt_im, gt_d,
         w2c) = ctx.saved_tensors
        t, T, scols, n, cam, cfg = ctx.meta
        nones = (None,) * 13
        records = getattr(ctx, "records", None)
        if ctx.pre is not None and g is not None and g.data_ptr() == ctx.pre[2].data_ptr():
            dim, dds = ctx.pre[0], ctx.pre[1]
            if records is not None:  # the render backward ran in the forward: its sums are in records
                dim, dds = im, ds    # (placeholders of the right shape: not read)
        else:
            records = None  # another loss seed: the render backward runs from the recomputed gradient images
            if g is None:
                return nones
            if im is None:
                raise RuntimeError("tracking_iteration(images=False) rendered without storing its images: "
                                   "backpropagate the static loss seed it was given")
            H, W = cam.image_height, cam.image_width
            g = g.contiguous()
            dim, dds = torch.empty_like(im), torch.empty_like(ds)
            rc = lib.gsr_track_l1_bwd(H, W, im.data_ptr(), ds.data_ptr(), gt_im.data_ptr(), gt_d.data_ptr(),
                                      float(cfg.sil_thres), float(cfg.w_im), float(cfg.w_depth), g.data_ptr(),
                                      dim.data_ptr(), dds.data_ptr(), _stream(im))
            _check(rc, "track_l1_bwd")
        P = mw.shape[0]
        scratch = _scratch(mw, lib.gsr_track_backward_scratch_floats(P))
        opt = ctx.pose_adam
        rot_in = rot  # the rendered (camera-frame) rotations: their gradient feeds the pose (anisotropic maps)
        if opt is not None:
            _C.track_backward_dual(cam, means, radii, rgb, dcol, scales, rot_in, dim, dds, geom, n, binning, img, mw,
                                   ur, scols, cam_rots.data_ptr() + 4 * t, cam_trans.data_ptr() + 4 * t, T, w2c,
                                   scratch, adam=(opt.lr_q, opt.lr_t, float(opt.betas[0]), float(opt.betas[1]),
                                                  opt.eps, opt.state), track=opt.track(ctx.loss_ptr),
                                   log_scales=ctx.log_scales, records=records)
            return nones
        dq, dt = torch.zeros_like(cam_rots), torch.zeros_like(cam_trans)
        _C.track_backward_dual(cam, means, radii, rgb, dcol, scales, rot_in, dim, dds, geom, n, binning, img, mw, ur,
                               scols, cam_rots.data_ptr() + 4 * t, cam_trans.data_ptr() + 4 * t, T, w2c, scratch,
                               dq_ptr=dq.data_ptr() + 4 * t, dt_ptr=dt.data_ptr() + 4 * t, log_scales=ctx.log_scales,
                               records=records)
        return (dq, dt) + (None,) * 11


def tracking_iteration(params: dict, curr: dict, time_idx: int, cfg, pose_adam: PoseAdam | None = None,
                       capacity: int = 0, status=None, seed=None, images: bool = True, alive=None):
    """get_loss(tracking=True) as one fused forward (transform, dual rasterization, masked L1) whose backward
    runs the render backward and the per-Gaussian backward with the pose chain (+ pose Adam) fused in:
    no per-Gaussian gradient array, no separate pose-reduction launch.  Returns (loss, radii).
    images=False: with the render backward fused into the forward's launch (static mode and seed), the
    rendered images are not stored at all (get_loss reads them only for the loss, formed in the same launch);
    the backward must then be taken from `seed`.  alive (uint8 [P], static form only): the Gaussians with
    alive[i] == 0 are culled (a capacity-padded map's free and pruned slots)."""
    return _TrackIteration.apply(params["cam_unnorm_rots"], params["cam_trans"], params, curr, int(time_idx), cfg,
                                 pose_adam, int(capacity), status, None, seed, bool(images), alive)


class _DualRenderL1(torch.autograd.Function):
    """Static dual rasterization + SplaTAM's tracking L1 loss in one forward
    (gsr_track_forward_dual_static: loss and gradient images from the render epilogue), backward
    through gsr_backward_dual with the precomputed gradient images when seeded with the static seed."""

    @staticmethod
    def forward(ctx, means3D, colors, colors2, opacities, scales, rotations, st, capacity, status, gt_im, gt_depth,
                cfg, seed):
        from . import _C
        H, W = st.image_height, st.image_width
        scratch = _scratch(means3D, lib.gsr_track_forward_scratch_floats(W, H))
        (n, im, ds, radii, geom, binning, img, _, loss, dim, dds) = _C.track_forward_dual_static(
            st, means3D, colors, colors2, opacities, scales, rotations, capacity, status, gt_im, gt_depth,
            cfg.sil_thres, cfg.w_im, cfg.w_depth, seed, scratch)
        ctx.save_for_backward(colors, colors2, means3D, scales, rotations, radii, geom, binning, img, im, ds, gt_im,
                              gt_depth)
        ctx.meta = (st, int(n), cfg)
        ctx.pre = (dim, dds, seed)
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)
        return loss, radii

    @staticmethod
    def backward(ctx, g, _g_radii):
        from . import _C
        colors, colors2, means3D, scales, rotations, radii, geom, binning, img, im, ds, gt_im, gt_d = ctx.saved_tensors
        st, n, cfg = ctx.meta
        if g is None:
            return (None,) * 13
        if g.data_ptr() == ctx.pre[2].data_ptr():
            dim, dds = ctx.pre[0], ctx.pre[1]
        else:
            g = g.contiguous()
            dim, dds = torch.empty_like(im), torch.empty_like(ds)
            rc = lib.gsr_track_l1_bwd(st.image_height, st.image_width, im.data_ptr(), ds.data_ptr(), gt_im.data_ptr(),
                                      gt_d.data_ptr(), float(cfg.sil_thres), float(cfg.w_im), float(cfg.w_depth),
                                      g.data_ptr(), dim.data_ptr(), dds.data_ptr(), _stream(im))
            _check(rc, "track_l1_bwd")
        nd = ctx.needs_input_grad  # (means3D, colors, colors2, opacities, scales, rotations, ...)
        needs = (False, nd[1], nd[2], nd[3], nd[0], False, False, nd[4], nd[5])
        empty = torch.Tensor([])
        (_, g_col, g_col2, g_op, g_m3, _, _, g_sc, g_rot) = _C.rasterize_gaussians_dual_backward(
            st.bg, means3D, radii, colors, colors2, scales, rotations, st.scale_modifier, empty, st.viewmatrix,
            st.projmatrix, st.tanfovx, st.tanfovy, dim, dds, empty, st.sh_degree, st.campos, geom, n, binning, img,
            needs=needs, dl2_channels=1)
        return (g_m3 if nd[0] else None, g_col, g_col2, g_op, g_sc, g_rot) + (None,) * 7


def dual_render_tracking_l1(means3D, colors, colors2, opacities, scales, rotations, raster_settings, capacity, status,
                            gt_im, gt_depth, cfg, seed):
    """(loss, radii) of the tracking iteration's two renders + L1 loss, one static dual rasterization with
    the loss formed in the render epilogue (HIP-graph capturable; check `status` for overflow)."""
    return _DualRenderL1.apply(means3D, colors, colors2, opacities, scales, rotations, raster_settings, int(capacity),
                               status, gt_im, gt_depth, cfg, seed)
