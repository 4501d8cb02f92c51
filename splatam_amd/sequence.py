"""SplaTAM's per-frame loop on one capture: a SLAM sequence whose frames reuse one HIP-graph tracker and one
HIP-graph mapper.

scripts/splatam.py:697-929 runs, per frame t: the constant-velocity pose initialisation (initialize_camera_pose,
:429-448), `num_iters` tracking iterations with the best candidate written back (:700-763), add_new_gaussians
(:384-426: Gaussians from the pixels the map does not explain, appended to every parameter tensor), the mapping
iterations over a keyframe window (:796-905, prune_gaussians inside), and the keyframe bookkeeping.  P changes
every frame, and a captured graph needs fixed shapes, so the per-frame GraphTracker / GraphMapper of
splatam_amd.tracker / splatam_amd.mapper would be rebuilt every frame (probe, warm-up, capture: tens of ms).

Here the map lives in a capacity-padded buffer: every per-Gaussian tensor has `capacity + 1` rows, a device
`alive` mask marks the live ones (the rasterizer culls the others like Gaussians behind the camera: radius 0, no
instances, zero gradients), and `n_live` (device) counts the appended rows.  add_new_gaussians becomes
`densify_static`: the silhouette render, the masks and the point cloud of every pixel on the device, the new
rows scattered to n_live + (their rank among the selected pixels) -- no host synchronisation, no reallocation.
After a frame's pruning, compact_static moves the live rows to the front in order (remove_points without
a reallocation), so the padded map's live rows are always the reference map's rows in its order; the sequence
raises (check()) when the capacity is exhausted.  The tracker renders
from a one-column pose slot and slot targets that each frame fills; the mapper draws from a keyframe window
set per frame (GraphMapper.set_keyframes).  Keyframe selection is the window of the last `window - 1` keyframes
plus the current frame (keyframe_selection_overlap, :820-836, ranks keyframes by the overlap of a random
pixel sample -- control logic outside the rasterizer path, not restated).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .mapper import GAUSS_KEYS, GraphMapper
from .slam import MappingConfig, TrackingConfig, build_rotation, color_key, transform_to_frame, \
    transformed_params2depthplussilhouette
from .tracker import GraphTracker

# dead rows: finite values (the pose-fused backward forms every row's pose partials, zero for culled rows)
_DEAD = {"means3D": 0.0, "rgb_colors": 0.0, "logit_opacities": -20.0, "log_scales": -10.0}


def pad_map(params: dict, capacity: int) -> tuple[dict, torch.Tensor, torch.Tensor]:
    """(padded params, alive uint8 [capacity + 1], n_live int64 [1]): every per-Gaussian tensor copied into
    `capacity + 1` rows (the last one a scatter sink that is never live), the camera tensors as they are."""
    P = params["means3D"].shape[0]
    if P > capacity:
        raise ValueError(f"capacity {capacity} < the map's {P} Gaussians")
    dev = params["means3D"].device
    out = {}
    for k, v in params.items():
        if k in ("cam_unnorm_rots", "cam_trans") or not torch.is_tensor(v) or v.dim() == 0 or v.shape[0] != P:
            out[k] = v
            continue
        t = torch.empty((capacity + 1,) + tuple(v.shape[1:]), dtype=v.dtype, device=dev)
        if k == "unnorm_rotations":
            t.zero_()
            t[:, 0] = 1.0
        else:
            t.fill_(_DEAD.get(k, 0.0))
        t[:P] = v.detach()
        out[k] = t
    alive = torch.zeros(capacity + 1, dtype=torch.uint8, device=dev)
    alive[:P] = 1
    return out, alive, torch.full((1,), P, dtype=torch.int64, device=dev)


def initialize_camera_pose(params: dict, t: int, forward_prop: bool = True):
    """initialize_camera_pose (scripts/splatam.py:429-448): the constant-velocity model from t - 1 and t - 2,
    else the previous pose; device tensor ops only."""
    with torch.no_grad():
        q, tr = params["cam_unnorm_rots"], params["cam_trans"]
        if t > 1 and forward_prop:
            r1, r2 = F.normalize(q[..., t - 1].detach()), F.normalize(q[..., t - 2].detach())
            q[..., t] = F.normalize(r1 + (r1 - r2)).detach()
            t1, t2 = tr[..., t - 1].detach(), tr[..., t - 2].detach()
            tr[..., t] = (t1 + (t1 - t2)).detach()
        else:
            q[..., t] = q[..., t - 1].detach()
            tr[..., t] = tr[..., t - 1].detach()


def frame_pointcloud(params: dict, curr: dict, t: int, intrinsics) -> dict:
    """get_pointcloud + initialize_new_params (scripts/splatam.py:73-124,356-381; projective scales, isotropic)
    for EVERY pixel of the frame: the new Gaussian each pixel would add (world-frame mean from the depth and the
    pose of column t, the pixel's colour, log_scale = log(sqrt((z / mean focal)^2)), opacity logit 0, identity
    rotation)."""
    im, depth = curr["im"], curr["depth"]
    H, W = im.shape[1], im.shape[2]
    fx, fy, cx, cy = intrinsics
    dev = im.device
    with torch.no_grad():
        rot = F.normalize(params["cam_unnorm_rots"][..., t].detach())
        w2c = torch.eye(4, device=dev, dtype=torch.float32)
        w2c[:3, :3] = build_rotation(rot)
        w2c[:3, 3] = params["cam_trans"][..., t].detach()
        # c2w: the rigid transform's closed-form inverse [R^T, -R^T t] (the reference's torch.inverse forms the
        # same matrix by LU; both SplaTAM forms here use this one)
        c2w = torch.eye(4, device=dev, dtype=torch.float32)
        rt = w2c[:3, :3].transpose(0, 1)
        c2w[:3, :3] = rt
        c2w[:3, 3] = -(rt @ w2c[:3, 3])
        xg, yg = torch.meshgrid(torch.arange(W, device=dev).float(), torch.arange(H, device=dev).float(), indexing="xy")
        xx, yy = ((xg - cx) / fx).reshape(-1), ((yg - cy) / fy).reshape(-1)
        z = depth[0].reshape(-1)
        pts4 = torch.stack((xx * z, yy * z, z, torch.ones_like(z)), dim=-1)
        pts = (c2w @ pts4.T).T[:, :3]
        mean3_sq_dist = (z / ((fx + fy) / 2)) ** 2
        n = pts.shape[0]
        return {"means3D": pts.contiguous(), "rgb_colors": im.permute(1, 2, 0).reshape(-1, 3).contiguous(),
                "unnorm_rotations": torch.tensor([1.0, 0.0, 0.0, 0.0], device=dev).repeat(n, 1),
                "logit_opacities": torch.zeros(n, 1, device=dev),
                "log_scales": torch.log(torch.sqrt(mean3_sq_dist))[..., None].contiguous()}


def non_presence_mask(depth_sil: torch.Tensor, gt_depth: torch.Tensor, sil_thres: float) -> torch.Tensor:
    """add_new_gaussians' pixel selection (scripts/splatam.py:391-410), flattened: silhouette below sil_thres,
    or rendered depth behind the measured depth by more than 50x the median depth error; valid depth only."""
    sil = depth_sil[1]
    gt = gt_depth[0]
    rd = depth_sil[0]
    err = torch.abs(gt - rd) * (gt > 0)
    m = (sil < sil_thres) | ((rd > gt) & (err > 50 * err.median()))
    return (m & (gt > 0)).reshape(-1)


def render_depth_sil(params: dict, curr: dict, t: int, alive=None, capacity: int = 0, status=None):
    """The depth / silhouette render of add_new_gaussians (transform_to_frame + the [z, 1, z^2] rendervars,
    slam_helpers.py:234-304) through the rasterizer: static-capacity with the alive mask when given."""
    from .rasterizer import GaussianRasterizer, rasterize_gaussians_dual
    with torch.no_grad():
        tg = transform_to_frame(params, t, gaussians_grad=False, camera_grad=False)
        rv = transformed_params2depthplussilhouette(params, curr["w2c"], tg)
        if alive is None and capacity <= 0:
            ds, _, _ = GaussianRasterizer(raster_settings=curr["cam"])(**rv)
            return ds
        _, ds, _, _ = rasterize_gaussians_dual(rv["means3D"], torch.zeros_like(rv["means3D"]), None,
                                               rv["colors_precomp"], rv["colors_precomp"], rv["opacities"],
                                               rv["scales"], rv["rotations"], None, curr["cam"], capacity, status,
                                               grad2_channels=1, alive=alive)
        return ds


def add_new_gaussians_literal(params: dict, curr: dict, t: int, intrinsics, sil_thres: float = 0.5) -> dict:
    """add_new_gaussians (scripts/splatam.py:384-426) on an unpadded map: the selected pixels' Gaussians
    appended with torch.cat (the reference's reallocation; one host synchronisation for the selection).
    Returns the new params dict (Gaussian tensors new leaves; the camera tensors as they were)."""
    ds = render_depth_sil(params, curr, t)
    mask = non_presence_mask(ds, curr["depth"], sil_thres)
    new = frame_pointcloud(params, curr, t, intrinsics)
    out = dict(params)
    for k, v in new.items():
        out[k] = torch.cat((params[k].detach(), v[mask]), dim=0).requires_grad_(params[k].requires_grad)
    return out


def densify_static(params: dict, alive: torch.Tensor, n_live: torch.Tensor, overflow: torch.Tensor, curr: dict,
                   t: int, intrinsics, sil_thres: float, capacity: int, bin_capacity: int, status):
    """add_new_gaussians on a capacity-padded map, without a host synchronisation: the selected pixels'
    Gaussians (frame_pointcloud) land in rows n_live + rank, every other pixel writes to the sink row
    `capacity`; alive marks the new rows, n_live grows (clamped; `overflow` set when the map is full)."""
    ds = render_depth_sil(params, curr, t, alive, bin_capacity, status)
    with torch.no_grad():
        mask = non_presence_mask(ds, curr["depth"], sil_thres)
        new = frame_pointcloud(params, curr, t, intrinsics)
        incl = torch.cumsum(mask.to(torch.int64), 0)
        dest = n_live + incl - 1
        ok = mask & (dest < capacity)
        dest = torch.where(ok, dest, torch.full_like(dest, capacity))
        for k, v in new.items():
            params[k].data.index_put_((dest,), v)
        alive.index_put_((dest,), ok.to(torch.uint8))
        total = n_live + incl[-1:]
        overflow.logical_or_(total > capacity)
        n_live.copy_(torch.clamp(total, max=capacity))


def compact_static(params: dict, alive: torch.Tensor, n_live: torch.Tensor, capacity: int):
    """remove_points (utils/slam_external.py:141-163) on a capacity-padded map, without a host
    synchronisation or a reallocation: the live rows move, in order, to the front (their rank among the live
    rows; the dead ones to the sink row), alive becomes the prefix [0, count), n_live the count.  The map's
    rows are then those of the compacted reference map, in the same order, so the next frame's densified
    rows land where torch.cat puts them."""
    with torch.no_grad():
        keep = alive.bool()
        rank = torch.cumsum(keep.to(torch.int64), 0) - 1
        dest = torch.where(keep, rank, torch.full_like(rank, capacity))
        for k, v in params.items():
            if k in ("cam_unnorm_rots", "cam_trans") or not torch.is_tensor(v) or v.dim() == 0 or \
                    v.shape[0] != capacity + 1:
                continue
            v.data.index_put_((dest,), v.detach().clone())
        count = rank[-1:] + 1
        alive.copy_((torch.arange(capacity + 1, device=alive.device) < count).to(torch.uint8))
        n_live.copy_(count)


class SlamSequence:
    """Frames of SplaTAM's loop on a capacity-padded map with one GraphTracker and one GraphMapper.

    params: the initial map (SplaTAM's init from frame 0; isotropic, rgb colours) with one pose column per frame;
    frames: per frame {"im", "depth"} targets (all sharing `cam` / `w2c`, the first frame's, like the reference);
    intrinsics (fx, fy, cx, cy).  frame(t) runs one frame; run(frames) a range of them."""

    def __init__(self, params: dict, frames: list, cam, w2c, intrinsics, capacity: int, bin_capacity: int,
                 tracking_iters: int = 40, mapping_iters: int = 60, track_replay: int = 20, window: int = 8,
                 keyframe_every: int = 5, sil_thres: float = 0.5, track_cfg: TrackingConfig = TrackingConfig(),
                 map_cfg: MappingConfig = MappingConfig(), prune: bool | None = None, seed: int = 0,
                 scene_radius=None):
        if color_key(params) != "rgb_colors" or params["log_scales"].shape[1] != 1:
            raise ValueError("SlamSequence: SplaTAM's isotropic rgb map (the tracking fast path's form)")
        if tracking_iters % track_replay:
            raise ValueError("tracking_iters must be a multiple of track_replay")
        self.frames, self.cam, self.w2c, self.intrinsics = frames, cam, w2c, intrinsics
        self.bin_capacity = int(bin_capacity)
        self.tracking_iters, self.mapping_iters, self.window = tracking_iters, mapping_iters, window
        self.keyframe_every, self.sil_thres = keyframe_every, sil_thres
        self.track_replay, self.track_cfg, self.map_cfg, self.prune, self.seed = \
            track_replay, track_cfg, map_cfg, prune, seed
        if scene_radius is None:  # initialize_first_timestep: max depth / scene_radius_depth_ratio (3, the config's)
            scene_radius = frames[0]["depth"].max() / 3.0
        self.scene_radius = scene_radius
        self.keyframes = [self._kf(0)]
        self.rng = np.random.RandomState(seed)
        self.draws = []  # the mapper's keyframe draws per frame (window indices)
        dev = params["means3D"].device
        self.overflow = torch.zeros(1, dtype=torch.bool, device=dev)
        self.dstatus = torch.zeros(4, dtype=torch.int32, device=dev)
        self._build(params, int(capacity))

    def _build(self, params: dict, capacity: int):
        """The padded map of `params` (its per-Gaussian rows live) and the tracker / mapper graphs over it."""
        self.capacity = capacity
        self.params, self.alive, self.n_live = pad_map(params, self.capacity)
        for k in GAUSS_KEYS + ("rgb_colors",):
            self.params[k].requires_grad_(True)
        q, tr = params["cam_unnorm_rots"], params["cam_trans"]
        self.params["cam_unnorm_rots"] = q.detach().clone()
        self.params["cam_trans"] = tr.detach().clone()
        # the tracker's pose slot (one column) and targets: filled per frame; the map tensors as detached views
        # (the same storage: every replay reads the current map; tracking differentiates the pose only)
        self.slot = {k: (v.detach() if k in GAUSS_KEYS + ("rgb_colors",) else v) for k, v in self.params.items()}
        self.slot["cam_unnorm_rots"] = q[..., :1].detach().clone().requires_grad_(True)
        self.slot["cam_trans"] = tr[..., :1].detach().clone().requires_grad_(True)
        f0 = self.frames[0]
        self.slot_curr = {"cam": self.cam, "w2c": self.w2c, "im": f0["im"].clone(), "depth": f0["depth"].clone()}
        self.tracker = GraphTracker(self.slot, self.slot_curr, 0, iters_per_graph=self.track_replay,
                                    cfg=self.track_cfg, warmup_iters=1, fuse_pose=True, alive=self.alive,
                                    capacity=self.bin_capacity)
        self.mapper = GraphMapper(self.params, self.keyframes, iters_per_graph=self.mapping_iters, cfg=self.map_cfg,
                                  seed=self.seed, prune=self.prune, scene_radius=self.scene_radius,
                                  alive=self.alive, capacity=self.bin_capacity)

    def ensure_headroom(self, free: int) -> bool:
        """One host read of n_live: when fewer than `free` rows are left, move the map into a larger buffer
        (max(2 x capacity, n_live + free) rows) and rebuild the two graphs -- the live rows and their order
        unchanged, so the results are the same bits.  Every per-Gaussian launch covers the whole capacity
        (bench.py's sequence leg: 45.6 frames/s at 342 k rows, 27.1 at 1.84 M for the same 293 k live
        Gaussians), so size it to the map and grow on demand.  Returns True when it grew."""
        n = int(self.n_live.item())
        if self.capacity - n >= free:
            return False
        self._build(self.live_params(), max(2 * self.capacity, n + int(free)))
        return True

    def _kf(self, t: int) -> dict:
        return {"cam": self.cam, "w2c": self.w2c, "im": self.frames[t]["im"], "depth": self.frames[t]["depth"], "id": t}

    def track(self, t: int):
        """initialize_camera_pose, then tracking_iters iterations from the pose slot (best candidate written
        back into column t)."""
        p = self.params
        initialize_camera_pose(p, t)
        with torch.no_grad():
            self.slot["cam_unnorm_rots"][..., 0] = p["cam_unnorm_rots"][..., t]
            self.slot["cam_trans"][..., 0] = p["cam_trans"][..., t]
            self.slot_curr["im"].copy_(self.frames[t]["im"])
            self.slot_curr["depth"].copy_(self.frames[t]["depth"])
        self.tracker.track_frame(self.tracking_iters, check=False)
        with torch.no_grad():
            p["cam_unnorm_rots"][..., t] = self.slot["cam_unnorm_rots"][..., 0]
            p["cam_trans"][..., t] = self.slot["cam_trans"][..., 0]

    def densify(self, t: int):
        densify_static(self.params, self.alive, self.n_live, self.overflow, self._kf(t), t, self.intrinsics,
                       self.sil_thres, self.capacity, self.bin_capacity, self.dstatus)

    def map(self, t: int, sequence=None):
        """The mapping frame over the window (the last window - 1 keyframes + frame t), keyframe draws from the
        sequence's numpy stream (np.random.randint, scripts/splatam.py:851) unless `sequence` is given."""
        win = self.keyframes[-(self.window - 1):] + ([self._kf(t)] if self.keyframes[-1]["id"] != t else [])
        self.mapper.set_keyframes(win)
        seq = [int(self.rng.randint(0, len(win))) for _ in range(self.mapping_iters)] if sequence is None else sequence
        self.draws.append(seq)
        self.mapper.run(check=False, sequence=seq)
        if self.mapper.prune_at:  # the frame's pruned Gaussians removed for good (in place, no sync)
            compact_static(self.params, self.alive, self.n_live, self.capacity)
        # keyframes: frame 0 and every keyframe_every-th frame (scripts/splatam.py:907-913)
        if t > 0 and (t + 1) % self.keyframe_every == 0:
            self.keyframes.append(self._kf(t))

    def frame(self, t: int, sequence=None):
        """One frame of scripts/splatam.py:697-929: tracking (t > 0), densification (t > 0), mapping."""
        if t > 0:
            self.track(t)
            self.densify(t)
        self.map(t, sequence)

    def check(self):
        """One host synchronisation: raises if a binning capacity or the map capacity overflowed."""
        if self.tracker.overflowed() or self.mapper.overflowed() or bool(self.overflow.item()):
            raise RuntimeError("SlamSequence: a binning capacity or the map capacity was exceeded")
        st = self.dstatus.cpu()
        if int(st[0]) > self.bin_capacity or int(st[1]) != 0:
            raise RuntimeError("SlamSequence: the densification render overflowed its binning capacity")

    def live_params(self) -> dict:
        """The live rows (slot order) of every per-Gaussian tensor, and the camera tensors."""
        keep = self.alive.bool()
        return {k: (v.detach()[keep] if torch.is_tensor(v) and v.dim() > 0 and v.shape[0] == keep.shape[0] else v)
                for k, v in self.params.items()}


class PerFrameSlam:
    """The same frames in the form a shape-changing map forces on captured graphs: per frame a fresh
    GraphTracker on the frame's pose (probe, warm-up, capture), add_new_gaussians by torch.cat, a fresh
    GraphMapper on the grown map (probe, warm-up, capture) and, after its pruning, compact().  The comparison
    form for SlamSequence (tests/test_gpu_sequence.py; bench.py's sequence leg times both).  bin_capacity None:
    each tracker / mapper probes its own (what a per-frame loop must do); given: every one uses it."""

    def __init__(self, params: dict, frames: list, cam, w2c, intrinsics, tracking_iters: int = 40,
                 mapping_iters: int = 60, track_replay: int = 20, window: int = 8, keyframe_every: int = 5,
                 sil_thres: float = 0.5, track_cfg: TrackingConfig = TrackingConfig(),
                 map_cfg: MappingConfig = MappingConfig(), prune: bool | None = None, scene_radius=None,
                 bin_capacity: int | None = None):
        self.p = {k: v.detach().clone() for k, v in params.items()}
        self.frames, self.cam, self.w2c, self.intrinsics = frames, cam, w2c, intrinsics
        self.tracking_iters, self.mapping_iters, self.track_replay = tracking_iters, mapping_iters, track_replay
        self.window, self.keyframe_every, self.sil_thres = window, keyframe_every, sil_thres
        self.track_cfg, self.map_cfg, self.prune, self.bin_capacity = track_cfg, map_cfg, prune, bin_capacity
        self.scene_radius = frames[0]["depth"].max() / 3.0 if scene_radius is None else scene_radius
        self.keyframes = [self._kf(0)]

    def _kf(self, t: int) -> dict:
        return {"cam": self.cam, "w2c": self.w2c, "im": self.frames[t]["im"], "depth": self.frames[t]["depth"], "id": t}

    def frame(self, t: int, sequence):
        p = self.p
        if t > 0:
            initialize_camera_pose(p, t)
            tp = dict(p)
            tp["cam_unnorm_rots"] = p["cam_unnorm_rots"][..., t:t + 1].clone().requires_grad_(True)
            tp["cam_trans"] = p["cam_trans"][..., t:t + 1].clone().requires_grad_(True)
            curr = {"cam": self.cam, "w2c": self.w2c, "im": self.frames[t]["im"], "depth": self.frames[t]["depth"]}
            GraphTracker(tp, curr, 0, iters_per_graph=self.track_replay, cfg=self.track_cfg, warmup_iters=1,
                         fuse_pose=True, capacity=self.bin_capacity).track_frame(self.tracking_iters)
            with torch.no_grad():
                p["cam_unnorm_rots"][..., t] = tp["cam_unnorm_rots"][..., 0]
                p["cam_trans"][..., t] = tp["cam_trans"][..., 0]
            p = add_new_gaussians_literal(p, self._kf(t), t, self.intrinsics, self.sil_thres)
        mp = {k: (v.detach().requires_grad_(True) if k in GAUSS_KEYS + ("rgb_colors",) else v) for k, v in p.items()}
        win = self.keyframes[-(self.window - 1):] + ([self._kf(t)] if self.keyframes[-1]["id"] != t else [])
        m = GraphMapper(mp, win, iters_per_graph=self.mapping_iters, cfg=self.map_cfg, seed=0, prune=self.prune,
                        scene_radius=self.scene_radius, capacity=self.bin_capacity)
        m.run(sequence=sequence)
        if m.prune_at:
            mp, _, _ = m.compact()
        self.p = {k: (v.detach() if torch.is_tensor(v) else v) for k, v in mp.items()}
        if t > 0 and (t + 1) % self.keyframe_every == 0:
            self.keyframes.append(self._kf(t))
