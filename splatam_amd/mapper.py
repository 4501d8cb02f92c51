"""SplaTAM's per-frame mapping loop replayed as one HIP graph.

scripts/splatam.py:842-905 maps every frame with `num_iters` iterations
(configs/replica/splatam.py:16: 60) of get_loss(mapping=True) + backward + Adam
over the Gaussian parameters, with a freshly initialised optimizer per frame
(initialize_optimizer, splatam.py:166-172) and, per iteration, a keyframe drawn
uniformly from the mapping window (np.random.randint, splatam.py:851).

GraphMapper captures one frame's mapping -- the optimizer-state reset plus all
`iters_per_graph` iterations -- into a torch.cuda.CUDAGraph: the Adam step runs
inside the transform backward (gsr_map_transform_bwd_adam, step numbers 1..N
baked into the captured launches) and the rasterization uses the static-capacity
dual forward.  The keyframes are drawn per replay, like the reference draws per
iteration: every `run()` draws `iters_per_graph` indices from numpy's global random
stream (np.random.randint, the reference's own draw; `seed`: a seeded
np.random.RandomState) and gathers the drawn keyframes' target image, depth and
camera pose into per-iteration slots the captured iterations read (three gathers
per replay, enqueued before it; the keyframes must share one camera settings object,
one w2c and one image size -- otherwise the sequence drawn at construction is baked
into the graph, `redraw` False).  `sequence` is the last replay's draw.
Each replay is one frame's mapping.  An iteration whose forward overflows the
binning capacity skips its Adam step on the device (its status row, sticky
across replays, reports it).

Pruning runs inside the frame, where the reference runs it: scripts/splatam.py:876-878 calls
prune_gaussians between loss.backward() and optimizer.step() of every mapping iteration, and with
configs/replica/splatam.py:101-111 (prune_every = stop_after = 20) it removes Gaussians at iterations
0 and 20 of each frame.  P cannot change inside a captured graph, so the removal is a device mask:
at a pruning iteration gsr_map_prune clears alive[i] for the Gaussians remove_points would drop
(utils/slam_external.py:174-181), and every later forward of the frame culls them
(gsr_forward_dual_static_alive: radius 0, no instances, zero gradients), so the survivors render,
differentiate and step exactly as the compacted set does.  At a pruning iteration the reference's
optimizer.step() updates no Gaussian parameter at all -- remove_points replaced every one of them by a
new tensor without .grad, so torch.optim.Adam skips them and their state["step"] does not advance --
hence that iteration is captured as its loss forward plus the mask update, with no backward and no
Adam step (the fused steps' step counts follow: 1..19, then 20..58 for a 60-iteration frame).
The mask persists across replays: a Gaussian pruned in one replay stays removed in the next, as after the
reference's remove_points.  compact() then removes the pruned Gaussians from the parameters, the Adam state
and SplaTAM's per-Gaussian variables for real (remove_points).  Densification (GS-style, off in the default configs) changes P and
stays outside the graph.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _C
from .glue import MapAdam, map_transform
from .layout import views
from .slam import MappingConfig, _get_loss_mapping_fused, color_key, fused_mapping_eligible

TILE_SORT_CAP = 4096  # longest tile list the static mode handles (render_fwd's per-tile sort)
GAUSS_KEYS = ("means3D", "unnorm_rotations", "logit_opacities", "log_scales")


def probe_num_rendered(params, curr_data, time_idx) -> tuple[int, int]:
    """(num_rendered, longest tile list) of a keyframe at its current pose (eager, synchronous)."""
    cam = curr_data["cam"]
    key = color_key(params)
    with torch.no_grad():
        means, rots, dcol, opac, scales, col = map_transform(params, time_idx, curr_data["w2c"], key)
        sh, colors = (col, torch.Tensor([])) if key == "shs" else (torch.Tensor([]), col)
        out = _C.rasterize_gaussians_dual(cam.bg, means, colors, dcol, opac, scales, rots, cam.scale_modifier,
                                          torch.Tensor([]), cam.viewmatrix, cam.projmatrix, cam.tanfovx, cam.tanfovy,
                                          cam.image_height, cam.image_width, sh, cam.sh_degree, cam.campos,
                                          cam.prefiltered)
        n, img, binning = out[0], out[6], out[5]
        r = views(img, binning, cam.image_width, cam.image_height, n)["ranges"]
        longest = int((r[:, 1] - r[:, 0]).max().item()) if r.numel() else 0
    return int(n), longest


class GraphMapper:
    def __init__(self, params: dict, keyframes: list, iters_per_graph: int = 60, cfg: MappingConfig = MappingConfig(),
                 headroom: float = 1.5, min_extra: int = 65536, seed: int | None = None, timing: bool = False,
                 prune: bool | None = None, scene_radius=None, alive=None, capacity: int | None = None,
                 clock_stages=None):
        if not keyframes:
            raise RuntimeError("GraphMapper needs at least one keyframe")
        for kf in keyframes:
            if not fused_mapping_eligible(params, kf, cfg):
                raise RuntimeError("GraphMapper needs the fused mapping configuration (camera fixed, L1 + SSIM)")
        key = color_key(params)
        for k in GAUSS_KEYS + (key,):
            p = params[k]
            if not (p.is_leaf and p.requires_grad):
                raise RuntimeError(f"params[{k!r}] must be a leaf tensor requiring grad")
        self.params, self.keyframes, self.cfg = params, keyframes, cfg
        dev = params["means3D"].device
        self._setup_pruning(cfg if prune is None else None, bool(prune), scene_radius, int(iters_per_graph),
                            params["means3D"].shape[0], dev)
        # alive: an external uint8 [P] mask (a capacity-padded map's live slots, splatam_amd.sequence): every
        # forward culls the cleared slots and the in-frame pruning clears more
        self.external_alive = alive is not None
        if alive is not None:
            if alive.dtype != torch.uint8 or alive.numel() != params["means3D"].shape[0] or alive.device != dev:
                raise RuntimeError("alive: uint8 [P] on the parameters' device")
            self.alive = alive
        if capacity is None:
            probes = [probe_num_rendered(params, kf, kf["id"]) for kf in keyframes]
            longest = max(p[1] for p in probes)
            if longest > TILE_SORT_CAP:
                raise RuntimeError(f"a tile list of {longest} > {TILE_SORT_CAP}: use the eager (synchronous) path")
            capacity = max(1, int(headroom * max(p[0] for p in probes)) + int(min_extra))
        self.capacity = int(capacity)
        self.iters = int(iters_per_graph)
        self.rng = np.random if seed is None else np.random.RandomState(seed)
        kf0 = keyframes[0]
        self.redraw = all(kf["cam"] is kf0["cam"] and kf["w2c"] is kf0["w2c"] and kf["im"].shape == kf0["im"].shape
                          and kf["depth"].shape == kf0["depth"].shape for kf in keyframes)
        if self.redraw:
            self._make_slots(params, keyframes, dev)
            self.sequence = [0] * self.iters  # warm-up / capture content; run() draws before every replay
            self._load(self.sequence)
        else:
            self.sequence = [int(self.rng.randint(0, len(keyframes))) for _ in range(self.iters)]  # splatam.py:851
        self.status = torch.zeros(self.iters, 4, dtype=torch.int32, device=dev)
        self.adam = MapAdam(params, cfg.lrs, color_key=key)
        self.adam.capacity = self.capacity
        self.seed = torch.ones((), dtype=torch.float32, device=dev)           # static loss-gradient seed
        self.means2D = torch.zeros(params["means3D"].shape[0], 3, device=dev)  # no grad (no densification stats)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        snapshot = {k: params[k].detach().clone() for k in GAUSS_KEYS + (key,)}
        alive0 = self.alive.clone()
        with torch.cuda.stream(side):  # warm-up iterations outside the capture, then the state is restored
            for k in range(min(2, self.iters)):
                self._iteration(k)
            with torch.no_grad():
                for k, v in snapshot.items():
                    params[k].copy_(v)
            self.status.zero_()
            self.alive.copy_(alive0)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        del snapshot
        if timing:  # in-kernel stage clocks captured into the graph (clock_stages: which; default every stage --
            # each clocked launch pays its workgroups' clock atomics, ~15 us for config 4's preprocess)
            from . import profiling
            profiling.enable_timing(clock_stages=profiling.CLOCK_STAGES if clock_stages is None else
                                    tuple(clock_stages))
        self.graph = torch.cuda.CUDAGraph()
        self.stream = side
        with torch.cuda.graph(self.graph, stream=side):
            self.adam.reset()          # initialize_optimizer per frame: zero moments, step 0
            # (the alive mask is NOT reset per replay: a Gaussian pruned in one replay stays removed in the next,
            # as remove_points removes it for good -- its parameters drift under their moments with zero
            # gradient for the rest of that frame, but it is never rendered again; compact() drops it)
            for k in range(self.iters):
                self.loss = self._iteration(k)
        self.stale = False

    def _setup_pruning(self, cfg, prune, scene_radius, iters, P, dev):
        """The frame's pruning iterations (glue.prune_step over 0..iters-1) and the alive mask."""
        from .glue import prune_step
        on = cfg.prune_gaussians if cfg is not None else prune
        pd = self.cfg.pruning_dict
        self.prune_at = {}
        if on:
            for k in range(iters):
                remove, thr, big, reset = prune_step(k, pd)
                if reset:
                    raise ValueError("reset_opacities inside a captured frame would need per-group Adam step "
                                     "counts (update_params_and_optimizer skips one group's step): map eagerly")
                if remove:
                    self.prune_at[k] = (thr, big)
        self.big_thr = None
        if any(big for _, big in self.prune_at.values()):
            if scene_radius is None:
                raise ValueError("pruning big Gaussians needs variables['scene_radius'] (scene_radius=)")
            r = scene_radius if torch.is_tensor(scene_radius) else torch.tensor(float(scene_radius))
            self.big_thr = float((0.1 * r.to(device=dev, dtype=torch.float32)).item())  # as the reference forms it
        self.alive = torch.ones(P, dtype=torch.uint8, device=dev)

    def _make_slots(self, params, keyframes, dev):
        """Per-iteration keyframe slots read by the captured iterations: target image / depth, and the
        camera pose columns (a params view whose cam_unnorm_rots / cam_trans hold iteration k's pose in
        column k; the Gaussian tensors are the mapped ones)."""
        K = self.iters
        self._kf_im = torch.stack([kf["im"] for kf in keyframes]).contiguous()
        self._kf_depth = torch.stack([kf["depth"] for kf in keyframes]).contiguous()
        self._kf_ids = [int(kf["id"]) for kf in keyframes]
        self._slot_im = torch.empty((K,) + tuple(keyframes[0]["im"].shape), device=dev)
        self._slot_depth = torch.empty((K,) + tuple(keyframes[0]["depth"].shape), device=dev)
        cr, ct = params["cam_unnorm_rots"], params["cam_trans"]
        self._slot_params = dict(params)
        self._slot_params["cam_unnorm_rots"] = torch.empty(cr.shape[:-1] + (K,), dtype=cr.dtype, device=dev)
        self._slot_params["cam_trans"] = torch.empty(ct.shape[:-1] + (K,), dtype=ct.dtype, device=dev)
        kf0 = keyframes[0]
        self._slot_kfs = [{"cam": kf0["cam"], "w2c": kf0["w2c"], "im": self._slot_im[k], "depth": self._slot_depth[k],
                           "id": k} for k in range(K)]
        self._idx_host = torch.empty(2, K, dtype=torch.int64, pin_memory=True)
        self._idx_dev = torch.empty(2, K, dtype=torch.int64, device=dev)
        self._idx_event = None

    def _load(self, seq):
        """Gather the keyframes of `seq` (one index per iteration) into the slots, on the current stream."""
        if self._idx_event is not None:  # the pinned index buffer of the previous load has been read
            self._idx_event.synchronize()
        self._idx_host[0] = torch.tensor(seq, dtype=torch.int64)
        self._idx_host[1] = torch.tensor([self._kf_ids[j] for j in seq], dtype=torch.int64)
        self._idx_dev.copy_(self._idx_host, non_blocking=True)
        self._idx_event = torch.cuda.Event()
        self._idx_event.record()
        with torch.no_grad():
            torch.index_select(self._kf_im, 0, self._idx_dev[0], out=self._slot_im)
            torch.index_select(self._kf_depth, 0, self._idx_dev[0], out=self._slot_depth)
            p = self.params
            torch.index_select(p["cam_unnorm_rots"].detach(), -1, self._idx_dev[1],
                               out=self._slot_params["cam_unnorm_rots"])
            torch.index_select(p["cam_trans"].detach(), -1, self._idx_dev[1], out=self._slot_params["cam_trans"])

    def _iteration(self, k: int):
        if self.redraw:
            kf, params, t = self._slot_kfs[k], self._slot_params, k
        else:
            kf = self.keyframes[self.sequence[k]]
            params, t = self.params, kf["id"]
        self.adam.status = self.status[k]  # this iteration's forward guards its Adam step
        alive = self.alive if (self.prune_at or self.external_alive) else None
        loss, _, _ = _get_loss_mapping_fused(params, kf, t, self.cfg, adam=self.adam, capacity=self.capacity,
                                             status=self.status[k], means2D=self.means2D, alive=alive)
        if k in self.prune_at:
            # prune_gaussians after loss.backward(): the gradients of this iteration reach no parameter (every
            # Gaussian tensor is replaced by remove_points, so optimizer.step() skips them), so no backward runs
            from .glue import map_prune
            thr, big = self.prune_at[k]
            map_prune(self.params, self.alive, thr, self.big_thr if big else None)
            return loss.detach()
        torch.autograd.backward(loss, self.seed)
        return loss.detach()

    def set_keyframes(self, keyframes: list):
        """A new keyframe window for the next replays (SplaTAM selects one per mapped frame, scripts/splatam.py:
        820-836): the captured iterations read per-iteration slots that run() fills from this window, so the
        graph is not re-captured.  Needs the redraw form; the keyframes must share the camera settings object,
        the w2c and the image size of the ones the mapper was built with."""
        if not self.redraw:
            raise RuntimeError("set_keyframes needs the redraw form (keyframes sharing cam / w2c / image size)")
        kf0 = self._slot_kfs[0]
        for kf in keyframes:
            if kf["cam"] is not kf0["cam"] or kf["w2c"] is not kf0["w2c"] or kf["im"].shape != self._slot_im.shape[1:]:
                raise RuntimeError("set_keyframes: every keyframe must share the mapper's camera, w2c and image size")
        self.keyframes = list(keyframes)
        self._kf_im = torch.stack([kf["im"] for kf in keyframes]).contiguous()
        self._kf_depth = torch.stack([kf["depth"] for kf in keyframes]).contiguous()
        self._kf_ids = [int(kf["id"]) for kf in keyframes]

    def survivors(self) -> torch.Tensor:
        """Boolean [P] mask of the Gaussians every replay so far kept (the mask persists across replays)."""
        return self.alive.bool()

    VARIABLE_KEYS = ("means2D_gradient_accum", "denom", "max_2D_radius", "timestep")

    def compact(self, variables: dict | None = None):
        """After a replay, remove the pruned Gaussians for real: remove_points (utils/slam_external.py:141-163)
        on the parameters, the frame's Adam moments and -- when `variables` is given -- the per-Gaussian
        SplaTAM variables remove_points compacts too (means2D_gradient_accum, denom, max_2D_radius and, when
        present, timestep; assigned into the caller's dict as remove_points does, so get_loss's
        `variables['max_2D_radius'][seen]` and the saved params['timestep'] keep lining up with means3D).
        Returns (params, exp_avg, exp_avg_sq): a new params dict (every per-Gaussian tensor compacted, new
        leaves requiring grad; the camera tensors as they were) and the moments by parameter name.  P changes,
        so this mapper is stale afterwards (run() raises): build the next frame's mapper on the returned
        parameters."""
        keep = self.survivors()
        P = keep.shape[0]
        out = dict(self.params)
        m, v = {}, {}
        with torch.no_grad():
            for k, em, ev in zip(self.adam.keys, self.adam.exp_avg, self.adam.exp_avg_sq):
                out[k] = self.params[k].detach()[keep].clone().requires_grad_(True)
                m[k], v[k] = em[keep].clone(), ev[keep].clone()
            for k, t in self.params.items():  # any other per-Gaussian parameter (remove_points: every non-camera key)
                if k in m or k in ("cam_unnorm_rots", "cam_trans") or not torch.is_tensor(t) or t.dim() == 0:
                    continue
                if t.shape[0] == P:
                    out[k] = t.detach()[keep].clone().requires_grad_(t.requires_grad)
            if variables is not None:
                for k in self.VARIABLE_KEYS:
                    t = variables.get(k)
                    if torch.is_tensor(t) and t.dim() > 0 and t.shape[0] == P:
                        variables[k] = t[keep.to(t.device)]
        self.stale = True
        return out, m, v

    def run(self, check: bool = True, sequence=None):
        """Enqueue one frame's mapping (one graph launch).  With `redraw` the keyframe of every iteration
        is drawn now (splatam.py:851; `sequence` overrides the draw) and gathered into the slots.  An
        iteration whose forward overflowed skips its Adam step, and so does every later iteration of the
        frame (MapAdam.halted_word, sticky on the device), so the parameters are those of the last good
        iteration and no step uses mismatched bias corrections.  `check` (the default) ends the replay
        with one host sync and raises on an overflow, so the caller can rebuild with more headroom and
        re-map the frame; check=False (timing loops) enqueues without a sync -- read overflowed()
        afterwards."""
        if self.stale:
            raise RuntimeError("this mapper was compacted (P changed): build a new one for the next frame")
        if self.redraw:
            n = len(self.keyframes)
            seq = [int(self.rng.randint(0, n)) for _ in range(self.iters)] if sequence is None else \
                [int(j) for j in sequence]
            if len(seq) != self.iters or not all(0 <= j < n for j in seq):
                raise ValueError(f"sequence: {self.iters} keyframe indices in [0, {n})")
            self.sequence = seq
            self._load(seq)
        elif sequence is not None:
            raise RuntimeError("this mapper bakes its keyframe sequence into the graph (redraw False)")
        if check:
            self.reset_status()
        self.graph.replay()
        if check and self.overflowed():
            raise RuntimeError(f"binning capacity {self.capacity} exceeded during mapping: rebuild the mapper "
                               "with more headroom and re-run the frame")

    def reset_status(self):
        self.status.zero_()

    def overflowed(self) -> bool:
        """True if any iteration since the last reset_status() exceeded the binning capacity, or the last
        replay's optimizer halted (one host sync)."""
        st = self.status.cpu()
        return bool((st[:, 0] > self.capacity).any() or (st[:, 2] > TILE_SORT_CAP).any() or (st[:, 1] != 0).any()
                    or self.adam.halted())

    def num_rendered(self) -> list[int]:
        return [int(x) for x in self.status[:, 0].cpu()]
