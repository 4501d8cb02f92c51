"""Headline benchmark: SplaTAM tracking iterations through the MI355X rasterizer.

BASELINE.json metric "rasterize fwd+bwd frames/sec @640x480, 300k Gaussians;
HBM GB/s vs peak" on config 3: 300k isotropic Gaussians, 640x480, full
tracking-iteration loss (scripts/splatam.py:220-353 with tracking=True).
One step = one frame = RGB render fwd+bwd + depth/silhouette ([z,1,z^2])
render fwd+bwd + masked L1 loss + Adam step on the camera pose.  The two renders
share one dual rasterization (gsr_forward_dual) and the glue runs as the fused
HIP kernels of include/gsr_glue.h (splatam_amd/slam.py get_loss_tracking).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU; every rank tracks its own frame against the same
Gaussian map (frame sharding); rank 0 broadcasts the canonical
Gaussian set over RCCL every --bcast-every steps (inside the timed region).
`value` = frames processed by all ranks / max-over-ranks wall time.

The JSON line carries:
  roofline      -- render-backward kernel (one dual launch per frame): SURVEY.md
                   8(d) algorithmic bytes per launch extended to both colour sets
                   (8*Tt + 52*I + 32*N + 56*P, measured I) over its average
                   duration during the timed region, measured on its launch
                   stream: device wall-clock stamps around every launch (graph
                   mode; hipEvent records cannot be captured) or hipEvents (eager);
  cpu_baseline  -- rank 0 at N=1 only: the float32 C oracle (oracle/) on one
                   frame of the same workload, single thread.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "rasterize fwd+bwd frames/sec @640×480, 300k Gaussians; HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TFLOPS = 157.3  # FP32 vector (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=None, help="BASELINE config (default: 3 tracking, 4 mapping)")
    ap.add_argument("--workload", choices=("tracking", "mapping"), default="tracking",
                    help="tracking: the headline metric (config 3); mapping: SplaTAM mapping iterations "
                         "(config 4: 1M anisotropic Gaussians, SH degree 3, 1200x680)")
    ap.add_argument("--keyframes", type=int, default=4, help="mapping: keyframes in the window")
    ap.add_argument("--bcast-every", type=int, default=40,
                    help="broadcast the Gaussian map every k steps (Replica: 40 tracking iters/frame)")
    ap.add_argument("--cpu-baseline", choices=("auto", "on", "off"), default="auto")
    ap.add_argument("--graph", type=int, default=1, help="1: replay the tracking iterations as a HIP graph")
    ap.add_argument("--iters-per-graph", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=50.0,
                    help="tracking: untimed priming replays (undone) until this much wall time has passed, so "
                         "the timed region does not start on the GPU's clock ramp (0: one priming replay)")
    ap.add_argument("--frame-iters", type=int, default=40,
                    help="tracking iterations per frame (configs/replica/splatam.py:15); the timed loop runs whole "
                         "frames: fresh optimizer, replays, best-candidate pose written back")
    ap.add_argument("--fuse-pose", type=int, default=1,
                    help="tracking: 1 = pose chain + Adam inside the per-Gaussian backward (one launch fewer), "
                         "0 = separate pose kernel")
    ap.add_argument("--dropin", choices=("on", "off"), default="on",
                    help="also time the unchanged-caller path: SURVEY 8(d)'s unit through "
                         "diff_gaussian_rasterization.GaussianRasterizer, eager (the 'dropin' object)")
    ap.add_argument("--dropin-frames", type=int, default=3, help="dropin: timed frames of 40 iterations")
    ap.add_argument("--fisher", choices=("on", "off"), default="on",
                    help="also time the batched Fisher / EIG view scoring (backward_power 2) on the same map")
    ap.add_argument("--mapping", choices=("auto", "on", "off"), default="auto",
                    help="also time the mapping workload (config 4) into a 'mapping' object (auto: N=1 only)")
    ap.add_argument("--mapping-steps", type=int, default=120, help="mapping leg: timed iterations (whole frames)")
    ap.add_argument("--map-frame-iters", type=int, default=60,
                    help="mapping: iterations per frame = per HIP graph (configs/replica/splatam.py:16: 60)")
    ap.add_argument("--map-prune", type=int, default=1,
                    help="mapping: prune_gaussians inside the frame (configs/replica/splatam.py:101-111), 0: off")
    ap.add_argument("--map-binning", choices=("culled", "reference"), default="culled",
                    help="mapping: tile lists without the culled instances (default) or the reference's lists "
                         "(A/B of the tile cull's effect on the mapping kernels)")
    ap.add_argument("--map-prunable", type=float, default=0.02,
                    help="mapping: fraction of the map's Gaussians given opacities under prune_gaussians' 0.005 "
                         "threshold (removed at the frame's first pruning iteration, as faded Gaussians are)")
    ap.add_argument("--sequence", choices=("auto", "on", "off"), default="auto",
                    help="SLAM sequence leg (splatam_amd.sequence) at config 3 (auto: N=1 only)")
    ap.add_argument("--seq-frames", type=int, default=4, help="sequence: timed frames (after frames 0 and 1)")
    ap.add_argument("--seq-headroom", type=int, default=None,
                    help="sequence: map capacity beyond the initial map, in Gaussians (default W*H/3); every "
                         "per-Gaussian launch covers the whole capacity")
    ap.add_argument("--fisher-k", type=int, default=16, help="fisher: poses per HIP-graph launch")
    ap.add_argument("--configs", choices=("auto", "on", "off"), default="auto",
                    help="BASELINE configs 1 (forward only) and 2 (fwd+bwd RGB + depth) on the GPU and the CPU "
                         "oracle beside the headline (auto: N=1 only)")
    ap.add_argument("--fuse-render", type=int, default=1,
                    help="tracking: 1 = the render forward and render backward of an iteration in one launch "
                         "(render_track_kernel), 0 = separate render_fwd / render_bwd launches")
    ap.add_argument("--unfused-leg", choices=("on", "off"), default="on",
                    help="with --fuse-render 1 at N=1: also time a few iterations with separate render launches "
                         "(roofline.unfused: render_bwd's own time and roofline)")
    ap.add_argument("--stage-clocks", choices=("all", "render"), default="render",
                    help="tracking: the kernels whose in-kernel stage clocks run in the timed replays (render: the "
                         "render kernel only, stages_us from a separate pass with every clock on; all: every stage "
                         "in the timed replays, ~5 us per iteration of stamps)")
    ap.add_argument("--stage-breakdown", choices=("on", "off"), default="on",
                    help="tracking: the separate all-clocks pass after the timed region that gives stages_us (off: "
                         "profiling runs, whose kernel averages it would mix with the clocked launches)")
    ap.add_argument("--timing", type=int, default=1,
                    help="0: no device-clock timing of render_bwd in the graph (A/B check; no roofline)")
    return ap.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        backend = os.environ.get("GSR_DIST_BACKEND", "nccl")  # nccl = RCCL; gloo only to rehearse ranks on one GPU
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def img_n_contrib_sum(img_buffer: torch.Tensor, W: int, H: int) -> int:
    """Sum of per-pixel n_contrib (= pairs the backward evaluates); ImgLayout in csrc/gsr_common.h."""
    N = W * H
    off = (4 * N + 255) // 256 * 256
    nc = img_buffer[off:off + 4 * N].view(torch.int32)
    return int(nc.sum().item())


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if args.config is None:
        args.config = 4 if args.workload == "mapping" else 3
    if args.workload == "mapping":
        return main_mapping(args, world, rank, dev)

    from splatam_amd import profiling
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import camera_settings, get_loss_tracking, init_tracking_params, transformed_params2rendervar, \
        transformed_params2depthplussilhouette, transform_to_frame
    from splatam_amd.rasterizer import GaussianRasterizer

    from splatam_amd import dist as sd
    scene = config_scene(args.config)
    P, W, H = scene.P, scene.cam.W, scene.cam.H
    from splatam_amd.workloads import tracking_frame
    frame = sd.frames_for_rank(world)[0] if world > 1 else 0  # frame sharding: rank r tracks frame r
    # the map of init_tracking_params and the frame's target rendered at the unperturbed pose -- the workload
    # tests/test_gpu_pinned.py compares with the literal get_loss loop at this size
    params, curr = tracking_frame(scene, dev, num_frames=max(world, 1), frame=frame)
    fm = sd.FlatMap(params)                     # the map as one contiguous buffer: one collective per broadcast
    sd.broadcast_flat(fm)                       # canonical Gaussian map from rank 0
    bc = sd.MapBroadcaster(fm)                  # double-buffered broadcast, overlapped with the frames' replays
    cam, w2c = curr["cam"], curr["w2c"]
    params["cam_unnorm_rots"].requires_grad_(True)
    params["cam_trans"].requires_grad_(True)
    # configs/replica/splatam.py:71-80 tracking learning rates; torch's fused (single-kernel) Adam
    opt = torch.optim.Adam([{"params": [params["cam_unnorm_rots"]], "lr": 0.0004},
                            {"params": [params["cam_trans"]], "lr": 0.002}], fused=True)

    def step():
        opt.zero_grad(set_to_none=True)
        loss, _, _ = get_loss_tracking(params, curr, frame)
        loss.backward()
        opt.step()
        return loss

    tracker = None
    steps = args.steps
    FI = max(1, args.frame_iters)
    if args.graph:
        # HIP graph of S tracking iterations (splatam_amd/tracker.py).  Exactly `steps` iterations are
        # timed: frames of FI iterations (fresh optimizer, best-candidate write-back), the last one
        # partial when FI does not divide steps; S divides both so every frame is whole replays.
        from splatam_amd import glue
        from splatam_amd.tracker import GraphTracker
        glue._RENDER_FUSED = glue._RENDER_FUSED and bool(args.fuse_render)
        S = math.gcd(math.gcd(max(1, args.iters_per_graph), FI), max(1, steps))
        # warm-up: W eager tracking iterations plus one priming replay, all undone (pose restored,
        # optimizer reset) before the timed frames
        clock_stages = profiling.CLOCK_STAGES if args.stage_clocks == "all" else ("render_fwd", "render_bwd")
        tracker = GraphTracker(params, curr, frame, iters_per_graph=S, timing=bool(args.timing),
                               fuse_pose=bool(args.fuse_pose), warmup_iters=max(1, args.warmup), prime=True,
                               prime_ms=args.settle_ms, clock_stages=clock_stages)
    else:
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if tracker is None:
        profiling.enable_timing(True)
    else:  # reset the device-clock accumulators the captured stamps add to
        profiling.enable_timing(clock_stages=tracker.clock_stages)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if tracker is not None:
        per_bcast = max(1, args.bcast_every // FI) if args.bcast_every > 0 else 0
        done, f, n_bcast = 0, 0, 0
        while done < steps:
            if world > 1 and per_bcast and f % per_bcast == 0:
                bc.finish()                    # the map version broadcast at the last boundary goes live
                bc.start()                     # map update -> one RCCL broadcast over xGMI, side stream
                n_bcast += 1
            n = min(FI, steps - done)
            tracker.track_frame(n, check=False)  # one frame: fresh optimizer, replays, best pose written back
            #   (overflow checked once after the timed loop, below)
            done += n
            f += 1
        bc.finish()
    else:
        for i in range(steps):
            if world > 1 and args.bcast_every > 0 and i % args.bcast_every == 0:
                sd.broadcast_map(params)           # map update -> RCCL broadcast over xGMI
            step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    stages = profiling.read_timing()
    profiling.enable_timing(False)
    if tracker is not None and tracker.overflowed():
        raise SystemExit(f"binning capacity overflow during the timed replays (capacity {tracker.capacity}, "
                         f"status rows {tracker.status.cpu().tolist()}): measurement invalid")
    elapsed = sd.max_over_ranks(t1 - t0, device=dev)
    frames = steps * world
    value = frames / elapsed
    # Per-stage breakdown: every kernel's in-kernel clock on, in a separate pass of the same frames after the
    # timed region (the stamps cost ~5 us per iteration -- 6510 vs 6290 frames/s interleaved,
    # profiles/r9i_ab_stage_clocks.txt -- so the timed replays clock the render kernel only)
    stages_timed = {k: round(v["avg_us"], 2) for k, v in stages.items() if v["launches"]}
    stages_breakdown, stages_source = stages_timed, "the timed replays' in-kernel stage clocks"
    if tracker is not None and args.timing and args.stage_clocks == "render" and args.stage_breakdown == "on":
        bt = GraphTracker(params, curr, frame, iters_per_graph=S, timing=True, fuse_pose=bool(args.fuse_pose),
                          warmup_iters=1, prime=True, prime_ms=args.settle_ms, clock_stages=profiling.CLOCK_STAGES)
        profiling.enable_timing(clock_stages=profiling.CLOCK_STAGES)
        done = 0
        while done < steps:
            n = min(FI, steps - done)
            bt.track_frame(n, check=False)
            done += n
        torch.cuda.synchronize()
        stages_breakdown = {k: round(v["avg_us"], 2) for k, v in profiling.read_timing().items() if v["launches"]}
        profiling.enable_timing(False)
        if bt.overflowed():
            raise SystemExit("binning capacity overflow in the stage-breakdown pass")
        stages_source = (f"a separate pass of the same {steps} iterations after the timed region with every "
                         "kernel's in-kernel stage clock on (the timed replays clock the render kernel only)")
        del bt
    if stages["render_bwd"]["launches"] == 0 and stages["render_fwd"]["launches"] > 0:  # fused: render_track
        stages_breakdown = {("render_track" if k == "render_fwd" else k): v for k, v in stages_breakdown.items()}
    # the same timed frames without the broadcast, and the broadcast alone
    bcast_split = None
    if world > 1 and tracker is not None:
        dist.barrier()
        torch.cuda.synchronize()
        tb0 = time.perf_counter()
        done = 0
        while done < steps:
            n = min(FI, steps - done)
            tracker.track_frame(n, check=False)
            done += n
        torch.cuda.synchronize()
        dist.barrier()
        el_nb = sd.max_over_ranks(time.perf_counter() - tb0, device=dev)
        nb = 5
        dist.barrier()
        torch.cuda.synchronize()
        tc0 = time.perf_counter()
        for _ in range(nb):
            sd.broadcast_flat(fm)
        torch.cuda.synchronize()
        dist.barrier()
        el_b = sd.max_over_ranks(time.perf_counter() - tc0, device=dev)
        if tracker.overflowed():
            raise SystemExit("binning capacity overflow during the no-broadcast replays: measurement invalid")
        bcast_split = {"value_no_broadcast": round(frames / el_nb, 3), "ms_per_step_no_broadcast":
                       round(1000.0 * el_nb / steps, 4), "broadcast_ms": round(1000.0 * el_b / nb, 4),
                       "broadcasts_in_timed_region": n_bcast, "broadcast_bytes": int(fm.nbytes),
                       # the receiving ranks track against the map of the previous broadcast boundary (the
                       # double-buffered broadcast goes live one boundary after it starts)
                       "map_staleness_boundaries": 1,
                       "broadcast_path": "one RCCL broadcast of the flat map buffer (splatam_amd.dist.FlatMap) "
                                         "per map update, on a side stream overlapped with the next frame's "
                                         "replays (MapBroadcaster, double-buffered); broadcast_ms: the blocking "
                                         "single call alone"}

    # ---- roofline of the dominant kernel (render backward) ------------------
    rb = stages["render_bwd"]
    Tt = ((W + 15) // 16) * ((H + 15) // 16)
    N = W * H
    if tracker is not None:  # static-mode launches report capacity as units; use the measured counters
        nr = tracker.num_rendered()
        I_avg = sum(nr) / len(nr)
    else:
        I_avg = rb["units"] / max(rb["launches"], 1)
    # SURVEY.md 8(d) per-rasterization bytes 8*Tt + 40*I + 20*N + 44*P, for the dual launch
    # (both colour sets): + colors2 gather 12*I, + dL_dpix2 12*N, + dcolors2 12*P
    bwd_bytes = 8 * Tt + 52 * I_avg + 32 * N + 56 * P
    # render fwd 8*Tt + 44*I + 24*N per rasterization, dual: + colors2 gather 12*I, + out_color2 12*N
    fwd_bytes = 8 * Tt + 56 * I_avg + 36 * N
    fused = rb["launches"] == 0 and stages["render_fwd"]["launches"] > 0
    if fused:  # render_track_kernel: the tracking forward and render backward in one launch (stage render_fwd)
        rk, bytes_per_launch, kname = stages["render_fwd"], fwd_bytes + bwd_bytes, "render_track_kernel"
        traffic, traffic_source = committed_traffic("render_track_pmc.json")
    else:
        rk, bytes_per_launch, kname = rb, bwd_bytes, "render_bwd_kernel"
        # traffic: HBM bytes per launch from a separate rocprofv3 PMC pass (FETCH_SIZE / WRITE_SIZE,
        # calibrated; counters cannot be collected inside the timed run) -- committed, so the line names
        # where it came from
        traffic, traffic_source = committed_traffic("render_bwd_pmc.json")
    dur_s = rk["avg_us"] * 1e-6
    achieved = bytes_per_launch / dur_s / 1e9 if dur_s > 0 else 0.0
    roofline = {"kernel": kname, "bound": "hbm", "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic, "traffic_source": traffic_source, "alg_bytes_per_launch": int(bytes_per_launch),
                "avg_us": round(rk["avg_us"], 2), "num_rendered_avg": int(I_avg), "launches_timed": int(rk["launches"]),
                "timing": "in-kernel wall_clock64 (first workgroup start to last workgroup end) of every launch in the timed HIP-graph replays" if tracker is not None
                else "hipEvents around each launch"}
    if fused:
        roofline["fused"] = ("the tracking iteration's render forward (+ L1 loss) and render backward in one "
                             "launch per tile (gsr_track_forward_backward_dual_static_xf); the rendered images, "
                             "final_T / n_contrib and the loss gradient images stay in registers (GraphTracker: "
                             "images=False, nothing reads them after the launch); alg bytes = SURVEY 8(d)'s "
                             "dual render fwd + render bwd, which count those image writes and reads")
        if world == 1 and args.unfused_leg == "on":
            roofline["unfused"] = unfused_render_leg(params, curr, frame, tracker.iters, P, W, H, Tt, N)

    dropin = dropin_leg(args, scene, dev) if args.dropin == "on" else None
    configs = None
    if args.configs == "on" or (args.configs == "auto" and world == 1):
        configs = configs_leg(dev, want_cpu=rank == 0 and args.cpu_baseline != "off")
        stream = hbm_stream_gbs()
        if stream:
            # not a peak: the rate plain copies reach on this box (the roofline's `peak` stays the 8 TB/s spec)
            roofline["stream_measured"] = {
                "copy_gbs": stream["copy_gbs"], "triad_gbs": stream["triad_gbs"],
                "copy_tile_gbs": stream.get("copy_tile_gbs"), "copy_tile_form": stream.get("copy_tile_form"),
                "source": "tools/micro/stream (1 GiB float4 arrays, best of 20 launches): grid-stride "
                          "copy / triad, and block-tile copies with 4-16 loads in flight per thread "
                          "(plain or nontemporal)"}
    fisher = fisher_leg(args, scene, dev, world=world, rank=rank) if args.fisher == "on" else None
    mapping = None
    if args.mapping == "on" or (args.mapping == "auto" and world == 1):
        mapping = mapping_leg(args, dev)
        if args.dropin == "on":
            mapping["dropin"] = dropin_mapping_leg(args, dev)

    sequence = None
    if args.sequence == "on" or (args.sequence == "auto" and world == 1):
        sequence = sequence_leg(args, dev)

    # ---- CPU baseline: the float32 C oracle on one frame (rank 0, N=1) ------
    cpu = None
    want_cpu = args.cpu_baseline == "on" or (args.cpu_baseline == "auto" and world == 1)
    if want_cpu and rank == 0:
        import numpy as np
        from oracle import oracle as orc
        with torch.no_grad():
            tg = transform_to_frame(params, frame, False, False)
            rv = transformed_params2rendervar(params, tg)
            dv = transformed_params2depthplussilhouette(params, w2c, tg)
        c = scene.cam
        common = dict(view=c.viewmatrix.numpy(), proj=c.projmatrix.numpy(), campos=c.campos.numpy(),
                      tanfovx=c.tanfovx, tanfovy=c.tanfovy, H=H, W=W)
        rng = np.random.RandomState(0)
        dpix = [rng.randn(3, H, W).astype(np.float32) for _ in range(2)]
        inputs = [(r["means3D"].cpu().numpy(), r["opacities"].cpu().numpy(), r["colors_precomp"].cpu().numpy(),
                   r["scales"].cpu().numpy(), r["rotations"].cpu().numpy()) for r in (rv, dv)]

        def cpu_frame():
            ev = ct = 0
            for (m, o, col, sc, ro), dp in zip(inputs, dpix):
                fr = orc.forward(m, o, colors=col, scales=sc, rotations=ro, **common)
                g = orc.backward(fr, dp)
                ev += g["pair_evals"]
                ct += g["pair_contrib"]
            return ev, ct

        # BASELINE.md / SURVEY 8(d) protocol: every host thread the process has (OpenMP over tiles;
        # OMP_NUM_THREADS on the GPU box), 1 warm-up, median of 3 timed frames
        evals, contrib = cpu_frame()
        times = []
        for _ in range(3):
            t_cpu = time.perf_counter()
            cpu_frame()
            times.append(time.perf_counter() - t_cpu)
        t_cpu = sorted(times)[1]
        cores = orc.threads()
        cpu = {"value": round(1.0 / t_cpu, 5), "unit": "frames/s", "cores": cores, "kind": "port",
               "sample": f"1 frame (RGB + depth/silhouette render fwd+bwd) of config {args.config} "
                         f"({P} Gaussians, {W}x{H}) through oracle/gsr_oracle.c float32 on {cores} OpenMP "
                         f"threads (tiles in parallel), 1 warm-up + median of 3: "
                         f"{', '.join(f'{t:.2f}' for t in times)} s"}
        # VALU view of the same kernel: F_eval=12 per evaluated pair, +45 per contributing pair
        # for one colour set, +9 for the second set of the dual launch (dot product, 3 products, 3 sums);
        # one dual launch evaluates each pair once for both renders (the oracle counts both renders)
        flops = 12 * evals / 2 + 54 * contrib / 2
        if fused:  # + the forward's: F_eval 12 per evaluated pair, +14 per contributing pair (+3 for colours2)
            flops += 12 * evals / 2 + 17 * contrib / 2
        roofline["valu"] = {"achieved_tflops": round(flops / dur_s / 1e12, 3) if dur_s > 0 else None,
                            "peak_tflops": VALU_PEAK_TFLOPS,
                            "frac": round(flops / dur_s / 1e12 / VALU_PEAK_TFLOPS, 4) if dur_s > 0 else None,
                            "pairs_evaluated": int(evals / 2), "pairs_contributing": int(contrib / 2)}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "frames/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "execution": (f"{steps} timed tracking iterations in frames of up to {FI} (fresh optimizer per "
                          f"frame, best-candidate pose written back): HIP graph of {tracker.iters} iterations "
                          f"replayed {-(-steps // tracker.iters)}x; warm-up {args.warmup} eager iterations + "
                          f"{tracker.prime_replays} priming replays ({tracker.prime_ms:.0f} ms: graph upload and "
                          f"GPU clock settle, --settle-ms {args.settle_ms:g}), undone; binning capacity "
                          f"{tracker.capacity}, no overflow"
                          if tracker is not None else "eager"),
            "data": "synthetic (SURVEY.md 8(d) seeded scene; targets rendered at the unperturbed pose)",
            "config": {"workload": f"config {args.config}: {P} isotropic Gaussians, {W}x{H}, SplaTAM tracking "
                                   "iteration (RGB + depth/silhouette render fwd+bwd, masked L1, Adam on pose)",
                       "gaussians": P, "width": W, "height": H, "frames_per_step_per_gpu": 1,
                       "broadcast_every": args.bcast_every if world > 1 else None,
                       "parallelism": f"frame-sharded x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            # per launch, from in-kernel stage clocks (the per-tile sort runs inside render_fwd / render_track: no
            # "sort" stage; "ranges" is the tile-count column scan)
            "stages_us": stages_breakdown, "stages_source": stages_source,
            "dropin": dropin,
            "fisher": fisher,
            "mapping": mapping,
            "sequence": sequence,
            "configs": configs,
            "broadcast": bcast_split,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def configs_leg(dev, want_cpu: bool):
    """BASELINE.json configs 1 and 2 in SURVEY 8(d)'s unit (1 frame = the RGB render plus the [z, 1, z^2]
    depth/silhouette render of the same Gaussians and camera): config 1 (10k isotropic, 320x240) forward
    only, config 2 (100k isotropic, 640x480, Replica room0 intrinsics) forward + backward of both renders
    with seeded N(0,1) pixel gradients.  GPU, two ways: `unit` = SURVEY's own measurement, 2 x
    diff_gaussian_rasterization.GaussianRasterizer (+ backward) from Python with a synchronize around the
    timed frames (every input a leaf requiring grad), and `fused` = one rasterize_gaussians_dual call (+ its
    backward) per frame, eager.  CPU: the float32 C oracle on the same frame, every host thread, 1 warm-up +
    median of 3 (config 1: 10 frames per sample)."""
    import numpy as np
    import diff_gaussian_rasterization as dgr
    from splatam_amd.rasterizer import rasterize_gaussians_dual
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import camera_settings, init_tracking_params, transform_to_frame, \
        transformed_params2depthplussilhouette, transformed_params2rendervar
    out = {}
    for cfg, fwd_only in ((1, True), (2, False)):
        scene = config_scene(cfg)
        P, W, H = scene.P, scene.cam.W, scene.cam.H
        params = init_tracking_params(scene, num_frames=1, device=dev)
        cam = camera_settings(scene.cam, dev)
        w2c = torch.eye(4, device=dev)
        with torch.no_grad():
            tg = transform_to_frame(params, 0, False, False)
            rv1 = transformed_params2rendervar(params, tg)
            rv2 = transformed_params2depthplussilhouette(params, w2c, tg)
        leaf = lambda d: {k: v.detach().clone().requires_grad_(not fwd_only) for k, v in d.items()}  # noqa: E731
        rv1, rv2 = leaf(rv1), leaf(rv2)
        rv2["means3D"] = rv1["means3D"]
        gen = torch.Generator().manual_seed(0)
        g1 = torch.randn(3, H, W, generator=gen).to(dev)
        g2 = torch.randn(3, H, W, generator=gen).to(dev)
        R = dgr.GaussianRasterizer

        def unit():
            if fwd_only:
                with torch.no_grad():
                    R(cam)(**rv1)
                    R(cam)(**rv2)
                return
            for d in (rv1, rv2):
                for v in d.values():
                    v.grad = None
            im, _, _ = R(cam)(**rv1)
            ds, _, _ = R(cam)(**rv2)
            ((im * g1).sum() + (ds * g2).sum()).backward()

        def fused():
            if fwd_only:
                with torch.no_grad():
                    rasterize_gaussians_dual(rv1["means3D"], rv1["means2D"], None, rv1["colors_precomp"],
                                             rv2["colors_precomp"], rv1["opacities"], rv1["scales"],
                                             rv1["rotations"], None, cam)
                return
            for d in (rv1, rv2):
                for v in d.values():
                    v.grad = None
            im, ds, _, _ = rasterize_gaussians_dual(rv1["means3D"], rv1["means2D"], None, rv1["colors_precomp"],
                                                    rv2["colors_precomp"], rv1["opacities"], rv1["scales"],
                                                    rv1["rotations"], None, cam)
            ((im * g1).sum() + (ds * g2).sum()).backward()

        res = {"workload": f"config {cfg}: {P} isotropic Gaussians, {W}x{H}, "
                           + ("forward only" if fwd_only else "forward + backward") + " of RGB + depth/silhouette"}
        for name, fn in (("unit", unit), ("fused", fused)):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            n = 200 if fwd_only else 100
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            res[name] = {"value": round(1.0 / dt, 2), "unit": "frames/s", "ms_per_frame": round(1000 * dt, 4)}
        # the eager calls above are host-bound (each forward waits for num_rendered, as the reference's
        # does): the device time of the fused frame's own kernels, from hipEvents around every stage
        from splatam_amd import profiling
        nd = 20
        profiling.enable_timing(True)
        for _ in range(nd):
            fused()
        torch.cuda.synchronize()
        st = profiling.read_timing()
        profiling.enable_timing(False)
        dev_us = sum(v["ms"] for v in st.values()) * 1000.0 / nd
        res["fused"]["device_us_per_frame"] = round(dev_us, 2)
        res["fused"]["device_bound_frames_per_s"] = round(1e6 / dev_us, 1) if dev_us > 0 else None
        res["fused"]["stages_us_per_frame"] = {k: round(v["ms"] * 1000.0 / nd, 2) for k, v in st.items() if v["ms"]}
        if want_cpu:
            from oracle import oracle as orc
            c = scene.cam
            common = dict(view=c.viewmatrix.numpy(), proj=c.projmatrix.numpy(), campos=c.campos.numpy(),
                          tanfovx=c.tanfovx, tanfovy=c.tanfovy, H=H, W=W)
            inputs = [tuple(r[k].detach().cpu().numpy() for k in ("means3D", "opacities", "colors_precomp", "scales",
                                                                   "rotations")) for r in (rv1, rv2)]
            dps = [g1.cpu().numpy(), g2.cpu().numpy()]
            reps = 10 if fwd_only else 1

            def cpu_frame():
                for _ in range(reps):
                    for (m, o, col, sc, ro), dp in zip(inputs, dps):
                        fr = orc.forward(m, o, colors=col, scales=sc, rotations=ro, **common)
                        if not fwd_only:
                            orc.backward(fr, dp)

            cpu_frame()
            times = []
            for _ in range(3):
                t0 = time.perf_counter()
                cpu_frame()
                times.append((time.perf_counter() - t0) / reps)
            tc = sorted(times)[1]
            res["cpu"] = {"value": round(1.0 / tc, 4), "unit": "frames/s", "cores": orc.threads(), "kind": "port",
                          "sample": f"{reps} frame(s) per sample through oracle/gsr_oracle.c float32, 1 warm-up + "
                                    f"median of 3: {', '.join(f'{t:.4f}' for t in times)} s per frame"}
        out[str(cfg)] = res
        del params, rv1, rv2
        torch.cuda.empty_cache()
    return out


def hbm_stream_gbs():
    """STREAM-style copy / triad on this GPU (tools/micro/stream, built in-tree): the measured HBM peak the
    roofline's spec peak is compared with; None when the binary is absent."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "micro", "stream")
    if not os.path.exists(exe):
        return None
    try:
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        return json.loads(r.stdout.strip().split("\n")[-1])
    except Exception:
        return None


def dropin_leg(args, scene, dev, iters_per_frame: int = 40):
    """SURVEY.md 8(d)'s unit of work as an unchanged scripts/splatam.py runs it: every parameter an
    nn.Parameter requiring grad (splatam.py:150-155), the literal get_loss(tracking=True) with two
    diff_gaussian_rasterization.GaussianRasterizer calls (:255,259), loss.backward() (:722), torch Adam over
    every group (:166-172,723-724), the best-candidate pose (:726-731,760-763) -- eager, one Python
    iteration at a time.  Returns frames(=iterations)/s and the render-backward kernel's average."""
    import diff_gaussian_rasterization as dgr
    from splatam_amd import profiling
    from splatam_amd.rasterizer import GaussianRasterizer
    from splatam_amd.slam import as_parameters, camera_settings, init_tracking_params, track_frame_literal, \
        tracking_variables, transform_to_frame, transformed_params2depthplussilhouette, transformed_params2rendervar
    P, W, H = scene.P, scene.cam.W, scene.cam.H
    nf = max(1, args.dropin_frames) + 1
    base = init_tracking_params(scene, num_frames=nf, device=dev)
    cam = camera_settings(scene.cam, dev)
    w2c = torch.eye(4, device=dev)
    with torch.no_grad():
        gt = dict(base)
        gt["cam_unnorm_rots"] = torch.zeros_like(base["cam_unnorm_rots"])
        gt["cam_unnorm_rots"][0, 0] = 1.0
        gt["cam_trans"] = torch.zeros_like(base["cam_trans"])
        tg = transform_to_frame(gt, 0, False, False)
        im, _, _ = GaussianRasterizer(cam)(**transformed_params2rendervar(gt, tg))
        ds, _, _ = GaussianRasterizer(cam)(**transformed_params2depthplussilhouette(gt, w2c, tg))
    curr = {"cam": cam, "w2c": w2c, "im": im.clone(), "depth": ds[0:1].clone()}
    params = as_parameters(base)
    variables = tracking_variables(P, dev)
    R = dgr.GaussianRasterizer
    track_frame_literal(params, variables, curr, 0, 10, renderer=R)  # warm-up (allocator, kernels)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(1, nf):
        track_frame_literal(params, variables, curr, f, iters_per_frame, renderer=R)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    iters = (nf - 1) * iters_per_frame
    # SURVEY 8(d)'s unit on its own: 2 x (GaussianRasterizer(...) + backward) from Python, eager, every
    # rasterizer input a leaf requiring grad, no caller glue (the rest of the loop body above is caller code)
    with torch.no_grad():
        tg = transform_to_frame(params, 0, False, False)
        rv1 = transformed_params2rendervar(params, tg)
        rv2 = transformed_params2depthplussilhouette(params, w2c, tg)
    leaf = lambda d: {k: v.detach().clone().requires_grad_(True) for k, v in d.items()}  # noqa: E731
    rv1, rv2 = leaf(rv1), leaf(rv2)
    rv2["means3D"] = rv1["means3D"]  # get_loss passes the same transformed means to both calls
    g1 = torch.randn(3, H, W, device=dev)
    g2 = torch.randn(3, H, W, device=dev)

    def unit():
        for d in (rv1, rv2):
            for v in d.values():
                v.grad = None
        im_, _, _ = R(cam)(**rv1)
        ds_, _, _ = R(cam)(**rv2)
        ((im_ * g1).sum() + (ds_ * g2).sum()).backward()

    for _ in range(5):
        unit()
    torch.cuda.synchronize()
    nu = 200
    t1 = time.perf_counter()
    for _ in range(nu):
        unit()
    torch.cuda.synchronize()
    du = (time.perf_counter() - t1) / nu
    profiling.enable_timing(True)  # separate pass: hipEvents around every stage
    track_frame_literal(params, variables, curr, 0, 10, renderer=R)
    torch.cuda.synchronize()
    st = profiling.read_timing()
    profiling.enable_timing(False)
    rb = st["render_bwd"]
    I_avg = st["render_fwd"]["units"] / max(st["render_fwd"]["launches"], 1)
    Tt = ((W + 15) // 16) * ((H + 15) // 16)
    alg = 8 * Tt + 40 * I_avg + 20 * W * H + 44 * P  # one single-image render backward
    return {"value": round(iters / dt, 3), "unit": "frames/s", "ms_per_step": round(1000 * dt / iters, 4),
            "iterations": iters,
            "path": "unchanged scripts/splatam.py tracking loop body: literal get_loss(tracking=True), "
                    "2x diff_gaussian_rasterization.GaussianRasterizer + loss.backward() + torch.optim.Adam "
                    "(all 7 groups) + best-candidate pose, eager",
            "render_bwd": {"avg_us": round(rb["avg_us"], 2), "launches_per_step": 2,
                           "alg_bytes_per_launch": int(alg),
                           "frac": round(alg / (rb["avg_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 5) if rb["avg_us"] else None},
            "stages_us": {k: round(v["avg_us"], 2) for k, v in st.items()},
            "raster_unit": {"value": round(1.0 / du, 3), "unit": "frames/s", "ms_per_step": round(1000 * du, 4),
                            "path": "SURVEY 8(d) unit alone: 2x diff_gaussian_rasterization.GaussianRasterizer "
                                    "(RGB, depth/silhouette) + backward from Python, eager, every input a leaf "
                                    "requiring grad (means3D shared by both calls, as in get_loss); the difference "
                                    "to ms_per_step is the caller's torch glue"}}


def dropin_mapping_leg(args, dev, iters: int = 60):
    """The unchanged mapping loop (scripts/splatam.py:841-905) at config 4: every parameter an
    nn.Parameter, a fresh torch.optim.Adam per frame over every group (eps 1e-15), per iteration a random
    keyframe, the literal get_loss(mapping=True) with two diff_gaussian_rasterization.GaussianRasterizer
    calls (SH colours, [z,1,z^2]), L1 + SSIM (torch conv2d) + masked depth L1, loss.backward(), step --
    eager, one Python iteration at a time, beside the HIP-graph mapping number."""
    import numpy as np
    import diff_gaussian_rasterization as dgr
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import MappingConfig, as_parameters, map_frame_literal, tracking_variables
    from splatam_amd.workloads import mapping_workload
    scene = config_scene(4)
    P, W, H = scene.P, scene.cam.W, scene.cam.H
    K = max(1, args.keyframes)
    base, cam, kfs = mapping_workload(scene, K, dev, prunable=args.map_prunable)  # the HIP-graph leg's window
    params = as_parameters(base)
    del base
    variables = tracking_variables(P, dev)
    variables["scene_radius"] = torch.max(kfs[0]["depth"]) / 3.0  # initialize_first_timestep (splatam.py:212)
    cfg = MappingConfig()
    rng = np.random.RandomState(0)
    map_frame_literal(params, variables, kfs, 3, cfg, renderer=dgr.GaussianRasterizer, rng=rng)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    map_frame_literal(params, variables, kfs, iters, cfg, renderer=dgr.GaussianRasterizer, rng=rng)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    survivors = int(params["means3D"].shape[0])
    del params, variables, kfs
    torch.cuda.empty_cache()
    return {"value": round(iters / dt, 3), "unit": "iterations/s", "ms_per_step": round(1000 * dt / iters, 4),
            "iterations": iters,
            "path": f"unchanged scripts/splatam.py mapping loop body at config 4 ({P} Gaussians, SH degree "
                    f"{scene.sh_degree}, {W}x{H}, {K} keyframes): literal get_loss(mapping=True) with 2x "
                    "diff_gaussian_rasterization.GaussianRasterizer, torch L1 + calc_ssim + masked depth L1, "
                    "loss.backward(), prune_gaussians at iterations 0 and 20 (configs/replica/splatam.py:101-111, "
                    "remove_points on the optimizer), torch.optim.Adam over every group (fresh per frame), eager; "
                    f"one {iters}-iteration frame; GS densification off (the config's default)",
            "survivors": survivors}


def fisher_leg(args, scene, dev, launches: int = 6, world: int = 1, rank: int = 0):
    """Fisher / EIG view scoring (scripts/ros_handler.py:807-902) on the bench map:
    the visited-pose Hessian sum H = sum_k [dL/dmeans_cam, dL/dopacity] of backward_power=2 renders seeded
    with 1e-3, K poses per HIP-graph launch (fisher.BatchedFisher), against the per-pose eager path.
    N > 1: the visited poses shard over the ranks (rank r scores poses rK .. rK + K - 1 of the ring, weak
    scaling) and the ranks' H sums meet in one all-reduce (compute_H_visited_inv's sum,
    ros_handler.py:807-829), inside the timed region; value = all ranks' poses / max-over-ranks time."""
    import math
    from splatam_amd import dist as sd
    from splatam_amd.fisher import BatchedFisher, FisherScorer
    from splatam_amd.slam import camera_settings, init_tracking_params
    params = init_tracking_params(scene, num_frames=1, device=dev)
    cam = camera_settings(scene.cam, dev)
    sc = FisherScorer(params, cam)
    K = max(1, args.fisher_k)

    def pose(k):  # a ring of views around the frame's camera: 0.5 deg yaw steps, 1 cm translations
        a = math.radians(0.5 * (k - K / 2))
        w = torch.eye(4, device=dev)
        w[0, 0], w[0, 2], w[2, 0], w[2, 2] = math.cos(a), math.sin(a), -math.sin(a), math.cos(a)
        w[:3, 3] = torch.tensor([0.01 * math.sin(k), 0.01 * math.cos(k), 0.0], device=dev)
        return w

    poses = [pose(k + rank * K) for k in range(K)]  # this rank's share of the visited poses
    bf = BatchedFisher(sc, K, mode="sum", probe_w2cs=poses)
    bf.hessian_sum(poses)
    H = torch.zeros_like(bf.out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(launches):
        h = bf.hessian_sum(poses)  # the default (checked) call: one host sync per launch
        if h is None:
            return {"error": "binning capacity overflow"}
        H.add_(h)
    sd.all_reduce_sum_(H)  # the visited-pose sum over all ranks' shares
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = sd.max_over_ranks(time.perf_counter() - t0, device=dev)
    sc.hessian(poses[0])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for w in poses[:4]:
        sc.hessian(w)
    torch.cuda.synchronize()
    de = (time.perf_counter() - t1) / 4
    dropin = fisher_dropin(params, cam, poses, dev)
    return {"value": round(K * launches * world / dt, 2), "unit": "poses/s", "poses_per_launch": K,
            "ranks": world, "ms_per_pose": round(1000 * dt / (K * launches), 4),
            "eager_ms_per_pose": round(1000 * de, 4),
            "dropin": dropin,
            "workload": f"H_train of {K} visited poses per HIP-graph launch over the {scene.P}-Gaussian "
                        f"{scene.cam.W}x{scene.cam.H} map: static forward + backward_power=2 per pose, "
                        "H accumulated on the device"}


def fisher_dropin(params, cam, poses, dev):
    """The reference's own Fisher caller, unchanged (scripts/ros_handler.py:839-902 compute_Hessian with
    return_points=True): per pose the map is moved into the candidate frame by torch glue, every rendervar
    is made to require grad, hessian_diff_gaussian_rasterization_w_depth.GaussianRasterizer(..,
    backward_power=2) renders, im.backward(1e-3 * ones) runs the full-gradient power-2 backward, and H =
    [transformed_pts.grad, opacities.grad].  Eager, one pose at a time; the render-backward kernels' own
    time is read from the stage timers in a separate pass."""
    import torch.nn.functional as F
    from hessian_diff_gaussian_rasterization_w_depth import GaussianRasterizer as Renderer
    from splatam_amd import profiling

    def compute_hessian(rel_w2c):
        with torch.no_grad():
            pts = params["means3D"]
            pts_ones = torch.ones(pts.shape[0], 1, device=dev).float()
            pts4 = torch.cat((pts, pts_ones), dim=1)
            transformed_pts = (rel_w2c @ pts4.T).T[:, :3]
            rgb_colors = params["rgb_colors"]
            rotations = F.normalize(params["unnorm_rotations"])
            opacities = torch.sigmoid(params["logit_opacities"])
            scales = torch.exp(params["log_scales"])
            if scales.shape[-1] == 1:
                scales = torch.tile(scales, (1, 3))
        num_points = transformed_pts.shape[0]
        rendervar = {"means3D": transformed_pts.requires_grad_(True),
                     "colors_precomp": rgb_colors.detach().clone().requires_grad_(True),
                     "rotations": rotations.requires_grad_(True), "opacities": opacities.requires_grad_(True),
                     "scales": scales.requires_grad_(True),
                     "means2D": torch.zeros_like(transformed_pts, requires_grad=True, device=dev) + 0}
        rendervar["means2D"].retain_grad()
        im, _, _ = Renderer(raster_settings=cam, backward_power=2)(**rendervar)
        im.backward(gradient=torch.ones_like(im) * 1e-3)
        cur_H = torch.cat([transformed_pts.grad.detach().reshape(num_points, -1),
                           opacities.grad.detach().reshape(num_points, -1)], dim=1)
        for v in rendervar.values():
            v.grad.fill_(0.)
        return cur_H

    for w in poses[:2]:
        compute_hessian(w)
    torch.cuda.synchronize()
    n = len(poses)
    t0 = time.perf_counter()
    for w in poses:
        compute_hessian(w)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    profiling.enable_timing(True)
    for w in poses[:4]:
        compute_hessian(w)
    torch.cuda.synchronize()
    st = profiling.read_timing()
    profiling.enable_timing(False)
    return {"value": round(1.0 / dt, 2), "unit": "poses/s", "ms_per_pose": round(1000 * dt, 4),
            "render_bwd_us": round(st["render_bwd"]["avg_us"], 2), "gauss_bwd_us": round(st["gauss_bwd"]["avg_us"], 2),
            "path": "unchanged scripts/ros_handler.py compute_Hessian: torch glue + hessian_diff_gaussian_"
                    "rasterization_w_depth.GaussianRasterizer(backward_power=2) with every rendervar requiring "
                    "grad + im.backward(1e-3), eager, one pose at a time"}


def unfused_render_leg(params, curr, frame, S, P, W, H, Tt, N, replays: int = 4):
    """The same tracking iterations with render_fwd and render_bwd as separate launches
    (GSR_TRACK_RENDER_FUSED=0's path): both kernels' in-kernel times, render_bwd's own roofline, frames/s."""
    from splatam_amd import glue, profiling
    from splatam_amd.tracker import GraphTracker
    prev = glue._RENDER_FUSED
    glue._RENDER_FUSED = False
    try:
        with torch.no_grad():
            q0 = params["cam_unnorm_rots"][..., frame].clone()
            t0 = params["cam_trans"][..., frame].clone()
        tr = GraphTracker(params, curr, frame, iters_per_graph=S, fuse_pose=True, warmup_iters=1, prime=True,
                          timing=True)
        profiling.enable_timing(clock_stages=profiling.CLOCK_STAGES)
        torch.cuda.synchronize()
        ta = time.perf_counter()
        tr.track_frame(S * replays, check=False)
        torch.cuda.synchronize()
        el = time.perf_counter() - ta
        st = profiling.read_timing()
        profiling.enable_timing(False)
        overflow = tr.overflowed()
        nr = tr.num_rendered()
        with torch.no_grad():
            params["cam_unnorm_rots"][..., frame] = q0
            params["cam_trans"][..., frame] = t0
        del tr
    finally:
        glue._RENDER_FUSED = prev
    I_avg = sum(nr) / len(nr)
    rb = st["render_bwd"]
    alg = 8 * Tt + 52 * I_avg + 32 * N + 56 * P
    dur = rb["avg_us"] * 1e-6
    return {"frames_per_s": round(S * replays / el, 2), "render_fwd_us": round(st["render_fwd"]["avg_us"], 2),
            "render_bwd_us": round(rb["avg_us"], 2), "render_bwd_alg_bytes": int(alg),
            "render_bwd_frac": round(alg / dur / 1e9 / HBM_PEAK_GBS, 5) if dur > 0 else None,
            "overflow": bool(overflow), "iterations": S * replays}


def committed_traffic(name):
    """roofline.traffic: calibrated HBM bytes per launch from a separate rocprofv3 PMC pass (FETCH_SIZE /
    WRITE_SIZE; counters cannot be collected inside the timed run), committed under profiles/ by
    tools/make_profiles.py -- returned with where it came from (file, summary, commit of the pass)."""
    pmc = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(pmc):
        return None, None
    try:
        d = json.load(open(pmc))
    except Exception:
        return None, None
    return d.get("hbm_bytes_per_launch"), {"kind": "committed PMC pass, not measured in this run",
                                           "file": f"profiles/{name}", "summary": d.get("source"),
                                           "commit": d.get("commit"), "kernel_avg_us_in_pass": d.get("kernel_avg_us")}


def render_bwd_roofline(rb, I_avg, P, W, H, graph: bool):
    """SURVEY.md 8(d) algorithmic bytes of one dual render-backward launch over its measured duration."""
    Tt = ((W + 15) // 16) * ((H + 15) // 16)
    N = W * H
    # 8*Tt + 40*I + 20*N + 44*P per rasterization, for the dual launch (both colour sets):
    # + colors2 gather 12*I, + dL_dpix2 12*N, + dcolors2 12*P
    bytes_per_launch = 8 * Tt + 52 * I_avg + 32 * N + 56 * P
    dur_s = rb["avg_us"] * 1e-6
    achieved = bytes_per_launch / dur_s / 1e9 if dur_s > 0 else 0.0
    return {"kernel": "render_bwd_kernel", "bound": "hbm", "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": None, "alg_bytes_per_launch": int(bytes_per_launch), "avg_us": round(rb["avg_us"], 2),
            "num_rendered_avg": int(I_avg), "launches_timed": int(rb["launches"]),
            "timing": "in-kernel wall_clock64 (first workgroup start to last workgroup end) of every launch in "
                      "the timed HIP-graph replays" if graph else "hipEvents around each launch"}


def sequence_leg(args, dev):
    """SplaTAM's per-frame loop (scripts/splatam.py:697-929) at config 3's scene: --seq-frames frames, each
    40 tracking iterations (constant-velocity start, best candidate written back), add_new_gaussians and 60
    mapping iterations over the keyframe window (prune_gaussians at 0 and 20).  `value`: frames/s of
    SlamSequence (capacity-padded map, one GraphTracker + one GraphMapper for the whole sequence, densification
    on the device without a host sync); `per_frame`: the same frames with a fresh GraphTracker and GraphMapper
    per frame (probe + warm-up + capture each, torch.cat densification, compaction after pruning) -- everything
    a shape-changing map costs, inside the timed region.  Construction and frames 0 (mapping only) and 1 (the
    first densification) untimed, for both forms; the timed frames are 2 .. K + 1."""
    from splatam_amd.scenes import config_scene
    from splatam_amd.sequence import PerFrameSlam, SlamSequence
    from splatam_amd.tracker import probe_num_rendered
    from splatam_amd.workloads import sequence_workload

    K = max(1, args.seq_frames)
    scene = config_scene(3)
    P, W, H = scene.P, scene.cam.W, scene.cam.H
    params, frames, cam, w2c, intr, (q_gt, t_gt) = sequence_workload(scene, K + 2, dev, prunable=args.map_prunable)
    P0 = params["means3D"].shape[0]
    n, _ = probe_num_rendered(params, {"cam": cam, "w2c": w2c, **frames[0]}, 0)
    headroom = args.seq_headroom if args.seq_headroom is not None else W * H // 3
    capacity, bin_cap = P0 + headroom, 2 * n + 2_000_000
    t0 = time.perf_counter()
    seq = SlamSequence(params, frames, cam, w2c, intr, capacity=capacity, bin_capacity=bin_cap, seed=0)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    W0 = 2  # untimed warm-up frames: 0 (mapping only) and 1 (the first densification: allocator, kernels)
    for t in range(W0):
        seq.frame(t)
    seq.check()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j, t in enumerate(range(W0, W0 + K)):
        ev[j][0].record()
        seq.track(t)
        ev[j][1].record()
        seq.densify(t)
        ev[j][2].record()
        seq.map(t)
        ev[j][3].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    seq.check()
    phases = {name: round(sum(e[i].elapsed_time(e[i + 1]) for e in ev) / K, 3)
              for i, name in enumerate(("tracking_ms", "densify_ms", "mapping_ms"))}
    n_live = int(seq.n_live.item())
    live = int(seq.alive.sum().item())
    te = float((seq.params["cam_trans"][..., 1:W0 + K] - t_gt[..., 1:W0 + K]).norm(dim=1).max())
    # the per-frame form on the same frames and keyframe draws (its own probes; checked runs)
    ref = PerFrameSlam(params, frames, cam, w2c, intr)
    for t in range(W0):
        ref.frame(t, seq.draws[t])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(W0, W0 + K):
        ref.frame(t, seq.draws[t])
    torch.cuda.synchronize()
    elapsed_ref = time.perf_counter() - t0
    dpose = float((seq.params["cam_trans"] - ref.p["cam_trans"]).abs().max())
    out = {"metric": "SLAM frames/sec (40 tracking + densification + 60 mapping iterations per frame)",
           "value": round(K / elapsed, 3), "unit": "frames/s", "ms_per_frame": round(1000.0 * elapsed / K, 3),
           "frames": K, "phases_ms": phases,
           "per_frame": {"value": round(K / elapsed_ref, 3), "ms_per_frame": round(1000.0 * elapsed_ref / K, 3),
                         "form": "fresh GraphTracker + GraphMapper per frame (probe, warm-up, capture), torch.cat "
                                 "densification, compact() after pruning",
                         "max_pose_diff_m": dpose, "gaussians": int(ref.p["means3D"].shape[0])},
           "map": {"initial": P0, "appended": n_live - P0, "live": live, "capacity": capacity,
                   "binning_capacity": bin_cap},
           "pose_error_m": round(te, 5), "setup_s": round(t_build, 3),
           "config": {"workload": f"config 3 scene ({P} isotropic Gaussians, {W}x{H}); the map starts without "
                                  f"the left 20 % of frame 0 (densified), {args.map_prunable:g} of it prunable; "
                                  "camera 2 cm + 0.3 deg per frame", "gaussians": P, "width": W, "height": H},
           "data": "synthetic (splatam_amd.workloads.sequence_workload: targets rendered from the full scene "
                   "along the trajectory, 1 % depth noise)"}
    del seq, ref
    torch.cuda.empty_cache()
    return out


def main_mapping(args, world, rank, dev):
    line = run_mapping(args, world, rank, dev)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def mapping_leg(args, dev):
    """BASELINE config 4 (the mapping workload) inside the default bench line, so the round-end driver run
    records it too: the same measurement as `--workload mapping` (rank 0, N=1 only)."""
    import copy
    a = copy.copy(args)
    a.config, a.steps, a.warmup = 4, max(1, args.mapping_steps), args.map_frame_iters
    line = run_mapping(a, 1, 0, dev)
    keep = ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "execution", "config", "roofline",
            "stages_us", "stages_source", "pruning")
    return {k: line[k] for k in keep}


def run_mapping(args, world, rank, dev):
    """SplaTAM mapping iterations (scripts/splatam.py:842-905, get_loss mapping=True): one step = one
    iteration = transform + RGB(SH) and depth/silhouette render fwd+bwd (one dual rasterization) +
    0.8 L1 + 0.2 (1 - SSIM) + masked depth L1 + Adam on every Gaussian parameter; replayed as a HIP
    graph of --iters-per-graph iterations (one frame's mapping with a fresh optimizer), keyframes drawn
    from a window of --keyframes synthetic frames.  Frame-sharded over ranks like tracking."""
    from splatam_amd import dist as sd
    from splatam_amd import profiling
    from splatam_amd.mapper import GraphMapper
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import MappingConfig, color_key
    from splatam_amd.workloads import mapping_workload

    scene = config_scene(args.config)
    P, W, H = scene.P, scene.cam.W, scene.cam.H
    K = max(1, args.keyframes)
    # keyframe targets: the map with perturbed colours; --map-prunable of the Gaussians faded under
    # prune_gaussians' 0.005 opacity threshold, so the frame's pruning iterations remove them
    params, cam, kfs = mapping_workload(scene, K, dev, rank=rank, world=world, prunable=args.map_prunable)
    sd.broadcast_map(params, keys=tuple(k for k in params))
    w2c = torch.eye(4, device=dev)
    key = color_key(params)
    for k in ("means3D", "unnorm_rotations", "logit_opacities", "log_scales", key):
        params[k].requires_grad_(True)
    # one replay = one frame of --map-frame-iters iterations (fresh Adam, prune_gaussians at the iterations
    # pruning_dict names: 0 and 20 of 60); exactly `steps` timed iterations, rounded up to whole frames
    S = max(1, args.map_frame_iters)
    steps = S * max(1, -(-max(1, args.steps) // S))
    scene_radius = torch.max(kfs[0]["depth"]) / 3.0  # initialize_first_timestep (splatam.py:212), ratio 3 (replica)
    import contextlib
    from splatam_amd import _C
    binning = _C.reference_binning() if getattr(args, "map_binning", "culled") == "reference" else \
        contextlib.nullcontext()
    snap = {k: params[k].detach().clone() for k in ("means3D", "unnorm_rotations", "logit_opacities", "log_scales",
                                                     key)}  # (the stage-breakdown pass starts from the same map)
    with binning:  # (captured into the graph: every replay bins this way)
        # the timed replays clock the render kernels only (each clocked launch pays its workgroups' clock
        # atomics); the other stages come from a separate all-clocks mapper after the timed region
        mapper = GraphMapper(params, kfs, iters_per_graph=S, cfg=MappingConfig(), timing=bool(args.timing),
                             prune=bool(args.map_prune), scene_radius=scene_radius,
                             clock_stages=("render_fwd", "render_bwd"))
    for _ in range(max(1, -(-args.warmup // S))):  # >= W untimed iterations (whole replays)
        mapper.run()  # checked: raises on an overflow
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    profiling.enable_timing(clock_stages=profiling.CLOCK_STAGES)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // S):
        mapper.run(check=False)  # no host sync inside the timed region; overflowed() read after it
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    stages = profiling.read_timing()
    profiling.enable_timing(False)
    if mapper.overflowed():
        raise SystemExit(f"binning capacity overflow during the timed replays (capacity {mapper.capacity}): "
                         "measurement invalid")
    survivors = int(mapper.survivors().sum().item())
    nr = mapper.num_rendered()
    mcap, prune_iters = mapper.capacity, sorted(mapper.prune_at)
    stages_all = None
    if args.timing and getattr(args, "stage_breakdown", "on") == "on":  # every stage clocked, one untimed frame
        del mapper
        with torch.no_grad():
            for k, v in snap.items():
                params[k].copy_(v)
        with binning:
            mb = GraphMapper(params, kfs, iters_per_graph=S, cfg=MappingConfig(), timing=True,
                             prune=bool(args.map_prune), scene_radius=scene_radius, capacity=mcap)
        profiling.enable_timing(clock_stages=profiling.CLOCK_STAGES)
        mb.run(check=False)
        torch.cuda.synchronize()
        stages_all = profiling.read_timing()
        profiling.enable_timing(False)
        del mb
    del snap
    elapsed = sd.max_over_ranks(t1 - t0, device=dev)
    value = steps * world / elapsed
    roofline = render_bwd_roofline(stages["render_bwd"], sum(nr) / len(nr), P, W, H, graph=True)
    roofline["traffic"], roofline["traffic_source"] = committed_traffic("mapping_render_bwd_pmc.json")
    line = {
        "metric": f"mapping iterations/sec @{W}x{H}, {P // 1000}k anisotropic Gaussians, SH degree "
                  f"{scene.sh_degree}", "value": round(value, 3), "unit": "iterations/s", "n_gpus": world,
        "steps": steps, "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "execution": f"HIP graph of {S} mapping iterations (one frame, fresh Adam), replayed "
                     f"{steps // S}x; binning capacity {mcap}, no overflow",
        "pruning": ({"iterations": prune_iters, "survivors": survivors, "gaussians": P,
                     "path": "prune_gaussians inside the frame (scripts/splatam.py:876-878, configs/replica/"
                             "splatam.py:101-111): device alive mask (gsr_map_prune), pruned Gaussians culled by "
                             "the static forward; a pruning iteration is its loss forward only (the reference's "
                             "optimizer.step() updates no Gaussian there: remove_points drops every .grad)"}
                    if prune_iters else None),
        "data": f"synthetic (SURVEY.md 8(d) seeded scene; {K} keyframe targets rendered from a perturbed map)",
        "config": {"workload": f"config {args.config}: {P} Gaussians, {W}x{H}, SplaTAM mapping iteration "
                               "(SH colour + depth/silhouette render fwd+bwd, L1 + SSIM + depth L1, Adam on "
                               "all Gaussian parameters)", "gaussians": P, "width": W, "height": H,
                   "keyframes": K, "parallelism": f"frame-sharded x{world}",
                   "binning": getattr(args, "map_binning", "culled")},
        "roofline": roofline,
        "stages_us": {k: round(v["avg_us"], 2) for k, v in (stages_all or stages).items() if v["launches"]},
        "stages_source": ("a separate untimed frame with every kernel's in-kernel stage clock on (the timed "
                          "replays clock the render kernels only)" if stages_all else
                          "the timed replays' in-kernel stage clocks (render kernels)"),
    }
    del params, kfs
    torch.cuda.empty_cache()
    return line


if __name__ == "__main__":
    main()
