"""Frame-sharding orchestration (splatam_amd.dist) with world_size 2 on gloo (CPU)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splatam_amd import dist as sd
    from splatam_amd.scenes import make_scene
    from splatam_amd.slam import init_tracking_params
    scene = make_scene(100, 32, 32, seed=rank)          # ranks start from different maps
    params = init_tracking_params(scene, num_frames=4, device="cpu")
    sent = sd.broadcast_map(params)
    ref = init_tracking_params(make_scene(100, 32, 32, seed=0), num_frames=4, device="cpu")
    same = all(torch.equal(params[k], ref[k]) for k in sd.MAP_KEYS)
    frames = sd.frames_for_rank(5)
    h = torch.full((100, 4), float(rank + 1))
    sd.all_reduce_sum_(h)
    t = sd.max_over_ranks(0.5 + rank)
    q.put((rank, same, frames, float(h[0, 0]), t, sent))
    dist.destroy_process_group()


def test_frame_sharding_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, same0, f0, h0, t0, sent0), (r1, same1, f1, h1, t1, sent1) = res
    assert same0 and same1                       # rank 1 received rank 0's map
    assert f0 == [0, 2, 4] and f1 == [1, 3]      # disjoint, covering frames
    assert h0 == h1 == 3.0                       # Fisher / Hessian merge
    assert t0 == t1 == 1.5                       # max-over-ranks timing
    assert sent0 == 100 * (3 + 3 + 4 + 1 + 1) * 4


def _fisher_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splatam_amd.fisher import FisherScorer

    def fake_hessian(w2c):  # deterministic per pose, positive like a Fisher diagonal
        s = float(w2c[0, 3]) + 1.0
        return torch.arange(40, dtype=torch.float32).reshape(10, 4) * s + s

    params = {"means3D": torch.zeros(10, 3)}
    sc = FisherScorer(params, None, hessian_fn=fake_hessian)
    visited = [torch.eye(4) for _ in range(3)]
    for j, v in enumerate(visited):
        v[0, 3] = float(j)
    cands = [torch.eye(4) for _ in range(5)]
    for j, c in enumerate(cands):
        c[0, 3] = 0.5 * j
    hinv = sc.fit_visited(visited)
    scores = sc.eig_scores(cands)
    # plain lists: a tensor on a multiprocessing queue is shared through the sender's file
    # descriptors, which vanish when the sender exits before the parent reads it
    q.put((rank, hinv.tolist(), scores.tolist()))
    dist.destroy_process_group()


def test_fisher_scoring_sharded_world2():
    """Visited-pose Hessians summed across ranks (all-reduce) and candidate EIG scores
    gathered in pose order equal the single-process result (ros_handler.py:807-836)."""
    from splatam_amd.fisher import FisherScorer
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fisher_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    def fake_hessian(w2c):
        s = float(w2c[0, 3]) + 1.0
        return torch.arange(40, dtype=torch.float32).reshape(10, 4) * s + s

    ref = FisherScorer({"means3D": torch.zeros(10, 3)}, None, hessian_fn=fake_hessian)
    visited = [torch.eye(4) for _ in range(3)]
    for j, v in enumerate(visited):
        v[0, 3] = float(j)
    cands = [torch.eye(4) for _ in range(5)]
    for j, c in enumerate(cands):
        c[0, 3] = 0.5 * j
    hinv = ref.fit_visited(visited)
    scores = ref.eig_scores(cands)
    for _, h, s in res:
        assert torch.allclose(torch.tensor(h, dtype=hinv.dtype), hinv) and torch.allclose(torch.tensor(s, dtype=scores.dtype), scores)
    assert bool((scores[1:] > scores[:-1]).all())


def _flat_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from splatam_amd import dist as sd
    from splatam_amd.scenes import make_scene
    from splatam_amd.slam import init_tracking_params
    params = init_tracking_params(make_scene(100, 32, 32, seed=rank), num_frames=4, device="cpu")
    objs = {k: params[k] for k in sd.MAP_KEYS}
    fm = sd.FlatMap(params)
    seated = all(params[k] is objs[k] for k in sd.MAP_KEYS) and fm.check()  # same tensor objects, new storage
    sent = sd.broadcast_flat(fm)  # one collective: rank 1 now holds rank 0's map
    ref0 = init_tracking_params(make_scene(100, 32, 32, seed=0), num_frames=4, device="cpu")
    same = all(torch.equal(params[k], ref0[k]) for k in sd.MAP_KEYS)
    # double-buffered: rank 0 updates its map, starts the broadcast, keeps updating; rank 1 keeps the old
    # version until finish(), then holds exactly the version rank 0 had at start()
    bc = sd.MapBroadcaster(fm)
    if rank == 0:
        with torch.no_grad():
            params["means3D"].add_(1.0)
    v1 = params["means3D"].clone() if rank == 0 else None
    bc.start()
    stale = torch.equal(params["means3D"], ref0["means3D"]) if rank == 1 else True
    if rank == 0:
        with torch.no_grad():
            params["means3D"].add_(5.0)  # after start(): not part of this broadcast
    bc.finish()
    got = params["means3D"].clone()
    dist.broadcast(v1 if rank == 0 else (v1 := torch.empty_like(got)), src=0)  # rank 0's start() version
    fresh = torch.equal(got, v1) if rank == 1 else torch.equal(got, v1 + 5.0)
    q.put((rank, seated, sent, same, stale, fresh))
    dist.destroy_process_group()


def test_flat_map_broadcast_world2():
    """FlatMap re-seats the map tensors as views of one buffer (the same tensor objects) and broadcast_flat
    moves the whole map in one collective; MapBroadcaster's double buffer leaves the receiving rank on the
    old map until finish(), then on exactly the version the source had at start() (bitwise)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_flat_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, seated, sent, same, stale, fresh in res:
        assert seated and same and stale and fresh, (rank, seated, same, stale, fresh)
        assert sent == 100 * (3 + 3 + 4 + 1 + 1) * 4
