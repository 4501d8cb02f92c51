"""The multi-process bench path on the GPU: two ranks, one process each, launched by
torch.distributed.run exactly as the driver launches bench.py for N > 1, sharing this box's one GPU.
Collectives go over gloo here (GSR_DIST_BACKEND=gloo: RCCL refuses two ranks on one device); the
per-rank work -- frame sharding, the map broadcast between HIP-graph replays, the max-over-ranks clock,
the whole-job value -- is the nccl path's.  (The 8-GPU RCCL run is the driver's.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks(cuda):
    env = dict(os.environ, GSR_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29517", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "40", "--warmup", "5", "--bcast-every", "40", "--dropin", "off", "--fisher", "off",
           "--mapping", "off", "--cpu-baseline", "off"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one JSON line
    b = lines[0]
    print(json.dumps({k: b[k] for k in ("value", "n_gpus", "steps", "ms_per_step", "scaling")}))
    assert b["n_gpus"] == 2 and b["steps"] == 40 and b["scaling"] == "weak"
    assert b["config"]["parallelism"] == "frame-sharded x2" and b["config"]["broadcast_every"] == 40
    # value = frames of both ranks / max-over-ranks wall time
    assert abs(b["value"] - 2 * 40 / (b["ms_per_step"] * 40 / 1e3)) <= 0.01 * b["value"]
    assert b["roofline"]["launches_timed"] == 40 and b["roofline"]["avg_us"] > 0
    # the N > 1 line: the single-call flat-buffer broadcast timed alone, and the frames without it
    bs = b["broadcast"]
    assert bs["broadcast_ms"] > 0 and bs["value_no_broadcast"] > 0 and bs["broadcasts_in_timed_region"] == 1
    assert bs["broadcast_bytes"] == 300000 * (3 + 3 + 4 + 1 + 1) * 4 and "one RCCL broadcast" in bs["broadcast_path"]


_RCCL_SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from splatam_amd import dist as sd
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))  # bench.py's call (RCCL)
p = {"means3D": torch.arange(12., device="cuda").reshape(4, 3), "rgb_colors": torch.ones(4, 3, device="cuda")}
n = sd.broadcast_map(p, keys=("means3D", "rgb_colors"))
for k in ("means3D", "rgb_colors"):  # the collectives the helpers issue when world > 1, issued directly
    dist.broadcast(p[k].data, src=0)
dist.barrier()
t = torch.full((3,), 2.0, device="cuda")
dist.all_reduce(t, op=dist.ReduceOp.SUM)
x = torch.tensor([0.25], dtype=torch.float64, device="cuda")
dist.all_reduce(x, op=dist.ReduceOp.MAX)
m = sd.max_over_ranks(float(x), device=torch.device("cuda", 0))
print("RCCL", dist.get_backend(), dist.get_world_size(), n, t.tolist(), m, float(p["means3D"].sum()))
dist.destroy_process_group()
"""


def test_rccl_single_rank(cuda):
    """bench.py's RCCL calls (init_process_group("nccl", device_id), map broadcast, barrier, all-reduce,
    max over ranks) on this box's one GPU with one rank: the nccl backend is RCCL on ROCm, and this is the
    code path the driver's multi-GPU runs take (two ranks cannot share one device under RCCL)."""
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29531")
    r = subprocess.run([sys.executable, "-c", _RCCL_SCRIPT, ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RCCL")][-1]
    print(line)
    f = line.split()
    assert f[1] == "nccl" and f[2] == "1" and f[-1] == "66.0"


_FISHER_SCRIPT = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from splatam_amd import dist as sd
from splatam_amd.fisher import BatchedFisher, FisherScorer
from splatam_amd.scenes import make_scene
from splatam_amd.slam import camera_settings, init_tracking_params
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
scene = make_scene(20000, 160, 120, seed=4)
params = init_tracking_params(scene, num_frames=1, device=dev)
sc = FisherScorer(params, camera_settings(scene.cam, dev))
K = 4
def pose(k):
    w = torch.eye(4, device=dev)
    w[:3, 3] = torch.tensor([0.01 * k, -0.005 * k, 0.02], device=dev)
    return w
allp = [pose(k) for k in range(K * world)]
bf = BatchedFisher(sc, K, mode="sum", probe_w2cs=allp)
H = bf.hessian_sum(allp[rank * K:(rank + 1) * K]).clone()   # this rank's share
sd.all_reduce_sum_(H)                                        # the visited-pose sum over the ranks
ok = True
if rank == 0:                                                # one rank, every pose, the same two launch sums
    ref = bf.hessian_sum(allp[0:K]).clone() + bf.hessian_sum(allp[K:2 * K]).clone()
    ok = torch.equal(H, ref) and float(H.abs().sum()) > 0
print("FISHER", rank, world, ok)
dist.destroy_process_group()
"""


def test_fisher_sharded_sum_two_ranks(cuda):
    """bench.py's sharded Fisher leg: two ranks (gloo, this box's GPU) each sum the Hessians of their half of
    the visited poses and all-reduce; the result is bitwise the one-rank sum of the same two launch sums."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29523", "--no-python", sys.executable, "-c", _FISHER_SCRIPT,
           ROOT]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = sorted(l for l in r.stdout.splitlines() if l.startswith("FISHER"))
    assert lines == ["FISHER 0 2 True", "FISHER 1 2 True"], r.stdout[-2000:]
