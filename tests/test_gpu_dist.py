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
