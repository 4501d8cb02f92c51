"""Fisher / EIG scoring alone (bench.py's fisher leg without the tracking run): BatchedFisher over the
config-3 map, K poses per HIP-graph launch, `--launches` timed launches.  For rocprofv3 kernel traces of
the per-pose pipeline.  Usage: python tools/fisher_bench.py [--k 16] [--launches 20]"""
import argparse
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--config", type=int, default=3)
    a = ap.parse_args()
    from splatam_amd.fisher import BatchedFisher, FisherScorer
    from splatam_amd.scenes import config_scene
    from splatam_amd.slam import camera_settings, init_tracking_params
    dev = torch.device("cuda", 0)
    scene = config_scene(a.config)
    params = init_tracking_params(scene, num_frames=1, device=dev)
    sc = FisherScorer(params, camera_settings(scene.cam, dev))
    K = a.k

    def pose(k):
        ang = math.radians(0.5 * (k - K / 2))
        w = torch.eye(4, device=dev)
        w[0, 0], w[0, 2], w[2, 0], w[2, 2] = math.cos(ang), math.sin(ang), -math.sin(ang), math.cos(ang)
        w[:3, 3] = torch.tensor([0.01 * math.sin(k), 0.01 * math.cos(k), 0.0], device=dev)
        return w

    poses = [pose(k) for k in range(K)]
    bf = BatchedFisher(sc, K, mode="sum", probe_w2cs=poses)
    bf.hessian_sum(poses)
    torch.cuda.synchronize()
    bf.status.zero_()
    t0 = time.perf_counter()
    for _ in range(a.launches):
        bf.hessian_sum(poses, check=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert not bf.overflowed()
    print(f"fisher: {K * a.launches / dt:.1f} poses/s, {1e3 * dt / (K * a.launches):.4f} ms/pose")


if __name__ == "__main__":
    main()
