"""Diagnostic: status rows of static-mode dual forwards (eager and graph-replayed)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from splatam_amd import profiling  # noqa: E402
from splatam_amd.scenes import config_scene  # noqa: E402
from splatam_amd.slam import _get_loss_tracking_fused, TrackingConfig, camera_settings, init_tracking_params  # noqa
from splatam_amd.tracker import GraphTracker, probe_num_rendered  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    s = config_scene(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
    params = init_tracking_params(s, 1, dev)
    cam = camera_settings(s.cam, dev)
    curr = {"cam": cam, "w2c": torch.eye(4, device=dev), "im": torch.rand(3, s.cam.H, s.cam.W, device=dev),
            "depth": torch.rand(1, s.cam.H, s.cam.W, device=dev) + 1}
    params["cam_unnorm_rots"].requires_grad_(True)
    params["cam_trans"].requires_grad_(True)
    n, longest = probe_num_rendered(params, curr, 0)
    print("probe", n, longest)
    cap = int(1.5 * n) + 65536
    st = torch.zeros(20, 4, dtype=torch.int32, device=dev)
    opt = torch.optim.Adam([params["cam_unnorm_rots"], params["cam_trans"]], lr=1e-3, fused=True)
    for k in range(20):  # eager static iterations, forward + backward + Adam
        opt.zero_grad(set_to_none=True)
        loss, _, _ = _get_loss_tracking_fused(params, curr, 0, TrackingConfig(), True, cap, st[k])
        loss.backward()
        opt.step()
        del loss
    torch.cuda.synchronize()
    rows = st.cpu()
    print("eager static bad rows", [i for i in range(20) if rows[i, 1] != 0 or rows[i, 0] > cap])
    for p_ in (params["cam_unnorm_rots"], params["cam_trans"]):
        p_.grad = None
    for timing in (False, True):
        tr = GraphTracker(params, curr, 0, iters_per_graph=20, timing=timing)
        for r in range(3):
            tr.run()
            torch.cuda.synchronize()
            rows = tr.status.cpu()
            bad = [i for i in range(rows.shape[0]) if rows[i, 1] != 0 or rows[i, 0] > tr.capacity]
            print("graph timing", timing, "replay", r, "bad rows", bad, [rows[i].tolist() for i in bad][:4])
    profiling.enable_timing(False)


if __name__ == "__main__":
    main()
