"""Microbenchmark of the tracking pose backward (gsr_track_transform_bwd[_adam]):
duration against P, to split the per-Gaussian streaming part from the fixed
reduction tail (last workgroup + pose_fin)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from splatam_amd._lib import lib  # noqa: E402


def run(P, adam, iters=200):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    mw = torch.randn(P, 3, device=dev, generator=g)
    ur = torch.randn(P, 4, device=dev, generator=g)
    mc = torch.randn(P, 3, device=dev, generator=g)
    gm = torch.randn(P, 3, device=dev, generator=g)
    gd = torch.randn(P, 3, device=dev, generator=g)
    q = torch.tensor([[1.0], [0.0], [0.0], [0.0]], device=dev)
    t = torch.zeros(3, 1, device=dev)
    w2c = torch.eye(4, device=dev)
    state = torch.zeros(32, device=dev)
    scratch = torch.zeros(lib.gsr_track_scratch_floats(P), device=dev)
    dq = torch.zeros_like(q)
    dt = torch.zeros_like(t)
    s = torch.cuda.current_stream().cuda_stream

    def once():
        if adam:
            rc = lib.gsr_track_transform_bwd_adam(P, mw.data_ptr(), ur.data_ptr(), 1, q.data_ptr(), t.data_ptr(), 1,
                                                  mc.data_ptr(), w2c.data_ptr(), gm.data_ptr(), None, gd.data_ptr(),
                                                  1e-4, 1e-3, 0.9, 0.999, 1e-8, state.data_ptr(), scratch.data_ptr(), s)
        else:
            rc = lib.gsr_track_transform_bwd(P, mw.data_ptr(), ur.data_ptr(), 1, q.data_ptr(), mc.data_ptr(),
                                             w2c.data_ptr(), gm.data_ptr(), None, gd.data_ptr(), dq.data_ptr(),
                                             dt.data_ptr(), 1, scratch.data_ptr(), s)
        assert rc == 0

    for _ in range(20):
        once()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        once()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / iters


if __name__ == "__main__":
    for adam in (False, True):
        for P in (1000, 65536, 300000, 600000):
            print(f"adam={adam} P={P:7d}: {run(P, adam):7.2f} us/launch (back-to-back)")
