"""SLAM sequence on one HIP-graph tracker and one HIP-graph mapper (splatam_amd.sequence) against the
per-frame loop of fresh GraphTrackers / GraphMappers on an unpadded map that grows by torch.cat
(add_new_gaussians_literal) -- the form in which P changes every frame, scripts/splatam.py:697-929.

The capacity-padded map keeps its free rows dead (culled by the alive mask), appends the densified Gaussians
at n_live + rank and, after a frame's pruning, moves the live rows to the front in order (compact_static); its
live rows are then the literal map's rows in the literal map's order, both forms run the same kernels on the
same Gaussians in the same order, and the poses and the map agree bitwise -- with and without pruning, and
when the map outgrows its buffer mid-sequence (ensure_headroom: a larger buffer, the graphs rebuilt)."""
import pytest
import torch

from splatam_amd.mapper import GAUSS_KEYS
from splatam_amd.scenes import make_scene
from splatam_amd.sequence import PerFrameSlam, SlamSequence
from splatam_amd.workloads import sequence_workload

pytestmark = pytest.mark.gpu

N_FRAMES = 3


@pytest.fixture(scope="module")
def capture(cuda):
    scene = make_scene(20_000, 320, 240, seed=7)
    return sequence_workload(scene, N_FRAMES, torch.device(cuda))


def _literal(params0, frames, cam, w2c, intr, draws, bin_cap, prune):
    ref = PerFrameSlam(params0, frames, cam, w2c, intr, prune=prune, bin_capacity=bin_cap)
    for t in range(N_FRAMES):
        ref.frame(t, draws[t])
    torch.cuda.synchronize()
    return ref.p


def _run_sequence(capture, prune, grow=False):
    params, frames, cam, w2c, intr, _ = capture
    from splatam_amd.tracker import probe_num_rendered
    n, _ = probe_num_rendered(params, {"cam": cam, "w2c": w2c, "im": frames[0]["im"], "depth": frames[0]["depth"]}, 0)
    bin_cap = 4 * n + 400_000
    P0 = params["means3D"].shape[0]
    seq = SlamSequence(params, frames, cam, w2c, intr, capacity=P0 + (1000 if grow else 2 * 320 * 240),
                       bin_capacity=bin_cap, prune=prune, seed=0)
    grew = 0
    for t in range(N_FRAMES):
        if grow:  # the capacity runs out after frame 0: the map moves to a larger buffer, graphs rebuilt
            grew += seq.ensure_headroom(320 * 240)
        seq.frame(t)
    if grow:
        assert grew >= 1 and seq.capacity > P0 + 1000
    seq.check()
    torch.cuda.synchronize()
    return seq, bin_cap


@pytest.mark.parametrize("prune,grow", [(False, False), (True, False), (True, True)])
def test_sequence_equals_per_frame_loop(cuda, capture, prune, grow):
    params, frames, cam, w2c, intr, (q_gt, t_gt) = capture
    seq, bin_cap = _run_sequence(capture, prune, grow)
    ref = _literal(params, frames, cam, w2c, intr, seq.draws, bin_cap, prune)
    live = seq.live_params()
    P0, Pn = params["means3D"].shape[0], live["means3D"].shape[0]
    added = int(seq.n_live.item()) - P0
    print(f"prune={prune}: P0 {P0}, appended {added}, live {Pn}, literal {ref['means3D'].shape[0]}")
    assert added > 1000  # the hole was densified
    assert Pn == ref["means3D"].shape[0]
    dq = float((seq.params["cam_unnorm_rots"] - ref["cam_unnorm_rots"]).abs().max())
    dt = float((seq.params["cam_trans"] - ref["cam_trans"]).abs().max())
    errs = {k: float((live[k] - ref[k]).abs().max()) for k in GAUSS_KEYS + ("rgb_colors",)}
    print(f"  pose max |d| q {dq:.3e} t {dt:.3e}; map {errs}")
    # tracking follows the trajectory (2 cm / 0.3 deg per frame)
    te = float((seq.params["cam_trans"][..., 1:] - t_gt[..., 1:]).abs().max())
    print(f"  translation error {te:.4f} m")
    assert te < 1e-2
    assert dq == 0.0 and dt == 0.0
    assert all(e == 0.0 for e in errs.values())
