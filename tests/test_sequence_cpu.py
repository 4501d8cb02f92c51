"""Host-side pieces of the SLAM sequence (splatam_amd.sequence) on the CPU: the capacity-padded map, its
in-place compaction after pruning (remove_points' result, utils/slam_external.py:141-163, without a
reallocation) and the constant-velocity pose initialisation (scripts/splatam.py:429-448)."""
import torch
import torch.nn.functional as F

from splatam_amd.sequence import compact_static, initialize_camera_pose, pad_map


def _map(P, T=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    return {"means3D": torch.randn(P, 3, generator=g), "rgb_colors": torch.rand(P, 3, generator=g),
            "unnorm_rotations": torch.randn(P, 4, generator=g), "logit_opacities": torch.randn(P, 1, generator=g),
            "log_scales": torch.randn(P, 1, generator=g), "cam_unnorm_rots": torch.randn(1, 4, T, generator=g),
            "cam_trans": torch.randn(1, 3, T, generator=g)}


def test_pad_map_rows_and_dead_fill():
    m = _map(50)
    p, alive, n = pad_map(m, 80)
    assert int(n) == 50 and alive.shape == (81,) and int(alive.sum()) == 50 and bool(alive[:50].all())
    for k in ("means3D", "rgb_colors", "unnorm_rotations", "logit_opacities", "log_scales"):
        assert p[k].shape[0] == 81 and torch.equal(p[k][:50], m[k])
        assert torch.isfinite(p[k]).all()
    assert torch.equal(p["unnorm_rotations"][50:], torch.tensor([1.0, 0, 0, 0]).expand(31, 4))
    assert p["cam_trans"] is m["cam_trans"]  # camera tensors as they are


def test_compact_static_equals_boolean_compaction():
    m = _map(200, seed=1)
    p, alive, n = pad_map(m, 300)
    g = torch.Generator().manual_seed(7)
    dead = torch.randperm(200, generator=g)[:37]
    alive[dead] = 0
    keep = alive[:200].bool()
    want = {k: m[k][keep] for k in ("means3D", "rgb_colors", "unnorm_rotations", "logit_opacities", "log_scales")}
    compact_static(p, alive, n, 300)
    assert int(n) == 163 and int(alive.sum()) == 163 and bool(alive[:163].all()) and not bool(alive[163:].any())
    for k, v in want.items():
        assert torch.equal(p[k][:163], v), k  # the survivors, in order, at the front


def test_initialize_camera_pose_constant_velocity():
    m = _map(4, T=4, seed=3)
    q, t = m["cam_unnorm_rots"].clone(), m["cam_trans"].clone()
    initialize_camera_pose(m, 1)  # t = 1: the previous pose
    assert torch.equal(m["cam_unnorm_rots"][..., 1], q[..., 0]) and torch.equal(m["cam_trans"][..., 1], t[..., 0])
    initialize_camera_pose(m, 2)  # t > 1: r1 + (r1 - r2), normalised; t1 + (t1 - t2)
    r1, r2 = F.normalize(m["cam_unnorm_rots"][..., 1]), F.normalize(m["cam_unnorm_rots"][..., 0])
    assert torch.equal(m["cam_unnorm_rots"][..., 2], F.normalize(r1 + (r1 - r2)))
    t1, t2 = m["cam_trans"][..., 1], m["cam_trans"][..., 0]
    assert torch.equal(m["cam_trans"][..., 2], t1 + (t1 - t2))
