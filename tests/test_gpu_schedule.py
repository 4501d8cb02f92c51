"""The render schedule (tile_plan in the bucketed duplicate, gsr_forward.hip): render workgroup i renders tile
order[i].  It must be a permutation of the tiles (every tile rendered once -- the rasterized images of every
parity test depend on it only through that), and it deals the tiles so that the CUs rendering one tile fewer
(slots s with s mod ncu >= ntiles mod ncu) take the longest lists: with lengths bucketed by 4 (the counting
sort's key), no list dealt to those CUs is shorter than a list dealt to the others.  Checked at config 2
(1200 tiles), config 4 (3200 tiles) and the Habitat portrait grid (30 x 40)."""
import numpy as np
import pytest
import torch

from splatam_amd.scenes import config_scene, make_scene

pytestmark = pytest.mark.gpu


def _scene(cfg):
    if cfg == "habitat":
        return make_scene(300_000, 480, 640, seed=0, intrinsics=(625.22, 625.22, 240.5, 320.5))
    return config_scene(cfg)


@pytest.mark.parametrize("cfg", [2, 4, "habitat"])
def test_render_schedule_permutation_and_balance(cuda, cfg):
    from splatam_amd import _C
    from splatam_amd.layout import views
    s = _scene(cfg)
    c = s.cam
    e = torch.Tensor([])
    shs = s.shs.to(cuda) if s.shs is not None else e
    cols = s.colors.to(cuda) if s.shs is None else e
    out = _C.rasterize_gaussians(torch.zeros(3, device=cuda), s.means3D.to(cuda), cols, s.opacities.to(cuda),
                                 s.scales.to(cuda), s.rotations.to(cuda), 1.0, e, c.viewmatrix.to(cuda),
                                 c.projmatrix.to(cuda), c.tanfovx, c.tanfovy, c.H, c.W, shs,
                                 s.sh_degree if s.shs is not None else 0, c.campos.to(cuda), False)
    n, img, binning = out[0], out[5], out[4]
    v = views(img, binning, c.W, c.H, n)
    torch.cuda.synchronize()
    order = v["order"].cpu().numpy().astype(np.int64)
    rng = v["ranges"].cpu().numpy().astype(np.int64)
    T = ((c.W + 15) // 16) * ((c.H + 15) // 16)
    np.testing.assert_array_equal(np.sort(order), np.arange(T))  # every tile exactly once
    ncu = torch.cuda.get_device_properties(cuda).multi_processor_count
    q, m = divmod(T, ncu)
    length = rng[:, 1] - rng[:, 0]
    bucket = np.minimum(length >> 2, 1023)  # the plan's counting-sort key (PLAN_SHIFT, PLAN_BUCKETS)
    slot_cls = np.arange(T) % ncu           # slot s renders on the CU class s mod ncu
    heavy = bucket[order[slot_cls >= m]]    # tiles of the CUs that render q tiles
    light = bucket[order[slot_cls < m]]     # ... and of those that render q + 1
    if length.max() > 4096:  # (a list beyond TILE_SORT_CAP: the radix-sort binning renders in row-major order)
        pytest.skip(f"config {cfg}: longest tile list {length.max()} > 4096")
    if q > 0 and m > 0:
        assert heavy.min() >= light.max(), (cfg, heavy.min(), light.max())
    # per-CU list sums stay close to the mean (the alternating deal inside each group)
    per_cu = np.bincount(slot_cls, weights=length[order], minlength=ncu)
    mean = length.sum() / ncu
    print(f"config {cfg}: {T} tiles on {ncu} CUs (q {q}, m {m}), per-CU list sum max/mean "
          f"{per_cu.max() / mean:.3f}, min/mean {per_cu.min() / mean:.3f}")
    assert per_cu.max() <= 1.25 * mean
