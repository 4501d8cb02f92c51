"""BASELINE.json configurations at full size, rasterizer vs the CPU oracle (fwd+bwd
through the C ABI):

  * config 1: 10k isotropic Gaussians, 320x240;
  * config 2: 100k isotropic Gaussians, 640x480 (Replica room0 intrinsics);
  * config 3: 300k isotropic Gaussians, 640x480 (the bench workload);
  * config 4: 1M anisotropic Gaussians + SH degree 3, 1200x680 (Replica native
    intrinsics, SURVEY.md 8(d) substitution for ScanNet++);
  * the fork's Habitat orientation (configs/data/habitat.yaml:3-8): 480 wide x 640
    high portrait, fx = fy = 625.22, 300k Gaussians (the tile grid
    is 30x40 instead of 40x30).

Criteria:
  * integer work bit-exact against the float32 oracle (the reference's float32
    arithmetic): num_rendered, every tile range, the sorted Gaussian-id list,
    every radius, and n_contrib at every pixel without an alpha / T decision near
    its threshold;
  * forward RGB within 1e-4 * max(1, |ref|) at every pixel without such a decision
    (and on >= 99.9 % overall), median depth equal except where T = 0.5 is crossed
    near the threshold;
  * gradients against the float64 oracle per tensor and per element
    (harness.check_grad_accuracy), plus relative L2 <= 1e-4 against the float32 oracle.

The oracle runs multi-threaded C (OpenMP; results independent of the thread count)."""
import numpy as np
import pytest

from oracle import harness
from splatam_amd.scenes import config_scene, make_scene

pytestmark = pytest.mark.gpu

# Upper bounds on the oracle's near-threshold sets (fractions; measured on these seeded scenes:
# Gaussians 0.40 / 1.03 / 2.38 / 8.12 / 1.61 % of the visible ones, pixels <= 0.124 %).  A Gaussian is
# excluded from the per-element gradient check when any pixel it contributes to has a decision near its
# threshold (oracle/gsr_oracle.c ALPHA_BAND / T_BAND, forward.cu:311-381): one such pixel excludes every
# Gaussian composited in front of its terminating pair, hence the larger share at config 4 (~80 per pixel).
UNSTABLE_MAX = {1: 0.01, 2: 0.015, 3: 0.03, 4: 0.10, "habitat": 0.02}
UNSTABLE_PIX_MAX = 0.002


def _scene(cfg):
    if cfg == "habitat":
        return make_scene(300_000, 480, 640, seed=0, intrinsics=(625.22, 625.22, 240.5, 320.5))
    return config_scene(cfg)


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, "habitat"])
def test_baseline_config_parity(cuda, cfg):
    scene = _scene(cfg)
    c = scene.cam
    use_sh = scene.shs is not None
    dpix = np.random.RandomState(11).randn(3, c.H, c.W).astype(np.float32)
    gpu = harness.run_gpu(scene, dpix, use_sh=use_sh)
    binning = harness.binning_gpu(scene, use_sh=use_sh)
    fr, ref = harness.run_oracle(scene, dpix, use_sh=use_sh)
    fr64, ref64 = harness.run_oracle(scene, dpix, use_sh=use_sh, dtype=np.float64, error_scale=True)

    # ---- integer work: bit-exact -------------------------------------------------
    assert fr.num_rendered > 0 and int(fr.tiles_touched.sum()) == fr.num_rendered
    assert binning["num_rendered"] == fr.num_rendered
    np.testing.assert_array_equal(gpu["radii"], fr.radii)
    np.testing.assert_array_equal(binning["radii"], fr.radii)
    cnt = fr.ranges[:, 1] - fr.ranges[:, 0]
    np.testing.assert_array_equal(binning["ranges"][:, 1] - binning["ranges"][:, 0], cnt)
    np.testing.assert_array_equal(binning["ranges"][cnt > 0], fr.ranges[cnt > 0])  # empty tiles: any start
    np.testing.assert_array_equal(binning["point_list"], fr.point_list)
    settled = ~fr.unstable_pix
    # pixels with an alpha / T decision near its threshold: reported and bounded (the oracle's count on
    # these seeded scenes is deterministic; the bound guards against a widened exclusion)
    n_upix = int(fr.unstable_pix.astype(bool).sum())
    assert n_upix <= UNSTABLE_PIX_MAX * c.W * c.H, (cfg, n_upix, c.W * c.H)
    nc = binning["n_contrib"].reshape(c.H, c.W)
    assert np.array_equal(nc[settled], fr.n_contrib[settled])

    # ---- forward images -------------------------------------------------------------
    fwd = harness.compare_forward(gpu, fr)
    assert fwd["frac_bad"] <= 1e-3, fwd
    col = np.asarray(gpu["color"], np.float64)
    bad = (np.abs(col - fr.color) > 1e-4 * np.maximum(1.0, np.abs(fr.color))).any(axis=0)
    assert not (bad & settled).any(), int((bad & settled).sum())
    depth_ok = (np.asarray(gpu["depth"])[0] == fr.depth[0]) | fr.unstable_depth_pix | fr.unstable_pix
    assert depth_ok.all(), int((~depth_ok).sum())

    # ---- gradients --------------------------------------------------------------------
    errs = harness.compare_grads(gpu["grads"], ref)
    assert not {k: v for k, v in errs.items() if v > 1e-4}, errs
    stable = ~(fr.unstable | fr64.unstable)
    visible = int((fr.radii > 0).sum())
    n_unstable = int((~stable).sum())
    g, o = harness.check_grad_accuracy(gpu["grads"], ref, ref64, stable)
    print(f"config {cfg}: {n_unstable} of {visible} visible Gaussians excluded from the per-element check "
          f"({n_unstable / max(visible, 1):.3%}), {n_upix} near-threshold pixels; forward {fwd}; "
          f"rel L2 vs f32 {({k: f'{v:.2e}' for k, v in errs.items()})}")
    for k in g:
        print(f"  {k}: gpu {g[k]}  oracle_f32 {o[k]}")
    assert n_unstable <= UNSTABLE_MAX[cfg] * visible, (cfg, n_unstable, visible)
    # the excluded Gaussians are checked too, against the float32 oracle's own error on the same subset:
    # a float32 rasterizer may flip the near-threshold pairs, but no worse than the reference arithmetic
    # (measured r3a: the product's subset errors equal the float32 oracle's to 1-7 %, all configs)
    us = harness.unstable_grad_stats(gpu["grads"], ref, ref64, ~stable)
    for k, d in us.items():
        print(f"  unstable {k}: {d}")
    worse = {k: d for k, d in us.items()
             if d["gpu_rel_l2"] > max(1e-4, 1.5 * d["f32_rel_l2"]) or d["gpu_q99"] > max(1e-3, 1.5 * d["f32_q99"])}
    assert not worse, worse
