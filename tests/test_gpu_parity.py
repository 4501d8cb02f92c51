"""GPU parity: the HIP rasterizer (through the C ABI, via GaussianRasterizer)
against the CPU oracle on the same seeded inputs.

Tolerances (north star: 1e-4 relative):
  * forward RGB: |d| <= 1e-4 * max(1, |ref|) on >= 99.9 % of pixels; the rest
    are pixels where an alpha / T threshold flips between float32 exp
    implementations;
  * radii (float-derived integers): exact on >= 99.9 % of Gaussians
    (the preprocess is compiled without FMA contraction to match the oracle);
  * median depth: exact on >= 99.5 % of pixels (T ~ 0.5 crossings excepted);
  * gradients: relative L2 <= 1e-4 per tensor against the float32 oracle.
"""
import contextlib
import dataclasses

import numpy as np
import pytest
import torch

from oracle import harness
from splatam_amd.scenes import make_scene

pytestmark = pytest.mark.gpu

CASES = [
    dict(name="iso", P=2000, W=128, H=96, aniso=False, sh=0),
    dict(name="aniso", P=2000, W=128, H=96, aniso=True, sh=0),
    dict(name="ragged", P=1500, W=100, H=75, aniso=True, sh=0),     # image not a multiple of 16
    dict(name="sh1", P=1500, W=96, H=64, aniso=True, sh=1),
    dict(name="sh3", P=1500, W=96, H=64, aniso=True, sh=3),
    dict(name="dense", P=6000, W=64, H=48, aniso=False, sh=0),     # long tile lists, > 1 LDS batch
]


def _check(gpu, fr, ref):
    fwd = harness.compare_forward(gpu, fr)
    assert fwd["frac_bad"] <= 1e-3, fwd
    assert fwd["radii_match"] >= 0.999, fwd
    assert fwd["depth_match"] >= 0.995, fwd
    errs = harness.compare_grads(gpu["grads"], ref)
    bad = {k: v for k, v in errs.items() if v > 1e-4}
    assert not bad, errs
    return fwd, errs


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_forward_backward_parity(cuda, case):
    scene = make_scene(case["P"], case["W"], case["H"], seed=7, anisotropic=case["aniso"], sh_degree=case["sh"])
    dpix = np.random.RandomState(1).randn(3, case["H"], case["W"]).astype(np.float32)
    use_sh = case["sh"] > 0
    gpu = harness.run_gpu(scene, dpix, use_sh=use_sh)
    fr, ref = harness.run_oracle(scene, dpix, use_sh=use_sh)
    _check(gpu, fr, ref)


def test_background_and_cov_precomp(cuda):
    scene = make_scene(1500, 80, 64, seed=11, anisotropic=True)
    dpix = np.random.RandomState(2).randn(3, 64, 80).astype(np.float32)
    bg = (0.2, 0.5, 0.9)
    gpu = harness.run_gpu(scene, dpix, bg=bg, use_cov=True)
    fr, ref = harness.run_oracle(scene, dpix, bg=bg, use_cov=True)
    _check(gpu, fr, ref)


def test_reduce9_lane_mapping(cuda):
    from splatam_amd._C import lib
    x = torch.randn(64, 9, device=cuda, dtype=torch.float32)
    out = torch.zeros(9, device=cuda)
    rc = lib.gsr_selftest_reduce9(x.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), x.sum(0).cpu(), rtol=1e-5, atol=1e-5)


def test_empty_and_culled(cuda):
    from splatam_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer
    scene = make_scene(64, 32, 32, seed=1)
    c = scene.cam
    st = GaussianRasterizationSettings(32, 32, c.tanfovx, c.tanfovy, torch.tensor([0.1, 0.2, 0.3], device=cuda), 1.0,
                                       c.viewmatrix.to(cuda), c.projmatrix.to(cuda), 0, c.campos.to(cuda), False)
    ras = GaussianRasterizer(st)
    # P == 0: reference returns zeros (rasterize_points.cu:67-81)
    z = torch.zeros(0, 3, device=cuda)
    color, radii, depth = ras(means3D=z, means2D=z, opacities=torch.zeros(0, 1, device=cuda),
                              colors_precomp=z, scales=z, rotations=torch.zeros(0, 4, device=cuda))
    assert color.shape == (3, 32, 32) and float(color.abs().sum()) == 0.0 and radii.numel() == 0
    # every Gaussian behind the camera: background everywhere, depth 15, zero grads
    m = scene.means3D.clone().to(cuda)
    m[:, 2] = -1.0
    m.requires_grad_(True)
    m2 = torch.zeros_like(m, requires_grad=True)
    color, radii, depth = ras(means3D=m, means2D=m2, opacities=scene.opacities.to(cuda),
                              colors_precomp=scene.colors.to(cuda), scales=scene.scales.to(cuda),
                              rotations=scene.rotations.to(cuda))
    assert int(radii.abs().sum()) == 0
    torch.testing.assert_close(color[:, 0, 0].cpu(), torch.tensor([0.1, 0.2, 0.3]))
    assert float(depth.min()) == 15.0
    color.sum().backward()
    assert float(m.grad.abs().sum()) == 0.0


def test_bitwise_deterministic_backward(cuda):
    scene = make_scene(3000, 128, 96, seed=5, anisotropic=True)
    dpix = np.random.RandomState(3).randn(3, 96, 128).astype(np.float32)
    a = harness.run_gpu(scene, dpix)
    b = harness.run_gpu(scene, dpix)
    for k in a["grads"]:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


def _binning_gpu(scene, cuda, mode=2):
    """The dynamic forward's binning; mode 2: the reference's lists (gsr_settings.binning = REFERENCE), 3: the
    tile-culled lists (the default)."""
    from splatam_amd import _C
    from splatam_amd.layout import views
    c = scene.cam
    with (_C.reference_binning() if mode == 2 else contextlib.nullcontext()):
        out = _C.rasterize_gaussians(torch.zeros(3, device=cuda), scene.means3D.to(cuda), scene.colors.to(cuda),
                                     scene.opacities.to(cuda), scene.scales.to(cuda), scene.rotations.to(cuda), 1.0,
                                     torch.Tensor([]), c.viewmatrix.to(cuda), c.projmatrix.to(cuda), c.tanfovx,
                                     c.tanfovy, c.H, c.W, torch.Tensor([]), 0, c.campos.to(cuda), False)
    n, color, radii, geom, binning, img, depth = out
    v = views(img, binning, c.W, c.H, n)
    res = {k: t.cpu().numpy() for k, t in v.items()}
    res["radii"] = radii.cpu().numpy()
    res["color"], res["depth"] = color.cpu().numpy(), depth.cpu().numpy()
    return n, res


BIN_CASES = [
    dict(name="cfg1_like", P=4000, W=160, H=120, aniso=False),
    dict(name="aniso", P=3000, W=128, H=96, aniso=True),
    dict(name="long_lists", P=12000, W=48, H=32, aniso=False, near=True, scale=12.0),  # > TILE_SORT_CAP -> radix
    # lists of 1025-2048 / 2049-3072 / 3073-4096 keys: 2, 3 and 4 sorted chunks merged by rank in render_fwd
    dict(name="chunked_lists", P=6000, W=96, H=64, aniso=False, near=True, scale=7.0),
    dict(name="many_tiles", P=6000, W=2080, H=2080, aniso=True),  # > MAX_LDS_TILES -> global-atomic counts
]


@pytest.mark.parametrize("case", BIN_CASES, ids=[c["name"] for c in BIN_CASES])
def test_binning_bit_exact(cuda, case):
    """Integer work is bit-exact: num_rendered, per-tile ranges and the sorted
    Gaussian-id list equal the oracle's (tile, depth, id) order."""
    scene = make_scene(case["P"], case["W"], case["H"], seed=13, anisotropic=case["aniso"],
                       z_range=(0.5, 1.0) if case.get("near") else (0.5, 5.0))
    scene.scales *= case.get("scale", 1.0)
    fr, _ = harness.run_oracle(scene, backward=False)
    n, v = _binning_gpu(scene, cuda)
    assert n == fr.num_rendered
    cnt_gpu = v["ranges"][:, 1] - v["ranges"][:, 0]
    cnt_ref = fr.ranges[:, 1] - fr.ranges[:, 0]
    np.testing.assert_array_equal(cnt_gpu, cnt_ref)
    nz = cnt_ref > 0
    np.testing.assert_array_equal(v["ranges"][nz, 0], fr.ranges[nz, 0])
    np.testing.assert_array_equal(v["point_list"], fr.point_list)
    if case["name"] == "long_lists":
        assert cnt_ref.max() > 4096
    if case["name"] == "chunked_lists":
        assert cnt_ref.max() <= 4096
        for lo, hi in ((1024, 2048), (2048, 3072), (3072, 4096)):
            assert ((cnt_ref > lo) & (cnt_ref <= hi)).any(), (lo, hi)


@pytest.mark.parametrize("case", BIN_CASES, ids=[c["name"] for c in BIN_CASES])
def test_tile_cull_drops_only_unreached_instances(cuda, case):
    """Tile culling in the dynamic drop-in forward (the default gsr_settings.binning, every binning path: bucketed,
    chunked, radix fallback with the culled instances keyed behind every tile, global-atomic counts): every
    tile list is an order-preserving subsequence of the reference's list (mode 2), an instance is dropped only
    where no pixel of its tile reaches alpha >= 1/255 (float64, margin), num_rendered, radii, images and every
    gradient are bitwise those of the reference's lists."""
    from splatam_amd import _C
    scene = make_scene(case["P"], case["W"], case["H"], seed=13, anisotropic=case["aniso"],
                       z_range=(0.5, 1.0) if case.get("near") else (0.5, 5.0))
    scene.scales *= case.get("scale", 1.0)
    c = scene.cam
    fr, _ = harness.run_oracle(scene, backward=False)
    n2, v2 = _binning_gpu(scene, cuda, mode=2)
    n3, v3 = _binning_gpu(scene, cuda, mode=3)
    assert n2 == n3 == fr.num_rendered
    for k in ("radii", "color", "depth"):
        assert np.array_equal(v2[k], v3[k]), k
    gx = (c.W + 15) // 16
    m2, co = fr.means2D.astype(np.float64), fr.conic_opacity.astype(np.float64)
    ly, lx = np.meshgrid(np.arange(16), np.arange(16), indexing="ij")
    dropped = 0
    for t in range(len(v2["ranges"])):
        a2, b2 = (int(x) for x in v2["ranges"][t])
        a3, b3 = (int(x) for x in v3["ranges"][t])
        full = v2["point_list"][a2:b2].astype(np.int64) if b2 > a2 else np.zeros(0, np.int64)
        kept = v3["point_list"][a3:b3].astype(np.int64) if b3 > a3 else np.zeros(0, np.int64)
        sel = np.isin(full, kept)
        np.testing.assert_array_equal(full[sel], kept)  # an order-preserving subsequence
        gone = full[~sel].astype(np.int64)
        dropped += len(gone)
        if len(gone):
            X, Y = (t % gx) * 16 + lx.ravel(), (t // gx) * 16 + ly.ravel()
            inside = (X < c.W) & (Y < c.H)
            dx, dy = m2[gone, 0][:, None] - X[None], m2[gone, 1][:, None] - Y[None]
            A, B, C, o = (co[gone, k][:, None] for k in range(4))
            power = -0.5 * (A * dx * dx + C * dy * dy) - B * dx * dy
            alpha = o * np.exp(np.minimum(power, 0.0))
            assert not ((power <= 0) & (alpha >= 0.99 / 255.0) & inside[None]).any(), t
    print(f"{case['name']}: {dropped} of {n2} instances culled")
    if case["name"] not in ("many_tiles", "long_lists"):  # (long_lists: every Gaussian reaches all six tiles)
        assert dropped > 0
    dpix = np.random.RandomState(3).randn(3, c.H, c.W).astype(np.float32)
    with _C.reference_binning():
        a = harness.run_gpu(scene, dpix)
    b = harness.run_gpu(scene, dpix)
    for k in a["grads"]:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


@pytest.mark.parametrize("case", BIN_CASES, ids=[c["name"] for c in BIN_CASES])
def test_point_list_holds_num_rendered_valid_ids(cuda, case):
    """The binning buffer's contract (rasterizer_impl.cu:290-315 walks num_rendered entries): with culling on
    (the default) and off, every one of the num_rendered point-list entries is a Gaussian id in [0, P), and
    their multiset is the reference's (Gaussian i listed tiles_touched(i) times).  Culled instances sit in
    the tail [L, num_rendered) (L = the ranges' total) with an empty block mask.  The r7s abort came from
    reading that tail before the library wrote it."""
    scene = make_scene(case["P"], case["W"], case["H"], seed=13, anisotropic=case["aniso"],
                       z_range=(0.5, 1.0) if case.get("near") else (0.5, 5.0))
    scene.scales *= case.get("scale", 1.0)
    fr, _ = harness.run_oracle(scene, backward=False)
    want = np.bincount(fr.point_list.astype(np.int64), minlength=scene.P)
    for mode in (2, 3):
        n, v = _binning_gpu(scene, cuda, mode=mode)
        assert n == fr.num_rendered
        ids = v["point_list"][:n].astype(np.int64)
        assert ids.min() >= 0 and ids.max() < scene.P, mode
        np.testing.assert_array_equal(np.bincount(ids, minlength=scene.P), want)
        L = int((v["ranges"][:, 1] - v["ranges"][:, 0]).clip(min=0).sum())
        assert L <= n
        if mode == 2:
            assert L == n
        assert not (v["block_masks"][L:n] & 0xFFFF).any(), mode
        print(f"{case['name']} mode {mode}: {n - L} of {n} entries in the culled tail")


def test_point_list_valid_in_static_mode(cuda):
    """The static (capacity) forward: the first status[0] = num_rendered entries are valid ids, culled or not:
    the tile lists, then (culled) padding entries -- the owners of the last rect instance slots -- with empty
    block masks (include/gsr.h: the exact culled instances are written by the dynamic forward only)."""
    from splatam_amd import _C
    from splatam_amd.layout import views
    scene = make_scene(20000, 320, 240, seed=3)
    c = scene.cam
    dev = torch.device(cuda)
    e = torch.Tensor([])
    for mode in (2, 3):
        status = torch.zeros(4, dtype=torch.int32, device=dev)
        with (_C.reference_binning() if mode == 2 else contextlib.nullcontext()):
            out = _C.rasterize_gaussians(torch.zeros(3, device=dev), scene.means3D.to(dev), scene.colors.to(dev),
                                         scene.opacities.to(dev), scene.scales.to(dev), scene.rotations.to(dev), 1.0,
                                         e, c.viewmatrix.to(dev), c.projmatrix.to(dev), c.tanfovx, c.tanfovy, c.H, c.W,
                                         e, 0, c.campos.to(dev), False, capacity=200000, status=status)
        torch.cuda.synchronize()
        n = int(status[0])
        assert 0 < n <= 200000
        v = views(out[5], out[4], c.W, c.H, n)
        ids = v["point_list"][:n].long()
        assert int(ids.min()) >= 0 and int(ids.max()) < scene.P
        rng = v["ranges"].long()
        L = int((rng[:, 1] - rng[:, 0]).clamp(min=0).sum())
        assert (L == n) if mode == 2 else (L < n)
        assert not bool((v["block_masks"][L:n] & 0xFFFF).any())
        assert bool((out[2][ids] > 0).all())  # every listed or padding id has a rect (radius > 0)


def test_binning_mode_is_per_call_across_threads(cuda):
    """gsr_settings.binning is a per-call argument (no process-wide mode): two threads, each with its own
    stream, one forwarding with the reference's lists and one with culled lists, interleaved, each get their
    own lists -- bitwise those of a single-threaded call."""
    import threading
    scene = make_scene(8000, 160, 120, seed=19)
    ref = {m: _binning_gpu(scene, cuda, mode=m) for m in (2, 3)}
    assert ref[2][0] == ref[3][0]
    assert not np.array_equal(ref[2][1]["ranges"], ref[3][1]["ranges"])  # the modes differ on this scene
    errors = []

    def worker(mode):
        try:
            s = torch.cuda.Stream(device=cuda)
            with torch.cuda.stream(s):
                for _ in range(12):
                    n, v = _binning_gpu(scene, cuda, mode=mode)
                    for k in ("ranges", "point_list"):
                        if not np.array_equal(v[k], ref[mode][1][k]):
                            errors.append((mode, k))
        except Exception as exc:  # pragma: no cover - reported below
            errors.append((mode, repr(exc)))

    ts = [threading.Thread(target=worker, args=(m,)) for m in (2, 3, 2, 3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:4]


POWER_CASES = [
    dict(name="p2_iso", P=2000, W=128, H=96, aniso=False, sh=0, power=2),     # SplaTAM's Fisher scoring
    dict(name="p2_aniso_sh1", P=1500, W=96, H=64, aniso=True, sh=1, power=2),
    dict(name="p2_sh3", P=1200, W=96, H=64, aniso=True, sh=3, power=2),
    dict(name="p3_ragged", P=1500, W=100, H=75, aniso=True, sh=0, power=3),
    dict(name="p2_dense", P=6000, W=64, H=48, aniso=False, sh=0, power=2),   # > 1 LDS batch per tile
]


@pytest.mark.parametrize("case", POWER_CASES, ids=[c["name"] for c in POWER_CASES])
def test_backward_power_parity(cuda, case):
    """backward_power != 1: per-pair powf before summation (renderCUDAFused,
    backward.cu:850-1140) against the oracle's FUSED mode; same 1e-4 relative L2."""
    scene = make_scene(case["P"], case["W"], case["H"], seed=17, anisotropic=case["aniso"], sh_degree=case["sh"])
    dpix = np.random.RandomState(4).randn(3, case["H"], case["W"]).astype(np.float32)
    use_sh = case["sh"] > 0
    gpu = harness.run_gpu(scene, dpix, use_sh=use_sh, power=case["power"])
    fr, ref = harness.run_oracle(scene, dpix, use_sh=use_sh, power=case["power"])
    _check(gpu, fr, ref)


def test_backward_power_bg_cov_deterministic(cuda):
    scene = make_scene(1500, 80, 64, seed=19, anisotropic=True)
    dpix = np.random.RandomState(5).randn(3, 64, 80).astype(np.float32)
    bg = (0.3, 0.1, 0.7)
    a = harness.run_gpu(scene, dpix, bg=bg, use_cov=True, power=2)
    b = harness.run_gpu(scene, dpix, bg=bg, use_cov=True, power=2)
    fr, ref = harness.run_oracle(scene, dpix, bg=bg, use_cov=True, power=2)
    _check(a, fr, ref)
    for k in a["grads"]:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


@pytest.mark.parametrize("aniso", [False, True], ids=["iso", "aniso"])
def test_dual_render_matches_two_calls_and_oracle(cuda, aniso):
    """gsr_forward_dual / gsr_backward_dual: each image is
    bitwise the single-call image; colour gradients equal the single calls';
    geometric gradients equal the sum of the two oracle backward passes (1e-4)."""
    from splatam_amd.rasterizer import rasterize_gaussians_dual
    scene = make_scene(3000, 128, 96, seed=23, anisotropic=aniso)
    H, W = 96, 128
    rs = np.random.RandomState(6)
    dpix, dpix2 = rs.randn(3, H, W).astype(np.float32), rs.randn(3, H, W).astype(np.float32)
    z = scene.means3D[:, 2:3]
    colors2 = torch.cat([z, torch.ones_like(z), z * z], 1)  # SplaTAM's [z, 1, z^2]
    a = harness.run_gpu(scene, dpix)
    scene2 = dataclasses.replace(scene, colors=colors2)
    b = harness.run_gpu(scene2, dpix2)
    c = scene.cam
    from splatam_amd.rasterizer import GaussianRasterizationSettings
    st = GaussianRasterizationSettings(H, W, c.tanfovx, c.tanfovy, torch.zeros(3, device=cuda), 1.0,
                                       c.viewmatrix.to(cuda), c.projmatrix.to(cuda), 0, c.campos.to(cuda), False)
    leaf = lambda t: t.detach().to(cuda).clone().requires_grad_(True)  # noqa: E731
    m3, op, col, col2, sc, ro = (leaf(scene.means3D), leaf(scene.opacities), leaf(scene.colors), leaf(colors2),
                                 leaf(scene.scales), leaf(scene.rotations))
    m2 = torch.zeros_like(m3, requires_grad=True)
    im, im2, radii, depth = rasterize_gaussians_dual(m3, m2, None, col, col2, op, sc, ro, None, st,
                                                     means2D_grad_sum=True)
    assert np.array_equal(im.detach().cpu().numpy(), a["color"])
    assert np.array_equal(im2.detach().cpu().numpy(), b["color"])
    assert np.array_equal(radii.cpu().numpy(), a["radii"])
    assert np.array_equal(depth.cpu().numpy(), a["depth"])
    (im * torch.as_tensor(dpix, device=cuda)).sum().backward(retain_graph=True)
    (im2 * torch.as_tensor(dpix2, device=cuda)).sum().backward()
    np.testing.assert_array_equal(col.grad.cpu().numpy(), a["grads"]["dcolors"])
    np.testing.assert_array_equal(col2.grad.cpu().numpy(), b["grads"]["dcolors"])
    # geometric gradients: sum of the two single-render oracle passes
    _, ra = harness.run_oracle(scene, dpix)
    _, rb = harness.run_oracle(scene2, dpix2)
    got = {"dmeans3D": m3.grad, "dmeans2D": m2.grad, "dopacity": op.grad, "dscales": sc.grad, "drot": ro.grad}
    for k, v in got.items():
        ref = ra[k].reshape(v.shape) + rb[k].reshape(v.shape)
        assert harness.rel_l2(v.detach().cpu().numpy(), ref) <= 1e-4, k
    # by default the dual render gives means2D no gradient: the reference's densification statistics
    # read the RGB render's own means2D gradient (scripts/splatam.py:256), which the sum is not
    m2b = torch.zeros_like(m3, requires_grad=True)
    im, im2, _, _ = rasterize_gaussians_dual(m3, m2b, None, col, col2, op, sc, ro, None, st)
    ((im * torch.as_tensor(dpix, device=cuda)).sum() + (im2 * torch.as_tensor(dpix2, device=cuda)).sum()).backward()
    assert m2b.grad is None


def test_fused_mapping_refuses_densification(cuda):
    """Gaussian-splatting densification needs the RGB render's own means2D gradient: the fused
    (one-rasterization) mapping path declines it and the literal two-call path runs."""
    from splatam_amd import slam
    scene = make_scene(500, 64, 48, seed=3)
    params = slam.init_mapping_params(scene, num_frames=1, device=cuda)
    cam = slam.camera_settings(scene.cam, cuda)
    curr = {"cam": cam, "w2c": torch.eye(4, device=cuda), "im": torch.rand(3, 48, 64, device=cuda),
            "depth": torch.rand(1, 48, 64, device=cuda)}
    assert slam.fused_mapping_eligible(params, curr, slam.MappingConfig())
    assert not slam.fused_mapping_eligible(params, curr, slam.MappingConfig(use_gaussian_splatting_densification=True))


def test_dual_render_skips_unneeded_gradients(cuda):
    """Only means3D and colors2 require grad (SplaTAM tracking): the lean
    backward variant gives bitwise the full variant's gradients for them."""
    from splatam_amd.rasterizer import GaussianRasterizationSettings, rasterize_gaussians_dual
    scene = make_scene(3000, 128, 96, seed=29, anisotropic=True)
    c = scene.cam
    st = GaussianRasterizationSettings(96, 128, c.tanfovx, c.tanfovy, torch.zeros(3, device=cuda), 1.0,
                                       c.viewmatrix.to(cuda), c.projmatrix.to(cuda), 0, c.campos.to(cuda), False)
    rs = np.random.RandomState(8)
    g1 = torch.as_tensor(rs.randn(3, 96, 128).astype(np.float32), device=cuda)
    g2 = torch.as_tensor(rs.randn(3, 96, 128).astype(np.float32), device=cuda)
    z = scene.means3D[:, 2:3]
    c2 = torch.cat([z, torch.ones_like(z), z * z], 1)
    res = []
    for lean in (False, True):
        t = lambda x, rg: x.detach().to(cuda).clone().requires_grad_(rg)  # noqa: E731
        m3, col2 = t(scene.means3D, True), t(c2, True)
        op, col, sc, ro = (t(scene.opacities, not lean), t(scene.colors, not lean), t(scene.scales, not lean),
                           t(scene.rotations, not lean))
        m2 = torch.zeros_like(m3, requires_grad=not lean)
        im, im2, _, _ = rasterize_gaussians_dual(m3, m2, None, col, col2, op, sc, ro, None, st)
        ((im * g1).sum() + (im2 * g2).sum()).backward()
        res.append((m3.grad.cpu(), col2.grad.cpu(), op.grad))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert res[1][2] is None


def test_single_render_skips_unneeded_gradients(cuda):
    """GaussianRasterizer forms only the gradients autograd asks for (ctx.needs_input_grad):
    with only means3D / colors requiring grad, their gradients are bitwise those of the
    all-inputs call and the other inputs receive None."""
    from splatam_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer
    scene = make_scene(3000, 128, 96, seed=31, anisotropic=True)
    c = scene.cam
    st = GaussianRasterizationSettings(96, 128, c.tanfovx, c.tanfovy, torch.zeros(3, device=cuda), 1.0,
                                       c.viewmatrix.to(cuda), c.projmatrix.to(cuda), 0, c.campos.to(cuda), False)
    g1 = torch.as_tensor(np.random.RandomState(9).randn(3, 96, 128).astype(np.float32), device=cuda)
    res = []
    for lean in (False, True):
        t = lambda x, rg: x.detach().to(cuda).clone().requires_grad_(rg)  # noqa: E731
        m3, col = t(scene.means3D, True), t(scene.colors, True)
        op, sc, ro = t(scene.opacities, not lean), t(scene.scales, not lean), t(scene.rotations, not lean)
        m2 = torch.zeros_like(m3, requires_grad=not lean)
        im, _, _ = GaussianRasterizer(st)(means3D=m3, means2D=m2, opacities=op, colors_precomp=col, scales=sc,
                                          rotations=ro)
        (im * g1).sum().backward()
        res.append((m3.grad.cpu(), col.grad.cpu(), op.grad, sc.grad, ro.grad, m2.grad))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert all(g is not None for g in res[0][2:]) and all(g is None for g in res[1][2:])


def test_dual_render_depth_channel_only_gradient(cuda):
    """grad2_channels=1 (SplaTAM tracking: the loss reads only the depth channel
    of the depth/silhouette render) matches the 3-channel backward when the
    incoming gradient of channels 1, 2 is zero; dcolors2[:, 1:] is exactly 0."""
    from splatam_amd.rasterizer import GaussianRasterizationSettings, rasterize_gaussians_dual
    scene = make_scene(3000, 128, 96, seed=31, anisotropic=False)
    c = scene.cam
    st = GaussianRasterizationSettings(96, 128, c.tanfovx, c.tanfovy, torch.zeros(3, device=cuda), 1.0,
                                       c.viewmatrix.to(cuda), c.projmatrix.to(cuda), 0, c.campos.to(cuda), False)
    rs = np.random.RandomState(9)
    g1 = torch.as_tensor(rs.randn(3, 96, 128).astype(np.float32), device=cuda)
    g2 = torch.zeros(3, 96, 128, device=cuda)
    g2[0] = torch.as_tensor(rs.randn(96, 128).astype(np.float32), device=cuda)
    z = scene.means3D[:, 2:3]
    c2 = torch.cat([z, torch.ones_like(z), z * z], 1)
    res = []
    for ch in (3, 1):
        t = lambda x, rg: x.detach().to(cuda).clone().requires_grad_(rg)  # noqa: E731
        m3, col2 = t(scene.means3D, True), t(c2, True)
        op, col, sc, ro = (t(scene.opacities, False), t(scene.colors, False), t(scene.scales, False),
                           t(scene.rotations, False))
        m2 = torch.zeros_like(m3)
        im, im2, _, _ = rasterize_gaussians_dual(m3, m2, None, col, col2, op, sc, ro, None, st, grad2_channels=ch)
        ((im * g1).sum() + (im2 * g2).sum()).backward()
        res.append((m3.grad.cpu().numpy(), col2.grad.cpu().numpy()))
    (m3_full, c2_full), (m3_lean, c2_lean) = res
    # tolerance: the lean variant drops two exact-zero FMAs from the per-pair colour
    # dot product, which reorders one rounding step (fp32, relative L2 1e-5)
    assert harness.rel_l2(m3_lean, m3_full) <= 1e-5
    assert harness.rel_l2(c2_lean[:, 0], c2_full[:, 0]) <= 1e-5
    assert np.all(c2_lean[:, 1:] == 0)
    assert np.abs(c2_full[:, 0]).sum() > 0


@pytest.mark.parametrize("aniso", [False, True])
def test_block_masks_are_conservative(cuda, aniso):
    """The exact ellipse-vs-block masks carried by the sorted tile lists (block_mask_exact)
    never drop a 4x4 block in which the Gaussian reaches alpha >= 1/255 at some pixel
    (evaluated per pixel in float32 with the render kernels' formula), and cull blocks the
    bounding box keeps."""
    from splatam_amd import _C
    from splatam_amd.layout import views
    scene = make_scene(4000, 160, 112, seed=41, anisotropic=aniso)
    c = scene.cam
    dev = torch.device(cuda)
    e = torch.Tensor([])
    out = _C.rasterize_gaussians(torch.zeros(3, device=dev), scene.means3D.to(dev), scene.colors.to(dev),
                                 scene.opacities.to(dev), scene.scales.to(dev), scene.rotations.to(dev), 1.0, e,
                                 c.viewmatrix.to(dev), c.projmatrix.to(dev), c.tanfovx, c.tanfovy, c.H, c.W, e, 0,
                                 c.campos.to(dev), False)
    n, geom, binning, img = out[0], out[3], out[4], out[5]
    v = views(img, binning, c.W, c.H, n)
    P = scene.P
    rr = geom[:64 * P].view(torch.float32).reshape(P, 16)
    k_ac, k_b = -0.5 * 1.4426950408889634, -1.4426950408889634
    x, y, A, C, B, o = rr[:, 0], rr[:, 1], rr[:, 2] / k_ac, rr[:, 3] / k_ac, rr[:, 4] / k_b, rr[:, 5]
    rng = v["ranges"].long()
    gx = (c.W + 15) // 16
    tile_of = torch.repeat_interleave(torch.arange(rng.shape[0], device=dev), (rng[:, 1] - rng[:, 0]).clamp(min=0))
    # the listed entries: the ranges' total (num_rendered counts record slots, culled instances included)
    nl = int((rng[:, 1] - rng[:, 0]).clamp(min=0).sum())
    assert nl <= n
    gid = v["point_list"].long()[:nl]
    mask = v["block_masks"].long()[:nl] & 0xFFFF
    ty, tx = tile_of // gx, tile_of % gx
    ly, lx = torch.meshgrid(torch.arange(16, device=dev), torch.arange(16, device=dev), indexing="ij")
    px = (tx * 16)[:, None, None] + lx[None]
    py = (ty * 16)[:, None, None] + ly[None]
    dx, dy = x[gid][:, None, None] - px, y[gid][:, None, None] - py
    pw = -0.5 * (A[gid][:, None, None] * dx * dx + C[gid][:, None, None] * dy * dy) - B[gid][:, None, None] * dx * dy
    al = torch.clamp(o[gid][:, None, None] * torch.exp(pw), max=0.99)
    ok = (pw <= 0) & (al >= 1.0 / 255.0 * 0.999) & (px < c.W) & (py < c.H)
    # block (cx, cy) of the tile -> mask bit 4 (2 (cy >> 1) + (cx >> 1)) + 2 (cy & 1) + (cx & 1)
    blk = ok.reshape(-1, 4, 4, 4, 4).any(4).any(2)  # [inst, cy, cx]
    bits = torch.zeros(nl, dtype=torch.long, device=dev)
    for cy in range(4):
        for cx in range(4):
            bit = 4 * (2 * (cy >> 1) + (cx >> 1)) + 2 * (cy & 1) + (cx & 1)
            bits |= blk[:, cy, cx].long() << bit
    # the mask reaches the sorted entry when render_fwd stages it: every entry up to the tile's last
    # contributor (the entries render_bwd stages)
    nc = v["n_contrib"].reshape(c.H, c.W).long()
    nc = torch.nn.functional.pad(nc, (0, gx * 16 - c.W, 0, ((c.H + 15) // 16) * 16 - c.H))
    tile_last = nc.reshape((c.H + 15) // 16, 16, gx, 16).amax(dim=(1, 3)).reshape(-1)
    pos = torch.arange(nl, device=dev) - rng[tile_of, 0]
    staged = pos < tile_last[tile_of]
    missed = ((bits & ~mask) != 0) & staged
    assert int(staged.sum()) > 0
    assert int(missed.sum()) == 0, int(missed.sum())
    kept = torch.stack([(mask[staged] >> b) & 1 for b in range(16)], 1).sum()
    assert int(kept) < 16 * int(staged.sum())  # it does cull


def test_mark_visible_matches_oracle(cuda):
    """GaussianRasterizer.markVisible (__init__.py:159-168 -> rasterize_points.cu:198-216 ->
    checkFrustum, rasterizer_impl.cu:54-67): view_z > 0.001, against the oracle, including points
    behind, on and just in front of the near limit and a non-identity view."""
    from oracle import oracle
    from splatam_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer
    from splatam_amd.scenes import setup_camera
    g = torch.Generator().manual_seed(21)
    P = 5000
    pts = torch.randn(P, 3, generator=g) * 2.0
    pts[:16, 2] = torch.tensor([0.001, 0.0010001, 0.0009999, -0.001, 0.0, 1e-7, -1e-7, 0.002] * 2)
    w2c = torch.eye(4)
    w2c[:3, 3] = torch.tensor([0.1, -0.2, 0.3])
    cam = setup_camera(64, 48, 50.0, 50.0, 31.5, 23.5, w2c=w2c)
    st = GaussianRasterizationSettings(image_height=48, image_width=64, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
                                       bg=torch.zeros(3, device=cuda), scale_modifier=1.0,
                                       viewmatrix=cam.viewmatrix.to(cuda), projmatrix=cam.projmatrix.to(cuda),
                                       sh_degree=0, campos=cam.campos.to(cuda), prefiltered=False)
    vis = GaussianRasterizer(st).markVisible(pts.to(cuda))
    assert vis.dtype == torch.bool and vis.shape == (P,)
    ref = oracle.mark_visible(pts.numpy(), cam.viewmatrix.numpy())
    np.testing.assert_array_equal(vis.cpu().numpy(), ref)
    assert 0 < int(vis.sum()) < P


def _geom_pair(cuda, seed, perturb_second=False, cache=True):
    """SplaTAM's two Renderer calls (scripts/splatam.py:255,259): same means3D tensor and camera,
    rotations / opacities / scales recomputed (new tensors, equal values), different colours."""
    from splatam_amd import _C
    from splatam_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer
    scene = make_scene(4000, 160, 120, seed=seed, anisotropic=True)
    c = scene.cam
    st = GaussianRasterizationSettings(120, 160, c.tanfovx, c.tanfovy, torch.zeros(3, device=cuda), 1.0,
                                       c.viewmatrix.to(cuda), c.projmatrix.to(cuda), 0, c.campos.to(cuda), False)
    rs = np.random.RandomState(seed)
    g1 = torch.as_tensor(rs.randn(3, 120, 160).astype(np.float32), device=cuda)
    g2 = torch.as_tensor(rs.randn(3, 120, 160).astype(np.float32), device=cuda)
    old = _C._GEOM_CACHE
    if cache is not None:  # (None: leave the current setting -- callers on several threads)
        _C.set_geom_cache(cache)
    try:
        m3 = scene.means3D.to(cuda).requires_grad_(True)
        u_rot = scene.rotations.to(cuda).requires_grad_(True)
        lo = torch.logit(scene.opacities.to(cuda).clamp(1e-4, 1 - 1e-4)).requires_grad_(True)
        ls = torch.log(scene.scales.to(cuda)).requires_grad_(True)
        col = scene.colors.to(cuda).requires_grad_(True)
        outs = []
        rendervars = []  # held like get_loss holds its two rendervar dicts (slam_helpers.py:124-139,234-249)
        for k in range(2):
            z = m3[:, 2:3]
            rendervars.append(dict(
                means3D=m3, means2D=torch.zeros_like(m3, requires_grad=True), opacities=torch.sigmoid(lo),
                colors_precomp=col if k == 0 else torch.cat([z, torch.ones_like(z), z * z], 1),
                scales=torch.exp(ls) * (1.001 if (perturb_second and k == 1) else 1.0),
                rotations=torch.nn.functional.normalize(u_rot)))
        for k in range(2):
            outs.append(GaussianRasterizer(st)(**rendervars[k]))
        ((outs[0][0] * g1).sum() + (outs[1][0] * g2).sum()).backward()
        res = [o[0].detach().cpu() for o in outs] + [o[1].cpu() for o in outs] + [o[2].detach().cpu() for o in outs]
        res += [t.grad.cpu() for t in (m3, u_rot, lo, ls, col)]
        return res
    finally:
        if cache is not None:
            _C.set_geom_cache(old)


@pytest.mark.parametrize("native", [True, False])
def test_geometry_reuse_matches_two_full_calls(cuda, native):
    """The second of two calls on identical geometry reuses the first call's preprocess / binning
    (gsr_forward_reuse_if_equal, comparison and gating on the device): images, radii, depth and every
    gradient bitwise those of two full calls -- through the native binding and the ctypes one."""
    from splatam_amd import _C
    with _binding(native):
        hits = _C.reuse_stats()["hits"]
        a = _geom_pair(cuda, 41, cache=True)
        assert _C.reuse_stats()["hits"] == hits + 1, _C.reuse_stats()  # the second call took the reuse form
        b = _geom_pair(cuda, 41, cache=False)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("native", [True, False])
def test_geometry_reuse_refused_on_changed_geometry(cuda, native):
    """Scales differing in the second call (bitwise comparison on the device) -> the full forward ran."""
    from splatam_amd import _C
    with _binding(native):
        st = _C.reuse_stats()
        hits, content = st["hits"], st.get("content", 0)
        a = _geom_pair(cuda, 43, perturb_second=True, cache=True)
        st = _C.reuse_stats()
        assert st["hits"] == hits and st["content"] == content + 1, st
        b = _geom_pair(cuda, 43, perturb_second=True, cache=False)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_geometry_reuse_concurrent_threads(cuda):
    """Two threads, each on its own stream, running RGB / depth pairs with the reuse on: every image, radius
    and gradient bitwise that of the same pair with the reuse off (the gate word lives in each call's own
    geometry buffer, the previous-call state is per thread)."""
    import threading
    from splatam_amd import _C
    seeds = [(61, 62), (63, 64)]
    ref = {sd: _geom_pair(cuda, sd, cache=False) for pair in seeds for sd in pair}
    old = _C._GEOM_CACHE
    _C.set_geom_cache(True)
    hits = _C.reuse_stats()["hits"]
    out, errs = {}, []

    def worker(pair):
        try:
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                for sd in pair:
                    out[sd] = _geom_pair(cuda, sd, cache=None)
            st.synchronize()
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(e)

    try:
        th = [threading.Thread(target=worker, args=(pair,)) for pair in seeds]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
    finally:
        _C.set_geom_cache(old)
    assert not errs, errs
    assert _C.reuse_stats()["hits"] >= hits + 4, _C.reuse_stats()
    for sd, r in ref.items():
        for x, y in zip(out[sd], r):
            assert torch.equal(x, y), sd


@contextlib.contextmanager
def _binding(native):
    """The native torch binding (the default for the dynamic forward) or the ctypes path."""
    from splatam_amd import _C
    old = _C._NATIVE_ON
    if native and _C._native() is None:
        pytest.fail("the native torch binding did not load")
    _C._NATIVE_ON = bool(native)
    try:
        yield
    finally:
        _C._NATIVE_ON = old


def test_speculation_overflow_relaunch(cuda):
    """The dynamic forward sizes its binning from the last calls' instances per Gaussian and enqueues the
    render before it knows num_rendered; a call with far more instances per Gaussian than the last overflows
    that capacity and re-runs the duplicate and render at the exact size.  That re-launch gives bitwise the
    outputs of the same call made once the size hint has caught up, and the counters the host reads (after
    the duplicate stored them into the pinned snapshot) are this call's."""
    from splatam_amd import _C
    dev = torch.device(cuda)
    e = torch.Tensor([])
    small = make_scene(20000, 320, 240, seed=5)
    big = make_scene(20000, 320, 240, seed=6)
    big.scales = big.scales * 6.0  # many more tiles per Gaussian than the small scene's

    def call(s):
        c = s.cam
        out = _C.rasterize_gaussians(torch.zeros(3, device=dev), s.means3D.to(dev), s.colors.to(dev),
                                     s.opacities.to(dev), s.scales.to(dev), s.rotations.to(dev), 1.0, e,
                                     c.viewmatrix.to(dev), c.projmatrix.to(dev), c.tanfovx, c.tanfovy, c.H, c.W, e, 0,
                                     c.campos.to(dev), False)
        torch.cuda.synchronize()
        return out[0], out[1].cpu(), out[2].cpu(), out[6].cpu()

    n_small = call(small)[0]
    for _ in range(3):
        call(small)  # the hint: the small scene's instances per Gaussian
    first = call(big)  # beyond 1.5x that hint: the re-launch
    again = call(big)  # the hint now matches
    assert first[0] == again[0] and first[0] > 1.5 * n_small * 1.2, (first[0], n_small)
    for a, b in zip(first[1:], again[1:]):
        assert torch.equal(a, b)
