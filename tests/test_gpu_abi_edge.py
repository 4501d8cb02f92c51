"""C-ABI edge cases on the GPU (include/gsr_glue.h): an empty map through the static tracking-L1 forward."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_static_l1_empty_map_zeroes_loss(cuda):
    """gsr_track_forward_dual_static with P = 0 (a caller's non-null colour pointer): the zero silhouette masks
    every pixel, so the loss and the gradient images are zero -- written, not left as whatever the caller's
    buffers held (get_loss on an empty render gives 0: rasterize_points.cu:67-81 returns zero images)."""
    from splatam_amd import _C
    from splatam_amd._lib import GsrGaussians, lib
    from splatam_amd.scenes import make_scene
    from splatam_amd.slam import camera_settings
    scene = make_scene(10, 48, 32, seed=0)
    st = camera_settings(scene.cam, cuda)
    H, W = st.image_height, st.image_width
    s, keep = _C._settings(st.bg, st.viewmatrix, st.projmatrix, st.campos, st.tanfovx, st.tanfovy, H, W,
                           st.scale_modifier, st.sh_degree, st.prefiltered, cuda)
    g = GsrGaussians(P=0, M=0)
    c2 = torch.zeros(1, 3, device=cuda)  # non-null, no rows
    f32 = dict(dtype=torch.float32, device=cuda)
    imgs = [torch.full((3, H, W), 5.0, **f32) for _ in range(2)] + [torch.full((1, H, W), 5.0, **f32)]
    gt_im, gt_d = torch.rand(3, H, W, **f32), torch.rand(1, H, W, **f32) + 0.5
    seed = torch.ones((), **f32)
    loss = torch.full((), 123.0, **f32)
    dim, dds = torch.full((3, H, W), 7.0, **f32), torch.full((3, H, W), 7.0, **f32)
    scratch = torch.zeros(lib.gsr_track_forward_scratch_floats(W, H), **f32)
    status = torch.zeros(4, dtype=torch.int32, device=cuda)
    _C._begin(cuda)
    rc = lib.gsr_track_forward_dual_static(ctypes.byref(s), ctypes.byref(g), c2.data_ptr(), 64, status.data_ptr(),
                                           imgs[0].data_ptr(), imgs[1].data_ptr(), imgs[2].data_ptr(), None,
                                           gt_im.data_ptr(), gt_d.data_ptr(), 0.99, 0.5, 1.0, seed.data_ptr(),
                                           loss.data_ptr(), dim.data_ptr(), dds.data_ptr(), scratch.data_ptr(),
                                           _C._ALLOC_CB, None, _C._stream(cuda))
    assert rc >= 0, lib.gsr_last_error()
    torch.cuda.synchronize()
    assert float(loss) == 0.0
    assert not dim.any() and not dds.any() and not any(t.any() for t in imgs)


def test_mapping_xf_forward_contract(cuda):
    """gsr_forward_dual_static_xf (the mapping transform inside preprocess): refuses store_rendervars = 0 and
    SH colours with GSR_ERR_INVALID_ARG and a message, and an empty map returns zero images."""
    from splatam_amd import _C
    from splatam_amd._lib import GsrGaussians, GsrTrackXform, lib
    from splatam_amd.scenes import make_scene
    from splatam_amd.slam import camera_settings
    scene = make_scene(10, 48, 32, seed=0)
    st = camera_settings(scene.cam, cuda)
    H, W = st.image_height, st.image_width
    s, keep = _C._settings(st.bg, st.viewmatrix, st.projmatrix, st.campos, st.tanfovx, st.tanfovy, H, W,
                           st.scale_modifier, st.sh_degree, st.prefiltered, cuda)
    f32 = dict(dtype=torch.float32, device=cuda)
    P = 4
    mw, ur = torch.rand(P, 3, **f32), torch.rand(P, 4, **f32)
    lo, ls = torch.zeros(P, 1, **f32), torch.full((P, 1), -3.0, **f32)
    q, t, w2c = torch.tensor([1.0, 0, 0, 0], **f32), torch.zeros(3, **f32), torch.eye(4, **f32)
    outs = {k: torch.empty(P, n, **f32) for k, n in (("means", 3), ("rot", 4), ("dcol", 3), ("opac", 1),
                                                      ("scales", 3), ("rgb", 3))}
    status = torch.zeros(4, dtype=torch.int32, device=cuda)
    imgs = [torch.full((3, H, W), 5.0, **f32) for _ in range(2)] + [torch.full((1, H, W), 5.0, **f32)]
    radii = torch.empty(P, dtype=torch.int32, device=cuda)

    def call(p, store, shs=None):
        g = GsrGaussians(P=p, M=16 if shs is not None else 0, means3D=outs["means"].data_ptr(),
                         shs=shs.data_ptr() if shs is not None else None,
                         colors_precomp=outs["rgb"].data_ptr() if shs is None else None,
                         opacities=outs["opac"].data_ptr(), scales=outs["scales"].data_ptr(),
                         rotations=outs["rot"].data_ptr())
        xf = GsrTrackXform(means_world=mw.data_ptr(), unnorm_rot=ur.data_ptr(), logit_opac=lo.data_ptr(),
                           log_scales=ls.data_ptr(), scale_cols=1, cam_q=q.data_ptr(), cam_t=t.data_ptr(), q_stride=1,
                           w2c=w2c.data_ptr(), store_rendervars=store, alive=None)
        _C._begin(cuda)
        return lib.gsr_forward_dual_static_xf(ctypes.byref(s), ctypes.byref(g), outs["dcol"].data_ptr(),
                                              ctypes.byref(xf), 1024, status.data_ptr(), imgs[0].data_ptr(),
                                              imgs[1].data_ptr(), imgs[2].data_ptr(), radii.data_ptr(), _C._ALLOC_CB,
                                              None, _C._stream(cuda))

    assert call(P, 0) < 0 and b"store_rendervars" in lib.gsr_last_error()
    assert call(P, 1, shs=torch.zeros(P, 16, 3, **f32)) < 0 and b"precomputed colours" in lib.gsr_last_error()
    assert call(0, 1) >= 0, lib.gsr_last_error()
    torch.cuda.synchronize()
    assert not any(t.any() for t in imgs)
