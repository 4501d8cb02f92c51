"""Loads libgsr.so (the C ABI of include/gsr.h) with ctypes.

Fails loudly: there is no CPU or eager-PyTorch fallback for the rasterizer.
Set GSR_LIB to load a library from another path (same strict symbol / ABI checks).  GSR_LIB_AB=1 in
addition relaxes them for an A/B baseline built from an older revision (build.build_from_rev): entry
points added since that revision may be absent and ABI versions 4 / 5 are accepted.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSR_LIB", os.path.join(_HERE, "libgsr.so"))

c_int, c_float, c_void_p, c_size_t = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
c_double = ctypes.c_double


class GsrSettings(ctypes.Structure):
    """gsr_settings (include/gsr.h)."""
    _fields_ = [("image_height", c_int), ("image_width", c_int), ("tan_fovx", c_float), ("tan_fovy", c_float),
                ("bg", c_void_p), ("scale_modifier", c_float), ("viewmatrix", c_void_p), ("projmatrix", c_void_p),
                ("sh_degree", c_int), ("campos", c_void_p), ("prefiltered", c_int), ("binning", c_int)]


class GsrGaussians(ctypes.Structure):
    """gsr_gaussians (include/gsr.h)."""
    _fields_ = [("P", c_int), ("M", c_int), ("means3D", c_void_p), ("shs", c_void_p), ("colors_precomp", c_void_p),
                ("opacities", c_void_p), ("scales", c_void_p), ("rotations", c_void_p), ("cov3D_precomp", c_void_p)]


class GsrGrads(ctypes.Structure):
    """gsr_grads (include/gsr.h)."""
    _fields_ = [("dmeans2D", c_void_p), ("dcolors", c_void_p), ("dopacity", c_void_p), ("dmeans3D", c_void_p),
                ("dcov3D", c_void_p), ("dsh", c_void_p), ("dscales", c_void_p), ("drotations", c_void_p)]


class GsrMapAdam(ctypes.Structure):
    """gsr_map_adam (include/gsr_glue.h)."""
    _fields_ = [("exp_avg", c_void_p * 5), ("exp_avg_sq", c_void_p * 5), ("lr", c_double * 5), ("step", c_int),
                ("beta1", c_double), ("beta2", c_double), ("eps", c_double), ("status", c_void_p),
                ("capacity", ctypes.c_uint), ("halted", c_void_p)]


class GsrTrackXform(ctypes.Structure):
    """gsr_track_xform (include/gsr_glue.h)."""
    _fields_ = [("means_world", c_void_p), ("unnorm_rot", c_void_p), ("logit_opac", c_void_p),
                ("log_scales", c_void_p), ("scale_cols", c_int), ("cam_q", c_void_p), ("cam_t", c_void_p),
                ("q_stride", c_int), ("w2c", c_void_p), ("store_rendervars", c_int), ("alive", c_void_p)]


class GsrPoseTrack(ctypes.Structure):
    """gsr_pose_track (include/gsr_glue.h)."""
    _fields_ = [("status", c_void_p), ("capacity", ctypes.c_uint), ("loss", c_void_p), ("best", c_void_p)]


class GsrAdamTensor(ctypes.Structure):
    """gsr_adam_tensor (include/gsr_glue.h)."""
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("n", ctypes.c_longlong), ("lr", c_double)]


ALLOC_FN = ctypes.CFUNCTYPE(c_void_p, c_void_p, c_int, c_size_t)

# every symbol declared in include/gsr.h: (name, restype, argtypes)
SIGNATURES = {
    "gsr_forward": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p, c_void_p, c_void_p,
                            ALLOC_FN, c_void_p, c_void_p]),
    "gsr_backward": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p, c_void_p, c_int,
                             c_void_p, c_void_p, c_void_p, c_int, ctypes.POINTER(GsrGrads), ALLOC_FN, c_void_p,
                             c_void_p]),
    "gsr_forward_dual": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, ALLOC_FN, c_void_p, c_void_p]),
    "gsr_forward_static": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_int, c_void_p,
                                   c_void_p, c_void_p, c_void_p, ALLOC_FN, c_void_p, c_void_p]),
    "gsr_forward_dual_static": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p, c_int,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ALLOC_FN, c_void_p,
                                        c_void_p]),
    "gsr_backward_dual": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, ctypes.POINTER(GsrGrads),
                                  c_void_p, c_int, ALLOC_FN, c_void_p, c_void_p]),
    "gsr_forward_reuse": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_int, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ALLOC_FN, c_void_p,
                                  c_void_p]),
    "gsr_forward_reuse_if_equal": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_int,
                                           c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ALLOC_FN, c_void_p,
                                           c_void_p]),
    "gsr_bitwise_equal": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsr_mark_visible": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsr_geom_buffer_bytes": (c_size_t, [c_int]),
    "gsr_geom_counters_offset": (c_size_t, [c_int]),
    "gsr_binning_buffer_bytes": (c_size_t, [c_int, c_int, c_int]),
    "gsr_image_buffer_bytes": (c_size_t, [c_int, c_int]),
    "gsr_last_error": (ctypes.c_char_p, []),
    "gsr_abi_version": (c_int, []),
    "gsr_selftest_reduce9": (c_int, [c_void_p, c_void_p, c_void_p]),
    "gsr_timing_enable": (c_int, [c_int]),
    "gsr_timing_read": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
    # include/gsr_glue.h: fused SplaTAM tracking glue
    "gsr_track_scratch_floats": (c_int, [c_int]),
    "gsr_track_transform_fwd": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                        c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsr_track_transform_bwd": (c_int, [c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "gsr_track_transform_bwd_adam": (c_int, [c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_void_p, c_double, c_double,
                                             c_double, c_double, c_double, c_void_p, c_void_p,
                                             ctypes.POINTER(GsrPoseTrack), c_void_p]),
    "gsr_track_l1_fwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float,
                                 ctypes.c_float, ctypes.c_float, c_void_p, c_void_p, c_void_p]),
    "gsr_track_l1_bwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float,
                                 ctypes.c_float, ctypes.c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsr_track_l1_fwd_bwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_float,
                                     ctypes.c_float, ctypes.c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
    "gsr_track_forward_scratch_floats": (c_int, [c_int, c_int]),
    "gsr_track_forward_dual_static": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p,
                                              c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p, ALLOC_FN, c_void_p, c_void_p]),
    "gsr_track_forward_dual_static_xf": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p,
                                                 ctypes.POINTER(GsrTrackXform), c_int, c_void_p, c_void_p, c_void_p,
                                                 c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_float,
                                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ALLOC_FN, c_void_p,
                                                 c_void_p]),
    "gsr_track_records_floats": (c_int, [c_int]),
    "gsr_track_forward_backward_dual_static_xf": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians),
                                                          c_void_p, ctypes.POINTER(GsrTrackXform), c_int, c_void_p,
                                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                          c_float, c_float, c_float, c_void_p, c_void_p, c_void_p,
                                                          c_void_p, ALLOC_FN, c_void_p, c_void_p]),
    "gsr_track_backward_dual_records": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p,
                                                c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                c_int, c_void_p, c_void_p, c_int, c_void_p, c_double, c_double,
                                                c_double, c_double, c_double, c_void_p, c_void_p, c_void_p, c_void_p,
                                                ctypes.POINTER(GsrPoseTrack), c_void_p, c_void_p, ALLOC_FN, c_void_p,
                                                c_void_p]),
    "gsr_backward_dual_sh_adam": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                          ctypes.POINTER(GsrGrads), c_void_p, c_int, ctypes.POINTER(GsrMapAdam),
                                          ALLOC_FN, c_void_p, c_void_p]),
    "gsr_track_backward_scratch_floats": (c_int, [c_int]),
    "gsr_track_backward_dual": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_int, c_void_p, c_void_p, c_int, c_void_p, c_double, c_double, c_double,
                                        c_double, c_double, c_void_p, c_void_p, c_void_p, c_void_p,
                                        ctypes.POINTER(GsrPoseTrack), c_void_p, ALLOC_FN, c_void_p, c_void_p]),
    # include/gsr_glue.h: fused SplaTAM mapping glue and optimizer
    "gsr_map_loss_scratch_floats": (c_int, [c_int, c_int]),
    "gsr_map_loss_state_floats": (c_int, [c_int, c_int]),
    "gsr_map_loss_fwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_void_p,
                                 c_void_p, c_void_p, c_void_p]),
    "gsr_map_loss_bwd": (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsr_map_transform_bwd": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p]),
    "gsr_map_transform_bwd_adam": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                                           c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, ctypes.POINTER(GsrMapAdam), c_void_p]),
    "gsr_adam_step": (c_int, [c_int, ctypes.POINTER(GsrAdamTensor), c_int, c_double, c_double, c_double, c_void_p]),
    "gsr_map_prune": (c_int, [c_int, c_void_p, c_void_p, c_int, c_float, c_float, c_int, c_void_p, c_void_p]),
    "gsr_forward_dual_static_alive": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p,
                                              c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              ALLOC_FN, c_void_p, c_void_p]),
    "gsr_forward_dual_static_xf": (c_int, [ctypes.POINTER(GsrSettings), ctypes.POINTER(GsrGaussians), c_void_p,
                                           ctypes.POINTER(GsrTrackXform), c_int, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, ALLOC_FN, c_void_p, c_void_p]),
    # include/gsr_glue.h: Fisher scoring glue
    "gsr_points_to_camera": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gsr_fisher_accumulate": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
}


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(f"libgsr.so not found at {path}: build it with `python -m splatam_amd.build` "
                          "(no CPU fallback exists for the rasterizer)")
    lib = ctypes.CDLL(path)
    # an A/B baseline built from an older revision (build.build_from_rev): explicit opt-in only
    ab = os.environ.get("GSR_LIB_AB") == "1" and bool(os.environ.get("GSR_LIB"))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if ab:  # (entry points added since that revision: absent, the callers fall back)
                continue
            raise ImportError(f"libgsr.so lacks {name}")
        fn.restype = res
        fn.argtypes = args
    v = lib.gsr_abi_version()
    if v != 8:
        # an older revision may differ in the glue structs only (ABI 4: gsr_map_adam without `halted`;
        # ABI 5: no fused tracking render; ABI 6: gsr_settings without `binning`, which such a library does
        # not read; ABI 7: no gsr_forward_reuse_if_equal); the rasterizer calls are unchanged
        if not (ab and v in (4, 5, 6, 7)):
            raise ImportError("libgsr.so ABI version mismatch")
    return lib


lib = load()
