"""splatam_amd -- MI355X-native (HIP / gfx950) differentiable Gaussian rasterizer
for SplaTAM, a drop-in for diff_gaussian_rasterization /
hessian_diff_gaussian_rasterization_w_depth.

The rasterizer classes are imported lazily so that the host-only helpers
(scenes, build) work without libgsr.so.
"""
__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians"]


def __getattr__(name):
    if name in __all__:
        from . import rasterizer
        return getattr(rasterizer, name)
    raise AttributeError(name)
