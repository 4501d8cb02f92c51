"""Drop-in for the vendored ``hessian_diff_gaussian_rasterization_w_depth``
(GaussianRasterizer(raster_settings, backward_power=1)), backed by splatam_amd."""
from splatam_amd import _C  # noqa: F401  (module attribute `_C`, like the reference)
from splatam_amd.rasterizer import (GaussianRasterizationSettings, GaussianRasterizer,  # noqa: F401
                                    _RasterizeGaussians, rasterize_gaussians)
