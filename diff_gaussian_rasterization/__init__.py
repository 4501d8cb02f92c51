"""Drop-in for upstream ``diff_gaussian_rasterization`` (JonathonLuiten/diff-gaussian-rasterization-w-depth
@cb65e4b, requirements.txt:16), the module SplaTAM's main loop imports.  Same API
as the vendored fork with ``backward_power`` fixed at 1."""
import torch.nn as nn

from splatam_amd import _C  # noqa: F401
from splatam_amd.rasterizer import GaussianRasterizationSettings, _RasterizeGaussians  # noqa: F401
from splatam_amd.rasterizer import GaussianRasterizer as _Rasterizer
from splatam_amd.rasterizer import rasterize_gaussians as _rasterize


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _rasterize(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                      raster_settings, 1)


class GaussianRasterizer(_Rasterizer):
    def __init__(self, raster_settings):
        nn.Module.__init__(self)
        self.raster_settings = raster_settings
        self.backward_power = 1
