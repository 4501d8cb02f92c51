"""Python surface of the rasterizer: a drop-in for SplaTAM's
``GaussianRasterizer`` / ``GaussianRasterizationSettings``.

Mirrors hessian-diff-gaussian-rasterization-w-depth/hessian_diff_gaussian_rasterization_w_depth/__init__.py
(names, argument order, validation messages, output tuples and gradient
order), with the kernels behind it replaced by libgsr.so (HIP, gfx950) via
``splatam_amd._C``.
"""
from __future__ import annotations

from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C
from ._lib import lib


class GaussianRasterizationSettings(NamedTuple):
    """__init__.py:140-151 -- field order matters (positional construction)."""
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings, backward_power=1):
    """__init__.py:17-40."""
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings, backward_power)


class _RasterizeGaussians(torch.autograd.Function):
    """__init__.py:42-138.  Forward returns (color[3,H,W], radii[P], depth[1,H,W]);
    gradients arriving at depth and radii are ignored (__init__.py:92), as in the reference."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings, backward_power):
        s = raster_settings
        num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer, depth = _C.rasterize_gaussians(
            s.bg, means3D, colors_precomp, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
            s.campos, s.prefiltered)
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.backward_power = backward_power
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer,
                              binningBuffer, imgBuffer)
        # the gradients of radii and depth are ignored: no zero tensors materialised for them (two fill
        # launches per call otherwise); the depth output keeps requires_grad, as the reference's does
        ctx.set_materialize_grads(False)
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_out_color, _grad_radii, _grad_depth):
        s = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer,
         imgBuffer) = ctx.saved_tensors
        if grad_out_color is None:  # (a loss that reads only the depth output: what materialisation gave)
            grad_out_color = torch.zeros(3, s.image_height, s.image_width, device=means3D.device)
        # inputs: (means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, ...);
        # outputs of the binding: (dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drotations)
        n = ctx.needs_input_grad
        needs = (n[1], n[3], n[4], True, n[7], n[2], n[5], n[6])
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh, grad_scales,
         grad_rotations) = _C.rasterize_gaussians_backward(
            s.bg, means3D, radii, colors_precomp, scales, rotations, s.scale_modifier, cov3Ds_precomp, s.viewmatrix,
            s.projmatrix, s.tanfovx, s.tanfovy, grad_out_color, sh, s.sh_degree, s.campos, geomBuffer,
            ctx.num_rendered, binningBuffer, imgBuffer, ctx.backward_power, needs=needs)
        if not n[0]:
            grad_means3D = None
        return (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales, grad_rotations,
                grad_cov3Ds_precomp, None, None)


def rasterize_gaussians_dual(means3D, means2D, sh, colors_precomp, colors2, opacities, scales, rotations,
                             cov3Ds_precomp, raster_settings, capacity=0, status=None, grad2_channels=3,
                             means2D_grad_sum=False, sh_adam=None, guard_sink=None, alive=None, xform=None):
    """Two GaussianRasterizer calls on identical geometry fused into one
    rasterization: SplaTAM renders RGB and the [z, 1, z^2]
    depth/silhouette image from the same means / scales / rotations / opacities
    and camera (scripts/splatam.py:255,259).  Returns (color, color2, radii,
    depth); each image is bitwise what a separate call returns, and the gradients
    of the shared inputs are the sums over both images, as autograd would
    accumulate them over two calls.  means2D: the reference's densification statistics read the
    gradient of the RGB render's own means2D (scripts/splatam.py:256), which one rasterization of
    both images does not separate, so means2D receives no gradient unless means2D_grad_sum=True
    asks for the sum over both images; callers that need the RGB-only statistic render the two
    images with two GaussianRasterizer calls.
    capacity > 0: synchronisation-free static mode (gsr_forward_dual_static),
    for HIP-graph capture; check `status` (device int32[4]) afterwards.
    grad2_channels=1: the caller's loss reads only channel 0 of color2 (SplaTAM
    tracking uses the depth, not the silhouette or depth^2, in its loss), so the
    backward skips the other two channels; their incoming gradient must be zero.
    sh_adam: the mapping optimizer (glue.MapAdam) whose colour group steps `sh` in place inside the
    backward (gsr_backward_dual_sh_adam); `sh` then receives no gradient (the caller's own colour step,
    gsr_map_transform_bwd_adam, sees none and leaves the colours to this one).
    alive: uint8 [P] pruning mask for the static mode (0 = removed: culled, zero gradients; GraphMapper's
    in-frame prune_gaussians).
    xform: the mapping transform deferred into this forward (glue.map_transform(defer=...)): preprocess forms
    means3D / rotations / colors2 / opacities / scales from the world-frame map and writes them
    (gsr_forward_dual_static_xf; static mode, precomputed colours)."""
    empty = torch.Tensor([])
    return _RasterizeGaussiansDual.apply(means3D, means2D, empty if sh is None else sh,
                                         empty if colors_precomp is None else colors_precomp, colors2, opacities,
                                         empty if scales is None else scales,
                                         empty if rotations is None else rotations,
                                         empty if cov3Ds_precomp is None else cov3Ds_precomp, raster_settings,
                                         capacity, status, grad2_channels, bool(means2D_grad_sum), sh_adam,
                                         guard_sink, alive, xform)


class _RasterizeGaussiansDual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, colors2, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings, capacity, status, grad2_channels, means2D_grad_sum, sh_adam=None, guard_sink=None,
                alive=None, xform=None):
        s = raster_settings
        num_rendered, color, color2, radii, geomBuffer, binningBuffer, imgBuffer, depth = _C.rasterize_gaussians_dual(
            s.bg, means3D, colors_precomp, colors2, opacities, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, s.image_height, s.image_width, sh, s.sh_degree,
            s.campos, s.prefiltered, capacity=capacity, status=status, alive=alive, xform=xform)
        if guard_sink is not None:
            if capacity > 0:
                # the fused optimizer steps of this iteration guard on this forward's own counters
                # (the geometry buffer stays referenced until the next iteration replaces it); the
                # geometry layout depends on the device's CU count, so the offset is taken on its device
                with torch.cuda.device(means3D.device):
                    off = int(lib.gsr_geom_counters_offset(means3D.shape[0]))
                guard_sink.guard = (geomBuffer, off, int(num_rendered))
            else:
                # an eager forward (no static capacity) never overflows silently: no stale guard from an
                # earlier static forward may decide this iteration's optimizer steps
                guard_sink.guard = None
        ctx.raster_settings = s
        ctx.num_rendered = num_rendered
        ctx.grad2_channels = grad2_channels
        ctx.means2D_grad_sum = means2D_grad_sum
        ctx.sh_adam = sh_adam
        ctx.save_for_backward(colors_precomp, colors2, means3D, scales, rotations, cov3Ds_precomp, radii, sh,
                              geomBuffer, binningBuffer, imgBuffer)
        ctx.mark_non_differentiable(radii, depth)
        ctx.set_materialize_grads(False)  # radii / depth never carry gradients: no zero fills
        return color, color2, radii, depth

    @staticmethod
    def backward(ctx, grad_color, grad_color2, _grad_radii, _grad_depth):
        s = ctx.raster_settings
        (colors_precomp, colors2, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer,
         imgBuffer) = ctx.saved_tensors
        if grad_color is None:
            grad_color = torch.zeros(3, s.image_height, s.image_width, device=means3D.device)
        if grad_color2 is None:
            grad_color2 = torch.zeros(3, s.image_height, s.image_width, device=means3D.device)
        n = ctx.needs_input_grad  # (means3D, means2D, sh, colors_precomp, colors2, opacities, scales, rotations, cov3D)
        needs = (n[1] and ctx.means2D_grad_sum, n[3], n[4], n[5], n[0], n[8], n[2], n[6], n[7])
        sa = None
        if ctx.sh_adam is not None:  # the colour group's upcoming step (the transform backward counts it)
            sa = ctx.sh_adam.struct()
            sa.step = ctx.sh_adam.step + 1
        (g_m2, g_col, g_col2, g_op, g_m3, g_cov, g_sh, g_sc, g_rot) = _C.rasterize_gaussians_dual_backward(
            s.bg, means3D, radii, colors_precomp, colors2, scales, rotations, s.scale_modifier, cov3Ds_precomp,
            s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, grad_color, grad_color2, sh, s.sh_degree, s.campos,
            geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, needs=needs,
            dl2_channels=ctx.grad2_channels if grad_color2 is not None else 3, sh_adam=sa)
        if not n[0]:
            g_m3 = None
        return g_m3, g_m2, g_sh, g_col, g_col2, g_op, g_sc, g_rot, g_cov, None, None, None, None, None, None, None, None, \
            None


class GaussianRasterizer(nn.Module):
    """__init__.py:153-204.  ``backward_power`` is the fork's Fisher knob (1 = standard gradients)."""

    def __init__(self, raster_settings, backward_power: int = 1):
        super().__init__()
        self.raster_settings = raster_settings
        self.backward_power = backward_power

    def markVisible(self, positions):
        with torch.no_grad():
            s = self.raster_settings
            return _C.mark_visible(positions, s.viewmatrix, s.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        s = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        empty = torch.Tensor([])
        shs = empty if shs is None else shs
        colors_precomp = empty if colors_precomp is None else colors_precomp
        scales = empty if scales is None else scales
        rotations = empty if rotations is None else rotations
        cov3D_precomp = empty if cov3D_precomp is None else cov3D_precomp
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations,
                                   cov3D_precomp, s, self.backward_power)
