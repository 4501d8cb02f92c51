/*
 * gsr.h -- C ABI of the MI355X-native differentiable Gaussian rasterizer
 * (libgsr.so, built from the splatam_amd/csrc HIP sources for gfx950).
 *
 * This is the drop-in boundary for the reference's torch extension `_C`
 * (hessian-diff-gaussian-rasterization-w-depth/ext.cpp:15-18).  Every entry
 * point takes plain device pointers, sizes and a hipStream_t (as void*); no
 * torch types cross it.  The Python binding splatam_amd/_C.py (ctypes) is the
 * ~100-line tensor -> pointer marshalling layer on top of it; INTEGRATION.md
 * shows the binding a maintainer would add on the reference side.
 *
 * Conventions:
 *   - every float array is float32, contiguous, on the device the stream belongs to;
 *   - "absent" inputs (shs, colors_precomp, scales, rotations, cov3D_precomp)
 *     are NULL pointers (the reference turns an empty tensor into nullptr);
 *   - viewmatrix / projmatrix are the reference's column-major 4x4 (16 floats,
 *     element (r,c) at index 4c+r), campos / bg are 3 floats, all on device;
 *   - opaque state buffers are allocated through the caller's allocator
 *     callback and must be passed back unchanged to gsr_backward;
 *   - all work is enqueued on `stream`; gsr_forward synchronises the stream
 *     once to read num_rendered (rasterizer_impl.cu:282 does the same);
 *   - negative return values are errors; gsr_last_error() gives the message
 *     (thread-local).  Re-entrant across devices and threads: the only host-side
 *     state is kept per device of the launch stream (the binning-capacity hint,
 *     the stage timing) and per (thread, device) (the pinned num_rendered staging
 *     word and its event).
 */
#ifndef GSR_H
#define GSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ABI_VERSION 8

/* error codes */
#define GSR_OK 0
#define GSR_ERR_INVALID_ARG (-1)
#define GSR_ERR_ALLOC (-2)
#define GSR_ERR_HIP (-3)
#define GSR_ERR_PREFILTERED (-4) /* auxiliary.h:154-160 traps; we report instead */

/* buffer kinds handed to the allocator callback */
#define GSR_BUF_GEOM 0    /* per-Gaussian state   (reference geomBuffer)    */
#define GSR_BUF_BINNING 1 /* per-instance state   (reference binningBuffer) */
#define GSR_BUF_IMAGE 2   /* per-pixel/tile state (reference imgBuffer)     */
#define GSR_BUF_SCRATCH 3 /* backward scratch, released by the caller after gsr_backward */

/* Returns a device pointer to at least `bytes` bytes (256-byte aligned), or
 * NULL on failure.  Replaces resizeFunctional (rasterize_points.cu:27-33). */
typedef void* (*gsr_alloc_fn)(void* ctx, int kind, size_t bytes);

/* GaussianRasterizationSettings (hessian_diff_gaussian_rasterization_w_depth/__init__.py:140-151) */
typedef struct gsr_settings {
    int image_height;
    int image_width;
    float tan_fovx;
    float tan_fovy;
    const float* bg;          /* [3] */
    float scale_modifier;
    const float* viewmatrix;  /* [16] column-major */
    const float* projmatrix;  /* [16] column-major */
    int sh_degree;
    const float* campos;      /* [3] */
    int prefiltered;
    /* Not in the reference's settings (its binning is internal to the forward / backward pair); a
     * per-call choice, no process-wide state.  GSR_BINNING_CULLED (0, the default of a zero-initialised
     * struct): a (Gaussian, tile) instance whose alpha >= 1/255 ellipse reaches no 4x4 block of the tile
     * is left out of the tile's sorted list -- it would be staged but never evaluated.  Images, radii,
     * num_rendered and gradients are bitwise those of the reference's lists.  GSR_BINNING_REFERENCE (1):
     * every rect instance listed, rasterizer_impl.cu:290-315 entry for entry.  Either way the binning
     * buffer's point list holds num_rendered valid entries: point_list[0, L) are the tiles' sorted lists
     * (L = the ranges' total) and point_list[L, num_rendered) has an empty block mask and a valid Gaussian
     * id -- in gsr_forward / gsr_forward_dual (the buffers a caller reads like the reference's) the culled
     * instances themselves, so the ids are the reference's multiset (Gaussian i appears tiles_touched(i)
     * times); in the static-capacity forwards, whose buffers only this library reads, padding (the Gaussian
     * owning each of the last rect instance slots), which costs the binning nothing. */
    int binning;
} gsr_settings;

#define GSR_BINNING_CULLED 0
#define GSR_BINNING_REFERENCE 1

/* Per-Gaussian inputs (rasterize_points.cu:36-54 argument list) */
typedef struct gsr_gaussians {
    int P;                      /* number of Gaussians */
    int M;                      /* SH coefficients per Gaussian (0 when shs == NULL) */
    const float* means3D;       /* [P,3] */
    const float* shs;           /* [P,M,3] or NULL */
    const float* colors_precomp;/* [P,3]   or NULL */
    const float* opacities;     /* [P,1] */
    const float* scales;        /* [P,3]   or NULL */
    const float* rotations;     /* [P,4]   or NULL (w,x,y,z; not normalised in-kernel) */
    const float* cov3D_precomp; /* [P,6]   or NULL */
} gsr_gaussians;

/* Output of rasterize_gaussians_backward (rasterize_points.cu:195), each
 * written in full by gsr_backward (no zero-initialisation needed); with
 * power == 1 a NULL pointer (other than dmeans3D) skips that gradient. */
typedef struct gsr_grads {
    float* dmeans2D;    /* [P,3] (z component 0) */
    float* dcolors;     /* [P,3] */
    float* dopacity;    /* [P,1] */
    float* dmeans3D;    /* [P,3] */
    float* dcov3D;      /* [P,6] */
    float* dsh;         /* [P,M,3] (NULL allowed when M == 0) */
    float* dscales;     /* [P,3] */
    float* drotations;  /* [P,4] */
} gsr_grads;

/* Forward rasterization.  Replaces CudaRasterizer::Rasterizer::forward
 * (rasterizer_impl.cu:198-339) behind RasterizeGaussiansCUDA
 * (rasterize_points.cu:35-115).  Writes out_color [3,H,W], out_depth [1,H,W]
 * (median depth, 15 when T never crosses 0.5) and radii [P].  Returns
 * num_rendered (>= 0) or a negative error code. */
int gsr_forward(const gsr_settings* settings, const gsr_gaussians* gaussians,
                float* out_color, float* out_depth, int* radii,
                gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* Backward.  Replaces CudaRasterizer::Rasterizer::backward
 * (rasterizer_impl.cu:343-434) behind RasterizeGaussiansBackwardCUDA
 * (rasterize_points.cu:117-196).  `power` is the vendored fork's
 * backward_power (backward.cu:1093-1137): gradients are summed over
 * (pixel, Gaussian) pairs of powf(per-pair gradient, power); power == 1 is the
 * standard 3DGS backward.  H/W come from settings (the reference reads them
 * from dL_dout_color).  With power == 1 every gradient pointer except
 * dmeans3D may be NULL: that gradient is skipped, and render_bwd does not form
 * the per-pair sums only it needs (dopacity, dcolors without SH).  Returns
 * GSR_OK or a negative error code. */
int gsr_backward(const gsr_settings* settings, const gsr_gaussians* gaussians,
                 const int* radii, const float* dL_dout_color, int num_rendered,
                 const void* geom_buffer, const void* binning_buffer, const void* image_buffer,
                 int power, const gsr_grads* grads,
                 gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* Dual render: one rasterization composites a second colour set colors2
 * [P,3] (precomputed) with the same alpha / transmittance, i.e. the two
 * GaussianRasterizer calls SplaTAM makes per iteration on identical geometry
 * (RGB and [z, 1, z^2], scripts/splatam.py:255,259), sharing preprocess,
 * binning and the per-pair evaluation.  out_color and
 * out_color2 are bitwise the images two gsr_forward calls would produce. */
int gsr_forward_dual(const gsr_settings* settings, const gsr_gaussians* gaussians,
                     const float* colors2, float* out_color, float* out_color2, float* out_depth,
                     int* radii, gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* Static-capacity, synchronisation-free gsr_forward_dual (capturable in a HIP
 * graph).  The binning buffer holds `capacity` instances; nothing waits on the
 * host.  The device counters are merged into `status` (device, 4 x u32) when
 * the stream reaches that point: [0] = max(num_rendered), [1] |= prefiltered
 * violation, [2] = max(longest tile list), [3] = the longest list the per-tile
 * sort handles (4096).  The row is sticky: an overflow in any call (e.g. any
 * replay of a captured graph) stays visible until the caller zeroes the row.
 * This call's outputs are valid iff its num_rendered <= capacity and its
 * longest list <= 4096 (longer lists need gsr_forward_dual); otherwise every
 * kernel after the scan skipped its work (no out-of-bounds writes), the fused
 * optimizer steps of include/gsr_glue.h skip theirs, and the call must be
 * repeated with a larger capacity or in the synchronous mode.  Returns
 * `capacity`: pass it as num_rendered to gsr_backward_dual (it sizes the
 * buffer layouts). */
int gsr_forward_dual_static(const gsr_settings* settings, const gsr_gaussians* gaussians,
                            const float* colors2, int capacity, unsigned* status,
                            float* out_color, float* out_color2, float* out_depth, int* radii,
                            gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* Geometry-reuse forward (SURVEY.md 8(f) row 1 for unchanged callers): the
 * second of two gsr_forward calls on identical geometry and camera -- SplaTAM's
 * RGB then depth/silhouette Renderer calls (scripts/splatam.py:255,259), each
 * through RasterizeGaussiansCUDA (rasterize_points.cu:35-115) -- skips
 * preprocess, binning and the tile sort: the new geometry buffer is the
 * previous one with the colours of `gaussians` (colors_precomp, required; no
 * SH) written into its render records, the binning and image buffers of the
 * previous call are reused in place (their content is what this call would
 * compute), radii are copied.  The caller guarantees (gsr_bitwise_equal on
 * the device, identity of the unchanged tensors on the host) that means3D,
 * scales, rotations, opacities and every setting equal those of the call that
 * produced prev_geom / binning_buffer / image_buffer, which must still be
 * alive.  Returns num_rendered (the previous call's) or a negative error. */
int gsr_forward_reuse(const gsr_settings* settings, const gsr_gaussians* gaussians, int num_rendered,
                      const void* prev_geom, void* binning_buffer, void* image_buffer, const int* prev_radii,
                      float* out_color, float* out_depth, int* radii,
                      gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* gsr_forward with the geometry reuse decided on the device (SplaTAM's second
 * Renderer call of an iteration, scripts/splatam.py:255,259): the `npairs`
 * (<= 8) float arrays a[k] / b[k] of n[k] elements -- this call's and the
 * previous call's rotations / opacities / scales -- are compared bitwise on the
 * device, and both forms are enqueued, each launch gated on the result: equal
 * -> the gsr_forward_reuse form (the previous call's geometry with this call's
 * colours, its sorted lists; *reused = 1, num_rendered = prev_num_rendered, and
 * the binning and image buffers the backward must get are prev_binning /
 * prev_image, whose final_T / n_contrib are rewritten with the same values);
 * different -> the full gsr_forward (*reused = 0, this call's own buffers).
 * The host waits once, on the counter copy gsr_forward waits on anyway.  The
 * caller guarantees what gsr_forward_reuse requires of everything else (same
 * means3D, camera and settings; colors_precomp, no SH; the previous call's
 * buffers alive).  Returns num_rendered or a negative error. */
int gsr_forward_reuse_if_equal(const gsr_settings* settings, const gsr_gaussians* gaussians, int npairs,
                               const float* const* a, const float* const* b, const long long* n,
                               int prev_num_rendered, const void* prev_geom, void* prev_binning, void* prev_image,
                               const int* prev_radii, float* out_color, float* out_depth, int* radii, int* reused,
                               gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* Zeroes *flag (device int) and sets it to non-zero when any of the
 * `npairs` (<= 8) float arrays a[k][0..n[k]) and b[k][0..n[k]) differ bitwise.
 * Enqueued on `stream`; the host reads the flag after a stream sync. */
int gsr_bitwise_equal(int npairs, const float* const* a, const float* const* b, const long long* n, int* flag,
                      void* stream);

/* Static-capacity, synchronisation-free gsr_forward (one colour set): the
 * gsr_forward_dual_static contract (capacity, sticky status row, returns
 * `capacity` for gsr_backward's num_rendered) for a single render -- e.g. the
 * HIP-graph-captured Fisher scoring of a batch of poses (backward_power 2). */
int gsr_forward_static(const gsr_settings* settings, const gsr_gaussians* gaussians, int capacity,
                       unsigned* status, float* out_color, float* out_depth, int* radii,
                       gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* Backward of gsr_forward_dual (power 1): every geometric gradient in `grads`
 * is the sum of the two renders' (as autograd would accumulate it over two
 * calls), grads->dcolors is d/dcolors of the first set and dcolors2 [P,3]
 * that of colors2 (NULL skips it, as for the pointers in `grads`).
 * dl2_channels: 3, or 1 when the caller guarantees channels 1 and 2 of
 * dL_dout_color2 are zero (SplaTAM tracking differentiates only the depth of
 * the [depth, silhouette, depth^2] render); those channels are then not read
 * and dcolors2[:,1:] is written as zero. */
int gsr_backward_dual(const gsr_settings* settings, const gsr_gaussians* gaussians,
                      const int* radii, const float* colors2, const float* dL_dout_color,
                      const float* dL_dout_color2, int num_rendered, const void* geom_buffer,
                      const void* binning_buffer, const void* image_buffer, const gsr_grads* grads,
                      float* dcolors2, int dl2_channels, gsr_alloc_fn alloc, void* alloc_ctx,
                      void* stream);

/* Frustum test view_z > 0.001.  Replaces markVisible / checkFrustum
 * (rasterize_points.cu:198-216, rasterizer_impl.cu:54-67,141-153).
 * visible: [P] bytes (0/1, torch.bool layout). */
int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix,
                     const float* projmatrix, uint8_t* visible, void* stream);

/* Byte sizes of the opaque buffers (for tests and pre-sizing).  The geometry buffer's size (and the
 * counters' offset) depends on P and on the current device's CU count: its per-row scan arrays hold one
 * entry per 512 or 1024 Gaussians (rows of 512 when rows of 1024 would leave fewer than two per CU). */
size_t gsr_geom_buffer_bytes(int P);
size_t gsr_binning_buffer_bytes(int num_rendered, int image_width, int image_height);
size_t gsr_image_buffer_bytes(int image_width, int image_height);
/* Byte offset, inside a geometry buffer of P Gaussians, of the forward's device counters
 * (4 x u32, the status-row layout of gsr_forward_dual_static: num_rendered, prefiltered
 * violation, longest tile list, sort cap).  Passed as gsr_map_adam.status, they make the
 * fused optimizer steps guard on that one call's forward instead of a sticky status row. */
size_t gsr_geom_counters_offset(int P);

const char* gsr_last_error(void);
int gsr_abi_version(void);

/* Per-stage device timing (diagnostics, bench.py).  When enabled, every stage
 * below is bracketed by hipEvents recorded on the launch stream; read returns
 * accumulated milliseconds, launch counts and work units (P for per-Gaussian
 * stages, num_rendered for per-instance stages) since the last enable.
 * Per device: enable / read act on the calling thread's current device and
 * cover launches on that device from any thread (autograd runs backward on its
 * own thread).  gsr_timing_read synchronises on the recorded events. */
#define GSR_STAGE_PREPROCESS 0 /* preprocess + tile-count scan  */
#define GSR_STAGE_DUPLICATE 1  /* duplicateWithKeys              */
#define GSR_STAGE_SORT 2       /* radix sort (all passes)        */
#define GSR_STAGE_RANGES 3     /* identifyTileRanges + id gather */
#define GSR_STAGE_RENDER_FWD 4 /* renderCUDA forward             */
#define GSR_STAGE_RENDER_BWD 5 /* render backward                */
#define GSR_STAGE_GAUSS_BWD 6  /* per-Gaussian chain rule        */
#define GSR_NUM_STAGES 7
/* on: 0 off, 1 hipEvents around every stage (not usable under stream capture),
 * GSR_TIMING_CLOCK | stage_mask: device-clock mode -- the stages in stage_mask
 * (bit = stage id) are timed with wall_clock64() on the device and accumulated
 * there, so captured HIP graphs accumulate over every replay.  The render
 * stages stamp themselves inside the kernel (first workgroup start -> last
 * workgroup end, no extra launches); other stages get one-thread stamp kernels
 * before/after their launches. */
#define GSR_TIMING_CLOCK 0x100
int gsr_timing_enable(int on);
int gsr_timing_read(double* ms, long long* launches, long long* units, int n);

/* Test hook (tests/test_gpu_kernels.py): wave64 transposed reduction of
 * in_dev[64*9] (lane-major) into out_dev[9]; checks the permlane/DPP lane
 * mapping the backward relies on. */
int gsr_selftest_reduce9(const float* in_dev, float* out_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H */
