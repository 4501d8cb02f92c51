/* gsr_glue.h -- fused SplaTAM caller glue around the rasterizer.
 *
 * SplaTAM's tracking iteration (scripts/splatam.py:220-353, tracking=True)
 * spends more GPU time in ~300 small torch kernels around the two rasterizer
 * calls than in the rasterizer itself.  These entry points restate that glue
 * as a handful of HIP kernels with exactly the reference's math:
 *
 *   gsr_track_transform_fwd / _bwd
 *       transform_to_frame(params, t, gaussians_grad=False, camera_grad=True)
 *           (utils/slam_helpers.py:252-304)
 *       + transformed_params2rendervar / ...depthplussilhouette rotations,
 *         opacities and scales (slam_helpers.py:124-139, 234-249)
 *       + get_depth_and_silhouette colours [z, 1, z^2] (slam_helpers.py:196-213)
 *       Backward: gradient w.r.t. the frame's unnormalised camera quaternion and
 *       translation only (the Gaussians are detached in tracking), through
 *       F.normalize, build_rotation's own normalisation (slam_external.py:25-42)
 *       and, for anisotropic maps, quat_mult(cam_rot, normalize(q)).
 *       Deterministic: fixed-order two-level reduction.
 *
 *   gsr_track_l1_fwd / _bwd
 *       get_loss's tracking L1 terms (splatam.py:262-296 with use_l1,
 *       use_sil_for_loss, ignore_outlier_depth_loss=False): mask =
 *       (gt_depth > 0) & !isnan(depth) & !isnan(depth_sq - depth^2) &
 *       (silhouette > sil_thres); loss = w_im * sum(mask * |gt_im - im|) +
 *       w_depth * sum(mask * |gt_depth - depth|), and its gradient w.r.t. the
 *       RGB render and the [depth, silhouette, depth^2] render.
 *
 * All pointers are device float32 (contiguous), sizes in elements, `stream`
 * a hipStream_t.  Return GSR_OK (0) or a negative GSR_ERR_* (see gsr.h).
 */
#ifndef GSR_GLUE_H
#define GSR_GLUE_H

#include "gsr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Scratch floats needed by gsr_track_transform_bwd(_adam) (n = P) and
 * gsr_track_l1_fwd(_bwd) (n = H*W): per-workgroup partials followed by an
 * arrival counter.  The scratch must be zero-filled before its first use; every
 * call leaves it zero-filled, so one buffer serves any number of calls on one
 * stream (not calls running concurrently). */
int gsr_track_scratch_floats(int n);

/* cam_q: the frame's unnormalised (w,x,y,z) quaternion, element k at cam_q[k * q_stride]
 *        (params["cam_unnorm_rots"][..., t] is a strided view); cam_t likewise (3 values).
 * unnorm_rot [P,4], logit_opac [P,1], log_scales [P,S] (S = 1 isotropic -> tiled to 3, or 3).
 * w2c [4,4] row-major: curr_data["w2c"] used for the depth colours.
 * Outputs [P,3] means_cam, [P,4] rotations (normalised, rendervar form), [P,3] depth_colors,
 *         [P,1] opacities, [P,3] scales. */
int gsr_track_transform_fwd(int P, const float* means_world, const float* unnorm_rot, const float* logit_opac,
                            const float* log_scales, int scale_cols, const float* cam_q, const float* cam_t,
                            int q_stride, const float* w2c, float* means_cam, float* rotations, float* depth_colors,
                            float* opacities, float* scales, void* stream);

/* dL_dmeans_cam [P,3] (sum over both renders), dL_drot [P,4] (may be NULL), dL_ddepth_colors [P,3]
 * (may be NULL).  Writes dL/dcam_q (4 values, stride q_stride) and dL/dcam_t (3 values, stride
 * q_stride); scratch: gsr_track_scratch_floats(P) floats. */
int gsr_track_transform_bwd(int P, const float* means_world, const float* unnorm_rot, int scale_cols,
                            const float* cam_q, const float* means_cam, const float* w2c,
                            const float* dL_dmeans_cam, const float* dL_drot, const float* dL_ddepth_colors,
                            float* dL_dcam_q, float* dL_dcam_t, int q_stride, float* scratch, void* stream);

/* gsr_track_transform_bwd with the optimizer step fused in:
 * instead of writing the pose gradient, applies torch.optim.Adam (no weight
 * decay, no amsgrad; the tracking optimizer of scripts/splatam.py) to the
 * frame's pose column in place: cam_q (4 values) / cam_t (3 values) at stride
 * q_stride.  Hyperparameters are doubles (torch's are python floats: 1 - beta2
 * rounded from a float beta2 would be 1.3e-5 off).  adam_state: device, 15 floats [m_q 4, v_q 4, m_t 3, v_t 3, step],
 * zero-initialised by the caller per frame (SplaTAM re-creates the optimizer per
 * frame). */
/* Optional per-iteration bookkeeping of the fused pose optimizer (may be NULL):
 *   status / capacity: the static-mode status row of this iteration's forward and its binning
 *       capacity; when the row shows an overflow ([0] > capacity, [2] > [3], or [1] != 0) the
 *       Adam step is skipped -- pose and optimizer state stay as they were (the outputs of an
 *       overflowing forward are invalid);
 *   loss / best: scripts/splatam.py:726-731 best-candidate selection: after the step, if
 *       *loss < best[0] then best[0] = *loss, best[1..4] = the updated quaternion and
 *       best[5..7] = the updated translation (a NaN loss never replaces the candidate).  The
 *       caller starts a frame with best[0] = 1e20 and writes best[1..7] back after its last
 *       iteration (:760-763). */
typedef struct gsr_pose_track {
    const unsigned* status;
    unsigned capacity;
    const float* loss;
    float* best;
} gsr_pose_track;

int gsr_track_transform_bwd_adam(int P, const float* means_world, const float* unnorm_rot, int scale_cols,
                                 float* cam_q, float* cam_t, int q_stride, const float* means_cam,
                                 const float* w2c, const float* dL_dmeans_cam, const float* dL_drot,
                                 const float* dL_ddepth_colors, double lr_q, double lr_t, double beta1,
                                 double beta2, double eps, float* adam_state, float* scratch,
                                 const gsr_pose_track* track, void* stream);

/* im [3,H,W], depth_sil [3,H,W] (depth, silhouette, depth^2), gt_im [3,H,W], gt_depth [1,H,W].
 * loss: 1 float (device).  scratch: gsr_track_scratch_floats(H*W) floats. */
int gsr_track_l1_fwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im,
                     const float* gt_depth, float sil_thres, float w_im, float w_depth, float* loss, float* scratch,
                     void* stream);

/* gsr_track_l1_fwd and gsr_track_l1_bwd in one pass (one launch): dL_dloss is
 * read when the kernel runs, so the caller's loss seed must already hold its
 * value (a static seed, e.g. the tracker's ones). */
int gsr_track_l1_fwd_bwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im,
                         const float* gt_depth, float sil_thres, float w_im, float w_depth, const float* dL_dloss,
                         float* loss, float* dL_dim, float* dL_ddepth_sil, float* scratch, void* stream);

/* dL_dloss: 1 float (device).  Writes dL_dim [3,H,W] and dL_ddepth_sil [3,H,W]. */
int gsr_track_l1_bwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im,
                     const float* gt_depth, float sil_thres, float w_im, float w_depth, const float* dL_dloss,
                     float* dL_dim, float* dL_ddepth_sil, void* stream);

/* gsr_forward_dual_static with the tracking L1 loss (gsr_track_l1_fwd_bwd
 * semantics) formed in the render's per-pixel epilogue: the loss (1 float) and
 * its gradient images dL_dim [3,H,W] / dL_ddepth_sil [3,H,W] are written without
 * reading the rendered images back; dL_dloss (device scalar, the caller's static
 * loss seed) is read when the kernel runs.  scratch:
 * gsr_track_forward_scratch_floats(W, H) floats, zero-filled before first use, left
 * zero-filled.  The loss is valid iff the status reports no overflow. */
int gsr_track_forward_scratch_floats(int image_width, int image_height);
int gsr_track_forward_dual_static(const gsr_settings* settings, const gsr_gaussians* gaussians, const float* colors2,
                                  int capacity, unsigned* status, float* out_color, float* out_color2,
                                  float* out_depth, int* radii, const float* gt_im, const float* gt_depth,
                                  float sil_thres, float w_im, float w_depth, const float* dL_dloss, float* loss,
                                  float* dL_dim, float* dL_ddepth_sil, float* scratch, gsr_alloc_fn alloc,
                                  void* alloc_ctx, void* stream);

/* gsr_track_transform_fwd fused into gsr_track_forward_dual_static (SURVEY.md 8(f) row 3:
 * "transform-to-frame plus the [z,1,z^2] colours fused into preprocess"): the rasterizer's
 * preprocess forms each Gaussian's camera-frame rendervars from the world-frame map and the
 * frame's pose itself, so the transform is not a launch of its own and its outputs are not read
 * back.  Same results, bit for bit, as gsr_track_transform_fwd(xform -> gaussians->means3D,
 * ->rotations, colors2, ->opacities, ->scales) followed by gsr_track_forward_dual_static with
 * those arrays: here they are OUTPUTS (written by the forward, device [P,3] / [P,4] / [P,3] /
 * [P,1] / [P,3]) for the backward (gsr_track_backward_dual), unless store_rendervars is 0: then
 * nothing is written to them (storing them cost preprocess ~6 us at 300 k Gaussians) and the
 * backward recomputes the geometric ones from the world-frame map (its log_scales argument).  gaussians->colors_precomp: the
 * RGB colours [P,3] (input); shs and cov3D_precomp must be NULL. */
typedef struct gsr_track_xform {
    const float* means_world;  /* [P,3] */
    const float* unnorm_rot;   /* [P,4] */
    const float* logit_opac;   /* [P,1] */
    const float* log_scales;   /* [P,scale_cols] */
    int scale_cols;            /* 1 (isotropic, tiled to 3) or 3 */
    const float* cam_q;        /* the frame's quaternion, element k at cam_q[k * q_stride] */
    const float* cam_t;        /* the frame's translation, likewise */
    int q_stride;
    const float* w2c;          /* [4,4] row-major: depth colours */
    int store_rendervars;      /* 1: write the rendervars (outputs below); 0: do not -- the
                                  backward then recomputes them (gsr_track_backward_dual log_scales) */
    const uint8_t* alive;      /* (ABI 7) [P] or NULL: alive[i] == 0 culls Gaussian i like one behind the
                                  camera (radius 0, no instances, zero gradients) -- a capacity-padded map's
                                  free and pruned slots (splatam_amd.sequence) */
} gsr_track_xform;

int gsr_track_forward_dual_static_xf(const gsr_settings* settings, const gsr_gaussians* gaussians, float* colors2,
                                     const gsr_track_xform* xform, int capacity, unsigned* status, float* out_color,
                                     float* out_color2, float* out_depth, int* radii, const float* gt_im,
                                     const float* gt_depth, float sil_thres, float w_im, float w_depth,
                                     const float* dL_dloss, float* loss, float* dL_dim, float* dL_ddepth_sil,
                                     float* scratch, gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* Tracking backward with the pose chain fused into the rasterizer's per-Gaussian
 * backward: gsr_backward_dual's render backward (depth channel of the second
 * image, no opacity / colour sums), then one per-Gaussian kernel whose
 * dL/dmeans_cam, dL/d[z,1,z^2] and (anisotropic) dL/drotation feed the 16 pose
 * sums of gsr_track_transform_bwd directly -- no per-Gaussian gradient reaches
 * memory.  The last workgroup applies the pose chain and, with adam_state, the
 * Adam step in place (gsr_track_transform_bwd_adam semantics); without it the
 * pose gradient goes to dL_dcam_q / dL_dcam_t (stride q_stride).  settings,
 * gaussians (camera-frame rendervars), radii, colors2 ([z,1,z^2]) and the buffers
 * are those of the gsr_forward_dual(_static) call; means_world / unnorm_rot /
 * scale_cols / cam_q / cam_t / w2c those of gsr_track_transform_fwd.  scratch:
 * gsr_track_backward_scratch_floats(P) floats, zero-filled before first use,
 * left zero-filled.  The Adam step is skipped when the forward's own device
 * counters show an overflow of num_rendered (its capacity); `track` (may be
 * NULL) adds the best-candidate selection (its status / capacity are not used).
 * log_scales [P, scale_cols] (may be NULL): recompute each Gaussian's camera-frame mean, rotation
 * and scale from means_world / unnorm_rot / log_scales and the frame's (pre-step) pose instead of
 * reading gaussians->means3D / rotations / scales -- for a forward that did not store them
 * (gsr_track_forward_dual_static_xf with store_rendervars = 0); bitwise the same values. */
int gsr_track_backward_scratch_floats(int P);
int gsr_track_backward_dual(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                            const float* colors2, const float* dL_dout_color, const float* dL_dout_color2,
                            int num_rendered, const void* geom_buffer, const void* binning_buffer,
                            const void* image_buffer, const float* means_world, const float* unnorm_rot,
                            int scale_cols, float* cam_q, float* cam_t, int q_stride, const float* w2c, double lr_q,
                            double lr_t, double beta1, double beta2, double eps, float* adam_state,
                            float* dL_dcam_q, float* dL_dcam_t, float* scratch, const gsr_pose_track* track,
                            const float* log_scales, gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* The tracking iteration's render forward and render backward in ONE launch (render_track_kernel) --
 * what scripts/splatam.py:255-296 (get_loss(tracking=True)) + :722 (loss.backward()) run as
 * CudaRasterizer::Rasterizer::forward (rasterizer_impl.cu:198-339) and ::backward (:343-434) per
 * Renderer call:
 * gsr_track_forward_dual_static_xf's forward + L1 loss, then in the same workgroup the back-to-front
 * walk of gsr_track_backward_dual's render backward -- SplaTAM's tracking loss gradient is per pixel
 * (dL/dloss is the static seed dL_dloss), so a tile's backward needs nothing from other tiles and runs
 * from the pixel state still in registers.  inst_records: gsr_track_records_floats(capacity) floats
 * (device), receiving the per-instance sums gsr_track_backward_dual_records reads; they equal, bit for
 * bit, what gsr_track_backward_dual's render backward forms.  The gradient images are not formed.
 * out_color, out_color2 and out_depth all NULL: the rendered images are not stored either (the loss and
 * the backward consume them in registers; nor are the image buffer's final_T / n_contrib, so a render
 * backward from another loss seed cannot follow such a call). */
int gsr_track_records_floats(int capacity);

int gsr_track_forward_backward_dual_static_xf(const gsr_settings* settings, const gsr_gaussians* gaussians,
                                              float* colors2, const gsr_track_xform* xform, int capacity,
                                              unsigned* status, float* out_color, float* out_color2,
                                              float* out_depth, int* radii, const float* gt_im,
                                              const float* gt_depth, float sil_thres, float w_im, float w_depth,
                                              const float* dL_dloss, float* loss, float* scratch,
                                              float* inst_records, gsr_alloc_fn alloc, void* alloc_ctx,
                                              void* stream);
/* gsr_track_backward_dual after gsr_track_forward_backward_dual_static_xf: only the pose-fused
 * per-Gaussian backward (the render backward's records come from inst_records). */
int gsr_track_backward_dual_records(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                                    const float* colors2, int num_rendered, const void* geom_buffer,
                                    const void* binning_buffer, const void* image_buffer, const float* means_world,
                                    const float* unnorm_rot, int scale_cols, float* cam_q, float* cam_t, int q_stride,
                                    const float* w2c, double lr_q, double lr_t, double beta1, double beta2,
                                    double eps, float* adam_state, float* dL_dcam_q, float* dL_dcam_t,
                                    float* scratch, const gsr_pose_track* track, const float* log_scales,
                                    const float* inst_records, gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* ------------------------------------------------------------------ mapping --
 * get_loss(mapping=True, do_ba=False) (scripts/splatam.py:220-353) with the
 * Replica mapping config (configs/replica/splatam.py:82-103: use_l1,
 * use_sil_for_loss=False, ignore_outlier_depth_loss=False, weights im 0.5 /
 * depth 1.0), and the mapping optimizer (splatam.py:166-172).  Forward of the
 * transform is gsr_track_transform_fwd (identical outputs). */

/* Persistent zero-filled scratch (same contract as gsr_track_scratch_floats)
 * and the per-call state gsr_map_loss_fwd hands to gsr_map_loss_bwd. */
int gsr_map_loss_scratch_floats(int H, int W);
int gsr_map_loss_state_floats(int H, int W);

/* loss = w_im * (0.8 * mean|im - gt_im| + 0.2 * (1 - calc_ssim(im, gt_im)))
 *      + w_depth * mean over mask of |gt_depth - depth|,
 * mask = (gt_depth > 0) & !isnan(depth) & !isnan(depth_sq - depth^2)
 * (gs_helpers.py:18-19 l1_loss_v1, slam_external.py:66-97 calc_ssim with an
 * 11x11 sigma-1.5 window and zero padding).  im/gt_im/depth_sil [3,H,W],
 * gt_depth [1,H,W]; loss: 1 float (device); state: gsr_map_loss_state_floats. */
int gsr_map_loss_fwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im, const float* gt_depth,
                     float w_im, float w_depth, float* loss, float* state, float* scratch, void* stream);

/* Gradient of the loss above w.r.t. im [3,H,W] and depth_sil [3,H,W] (channels
 * 1, 2 written as zero), given dL_dloss (1 float, device) and the forward's state. */
int gsr_map_loss_bwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im, const float* gt_depth,
                     float w_im, float w_depth, const float* dL_dloss, const float* state, float* dL_dim,
                     float* dL_ddepth_sil, void* stream);

/* Backward of transform_to_frame(gaussians_grad=True, camera_grad=False) + the
 * rendervar builders: from the gradients of (means_cam, rotations, depth
 * colours, opacities, scales) [any but dL_dmeans_cam may be NULL] to the
 * gradients of means3D [P,3], unnorm_rotations [P,4], logit_opacities [P,1] and
 * log_scales [P,scale_cols] (outputs other than dL_dmeans may be NULL). */
int gsr_map_transform_bwd(int P, const float* unnorm_rot, const float* logit_opac, const float* log_scales,
                          int scale_cols, const float* cam_q, int q_stride, const float* means_cam, const float* w2c,
                          const float* dL_dmeans_cam, const float* dL_drot, const float* dL_ddepth_colors,
                          const float* dL_dopac, const float* dL_dscales, float* dL_dmeans, float* dL_dunnorm_rot,
                          float* dL_dlogit_opac, float* dL_dlog_scales, void* stream);

/* torch.optim.Adam state of the mapping optimizer for the five Gaussian
 * parameter tensors [means3D, unnorm_rotations, logit_opacities, log_scales,
 * colours (rgb_colors [P,3] or shs [P,M,3])]: exp_avg / exp_avg_sq of each
 * tensor's shape, per-tensor lr, and the optimizer step (>= 1, i.e. already
 * incremented) this update uses. */
typedef struct gsr_map_adam {
    float* exp_avg[5];
    float* exp_avg_sq[5];
    double lr[5];
    int step;
    double beta1, beta2, eps;
    /* optional: the counters of this iteration's static-mode forward and its binning capacity;
     * an overflow there (see gsr_pose_track) skips the step -- parameters and state unchanged.
     * Point it at the forward's own counters (geom_buffer + gsr_geom_counters_offset(P)); a
     * sticky status row would skip every later step once any earlier call overflowed.
     * gsr_backward_dual_sh_adam ignores it and guards on its own forward's counters. */
    const unsigned* status;
    unsigned capacity;
    /* optional device word, zero at the start of a frame (torch.optim.Adam's fresh state): a step
     * skipped because its forward overflowed sets it, and every later fused step (colour group,
     * transform backward) is skipped while it is set -- so the device never applies a step whose
     * bias corrections assume a step count the skipped one did not reach.  The caller re-runs the
     * frame from fresh state (splatam_amd.glue.MapAdam.reset) after reading it as non-zero. */
    unsigned* halted;
} gsr_map_adam;

/* gsr_backward_dual with the mapping optimizer's colour group (sh_adam->exp_avg[4] / exp_avg_sq[4] /
 * lr[4], step, betas, eps) applied to the SH coefficients gaussians->shs in place inside the
 * SH backward stage, instead of writing grads->dsh (which may be NULL) for
 * gsr_map_transform_bwd_adam to step: the 192-B-per-Gaussian gradient never makes the HBM round
 * trip.  Same element update (bitwise) as gsr_map_transform_bwd_adam's; call that one afterwards
 * with dL_dcolors = NULL.  Needs staged SH colours (M == (sh_degree+1)^2). */
int gsr_backward_dual_sh_adam(const gsr_settings* settings, const gsr_gaussians* gaussians, const int* radii,
                              const float* colors2, const float* dL_dout_color, const float* dL_dout_color2,
                              int num_rendered, const void* geom_buffer, const void* binning_buffer,
                              const void* image_buffer, const gsr_grads* grads, float* dcolors2, int dl2_channels,
                              const gsr_map_adam* sh_adam, gsr_alloc_fn alloc, void* alloc_ctx, void* stream);

/* gsr_map_transform_bwd with the optimizer step fused in: the parameters are
 * updated in place, no gradient is written.  dL_dcolors (the rasterizer's
 * gradient of the colour parameters, [P, color_cols]) steps `colors`; NULL
 * leaves them (and their state) untouched. */
int gsr_map_transform_bwd_adam(int P, float* means_world, float* unnorm_rot, float* logit_opac, float* log_scales,
                               int scale_cols, float* colors, int color_cols, const float* cam_q, int q_stride,
                               const float* means_cam, const float* w2c, const float* dL_dmeans_cam,
                               const float* dL_drot, const float* dL_ddepth_colors, const float* dL_dopac,
                               const float* dL_dscales, const float* dL_dcolors, const gsr_map_adam* adam,
                               void* stream);

/* SplaTAM's pruning inside a captured mapping frame (prune_gaussians, utils/slam_external.py:167-188, with
 * scripts/splatam.py:876-878 calling it between loss.backward() and optimizer.step()) without changing P:
 *   gsr_map_prune: alive[i] (uint8, 1 = kept) is cleared where the reference's remove_points would drop
 *     Gaussian i: sigmoid(logit_opac[i]) < opac_thr, or (remove_big) max_j exp(log_scales[i, j]) > big_thr
 *     (big_thr = 0.1 * scene_radius as the caller's float32 tensor holds it); each value formed as torch
 *     forms it (1 / (1 + exp(-x)), exp) so the decision is the reference's.  Already cleared entries stay.
 *   gsr_forward_dual_static_alive: gsr_forward_dual_static (include/gsr.h) where a Gaussian with
 *     alive[i] == 0 is culled like one behind the camera (radius 0, no instances, zero gradients); the
 *     others' images, binning order, gradients and optimizer steps are exactly those of the compacted
 *     set (the per-tile (depth, id) order of the survivors does not depend on the removed ids). */
int gsr_map_prune(int P, const float* logit_opac, const float* log_scales, int scale_cols, float opac_thr,
                  float big_thr, int remove_big, unsigned char* alive, void* stream);
int gsr_forward_dual_static_alive(const gsr_settings* settings, const gsr_gaussians* gaussians, const float* colors2,
                                  int capacity, unsigned* status, float* out_color, float* out_color2,
                                  float* out_depth, int* radii, const unsigned char* alive, gsr_alloc_fn alloc,
                                  void* alloc_ctx, void* stream);

/* The mapping iteration's transform fused into its forward (as
 * gsr_track_forward_dual_static_xf for tracking): gsr_track_transform_fwd(xform -> gaussians->means3D,
 * ->rotations, colors2, ->opacities, ->scales) followed by gsr_forward_dual_static_alive(..., xform->alive)
 * with those arrays, in one pass of preprocess -- the same results bit for bit, without the transform's
 * launch.  The five arrays are OUTPUTS (xform->store_rendervars must be 1: the mapping backward reads
 * them); gaussians->colors_precomp the RGB colours [P,3] (input); shs and cov3D_precomp must be NULL
 * (SH colours are evaluated ahead of preprocess, from the camera-frame means). */
int gsr_forward_dual_static_xf(const gsr_settings* settings, const gsr_gaussians* gaussians, float* colors2,
                               const gsr_track_xform* xform, int capacity, unsigned* status, float* out_color,
                               float* out_color2, float* out_depth, int* radii, gsr_alloc_fn alloc, void* alloc_ctx,
                               void* stream);

/* torch.optim.Adam (foreach implementation, no weight decay / amsgrad /
 * maximize) over up to 16 float32 tensors in one launch; every tensor shares
 * `step` (>= 1, already incremented) and has its own lr. */
typedef struct gsr_adam_tensor {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    long long n;
    double lr;
} gsr_adam_tensor;
int gsr_adam_step(int n_tensors, const gsr_adam_tensor* tensors, int step, double beta1, double beta2, double eps,
                  void* stream);

/* Fisher / EIG view scoring glue (scripts/ros_handler.py:847-902).
 * gsr_points_to_camera: pts [P,3] = the Gaussians' means [P,3] in a candidate camera frame,
 *     (rel_w2c @ [means, 1]^T)^T[:, :3] (ros_handler.py:863-866); w2c [4,4] row-major (device),
 *     each coordinate summed left to right without contraction.
 * gsr_fisher_accumulate: H [P,4] (16-byte aligned) += [dmeans3D [P,3], dopacity [P,1]] * (*weight)
 *     (weight: device scalar), product and sum each rounded -- torch's
 *     H.add_(torch.cat([pts.grad, opacities.grad], 1) * w) in one launch (the visited-pose sum of
 *     compute_H_visited_inv, ros_handler.py:807-829). */
int gsr_points_to_camera(int P, const float* means, const float* w2c, float* pts, void* stream);
int gsr_fisher_accumulate(int P, const float* dmeans3D, const float* dopacity, const float* weight, float* H,
                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_GLUE_H */
