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
 * q_stride.  adam_state: device, 15 floats [m_q 4, v_q 4, m_t 3, v_t 3, step],
 * zero-initialised by the caller per frame (SplaTAM re-creates the optimizer per
 * frame). */
int gsr_track_transform_bwd_adam(int P, const float* means_world, const float* unnorm_rot, int scale_cols,
                                 float* cam_q, float* cam_t, int q_stride, const float* means_cam,
                                 const float* w2c, const float* dL_dmeans_cam, const float* dL_drot,
                                 const float* dL_ddepth_colors, float lr_q, float lr_t, float beta1,
                                 float beta2, float eps, float* adam_state, float* scratch, void* stream);

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

#ifdef __cplusplus
}
#endif
#endif /* GSR_GLUE_H */
