// gsr_glue.hip -- SplaTAM's tracking-iteration glue as a few HIP kernels
// (include/gsr_glue.h).
//
//   track_transform_fwd   one lane per Gaussian: camera pose (F.normalize +
//                         build_rotation, slam_helpers.py:252-304 /
//                         slam_external.py:25-42) applied to the mean, the
//                         rendervar rotation / opacity / scale
//                         (slam_helpers.py:124-139) and the [z, 1, z^2] depth
//                         colours (slam_helpers.py:196-213) in one pass: 44 B in,
//                         64 B out per Gaussian (HBM-bound).
//   track_transform_bwd   one lane per Gaussian, grid-stride: the 16 pose
//                         partial sums (sum g, sum g p^T, sum dquat_mult^T dr)
//                         -> per-workgroup partials (transposed wave reduction +
//                         LDS); the last workgroup to finish sums them in a
//                         fixed order and applies the pose chain (R(n) -> n =
//                         c/|c| -> c = q/max(|q|, 1e-12)) and optionally Adam.
//                         One launch, bitwise reproducible.
//   track_l1              masked L1 tracking loss (splatam.py:262-296), same
//                         one-launch fixed-order sum; optionally its gradient
//                         w.r.t. both renders in the same pass;
//   track_l1_bwd          the gradient alone (any dL/dloss), one lane per pixel.
#include <math.h>

#include <algorithm>

#include "../../include/gsr.h"
#include "../../include/gsr_glue.h"
#include "gsr_glue_common.h"

namespace gsr {
namespace {

__global__ void __launch_bounds__(GLUE_BLOCK)
track_transform_fwd_kernel(int P, const float* __restrict__ mw, const float* __restrict__ ur,
                           const float* __restrict__ lo, const float* __restrict__ ls, int scols,
                           const float* __restrict__ cq, const float* __restrict__ ct, int qs,
                           const float* __restrict__ w2c, float* __restrict__ mc, float* __restrict__ rot,
                           float* __restrict__ dcol, float* __restrict__ opac, float* __restrict__ scl) {
    const int i = blockIdx.x * GLUE_BLOCK + threadIdx.x;
    if (i >= P) return;
    const Pose ps = make_pose(cq, ct, qs);
    TrackXf x;
    x.mw = mw; x.ur = ur; x.lo = lo; x.ls = ls; x.scols = scols; x.w2c = w2c;
    float m[3], c2[3], op, s[3];
    float4 q;
    track_xform_compute(x, ps, i, m, q, c2, op, s);
    track_xform_store(i, m, q, c2, op, s, mc, rot, dcol, opac, scl);
}

// Pose gradient in one launch: every workgroup publishes its partial of the 16
// sums (sum g, sum g p^T, sum dquat_mult^T dr); the last one to arrive adds the
// partials in a fixed order (bitwise reproducible) and runs pose_fin.
// scratch: 16 * gridDim.x partials, then the arrival counters (zero before the
// first launch; every launch leaves them zero).
__global__ void __launch_bounds__(GLUE_BLOCK)
track_transform_bwd_kernel(int P, const float* __restrict__ mw, const float* __restrict__ ur, int scols,
                           const float* __restrict__ cq, int qs, const float* __restrict__ mc,
                           const float* __restrict__ w2c, const float* __restrict__ gm,
                           const float* __restrict__ gr, const float* __restrict__ gd, float* __restrict__ part,
                           float* dq, float* dt, PoseAdam adam) {
    __shared__ float s_red[4 * POSE_PARTS];
    __shared__ float s_tot[POSE_PARTS];
    float v[POSE_PARTS];
#pragma unroll
    for (int k = 0; k < POSE_PARTS; k++) v[k] = 0.f;
    float c[4];
    if (scols != 1 && gr) {
        const Pose ps = make_pose(cq, nullptr, qs);  // only c is used
        for (int k = 0; k < 4; k++) c[k] = ps.c[k];
    }
    for (int i = blockIdx.x * GLUE_BLOCK + threadIdx.x; i < P; i += gridDim.x * GLUE_BLOCK) {
        const float g[3] = {gm[3 * i], gm[3 * i + 1], gm[3 * i + 2]};
        pose_partials(v, i, g, gd ? gd + 3 * i : nullptr, (scols != 1 && gr) ? gr + 4 * i : nullptr, mw, ur, mc, w2c,
                      c);
    }
    block_sum<POSE_PARTS>(v, s_red, s_tot);
    __syncthreads();
    if (threadIdx.x < POSE_PARTS) st_agent(part + POSE_PARTS * blockIdx.x + threadIdx.x, s_tot[threadIdx.x]);
    const int nb = gridDim.x;
    if (!last_block_arrive_grouped(reinterpret_cast<uint32_t*>(part + POSE_PARTS * nb))) return;
    // last workgroup: fixed-order sum of the partials
#pragma unroll
    for (int k = 0; k < POSE_PARTS; k++) v[k] = 0.f;
    gather_partials<POSE_PARTS, 2>(part, POSE_PARTS, nb, threadIdx.x, GLUE_BLOCK, v);
    __syncthreads();
    block_sum<POSE_PARTS>(v, s_red, s_tot);
    __syncthreads();
    if (threadIdx.x == 0) pose_fin(s_tot, cq, qs, dq, dt, adam);
}

// Masked L1 loss in one launch: per-workgroup partial sums published, the last
// workgroup adds them in a fixed order and writes the loss.  With dloss, the
// gradient images are written in the same pass (g = *dloss, read now: the
// caller's loss seed must already hold its value).  scratch: 4 * gridDim.x
// partials, then the arrival counter (zero before the first launch; left zero).
__global__ void __launch_bounds__(GLUE_BLOCK)
track_l1_kernel(int HW, const float* __restrict__ im, const float* __restrict__ ds,
                const float* __restrict__ gt_im, const float* __restrict__ gt_d, float thres, float w_im,
                float w_depth, float* __restrict__ part, float* __restrict__ loss, const float* __restrict__ dloss,
                float* __restrict__ dim, float* __restrict__ dds) {
    __shared__ float s_red[4 * 4];
    __shared__ float s_tot[4];
    const float g = dloss ? dloss[0] : 0.f;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int p = blockIdx.x * GLUE_BLOCK + threadIdx.x; p < HW; p += gridDim.x * GLUE_BLOCK) {
        const bool m = track_mask(p, HW, ds, gt_d, thres);
        if (m) {
            v[0] += fabsf(gt_im[p] - im[p]) + fabsf(gt_im[HW + p] - im[HW + p]) +
                    fabsf(gt_im[2 * HW + p] - im[2 * HW + p]);
            v[1] += fabsf(gt_d[p] - ds[p]);
        }
        if (dloss) {  // d|gt - x|/dx = -sgn(gt - x) (torch.abs backward: sgn, 0 at 0)
#pragma unroll
            for (int c = 0; c < 3; c++)
                dim[c * HW + p] = m ? (g * w_im) * neg_sgn(gt_im[c * HW + p] - im[c * HW + p]) : 0.f;
            dds[p] = m ? (g * w_depth) * neg_sgn(gt_d[p] - ds[p]) : 0.f;
            dds[HW + p] = 0.f;
            dds[2 * HW + p] = 0.f;
        }
    }
    block_sum<4>(v, s_red, s_tot);
    __syncthreads();
    if (threadIdx.x < 2) st_agent(part + 4 * blockIdx.x + threadIdx.x, s_tot[threadIdx.x]);
    const int nb = gridDim.x;
    if (!last_block_arrive_grouped(reinterpret_cast<uint32_t*>(part + 4 * nb))) return;
    v[0] = v[1] = v[2] = v[3] = 0.f;
    {
        float v2[2] = {0.f, 0.f};
        gather_partials<2, 4>(part, 4, nb, threadIdx.x, GLUE_BLOCK, v2);
        v[0] = v2[0];
        v[1] = v2[1];
    }
    __syncthreads();
    block_sum<4>(v, s_red, s_tot);
    __syncthreads();
    if (threadIdx.x == 0) loss[0] = w_im * s_tot[0] + w_depth * s_tot[1];
}

__global__ void __launch_bounds__(GLUE_BLOCK)
track_l1_bwd_kernel(int HW, const float* __restrict__ im, const float* __restrict__ ds,
                    const float* __restrict__ gt_im, const float* __restrict__ gt_d, float thres, float w_im,
                    float w_depth, const float* __restrict__ dloss, float* __restrict__ dim, float* __restrict__ dds) {
    const int p = blockIdx.x * GLUE_BLOCK + threadIdx.x;
    if (p >= HW) return;
    const float g = dloss[0];
    const bool m = track_mask(p, HW, ds, gt_d, thres);
    // d|gt - x|/dx = -sgn(gt - x) (torch.abs backward: sgn, 0 at 0)
#pragma unroll
    for (int c = 0; c < 3; c++) dim[c * HW + p] = m ? (g * w_im) * neg_sgn(gt_im[c * HW + p] - im[c * HW + p]) : 0.f;
    dds[p] = m ? (g * w_depth) * neg_sgn(gt_d[p] - ds[p]) : 0.f;
    dds[HW + p] = 0.f;
    dds[2 * HW + p] = 0.f;
}

// Fisher scoring glue (scripts/ros_handler.py:863-866, 884-889): the Gaussians' means moved into a
// candidate camera frame, and the visited-pose Hessian sum.
__global__ void __launch_bounds__(GLUE_BLOCK)
points_to_camera_kernel(int P, const float* __restrict__ means, const float* __restrict__ w2c, float* __restrict__ pts) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float m0 = means[3 * i], m1 = means[3 * i + 1], m2 = means[3 * i + 2];
#pragma unroll
    for (int r = 0; r < 3; r++)  // (rel_w2c @ [m, 1]^T)[r], left to right
        pts[3 * i + r] = ((w2c[4 * r] * m0 + w2c[4 * r + 1] * m1) + w2c[4 * r + 2] * m2) + w2c[4 * r + 3];
}
__global__ void __launch_bounds__(GLUE_BLOCK)
fisher_accumulate_kernel(int P, const float* __restrict__ dm, const float* __restrict__ dop, const float* __restrict__ w,
                         float* __restrict__ H) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float s = *w;
    float4 h = reinterpret_cast<float4*>(H)[i];
    h.x = h.x + dm[3 * i] * s;  // torch: H.add_(torch.cat([dm, dop], 1) * w), each op rounded
    h.y = h.y + dm[3 * i + 1] * s;
    h.z = h.z + dm[3 * i + 2] * s;
    h.w = h.w + dop[i] * s;
    reinterpret_cast<float4*>(H)[i] = h;
}

int blocks_for(int n) { return n <= 0 ? 1 : std::min(GLUE_MAX_BLOCKS, (n + GLUE_BLOCK - 1) / GLUE_BLOCK); }
// the pose reduction's last workgroup reads 16 partials per workgroup: fewer, fuller workgroups
constexpr int POSE_MAX_BLOCKS = 256;
int pose_blocks(int n) { return n <= 0 ? 1 : std::min(POSE_MAX_BLOCKS, (n + GLUE_BLOCK - 1) / GLUE_BLOCK); }

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

// partials of the widest reduction + the arrival counters (the L1 needs 4 per workgroup)
int gsr_track_scratch_floats(int n) { return POSE_PARTS * blocks_for(n) + ARRIVE_GROUPED_WORDS; }

int gsr_track_transform_fwd(int P, const float* means_world, const float* unnorm_rot, const float* logit_opac,
                            const float* log_scales, int scale_cols, const float* cam_q, const float* cam_t,
                            int q_stride, const float* w2c, float* means_cam, float* rotations, float* depth_colors,
                            float* opacities, float* scales, void* stream) {
    if (P < 0 || (scale_cols != 1 && scale_cols != 3) || q_stride < 1)
        return fail(GSR_ERR_INVALID_ARG, "track_transform_fwd: bad sizes");
    if (P == 0) return GSR_OK;
    if (!means_world || !unnorm_rot || !logit_opac || !log_scales || !cam_q || !cam_t || !w2c || !means_cam ||
        !rotations || !depth_colors || !opacities || !scales)
        return fail(GSR_ERR_INVALID_ARG, "track_transform_fwd: null pointer");
    hipLaunchKernelGGL(track_transform_fwd_kernel, dim3((P + GLUE_BLOCK - 1) / GLUE_BLOCK), dim3(GLUE_BLOCK), 0,
                       (hipStream_t)stream, P, means_world, unnorm_rot, logit_opac, log_scales, scale_cols, cam_q,
                       cam_t, q_stride, w2c, means_cam, rotations, depth_colors, opacities, scales);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "track_transform_fwd");
}

int gsr_track_transform_bwd(int P, const float* means_world, const float* unnorm_rot, int scale_cols,
                            const float* cam_q, const float* means_cam, const float* w2c,
                            const float* dL_dmeans_cam, const float* dL_drot, const float* dL_ddepth_colors,
                            float* dL_dcam_q, float* dL_dcam_t, int q_stride, float* scratch, void* stream) {
    if (P < 0 || (scale_cols != 1 && scale_cols != 3) || q_stride < 1)
        return fail(GSR_ERR_INVALID_ARG, "track_transform_bwd: bad sizes");
    if (!cam_q || !dL_dcam_q || !dL_dcam_t || !scratch || !w2c || (P > 0 && (!means_world || !means_cam ||
                                                                        !dL_dmeans_cam || !unnorm_rot)))
        return fail(GSR_ERR_INVALID_ARG, "track_transform_bwd: null pointer");
    hipLaunchKernelGGL(track_transform_bwd_kernel, dim3(pose_blocks(P)), dim3(GLUE_BLOCK), 0, (hipStream_t)stream, P,
                       means_world, unnorm_rot, scale_cols, cam_q, q_stride, means_cam, w2c, dL_dmeans_cam, dL_drot,
                       dL_ddepth_colors, scratch, dL_dcam_q, dL_dcam_t,
                       PoseAdam{0.0, 0.0, 0.0, 0.0, 0.f, 0.f, 0.f, nullptr, nullptr, nullptr});
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "track_transform_bwd");
}

int gsr_track_transform_bwd_adam(int P, const float* means_world, const float* unnorm_rot, int scale_cols,
                                 float* cam_q, float* cam_t, int q_stride, const float* means_cam, const float* w2c,
                                 const float* dL_dmeans_cam, const float* dL_drot, const float* dL_ddepth_colors,
                                 double lr_q, double lr_t, double beta1, double beta2, double eps, float* adam_state,
                                 float* scratch, const gsr_pose_track* track, void* stream) {
    if (P < 0 || (scale_cols != 1 && scale_cols != 3) || q_stride < 1)
        return fail(GSR_ERR_INVALID_ARG, "track_transform_bwd_adam: bad sizes");
    if (!cam_q || !cam_t || !adam_state || !scratch || !w2c ||
        (P > 0 && (!means_world || !means_cam || !dL_dmeans_cam || !unnorm_rot)))
        return fail(GSR_ERR_INVALID_ARG, "track_transform_bwd_adam: null pointer");
    hipLaunchKernelGGL(track_transform_bwd_kernel, dim3(pose_blocks(P)), dim3(GLUE_BLOCK), 0, (hipStream_t)stream, P,
                       means_world, unnorm_rot, scale_cols, cam_q, q_stride, means_cam, w2c, dL_dmeans_cam, dL_drot,
                       dL_ddepth_colors, scratch, nullptr, nullptr,
                       PoseAdam{lr_q, lr_t, beta1, beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps,
                                adam_state, cam_q, cam_t, track ? track->status : nullptr,
                                track ? track->capacity : 0u, track ? track->loss : nullptr,
                                track ? track->best : nullptr});
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "track_transform_bwd_adam");
}

int gsr_track_l1_fwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im,
                     const float* gt_depth, float sil_thres, float w_im, float w_depth, float* loss, float* scratch,
                     void* stream) {
    if (H <= 0 || W <= 0) return fail(GSR_ERR_INVALID_ARG, "track_l1_fwd: bad image size");
    if (!im || !depth_sil || !gt_im || !gt_depth || !loss || !scratch)
        return fail(GSR_ERR_INVALID_ARG, "track_l1_fwd: null pointer");
    const int HW = H * W;
    hipLaunchKernelGGL(track_l1_kernel, dim3(blocks_for(HW)), dim3(GLUE_BLOCK), 0, (hipStream_t)stream, HW, im,
                       depth_sil, gt_im, gt_depth, sil_thres, w_im, w_depth, scratch, loss, nullptr, nullptr, nullptr);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "track_l1_fwd");
}

int gsr_track_l1_fwd_bwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im,
                         const float* gt_depth, float sil_thres, float w_im, float w_depth, const float* dL_dloss,
                         float* loss, float* dL_dim, float* dL_ddepth_sil, float* scratch, void* stream) {
    if (H <= 0 || W <= 0) return fail(GSR_ERR_INVALID_ARG, "track_l1_fwd_bwd: bad image size");
    if (!im || !depth_sil || !gt_im || !gt_depth || !loss || !scratch || !dL_dloss || !dL_dim || !dL_ddepth_sil)
        return fail(GSR_ERR_INVALID_ARG, "track_l1_fwd_bwd: null pointer");
    const int HW = H * W;
    hipLaunchKernelGGL(track_l1_kernel, dim3(blocks_for(HW)), dim3(GLUE_BLOCK), 0, (hipStream_t)stream, HW, im,
                       depth_sil, gt_im, gt_depth, sil_thres, w_im, w_depth, scratch, loss, dL_dloss, dL_dim,
                       dL_ddepth_sil);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "track_l1_fwd_bwd");
}

int gsr_track_l1_bwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im,
                     const float* gt_depth, float sil_thres, float w_im, float w_depth, const float* dL_dloss,
                     float* dL_dim, float* dL_ddepth_sil, void* stream) {
    if (H <= 0 || W <= 0) return fail(GSR_ERR_INVALID_ARG, "track_l1_bwd: bad image size");
    if (!im || !depth_sil || !gt_im || !gt_depth || !dL_dloss || !dL_dim || !dL_ddepth_sil)
        return fail(GSR_ERR_INVALID_ARG, "track_l1_bwd: null pointer");
    const int HW = H * W;
    hipLaunchKernelGGL(track_l1_bwd_kernel, dim3((HW + GLUE_BLOCK - 1) / GLUE_BLOCK), dim3(GLUE_BLOCK), 0,
                       (hipStream_t)stream, HW, im, depth_sil, gt_im, gt_depth, sil_thres, w_im, w_depth, dL_dloss,
                       dL_dim, dL_ddepth_sil);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "track_l1_bwd");
}

int gsr_points_to_camera(int P, const float* means, const float* w2c, float* pts, void* stream) {
    if (P < 0) return fail(GSR_ERR_INVALID_ARG, "points_to_camera: bad size");
    if (P == 0) return GSR_OK;
    if (!means || !w2c || !pts) return fail(GSR_ERR_INVALID_ARG, "points_to_camera: null pointer");
    hipLaunchKernelGGL(points_to_camera_kernel, dim3((P + GLUE_BLOCK - 1) / GLUE_BLOCK), dim3(GLUE_BLOCK), 0,
                       (hipStream_t)stream, P, means, w2c, pts);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "points_to_camera");
}

int gsr_fisher_accumulate(int P, const float* dmeans3D, const float* dopacity, const float* weight, float* H,
                          void* stream) {
    if (P < 0) return fail(GSR_ERR_INVALID_ARG, "fisher_accumulate: bad size");
    if (P == 0) return GSR_OK;
    if (!dmeans3D || !dopacity || !weight || !H) return fail(GSR_ERR_INVALID_ARG, "fisher_accumulate: null pointer");
    if (((uintptr_t)H & 15u) != 0) return fail(GSR_ERR_INVALID_ARG, "fisher_accumulate: H must be 16-byte aligned");
    hipLaunchKernelGGL(fisher_accumulate_kernel, dim3((P + GLUE_BLOCK - 1) / GLUE_BLOCK), dim3(GLUE_BLOCK), 0,
                       (hipStream_t)stream, P, dmeans3D, dopacity, weight, H);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "fisher_accumulate");
}

}  // extern "C"
