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
    const float p0 = mw[3 * i], p1 = mw[3 * i + 1], p2 = mw[3 * i + 2];
    float m[3];
#pragma unroll
    for (int r = 0; r < 3; r++) m[r] = ps.R[r][0] * p0 + ps.R[r][1] * p1 + ps.R[r][2] * p2 + ps.t[r];
    mc[3 * i] = m[0]; mc[3 * i + 1] = m[1]; mc[3 * i + 2] = m[2];
    float un_norm;
    float4 q = normalize4(load4(ur + 4 * i), un_norm);          // F.normalize(unnorm_rotations)
    if (scols != 1) {                                          // anisotropic: compose with the camera
        float o_norm;
        q = normalize4(quat_mult(ps.c, q), o_norm);
    }
    rot[4 * i] = q.x; rot[4 * i + 1] = q.y; rot[4 * i + 2] = q.z; rot[4 * i + 3] = q.w;
    const float z = w2c[8] * m[0] + w2c[9] * m[1] + w2c[10] * m[2] + w2c[11];
    dcol[3 * i] = z; dcol[3 * i + 1] = 1.f; dcol[3 * i + 2] = z * z;
    opac[i] = 1.f / (1.f + expf(-lo[i]));
#pragma unroll
    for (int k = 0; k < 3; k++) scl[3 * i + k] = expf(ls[scols == 1 ? i : 3 * i + k]);
}

struct PoseAdam {  // torch.optim.Adam (no weight decay, no amsgrad) on the frame's pose column
    double lr_q, lr_t, beta1, beta2;   // torch's hyperparameters are python floats (double)
    float w1, omb2, eps;               // 1 - beta1, 1 - beta2 rounded from double, like torch's scalars
    float* state;     // device: m_q[4], v_q[4], m_t[3], v_t[3], step
    float* q;         // the frame's quaternion column (stride qs), updated in place
    float* t;         // the frame's translation column (stride qs)
};

// torch/optim/adam.py (foreach form): exp_avg.lerp_(g, 1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2);
// p.addcdiv_(exp_avg, sqrt(exp_avg_sq) / sqrt(1 - b2^s) + eps, -lr / (1 - b1^s)), the scalars
// formed in double like torch's python floats.
__device__ __forceinline__ void adam_update(float& p, float g, float& m, float& v, float neg_step, const PoseAdam& a,
                                            float bc2_sqrt) {
    m = m + a.w1 * (g - m);                      // exp_avg.lerp_(g, 1 - beta1)
    v = v * (float)a.beta2;                      // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
    v = v + a.omb2 * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + a.eps;
    p = p + neg_step * (m / denom);
}

// The pose chain on the 16 summed terms S: dR -> dn (build_rotation) -> dc
// (its own normalisation) -> dq (F.normalize), dt = S[0..2]; then either the
// gradient is written (dq, dt) or the Adam step is applied in place.
__device__ void pose_fin(const float* S, const float* cq, int qs, float* dq, float* dt, const PoseAdam& adam) {
    const Pose ps = make_pose(cq, nullptr, qs);
    // dR[j][k] = S[3 + 3j + k]; R = build_rotation(n), n = (r, x, y, z)
    const float r = ps.n[0], x = ps.n[1], y = ps.n[2], z = ps.n[3];
    const float d00 = S[3], d01 = S[4], d02 = S[5], d10 = S[6], d11 = S[7], d12 = S[8], d20 = S[9], d21 = S[10],
                d22 = S[11];
    const float4 dn = make_float4(
        2.f * (-z * d01 + y * d02 + z * d10 - x * d12 - y * d20 + x * d21),
        2.f * (y * d01 + z * d02 + y * d10 - 2.f * x * d11 - r * d12 + z * d20 + r * d21 - 2.f * x * d22),
        2.f * (-2.f * y * d00 + x * d01 + r * d02 + x * d10 + z * d12 - r * d20 + z * d21 - 2.f * y * d22),
        2.f * (-2.f * z * d00 - r * d01 + x * d02 + r * d10 - 2.f * z * d11 + y * d12 + x * d20 + y * d21));
    // n = c / |c| (build_rotation, no eps), then c = q / max(|q|, eps) (F.normalize)
    float4 dc = normalize4_bwd(make_float4(ps.n[0], ps.n[1], ps.n[2], ps.n[3]), ps.cn, dn);
    dc.x += S[12]; dc.y += S[13]; dc.z += S[14]; dc.w += S[15];
    const float4 g = normalize4_bwd(make_float4(ps.c[0], ps.c[1], ps.c[2], ps.c[3]), ps.qn, dc);
    if (adam.state) {  // optimizer step fused here: the pose gradient never leaves the kernel
        float* st = adam.state;
        const float step = st[14] + 1.f;
        st[14] = step;
        const double bc1 = 1.0 - pow(adam.beta1, (double)step);
        const float bc2_sqrt = (float)sqrt(1.0 - pow(adam.beta2, (double)step));
        const float ss_q = (float)(-adam.lr_q / bc1), ss_t = (float)(-adam.lr_t / bc1);
        const float gq[4] = {g.x, g.y, g.z, g.w};
        for (int k = 0; k < 4; k++) adam_update(adam.q[k * qs], gq[k], st[k], st[4 + k], ss_q, adam, bc2_sqrt);
        for (int k = 0; k < 3; k++) adam_update(adam.t[k * qs], S[k], st[8 + k], st[11 + k], ss_t, adam, bc2_sqrt);
        return;
    }
    dq[0] = g.x; dq[qs] = g.y; dq[2 * qs] = g.z; dq[3 * qs] = g.w;
    dt[0] = S[0]; dt[qs] = S[1]; dt[2 * qs] = S[2];
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
    const float wz0 = w2c[8], wz1 = w2c[9], wz2 = w2c[10];
    for (int i = blockIdx.x * GLUE_BLOCK + threadIdx.x; i < P; i += gridDim.x * GLUE_BLOCK) {
        float g0 = gm[3 * i], g1 = gm[3 * i + 1], g2 = gm[3 * i + 2];
        if (gd) {  // colours [z, 1, z^2]: dz = dc0 + 2 z dc2, z = w2c[2,:3] . m + w2c[2,3]
            const float z = wz0 * mc[3 * i] + wz1 * mc[3 * i + 1] + wz2 * mc[3 * i + 2] + w2c[11];
            const float dz = gd[3 * i] + 2.f * z * gd[3 * i + 2];
            g0 += dz * wz0; g1 += dz * wz1; g2 += dz * wz2;
        }
        const float p0 = mw[3 * i], p1 = mw[3 * i + 1], p2 = mw[3 * i + 2];
        v[0] += g0; v[1] += g1; v[2] += g2;
        v[3] += g0 * p0; v[4] += g0 * p1; v[5] += g0 * p2;
        v[6] += g1 * p0; v[7] += g1 * p1; v[8] += g1 * p2;
        v[9] += g2 * p0; v[10] += g2 * p1; v[11] += g2 * p2;
        if (scols != 1 && gr) {
            // rot = normalize(o), o = quat_mult(c, u), u = normalize(unnorm)
            float un_norm, o_norm;
            const float4 u = normalize4(load4(ur + 4 * i), un_norm);
            const float4 o = quat_mult(c, u);
            const float4 r = normalize4(o, o_norm);
            const float4 d = normalize4_bwd(r, o_norm, load4(gr + 4 * i));
            v[12] += d.x * u.x + d.y * u.y + d.z * u.z + d.w * u.w;
            v[13] += -d.x * u.y + d.y * u.x - d.z * u.w + d.w * u.z;
            v[14] += -d.x * u.z + d.y * u.w + d.z * u.x - d.w * u.y;
            v[15] += -d.x * u.w - d.y * u.z + d.z * u.y + d.w * u.x;
        }
    }
    block_sum<POSE_PARTS>(v, s_red, s_tot);
    __syncthreads();
    if (threadIdx.x < POSE_PARTS) st_agent(part + POSE_PARTS * blockIdx.x + threadIdx.x, s_tot[threadIdx.x]);
    const int nb = gridDim.x;
    if (!last_block_arrive_grouped(reinterpret_cast<uint32_t*>(part + POSE_PARTS * nb))) return;
    // last workgroup: fixed-order sum of the partials
#pragma unroll
    for (int k = 0; k < POSE_PARTS; k++) v[k] = 0.f;
    for (int b = threadIdx.x; b < nb; b += GLUE_BLOCK)
#pragma unroll
        for (int k = 0; k < POSE_PARTS; k++) v[k] += ld_agent(part + POSE_PARTS * b + k);
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
    for (int b = threadIdx.x; b < nb; b += GLUE_BLOCK) {
        v[0] += ld_agent(part + 4 * b);
        v[1] += ld_agent(part + 4 * b + 1);
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
                                 float* scratch, void* stream) {
    if (P < 0 || (scale_cols != 1 && scale_cols != 3) || q_stride < 1)
        return fail(GSR_ERR_INVALID_ARG, "track_transform_bwd_adam: bad sizes");
    if (!cam_q || !cam_t || !adam_state || !scratch || !w2c ||
        (P > 0 && (!means_world || !means_cam || !dL_dmeans_cam || !unnorm_rot)))
        return fail(GSR_ERR_INVALID_ARG, "track_transform_bwd_adam: null pointer");
    hipLaunchKernelGGL(track_transform_bwd_kernel, dim3(pose_blocks(P)), dim3(GLUE_BLOCK), 0, (hipStream_t)stream, P,
                       means_world, unnorm_rot, scale_cols, cam_q, q_stride, means_cam, w2c, dL_dmeans_cam, dL_drot,
                       dL_ddepth_colors, scratch, nullptr, nullptr,
                       PoseAdam{lr_q, lr_t, beta1, beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps,
                                adam_state, cam_q, cam_t});
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

}  // extern "C"
