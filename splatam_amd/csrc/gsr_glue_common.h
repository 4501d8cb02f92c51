// gsr_glue_common.h -- device helpers shared by the SplaTAM glue kernels
// (gsr_glue.hip: tracking, gsr_mapping.hip: mapping): camera pose / quaternion
// algebra of utils/slam_helpers.py + utils/slam_external.py, fixed-order
// workgroup sums, the L1 loss sign convention.
#pragma once
#include <math.h>

#include "gsr_common.h"

namespace gsr {
namespace {

constexpr int GLUE_BLOCK = 256;
constexpr int GLUE_MAX_BLOCKS = 1024;
constexpr int POSE_PARTS = 16;  // g (3), g p^T (9), dcam_rot via quat_mult (4)
constexpr float kNormEps = 1e-12f;  // F.normalize default eps

struct Pose {
    float c[4];    // F.normalize(q)
    float n[4];    // build_rotation's own normalisation of c
    float R[3][3];
    float t[3];
    float qn;      // |q|
    float cn;      // |c|
};

__device__ __forceinline__ Pose make_pose(const float* q, const float* t, int stride) {
    Pose p;
    const float q0 = q[0], q1 = q[stride], q2 = q[2 * stride], q3 = q[3 * stride];
    p.qn = sqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
    const float d = fmaxf(p.qn, kNormEps);
    p.c[0] = q0 / d; p.c[1] = q1 / d; p.c[2] = q2 / d; p.c[3] = q3 / d;
    p.cn = sqrtf(p.c[0] * p.c[0] + p.c[1] * p.c[1] + p.c[2] * p.c[2] + p.c[3] * p.c[3]);
    for (int k = 0; k < 4; k++) p.n[k] = p.c[k] / p.cn;
    const float r = p.n[0], x = p.n[1], y = p.n[2], z = p.n[3];
    p.R[0][0] = 1.f - 2.f * (y * y + z * z); p.R[0][1] = 2.f * (x * y - r * z); p.R[0][2] = 2.f * (x * z + r * y);
    p.R[1][0] = 2.f * (x * y + r * z); p.R[1][1] = 1.f - 2.f * (x * x + z * z); p.R[1][2] = 2.f * (y * z - r * x);
    p.R[2][0] = 2.f * (x * z - r * y); p.R[2][1] = 2.f * (y * z + r * x); p.R[2][2] = 1.f - 2.f * (x * x + y * y);
    p.t[0] = t ? t[0] : 0.f; p.t[1] = t ? t[stride] : 0.f; p.t[2] = t ? t[2 * stride] : 0.f;
    return p;
}

// quat_mult(a, b) (slam_helpers.py), (w, x, y, z)
__device__ __forceinline__ float4 quat_mult(const float a[4], float4 b) {
    return make_float4(a[0] * b.x - a[1] * b.y - a[2] * b.z - a[3] * b.w,
                       a[0] * b.y + a[1] * b.x + a[2] * b.w - a[3] * b.z,
                       a[0] * b.z - a[1] * b.w + a[2] * b.x + a[3] * b.y,
                       a[0] * b.w + a[1] * b.z - a[2] * b.y + a[3] * b.x);
}

__device__ __forceinline__ float4 normalize4(float4 v, float& norm) {
    norm = sqrtf(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w);
    const float d = fmaxf(norm, kNormEps);
    return make_float4(v.x / d, v.y / d, v.z / d, v.w / d);
}

// backward of y = x / max(|x|, eps) given y, |x| and dy
__device__ __forceinline__ float4 normalize4_bwd(float4 y, float norm, float4 dy) {
    if (norm <= kNormEps) return make_float4(dy.x / kNormEps, dy.y / kNormEps, dy.z / kNormEps, dy.w / kNormEps);
    const float dot = y.x * dy.x + y.y * dy.y + y.z * dy.z + y.w * dy.w;
    return make_float4((dy.x - y.x * dot) / norm, (dy.y - y.y * dot) / norm, (dy.z - y.z * dot) / norm,
                       (dy.w - y.w * dot) / norm);
}

__device__ __forceinline__ float4 load4(const float* p) { return make_float4(p[0], p[1], p[2], p[3]); }

// Sums `v` over the workgroup (4 waves) into out[0..N) in a fixed order.
template <int N>
__device__ __forceinline__ void block_sum(const float (&v)[N], float* s_red /*4*N*/, float* out) {
    float r[N / 4];
    wave_reduce_n<N>(v, r);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, row = lane >> 4;
    if ((lane & 15) == 0)
#pragma unroll
        for (int m = 0; m < N / 4; m++) s_red[w * N + row * (N / 4) + m] = r[m];
    __syncthreads();
    if (threadIdx.x < N) out[threadIdx.x] = (s_red[threadIdx.x] + s_red[N + threadIdx.x]) +
                                            (s_red[2 * N + threadIdx.x] + s_red[3 * N + threadIdx.x]);
}

// --------------------------------------------------------------- L1 loss --
__device__ __forceinline__ bool track_mask(int pid, int HW, const float* ds, const float* gt_depth, float thres) {
    const float d = ds[pid], sil = ds[HW + pid], dsq = ds[2 * HW + pid];
    const float unc = dsq - d * d;
    return gt_depth[pid] > 0.f && !isnan(d) && !isnan(unc) && sil > thres;
}

__device__ __forceinline__ float neg_sgn(float x) { return x > 0.f ? -1.f : (x < 0.f ? 1.f : 0.f); }

}  // namespace
}  // namespace gsr
