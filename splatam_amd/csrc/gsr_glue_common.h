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
// (explicit FMAs, contraction off here and in normalize4: the same bits in every kernel that inlines them)
__device__ __forceinline__ float4 quat_mult(const float a[4], float4 b) {
#pragma clang fp contract(off)
    // explicit fused multiply-adds (fixed, not left to the contraction of the caller's context)
    return make_float4(__builtin_fmaf(-a[3], b.w, __builtin_fmaf(-a[2], b.z, __builtin_fmaf(-a[1], b.y, a[0] * b.x))),
                       __builtin_fmaf(-a[3], b.z, __builtin_fmaf(a[2], b.w, __builtin_fmaf(a[1], b.x, a[0] * b.y))),
                       __builtin_fmaf(a[3], b.y, __builtin_fmaf(a[2], b.x, __builtin_fmaf(-a[1], b.w, a[0] * b.z))),
                       __builtin_fmaf(a[3], b.x, __builtin_fmaf(-a[2], b.y, __builtin_fmaf(a[1], b.z, a[0] * b.w))));
}

__device__ __forceinline__ float4 normalize4(float4 v, float& norm) {
#pragma clang fp contract(off)
    norm = sqrtf(__builtin_fmaf(v.w, v.w, __builtin_fmaf(v.z, v.z, __builtin_fmaf(v.y, v.y, v.x * v.x))));
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

// One Gaussian of transform_to_frame + the rendervar builders (slam_helpers.py:124-139,196-213,
// 252-304): camera-frame mean m, rendervar rotation q, depth colours c2 = [z, 1, z^2], opacity op,
// scales s.  Shared by track_transform_fwd_kernel and the transform-fused preprocess (same code,
// same bits).  Loads only: the stores (track_xform_store) go after every other global load of the
// calling kernel -- a load issued after a store waits for the store's completion too (vmcnt
// counts both on gfx950), which serialised ~5 store round trips in preprocess (6 us).
// The geometric part (mean, rotation, scale) alone: also what the tracking backward recomputes
// (PoseFuse::ls) instead of reading stored rendervars -- the same expressions, so the same bits.
// The transform's per-Gaussian inputs, loaded ahead of the arithmetic (the transform-fused
// preprocess issues them before its pose barrier, overlapping the pose's own loads).
struct XfRaw {
    float p[3];
    float4 ur;
    float ls[3];
    float lo;
};
__device__ __forceinline__ XfRaw track_xform_load(const TrackXf& x, int i, bool with_opacity) {
    XfRaw r;
    r.p[0] = x.mw[3 * i]; r.p[1] = x.mw[3 * i + 1]; r.p[2] = x.mw[3 * i + 2];
    r.ur = load4(x.ur + 4 * i);
#pragma unroll
    for (int k = 0; k < 3; k++) r.ls[k] = x.ls[x.scols == 1 ? i : 3 * i + k];
    r.lo = with_opacity ? x.lo[i] : 0.f;
    return r;
}
__device__ __forceinline__ void track_xform_geom_raw(const XfRaw& r, int scols, const Pose& ps, float (&m)[3],
                                                     float4& q, float (&s)[3]) {
    // explicit fused multiply-adds, contraction off otherwise: the same bits in every kernel that
    // inlines this (the forward's transform, the transform-fused preprocess, the backward's
    // recomputation), whatever the surrounding code
#pragma clang fp contract(off)
#pragma unroll
    for (int k = 0; k < 3; k++)
        m[k] = __builtin_fmaf(ps.R[k][2], r.p[2], __builtin_fmaf(ps.R[k][1], r.p[1], __builtin_fmaf(ps.R[k][0], r.p[0], ps.t[k])));
    float un_norm;
    q = normalize4(r.ur, un_norm);                               // F.normalize(unnorm_rotations)
    if (scols != 1) {                                            // anisotropic: compose with the camera
        float o_norm;
        q = normalize4(quat_mult(ps.c, q), o_norm);
    }
#pragma unroll
    for (int k = 0; k < 3; k++) s[k] = expf(r.ls[k]);
}
__device__ __forceinline__ void track_xform_geom(const TrackXf& x, const Pose& ps, int i, float (&m)[3], float4& q,
                                                 float (&s)[3]) {
    track_xform_geom_raw(track_xform_load(x, i, false), x.scols, ps, m, q, s);
}
__device__ __forceinline__ void track_xform_compute_raw(const TrackXf& x, const XfRaw& r, const Pose& ps,
                                                        float (&m)[3], float4& q, float (&c2)[3], float& op,
                                                        float (&s)[3]) {
#pragma clang fp contract(off)
    track_xform_geom_raw(r, x.scols, ps, m, q, s);
    const float z = __builtin_fmaf(x.w2c[10], m[2], __builtin_fmaf(x.w2c[9], m[1], __builtin_fmaf(x.w2c[8], m[0], x.w2c[11])));
    c2[0] = z; c2[1] = 1.f; c2[2] = z * z;
    op = 1.f / (1.f + expf(-r.lo));
}
__device__ __forceinline__ void track_xform_compute(const TrackXf& x, const Pose& ps, int i, float (&m)[3],
                                                    float4& q, float (&c2)[3], float& op, float (&s)[3]) {
    track_xform_compute_raw(x, track_xform_load(x, i, true), ps, m, q, c2, op, s);
}
__device__ __forceinline__ void track_xform_store(int i, const float (&m)[3], float4 q, const float (&c2)[3], float op,
                                                  const float (&s)[3], float* mc, float* rot, float* dcol,
                                                  float* opac, float* scl) {
#ifndef GSR_XF_NOSTORE
    mc[3 * i] = m[0]; mc[3 * i + 1] = m[1]; mc[3 * i + 2] = m[2];
    rot[4 * i] = q.x; rot[4 * i + 1] = q.y; rot[4 * i + 2] = q.z; rot[4 * i + 3] = q.w;
    dcol[3 * i] = c2[0]; dcol[3 * i + 1] = c2[1]; dcol[3 * i + 2] = c2[2];
    opac[i] = op;
#pragma unroll
    for (int k = 0; k < 3; k++) scl[3 * i + k] = s[k];
#endif
}

// Forward-state check of the fused optimizer steps: `st` is a forward's device counters or
// its static-mode status row ([0] num_rendered, [1] prefiltered violation, [2] longest tile
// list, [3] longest list the tile sort handled); the forward's outputs (and so the gradients)
// are invalid when it overflowed its binning capacity `cap`.  st == nullptr: no check.
__device__ __forceinline__ bool forward_overflowed(const uint32_t* st, uint32_t cap) {
    return st && (st[0] > cap || st[2] > st[3] || st[1] != 0u);
}
// The fused mapping steps' skip decision: the forward overflowed, or an earlier step of the frame
// was skipped (`halted`, gsr_map_adam.halted: sticky until the caller resets the optimizer).  A skip
// caused by an overflow sets `halted` (a plain vector store from one lane per workgroup; every
// workgroup of a launch takes the same decision from the same counters).
__device__ __forceinline__ bool fused_step_skipped(const uint32_t* st, uint32_t cap, uint32_t* halted) {
    if (halted && *reinterpret_cast<volatile uint32_t*>(halted) != 0u) return true;
    if (!forward_overflowed(st, cap)) return false;
    if (halted && threadIdx.x == 0) *halted = 1u;
    return true;
}

struct PoseAdam {  // torch.optim.Adam (no weight decay, no amsgrad) on the frame's pose column
    double lr_q, lr_t, beta1, beta2;   // torch's hyperparameters are python floats (double)
    float w1, omb2, eps;               // 1 - beta1, 1 - beta2 rounded from double, like torch's scalars
    float* state;     // device: m_q[4], v_q[4], m_t[3], v_t[3], step
    float* q;         // the frame's quaternion column (stride qs), updated in place
    float* t;         // the frame's translation column (stride qs)
    const uint32_t* guard = nullptr;  // forward counters / status row: skip the step on an overflow
    uint32_t cap = 0;
    const float* loss = nullptr;      // this iteration's loss (best-candidate selection), or nullptr
    float* best = nullptr;            // [min loss, q 4, t 3]
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

// beta^n for the Adam bias corrections, formed in double like torch's python floats: by
// squaring (n = the step count, an integer; within a few double ulps of pow(), so the float
// scalars derived from it are the same) -- 1 us faster than the device pow() on the one thread
// that runs the pose step (GSR_POW_INT=0: pow())
#ifndef GSR_POW_INT
#define GSR_POW_INT 1
#endif
__device__ __forceinline__ double adam_pow(double b, float step) {
#if GSR_POW_INT
    double r = 1.0;
    for (unsigned n = (unsigned)step; n; n >>= 1) {
        if (n & 1u) r *= b;
        b *= b;
    }
    return r;
#else
    return pow(b, (double)step);
#endif
}

// The pose chain on the 16 summed terms S: dR -> dn (build_rotation) -> dc
// (its own normalisation) -> dq (F.normalize), dt = S[0..2]; then either the
// gradient is written (dq, dt) or the Adam step is applied in place.
// Runs in one thread at the end of a launch, so every input (pose, optimizer state, guard
// counters, loss, best candidate) is loaded up front in one memory round trip, and every
// result stored at the end: element-wise updates through possibly aliasing pointers had
// serialised ~6 dependent round trips (~5 us of the fused pose backward).
__device__ void pose_fin(const float* S, const float* cq, int qs, float* dq, float* dt, const PoseAdam& adam) {
    float qv[4], qa[4] = {0.f, 0.f, 0.f, 0.f}, ta[3] = {0.f, 0.f, 0.f}, st[15];
    uint32_t gd[4] = {0u, 0u, 0u, 0u};
    float L = 0.f, b0 = 0.f;
    const bool fused = adam.state != nullptr;
    const bool track = fused && adam.loss && adam.best;
#pragma unroll
    for (int k = 0; k < 4; k++) qv[k] = cq[k * qs];
    if (fused) {
#pragma unroll
        for (int k = 0; k < 4; k++) qa[k] = adam.q[k * qs];
#pragma unroll
        for (int k = 0; k < 3; k++) ta[k] = adam.t[k * qs];
#pragma unroll
        for (int k = 0; k < 15; k++) st[k] = adam.state[k];
        if (adam.guard) {
#pragma unroll
            for (int k = 0; k < 4; k++) gd[k] = adam.guard[k];
        }
        if (track) {
            L = *adam.loss;
            b0 = adam.best[0];
        }
    }
    const Pose ps = make_pose(qv, nullptr, 1);
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
    if (fused) {  // optimizer step fused here: the pose gradient never leaves the kernel
        // forward_overflowed on the preloaded counters: invalid gradients, pose and state unchanged
        if (adam.guard && (gd[0] > adam.cap || gd[2] > gd[3] || gd[1] != 0u)) return;
        const float step = st[14] + 1.f;
        st[14] = step;
        const double bc1 = 1.0 - adam_pow(adam.beta1, step);
        const float bc2_sqrt = (float)sqrt(1.0 - adam_pow(adam.beta2, step));
        const float ss_q = (float)(-adam.lr_q / bc1), ss_t = (float)(-adam.lr_t / bc1);
        const float gq[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int k = 0; k < 4; k++) adam_update(qa[k], gq[k], st[k], st[4 + k], ss_q, adam, bc2_sqrt);
#pragma unroll
        for (int k = 0; k < 3; k++) adam_update(ta[k], S[k], st[8 + k], st[11 + k], ss_t, adam, bc2_sqrt);
#pragma unroll
        for (int k = 0; k < 4; k++) adam.q[k * qs] = qa[k];
#pragma unroll
        for (int k = 0; k < 3; k++) adam.t[k * qs] = ta[k];
#pragma unroll
        for (int k = 0; k < 15; k++) adam.state[k] = st[k];
        // scripts/splatam.py:726-731: keep the pose after this step if this iteration's loss is the
        // lowest so far (a NaN loss never is, like `loss < current_min_loss`)
        if (track && L < b0) {
            adam.best[0] = L;
#pragma unroll
            for (int k = 0; k < 4; k++) adam.best[1 + k] = qa[k];
#pragma unroll
            for (int k = 0; k < 3; k++) adam.best[5 + k] = ta[k];
        }
        return;
    }
    dq[0] = g.x; dq[qs] = g.y; dq[2 * qs] = g.z; dq[3 * qs] = g.w;
    dt[0] = S[0]; dt[qs] = S[1]; dt[2 * qs] = S[2];
}


// One Gaussian's contribution to the 16 pose sums (sum g, sum g p^T, sum dquat_mult^T dr):
// g = dL/dmeans_cam, gd = dL/d[z, 1, z^2] (or NULL), gr = dL/drotation of an anisotropic map
// (or NULL), c = F.normalize(cam quaternion) (used with gr only).
__device__ __forceinline__ void pose_partials_m(float (&v)[POSE_PARTS], int i, const float g_in[3], const float* gd,
                                              const float* gr, const float* __restrict__ mw,
                                              const float* __restrict__ ur, const float (&mci)[3],
                                              const float* __restrict__ w2c, const float c[4]) {
    float g0 = g_in[0], g1 = g_in[1], g2 = g_in[2];
    if (gd) {  // colours [z, 1, z^2]: dz = dc0 + 2 z dc2, z = w2c[2,:3] . m + w2c[2,3]
        const float wz0 = w2c[8], wz1 = w2c[9], wz2 = w2c[10];
        const float z = wz0 * mci[0] + wz1 * mci[1] + wz2 * mci[2] + w2c[11];
        const float dz = gd[0] + 2.f * z * gd[2];
        g0 += dz * wz0; g1 += dz * wz1; g2 += dz * wz2;
    }
    const float p0 = mw[3 * i], p1 = mw[3 * i + 1], p2 = mw[3 * i + 2];
    v[0] += g0; v[1] += g1; v[2] += g2;
    v[3] += g0 * p0; v[4] += g0 * p1; v[5] += g0 * p2;
    v[6] += g1 * p0; v[7] += g1 * p1; v[8] += g1 * p2;
    v[9] += g2 * p0; v[10] += g2 * p1; v[11] += g2 * p2;
    if (gr) {
        // rot = normalize(o), o = quat_mult(c, u), u = normalize(unnorm)
        float un_norm, o_norm;
        const float4 u = normalize4(load4(ur + 4 * i), un_norm);
        const float4 o = quat_mult(c, u);
        const float4 r = normalize4(o, o_norm);
        const float4 d = normalize4_bwd(r, o_norm, load4(gr));
        v[12] += d.x * u.x + d.y * u.y + d.z * u.z + d.w * u.w;
        v[13] += -d.x * u.y + d.y * u.x - d.z * u.w + d.w * u.z;
        v[14] += -d.x * u.z + d.y * u.w + d.z * u.x - d.w * u.y;
        v[15] += -d.x * u.w - d.y * u.z + d.z * u.y + d.w * u.x;
    }
}

__device__ __forceinline__ void pose_partials(float (&v)[POSE_PARTS], int i, const float g_in[3], const float* gd,
                                              const float* gr, const float* __restrict__ mw,
                                              const float* __restrict__ ur, const float* __restrict__ mc,
                                              const float* __restrict__ w2c, const float c[4]) {
    const float mci[3] = {mc[3 * i], mc[3 * i + 1], mc[3 * i + 2]};
    pose_partials_m(v, i, g_in, gd, gr, mw, ur, mci, w2c, c);
}

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
