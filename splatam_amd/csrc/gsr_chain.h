// gsr_chain.h -- per-Gaussian backward chain shared by the power-1 and the
// backward_power != 1 pipelines (gsr_backward.hip, gsr_backward_power.hip).
#pragma once
#include "gsr_common.h"

namespace gsr {

// The geometric inputs of Gaussian i: mean, and scale / rotation (when no cov3D is given) -- loaded
// from GaussIn, or recomputed from the world-frame map by the tracking backward (TrackXf).
struct GaussGeom {
    float3 m;
    float3 s;
    float4 q;
};
__device__ __forceinline__ GaussGeom load_geom(const GaussIn& g, int i) {
    GaussGeom r;
    r.m = make_float3(g.means3D[3 * i], g.means3D[3 * i + 1], g.means3D[3 * i + 2]);
    if (g.scales && g.rotations) {
        r.s = make_float3(g.scales[3 * i], g.scales[3 * i + 1], g.scales[3 * i + 2]);
        r.q = make_float4(g.rotations[4 * i], g.rotations[4 * i + 1], g.rotations[4 * i + 2], g.rotations[4 * i + 3]);
    } else {
        r.s = make_float3(0.f, 0.f, 0.f);
        r.q = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    return r;
}

// Conic of Gaussian i as preprocess computed it (same helpers, same inputs).
// (pj_out / c3_out: the projection and 3D covariance it formed, for gauss_chain to reuse)
__device__ inline void gaussian_conic(const Camera& cam, const GaussIn& g, const GaussGeom& gg, int i, float& ca,
                                      float& cb, float& cc, Proj* pj_out = nullptr, float* c3_out = nullptr) {
    const float3 m = gg.m;
    float c3[6];
    if (g.cov3D) {
#pragma unroll
        for (int k = 0; k < 6; k++) c3[k] = g.cov3D[6 * i + k];
    } else {
        cov3d_fwd(gg.s, cam.scale_modifier, gg.q, c3);
    }
    Proj pj;
    cov2d_fwd(m, cam.focal_x, cam.focal_y, cam.tan_fovx, cam.tan_fovy, c3, cam.view, pj);
    (void)conic_of(pj, ca, cb, cc);
    if (pj_out) *pj_out = pj;
    if (c3_out)
#pragma unroll
        for (int k = 0; k < 6; k++) c3_out[k] = c3[k];
}
__device__ inline void gaussian_conic(const Camera& cam, const GaussIn& g, int i, float& ca, float& cb, float& cc) {
    gaussian_conic(cam, g, load_geom(g, i), i, ca, cb, cc);
}

// SH backward (backward.cu:20-139) for one Gaussian: sh = its 3*M coefficients
// (any address space), drgb = dL/dcolor before the clamp mask.  Writes dsh_out[3*nsh],
// adds the view-direction term to dmean.
__device__ __forceinline__ void sh_chain_bwd(const Camera& cam, float3 m, const float* sh, const float* drgb,
                                             unsigned clamped, float* dsh_out, float dmean[3]) {
    const float dox = m.x - cam.campos[0], doy = m.y - cam.campos[1], doz = m.z - cam.campos[2];
    const float len = sqrtf(dox * dox + doy * doy + doz * doz);
    const float x = dox / len, y = doy / len, z = doz / len;
    const int D = cam.sh_degree;
    float ddir0 = 0.f, ddir1 = 0.f, ddir2 = 0.f;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        const float dRGB = ((clamped >> ch) & 1u) ? 0.f : drgb[ch];
#define SH(k) sh[3 * (k) + ch]
#define DSH(k) dsh_out[3 * (k) + ch]
        float dx_ = 0.f, dy_ = 0.f, dz_ = 0.f;
        DSH(0) = kSH_C0 * dRGB;
        if (D > 0) {
            DSH(1) = -kSH_C1 * y * dRGB;
            DSH(2) = kSH_C1 * z * dRGB;
            DSH(3) = -kSH_C1 * x * dRGB;
            dx_ = -kSH_C1 * SH(3);
            dy_ = -kSH_C1 * SH(1);
            dz_ = kSH_C1 * SH(2);
            if (D > 1) {
                const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                DSH(4) = kSH_C2[0] * xy * dRGB;
                DSH(5) = kSH_C2[1] * yz * dRGB;
                DSH(6) = kSH_C2[2] * (2.f * zz - xx - yy) * dRGB;
                DSH(7) = kSH_C2[3] * xz * dRGB;
                DSH(8) = kSH_C2[4] * (xx - yy) * dRGB;
                dx_ += kSH_C2[0] * y * SH(4) + kSH_C2[2] * 2.f * -x * SH(6) + kSH_C2[3] * z * SH(7) + kSH_C2[4] * 2.f * x * SH(8);
                dy_ += kSH_C2[0] * x * SH(4) + kSH_C2[1] * z * SH(5) + kSH_C2[2] * 2.f * -y * SH(6) + kSH_C2[4] * 2.f * -y * SH(8);
                dz_ += kSH_C2[1] * y * SH(5) + kSH_C2[2] * 2.f * 2.f * z * SH(6) + kSH_C2[3] * x * SH(7);
                if (D > 2) {
                    DSH(9) = kSH_C3[0] * y * (3.f * xx - yy) * dRGB;
                    DSH(10) = kSH_C3[1] * xy * z * dRGB;
                    DSH(11) = kSH_C3[2] * y * (4.f * zz - xx - yy) * dRGB;
                    DSH(12) = kSH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy) * dRGB;
                    DSH(13) = kSH_C3[4] * x * (4.f * zz - xx - yy) * dRGB;
                    DSH(14) = kSH_C3[5] * z * (xx - yy) * dRGB;
                    DSH(15) = kSH_C3[6] * x * (xx - 3.f * yy) * dRGB;
                    dx_ += kSH_C3[0] * SH(9) * 3.f * 2.f * xy + kSH_C3[1] * SH(10) * yz + kSH_C3[2] * SH(11) * -2.f * xy +
                           kSH_C3[3] * SH(12) * -3.f * 2.f * xz + kSH_C3[4] * SH(13) * (-3.f * xx + 4.f * zz - yy) +
                           kSH_C3[5] * SH(14) * 2.f * xz + kSH_C3[6] * SH(15) * 3.f * (xx - yy);
                    dy_ += kSH_C3[0] * SH(9) * 3.f * (xx - yy) + kSH_C3[1] * SH(10) * xz +
                           kSH_C3[2] * SH(11) * (-3.f * yy + 4.f * zz - xx) + kSH_C3[3] * SH(12) * -3.f * 2.f * yz +
                           kSH_C3[4] * SH(13) * -2.f * xy + kSH_C3[5] * SH(14) * -2.f * yz + kSH_C3[6] * SH(15) * -3.f * 2.f * xy;
                    dz_ += kSH_C3[1] * SH(10) * xy + kSH_C3[2] * SH(11) * 4.f * 2.f * yz +
                           kSH_C3[3] * SH(12) * 3.f * (2.f * zz - xx - yy) + kSH_C3[4] * SH(13) * 4.f * 2.f * xz +
                           kSH_C3[5] * SH(14) * (xx - yy);
                }
            }
        }
#undef SH
#undef DSH
        ddir0 += dx_ * dRGB;
        ddir1 += dy_ * dRGB;
        ddir2 += dz_ * dRGB;
    }
    const float sum2 = dox * dox + doy * doy + doz * doz;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);  // dnormvdv, auxiliary.h:107-117
    dmean[0] += ((sum2 - dox * dox) * ddir0 - doy * dox * ddir1 - doz * dox * ddir2) * invsum32;
    dmean[1] += (-dox * doy * ddir0 + (sum2 - doy * doy) * ddir1 - doz * doy * ddir2) * invsum32;
    dmean[2] += (-dox * doz * ddir0 - doy * doz * ddir1 + (sum2 - doz * doz) * ddir2) * invsum32;
}

// ------------------------------------------------------ per-Gaussian chain --
// g2: [0..1] dL/dmean2D (NDC units), [2..4] dL/dconic (A, B/2, C), [5] dL/dopacity,
// [6..8] dL/dcolor.  Outputs: dmean3D[3], dcov3D[6], dscale[3], drot[4], dsh[3*nsh].
// want_rs = false: dscale / drot are not wanted (left zero) -- the pose-fused tracking backward of an
// isotropic map, whose pose sums read neither
__device__ inline void gauss_chain(const Camera& cam, const GaussIn& g, const GaussGeom& gg, int i, const float g2[9],
                                   unsigned clamped, float dmean[3], float dcov[6], float dscale[3], float drot[4],
                                   float* dsh_out, int nsh, bool want_rs = true, const Proj* pj_in = nullptr,
                                   const float* c3_in = nullptr) {
    const float fx = cam.focal_x, fy = cam.focal_y;
    const float3 m = gg.m;
    float c3[6];
    Proj pj;
    if (pj_in) {  // gaussian_conic's (the same expressions on the same inputs)
        pj = *pj_in;
#pragma unroll
        for (int k = 0; k < 6; k++) c3[k] = c3_in[k];
    } else {
        if (g.cov3D) {
#pragma unroll
            for (int k = 0; k < 6; k++) c3[k] = g.cov3D[6 * i + k];
        } else {
            cov3d_fwd(gg.s, cam.scale_modifier, gg.q, c3);
        }
        // computeCov2DCUDA (backward.cu:144-274)
        cov2d_fwd(m, fx, fy, cam.tan_fovx, cam.tan_fovy, c3, cam.view, pj);
    }
    const float a = pj.a, b = pj.b, c = pj.c;
    const float gA = g2[2], gBh = g2[3], gC = g2[4];
    const float denom = a * c - b * b;
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
#pragma unroll
    for (int k = 0; k < 6; k++) dcov[k] = 0.f;
    if (denom2inv != 0.f) {
        dL_da = denom2inv * (-c * c * gA + 2.f * b * c * gBh + (denom - a * c) * gC);
        dL_dc = denom2inv * (-a * a * gC + 2.f * a * b * gBh + (denom - a * c) * gA);
        dL_db = denom2inv * 2.f * (b * c * gA - (denom + 2.f * b * b) * gBh + a * b * gC);
#pragma unroll
        for (int ii = 0; ii < 3; ii++)
#pragma unroll
            for (int jj = ii; jj < 3; jj++) {
                const float vv = pj.Mx[0][ii] * pj.Mx[0][jj] * dL_da + pj.Mx[1][ii] * pj.Mx[1][jj] * dL_dc +
                                 0.5f * (pj.Mx[0][ii] * pj.Mx[1][jj] + pj.Mx[1][ii] * pj.Mx[0][jj]) * dL_db;
                const int idx = (ii == 0) ? jj : (ii == 1 ? 2 + jj : 5);
                dcov[idx] = (ii == jj) ? vv : 2.f * vv;
            }
    }
    const float S[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    float dM[2][3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float ms0 = pj.Mx[0][0] * S[0][k] + pj.Mx[0][1] * S[1][k] + pj.Mx[0][2] * S[2][k];
        const float ms1 = pj.Mx[1][0] * S[0][k] + pj.Mx[1][1] * S[1][k] + pj.Mx[1][2] * S[2][k];
        dM[0][k] = 2.f * dL_da * ms0 + dL_db * ms1;
        dM[1][k] = 2.f * dL_dc * ms1 + dL_db * ms0;
    }
    const float* V = cam.view;
    const float dJ00 = dM[0][0] * V[0] + dM[0][1] * V[4] + dM[0][2] * V[8];
    const float dJ02 = dM[0][0] * V[2] + dM[0][1] * V[6] + dM[0][2] * V[10];
    const float dJ11 = dM[1][0] * V[1] + dM[1][1] * V[5] + dM[1][2] * V[9];
    const float dJ12 = dM[1][0] * V[2] + dM[1][1] * V[6] + dM[1][2] * V[10];
    const float tz = 1.f / pj.tz, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dtx = pj.xmul * -fx * tz2 * dJ02;
    const float dty = pj.ymul * -fy * tz2 * dJ12;
    const float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2.f * fx * pj.tx) * tz3 * dJ02 + (2.f * fy * pj.ty) * tz3 * dJ12;
    dmean[0] = V[0] * dtx + V[1] * dty + V[2] * dtz;
    dmean[1] = V[4] * dtx + V[5] * dty + V[6] * dtz;
    dmean[2] = V[8] * dtx + V[9] * dty + V[10] * dtz;
    // preprocessCUDA bwd (backward.cu:480-530): mean through the projection
    const float* pr = cam.proj;
    const float4 hom = xform4x4(m, pr);
    const float mw = 1.0f / (hom.w + 0.0000001f);
    const float mul1 = hom.x * mw * mw;
    const float mul2 = hom.y * mw * mw;
    const float gx2 = g2[0], gy2 = g2[1];
    dmean[0] += (pr[0] * mw - pr[3] * mul1) * gx2 + (pr[1] * mw - pr[3] * mul2) * gy2;
    dmean[1] += (pr[4] * mw - pr[7] * mul1) * gx2 + (pr[5] * mw - pr[7] * mul2) * gy2;
    dmean[2] += (pr[8] * mw - pr[11] * mul1) * gx2 + (pr[9] * mw - pr[11] * mul2) * gy2;
    // SH bwd (backward.cu:20-139)
    if (g.shs) sh_chain_bwd(cam, m, g.shs + (size_t)3 * g.M * i, g2 + 6, clamped, dsh_out, dmean);
    (void)nsh;
    // computeCov3D bwd (backward.cu:412-475); dL/dscale w.r.t. (modifier * scale), as the reference
#pragma unroll
    for (int k = 0; k < 3; k++) dscale[k] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; k++) drot[k] = 0.f;
    if (g.scales && want_rs) {
        const float4 q = gg.q;
        const float r = q.x, x = q.y, y = q.z, z = q.w;
        float R[3][3];
        rot_from_quat(q, R);
        const float s[3] = {cam.scale_modifier * gg.s.x, cam.scale_modifier * gg.s.y, cam.scale_modifier * gg.s.z};
        const float Gs[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                                {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                                {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
        float dR[3][3];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            float dMk[3];
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const float Mk0 = s[k] * R[0][k], Mk1 = s[k] * R[1][k], Mk2 = s[k] * R[2][k];
                dMk[j] = 2.f * (Mk0 * Gs[0][j] + Mk1 * Gs[1][j] + Mk2 * Gs[2][j]);
            }
            dscale[k] = dMk[0] * R[0][k] + dMk[1] * R[1][k] + dMk[2] * R[2][k];
#pragma unroll
            for (int ii = 0; ii < 3; ii++) dR[ii][k] = dMk[ii] * s[k];
        }
        drot[0] = 2.f * z * (dR[1][0] - dR[0][1]) + 2.f * y * (dR[0][2] - dR[2][0]) + 2.f * x * (dR[2][1] - dR[1][2]);
        drot[1] = 2.f * y * (dR[0][1] + dR[1][0]) + 2.f * z * (dR[0][2] + dR[2][0]) + 2.f * r * (dR[2][1] - dR[1][2]) - 4.f * x * (dR[1][1] + dR[2][2]);
        drot[2] = 2.f * x * (dR[0][1] + dR[1][0]) + 2.f * r * (dR[0][2] - dR[2][0]) + 2.f * z * (dR[1][2] + dR[2][1]) - 4.f * y * (dR[0][0] + dR[2][2]);
        drot[3] = 2.f * r * (dR[1][0] - dR[0][1]) + 2.f * x * (dR[0][2] + dR[2][0]) + 2.f * y * (dR[1][2] + dR[2][1]) - 4.f * z * (dR[0][0] + dR[1][1]);
    }
}
__device__ inline void gauss_chain(const Camera& cam, const GaussIn& g, int i, const float g2[9], unsigned clamped,
                                   float dmean[3], float dcov[6], float dscale[3], float drot[4], float* dsh_out,
                                   int nsh) {
    gauss_chain(cam, g, load_geom(g, i), i, g2, clamped, dmean, dcov, dscale, drot, dsh_out, nsh);
}

}  // namespace gsr
