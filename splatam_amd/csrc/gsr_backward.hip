// gsr_backward.hip -- backward pipeline of the MI355X-native Gaussian rasterizer.
//
// power == 1 (the standard 3DGS backward; SplaTAM's tracking/mapping path):
//   render_bwd  (backward.cu:586-748 semantics) one 16x16 tile per workgroup,
//               back-to-front over LDS batches.  Per (wave, Gaussian) the 9
//               per-pair 2D gradients are summed across the 64 lanes with a
//               transposed permlane/DPP reduction (~30 VALU), the 4 wave
//               partials are summed through LDS, and ONE plain 48-B record per
//               (tile, Gaussian) instance is stored at its unsorted position.
//               No global atomics at all: the reference issues ~25 float
//               atomics per contributing pair (backward.cu:1093-1137).
//   gauss_bwd   one lane per Gaussian: sums its instance records in a fixed
//               order (deterministic, bitwise reproducible) and applies the
//               per-Gaussian chain rule (backward.cu:144-274 cov2D,
//               412-475 cov3D, 480-530 projection, 20-139 SH).
#include "gsr_common.h"

namespace gsr {

__global__ void __launch_bounds__(TILE_PIX)
render_bwd_kernel(Camera cam, const uint2* __restrict__ ranges, const uint32_t* __restrict__ point_list,
                  const uint32_t* __restrict__ perm, const float4* __restrict__ rec_a,
                  const float4* __restrict__ rec_b, const float4* __restrict__ rec_c,
                  const float* __restrict__ final_T, const uint32_t* __restrict__ n_contrib,
                  const float* __restrict__ dL_dpix, float4* __restrict__ inst) {
    __shared__ float4 s_a[RENDER_BATCH];
    __shared__ float4 s_b[RENDER_BATCH];
    __shared__ float4 s_c[RENDER_BATCH];
    __shared__ uint32_t s_u[RENDER_BATCH];
    __shared__ float s_acc[4 * RENDER_BATCH * 9];
    __shared__ uint32_t s_wmax[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int tile = blockIdx.y * cam.gx + blockIdx.x;
    const int px = blockIdx.x * TILE_X + (tid & (TILE_X - 1));
    const int py = blockIdx.y * TILE_Y + (tid >> 4);
    const bool inside = px < cam.W && py < cam.H;
    const int pid = py * cam.W + px;
    const int HW = cam.W * cam.H;
    const uint2 range = ranges[tile];
    const float T_final = inside ? final_T[pid] : 0.f;
    const uint32_t last = inside ? n_contrib[pid] : 0u;
    float dp0 = 0.f, dp1 = 0.f, dp2 = 0.f;
    if (inside) {
        dp0 = dL_dpix[pid];
        dp1 = dL_dpix[HW + pid];
        dp2 = dL_dpix[2 * HW + pid];
    }
    uint32_t wmax = last;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o));
    if (lane == 0) s_wmax[w] = wmax;
    __syncthreads();
    const uint32_t bmax = max(max(s_wmax[0], s_wmax[1]), max(s_wmax[2], s_wmax[3]));
    // Instances behind every pixel's last contributor receive zero gradient.
    for (uint32_t k = range.x + bmax + tid; k < range.y; k += TILE_PIX) {
        const uint32_t u = perm[k];
        inst[3 * u] = make_float4(0.f, 0.f, 0.f, 0.f);
        inst[3 * u + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
        inst[3 * u + 2] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float bg_dot = cam.bg[0] * dp0 + cam.bg[1] * dp1 + cam.bg[2] * dp2;
    const float ddelx = (float)(0.5 * cam.W), ddely = (float)(0.5 * cam.H);  // backward.cu:935-936
    const float pxf = (float)px, pyf = (float)py;
    float T = T_final;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, lc0 = 0.f, lc1 = 0.f, lc2 = 0.f, last_alpha = 0.f;
    const int row = lane >> 4;
    for (int hi = (int)bmax; hi > 0; hi -= RENDER_BATCH) {
        const int cnt = min(RENDER_BATCH, hi);
        if (tid < cnt) {
            const uint32_t k = range.x + (uint32_t)(hi - 1 - tid);
            const uint32_t gi = point_list[k];
            s_u[tid] = perm[k];
            s_a[tid] = rec_a[gi];
            s_b[tid] = rec_b[gi];
            s_c[tid] = rec_c[gi];
        }
        for (int q = tid; q < 4 * RENDER_BATCH * 9 / 4; q += TILE_PIX)
            reinterpret_cast<float4*>(s_acc)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        __syncthreads();
        for (int j = 0; j < cnt; j++) {
            const uint32_t pos = (uint32_t)(hi - 1 - j);  // position in the tile list
            if (pos >= wmax) continue;                     // wave-uniform: no lane reaches it
            float v[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            bool contrib = false;
            if (pos < last) {
                const float4 a = s_a[j];
                const float4 b = s_b[j];
                const float dx = a.x - pxf, dy = a.y - pyf;
                const float power = -0.5f * (a.z * dx * dx + b.x * dy * dy) - a.w * dx * dy;
                const float G = __expf(power);
                const float alpha = fminf(0.99f, b.y * G);
                if (power <= 0.0f && alpha >= 1.0f / 255.0f) {
                    contrib = true;
                    const float4 c = s_c[j];
                    T = T / (1.f - alpha);
                    const float dchannel = alpha * T;
                    acc0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
                    acc1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
                    acc2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
                    lc0 = c.x; lc1 = c.y; lc2 = c.z;
                    float dL_dalpha = (c.x - acc0) * dp0 + (c.y - acc1) * dp1 + (c.z - acc2) * dp2;
                    v[6] = dchannel * dp0;
                    v[7] = dchannel * dp1;
                    v[8] = dchannel * dp2;
                    dL_dalpha *= T;
                    last_alpha = alpha;
                    dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                    const float dL_dG = b.y * dL_dalpha;
                    const float gdx = G * dx, gdy = G * dy;
                    const float dG_ddelx = -gdx * a.z - gdy * a.w;
                    const float dG_ddely = -gdy * b.x - gdx * a.w;
                    v[0] = dL_dG * dG_ddelx * ddelx;
                    v[1] = dL_dG * dG_ddely * ddely;
                    v[2] = -0.5f * gdx * dx * dL_dG;
                    v[3] = -0.5f * gdx * dy * dL_dG;
                    v[4] = -0.5f * gdy * dy * dL_dG;
                    v[5] = G * dL_dalpha;
                }
            }
            if (__ballot(contrib) == 0ull) continue;
            float r0, r1, r8;
            wave_reduce9(v, r0, r1, r8);
            if ((lane & 15) == 0) {
                float* dst = s_acc + (w * RENDER_BATCH + j) * 9;
                const int sl = reduce9_slot_r0(row);
                dst[sl] = r0;
                dst[4 + sl] = r1;
                if (row == 0) dst[8] = r8;
            }
        }
        __syncthreads();
        if (tid < cnt) {
            float s[9];
#pragma unroll
            for (int q = 0; q < 9; q++)
                s[q] = s_acc[(0 * RENDER_BATCH + tid) * 9 + q] + s_acc[(1 * RENDER_BATCH + tid) * 9 + q] +
                       s_acc[(2 * RENDER_BATCH + tid) * 9 + q] + s_acc[(3 * RENDER_BATCH + tid) * 9 + q];
            const uint32_t u = s_u[tid];
            inst[3 * u] = make_float4(s[0], s[1], s[2], s[3]);
            inst[3 * u + 1] = make_float4(s[4], s[5], s[6], s[7]);
            inst[3 * u + 2] = make_float4(s[8], 0.f, 0.f, 0.f);
        }
        __syncthreads();
    }
}

hipError_t launch_render_bwd(const Camera& cam, const uint2* ranges, const uint32_t* point_list,
                             const uint32_t* perm, GeomPtrs geo, const float* colors, const float* final_T,
                             const uint32_t* n_contrib, const float* dL_dpix, float4* inst, hipStream_t s) {
    (void)colors;
    hipLaunchKernelGGL(render_bwd_kernel, dim3(cam.gx, cam.gy), dim3(TILE_PIX), 0, s, cam, ranges, point_list, perm,
                       geo.rec_a, geo.rec_b, geo.rec_c, final_T, n_contrib, dL_dpix, inst);
    return hipGetLastError();
}

// ------------------------------------------------------ per-Gaussian chain --
// g2: [0..1] dL/dmean2D (NDC units), [2..4] dL/dconic (A, B/2, C), [5] dL/dopacity,
// [6..8] dL/dcolor.  Outputs: dmean3D[3], dcov3D[6], dscale[3], drot[4], dsh[3*nsh].
__device__ void gauss_chain(const Camera& cam, const GaussIn& g, int i, const float g2[9], unsigned clamped,
                            float dmean[3], float dcov[6], float dscale[3], float drot[4], float* dsh_out, int nsh) {
    const float fx = cam.focal_x, fy = cam.focal_y;
    const float3 m = make_float3(g.means3D[3 * i], g.means3D[3 * i + 1], g.means3D[3 * i + 2]);
    float c3[6];
    if (g.cov3D) {
#pragma unroll
        for (int k = 0; k < 6; k++) c3[k] = g.cov3D[6 * i + k];
    } else {
        float3 s = make_float3(g.scales[3 * i], g.scales[3 * i + 1], g.scales[3 * i + 2]);
        float4 q = make_float4(g.rotations[4 * i], g.rotations[4 * i + 1], g.rotations[4 * i + 2], g.rotations[4 * i + 3]);
        cov3d_fwd(s, cam.scale_modifier, q, c3);
    }
    // computeCov2DCUDA (backward.cu:144-274)
    Proj pj;
    cov2d_fwd(m, fx, fy, cam.tan_fovx, cam.tan_fovy, c3, cam.view, pj);
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
    if (g.shs) {
        const float* sh = g.shs + (size_t)3 * g.M * i;
        const float dox = m.x - cam.campos[0], doy = m.y - cam.campos[1], doz = m.z - cam.campos[2];
        const float len = sqrtf(dox * dox + doy * doy + doz * doz);
        const float x = dox / len, y = doy / len, z = doz / len;
        const int D = cam.sh_degree;
        float ddir0 = 0.f, ddir1 = 0.f, ddir2 = 0.f;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            const float dRGB = ((clamped >> ch) & 1u) ? 0.f : g2[6 + ch];
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
    (void)nsh;
    // computeCov3D bwd (backward.cu:412-475); dL/dscale w.r.t. (modifier * scale), as the reference
#pragma unroll
    for (int k = 0; k < 3; k++) dscale[k] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; k++) drot[k] = 0.f;
    if (g.scales) {
        const float4 q = make_float4(g.rotations[4 * i], g.rotations[4 * i + 1], g.rotations[4 * i + 2], g.rotations[4 * i + 3]);
        const float r = q.x, x = q.y, y = q.z, z = q.w;
        float R[3][3];
        rot_from_quat(q, R);
        const float s[3] = {cam.scale_modifier * g.scales[3 * i], cam.scale_modifier * g.scales[3 * i + 1],
                            cam.scale_modifier * g.scales[3 * i + 2]};
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

__global__ void __launch_bounds__(256)
gauss_bwd_kernel(Camera cam, GaussIn g, GeomPtrs geo, const int* __restrict__ radii, const float4* __restrict__ inst,
                 GradsOut out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.P) return;
    const int nsh = g.shs ? (cam.sh_degree + 1) * (cam.sh_degree + 1) : 0;
    float g2[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float dmean[3] = {0.f, 0.f, 0.f}, dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, dscale[3] = {0.f, 0.f, 0.f},
          drot[4] = {0.f, 0.f, 0.f, 0.f};
    float dsh[48];
#pragma unroll
    for (int k = 0; k < 48; k++) dsh[k] = 0.f;
    if (radii[i] > 0) {
        const uint32_t off = geo.offsets[i], cnt = geo.tiles[i];
        for (uint32_t e = 0; e < cnt; e++) {
            const float4 r0 = inst[3 * (off + e)];
            const float4 r1 = inst[3 * (off + e) + 1];
            const float r2 = inst[3 * (off + e) + 2].x;
            g2[0] += r0.x; g2[1] += r0.y; g2[2] += r0.z; g2[3] += r0.w;
            g2[4] += r1.x; g2[5] += r1.y; g2[6] += r1.z; g2[7] += r1.w;
            g2[8] += r2;
        }
        const unsigned clamped = __float_as_uint(geo.rec_c[i].w);
        gauss_chain(cam, g, i, g2, clamped, dmean, dcov, dscale, drot, dsh, nsh);
    }
    out.dmeans2D[3 * i] = g2[0];
    out.dmeans2D[3 * i + 1] = g2[1];
    out.dmeans2D[3 * i + 2] = 0.f;
    out.dcolors[3 * i] = g2[6];
    out.dcolors[3 * i + 1] = g2[7];
    out.dcolors[3 * i + 2] = g2[8];
    out.dopacity[i] = g2[5];
#pragma unroll
    for (int k = 0; k < 3; k++) out.dmeans3D[3 * i + k] = dmean[k];
#pragma unroll
    for (int k = 0; k < 6; k++) out.dcov3D[6 * i + k] = dcov[k];
#pragma unroll
    for (int k = 0; k < 3; k++) out.dscales[3 * i + k] = dscale[k];
#pragma unroll
    for (int k = 0; k < 4; k++) out.drot[4 * i + k] = drot[k];
    if (out.dsh && g.M > 0) {
        float* d = out.dsh + (size_t)3 * g.M * i;
#pragma unroll
        for (int k = 0; k < 48; k++)
            if (k < 3 * g.M) d[k] = (k < 3 * nsh) ? dsh[k] : 0.f;
        for (int k = 48; k < 3 * g.M; k++) d[k] = 0.f;
    }
}

hipError_t launch_gauss_bwd(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii, const float4* inst,
                            const GradsOut& out, hipStream_t s) {
    if (g.P == 0) return hipSuccess;
    hipLaunchKernelGGL(gauss_bwd_kernel, dim3((g.P + 255) / 256), dim3(256), 0, s, cam, g, geo, radii, inst, out);
    return hipGetLastError();
}

// ------------------------------------------------------------- self-test --
// Checks the permlane/DPP row mapping of wave_reduce9 on the hardware:
// in[64*9] (lane-major) -> out[9] wave totals.
__global__ void selftest_reduce9_kernel(const float* in, float* out) {
    const int lane = threadIdx.x;
    float v[9];
#pragma unroll
    for (int q = 0; q < 9; q++) v[q] = in[lane * 9 + q];
    float r0, r1, r8;
    wave_reduce9(v, r0, r1, r8);
    if ((lane & 15) == 0) {
        const int row = lane >> 4, sl = reduce9_slot_r0(row);
        out[sl] = r0;
        out[4 + sl] = r1;
        if (row == 0) out[8] = r8;
    }
}

hipError_t launch_selftest_reduce9(const float* in, float* out, hipStream_t s) {
    hipLaunchKernelGGL(selftest_reduce9_kernel, dim3(1), dim3(64), 0, s, in, out);
    return hipGetLastError();
}

}  // namespace gsr
