// gsr_backward_power.hip -- backward with backward_power != 1 (SplaTAM's Fisher /
// Hessian-diagonal scoring through the vendored fused kernel).
//
// Semantics (renderCUDAFused, backward.cu:850-1140; oracle/gsr_oracle.c mode
// GSR_ORACLE_FUSED): every contributing (pixel, Gaussian) pair is pushed through
// the whole per-Gaussian chain, each output component is raised to `power`
// PER PAIR, and only then summed.  The power-1 pipeline may sum first and chain
// once per Gaussian; here the nonlinearity forbids that, so:
//
//   gauss_jac         one lane per Gaussian: the chain is linear in the 9 per-pair
//                     2D gradients (fixed clamp bits), so it is tabulated once per
//                     Gaussian as an 84-float Jacobian pack (JAC_FLOATS; [80..82] the conic):
//                       [ 0..23] dmean3D  <- (dmean2D.xy, dconic.ABC, dRGB.rgb)  3x8
//                       [24..41] dcov3D   <- dconic                            6x3
//                       [42..50] dscale   <- dconic                            3x3
//                       [51..62] drot     <- dconic                            4x3
//                       [63..78] SH basis Y_k(dir) (dsh[k][c] = Y_k * dRGB_c)   16
//   render_bwd_power  per tile, back to front (same recurrence and quadrant culling
//                     as render_bwd_kernel); per pair it forms the NV = 22 + 3*nsh
//                     output components from the staged pack (LDS broadcast
//                     reads), applies powf per lane, reduces them across the wave
//                     with the transposed permlane/DPP reduction and stores one
//                     NV-float record per (tile, Gaussian) instance at its
//                     unsorted slot;
//   gauss_bwd_power   one lane per Gaussian: fixed-order sum of its records
//                     straight into the output tensors (deterministic).
//
// Deliberate difference from the vendored kernel (documented in DESIGN.md):
// SH gradients follow upstream (every coefficient, DC included, no pointer
// offset), as in the power-1 path.
#include <cstdlib>

#include "gsr_chain.h"

namespace gsr {

template <int NSH>
struct PowerShape {
    static constexpr int NV = 22 + 3 * NSH;          // values per pair / record
    static constexpr int NVP = (NV + 3) & ~3;        // padded to the reduction's multiple of 4
    static constexpr int BATCH = NSH >= 9 ? 32 : 64;  // LDS: acc 4*BATCH*NVP floats
};

int power_record_floats(int nsh) {
    switch (nsh) {
        case 0: return PowerShape<0>::NVP;
        case 1: return PowerShape<1>::NVP;
        case 4: return PowerShape<4>::NVP;
        case 9: return PowerShape<9>::NVP;
        case 16: return PowerShape<16>::NVP;
        default: return -1;
    }
}

// --------------------------------------------------------- Jacobian pack --
__global__ void __launch_bounds__(256)
gauss_jac_kernel(Camera cam, GaussIn g, const int* __restrict__ radii, float* __restrict__ jac) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.P || radii[i] <= 0) return;
    const int nsh = g.shs ? (cam.sh_degree + 1) * (cam.sh_degree + 1) : 0;
    float* J = jac + (size_t)JAC_FLOATS * i;
    // the geometry, conic, projection and 3D covariance once (as preprocess computed the conic); the
    // eight unit chain evaluations reuse them
    const GaussGeom gg = load_geom(g, i);
    float ca, cb, cc, c3[6];
    Proj pj;
    gaussian_conic(cam, g, gg, i, ca, cb, cc, &pj, c3);
    // column kk <- unit input g2[kin[kk]] (opacity, input 5, reaches no chained output)
    for (int kk = 0; kk < 8; kk++) {
        const int in = kk < 5 ? kk : kk + 1;
        float g2[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        g2[in] = 1.f;
        float dmean[3], dcov[6], dscale[3], drot[4], dsh[48];
        gauss_chain(cam, g, gg, i, g2, 0u, dmean, dcov, dscale, drot, dsh, nsh, true, &pj, c3);
        for (int r = 0; r < 3; r++) J[r * 8 + kk] = dmean[r];
        if (in >= 2 && in <= 4) {
            const int c = in - 2;
            for (int r = 0; r < 6; r++) J[24 + 3 * r + c] = dcov[r];
            for (int r = 0; r < 3; r++) J[42 + 3 * r + c] = dscale[r];
            for (int r = 0; r < 4; r++) J[51 + 3 * r + c] = drot[r];
        }
        if (in == 6)
            for (int k = 0; k < 16; k++) J[63 + k] = k < nsh ? dsh[3 * k] : 0.f;
    }
    J[79] = 0.f;
    J[JAC_CONIC] = ca;
    J[JAC_CONIC + 1] = cb;
    J[JAC_CONIC + 2] = cc;
    J[JAC_CONIC + 3] = 0.f;
}

hipError_t launch_gauss_jac(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii, float* jac,
                            hipStream_t s) {
    (void)geo;
    if (g.P == 0) return hipSuccess;
    hipLaunchKernelGGL(gauss_jac_kernel, dim3((g.P + 255) / 256), dim3(256), 0, s, cam, g, radii, jac);
    return hipGetLastError();
}

// --------------------------------------------------------- render backward --
__device__ __forceinline__ float pow_pair(float x, int p) { return p == 2 ? x * x : powf(x, (float)p); }

template <int NSH>
__global__ void __launch_bounds__(TILE_PIX)
render_bwd_power_kernel(Camera cam, int has_scales, int power, const uint2* __restrict__ ranges,
                        const PointEntry* __restrict__ point_list, const float4* __restrict__ rr,
                        const uint32_t* __restrict__ blocksums,
                        const uint32_t* __restrict__ clamp_bits,
                        const float4* __restrict__ jac, const float* __restrict__ final_T,
                        const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpix,
                        float4* __restrict__ rec, BwdGuard guard) {
    if (guard.overflow()) return;
    constexpr int NV = PowerShape<NSH>::NV, NVP = PowerShape<NSH>::NVP, B = PowerShape<NSH>::BATCH;
    constexpr int JF4 = JAC_FLOATS / 4;
    __shared__ float4 s_a[B];
    __shared__ float4 s_b[B];
    __shared__ float4 s_c[B];
    __shared__ uint32_t s_u[B];
    __shared__ uint32_t s_g[B];
    __shared__ float4 s_j[B * JF4];
    __shared__ __attribute__((aligned(16))) float s_acc[4 * B * NVP];
    __shared__ uint32_t s_wmax[4];
    __shared__ uint8_t s_mask[B];
    __shared__ __attribute__((aligned(16))) uint16_t s_list[4][B + 4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int tile = sched_tile(cam), tx = tile % cam.gx, ty = tile / cam.gx;
    const int px = tx * TILE_X + tile_px(tid);
    const int py = ty * TILE_Y + tile_py(tid);
    const bool inside = px < cam.W && py < cam.H;
    const int pid = py * cam.W + px;
    const float x0 = (float)(tx * TILE_X), y0 = (float)(ty * TILE_Y);
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
    for (uint32_t k = range.x + bmax + tid; k < range.y; k += TILE_PIX) {
        const uint32_t gk = pe_id(point_list[k]);
        const RenderRec r = load_rr(rr, gk);
        const uint32_t u = instance_slot(rr_rect(r), rr_offset(r, blocksums, gk, cam.pre_shift), tx, ty);
#pragma unroll
        for (int m = 0; m < NVP / 4; m++) rec[(size_t)u * (NVP / 4) + m] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float bg_dot = cam.bg[0] * dp0 + cam.bg[1] * dp1 + cam.bg[2] * dp2;
    const bool bg_on = cam.bg[0] != 0.f || cam.bg[1] != 0.f || cam.bg[2] != 0.f;
    const float ddelx = (float)(0.5 * cam.W), ddely = (float)(0.5 * cam.H);  // backward.cu:935-936
    const float pxf = (float)px, pyf = (float)py;
    float T = T_final;
    float acc_dot = 0.f, lc_dot = 0.f, last_alpha = 0.f;
    const int row = lane >> 4;
    for (int hi = (int)bmax; hi > 0; hi -= B) {
        const int cnt = min(B, hi);
        if (tid < cnt) {
            const uint32_t gi = pe_id(point_list[range.x + (uint32_t)(hi - 1 - tid)]);
            const RenderRec r = load_rr(rr, gi);
            const float4 pa = r.q0, pb = r.q1;
            s_g[tid] = gi;
            s_u[tid] = instance_slot(rr_rect(r), rr_offset(r, blocksums, gi, cam.pre_shift), tx, ty);
            s_a[tid] = pa;
            s_b[tid] = pb;
            s_c[tid] = make_float4(r.q2.x, r.q2.y, r.q2.z, __uint_as_float(clamp_bits[gi]));
            s_mask[tid] = (uint8_t)quad_mask(pa, pb, x0, y0);
        }
        for (int q = tid; q < 4 * B * NVP / 4; q += TILE_PIX)
            reinterpret_cast<float4*>(s_acc)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        __syncthreads();
        {  // every Jacobian-pack load issued before the first LDS store (one round trip, not one per float4)
            constexpr int NJ = (B * JF4 + TILE_PIX - 1) / TILE_PIX;
            float4 jv[NJ];
#pragma unroll
            for (int i = 0; i < NJ; i++) {
                const int q = min(tid + i * TILE_PIX, cnt * JF4 - 1);  // clamped: loads without a branch
                const int item = q / JF4, part = q - item * JF4;
                jv[i] = jac[(size_t)s_g[item] * JF4 + part];
            }
#pragma unroll
            for (int i = 0; i < NJ; i++) {
                const int q = tid + i * TILE_PIX;
                if (q < cnt * JF4) s_j[q] = jv[i];
            }
        }
        __syncthreads();
        const int n = build_wave_list(s_mask, cnt, w, hi - (int)wmax, s_list[w]);
        for (int i = 0; i < n; i++) {
            const int j = s_list[w][i];  // wave-uniform
            const float4 a = s_a[j], b = s_b[j];
            const v2f dd = pix_delta(a, v2f{pxf, pyf});
            const float dx = dd.x, dy = dd.y;
            const float p2 = eval_p2(a, b, dd);
            const float G = __builtin_amdgcn_exp2f(fminf(p2, 0.f));
            const float araw = b.y * G;
            const float alpha = fminf(0.99f, araw);
            const uint32_t pos = (uint32_t)(hi - 1 - j);
            const bool ok = pos < last && p2 <= 0.0f && alpha >= 1.0f / 255.0f;
            if (__ballot(ok) == 0ull) continue;
            const float4 c = s_c[j];
            const float inv = __builtin_amdgcn_rcpf(1.f - alpha);
            const float Tn = T * inv;
            const float cd = c.x * dp0 + c.y * dp1 + c.z * dp2;
            const float na_dot = last_alpha * lc_dot + (1.f - last_alpha) * acc_dot;
            float dL_dalpha = (cd - na_dot) * Tn;
            if (bg_on) dL_dalpha += (-T_final * inv) * bg_dot;
            const float dch = alpha * Tn;
            const float h = araw * dL_dalpha;  // G * dL/dG
            const float hx = h * dx, hy = h * dy;
            const float4* Jq = s_j + j * JF4;
            float Jv[JAC_FLOATS];
#pragma unroll
            for (int m = 0; m < JF4; m++) {
                const float4 t = Jq[m];
                Jv[4 * m] = t.x; Jv[4 * m + 1] = t.y; Jv[4 * m + 2] = t.z; Jv[4 * m + 3] = t.w;
            }
            // per-pair quantities of backward.cu:1020-1038
            float in8[8];
            in8[0] = -(Jv[JAC_CONIC] * hx + Jv[JAC_CONIC + 1] * hy) * ddelx;
            in8[1] = -(Jv[JAC_CONIC + 2] * hy + Jv[JAC_CONIC + 1] * hx) * ddely;
            in8[2] = -0.5f * hx * dx;
            in8[3] = -0.5f * hx * dy;
            in8[4] = -0.5f * hy * dy;
            const float col0 = dch * dp0, col1 = dch * dp1, col2 = dch * dp2;
            const unsigned clamped = __float_as_uint(c.w);
            in8[5] = (clamped & 1u) ? 0.f : col0;
            in8[6] = (clamped & 2u) ? 0.f : col1;
            in8[7] = (clamped & 4u) ? 0.f : col2;
            float v[NVP];
            v[0] = in8[0];
            v[1] = in8[1];
            v[2] = col0;
            v[3] = col1;
            v[4] = col2;
            v[5] = G * dL_dalpha;
#pragma unroll
            for (int r = 0; r < 3; r++) {
                float s = 0.f;
#pragma unroll
                for (int kk = 0; kk < 8; kk++) s += Jv[r * 8 + kk] * in8[kk];
                v[6 + r] = s;
            }
#pragma unroll
            for (int r = 0; r < 6; r++) v[9 + r] = Jv[24 + 3 * r] * in8[2] + Jv[25 + 3 * r] * in8[3] + Jv[26 + 3 * r] * in8[4];
#pragma unroll
            for (int r = 0; r < 3; r++) v[15 + r] = Jv[42 + 3 * r] * in8[2] + Jv[43 + 3 * r] * in8[3] + Jv[44 + 3 * r] * in8[4];
#pragma unroll
            for (int r = 0; r < 4; r++) v[18 + r] = Jv[51 + 3 * r] * in8[2] + Jv[52 + 3 * r] * in8[3] + Jv[53 + 3 * r] * in8[4];
#pragma unroll
            for (int k = 0; k < NSH; k++)
#pragma unroll
                for (int ch = 0; ch < 3; ch++) v[22 + 3 * k + ch] = Jv[63 + k] * in8[5 + ch];
#pragma unroll
            for (int m = 0; m < NVP; m++) {
                float x = m < NV ? pow_pair(v[m], power) : 0.f;
                if (!has_scales && m >= 15 && m < 22) x = 0.f;  // the reference skips scale/rot grads
                v[m] = ok ? x : 0.f;
            }
            if (ok) {
                T = Tn;
                acc_dot = na_dot;
                lc_dot = cd;
                last_alpha = alpha;
            }
            float r[NVP / 4];
            wave_reduce_n<NVP>(v, r);
            if ((lane & 15) == 0) {
                float* dst = s_acc + (w * B + j) * NVP + row * (NVP / 4);
#pragma unroll
                for (int m = 0; m < NVP / 4; m++) dst[m] = r[m];
            }
        }
        __syncthreads();
        for (int q = tid; q < cnt * (NVP / 4); q += TILE_PIX) {
            const int item = q / (NVP / 4), m = q - item * (NVP / 4);
            const float4* acc = reinterpret_cast<const float4*>(s_acc);
            const float4 s0 = acc[(0 * B + item) * (NVP / 4) + m], s1 = acc[(1 * B + item) * (NVP / 4) + m];
            const float4 s2 = acc[(2 * B + item) * (NVP / 4) + m], s3 = acc[(3 * B + item) * (NVP / 4) + m];
            rec[(size_t)s_u[item] * (NVP / 4) + m] =
                make_float4(s0.x + s1.x + s2.x + s3.x, s0.y + s1.y + s2.y + s3.y, s0.z + s1.z + s2.z + s3.z,
                            s0.w + s1.w + s2.w + s3.w);
        }
        __syncthreads();
    }
}

hipError_t launch_render_bwd_power(const Camera& cam, const GaussIn& g, const uint2* ranges,
                                   const uint64_t* point_list, GeomPtrs geo, const float* jac, const float* final_T,
                                   const uint32_t* n_contrib, const float* dL_dpix, int power, float* rec,
                                   BwdGuard guard, hipStream_t s) {
    const int nsh = g.shs ? (cam.sh_degree + 1) * (cam.sh_degree + 1) : 0;
    const int has_scales = g.scales != nullptr;
    const dim3 grid(cam.gx * cam.gy), block(TILE_PIX);
#define GSR_LAUNCH_POWER(NSH_)                                                                                      \
    hipLaunchKernelGGL(render_bwd_power_kernel<NSH_>, grid, block, 0, s, cam, has_scales, power, ranges, point_list, \
                       geo.rr, geo.blocksums, geo.clamp, (const float4*)jac, final_T,                                              \
                       n_contrib, dL_dpix, (float4*)rec, guard)
    switch (nsh) {
        case 0: GSR_LAUNCH_POWER(0); break;
        case 1: GSR_LAUNCH_POWER(1); break;
        case 4: GSR_LAUNCH_POWER(4); break;
        case 9: GSR_LAUNCH_POWER(9); break;
        case 16: GSR_LAUNCH_POWER(16); break;
        default: return hipErrorInvalidValue;
    }
#undef GSR_LAUNCH_POWER
    return hipGetLastError();
}

// ----------------------------------------------------- per-Gaussian sums --
template <int NSH>
__global__ void __launch_bounds__(256)
gauss_bwd_power_kernel(GaussIn g, GeomPtrs geo, const int* __restrict__ radii, const float4* __restrict__ rec,
                       GradsOut out, BwdGuard guard) {
    constexpr int NVP = PowerShape<NSH>::NVP;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.P) return;
    float s[NVP];
#pragma unroll
    for (int m = 0; m < NVP; m++) s[m] = 0.f;
    if (radii[i] > 0 && !guard.overflow()) {
        const uint32_t off = geo.offsets[i], cnt = geo.tiles[i];
        const uint32_t tl = reinterpret_cast<const uint32_t*>(geo.bin)[4 * (size_t)i + 3];  // (Camera::cull)
        for (uint32_t e = 0; e < cnt; e++) {
            if (!tile_live(tl, e)) continue;
            const float4* r = rec + (size_t)(off + e) * (NVP / 4);
#pragma unroll
            for (int m = 0; m < NVP / 4; m++) {
                const float4 t = r[m];
                s[4 * m] += t.x; s[4 * m + 1] += t.y; s[4 * m + 2] += t.z; s[4 * m + 3] += t.w;
            }
        }
    }
    out.dmeans2D[3 * i] = s[0];
    out.dmeans2D[3 * i + 1] = s[1];
    out.dmeans2D[3 * i + 2] = 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) out.dcolors[3 * i + k] = s[2 + k];
    out.dopacity[i] = s[5];
#pragma unroll
    for (int k = 0; k < 3; k++) out.dmeans3D[3 * i + k] = s[6 + k];
#pragma unroll
    for (int k = 0; k < 6; k++) out.dcov3D[6 * i + k] = s[9 + k];
#pragma unroll
    for (int k = 0; k < 3; k++) out.dscales[3 * i + k] = s[15 + k];
#pragma unroll
    for (int k = 0; k < 4; k++) out.drot[4 * i + k] = s[18 + k];
    if (out.dsh && g.M > 0) {
        float* d = out.dsh + (size_t)3 * g.M * i;
#pragma unroll
        for (int k = 0; k < 3 * NSH; k++)
            if (k < 3 * g.M) d[k] = s[22 + k];
        for (int k = 3 * NSH; k < 3 * g.M; k++) d[k] = 0.f;
    }
}

// ---------------------------------------------- Fisher-selective backward --
// The fork's Fisher / EIG scoring reads only transformed_pts.grad and opacities.grad of a
// backward_power render (scripts/ros_handler.py:884-889).  Without SH (colours precomputed) a
// pair's dL/dmeans3D is linear in its 2D terms u = h (dx, dy, dx^2, dx dy, dy^2), h = G dL/dG:
// backward.cu:1020-1038 forms dmean2D = -(Q h d) ddel and dconic = -1/2 h d d^T, and the
// per-Gaussian chain (computeCov2D / projection backward) maps those linearly to dmean3D.  With
// the conic and the NDC factor folded in, dmean3D_r = h * (M_r . (dx, dy, dx^2, dx dy, dy^2)) for a
// 3x5 matrix M per Gaussian (gauss_mpack_kernel), so a pair forms 4 values (3 mean components and
// G dL/dalpha), each raised to `power`, instead of the full path's 22 + 3 nsh.  The tile walk is
// render_bwd_kernel's: per-row lists of the 4x4-pixel blocks an entry's ellipse reaches (exact
// masks from the forward), compact per-(entry, block) slots, the transposed in-row reduction, one
// 16-B record per (tile, Gaussian) instance at its unsorted slot.
constexpr int MPACK_F4 = 4;  // M (15 floats, row-major) + 1 pad

__global__ void __launch_bounds__(256, 5)  // (5 workgroups per CU: a frame's ~1200 in one round)
gauss_mpack_kernel(Camera cam, GaussIn g, const int* __restrict__ radii, float4* __restrict__ mp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.P || radii[i] <= 0) return;
    const GaussGeom gg = load_geom(g, i);
    // the conic, projection and 3D covariance once; the five chain evaluations reuse them and skip the
    // rotation / scale terms (only dmean3D is tabulated)
    float ca, cb, cc, c3[6];
    Proj pj;
    gaussian_conic(cam, g, gg, i, ca, cb, cc, &pj, c3);
    float J[3][5];
#pragma unroll 1
    for (int kk = 0; kk < 5; kk++) {  // column kk <- unit dmean2D.x/.y, dconic.A/.B/.C
        float g2[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        g2[kk] = 1.f;
        float dmean[3], dcov[6], dscale[3], drot[4], dsh[48];
        gauss_chain(cam, g, gg, i, g2, 0u, dmean, dcov, dscale, drot, dsh, 0, false, &pj, c3);
#pragma unroll
        for (int r = 0; r < 3; r++) J[r][kk] = dmean[r];
    }
    const float ddelx = (float)(0.5 * cam.W), ddely = (float)(0.5 * cam.H);  // backward.cu:935-936
    float M[16];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        M[5 * r] = -(J[r][0] * ca * ddelx + J[r][1] * cb * ddely);
        M[5 * r + 1] = -(J[r][0] * cb * ddelx + J[r][1] * cc * ddely);
        M[5 * r + 2] = -0.5f * J[r][2];
        M[5 * r + 3] = -0.5f * J[r][3];
        M[5 * r + 4] = -0.5f * J[r][4];
    }
    M[15] = 0.f;
#pragma unroll
    for (int q = 0; q < MPACK_F4; q++) mp[(size_t)MPACK_F4 * i + q] = make_float4(M[4 * q], M[4 * q + 1], M[4 * q + 2], M[4 * q + 3]);
}

template <bool POW2>
__device__ __forceinline__ float pow_sel(float x, float p) { return POW2 ? x * x : powf(x, p); }

#ifndef GSR_FISHER_WAVES
#define GSR_FISHER_WAVES 4  // 128 VGPRs: room for a step's records and the next entry's M rows in flight
#endif
#ifndef GSR_FISHER_PF
#define GSR_FISHER_PF 1  // a step's geometry / colour records loaded up front, the next entry's M rows a pair ahead
#endif
template <bool POW2>
__global__ void __launch_bounds__(TILE_PIX, GSR_FISHER_WAVES)
render_bwd_fisher_kernel(Camera cam, float power, const uint2* __restrict__ ranges,
                         const PointEntry* __restrict__ point_list, const float4* __restrict__ rr,
                         const uint32_t* __restrict__ blocksums, const float4* __restrict__ mp,
                         const float* __restrict__ final_T, const uint32_t* __restrict__ n_contrib,
                         const float* __restrict__ dL_dpix, float* __restrict__ inst, BwdGuard guard) {
    if (guard.overflow()) return;  // invalid forward state (static-mode overflow): touch nothing
    constexpr int NV = 4, BB = 128, BS = 4 * BB, LS = BB + 4, SL = BB + 1;
    __shared__ float4 s_a[SL];
    __shared__ float4 s_b[SL];
    __shared__ float4 s_c[SL];
    __shared__ float4 s_m[MPACK_F4 * SL];
    __shared__ uint32_t s_u[BB];
    __shared__ uint16_t s_mask[BB];
    __shared__ uint16_t s_base[BB];
    __shared__ float4 s_acc4[BS + 1];
    __shared__ uint32_t s_rmax[16];
    __shared__ __attribute__((aligned(16))) uint32_t s_list[16 * LS];
    float* s_acc = reinterpret_cast<float*>(s_acc4);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, row = (tid >> 4) & 3;
    const int tile = sched_tile(cam), tx = tile % cam.gx, ty = tile / cam.gx;
    const int px = tx * TILE_X + tile_px(tid);
    const int py = ty * TILE_Y + tile_py(tid);
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
    uint32_t rmax = last;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, o));
    if ((lane & 15) == 0) s_rmax[4 * w + row] = rmax;
    __syncthreads();
    uint32_t bmax = 0;
#pragma unroll
    for (int b = 0; b < 16; b++) bmax = max(bmax, s_rmax[b]);
    const int rm[4] = {(int)s_rmax[4 * w], (int)s_rmax[4 * w + 1], (int)s_rmax[4 * w + 2], (int)s_rmax[4 * w + 3]};
    for (uint32_t k = range.x + bmax + tid; k < range.y; k += TILE_PIX) {  // behind every last contributor
        const uint32_t gk = pe_id(point_list[k]);
        const RenderRec r = load_rr(rr, gk);
        const uint32_t u = instance_slot(rr_rect(r), rr_offset(r, blocksums, gk, cam.pre_shift), tx, ty);
        reinterpret_cast<float4*>(inst)[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // background term of dL/dalpha (backward.cu:1014): -T_final / (1 - alpha) * (bg . dL/dpix)
    const float Tbg = -T_final * (cam.bg[0] * dp0 + cam.bg[1] * dp1 + cam.bg[2] * dp2);
    const v2f pix = v2f{(float)px, (float)py};
    const v2f dp01 = v2f{dp0, dp1};
    float T = T_final, A = 0.f;
    const int my_e = row_entry(lane);
    for (int q = tid; q < BS + 1; q += TILE_PIX) s_acc4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    const uint32_t* my_list = s_list + (4 * w + row) * LS;
    if (tid == 0) {
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        s_a[BB] = z;
        s_b[BB] = z;
        s_c[BB] = z;
#pragma unroll
        for (int q = 0; q < MPACK_F4; q++) s_m[MPACK_F4 * BB + q] = z;
    }
    // staging pipelined two batches deep (render_bwd_kernel): records + M of the next batch in
    // registers, sorted list entries of the batch after it
    float4 pa = make_float4(0.f, 0.f, 0.f, 0.f), pb = pa, pc = pa, pm0 = pa, pm1 = pa, pm2 = pa, pm3 = pa;
    uint32_t pbs = 0, pmask = 0, prh = 0, pgi = 0;
    PointEntry pn = 0;
    auto fetch_entry = [&](int hi_) {
        if (tid < min(BB, hi_)) pn = point_list[range.x + (uint32_t)(hi_ - 1 - tid)];
    };
    auto fetch_rec = [&](int hi_) {
        if (tid < min(BB, hi_)) {
            const uint32_t gi = pe_id(pn);
            pmask = pe_mask(pn);
            const RenderRec r = load_rr(rr, gi);
            pbs = blocksums[gi >> cam.pre_shift];
            pa = r.q0; pb = r.q1; pc = r.q2;
            prh = __float_as_uint(r.q3.w);
            pgi = gi;
        }
    };
    // the M rows are loaded after the walk (in flight during the entry totals), so they occupy no
    // registers while the batch is rasterised (16 VGPRs: the kernel spilled at 96)
    auto fetch_m = [&](int hi_) {
        if (tid < min(BB, hi_)) {
            const float4* m = mp + (size_t)MPACK_F4 * pgi;
            pm0 = m[0];
            pm1 = m[1];
            pm2 = m[2];
            pm3 = m[3];
        }
    };
    fetch_entry((int)bmax);
    fetch_rec((int)bmax);
    fetch_m((int)bmax);
    fetch_entry((int)bmax - BB);
    const uint32_t mean4 = sched_mean4(cam, guard.counters);
    int hi_pf = (int)bmax;
    for (int hi = (int)bmax; hi > 0;) {
        prio_by_remaining(hi, mean4, sched_multi_round(cam));
        if (hi != hi_pf) {  // the previous batch was cut by its slot budget: re-fetch (rare)
            fetch_entry(hi);
            fetch_rec(hi);
            fetch_m(hi);
            fetch_entry(hi - BB);
        }
        const int cmax = min(BB, hi);
        int ts_ = tid;
        asm volatile("" : "+v"(ts_));
        if (ts_ < cmax) {
            s_u[ts_] = instance_slot(make_uint2(__float_as_uint(pc.w), prh), pbs + __float_as_uint(pb.w), tx, ty);
            s_a[ts_] = pa;
            s_b[ts_] = pb;
            s_c[ts_] = pc;
            s_m[MPACK_F4 * ts_] = pm0;
            s_m[MPACK_F4 * ts_ + 1] = pm1;
            s_m[MPACK_F4 * ts_ + 2] = pm2;
            s_m[MPACK_F4 * ts_ + 3] = pm3;
            s_mask[ts_] = (uint16_t)pmask;
        }
        __syncthreads();
        fetch_rec(hi - BB);
        fetch_entry(hi - 2 * BB);
        hi_pf = hi - BB;
        const int jmin[4] = {hi - rm[0], hi - rm[1], hi - rm[2], hi - rm[3]};
        const SlotLists sl = build_row_slot_lists(s_mask, s_base, cmax, BS, w, jmin, s_list + 4 * w * LS, LS,
                                                  (uint32_t)BB | ((uint32_t)BS << 16));
        const int n = sl.len, cnt = sl.cnt;
        const int jlo = hi - (int)last;  // pos = hi-1-j < last  <=>  j >= jlo
        for (int i = 0; i < n; i += 4) {
            const uint4 gw = load_slot_group4(my_list, i);
            int jj[4];
            jj[0] = (int)(gw.x & 0xFFFFu);
            jj[1] = (int)(gw.y & 0xFFFFu);
            jj[2] = (int)(gw.z & 0xFFFFu);
            jj[3] = (int)(gw.w & 0xFFFFu);
            v2f d[4];
            float G[4], araw[4], alpha[4];
            bool ok[4];
#if GSR_FISHER_PF
            // one LDS round trip for the step's four geometry records (the compiler otherwise waits on each
            // entry's reads in turn: the kernel was LDS-latency-bound, SQ_WAIT_ANY 59 % of wave cycles)
            float4 ra[4], rb[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                ra[k] = s_a[jj[k]];
                rb[k] = s_b[jj[k]];
            }
#endif
#pragma unroll
            for (int k = 0; k < 4; k++) {
#if GSR_FISHER_PF
                const float4 a = ra[k], b = rb[k];
#else
                const float4 a = s_a[jj[k]], b = s_b[jj[k]];
#endif
                d[k] = pix_delta(a, pix);
                const float p2 = eval_p2(a, b, d[k]);
                G[k] = __builtin_amdgcn_exp2f(fminf(p2, 0.f));
                araw[k] = b.y * G[k];
                alpha[k] = fminf(0.99f, araw[k]);
                ok[k] = jj[k] >= jlo && p2 <= 0.0f && alpha[k] >= 1.0f / 255.0f;
                alpha[k] = ok[k] ? alpha[k] : 0.f;
            }
            // per pair, in list order: T and A, dL/dalpha; dL/dmeans3D = h * (M . (dx, dy, dx^2, dx dy,
            // dy^2)) with h = G dL/dG, dL/dopacity = G dL/dalpha, each powered (0 on non-contributing pairs)
            float v[4 * NV];
#if GSR_FISHER_PF
            float4 rc[4];
#pragma unroll
            for (int k = 0; k < 4; k++) rc[k] = s_c[jj[k]];
            float4 nm0 = s_m[MPACK_F4 * jj[0]], nm1 = s_m[MPACK_F4 * jj[0] + 1];
            float4 nm2 = s_m[MPACK_F4 * jj[0] + 2], nm3 = s_m[MPACK_F4 * jj[0] + 3];
#endif
#pragma unroll
            for (int k = 0; k < 4; k++) {
#if GSR_FISHER_PF
                const float4 c = rc[k];
                const float4 m0 = nm0, m1 = nm1, m2 = nm2, m3 = nm3;
                if (k < 3) {  // the next entry's M rows, in flight while this entry's values are formed
                    nm0 = s_m[MPACK_F4 * jj[k + 1]];
                    nm1 = s_m[MPACK_F4 * jj[k + 1] + 1];
                    nm2 = s_m[MPACK_F4 * jj[k + 1] + 2];
                    nm3 = s_m[MPACK_F4 * jj[k + 1] + 3];
                }
#else
                const float4 c = s_c[jj[k]];
#endif
                const v2f t = v2f{c.x, c.y} * dp01;
                const float cd = __builtin_fmaf(c.z, dp2, t.x + t.y);
                const float inv = __builtin_amdgcn_rcpf(1.f - alpha[k]);
                const float Tn = T * inv;                      // backward.cu:978
                const float e = cd - A;
                const bool o = ok[k];
                const float dLa = o ? __builtin_fmaf(Tbg, inv, e * Tn) : 0.f;
                T = Tn;  // masked pairs: alpha = 0, v_rcp_f32(1) == 1 exactly
                A = __builtin_fmaf(alpha[k], e, A);
#if !GSR_FISHER_PF
                const float4 m0 = s_m[MPACK_F4 * jj[k]], m1 = s_m[MPACK_F4 * jj[k] + 1];
                const float4 m2 = s_m[MPACK_F4 * jj[k] + 2], m3 = s_m[MPACK_F4 * jj[k] + 3];
#endif
                const float dx = d[k].x, dy = d[k].y;
                const float xx = dx * dx, xy = dx * dy, yy = dy * dy;
                const float h = araw[k] * dLa;
                const float q0 = m0.x * dx + m0.y * dy + m0.z * xx + m0.w * xy + m1.x * yy;
                const float q1 = m1.y * dx + m1.z * dy + m1.w * xx + m2.x * xy + m2.y * yy;
                const float q2 = m2.z * dx + m2.w * dy + m3.x * xx + m3.y * xy + m3.z * yy;
                float x0 = pow_sel<POW2>(h * q0, power), x1 = pow_sel<POW2>(h * q1, power);
                float x2 = pow_sel<POW2>(h * q2, power), x3 = pow_sel<POW2>(G[k] * dLa, power);
                // the entry's values formed here, unconditionally (no branch around the M reads), and its
                // M rows dead before the next entry's are read: all four entries' rows live at once spilled
                asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)::"memory");
                v[NV * k] = o ? x0 : 0.f;
                v[NV * k + 1] = o ? x1 : 0.f;
                v[NV * k + 2] = o ? x2 : 0.f;
                v[NV * k + 3] = o ? x3 : 0.f;
            }
            const uint32_t wlo = (my_e & 1) ? gw.y : gw.x, whi = (my_e & 1) ? gw.w : gw.z;
            const uint32_t we = (my_e & 2) ? whi : wlo;
            float r[RowReduce<NV>::R];
            row_reduce<NV>(v, r, lane);
            if ((lane & RowReduce<NV>::WRITER_MASK) == 0) {
                float* p = s_acc + (we >> 16) * NV + row_m0<NV>(lane);
#pragma unroll
                for (int m = 0; m < RowReduce<NV>::R; m++) p[m] = r[m];
            }
        }
        fetch_m(hi_pf);  // M rows of the next batch (its records were loaded after the staging barrier)
        __syncthreads();
        // entry totals: 2 threads per entry, each adds 2 values over the entry's block slots in block
        // order (deterministic), re-zeroes them, stores its half of the 16-B record
        int t_ = tid;
        asm volatile("" : "+v"(t_));
        const int e = t_ >> 1, q = t_ & 1;
        if (e < cnt) {
            float c0 = 0.f, c1 = 0.f;
            const int nb = __popc((uint32_t)s_mask[e]);
            float2* src = reinterpret_cast<float2*>(s_acc + (int)s_base[e] * NV) + q;
            for (int b = 0; b < nb; b++, src += 2) {
                const float2 x = *src;
                c0 += x.x;
                c1 += x.y;
                *src = make_float2(0.f, 0.f);
            }
            reinterpret_cast<float2*>(inst)[2 * (size_t)s_u[e] + q] = make_float2(c0, c1);
        }
        __syncthreads();
        hi -= cnt;
    }
}

// One lane per Gaussian: fixed-order sum of its 16-B instance records (deterministic) straight
// into dL/dmeans3D and dL/dopacity (nullptr: skipped).
__global__ void __launch_bounds__(256)
gauss_bwd_fisher_kernel(int P, GeomPtrs geo, const int* __restrict__ radii, const float4* __restrict__ rec,
                        float* __restrict__ dmeans3D, float* __restrict__ dopacity, BwdGuard guard) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (radii[i] > 0 && !guard.overflow()) {
        const uint32_t off = geo.offsets[i], cnt = geo.tiles[i];
        const uint32_t tl = reinterpret_cast<const uint32_t*>(geo.bin)[4 * (size_t)i + 3];  // (Camera::cull)
        constexpr int RU = 4;  // RU records' loads per memory round trip, added in instance order
        for (uint32_t e0 = 0; e0 < cnt; e0 += RU) {
            float4 v[RU];
#pragma unroll
            for (int k = 0; k < RU; k++)
                v[k] = (e0 + k < cnt && tile_live(tl, e0 + k)) ? rec[off + e0 + k] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int k = 0; k < RU; k++)
                if (e0 + k < cnt && tile_live(tl, e0 + k)) {
                    s.x += v[k].x;
                    s.y += v[k].y;
                    s.z += v[k].z;
                    s.w += v[k].w;
                }
        }
    }
    dmeans3D[3 * i] = s.x;
    dmeans3D[3 * i + 1] = s.y;
    dmeans3D[3 * i + 2] = s.z;
    if (dopacity) dopacity[i] = s.w;
}

hipError_t launch_gauss_mpack(const Camera& cam, const GaussIn& g, const int* radii, float* mpack, hipStream_t s) {
    if (g.P == 0) return hipSuccess;
    hipLaunchKernelGGL(gauss_mpack_kernel, dim3((g.P + 255) / 256), dim3(256), 0, s, cam, g, radii, (float4*)mpack);
    return hipGetLastError();
}

hipError_t launch_render_bwd_fisher(const Camera& cam, const uint2* ranges, const uint64_t* point_list, GeomPtrs geo,
                                    const float* mpack, const float* final_T, const uint32_t* n_contrib,
                                    const float* dL_dpix, int power, float* rec, BwdGuard guard, hipStream_t s) {
    auto k = power == 2 ? render_bwd_fisher_kernel<true> : render_bwd_fisher_kernel<false>;
    hipLaunchKernelGGL(k, dim3(cam.gx * cam.gy), dim3(TILE_PIX), 0, s, cam, (float)power, ranges, point_list, geo.rr,
                       geo.blocksums, (const float4*)mpack, final_T, n_contrib, dL_dpix, rec, guard);
    return hipGetLastError();
}

hipError_t launch_gauss_bwd_fisher(int P, GeomPtrs geo, const int* radii, const float* rec, float* dmeans3D,
                                   float* dopacity, BwdGuard guard, hipStream_t s) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(gauss_bwd_fisher_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, geo, radii,
                       (const float4*)rec, dmeans3D, dopacity, guard);
    return hipGetLastError();
}

hipError_t launch_gauss_bwd_power(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii,
                                  const float* rec, const GradsOut& out, BwdGuard guard, hipStream_t s) {
    if (g.P == 0) return hipSuccess;
    const int nsh = g.shs ? (cam.sh_degree + 1) * (cam.sh_degree + 1) : 0;
    const dim3 grid((g.P + 255) / 256), block(256);
    const float4* r = (const float4*)rec;
    switch (nsh) {
        case 0: hipLaunchKernelGGL(gauss_bwd_power_kernel<0>, grid, block, 0, s, g, geo, radii, r, out, guard); break;
        case 1: hipLaunchKernelGGL(gauss_bwd_power_kernel<1>, grid, block, 0, s, g, geo, radii, r, out, guard); break;
        case 4: hipLaunchKernelGGL(gauss_bwd_power_kernel<4>, grid, block, 0, s, g, geo, radii, r, out, guard); break;
        case 9: hipLaunchKernelGGL(gauss_bwd_power_kernel<9>, grid, block, 0, s, g, geo, radii, r, out, guard); break;
        case 16: hipLaunchKernelGGL(gauss_bwd_power_kernel<16>, grid, block, 0, s, g, geo, radii, r, out, guard); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace gsr
