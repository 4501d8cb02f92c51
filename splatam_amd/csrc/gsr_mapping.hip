// gsr_mapping.hip -- SplaTAM's mapping-iteration glue as HIP kernels
// (include/gsr_glue.h).
//
//   map_loss_fwd    get_loss(mapping=True) image terms (scripts/splatam.py:262-296
//                   with use_l1, no silhouette mask): 0.8 * l1_loss_v1 +
//                   0.2 * (1 - calc_ssim) on the RGB render (gs_helpers.py:18-19,
//                   slam_external.py:66-97) and the masked mean depth L1.  One
//                   workgroup per 64x16 output tile of one channel: the 11x11
//                   Gaussian window is applied separably to the five moments
//                   (x, y, x^2, y^2, xy) from an LDS halo tile; the per-pixel
//                   SSIM partials dS/dmu1, dS/dE[x^2], dS/dE[xy] are written for
//                   the backward; loss sums published with agent-scope stores and
//                   added in a fixed order by the last workgroup.
//   map_loss_bwd    dL/dim = sum_q w(q-p) g(q) [dS/dmu1 + 2 x(p) dS/dE[x^2] +
//                   y(p) dS/dE[xy]] (the window is symmetric: the transpose of the
//                   zero-padded convolution is the same convolution of the partial
//                   maps), plus the L1 sign term; the depth gradient of the masked
//                   mean.  Same tile / halo structure.
//   map_transform_bwd   transform_to_frame(gaussians_grad=True, camera_grad=False)
//                   (utils/slam_helpers.py:252-304) + rendervar builders
//                   (slam_helpers.py:124-139, 196-213, 234-249) backward: one lane
//                   per Gaussian; optionally the Adam step of the mapping
//                   optimizer (scripts/splatam.py:166-172, eps 1e-15) applied in
//                   place, including the colour parameters (coalesced k*P + i).
//   adam_step       torch.optim.Adam (foreach form) over up to 16 tensors in one
//                   launch, float4 streams (HBM-bound).
#include <math.h>

#include <algorithm>

#include "../../include/gsr.h"
#include "../../include/gsr_glue.h"
#include "gsr_glue_common.h"

namespace gsr {
namespace {

// ------------------------------------------------------------- SSIM tiles --
constexpr int SS_TW = 64;                 // output tile width (one wave per row)
#ifndef GSR_SS_TH
#define GSR_SS_TH 16
#endif
constexpr int SS_TH = GSR_SS_TH;          // output tile height
constexpr int SS_R = 5;                   // window radius (window_size 11)
constexpr int SS_IW = SS_TW + 2 * SS_R;   // 74
constexpr int SS_BLOCK = 256;
constexpr float SS_C1 = 0.01f * 0.01f;
constexpr float SS_C2 = 0.03f * 0.03f;
constexpr int MAP_PARTS = 4;  // sum ssim, sum |x - y|, sum masked |d - gt|, mask count

struct Window {
    float w[2 * SS_R + 1];
};

// create_window(11, C) (slam_external.py:54-63): gaussian(11, 1.5) in float32,
// normalised by its float32 sum; the 2-D window is its outer product, applied
// here as two 1-D passes.
Window make_window() {
    Window win;
    float g[2 * SS_R + 1], s = 0.f;
    for (int k = 0; k <= 2 * SS_R; k++) {
        g[k] = (float)exp(-(double)((k - SS_R) * (k - SS_R)) / (2.0 * 1.5 * 1.5));
        s += g[k];
    }
    for (int k = 0; k <= 2 * SS_R; k++) win.w[k] = g[k] / s;
    return win;
}

__device__ __forceinline__ bool map_mask_v(float d, float dsq, float gt_depth) {
    const float unc = dsq - d * d;
    return gt_depth > 0.f && !isnan(d) && !isnan(unc);
}

__device__ __forceinline__ float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }

// Loads NM maps' (TH + 10) x (TW + 10) halo tiles of channel plane `c` into LDS,
// zero outside the image (conv2d zero padding).
// Every load of the thread's elements is issued before the first LDS store: a load-then-store
// loop waits one HBM round trip per element (the halo phase set the kernels' time).
template <int TH, int NM>
__device__ __forceinline__ void load_halo(float (*dst)[TH + 2 * SS_R][SS_IW], const float* const (&src)[NM], int H,
                                          int W, int x0, int y0) {
    constexpr int SS_IH = TH + 2 * SS_R;
    constexpr int NE = (SS_IH * SS_IW + SS_BLOCK - 1) / SS_BLOCK;
    float v[NE][NM];
#pragma unroll
    for (int i = 0; i < NE; i++) {
        const int e = (int)threadIdx.x + i * SS_BLOCK;
        const int r = e / SS_IW, cc = e - r * SS_IW;
        const int y = y0 - SS_R + r, x = x0 - SS_R + cc;
        const bool in = e < SS_IH * SS_IW && y >= 0 && y < H && x >= 0 && x < W;
#pragma unroll
        for (int m = 0; m < NM; m++) v[i][m] = in ? src[m][y * W + x] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NE; i++) {
        const int e = (int)threadIdx.x + i * SS_BLOCK;
        if (e < SS_IH * SS_IW) {
            const int r = e / SS_IW, cc = e - r * SS_IW;
#pragma unroll
            for (int m = 0; m < NM; m++) dst[m][r][cc] = v[i][m];
        }
    }
}

// Separable window: horizontal pass over the halo rows into hs, then each
// thread forms the vertical pass for SS_ROWS_PER_THREAD output rows of one column.
template <int TH, int NI, int NO, typename F>
__device__ __forceinline__ void horizontal_pass(const float (*src)[TH + 2 * SS_R][SS_IW],
                                                float (*hs)[TH + 2 * SS_R][SS_TW], const Window& win, F moments) {
    constexpr int SS_IH = TH + 2 * SS_R;
    for (int e = threadIdx.x; e < SS_IH * SS_TW; e += SS_BLOCK) {
        const int r = e / SS_TW, cc = e - r * SS_TW;
        float acc[NO];
#pragma unroll
        for (int m = 0; m < NO; m++) acc[m] = 0.f;
#pragma unroll
        for (int k = 0; k <= 2 * SS_R; k++) {
            float in[NI];
#pragma unroll
            for (int m = 0; m < NI; m++) in[m] = src[m][r][cc + k];
            float mo[NO];
            moments(in, mo);
#pragma unroll
            for (int m = 0; m < NO; m++) acc[m] += win.w[k] * mo[m];
        }
#pragma unroll
        for (int m = 0; m < NO; m++) hs[m][r][cc] = acc[m];
    }
}

template <int TH, int NO>
__device__ __forceinline__ void vertical_pass(const float (*hs)[TH + 2 * SS_R][SS_TW], const Window& win, int col,
                                              int r0, float (&out)[TH / (SS_BLOCK / SS_TW)][NO]) {
    constexpr int SS_ROWS_PER_THREAD = TH / (SS_BLOCK / SS_TW);
#pragma unroll
    for (int j = 0; j < SS_ROWS_PER_THREAD; j++)
#pragma unroll
        for (int m = 0; m < NO; m++) out[j][m] = 0.f;
#pragma unroll
    for (int rr = 0; rr < SS_ROWS_PER_THREAD + 2 * SS_R; rr++) {
        float v[NO];
#pragma unroll
        for (int m = 0; m < NO; m++) v[m] = hs[m][r0 + rr][col];
#pragma unroll
        for (int j = 0; j < SS_ROWS_PER_THREAD; j++) {
            const int k = rr - j;
            if (k >= 0 && k <= 2 * SS_R)
#pragma unroll
                for (int m = 0; m < NO; m++) out[j][m] += win.w[k] * v[m];
        }
    }
}

// gmap: 3 partial maps x 3 channels x HW floats; part: MAP_PARTS * nblocks
// partials then the arrival counters; out: [0] depth mask count (read by the backward).
template <int TH>
__global__ void __launch_bounds__(SS_BLOCK)
map_loss_fwd_kernel(int H, int W, const float* __restrict__ im, const float* __restrict__ ds,
                    const float* __restrict__ gt_im, const float* __restrict__ gt_d, float w_im, float w_depth,
                    Window win, float* __restrict__ gmap, float* __restrict__ part, float* __restrict__ out,
                    float* __restrict__ loss) {
    constexpr int SS_TH = TH, SS_IH = TH + 2 * SS_R, SS_ROWS_PER_THREAD = TH / (SS_BLOCK / SS_TW);
    __shared__ float s_in[2][SS_IH][SS_IW];
    __shared__ float s_h[5][SS_IH][SS_TW];
    __shared__ float s_red[4 * MAP_PARTS];
    __shared__ float s_tot[MAP_PARTS];
    const int HW = H * W, c = blockIdx.z;
    const int x0 = blockIdx.x * SS_TW, y0 = blockIdx.y * SS_TH;
    const float* const src[2] = {im + (size_t)c * HW, gt_im + (size_t)c * HW};
    const int col = threadIdx.x % SS_TW, r0 = (threadIdx.x / SS_TW) * SS_ROWS_PER_THREAD;
    const int x = x0 + col;
    // the depth term's inputs (channel-0 workgroups), loaded up front: a load issued after the
    // gmap stores would wait for them (vmcnt counts both)
    float pd[SS_ROWS_PER_THREAD], pdsq[SS_ROWS_PER_THREAD], pgd[SS_ROWS_PER_THREAD];
#pragma unroll
    for (int j = 0; j < SS_ROWS_PER_THREAD; j++) {
        const int y = y0 + r0 + j;
        pd[j] = pdsq[j] = pgd[j] = 0.f;
        if (c == 0 && x < W && y < H) {
            const int pid = y * W + x;
            pd[j] = ds[pid];
            pdsq[j] = ds[2 * HW + pid];
            pgd[j] = gt_d[pid];
        }
    }
    load_halo<TH, 2>(s_in, src, H, W, x0, y0);
    __syncthreads();
    horizontal_pass<TH, 2, 5>(s_in, s_h, win, [](const float (&i)[2], float (&o)[5]) {
        o[0] = i[0]; o[1] = i[1]; o[2] = i[0] * i[0]; o[3] = i[1] * i[1]; o[4] = i[0] * i[1];
    });
    __syncthreads();
    float mo[SS_ROWS_PER_THREAD][5];
    vertical_pass<TH, 5>(s_h, win, col, r0, mo);
    float v[MAP_PARTS] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < SS_ROWS_PER_THREAD; j++) {
        const int y = y0 + r0 + j;
        if (x >= W || y >= H) continue;
        // _ssim (slam_external.py:72-97), same operation order as the torch expression
        const float mu1 = mo[j][0], mu2 = mo[j][1];
        const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
        const float s11 = mo[j][2] - mu1_sq, s22 = mo[j][3] - mu2_sq, s12 = mo[j][4] - mu1_mu2;
        const float A = 2.f * mu1_mu2 + SS_C1, B = 2.f * s12 + SS_C2;
        const float C = mu1_sq + mu2_sq + SS_C1, D = s11 + s22 + SS_C2;
        const float ssim = (A * B) / (C * D);
        const float inv_cd = 1.f / (C * D);
        // dS/dmu1 (through s11 = E11 - mu1^2 and s12 = E12 - mu1 mu2), dS/dE11, dS/dE12
        const float g0 = 2.f * mu2 * (B - A) * inv_cd - 2.f * mu1 * ssim * (1.f / C - 1.f / D);
        const float g1 = -ssim / D;
        const float g2 = 2.f * A * inv_cd;
        const size_t o = (size_t)c * HW + (size_t)y * W + x;
        gmap[o] = g0;
        gmap[3 * (size_t)HW + o] = g1;
        gmap[6 * (size_t)HW + o] = g2;
        v[0] += ssim;
        v[1] += fabsf(s_in[0][r0 + j + SS_R][col + SS_R] - s_in[1][r0 + j + SS_R][col + SS_R]);
        if (c == 0 && map_mask_v(pd[j], pdsq[j], pgd[j])) {
            v[2] += fabsf(pgd[j] - pd[j]);
            v[3] += 1.f;
        }
    }
    block_sum<MAP_PARTS>(v, s_red, s_tot);
    __syncthreads();
    const int nb = gridDim.x * gridDim.y * gridDim.z;
    const int b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (threadIdx.x < MAP_PARTS) st_agent(part + MAP_PARTS * b + threadIdx.x, s_tot[threadIdx.x]);
    if (!last_block_arrive_grouped(reinterpret_cast<uint32_t*>(part + MAP_PARTS * nb))) return;
#pragma unroll
    for (int k = 0; k < MAP_PARTS; k++) v[k] = 0.f;
    gather_partials<MAP_PARTS, 8>(part, MAP_PARTS, nb, threadIdx.x, SS_BLOCK, v);
    __syncthreads();
    block_sum<MAP_PARTS>(v, s_red, s_tot);
    __syncthreads();
    if (threadIdx.x == 0) {
        const float n = 3.f * (float)HW;
        // losses['im'] = 0.8 * l1 + 0.2 * (1 - ssim); losses['depth'] = masked mean (nan when empty)
        const float l_im = 0.8f * (s_tot[1] / n) + 0.2f * (1.f - s_tot[0] / n);
        const float l_d = s_tot[2] / s_tot[3];
        loss[0] = w_im * l_im + w_depth * l_d;
        out[0] = s_tot[3];
    }
}

template <int TH>
__global__ void __launch_bounds__(SS_BLOCK)
map_loss_bwd_kernel(int H, int W, const float* __restrict__ im, const float* __restrict__ ds,
                    const float* __restrict__ gt_im, const float* __restrict__ gt_d, float w_im, float w_depth,
                    Window win, const float* __restrict__ gmap, const float* __restrict__ fwd_out,
                    const float* __restrict__ dloss, float* __restrict__ dim, float* __restrict__ dds) {
    constexpr int SS_TH = TH, SS_IH = TH + 2 * SS_R, SS_ROWS_PER_THREAD = TH / (SS_BLOCK / SS_TW);
    __shared__ float s_in[3][SS_IH][SS_IW];
    __shared__ float s_h[3][SS_IH][SS_TW];
    const int HW = H * W, c = blockIdx.z;
    const int x0 = blockIdx.x * SS_TW, y0 = blockIdx.y * SS_TH;
    const float* const src[3] = {gmap + (size_t)c * HW, gmap + 3 * (size_t)HW + (size_t)c * HW,
                                 gmap + 6 * (size_t)HW + (size_t)c * HW};
    const int col = threadIdx.x % SS_TW, r0 = (threadIdx.x / SS_TW) * SS_ROWS_PER_THREAD;
    const int x = x0 + col;
    // the epilogue's per-pixel inputs, loaded up front (ahead of the gradient stores)
    float pxi[SS_ROWS_PER_THREAD], pyi[SS_ROWS_PER_THREAD];
    float pd[SS_ROWS_PER_THREAD], pdsq[SS_ROWS_PER_THREAD], pgd[SS_ROWS_PER_THREAD];
#pragma unroll
    for (int j = 0; j < SS_ROWS_PER_THREAD; j++) {
        const int y = y0 + r0 + j;
        pxi[j] = pyi[j] = pd[j] = pdsq[j] = pgd[j] = 0.f;
        if (x < W && y < H) {
            const int pid = y * W + x;
            pxi[j] = im[(size_t)c * HW + pid];
            pyi[j] = gt_im[(size_t)c * HW + pid];
            if (c == 0) {
                pd[j] = ds[pid];
                pdsq[j] = ds[2 * HW + pid];
                pgd[j] = gt_d[pid];
            }
        }
    }
    load_halo<TH, 3>(s_in, src, H, W, x0, y0);
    __syncthreads();
    horizontal_pass<TH, 3, 3>(s_in, s_h, win, [](const float (&i)[3], float (&o)[3]) {
        o[0] = i[0]; o[1] = i[1]; o[2] = i[2];
    });
    __syncthreads();
    float bl[SS_ROWS_PER_THREAD][3];
    vertical_pass<TH, 3>(s_h, win, col, r0, bl);
    const float g = dloss[0];
    const float n = 3.f * (float)HW;
    const float g_ssim = g * w_im * (-0.2f / n);  // d/dS of w_im * 0.2 * (1 - mean(S))
    const float g_l1 = g * w_im * (0.8f / n);
    const float count = fwd_out[0];
    const float g_d = g * w_depth / count;
#pragma unroll
    for (int j = 0; j < SS_ROWS_PER_THREAD; j++) {
        const int y = y0 + r0 + j;
        if (x >= W || y >= H) continue;
        const int pid = y * W + x;
        const size_t o = (size_t)c * HW + pid;
        const float xi = pxi[j], yi = pyi[j];
        dim[o] = g_ssim * (bl[j][0] + 2.f * xi * bl[j][1] + yi * bl[j][2]) + g_l1 * sgn(xi - yi);
        if (c == 0) {  // d|gt - d|/dd = -sgn(gt - d), over the masked mean
            dds[pid] = map_mask_v(pd[j], pdsq[j], pgd[j]) ? g_d * neg_sgn(pgd[j] - pd[j]) : 0.f;
            dds[HW + pid] = 0.f;
            dds[2 * HW + pid] = 0.f;
        }
    }
}

// ------------------------------------------------------------------- Adam --
constexpr int ADAM_MAX = 16;
constexpr int ADAM_BLOCK = 256;
constexpr int ADAM_VEC_PER_BLOCK = ADAM_BLOCK * 4;  // float4 per thread, 4 per thread per block

struct AdamArgs {
    float* p[ADAM_MAX];
    const float* g[ADAM_MAX];
    float* m[ADAM_MAX];
    float* v[ADAM_MAX];
    long long n[ADAM_MAX];
    float step_size[ADAM_MAX];   // -lr / (1 - beta1^step)   (double on the host, like torch's python floats)
    int blk0[ADAM_MAX + 1];      // first workgroup of each tensor
    int nt;
    float w1;                    // 1 - beta1 (lerp weight)
    float beta2, omb2;           // beta2, 1 - beta2
    float bc2_sqrt, eps;
    int vec;                     // bit t: tensor t is 16-byte aligned in all four streams
};

// torch/optim/adam.py _multi_tensor_adam (capturable=False, no weight decay, no
// amsgrad): m.lerp_(g, 1 - b1); v.mul_(b2).addcmul_(g, g, 1 - b2);
// p.addcdiv_(m, sqrt(v) / sqrt(bc2) + eps, -lr / bc1).
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float ss, const AdamArgs& a) {
    m = m + a.w1 * (g - m);
    v = v * a.beta2;
    v = v + a.omb2 * g * g;
    const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
    p = p + ss * (m / denom);
}

__global__ void __launch_bounds__(ADAM_BLOCK) adam_step_kernel(AdamArgs a) {
    int t = 0;
    while (t + 1 < a.nt && (int)blockIdx.x >= a.blk0[t + 1]) t++;
    const long long n = a.n[t];
    const long long base = (long long)(blockIdx.x - a.blk0[t]) * ADAM_VEC_PER_BLOCK * 4;
    float* __restrict__ p = a.p[t];
    const float* __restrict__ g = a.g[t];
    float* __restrict__ m = a.m[t];
    float* __restrict__ v = a.v[t];
    const float ss = a.step_size[t];
    if ((a.vec >> t) & 1) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const long long i = base + 4 * ((long long)k * ADAM_BLOCK + threadIdx.x);
            if (i + 3 < n) {
                float4 P4 = *reinterpret_cast<const float4*>(p + i), G4 = ld_stream(reinterpret_cast<const float4*>(g + i));
                float4 M4 = ld_stream(reinterpret_cast<const float4*>(m + i));
                float4 V4 = ld_stream(reinterpret_cast<const float4*>(v + i));
                adam_elem(P4.x, G4.x, M4.x, V4.x, ss, a);
                adam_elem(P4.y, G4.y, M4.y, V4.y, ss, a);
                adam_elem(P4.z, G4.z, M4.z, V4.z, ss, a);
                adam_elem(P4.w, G4.w, M4.w, V4.w, ss, a);
                st_stream(reinterpret_cast<float4*>(p + i), P4);
                st_stream(reinterpret_cast<float4*>(m + i), M4);
                st_stream(reinterpret_cast<float4*>(v + i), V4);
            } else {
                for (long long e = i; e < n; e++) adam_elem(p[e], g[e], m[e], v[e], ss, a);
            }
        }
    } else {
        for (int k = 0; k < 16; k++) {
            const long long i = base + (long long)k * ADAM_BLOCK + threadIdx.x;
            if (i < n) adam_elem(p[i], g[i], m[i], v[i], ss, a);
        }
    }
}

// ---------------------------------------------------- mapping transform bwd --
#ifndef GSR_NT_GRADS
#define GSR_NT_GRADS 1  // (config 4: map_transform_bwd 66.5 -> 61.8 us, profiles/r9z_ab_nt_grads.txt)
#endif
struct MapAdam {  // the mapping optimizer's state, applied in place (NULL p: write gradients instead)
    float* p[5];          // means3D, unnorm_rotations, logit_opacities, log_scales, colours
    float* m[5];
    float* v[5];
    float step_size[5];
    float w1, beta2, omb2, bc2_sqrt, eps;
    const uint32_t* guard;  // status row of the iteration's forward: skip the step on an overflow
    uint32_t cap;
    uint32_t* halted;       // gsr_map_adam.halted (sticky skip), or nullptr
};

__device__ __forceinline__ float adam_apply(float* p, float g, float* m, float* v, float ss, const MapAdam& a) {
    float mm = ld_stream(m), vv = ld_stream(v);
    const float np = adam_update_elem(*p, g, mm, vv, ss, a.w1, a.beta2, a.omb2, a.bc2_sqrt, a.eps);
    st_stream(m, mm);
    st_stream(v, vv);
    st_stream(p, np);
    return np;
}

// adam_apply on N elements p[k * stride] (k < N): every load is issued before the first
// store (the pointers may alias as far as the compiler knows, so element-wise calls would
// serialise one memory round trip per element); same arithmetic, same results
template <int N>
__device__ __forceinline__ void adam_apply_n(float* p, const float* g, float* m, float* v, size_t stride, float ss,
                                             const MapAdam& a) {
    float pv[N], mv[N], vv[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        pv[k] = p[k * stride];
        mv[k] = ld_stream(m + k * stride);
        vv[k] = ld_stream(v + k * stride);
    }
#pragma unroll
    for (int k = 0; k < N; k++) {
        float mm = mv[k], v2 = vv[k];
        const float np = adam_update_elem(pv[k], g[k], mm, v2, ss, a.w1, a.beta2, a.omb2, a.bc2_sqrt, a.eps);
        st_stream(m + k * stride, mm);
        st_stream(v + k * stride, v2);
        st_stream(p + k * stride, np);
    }
}

// One lane per Gaussian.  Forward (gsr_track_transform_fwd): m = R p + t,
// rot = normalize(u) (isotropic) or normalize(quat_mult(c, normalize(u))),
// opac = sigmoid(lo), scales = exp(ls) (tiled when S = 1), depth colours
// [z, 1, z^2] with z = w2c[2,:3] . m + w2c[2,3].  Colours pass through
// unchanged (their gradient is only stepped when `adam` is set).
__global__ void __launch_bounds__(GLUE_BLOCK)
map_transform_bwd_kernel(int P, const float* ur, const float* lo, const float* ls, int scols, const float* __restrict__ cq, int qs,
                         const float* __restrict__ mc, const float* __restrict__ w2c, const float* __restrict__ gm,
                         const float* __restrict__ gr, const float* __restrict__ gd, const float* __restrict__ go,
                         const float* __restrict__ gs, float* __restrict__ dmeans, float* __restrict__ dur,
                         float* __restrict__ dlo, float* __restrict__ dls, const float* __restrict__ gcol, int ccols,
                         MapAdam adam) {
    // ur / lo / ls alias adam.p[1..3] in the Adam variant (updated in place): no __restrict__,
    // and every lane reads its own elements before it stores them
    const int i = blockIdx.x * GLUE_BLOCK + threadIdx.x;
    const bool step = adam.p[0] != nullptr;
    if (step && fused_step_skipped(adam.guard, adam.cap, adam.halted)) return;  // invalid gradients: nothing changes
    if (step && gcol && i < P) {  // colour parameters: element k * P + i (coalesced across the wave)
        constexpr int CU = 4;  // colour columns per round trip
        int k = 0;
        for (; k + CU <= ccols; k += CU) {
            const size_t e = (size_t)k * P + i;
            float g[CU];
#pragma unroll
            for (int j = 0; j < CU; j++) g[j] = gcol[e + (size_t)j * P];
            adam_apply_n<CU>(adam.p[4] + e, g, adam.m[4] + e, adam.v[4] + e, (size_t)P, adam.step_size[4], adam);
        }
        for (; k < ccols; k++) {
            const size_t e = (size_t)k * P + i;
            adam_apply(adam.p[4] + e, gcol[e], adam.m[4] + e, adam.v[4] + e, adam.step_size[4], adam);
        }
    }
    if (i >= P) return;
    const Pose ps = make_pose(cq, nullptr, qs);
    // (the incoming gradients and camera-frame means are read once: GSR_NT_GRADS streams them nontemporally)
    auto ldg = [](const float* q) { return GSR_NT_GRADS ? ld_stream(q) : *q; };
    float g0 = gm ? ldg(gm + 3 * i) : 0.f, g1 = gm ? ldg(gm + 3 * i + 1) : 0.f, g2 = gm ? ldg(gm + 3 * i + 2) : 0.f;
    if (gd) {  // colours [z, 1, z^2]: dz = dc0 + 2 z dc2
        const float z = w2c[8] * ldg(mc + 3 * i) + w2c[9] * ldg(mc + 3 * i + 1) + w2c[10] * ldg(mc + 3 * i + 2) + w2c[11];
        const float dz = ldg(gd + 3 * i) + 2.f * z * ldg(gd + 3 * i + 2);
        g0 += dz * w2c[8]; g1 += dz * w2c[9]; g2 += dz * w2c[10];
    }
    // m = R p + t  ->  dp = R^T g
    float dp[3];
#pragma unroll
    for (int k = 0; k < 3; k++) dp[k] = ps.R[0][k] * g0 + ps.R[1][k] * g1 + ps.R[2][k] * g2;
    float4 du = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gr) {
        float un_norm;
        const float4 u = normalize4(load4(ur + 4 * i), un_norm);
        float4 d = make_float4(ldg(gr + 4 * i), ldg(gr + 4 * i + 1), ldg(gr + 4 * i + 2), ldg(gr + 4 * i + 3));
        if (scols != 1) {  // rot = normalize(o), o = quat_mult(c, u): do -> du = quat_mult(c, .)^T do
            float o_norm;
            const float4 o = quat_mult(ps.c, u);
            const float4 r = normalize4(o, o_norm);
            const float4 dq = normalize4_bwd(r, o_norm, d);
            const float* c = ps.c;
            d = make_float4(c[0] * dq.x + c[1] * dq.y + c[2] * dq.z + c[3] * dq.w,
                            -c[1] * dq.x + c[0] * dq.y + c[3] * dq.z - c[2] * dq.w,
                            -c[2] * dq.x - c[3] * dq.y + c[0] * dq.z + c[1] * dq.w,
                            -c[3] * dq.x + c[2] * dq.y - c[1] * dq.z + c[0] * dq.w);
        }
        du = normalize4_bwd(u, un_norm, d);
    }
    float dl = 0.f;
    if (go) {  // sigmoid backward: g * (1 - y) * y
        const float y = 1.f / (1.f + expf(-lo[i]));
        dl = ldg(go + i) * ((1.f - y) * y);
    }
    float dsc[3] = {0.f, 0.f, 0.f};
    if (gs) {  // exp backward: g * exp(x); tile backward sums the three columns
        if (scols == 1) {
            const float e = expf(ls[i]);
            dsc[0] = ldg(gs + 3 * i) * e + ldg(gs + 3 * i + 1) * e + ldg(gs + 3 * i + 2) * e;
        } else {
#pragma unroll
            for (int k = 0; k < 3; k++) dsc[k] = ldg(gs + 3 * i + k) * expf(ls[3 * i + k]);
        }
    }
    if (!step) {
        dmeans[3 * i] = dp[0]; dmeans[3 * i + 1] = dp[1]; dmeans[3 * i + 2] = dp[2];
        if (dur) { dur[4 * i] = du.x; dur[4 * i + 1] = du.y; dur[4 * i + 2] = du.z; dur[4 * i + 3] = du.w; }
        if (dlo) dlo[i] = dl;
        if (dls) for (int k = 0; k < scols; k++) dls[scols * i + k] = dsc[k];
        return;
    }
    // The four groups' parameters and moments are all loaded before the first store: a load issued
    // after a store waits for the store too (vmcnt counts both on gfx950), so the group-by-group
    // form serialised one store round trip per group.  Same element update, same results.
    const float duv[4] = {du.x, du.y, du.z, du.w};
    float pv[11], mv[11], vv[11], gv[11];
    float* const p0 = adam.p[0] + 3 * i;
    float* const p1 = adam.p[1] + 4 * i;
    float* const p2 = adam.p[2] + i;
    float* const p3 = adam.p[3] + scols * i;
    float* const m0 = adam.m[0] + 3 * i;
    float* const m1 = adam.m[1] + 4 * i;
    float* const m2 = adam.m[2] + i;
    float* const m3 = adam.m[3] + scols * i;
    float* const v0 = adam.v[0] + 3 * i;
    float* const v1 = adam.v[1] + 4 * i;
    float* const v2 = adam.v[2] + i;
    float* const v3 = adam.v[3] + scols * i;
#pragma unroll
    for (int k = 0; k < 3; k++) { pv[k] = p0[k]; mv[k] = ld_stream(m0 + k); vv[k] = ld_stream(v0 + k); gv[k] = dp[k]; }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        pv[3 + k] = p1[k]; mv[3 + k] = ld_stream(m1 + k); vv[3 + k] = ld_stream(v1 + k); gv[3 + k] = duv[k];
    }
    pv[7] = *p2; mv[7] = ld_stream(m2); vv[7] = ld_stream(v2); gv[7] = dl;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const bool on = k < scols;
        pv[8 + k] = on ? p3[k] : 0.f;
        mv[8 + k] = on ? ld_stream(m3 + k) : 0.f;
        vv[8 + k] = on ? ld_stream(v3 + k) : 0.f;
        gv[8 + k] = dsc[k];
    }
#pragma unroll
    for (int e = 0; e < 11; e++) {
        const float ss = adam.step_size[e < 3 ? 0 : (e < 7 ? 1 : (e < 8 ? 2 : 3))];
        pv[e] = adam_update_elem(pv[e], gv[e], mv[e], vv[e], ss, adam.w1, adam.beta2, adam.omb2, adam.bc2_sqrt,
                                 adam.eps);
    }
    // stores grouped by array (adjacent elements of one array in a row), so they merge into
    // dwordx3 / dwordx4 stores: interleaving p / m / v stores (possibly aliasing) kept them dwords
#pragma unroll
    for (int k = 0; k < 3; k++) st_stream(p0 + k, pv[k]);
#pragma unroll
    for (int k = 0; k < 3; k++) st_stream(m0 + k, mv[k]);
#pragma unroll
    for (int k = 0; k < 3; k++) st_stream(v0 + k, vv[k]);
#pragma unroll
    for (int k = 0; k < 4; k++) st_stream(p1 + k, pv[3 + k]);
#pragma unroll
    for (int k = 0; k < 4; k++) st_stream(m1 + k, mv[3 + k]);
#pragma unroll
    for (int k = 0; k < 4; k++) st_stream(v1 + k, vv[3 + k]);
    st_stream(p2, pv[7]); st_stream(m2, mv[7]); st_stream(v2, vv[7]);
    if (scols == 3) {
#pragma unroll
        for (int k = 0; k < 3; k++) st_stream(p3 + k, pv[8 + k]);
#pragma unroll
        for (int k = 0; k < 3; k++) st_stream(m3 + k, mv[8 + k]);
#pragma unroll
        for (int k = 0; k < 3; k++) st_stream(v3 + k, vv[8 + k]);
    } else {
        st_stream(p3, pv[8]); st_stream(m3, mv[8]); st_stream(v3, vv[8]);
    }
}

// The SSIM tile height: 16 rows (3 workgroups per CU by their LDS), or 32 (2 per CU) when that takes the frame's
// tiles into one dispatch round and 16 rows would not -- config 3's 640x480: 900 -> 450 workgroups on 256 CUs
// (mapping 14.68 -> 14.45-14.50 ms per 60-iteration frame, profiles/r10q_seq_ssim_rows.txt); at 1200x680 the
// 32-row tiles measured slower (GSR_SS_TH timing builds)
int map_loss_rows(int H, int W) {
    if (SS_TH != 16) return SS_TH;  // (a timing build's fixed height)
    const long cols = (W + SS_TW - 1) / SS_TW, cus = current_device_cus();
    const long b16 = 3 * cols * ((H + 15) / 16), b32 = 3 * cols * ((H + 31) / 32);
    return (b16 > 3 * cus && b32 <= 2 * cus) ? 32 : 16;
}
int map_loss_blocks(int H, int W, dim3& grid, int rows) {
    grid = dim3((W + SS_TW - 1) / SS_TW, (H + rows - 1) / rows, 3);
    return (int)(grid.x * grid.y * grid.z);
}

// torch forms these scalars from python floats (double) and rounds them to float in the kernels
void fill_adam_common(double beta1, double beta2, double eps, int step, float& w1, float& b2, float& omb2,
                      float& bc2_sqrt, float& e) {
    w1 = (float)(1.0 - beta1);
    b2 = (float)beta2;
    omb2 = (float)(1.0 - beta2);
    bc2_sqrt = (float)sqrt(1.0 - pow(beta2, (double)step));
    e = (float)eps;
}

// prune_gaussians' removal test (utils/slam_external.py:174-181) as an in-place mask update: one lane per
// Gaussian; sigmoid and exp formed the way torch's elementwise kernels form them (ATen: 1 / (1 + exp(-x)) in
// float, expf), max over the scale columns with torch.max's NaN propagation
__global__ void map_prune_kernel(int P, const float* __restrict__ logit_opac, const float* __restrict__ log_scales,
                                 int scols, float opac_thr, float big_thr, int remove_big, uint8_t* __restrict__ alive) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P || alive[i] == 0) return;
    const float op = 1.0f / (1.0f + expf(-logit_opac[i]));
    bool rm = op < opac_thr;
    if (remove_big) {
        float m = expf(log_scales[(size_t)scols * i]);
        for (int k = 1; k < scols; k++) {
            const float v = expf(log_scales[(size_t)scols * i + k]);
            m = (v > m || isnan(v)) && !isnan(m) ? v : m;
        }
        rm = rm || m > big_thr;
    }
    if (rm) alive[i] = 0;
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

int gsr_map_loss_scratch_floats(int H, int W) {
    dim3 grid;  // (sized for the smaller row count: at least as many workgroups as the height chosen)
    return MAP_PARTS * map_loss_blocks(H, W, grid, std::min(SS_TH, 16)) + ARRIVE_GROUPED_WORDS;
}

int gsr_map_loss_state_floats(int H, int W) { return 9 * H * W + 4; }

int gsr_map_loss_fwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im, const float* gt_depth,
                     float w_im, float w_depth, float* loss, float* state, float* scratch, void* stream) {
    if (H <= 0 || W <= 0) return fail(GSR_ERR_INVALID_ARG, "map_loss_fwd: bad image size");
    if (!im || !depth_sil || !gt_im || !gt_depth || !loss || !state || !scratch)
        return fail(GSR_ERR_INVALID_ARG, "map_loss_fwd: null pointer");
    dim3 grid;
    const int rows = map_loss_rows(H, W);
    map_loss_blocks(H, W, grid, rows);
    float* out = state + 9 * (size_t)H * W;
    hipLaunchKernelGGL(rows == 32 ? map_loss_fwd_kernel<32> : map_loss_fwd_kernel<SS_TH>, grid, dim3(SS_BLOCK), 0, (hipStream_t)stream, H, W, im, depth_sil, gt_im,
                       gt_depth, w_im, w_depth, make_window(), state, scratch, out, loss);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "map_loss_fwd");
}

int gsr_map_loss_bwd(int H, int W, const float* im, const float* depth_sil, const float* gt_im, const float* gt_depth,
                     float w_im, float w_depth, const float* dL_dloss, const float* state, float* dL_dim,
                     float* dL_ddepth_sil, void* stream) {
    if (H <= 0 || W <= 0) return fail(GSR_ERR_INVALID_ARG, "map_loss_bwd: bad image size");
    if (!im || !depth_sil || !gt_im || !gt_depth || !dL_dloss || !state || !dL_dim || !dL_ddepth_sil)
        return fail(GSR_ERR_INVALID_ARG, "map_loss_bwd: null pointer");
    dim3 grid;
    const int rows = map_loss_rows(H, W);
    map_loss_blocks(H, W, grid, rows);
    hipLaunchKernelGGL(rows == 32 ? map_loss_bwd_kernel<32> : map_loss_bwd_kernel<SS_TH>, grid, dim3(SS_BLOCK), 0, (hipStream_t)stream, H, W, im, depth_sil, gt_im,
                       gt_depth, w_im, w_depth, make_window(), state, state + 9 * (size_t)H * W, dL_dloss, dL_dim,
                       dL_ddepth_sil);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "map_loss_bwd");
}

int gsr_map_transform_bwd(int P, const float* unnorm_rot, const float* logit_opac, const float* log_scales,
                          int scale_cols, const float* cam_q, int q_stride, const float* means_cam, const float* w2c,
                          const float* dL_dmeans_cam, const float* dL_drot, const float* dL_ddepth_colors,
                          const float* dL_dopac, const float* dL_dscales, float* dL_dmeans, float* dL_dunnorm_rot,
                          float* dL_dlogit_opac, float* dL_dlog_scales, void* stream) {
    if (P < 0 || (scale_cols != 1 && scale_cols != 3) || q_stride < 1)
        return fail(GSR_ERR_INVALID_ARG, "map_transform_bwd: bad sizes");
    if (P == 0) return GSR_OK;
    if (!unnorm_rot || !logit_opac || !log_scales || !cam_q || !w2c || !means_cam || !dL_dmeans)
        return fail(GSR_ERR_INVALID_ARG, "map_transform_bwd: null pointer");
    MapAdam none{};
    hipLaunchKernelGGL(map_transform_bwd_kernel, dim3((P + GLUE_BLOCK - 1) / GLUE_BLOCK), dim3(GLUE_BLOCK), 0,
                       (hipStream_t)stream, P, unnorm_rot, logit_opac, log_scales, scale_cols, cam_q, q_stride,
                       means_cam, w2c, dL_dmeans_cam, dL_drot, dL_ddepth_colors, dL_dopac, dL_dscales, dL_dmeans,
                       dL_dunnorm_rot, dL_dlogit_opac, dL_dlog_scales, nullptr, 0, none);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "map_transform_bwd");
}

int gsr_map_transform_bwd_adam(int P, float* means_world, float* unnorm_rot, float* logit_opac, float* log_scales,
                               int scale_cols, float* colors, int color_cols, const float* cam_q, int q_stride,
                               const float* means_cam, const float* w2c, const float* dL_dmeans_cam,
                               const float* dL_drot, const float* dL_ddepth_colors, const float* dL_dopac,
                               const float* dL_dscales, const float* dL_dcolors, const gsr_map_adam* adam,
                               void* stream) {
    if (P < 0 || (scale_cols != 1 && scale_cols != 3) || q_stride < 1 || color_cols < 0 || !adam || adam->step < 1)
        return fail(GSR_ERR_INVALID_ARG, "map_transform_bwd_adam: bad sizes");
    if (P == 0) return GSR_OK;
    if (!means_world || !unnorm_rot || !logit_opac || !log_scales || !cam_q || !w2c || !means_cam ||
        (dL_dcolors && !colors))
        return fail(GSR_ERR_INVALID_ARG, "map_transform_bwd_adam: null pointer");
    for (int k = 0; k < 5; k++)
        if (!adam->exp_avg[k] || !adam->exp_avg_sq[k])
            if (k < 4 || dL_dcolors) return fail(GSR_ERR_INVALID_ARG, "map_transform_bwd_adam: null optimizer state");
    MapAdam a{};
    float* ps[5] = {means_world, unnorm_rot, logit_opac, log_scales, colors};
    const double bc1 = 1.0 - pow(adam->beta1, (double)adam->step);
    for (int k = 0; k < 5; k++) {
        a.p[k] = ps[k];
        a.m[k] = adam->exp_avg[k];
        a.v[k] = adam->exp_avg_sq[k];
        a.step_size[k] = (float)(-adam->lr[k] / bc1);
    }
    fill_adam_common(adam->beta1, adam->beta2, adam->eps, adam->step, a.w1, a.beta2, a.omb2, a.bc2_sqrt, a.eps);
    a.guard = adam->status;
    a.cap = adam->capacity;
    a.halted = adam->halted;
    hipLaunchKernelGGL(map_transform_bwd_kernel, dim3((P + GLUE_BLOCK - 1) / GLUE_BLOCK), dim3(GLUE_BLOCK), 0,
                       (hipStream_t)stream, P, unnorm_rot, logit_opac, log_scales, scale_cols, cam_q, q_stride,
                       means_cam, w2c, dL_dmeans_cam, dL_drot, dL_ddepth_colors, dL_dopac, dL_dscales, nullptr,
                       nullptr, nullptr, nullptr, dL_dcolors, color_cols, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "map_transform_bwd_adam");
}

int gsr_map_prune(int P, const float* logit_opac, const float* log_scales, int scale_cols, float opac_thr,
                  float big_thr, int remove_big, unsigned char* alive, void* stream) {
    if (P < 0 || scale_cols < 1) return fail(GSR_ERR_INVALID_ARG, "map_prune: bad sizes");
    if (P == 0) return GSR_OK;
    if (!logit_opac || !alive || (remove_big && !log_scales)) return fail(GSR_ERR_INVALID_ARG, "map_prune: null pointer");
    hipLaunchKernelGGL(map_prune_kernel, dim3((P + 255) / 256), dim3(256), 0, (hipStream_t)stream, P, logit_opac,
                       log_scales, scale_cols, opac_thr, big_thr, remove_big, alive);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "map_prune");
}

int gsr_adam_step(int n_tensors, const gsr_adam_tensor* tensors, int step, double beta1, double beta2, double eps,
                  void* stream) {
    if (n_tensors < 0 || n_tensors > ADAM_MAX || step < 1 || (n_tensors > 0 && !tensors))
        return fail(GSR_ERR_INVALID_ARG, "adam_step: bad arguments (at most 16 tensors, step >= 1)");
    AdamArgs a{};
    const double bc1 = 1.0 - pow(beta1, (double)step);
    int blocks = 0, nt = 0;
    for (int t = 0; t < n_tensors; t++) {
        const gsr_adam_tensor& x = tensors[t];
        if (x.n < 0) return fail(GSR_ERR_INVALID_ARG, "adam_step: negative size");
        if (x.n == 0) continue;
        if (!x.param || !x.grad || !x.exp_avg || !x.exp_avg_sq) return fail(GSR_ERR_INVALID_ARG, "adam_step: null pointer");
        a.p[nt] = x.param; a.g[nt] = x.grad; a.m[nt] = x.exp_avg; a.v[nt] = x.exp_avg_sq; a.n[nt] = x.n;
        a.step_size[nt] = (float)(-x.lr / bc1);
        const bool al = ((uintptr_t)x.param | (uintptr_t)x.grad | (uintptr_t)x.exp_avg | (uintptr_t)x.exp_avg_sq) % 16 == 0;
        if (al) a.vec |= 1 << nt;
        a.blk0[nt] = blocks;
        blocks += (int)((x.n + 4LL * ADAM_VEC_PER_BLOCK - 1) / (4LL * ADAM_VEC_PER_BLOCK));
        nt++;
    }
    if (nt == 0) return GSR_OK;
    a.blk0[nt] = blocks;
    a.nt = nt;
    fill_adam_common(beta1, beta2, eps, step, a.w1, a.beta2, a.omb2, a.bc2_sqrt, a.eps);
    hipLaunchKernelGGL(adam_step_kernel, dim3(blocks), dim3(ADAM_BLOCK), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GSR_OK : hip_fail(e, "adam_step");
}

}  // extern "C"
