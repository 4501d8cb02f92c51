// gsr_sh.hip -- spherical-harmonics colour stages with coalesced coefficient traffic.
//
// A Gaussian's 3 * (D+1)^2 SH coefficients are 192 contiguous bytes at D = 3, so
// one lane per Gaussian reading or writing them directly touches 64 cache lines
// per wave instruction, 48 times over.  Here a 256-Gaussian workgroup moves its
// coefficient block between HBM and LDS as one contiguous float4 stream and each
// lane works on its own LDS row (row stride 3*NSH + 1 floats: odd, so the 64
// lanes of a wave hit 64 distinct banks).
//
//   sh_eval_kernel  computeColorFromSH (forward.cu:20-73) -> rgb (handed to preprocess
//                   in the binning record bin[i]) and the clamp bits, before preprocess;
//   sh_bwd_kernel   the SH part of preprocessCUDA's backward (backward.cu:20-139):
//                   dsh (staged in LDS, written as one float4 stream) and the
//                   view-direction term added to dL/dmeans3D, after gauss_bwd has
//                   written dL/dcolor into a scratch array.
#include "gsr_chain.h"
#include "gsr_glue_common.h"

namespace gsr {
namespace {

constexpr int SH_BLOCK = 256;
#ifndef GSR_SH_SPLIT
#define GSR_SH_SPLIT 1  // sh_bwd_split_kernel for the fused colour Adam step (config 4: 205 -> 195 us)
#endif
constexpr int SH_SPLIT_BLOCK = 128;
#ifndef GSR_SH_BWD_NT
#define GSR_SH_BWD_NT 0  // sh_bwd's coefficient staging with nontemporal loads (its Adam step re-reads them)
#endif
// sh_eval: one wave per workgroup (12.5 KB of LDS at D = 3): the waves of a CU stage and evaluate
// independently instead of in barrier-coupled groups of four

template <int NSH>
struct ShTile {
    static constexpr int ROW = 3 * NSH;      // floats per Gaussian
    static constexpr int PITCH = ROW + 1;    // LDS row pitch (odd: conflict-free per-lane rows)
};

// Global [n x ROW] block (contiguous: M == NSH) -> LDS rows.
// NT: nontemporal loads (sh_eval's coefficient stream, read once there; sh_bwd's staging keeps the plain
// loads: its colour Adam step re-reads the same coefficients right after)
template <int NSH, int BLK = SH_BLOCK, bool NT = false>
__device__ __forceinline__ void stage_rows(float* s, const float* __restrict__ src, int n, int tix = -1) {
    const int tt = tix < 0 ? (int)threadIdx.x : tix;  // the staging thread's index among BLK
    using T = ShTile<NSH>;
    const int total = n * T::ROW;
    if (T::ROW % 4 == 0 && (reinterpret_cast<uintptr_t>(src) & 15u) == 0) {
        const float4* s4 = reinterpret_cast<const float4*>(src);
        if (n == BLK) {  // full block: every lane's ROW/4 loads issued before the first LDS store
            constexpr int IT = T::ROW / 4 > 0 ? T::ROW / 4 : 1;  // float4 per lane (ROW % 4 == 0 here)
            float4 v[IT];
#pragma unroll
            for (int k = 0; k < IT; k++) v[k] = NT ? ld_stream(s4 + tt + k * BLK) : s4[tt + k * BLK];
#pragma unroll
            for (int k = 0; k < IT; k++) {
                const int e = 4 * (tt + k * BLK), r = e / T::ROW, c = e - r * T::ROW;
                float* d = s + r * T::PITCH + c;
                d[0] = v[k].x; d[1] = v[k].y; d[2] = v[k].z; d[3] = v[k].w;
            }
            return;
        }
        for (int e4 = tt; 4 * e4 < total; e4 += BLK) {
            const float4 v = s4[e4];
            const int e = 4 * e4, r = e / T::ROW, c = e - r * T::ROW;  // ROW % 4 == 0: no row straddle
            float* d = s + r * T::PITCH + c;
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
    } else {
        for (int e = tt; e < total; e += BLK) {
            const int r = e / T::ROW, c = e - r * T::ROW;
            s[r * T::PITCH + c] = src[e];
        }
    }
}

template <int NSH>
__device__ __forceinline__ void unstage_rows(float* __restrict__ dst, const float* s, int n) {
    using T = ShTile<NSH>;
    const int total = n * T::ROW;
    if (T::ROW % 4 == 0 && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        float4* d4 = reinterpret_cast<float4*>(dst);
        for (int e4 = threadIdx.x; 4 * e4 < total; e4 += SH_BLOCK) {
            const int e = 4 * e4, r = e / T::ROW, c = e - r * T::ROW;
            const float* q = s + r * T::PITCH + c;
            d4[e4] = make_float4(q[0], q[1], q[2], q[3]);
        }
    } else {
        for (int e = threadIdx.x; e < total; e += SH_BLOCK) {
            const int r = e / T::ROW, c = e - r * T::ROW;
            dst[e] = s[r * T::PITCH + c];
        }
    }
}

// The colour Adam step over the workgroup's [n x ROW] block, gradients from the LDS rows: the
// parameters (the SH coefficients the block staged, updated in place), exp_avg and exp_avg_sq move
// as float4 streams.  The element update is adam_update_elem, as in map_transform_bwd's colour step, so
// fusing it here changes no bit of the optimizer's result.
template <int NSH>
__device__ __forceinline__ void adam_rows(float* p, float* m, float* v, const float* s, int n, const ShAdam& a) {
    using T = ShTile<NSH>;
    const int total = n * T::ROW;
    auto elem = [&](float& pp, float g, float& mm_, float& vv_) {
        pp = adam_update_elem(pp, g, mm_, vv_, a.ss, a.w1, a.beta2, a.omb2, a.bc2_sqrt, a.eps);
    };
    const bool vec = T::ROW % 4 == 0 && ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(m) |
                                          reinterpret_cast<uintptr_t>(v)) & 15u) == 0;
    if (vec) {
        float4* p4 = reinterpret_cast<float4*>(p);
        float4* m4 = reinterpret_cast<float4*>(m);
        float4* v4 = reinterpret_cast<float4*>(v);
        constexpr int U = 4;  // float4 groups per round trip: U loads of p, m and v in flight before the stores
        int e4 = threadIdx.x;
        for (; 4 * (e4 + (U - 1) * SH_BLOCK) < total; e4 += U * SH_BLOCK) {
            float4 pv[U], mv[U], vv[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                pv[u] = GSR_SH_BWD_NT ? ld_stream(p4 + e4 + u * SH_BLOCK) : p4[e4 + u * SH_BLOCK];
                mv[u] = ld_stream(m4 + e4 + u * SH_BLOCK);
                vv[u] = ld_stream(v4 + e4 + u * SH_BLOCK);
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int e = 4 * (e4 + u * SH_BLOCK), r = e / T::ROW, c = e - r * T::ROW;
                const float* q = s + r * T::PITCH + c;
                elem(pv[u].x, q[0], mv[u].x, vv[u].x);
                elem(pv[u].y, q[1], mv[u].y, vv[u].y);
                elem(pv[u].z, q[2], mv[u].z, vv[u].z);
                elem(pv[u].w, q[3], mv[u].w, vv[u].w);
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                st_stream(m4 + e4 + u * SH_BLOCK, mv[u]);
                st_stream(v4 + e4 + u * SH_BLOCK, vv[u]);
                st_stream(p4 + e4 + u * SH_BLOCK, pv[u]);
            }
        }
        for (; 4 * e4 < total; e4 += SH_BLOCK) {
            const int e = 4 * e4, r = e / T::ROW, c = e - r * T::ROW;
            const float* q = s + r * T::PITCH + c;
            float4 pv = p4[e4], mv = ld_stream(m4 + e4), vv = ld_stream(v4 + e4);
            elem(pv.x, q[0], mv.x, vv.x);
            elem(pv.y, q[1], mv.y, vv.y);
            elem(pv.z, q[2], mv.z, vv.z);
            elem(pv.w, q[3], mv.w, vv.w);
            st_stream(m4 + e4, mv);
            st_stream(v4 + e4, vv);
            st_stream(p4 + e4, pv);
        }
    } else {
        for (int e = threadIdx.x; e < total; e += SH_BLOCK) {
            const int r = e / T::ROW, c = e - r * T::ROW;
            float pv = p[e], mv = m[e], vv = v[e];
            elem(pv, s[r * T::PITCH + c], mv, vv);
            m[e] = mv;
            v[e] = vv;
            p[e] = pv;
        }
    }
}

// adam_rows with the parameters taken from the workgroup's own LDS copy (s_p, the staged coefficients)
// instead of re-reading them from HBM: only exp_avg / exp_avg_sq are read (the same bits: s_p holds what
// the block staged).  BLK lanes, gradients in s_g.
template <int NSH, int BLK>
__device__ __forceinline__ void adam_rows_lds(float* p, float* m, float* v, const float* s_p, const float* s_g, int n,
                                              const ShAdam& a) {
    using T = ShTile<NSH>;
    const int total = n * T::ROW;
    auto elem = [&](float& pp, float g, float& mm_, float& vv_) {
        pp = adam_update_elem(pp, g, mm_, vv_, a.ss, a.w1, a.beta2, a.omb2, a.bc2_sqrt, a.eps);
    };
    float4* p4 = reinterpret_cast<float4*>(p);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    constexpr int U = 4;
    int e4 = threadIdx.x;
    for (; 4 * (e4 + (U - 1) * BLK) < total; e4 += U * BLK) {
        float4 pv[U], mv[U], vv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            mv[u] = ld_stream(m4 + e4 + u * BLK);
            vv[u] = ld_stream(v4 + e4 + u * BLK);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int e = 4 * (e4 + u * BLK), r = e / T::ROW, c = e - r * T::ROW;
            const float* q = s_g + r * T::PITCH + c;
            const float* pp = s_p + r * T::PITCH + c;
            pv[u] = make_float4(pp[0], pp[1], pp[2], pp[3]);
            elem(pv[u].x, q[0], mv[u].x, vv[u].x);
            elem(pv[u].y, q[1], mv[u].y, vv[u].y);
            elem(pv[u].z, q[2], mv[u].z, vv[u].z);
            elem(pv[u].w, q[3], mv[u].w, vv[u].w);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            st_stream(m4 + e4 + u * BLK, mv[u]);
            st_stream(v4 + e4 + u * BLK, vv[u]);
            st_stream(p4 + e4 + u * BLK, pv[u]);
        }
    }
    for (; 4 * e4 < total; e4 += BLK) {
        const int e = 4 * e4, r = e / T::ROW, c = e - r * T::ROW;
        const float* q = s_g + r * T::PITCH + c;
        const float* pp = s_p + r * T::PITCH + c;
        float4 pv = make_float4(pp[0], pp[1], pp[2], pp[3]), mv = ld_stream(m4 + e4), vv = ld_stream(v4 + e4);
        elem(pv.x, q[0], mv.x, vv.x);
        elem(pv.y, q[1], mv.y, vv.y);
        elem(pv.z, q[2], mv.z, vv.z);
        elem(pv.w, q[3], mv.w, vv.w);
        st_stream(m4 + e4, mv);
        st_stream(v4 + e4, vv);
        st_stream(p4 + e4, pv);
    }
}

template <int NSH>
__global__ void __launch_bounds__(64) sh_eval_kernel(Camera cam, GaussIn g, GeomPtrs geo) {
    using T = ShTile<NSH>;
    __shared__ float s_sh[64 * T::PITCH];
    const int lane = threadIdx.x;
    const int base = blockIdx.x * 64;
    const int n = min(64, g.P - base);
    if (n <= 0) return;
    const int i = base + lane;
    const bool act = lane < n;
    // the lane's mean is loaded with the staging stream, not after it
    const float3 p = act ? make_float3(g.means3D[3 * i], g.means3D[3 * i + 1], g.means3D[3 * i + 2])
                         : make_float3(0.f, 0.f, 0.f);
    stage_rows<NSH, 64, true>(s_sh, g.shs + (size_t)T::ROW * base, n);
    __syncthreads();
    if (!act) return;
    float rgb[3];
    unsigned clamped = 0;
    sh_fwd(cam.sh_degree, p, cam.campos, s_sh + lane * T::PITCH, rgb, clamped);
    // handed to preprocess through bin[i] (dense 16-B rows, one full line per 4 Gaussians; preprocess
    // reads it first and overwrites it with the binning record) instead of the render record's rgb slot
    // (16 B every 64 B: partial-line writes here, 64-B line reads there)
    geo.bin[i] = make_uint4(__float_as_uint(rgb[0]), __float_as_uint(rgb[1]), __float_as_uint(rgb[2]), 0u);
    geo.clamp[i] = clamped;
}

// drgb: [P,3] dL/dcolor (unmasked) from gauss_bwd; dmeans3D: += view-direction term.
template <int NSH>
__global__ void __launch_bounds__(SH_BLOCK)
sh_bwd_kernel(Camera cam, GaussIn g, GeomPtrs geo, const int* __restrict__ radii, const float* __restrict__ drgb,
              float* __restrict__ dmeans3D, float* __restrict__ dsh, BwdGuard guard, ShAdam sa) {
    using T = ShTile<NSH>;
    __shared__ float s_sh[SH_BLOCK * T::PITCH];
    const int base = blockIdx.x * SH_BLOCK;
    const int n = min(SH_BLOCK, g.P - base);
    stage_rows<NSH, SH_BLOCK, GSR_SH_BWD_NT != 0>(s_sh, g.shs + (size_t)T::ROW * base, n);
    __syncthreads();
    if ((int)threadIdx.x < n) {
        const int i = base + threadIdx.x;
        float* row = s_sh + threadIdx.x * T::PITCH;
        if (radii[i] > 0 && !guard.overflow()) {
            const float3 m = make_float3(g.means3D[3 * i], g.means3D[3 * i + 1], g.means3D[3 * i + 2]);
            const float d[3] = {drgb[3 * i], drgb[3 * i + 1], drgb[3 * i + 2]};
            float dmean[3] = {dmeans3D[3 * i], dmeans3D[3 * i + 1], dmeans3D[3 * i + 2]};
            float dsh_r[T::ROW];
            sh_chain_bwd(cam, m, row, d, geo.clamp[i], dsh_r, dmean);
#pragma unroll
            for (int k = 0; k < T::ROW; k++) row[k] = dsh_r[k];  // own row: no other lane reads it
#pragma unroll
            for (int k = 0; k < 3; k++) dmeans3D[3 * i + k] = dmean[k];
        } else {
#pragma unroll
            for (int k = 0; k < T::ROW; k++) row[k] = 0.f;
        }
    }
    __syncthreads();
    if (sa.m) {  // the colour Adam step in place of the dsh round trip through HBM
        if (fused_step_skipped(sa.guard, sa.cap, sa.halted)) return;  // overflowing forward (or an earlier skip): no step
        const size_t o = (size_t)T::ROW * base;
        adam_rows<NSH>(const_cast<float*>(g.shs) + o, sa.m + o, sa.v + o, s_sh, n, sa);
    } else if (dsh) {
        unstage_rows<NSH>(dsh + (size_t)T::ROW * base, s_sh, n);
    }
}

// sh_bwd with the colour Adam step reading the coefficients from LDS: the gradient rows go to a second LDS
// array (two 128-Gaussian blocks of rows, 50 KB at D = 3), so the staged coefficients survive the chain
// and the step reads only the two moments from HBM (192 MB less per config-4 iteration than re-reading the
// coefficients).  Same element update, same bits.
template <int NSH>
__global__ void __launch_bounds__(SH_SPLIT_BLOCK)
sh_bwd_split_kernel(Camera cam, GaussIn g, GeomPtrs geo, const int* __restrict__ radii, const float* __restrict__ drgb,
                    float* __restrict__ dmeans3D, float* __restrict__ dsh, BwdGuard guard, ShAdam sa) {
    using T = ShTile<NSH>;
    constexpr int BLK = SH_SPLIT_BLOCK;
    __shared__ float s_sh[BLK * T::PITCH];
    __shared__ float s_g[BLK * T::PITCH];
    const int base = blockIdx.x * BLK;
    const int n = min(BLK, g.P - base);
    stage_rows<NSH, BLK>(s_sh, g.shs + (size_t)T::ROW * base, n);
    __syncthreads();
    if ((int)threadIdx.x < n) {
        const int i = base + threadIdx.x;
        const float* row = s_sh + threadIdx.x * T::PITCH;
        float* grow = s_g + threadIdx.x * T::PITCH;
        if (radii[i] > 0 && !guard.overflow()) {
            const float3 m = make_float3(g.means3D[3 * i], g.means3D[3 * i + 1], g.means3D[3 * i + 2]);
            const float d[3] = {drgb[3 * i], drgb[3 * i + 1], drgb[3 * i + 2]};
            float dmean[3] = {dmeans3D[3 * i], dmeans3D[3 * i + 1], dmeans3D[3 * i + 2]};
            float dsh_r[T::ROW];
            sh_chain_bwd(cam, m, row, d, geo.clamp[i], dsh_r, dmean);
#pragma unroll
            for (int k = 0; k < T::ROW; k++) grow[k] = dsh_r[k];
#pragma unroll
            for (int k = 0; k < 3; k++) dmeans3D[3 * i + k] = dmean[k];
        } else {
#pragma unroll
            for (int k = 0; k < T::ROW; k++) grow[k] = 0.f;
        }
    }
    __syncthreads();
    if (sa.m) {
        if (fused_step_skipped(sa.guard, sa.cap, sa.halted)) return;
        const size_t o = (size_t)T::ROW * base;
        adam_rows_lds<NSH, BLK>(const_cast<float*>(g.shs) + o, sa.m + o, sa.v + o, s_sh, s_g, n, sa);
    } else if (dsh) {
        const int total = n * T::ROW;
        for (int e = threadIdx.x; e < total; e += BLK) {
            const int r = e / T::ROW, c = e - r * T::ROW;
            dsh[(size_t)T::ROW * base + e] = s_g[r * T::PITCH + c];
        }
    }
}

template <int NSH>
hipError_t launch_sh_eval_t(const Camera& cam, const GaussIn& g, GeomPtrs geo, hipStream_t s) {
    constexpr int per = 64;
    hipLaunchKernelGGL(sh_eval_kernel<NSH>, dim3((g.P + per - 1) / per), dim3(per), 0, s, cam, g, geo);
    return hipGetLastError();
}

template <int NSH>
hipError_t launch_sh_bwd_t(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii, const float* drgb,
                           float* dmeans3D, float* dsh, BwdGuard guard, hipStream_t s, const ShAdam& sa) {
    using T = ShTile<NSH>;
    const bool aligned = ((reinterpret_cast<uintptr_t>(g.shs) | reinterpret_cast<uintptr_t>(sa.m) |
                           reinterpret_cast<uintptr_t>(sa.v)) & 15u) == 0;
    if (GSR_SH_SPLIT && sa.m && T::ROW % 4 == 0 && aligned) {  // (the float4 form of adam_rows_lds)
        hipLaunchKernelGGL(sh_bwd_split_kernel<NSH>, dim3((g.P + SH_SPLIT_BLOCK - 1) / SH_SPLIT_BLOCK),
                           dim3(SH_SPLIT_BLOCK), 0, s, cam, g, geo, radii, drgb, dmeans3D, dsh, guard, sa);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(sh_bwd_kernel<NSH>, dim3((g.P + SH_BLOCK - 1) / SH_BLOCK), dim3(SH_BLOCK), 0, s, cam, g, geo,
                       radii, drgb, dmeans3D, dsh, guard, sa);
    return hipGetLastError();
}

}  // namespace

// The staged kernels need M == (D+1)^2 (coefficient rows contiguous); otherwise the
// per-lane paths (preprocess / gauss_chain) keep handling SH.
bool sh_staged(const Camera& cam, const GaussIn& g) {
    return g.shs && cam.sh_degree >= 0 && cam.sh_degree <= 3 && g.M == (cam.sh_degree + 1) * (cam.sh_degree + 1);
}

hipError_t launch_sh_eval(const Camera& cam, const GaussIn& g, GeomPtrs geo, hipStream_t s) {
    if (g.P == 0) return hipSuccess;
    switch (cam.sh_degree) {
        case 0: return launch_sh_eval_t<1>(cam, g, geo, s);
        case 1: return launch_sh_eval_t<4>(cam, g, geo, s);
        case 2: return launch_sh_eval_t<9>(cam, g, geo, s);
        default: return launch_sh_eval_t<16>(cam, g, geo, s);
    }
}

hipError_t launch_sh_bwd(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii, const float* drgb,
                         float* dmeans3D, float* dsh, BwdGuard guard, hipStream_t s, const ShAdam& sa) {
    if (g.P == 0) return hipSuccess;
    switch (cam.sh_degree) {
        case 0: return launch_sh_bwd_t<1>(cam, g, geo, radii, drgb, dmeans3D, dsh, guard, s, sa);
        case 1: return launch_sh_bwd_t<4>(cam, g, geo, radii, drgb, dmeans3D, dsh, guard, s, sa);
        case 2: return launch_sh_bwd_t<9>(cam, g, geo, radii, drgb, dmeans3D, dsh, guard, s, sa);
        default: return launch_sh_bwd_t<16>(cam, g, geo, radii, drgb, dmeans3D, dsh, guard, s, sa);
    }
}

}  // namespace gsr
