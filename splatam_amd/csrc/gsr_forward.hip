// gsr_forward.hip -- forward pipeline of the MI355X-native Gaussian rasterizer.
//
//   preprocess  (forward.cu:155-256)     one lane per Gaussian, writes 48-B render records
//   scan        (rasterizer_impl.cu:277)  per-workgroup tile sums -> exclusive scan
//   duplicate   (rasterizer_impl.cu:70-111) load-balanced: a workgroup emits the
//               instances of its 256 Gaussians with consecutive lanes on consecutive
//               instances (binary search in LDS), so writes are coalesced
//   radix sort  (rasterizer_impl.cu:301-309) stable 8-bit LSD passes, wave64 ballot
//               match ranking (no atomics), values = unsorted instance index
//   ranges      (rasterizer_impl.cu:116-138) + point_list gather of Gaussian ids
//   render      (forward.cu:261-393) 16x16 tile per 256-lane workgroup, 256-entry
//               LDS batches, block-wide early exit
#include <cstdlib>

#include "gsr_glue_common.h"  // (includes gsr_common.h) track_xform_compute / _store: the transform-fused preprocess
#include "gsr_diag.h"
#include "gsr_render_fwd.h"

#ifndef GSR_CULL_TAIL
#define GSR_CULL_TAIL 1  // culled instances written to point_list's tail (0: timing experiments only)
#endif

namespace gsr {

constexpr bool kCullTail = GSR_CULL_TAIL != 0;


// ------------------------------------------------------------- preprocess --
// LDS_HIST: per-tile instance counts go to a workgroup histogram in LDS and
// leave as one row of the [workgroup x tile] matrix `counts` (no global
// atomics: ~680k scattered global atomics cost ~30 us on MI355X whatever their
// contention, tools/micro/atomics.hip).  Otherwise: global atomics on padded
// per-tile counters (fallback for > MAX_LDS_TILES tiles).
// XF: SplaTAM's tracking transform fused in (g.xf, TrackXf): the camera-frame rendervars are
// formed here from the world-frame map and the pose, and stored to g's arrays for the backward.
// CLK: the in-kernel stage clock (a separate instantiation: the production launches carry none of it)
// EXACT: the per-workgroup culled-instance counts of the dynamic forward's exact list tail (Camera::tail_exact);
// a separate instantiation because the bookkeeping, even skipped at run time, cost the static mapping
// preprocess 45 -> 58 us in code generation (profiles/r9y_ab_preprocess_tail.txt)
template <bool LDS_HIST, bool XF, bool CLK, bool EXACT>
__global__ void __launch_bounds__(PRE_BLOCK)
preprocess_kernel(Camera cam, GaussIn g, GeomPtrs geo, int* radii, uint32_t* __restrict__ counts, int ntiles,
                  unsigned long long* clk) {
#pragma clang fp contract(off)
    if (cam.gate.off()) return;
    if constexpr (CLK) kclock_begin(clk);  // (stage clock: first workgroup's start to the last one's end)
    extern __shared__ uint32_t s_hist[];
    __shared__ float s_pose[16];  // XF: the frame's pose (R 9, t 3, F.normalize(q) 4), formed once by wave 0
    const int i = (blockIdx.x << cam.pre_shift) + threadIdx.x;  // blockDim.x = 1 << pre_shift
    XfRaw xr{};  // XF: the Gaussian's transform inputs, in flight while wave 0 forms the pose
    if (XF && i < g.P) xr = track_xform_load(g.xf, i, true);
    // the per-Gaussian inputs used only once the rect is known (colour, opacity, second colour set)
    // are loaded here too, not after the projection: one memory round trip fewer per workgroup
    // (not in the transform-fused tracking form, where the early loads measured 0.6 us slower)
    float pre_rgb[3] = {0.f, 0.f, 0.f}, pre_c2[3] = {0.f, 0.f, 0.f}, pre_op = 0.f;
    if (!XF && i < g.P) {
        if (g.colors) {
            pre_rgb[0] = g.colors[3 * i]; pre_rgb[1] = g.colors[3 * i + 1]; pre_rgb[2] = g.colors[3 * i + 2];
        } else if (g.sh_staged) {  // sh_eval_kernel wrote rgb (in bin[i], overwritten below) and the clamp bits
            const uint4 c = geo.bin[i];
            pre_rgb[0] = __uint_as_float(c.x); pre_rgb[1] = __uint_as_float(c.y); pre_rgb[2] = __uint_as_float(c.z);
        }
        pre_op = g.opacities[i];
        if (g.colors2) {
            pre_c2[0] = g.colors2[3 * i]; pre_c2[1] = g.colors2[3 * i + 1]; pre_c2[2] = g.colors2[3 * i + 2];
        }
    }
    if (XF && threadIdx.x < 64) {
        const Pose ps = make_pose(g.xf.cq, g.xf.ct, g.xf.qs);
        if (threadIdx.x == 0) {
#pragma unroll
            for (int k = 0; k < 9; k++) s_pose[k] = ps.R[k / 3][k % 3];
#pragma unroll
            for (int k = 0; k < 3; k++) s_pose[9 + k] = ps.t[k];
#pragma unroll
            for (int k = 0; k < 4; k++) s_pose[12 + k] = ps.c[k];
        }
    }
    if (LDS_HIST)
        for (int t = threadIdx.x; t < ntiles; t += blockDim.x) s_hist[t] = 0u;
    if (LDS_HIST || XF) __syncthreads();
    if (i == 0) geo.counters[4] = 0u;  // tile_colscan_kernel's arrival counter (next launch)
    uint32_t tiles = 0, culled = 0;  // culled: rect tiles left out of the lists (Camera::cull)
    bool violation = false;  // prefiltered set but the point is culled (auxiliary.h:154-160)
    float4 q0, q1, q2, q3;
    if (i < g.P) {
        int radius = 0;
        float3 p;
        float xs[3], xc2[3], xop = 0.f;
        float4 xq;
        if (XF) {  // gsr_track_transform_fwd's outputs, formed in registers (and stored for the backward)
            Pose ps;  // (track_xform_compute reads R, t and c)
#pragma unroll
            for (int k = 0; k < 9; k++) ps.R[k / 3][k % 3] = s_pose[k];
#pragma unroll
            for (int k = 0; k < 3; k++) ps.t[k] = s_pose[9 + k];
#pragma unroll
            for (int k = 0; k < 4; k++) ps.c[k] = s_pose[12 + k];
            float m[3];
            track_xform_compute_raw(g.xf, xr, ps, m, xq, xc2, xop, xs);  // (stored below, after every load)
            p = make_float3(m[0], m[1], m[2]);
        } else {
            p = make_float3(g.means3D[3 * i], g.means3D[3 * i + 1], g.means3D[3 * i + 2]);
        }
        float4 hom = xform4x4(p, cam.proj);
        float pw = 1.0f / (hom.w + 0.0000001f);
        float3 pv = xform4x3(p, cam.view);
        bool ok = pv.z > 0.001f;  // auxiliary.h:154 (the 1.3 NDC test is commented out)
        if (!ok && cam.prefiltered) violation = true;
        // a pruned Gaussian (alive mask, prune_gaussians inside a captured mapping frame) is culled like one
        // behind the camera: radius 0, no instances, zero gradients -- the survivors render and
        // differentiate exactly as after remove_points (utils/slam_external.py:141-163)
        if (g.alive != nullptr && g.alive[i] == 0) ok = false;
        float cov3[6];
        Proj pj;
        float det = 0.f, ca = 0.f, cb = 0.f, cc = 0.f;
        if (ok) {
            if (g.cov3D) {
#pragma unroll
                for (int k = 0; k < 6; k++) cov3[k] = g.cov3D[6 * i + k];
            } else {
                float3 s = XF ? make_float3(xs[0], xs[1], xs[2])
                              : make_float3(g.scales[3 * i], g.scales[3 * i + 1], g.scales[3 * i + 2]);
                float4 q = XF ? xq : make_float4(g.rotations[4 * i], g.rotations[4 * i + 1], g.rotations[4 * i + 2],
                                                 g.rotations[4 * i + 3]);
                cov3d_fwd(s, cam.scale_modifier, q, cov3);
            }
            cov2d_fwd(p, cam.focal_x, cam.focal_y, cam.tan_fovx, cam.tan_fovy, cov3, cam.view, pj);
            det = conic_of(pj, ca, cb, cc);
            ok = det != 0.0f;
        }
        if (ok) {
            float mid = 0.5f * (pj.a + pj.c);
            float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
            float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
            float rad = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
            float px = ndc2pix(hom.x * pw, cam.W), py = ndc2pix(hom.y * pw, cam.H);
            int x0, y0, x1, y1;
            get_rect(px, py, (int)rad, cam.gx, cam.gy, x0, y0, x1, y1);
            tiles = (uint32_t)((x1 - x0) * (y1 - y0));
            if (tiles != 0) {
                float rgb[3] = {pre_rgb[0], pre_rgb[1], pre_rgb[2]};
                unsigned clamped = 0;
                if (XF && g.colors) {
                    rgb[0] = g.colors[3 * i]; rgb[1] = g.colors[3 * i + 1]; rgb[2] = g.colors[3 * i + 2];
                } else if (XF && g.sh_staged) {
                    const uint4 c = geo.bin[i];
                    rgb[0] = __uint_as_float(c.x); rgb[1] = __uint_as_float(c.y); rgb[2] = __uint_as_float(c.z);
                } else if (!g.colors && !g.sh_staged) {
                    sh_fwd(cam.sh_degree, p, cam.campos, g.shs + (size_t)3 * g.M * i, rgb, clamped);
                }
                radius = (int)rad;
                float c2[3] = {0.f, 0.f, 0.f};
                if (XF) {
                    c2[0] = xc2[0]; c2[1] = xc2[1]; c2[2] = xc2[2];
                } else if (g.colors2) {
                    c2[0] = pre_c2[0]; c2[1] = pre_c2[1]; c2[2] = pre_c2[2];
                }
                const uint32_t rlo = (uint32_t)x0 | ((uint32_t)y0 << 16), rhi = (uint32_t)x1 | ((uint32_t)y1 << 16);
                q0 = make_float4(px, py, K_AC * ca, K_AC * cc);  // render-record conic form
                q2 = make_float4(rgb[0], rgb[1], rgb[2], __uint_as_float(rlo));
                q3 = make_float4(c2[0], c2[1], c2[2], __uint_as_float(rhi));
                if (XF) {  // (tracking form: three quarters now, q1 after the scan measured 0.7 us faster)
                    float4* rr = geo.rr + (size_t)RR_F4 * i;
                    rr[0] = q0;
                    rr[2] = q2;
                    rr[3] = q3;
                }
                q1 = make_float4(K_B * cb, XF ? xop : pre_op, pv.z, 0.f);  // .w: workgroup-local instance offset, below
                // live-tile mask (Camera::cull): the render's own conservative block-mask test per rect tile
                uint32_t live = 0xFFFFFFFFu;
                if (cam.cull && tiles <= 32u) {
                    const MaskGeom mg = mask_geom(q0, q1);
                    live = 0u;
                    for (int ty = y0, k = 0; ty < y1; ty++)
                        for (int tx = x0; tx < x1; tx++, k++)
                            live |= (GSR_CULL_EXACT ? mask_of_geom(mg, (float)(tx * TILE_X), (float)(ty * TILE_Y)) != 0u
                                                    : tile_reached(mg, (float)(tx * TILE_X), (float)(ty * TILE_Y)))
                                        ? 1u << k : 0u;
                }
                if constexpr (kCullTail && EXACT) culled = culled_below(live, tiles);
                geo.bin[i] = make_uint4(rlo, rhi, __float_as_uint(pv.z), live);
                if (!g.sh_staged && !g.colors) geo.clamp[i] = clamped;  // (read only by the SH backward)
                for (int ty = y0, k = 0; ty < y1; ty++)  // per-tile instance counts -> bucket ranges
                    for (int tx = x0; tx < x1; tx++, k++) {
                        if (!tile_live(live, (uint32_t)k)) continue;
                        if (LDS_HIST) atomicAdd(&s_hist[ty * cam.gx + tx], 1u);
                        else atomicAdd(&counts[(ty * cam.gx + tx) * TILE_CTR_STRIDE], 1u);
                    }
            }
        }
        radii[i] = radius;
        geo.tiles[i] = tiles;
        if (tiles == 0) geo.bin[i] = make_uint4(0u, 0u, 0u, 0u);
        if (XF && g.xf.store) {  // the rendervars for the backward (the same values as gsr_track_transform_fwd's)
            const float m[3] = {p.x, p.y, p.z};
            track_xform_store(i, m, xq, xc2, xop, xs, const_cast<float*>(g.means3D), const_cast<float*>(g.rotations),
                              const_cast<float*>(g.colors2), const_cast<float*>(g.opacities),
                              const_cast<float*>(g.scales));
        }
    }
    // workgroup scan of tiles touched: the local instance offset goes into the render
    // record (q1.w; the render kernels add the scanned workgroup base, blocksums[i >> pre_shift]),
    // the workgroup total into wgsum (input of the two-level scan)
    __shared__ uint32_t wsum[PRE_BLOCK / 64], wcul[PRE_BLOCK / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t incl = wave_incl_scan(tiles);
    if (lane == 63) wsum[wv] = incl;
    if constexpr (kCullTail && EXACT) {  // the workgroup's culled instances (the exact tail, duplicate)
        const uint32_t cincl = wave_incl_scan(culled);
        if (lane == 63) wcul[wv] = cincl;
    }
    __syncthreads();
    uint32_t woff = 0;
    for (int k = 0; k < wv; k++) woff += wsum[k];
    if (tiles) {
        q1.w = __uint_as_float(woff + incl - tiles);
        float4* rr = geo.rr + (size_t)RR_F4 * i;
        if (!XF) {  // the whole 64-B record in one go, one full line (two partial writes of the line took
            rr[0] = q0;  // mapping's preprocess 49.7 us, this 41.5)
            rr[2] = q2;
            rr[3] = q3;
        }
        rr[1] = q1;
    }
    // top bit: prefiltered violation anywhere in the workgroup (folded into counters[1] by the scan)
    const bool viol = __syncthreads_or(violation);
    if (threadIdx.x == blockDim.x - 1) {
        geo.wgsum[blockIdx.x] = (woff + incl) | (viol ? 0x80000000u : 0u);
        if constexpr (kCullTail && EXACT) {
            uint32_t cw = 0;
            for (int k = 0; k < (int)(blockDim.x >> 6); k++) cw += wcul[k];
            geo.wgcull[blockIdx.x] = cw;
        }
    }
    if (LDS_HIST)
        for (int t = threadIdx.x; t < ntiles; t += blockDim.x) counts[(size_t)blockIdx.x * ntiles + t] = s_hist[t];
    if constexpr (CLK) kclock_end(clk);
}

hipError_t launch_preprocess(const Camera& cam, const GaussIn& g, GeomPtrs geo, int* radii, uint32_t* counts,
                             bool lds_hist, int ntiles, int nb, hipStream_t s, unsigned long long* clk) {
    if (nb == 0) return hipSuccess;
    const bool xf = g.xf.mw != nullptr;
    const bool exact = cam.tail_exact && cam.cull && !xf;  // (the transform-fused form is static-only)
    auto k = clk ? (lds_hist ? (xf ? preprocess_kernel<true, true, true, false>
                                   : (exact ? preprocess_kernel<true, false, true, true>
                                            : preprocess_kernel<true, false, true, false>))
                             : (xf ? preprocess_kernel<false, true, true, false>
                                   : (exact ? preprocess_kernel<false, false, true, true>
                                            : preprocess_kernel<false, false, true, false>)))
                 : (lds_hist ? (xf ? preprocess_kernel<true, true, false, false>
                                   : (exact ? preprocess_kernel<true, false, false, true>
                                            : preprocess_kernel<true, false, false, false>))
                             : (xf ? preprocess_kernel<false, true, false, false>
                                   : (exact ? preprocess_kernel<false, false, false, true>
                                            : preprocess_kernel<false, false, false, false>)));
    hipLaunchKernelGGL(k, dim3(nb), dim3(1 << cam.pre_shift), lds_hist ? sizeof(uint32_t) * ntiles : 0, s, cam, g,
                       geo, radii, counts, ntiles, clk);
    return hipGetLastError();
}

// Column scan of the [workgroup x tile] count matrix: in place, every entry
// becomes the workgroup's offset inside its tile's bucket; tot[t] = tile total.
// One workgroup per 16 tiles, 64 row segments each (coalesced across tiles): a
// frame's 1200 tiles give 75 workgroups, and a thread's <= CS_RQ column entries
// are loaded once, all in flight, and kept in registers for the offset pass
// (the previous 64-tile x 16-segment shape ran 19 workgroups of two dependent
// load passes: 16.5 us at config 3).
// Two shapes: 16 tiles x 64 parts (64-B row segments) for count matrices of <= 512 rows, 32 x 32
// (128-B segments, <= 32 rows per thread) above: 5.2 vs 5.8 us at config 3 (293 rows), 19.1 vs
// 16.2 us at config 4 (977 rows).
#ifndef GSR_CS_ROWS_SMALL
#define GSR_CS_ROWS_SMALL 640  // (config 3 has 586 rows of 512 Gaussians)
#endif
constexpr int CS_THREADS = 1024, CS_ROWS_SMALL = GSR_CS_ROWS_SMALL;
template <int CT>
struct ColscanShape {
    static constexpr int TILES = CT, PARTS = CS_THREADS / CT, RQ = PARTS == 64 ? 16 : 32;
};
template <bool AGENT_TILES>
__device__ void scan_counts_body(const uint32_t* __restrict__ wgsum, uint32_t* __restrict__ blocksums, uint32_t nb,
                                 const uint32_t* __restrict__ tile_count, uint32_t tile_stride, uint32_t ntiles,
                                 uint2* __restrict__ ranges, uint32_t* __restrict__ counters, uint32_t sort_cap,
                                 uint32_t* __restrict__ status);
constexpr int SCAN_THREADS = 1024;
constexpr int SCAN_ITEMS = 4;

// TAIL: ... and, in the same launch, the scan of scan_counts_kernel: the
// workgroups publish their tile totals (agent-scope stores), the last one to
// finish scans the workgroup sums and the tile totals (the arrival counter is
// GeomLayout counters[4], zeroed by preprocess).  Without TAIL (the bucketed
// path) every duplicate_bucket workgroup does those scans itself in its
// prologue, which removes this launch's serial tail (arrival + one-workgroup
// scan: ~10 us of latency at config 3).
template <bool TAIL, int CT>
__device__ __forceinline__ void tile_colscan_body(uint32_t* __restrict__ counts, int nb, int ntiles,
                                                  uint32_t* __restrict__ tot, GeomPtrs geo, uint2* __restrict__ ranges,
                                                  uint32_t sort_cap, uint32_t* __restrict__ status) {
    constexpr int CS_TILES = ColscanShape<CT>::TILES, CS_PARTS = ColscanShape<CT>::PARTS, CS_RQ = ColscanShape<CT>::RQ;
    __shared__ uint32_t s_part[CS_PARTS][CS_TILES];
    const int tl = threadIdx.x % CS_TILES, q = threadIdx.x / CS_TILES;
    const int t = blockIdx.x * CS_TILES + tl;
    const int rq = (nb + CS_PARTS - 1) / CS_PARTS;
    const int b0 = min(nb, q * rq), b1 = min(nb, b0 + rq);
    uint32_t sum = 0;
    uint32_t vals[CS_RQ];
    const bool in_regs = rq <= CS_RQ;
    if (t < ntiles) {
        if (in_regs) {
#pragma unroll
            for (int k = 0; k < CS_RQ; k++) {
                vals[k] = b0 + k < b1 ? counts[(size_t)(b0 + k) * ntiles + t] : 0u;
                sum += vals[k];
            }
        } else {
#pragma unroll 4
            for (int b = b0; b < b1; b++) sum += counts[(size_t)b * ntiles + t];
        }
    }
    s_part[q][tl] = sum;
    __syncthreads();
    {  // each wave scans 64 / CS_PARTS tile columns' part sums (lane = part) in place: exclusive prefixes
        static_assert(CS_PARTS == 64 || CS_PARTS == 32, "one or two tile columns per wave");
        constexpr int CPW = 64 / CS_PARTS;  // columns per wave
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int part = lane % CS_PARTS, colw = CPW * w + lane / CS_PARTS;
        const uint32_t v = s_part[part][colw];
        uint32_t inc = wave_incl_scan(v);
        if (CPW == 2) {  // the upper half-wave's column starts after the lower column's total
            const uint32_t lo_tot = (uint32_t)__shfl((int)inc, 31);
            if (lane >= 32) inc -= lo_tot;
        }
        s_part[part][colw] = inc - v;
    }
    __syncthreads();
    uint32_t run = s_part[q][tl];
    if (t < ntiles) {
        if (in_regs) {
#pragma unroll
            for (int k = 0; k < CS_RQ; k++)
                if (b0 + k < b1) {
                    counts[(size_t)(b0 + k) * ntiles + t] = run;
                    run += vals[k];
                }
        } else {
#pragma unroll 4
            for (int b = b0; b < b1; b++) {
                const uint32_t v = counts[(size_t)b * ntiles + t];
                counts[(size_t)b * ntiles + t] = run;
                run += v;
            }
        }
        if (q == CS_PARTS - 1) {
            if (TAIL) st_agent(&tot[t], run);
            else tot[t] = run;
        }
    }
    if (!TAIL) return;
    if (!last_block_arrive(&geo.counters[4])) return;
    scan_counts_body<true>(geo.wgsum, geo.blocksums, (uint32_t)nb, tot, 1u, (uint32_t)ntiles, ranges, geo.counters,
                           sort_cap, status);
}
template <bool TAIL, int CT, bool CLK>
__global__ void __launch_bounds__(CS_THREADS)
tile_colscan_kernel(uint32_t* __restrict__ counts, int nb, int ntiles, uint32_t* __restrict__ tot, GeomPtrs geo,
                    uint2* __restrict__ ranges, uint32_t sort_cap, uint32_t* __restrict__ status,
                    unsigned long long* clk, Gate gate) {
    if (gate.off()) return;
    if constexpr (CLK) kclock_begin(clk);
    tile_colscan_body<TAIL, CT>(counts, nb, ntiles, tot, geo, ranges, sort_cap, status);
    if constexpr (CLK) kclock_end(clk);
}

hipError_t launch_tile_colscan(uint32_t* counts, int nb, int ntiles, uint32_t* tot, GeomPtrs geo, uint2* ranges,
                               uint32_t* status, bool tail, hipStream_t s, unsigned long long* clk, Gate gate) {
    static_assert(CS_THREADS == SCAN_THREADS, "the last colscan workgroup runs the scan body");
    const int ct = nb <= CS_ROWS_SMALL ? 16 : 32;
    auto k = clk ? (tail ? (ct == 16 ? tile_colscan_kernel<true, 16, true> : tile_colscan_kernel<true, 32, true>)
                         : (ct == 16 ? tile_colscan_kernel<false, 16, true> : tile_colscan_kernel<false, 32, true>))
                 : (tail ? (ct == 16 ? tile_colscan_kernel<true, 16, false> : tile_colscan_kernel<true, 32, false>)
                         : (ct == 16 ? tile_colscan_kernel<false, 16, false> : tile_colscan_kernel<false, 32, false>));
    hipLaunchKernelGGL(k, dim3((ntiles + ct - 1) / ct), dim3(CS_THREADS), 0, s, counts, nb, ntiles, tot, geo, ranges,
                       (uint32_t)TILE_SORT_CAP, status, clk, gate);
    return hipGetLastError();
}

// -------------------------------------------------------- exclusive scan --
// One 1024-lane workgroup scans `n` u32 in place (exclusive) and writes the
// grand total.  Used for the per-workgroup tile sums and radix histograms.
__global__ void __launch_bounds__(SCAN_THREADS) exclusive_scan_kernel(uint32_t* data, uint32_t n, uint32_t* total) {
    __shared__ uint32_t wsums[SCAN_THREADS / 64];
    __shared__ uint32_t s_carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += SCAN_THREADS * SCAN_ITEMS) {
        uint32_t x[SCAN_ITEMS], sum = 0;
        const uint32_t i0 = base + (uint32_t)tid * SCAN_ITEMS;
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; k++) {
            x[k] = (i0 + k < n) ? data[i0 + k] : 0u;
            sum += x[k];
        }
        uint32_t incl = wave_incl_scan(sum);
        if (lane == 63) wsums[w] = incl;
        __syncthreads();
        if (w == 0) {
            uint32_t ws = (lane < SCAN_THREADS / 64) ? wsums[lane] : 0u;
            uint32_t wi = wave_incl_scan(ws);
            if (lane < SCAN_THREADS / 64) wsums[lane] = wi - ws;  // exclusive wave offsets
        }
        __syncthreads();
        uint32_t carry = s_carry;
        uint32_t run = carry + wsums[w] + incl - sum;
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; k++) {
            if (i0 + k < n) data[i0 + k] = run;
            run += x[k];
        }
        __syncthreads();
        if (tid == SCAN_THREADS - 1) s_carry = run;
        __syncthreads();
    }
    if (tid == 0 && total) *total = s_carry;
}

hipError_t launch_exclusive_scan(uint32_t* data, uint32_t n, uint32_t* total, hipStream_t s) {
    hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(SCAN_THREADS), 0, s, data, n, total);
    return hipGetLastError();
}

// One workgroup: exclusive scan of the per-workgroup tile sums (instance
// offsets, total = num_rendered) and of the per-tile instance counts, which
// directly gives every tile's [start, end) in the tile-major sorted list
// (identifyTileRanges, rasterizer_impl.cu:116-138, without reading keys).
// AGENT_TILES: the tile counts were published by other workgroups of the same
// launch (tile_colscan_kernel's last workgroup) and are read with agent-scope loads.
template <bool AGENT_TILES>
__device__ void scan_counts_body(const uint32_t* __restrict__ wgsum, uint32_t* __restrict__ blocksums, uint32_t nb,
                                 const uint32_t* __restrict__ tile_count, uint32_t tile_stride, uint32_t ntiles,
                                 uint2* __restrict__ ranges, uint32_t* __restrict__ counters, uint32_t sort_cap,
                                 uint32_t* __restrict__ status) {
    // Writes all four counters (no reset needed): [0] num_rendered, [1] prefiltered violation
    // (top bits of the workgroup sums), [2] longest tile list, [3] sort_cap; and a copy to
    // `status` (static mode).
    __shared__ uint32_t wsums[SCAN_THREADS / 64];
    __shared__ uint32_t s_carry, s_max, s_viol;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_viol = 0;
    for (int pass = 0; pass < 2; pass++) {
        const uint32_t n = pass == 0 ? nb : ntiles;
        const uint32_t* src = pass == 0 ? wgsum : tile_count;
        if (tid == 0) { s_carry = 0; s_max = 0; }
        __syncthreads();
        uint32_t vmax = 0, viol = 0;
        for (uint32_t base = 0; base < n; base += SCAN_THREADS * SCAN_ITEMS) {
            uint32_t x[SCAN_ITEMS], sum = 0;
            const uint32_t i0 = base + (uint32_t)tid * SCAN_ITEMS;
#pragma unroll
            for (int k = 0; k < SCAN_ITEMS; k++) {
                const uint32_t* ps = src + (size_t)(i0 + k) * (pass == 0 ? 1u : tile_stride);
                x[k] = (i0 + k < n) ? ((AGENT_TILES && pass == 1) ? ld_agent(ps) : *ps) : 0u;
                if (pass == 0) {  // workgroup sums carry the prefiltered-violation flag in bit 31
                    viol |= x[k] >> 31;
                    x[k] &= 0x7fffffffu;
                }
                sum += x[k];
                vmax = max(vmax, x[k]);
            }
            uint32_t incl = wave_incl_scan(sum);
            if (lane == 63) wsums[w] = incl;
            __syncthreads();
            if (w == 0) {
                uint32_t ws = (lane < SCAN_THREADS / 64) ? wsums[lane] : 0u;
                uint32_t wi = wave_incl_scan(ws);
                if (lane < SCAN_THREADS / 64) wsums[lane] = wi - ws;
            }
            __syncthreads();
            uint32_t run = s_carry + wsums[w] + incl - sum;
#pragma unroll
            for (int k = 0; k < SCAN_ITEMS; k++) {
                if (i0 + k < n) {
                    if (pass == 0) blocksums[i0 + k] = run;
                    else ranges[i0 + k] = make_uint2(run, run + x[k]);
                }
                run += x[k];
            }
            __syncthreads();
            if (tid == SCAN_THREADS - 1) s_carry = run;
            __syncthreads();
        }
        atomicMax(&s_max, vmax);
        if (viol) atomicOr(&s_viol, 1u);
        __syncthreads();
        if (tid == 0) {
            if (pass == 0) {
                counters[0] = s_carry;
                counters[1] = s_viol;
                if (status) status_merge(status, s_carry, s_viol, 0u, 0u);
            } else {
                counters[2] = s_max;
                counters[3] = sort_cap;  // longest list the tile sort will handle (BwdGuard)
                if (status) status_merge(status, 0u, 0u, s_max, sort_cap);
            }
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(SCAN_THREADS)
scan_counts_kernel(const uint32_t* __restrict__ wgsum, uint32_t* __restrict__ blocksums, uint32_t nb,
                   const uint32_t* __restrict__ tile_count,
                   uint32_t tile_stride, uint32_t ntiles, uint2* __restrict__ ranges,
                   uint32_t* __restrict__ counters, uint32_t sort_cap, uint32_t* __restrict__ status) {
    scan_counts_body<false>(wgsum, blocksums, nb, tile_count, tile_stride, ntiles, ranges, counters, sort_cap, status);
}

hipError_t launch_scan_counts(GeomPtrs geo, int nb, const uint32_t* tile_count, int tile_stride, int ntiles,
                              uint2* ranges, uint32_t* status, hipStream_t s) {
    hipLaunchKernelGGL(scan_counts_kernel, dim3(1), dim3(SCAN_THREADS), 0, s, geo.wgsum, geo.blocksums, (uint32_t)nb,
                       tile_count,
                       (uint32_t)tile_stride, (uint32_t)ntiles, ranges, geo.counters, (uint32_t)TILE_SORT_CAP,
                       status);
    return hipGetLastError();
}

// -------------------------------------------------------------- duplicate --
__global__ void __launch_bounds__(PRE_BLOCK)
duplicate_kernel(Camera cam, int P, GeomPtrs geo, uint64_t* __restrict__ keys, uint32_t* __restrict__ gid) {
    __shared__ uint32_t s_incl[PRE_BLOCK];   // inclusive scan of tiles touched
    __shared__ uint32_t s_x0[PRE_BLOCK], s_y0[PRE_BLOCK], s_w[PRE_BLOCK], s_depth[PRE_BLOCK], s_live[PRE_BLOCK];
    __shared__ uint32_t wsum[PRE_BLOCK / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, R = (int)blockDim.x;  // R = 1 << pre_shift
    const int i = (blockIdx.x << cam.pre_shift) + tid;
    uint32_t t = (i < P) ? geo.tiles[i] : 0u;
    uint32_t incl = wave_incl_scan(t);
    if (lane == 63) wsum[w] = incl;
    if (t) {
        const uint4 r = geo.bin[i];  // (rect lo, rect hi, depth bits, tiles)
        s_x0[tid] = r.x & 0xFFFFu;
        s_y0[tid] = r.x >> 16;
        s_w[tid] = (r.y & 0xFFFFu) - (r.x & 0xFFFFu);
        s_depth[tid] = r.z;
        s_live[tid] = r.w;
    }
    __syncthreads();
    uint32_t woff = 0;
    for (int k = 0; k < w; k++) woff += wsum[k];
    incl += woff;
    s_incl[tid] = incl;
    const uint32_t base = geo.blocksums[blockIdx.x];  // exclusive scan of workgroup totals
    if (i < P) geo.offsets[i] = base + incl - t;
    __syncthreads();
    const uint32_t total = s_incl[R - 1];
    for (uint32_t e = tid; e < total; e += R) {
        // owner j: first Gaussian whose inclusive sum exceeds e
        int lo = 0, hi = R - 1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (s_incl[mid] > e) hi = mid; else lo = mid + 1;
        }
        const uint32_t start = (lo == 0) ? 0u : s_incl[lo - 1];
        const uint32_t local = e - start;
        const uint32_t wdt = s_w[lo];
        const uint32_t ty = s_y0[lo] + local / wdt;
        const uint32_t tx = s_x0[lo] + local % wdt;
        const uint32_t u = base + e;
        const uint32_t gi = (blockIdx.x << cam.pre_shift) + lo;
        // a culled instance (Camera::cull) sorts behind every tile (tile id gx * gy, within the sorted bits), so
        // the live ones take the positions the culled tile counts' ranges give them
        const uint32_t tkey = tile_live(s_live[lo], local) ? ty * (uint32_t)cam.gx + tx : (uint32_t)(cam.gx * cam.gy);
        keys[u] = ((uint64_t)tkey << 32) | (uint64_t)s_depth[lo];
        gid[u] = gi;
    }
}

hipError_t launch_duplicate(const Camera& cam, int P, GeomPtrs geo, uint64_t* keys, uint32_t* gid,
                            int nb, hipStream_t s) {
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(duplicate_kernel, dim3(nb), dim3(1 << cam.pre_shift), 0, s, cam, P, geo, keys, gid);
    return hipGetLastError();
}

// Bucketed duplicate: every instance goes straight into its tile's bucket
// (slot from a per-tile cursor), keyed (depth bits << 32 | Gaussian id).  The
// order inside a bucket is arbitrary; render_fwd (tile_sort_bucket) restores the reference
// order (depth, then id: cub's stable LSD sort, rasterizer_impl.cu:304-309).
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v += (uint32_t)__shfl_xor((int)v, m);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, m));
    return v;
}

// ---- render schedule ---------------------------------------------------------
// All of a frame's render workgroups are resident at once (e.g. 1200 tiles on 256
// CUs at 5 workgroups per CU), workgroup i is dispatched to XCD i mod 8 and, inside
// it, round-robin over the XCD's CUs: workgroups i and i + ncu share a CU.  A render
// kernel therefore lasts as long as its most loaded CU (measured: the per-CU sum of
// tile work spread 0.81-1.18x of the mean with the row-major order, kernel span set
// by the top; tools/wgtime.py).  tile_plan deals the tiles, in descending order of
// list length (the render cost: 0.998 correlation with the tile's contributing
// pairs), to workgroup slots in rounds, alternating direction, so every CU's tiles
// add up to about the same work.  With n = q * ncu + m tiles, m CUs render q + 1
// tiles and ncu - m render q (config 3: 176 CUs x 5, 80 x 4; the per-CU end times
// follow the tile count first, `profiles/r4s_wgtime_fused.json`): the CUs with q
// tiles take the q (ncu - m) longest lists, dealt over their own q rounds, and the
// others the rest over q + 1 rounds.  Counting sort over length buckets of 4: ties
// land in arbitrary order, which changes only which workgroup renders a tile, never
// its results.
constexpr int PLAN_BUCKETS = 1024, PLAN_SHIFT = 2;
__device__ __forceinline__ uint32_t plan_bucket(uint32_t len) {  // descending length -> ascending bucket
    return (uint32_t)(PLAN_BUCKETS - 1) - min(len >> PLAN_SHIFT, (uint32_t)(PLAN_BUCKETS - 1));
}
__device__ __forceinline__ uint32_t plan_slot(uint32_t p, uint32_t n, uint32_t ncu) {
    const uint32_t q = n / ncu, m = n - q * ncu, heavy = q * (ncu - m);
    // group: CUs [g0, g0 + gs) (slot s renders on CU class s mod ncu), pp = position inside the group
    const bool hv = p < heavy;
    const uint32_t g0 = hv ? m : 0u, gs = hv ? ncu - m : m, pp = hv ? p : p - heavy;
    const uint32_t rd = pp / gs, k = pp - rd * gs;
    return rd * ncu + g0 + ((rd & 1u) ? gs - 1u - k : k);
}
// one workgroup of NT threads (PLAN_BUCKETS / NT consecutive buckets per thread); s_hist:
// PLAN_BUCKETS words of LDS, s_wsum: NT / 64
// TPT > 0: the tile totals come from registers, tv[k] = total of tile t0 + k (t0 + k < t1) -- no
// reload of `tot` after the caller's stores (a load issued after a store waits for it too)
template <int NT, int TPT = 0>
__device__ void tile_plan(const uint32_t* __restrict__ tot, int ntiles, int ncu, uint32_t* __restrict__ order,
                          uint32_t* s_hist, uint32_t* s_wsum, const uint32_t* tv = nullptr, int t0 = 0,
                          int t1 = 0) {
    constexpr int BPT = PLAN_BUCKETS / NT;
    static_assert(BPT * NT == PLAN_BUCKETS, "buckets per thread");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int k = 0; k < BPT; k++) s_hist[tid * BPT + k] = 0u;
    __syncthreads();
    if constexpr (TPT > 0) {
#pragma unroll
        for (int k = 0; k < TPT; k++)
            if (t0 + k < t1) atomicAdd(&s_hist[plan_bucket(tv[k])], 1u);
    } else {
        for (int u = tid; u < ntiles; u += NT) atomicAdd(&s_hist[plan_bucket(tot[u])], 1u);
    }
    __syncthreads();
    uint32_t c[BPT], cs = 0;
#pragma unroll
    for (int k = 0; k < BPT; k++) {
        c[k] = s_hist[tid * BPT + k];
        cs += c[k];
    }
    const uint32_t incl = wave_incl_scan(cs);
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    uint32_t run = incl - cs;
    for (int k = 0; k < w; k++) run += s_wsum[k];
#pragma unroll
    for (int k = 0; k < BPT; k++) {  // exclusive: first position of each bucket
        s_hist[tid * BPT + k] = run;
        run += c[k];
    }
    __syncthreads();
    if constexpr (TPT > 0) {
#pragma unroll
        for (int k = 0; k < TPT; k++)
            if (t0 + k < t1) {
                const uint32_t p = atomicAdd(&s_hist[plan_bucket(tv[k])], 1u);
                order[plan_slot(p, (uint32_t)ntiles, (uint32_t)ncu)] = (uint32_t)(t0 + k);
            }
    } else {
        for (int u = tid; u < ntiles; u += NT) {
            const uint32_t p = atomicAdd(&s_hist[plan_bucket(tot[u])], 1u);
            order[plan_slot(p, (uint32_t)ntiles, (uint32_t)ncu)] = (uint32_t)u;
        }
    }
}

__global__ void identity_order_kernel(uint32_t* __restrict__ order, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) order[i] = (uint32_t)i;
}
hipError_t launch_identity_order(uint32_t* order, int ntiles, hipStream_t s) {
    if (ntiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(identity_order_kernel, dim3((ntiles + 255) / 256), dim3(256), 0, s, order, ntiles);
    return hipGetLastError();
}

// DUP_T lanes per workgroup, each placing the instances of DUP_G consecutive Gaussians of a count-matrix
// row (DUP_G = 2 for rows of 1024, 1 for rows of 512): at 1024 lanes (98 VGPRs, one workgroup per CU) a
// frame's ~300 workgroups took two dispatch rounds on 37 CUs; at 512 two workgroups share a CU (one
// round).  Forcing 1024-lane workgroups to 64 VGPRs instead spilled and was slower.
constexpr int DUP_T = 512;
#ifndef GSR_DUP_LOOP_MAX
#define GSR_DUP_LOOP_MAX 16  // rows whose Gaussians touch at most this many tiles place instances per lane
#endif
#ifndef GSR_NO_PLAN
#define GSR_NO_PLAN 0  // timing experiment: row-major render order instead of tile_plan
#endif
// the snapshot the host reads after the duplicate (Camera::host_snap): two 16-B vector stores to the coherent
// pinned buffer, made visible to the host by the kernel's end-of-kernel release
__device__ __forceinline__ void store_host_snap(uint32_t* snap, uint4 lo, uint4 hi) {
    reinterpret_cast<uint4*>(snap)[0] = lo;
    reinterpret_cast<uint4*>(snap)[1] = hi;
}
// gated geometry reuse, equal geometry: the duplicate is skipped, and its workgroup 0 hands the counters the reuse
// copy wrote (the previous call's [0..3], this call's [4..7]) to the host instead
__device__ __forceinline__ void dup_gate_off_snap(const Camera& cam, const GeomPtrs& geo) {
    if (cam.host_snap && blockIdx.x == 0 && threadIdx.x == 0)
        store_host_snap(cam.host_snap, *reinterpret_cast<const uint4*>(geo.counters),
                        *reinterpret_cast<const uint4*>(geo.counters + 4));
}
template <bool LDS_HIST, int DUP_G, bool EXACT>
__device__ __forceinline__ void duplicate_bucket_body(Camera cam, int P, GeomPtrs geo, uint2* __restrict__ ranges,
                                                      const uint32_t* __restrict__ tot, uint32_t* __restrict__ cursor,
                                                      int ntiles, uint64_t* __restrict__ keys,
                                                      uint64_t* __restrict__ point_list, SpecGuard guard,
                                                      uint32_t sort_cap, uint32_t* __restrict__ status,
                                                      uint32_t* __restrict__ s_cur) {
    // LDS_HIST: cursor = the column-scanned count matrix; this workgroup's
    // instances of tile t go to start[t] + cursor[block][t] + (LDS rank)
    // Culled instances (Camera::cull) are in no bucket, so the tile lists fill point_list[0, L) with L <
    // num_rendered; the tail [L, num_rendered) is written too, so every one of the num_rendered entries the
    // forward returns is a valid Gaussian id with an empty block mask (PointEntry = mask << 32 | id):
    //   EXACT (the dynamic, drop-in forward): the culled instances themselves, in (Gaussian, rect tile) order --
    //     the ids are then the reference's multiset (Gaussian i listed tiles_touched(i) times);
    //   else (static mode: the library is the only reader): padding -- slot u of the tail holds the Gaussian
    //     owning rect instance slot u (offsets[i] <= u < offsets[i] + tiles[i]), which needs no global prefix of
    //     the culled counts (that bookkeeping cost the kernel 16 VGPRs and a second dispatch round).
    constexpr bool TAIL = kCullTail;
    constexpr int ROW = DUP_G * DUP_T;  // Gaussians per count-matrix row (1 << cam.pre_shift)
    __shared__ uint32_t s_incl[ROW];
    __shared__ uint32_t s_x0[ROW], s_y0[ROW], s_w[ROW], s_depth[ROW], s_live[ROW];
    __shared__ uint32_t s_cx[EXACT ? ROW : 1];
    __shared__ uint32_t wsum[DUP_T / 64], s_tmax[DUP_T / 64], s_cws[DUP_T / 64];
    __shared__ uint32_t s_cred[2][DUP_T / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i0 = blockIdx.x * ROW + DUP_G * tid;  // this lane's Gaussians i0 .. i0 + DUP_G - 1
    // the Gaussians' tile counts and rects, loaded ahead of the prologue's loads (one round trip)
    uint32_t t[DUP_G];
    uint4 r[DUP_G];
#pragma unroll
    for (int g = 0; g < DUP_G; g++) {
        t[g] = (i0 + g < P) ? geo.tiles[i0 + g] : 0u;
        r[g] = (i0 + g < P) ? geo.bin[i0 + g] : make_uint4(0u, 0u, 0u, 0u);  // (rect lo, rect hi, depth bits, tiles)
    }
    uint32_t base, ctail = 0, ltot = 0xFFFFFFFFu;  // ltot: L, the lists' total (padding tail)
    if (LDS_HIST) {
        // The scans of scan_counts_body, redone by every workgroup (the inputs are
        // a few KB, L2-resident): this workgroup's instance base from the raw
        // workgroup totals, num_rendered, the prefiltered flag, and the exclusive
        // scan of the tile totals (bucket starts).  Workgroup 0 publishes them
        // (ranges, counters, status) for the later launches and the host.
        constexpr int TPT = 4;  // tiles per thread kept in registers (<= 4 DUP_T tiles), else staged in LDS
        __shared__ uint32_t s_red[5][DUP_T / 64];
        const uint32_t b = blockIdx.x, nb = gridDim.x;
        const int per = (ntiles + DUP_T - 1) / DUP_T;  // contiguous tiles per thread
        const int t0 = min(ntiles, tid * per), t1 = min(ntiles, t0 + per);
        const bool in_regs = per <= TPT;
        uint32_t tv[TPT], cv[TPT];
#pragma unroll
        for (int k = 0; k < TPT; k++) {
            const bool ok = in_regs && t0 + k < t1;
            tv[k] = ok ? tot[t0 + k] : 0u;
            cv[k] = ok ? cursor[(size_t)b * ntiles + t0 + k] : 0u;
        }
        uint32_t pre = 0, all = 0, viol = 0, vmax = 0, cpre = 0, call = 0;
        // two workgroup sums per trip, both loads issued before either is used (config 3: 586 rows, so some
        // lanes read two -- one memory round trip instead of two ahead of the workgroup's first barrier)
        for (uint32_t k = tid; k < nb; k += 2 * DUP_T) {
            const uint32_t k2 = k + DUP_T;
            const uint32_t v = geo.wgsum[k], v2 = k2 < nb ? geo.wgsum[k2] : 0u;
            // (EXACT: preprocess wrote wgcull; loaded unconditionally, with the workgroup sums)
            const uint32_t c = (TAIL && EXACT) ? geo.wgcull[k] : 0u, c2 = (TAIL && EXACT && k2 < nb) ? geo.wgcull[k2] : 0u;
            viol |= (v | v2) >> 31;
            all += (v & 0x7fffffffu) + (v2 & 0x7fffffffu);
            pre += (k < b ? (v & 0x7fffffffu) : 0u) + (k2 < b ? (v2 & 0x7fffffffu) : 0u);
            if (TAIL && EXACT) {
                call += c + c2;
                cpre += (k < b ? c : 0u) + (k2 < b ? c2 : 0u);
            }
        }
        uint32_t csum = 0;
        if (in_regs) {
#pragma unroll
            for (int k = 0; k < TPT; k++) {
                csum += tv[k];
                vmax = max(vmax, tv[k]);
            }
        } else {
            for (int u = t0; u < t1; u++) {
                const uint32_t v = tot[u];
                s_cur[u] = v;
                csum += v;
                vmax = max(vmax, v);
            }
        }
        const uint32_t cincl = wave_incl_scan(csum);
        pre = wave_sum_u32(pre);
        all = wave_sum_u32(all);
        viol = wave_max_u32(viol);
        vmax = wave_max_u32(vmax);
        if (TAIL && EXACT && cam.cull) {
            cpre = wave_sum_u32(cpre);
            call = wave_sum_u32(call);
        }
        if (lane == 0) {
            s_red[0][w] = pre;
            s_red[1][w] = all;
            s_red[2][w] = viol;
            s_red[3][w] = vmax;
            if (TAIL && EXACT) {
                s_cred[0][w] = cpre;
                s_cred[1][w] = call;
            }
        }
        if (lane == 63) s_red[4][w] = cincl;
        __syncthreads();
        uint32_t woff = 0, lsum = 0;
        pre = all = viol = vmax = cpre = call = 0;
#pragma unroll
        for (int k = 0; k < DUP_T / 64; k++) {
            pre += s_red[0][k];
            all += s_red[1][k];
            viol |= s_red[2][k];
            vmax = max(vmax, s_red[3][k]);
            woff += k < w ? s_red[4][k] : 0u;
            if (TAIL && !EXACT) lsum += s_red[4][k];
            if (TAIL && EXACT) {
                cpre += s_cred[0][k];
                call += s_cred[1][k];
            }
        }
        if (TAIL && EXACT) ctail = all - call + cpre;  // this workgroup's first culled instance in point_list
        if (TAIL && !EXACT) ltot = lsum;
        uint32_t run = woff + cincl - csum;  // bucket start of this thread's first tile
        if (in_regs) {
#pragma unroll
            for (int k = 0; k < TPT; k++)
                if (t0 + k < t1) {
                    if (b == 0) ranges[t0 + k] = make_uint2(run, run + tv[k]);
                    s_cur[t0 + k] = run + cv[k];
                    run += tv[k];
                }
        } else {
            for (int u = t0; u < t1; u++) {
                const uint32_t v = s_cur[u];
                if (b == 0) ranges[u] = make_uint2(run, run + v);
                s_cur[u] = run + cursor[(size_t)b * ntiles + u];
                run += v;
            }
        }
        if (tid == 0) {
            geo.blocksums[b] = pre;
            if (b == 0) {
                // [0] num_rendered [1] prefiltered violation [2] longest tile list [3] sort cap
                geo.counters[0] = all;
                geo.counters[1] = viol;
                geo.counters[2] = vmax;
                geo.counters[3] = sort_cap;
                if (status) status_merge(status, all, viol, vmax, sort_cap);
                if (cam.host_snap)  // (Camera::host_snap; [4..7] were final before this launch)
                    store_host_snap(cam.host_snap, make_uint4(all, viol, vmax, sort_cap),
                                    *reinterpret_cast<const uint4*>(geo.counters + 4));
            }
        }
        if (b == 0 && cam.tile_order_out) {
#if GSR_NO_PLAN
            for (int u = tid; u < ntiles; u += DUP_T) cam.tile_order_out[u] = (uint32_t)u;
#else
            __shared__ uint32_t s_plan[PLAN_BUCKETS];
            if (in_regs)
                tile_plan<DUP_T, TPT>(tot, ntiles, cam.sched_cus, cam.tile_order_out, s_plan, wsum, tv, t0, t1);
            else
                tile_plan<DUP_T>(tot, ntiles, cam.sched_cus, cam.tile_order_out, s_plan, wsum);
#endif
        }
        base = pre;
        if (all > guard.cap_inst || vmax > guard.cap_tile) return;  // workgroup-uniform
    } else {
        if (guard.overflow()) return;
        base = geo.blocksums[blockIdx.x];
        if (TAIL && !EXACT && ntiles > 0) ltot = ranges[ntiles - 1].y;  // (the scan launch wrote the ranges)
        if (TAIL && EXACT && cam.cull) {  // (the global-atomic path, > MAX_LDS_TILES tiles) the culled totals' prefix
            const uint32_t b = blockIdx.x, nb = gridDim.x;
            uint32_t cpre = 0, call = 0;
            for (uint32_t k = tid; k < nb; k += DUP_T) {
                const uint32_t c = geo.wgcull[k];
                call += c;
                cpre += k < b ? c : 0u;
            }
            cpre = wave_sum_u32(cpre);
            call = wave_sum_u32(call);
            if (lane == 0) {
                s_cred[0][w] = cpre;
                s_cred[1][w] = call;
            }
            __syncthreads();
            cpre = call = 0;
#pragma unroll
            for (int k = 0; k < DUP_T / 64; k++) {
                cpre += s_cred[0][k];
                call += s_cred[1][k];
            }
            ctail = geo.counters[0] - call + cpre;
        }
    }
    uint32_t tsum = 0, tmax = 0, cg[DUP_G], csum = 0;
#pragma unroll
    for (int g = 0; g < DUP_G; g++) {
        tsum += t[g];
        tmax = max(tmax, t[g]);
        cg[g] = (TAIL && EXACT && cam.cull && t[g]) ? culled_below(r[g].w, t[g]) : 0u;
        csum += cg[g];
        const int q = DUP_G * tid + g;
        if (t[g]) {
            s_x0[q] = r[g].x & 0xFFFFu;
            s_y0[q] = r[g].x >> 16;
            s_w[q] = (r[g].y & 0xFFFFu) - (r[g].x & 0xFFFFu);
            s_depth[q] = r[g].z;
            s_live[q] = r[g].w;
        }
    }
    uint32_t incl = wave_incl_scan(tsum);
    const uint32_t cincl = (TAIL && EXACT && cam.cull) ? wave_incl_scan(csum) : 0u;
    tmax = wave_max_u32(tmax);
    __syncthreads();  // (wsum is also tile_plan's scratch)
    if (lane == 63) {
        wsum[w] = incl;
        if (TAIL && EXACT) s_cws[w] = cincl;
    }
    if (lane == 0) s_tmax[w] = tmax;
    __syncthreads();
    uint32_t run = incl - tsum, crun = ctail + cincl - csum;
    for (int k = 0; k < w; k++) {
        run += wsum[k];
        if (TAIL && EXACT) crun += s_cws[k];
    }
#pragma unroll
    for (int k = 0; k < DUP_T / 64; k++) tmax = max(tmax, s_tmax[k]);
    uint32_t cx[DUP_G];  // (EXACT) the Gaussians' first slots in point_list's culled tail
#pragma unroll
    for (int g = 0; g < DUP_G; g++) {  // Gaussian order: the workgroup-local instance offsets of preprocess
        const uint32_t off = base + run;
        if (i0 + g < P) geo.offsets[i0 + g] = off;
        if (TAIL && !EXACT && off + t[g] > ltot)  // padding tail: the owner of each rect slot >= L
            for (uint32_t u = max(off, ltot); u < off + t[g]; u++) point_list[u] = (uint64_t)(i0 + g);
        run += t[g];
        s_incl[DUP_G * tid + g] = run;
        cx[g] = crun;
        if (TAIL && EXACT) s_cx[DUP_G * tid + g] = crun;  // (read by the load-balanced path)
        crun += cg[g];
    }
    if (tmax <= (uint32_t)GSR_DUP_LOOP_MAX) {
        // few tiles per Gaussian in this row (config 3: at most 4; mapping duplicate 50.4 -> 48.1 us at 16 or
        // 64, tracking 13.4 -> 11.9 at 8): every lane places its own Gaussians'
        // instances (<= GSR_DUP_LOOP_MAX loop trips) instead of one binary search over the row's
        // inclusive sums per instance; the slots within a tile bucket still come from the LDS cursors
        // (the bucket order is the sort's input, any order)
#pragma unroll
        for (int g = 0; g < DUP_G; g++) {
            const uint32_t x0 = r[g].x & 0xFFFFu, y0 = r[g].x >> 16, wdt = (r[g].y & 0xFFFFu) - x0;
            const uint32_t gi = (uint32_t)(i0 + g);
            uint32_t ct = cx[g];
            for (uint32_t k = 0; k < t[g]; k++) {
                if (!tile_live(r[g].w, k)) {  // culled (Camera::cull): not in the bucket (EXACT: in the tail)
                    if (TAIL && EXACT) point_list[ct++] = (uint64_t)gi;
                    continue;
                }
                const uint32_t tile = (y0 + k / wdt) * (uint32_t)cam.gx + x0 + k % wdt;
                const uint32_t pos = LDS_HIST ? atomicAdd(&s_cur[tile], 1u)
                                              : ranges[tile].x + atomicAdd(&cursor[tile * TILE_CTR_STRIDE], 1u);
                keys[pos] = ((uint64_t)r[g].z << 32) | (uint64_t)gi;
            }
        }
        return;
    }
    __syncthreads();
    const uint32_t total = s_incl[ROW - 1];
    for (uint32_t e = tid; e < total; e += DUP_T) {
        int lo = 0, hi = ROW - 1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (s_incl[mid] > e) hi = mid; else lo = mid + 1;
        }
        const uint32_t local = e - ((lo == 0) ? 0u : s_incl[lo - 1]);
        if (!tile_live(s_live[lo], local)) {  // culled (Camera::cull): not in the bucket (EXACT: in the tail)
            if (TAIL && EXACT)
                point_list[s_cx[lo] + culled_below(s_live[lo], local)] = (uint64_t)(blockIdx.x * ROW + lo);
            continue;
        }
        const uint32_t wdt = s_w[lo];
        const uint32_t tile = (s_y0[lo] + local / wdt) * (uint32_t)cam.gx + s_x0[lo] + local % wdt;
        const uint32_t pos = LDS_HIST ? atomicAdd(&s_cur[tile], 1u)
                                      : ranges[tile].x + atomicAdd(&cursor[tile * TILE_CTR_STRIDE], 1u);
        const uint32_t gi = blockIdx.x * ROW + lo;
        keys[pos] = ((uint64_t)s_depth[lo] << 32) | (uint64_t)gi;
    }
}
// EXACT instantiations: at most 80 VGPRs (6 waves per SIMD), three 512-lane workgroups per CU, so config 3's 586
// count-matrix rows run in one dispatch round on 256 CUs (that bookkeeping took the kernel to 88 VGPRs: two
// workgroups per CU, a second round, 10.8 -> 14.5 us); the padding ones stay at 72-79 VGPRs by themselves
template <bool LDS_HIST, int DUP_G, bool CLK, bool EXACT>
__global__ void __launch_bounds__(DUP_T) __attribute__((amdgpu_waves_per_eu(6, 8)))
duplicate_bucket_kernel(Camera cam, int P, GeomPtrs geo, uint2* __restrict__ ranges, const uint32_t* __restrict__ tot,
                        uint32_t* __restrict__ cursor, int ntiles, uint64_t* __restrict__ keys,
                        uint64_t* __restrict__ point_list, SpecGuard guard, uint32_t sort_cap,
                        uint32_t* __restrict__ status, unsigned long long* clk) {
    extern __shared__ uint32_t s_cur[];
    if (cam.gate.off()) {
        dup_gate_off_snap(cam, geo);
        return;
    }
    if constexpr (CLK) kclock_begin(clk);
    duplicate_bucket_body<LDS_HIST, DUP_G, EXACT>(cam, P, geo, ranges, tot, cursor, ntiles, keys, point_list, guard,
                                                  sort_cap, status, s_cur);
    if constexpr (CLK) kclock_end(clk);
}
// The exact-tail form (the dynamic forward) needs ~88 VGPRs: at the 80-VGPR cap above it spills 80 B per
// lane; GSR_DUP_EXACT_WAVES sets its own occupancy target
#ifndef GSR_DUP_EXACT_WAVES
#define GSR_DUP_EXACT_WAVES 6
#endif
template <bool LDS_HIST, int DUP_G, bool CLK>
__global__ void __launch_bounds__(DUP_T) __attribute__((amdgpu_waves_per_eu(GSR_DUP_EXACT_WAVES, 8)))
duplicate_bucket_exact_kernel(Camera cam, int P, GeomPtrs geo, uint2* __restrict__ ranges,
                              const uint32_t* __restrict__ tot, uint32_t* __restrict__ cursor, int ntiles,
                              uint64_t* __restrict__ keys, uint64_t* __restrict__ point_list, SpecGuard guard,
                              uint32_t sort_cap, uint32_t* __restrict__ status, unsigned long long* clk) {
    extern __shared__ uint32_t s_cur[];
    if (cam.gate.off()) {
        dup_gate_off_snap(cam, geo);
        return;
    }
    if constexpr (CLK) kclock_begin(clk);
    duplicate_bucket_body<LDS_HIST, DUP_G, true>(cam, P, geo, ranges, tot, cursor, ntiles, keys, point_list, guard,
                                                 sort_cap, status, s_cur);
    if constexpr (CLK) kclock_end(clk);
}

template <bool CLK, bool EXACT>
static auto duplicate_bucket_variant(bool lds_hist, bool g2) {
    if constexpr (EXACT)
        return lds_hist ? (g2 ? duplicate_bucket_exact_kernel<true, 2, CLK> : duplicate_bucket_exact_kernel<true, 1, CLK>)
                        : (g2 ? duplicate_bucket_exact_kernel<false, 2, CLK> : duplicate_bucket_exact_kernel<false, 1, CLK>);
    else
        return lds_hist ? (g2 ? duplicate_bucket_kernel<true, 2, CLK, false> : duplicate_bucket_kernel<true, 1, CLK, false>)
                        : (g2 ? duplicate_bucket_kernel<false, 2, CLK, false> : duplicate_bucket_kernel<false, 1, CLK, false>);
}

hipError_t launch_duplicate_bucket(const Camera& cam, int P, GeomPtrs geo, uint2* ranges, const uint32_t* tot,
                                   uint32_t* cursor, bool lds_hist, int ntiles, uint64_t* keys, uint64_t* point_list,
                                   int nb, SpecGuard guard, uint32_t* status, hipStream_t s, unsigned long long* clk) {
    if (nb == 0) return hipSuccess;
    const bool g2 = cam.pre_shift == 10;  // rows of 1024: two Gaussians per lane; of 512: one
    const bool exact = cam.tail_exact != 0;
    auto k = clk ? (exact ? duplicate_bucket_variant<true, true>(lds_hist, g2)
                          : duplicate_bucket_variant<true, false>(lds_hist, g2))
                 : (exact ? duplicate_bucket_variant<false, true>(lds_hist, g2)
                          : duplicate_bucket_variant<false, false>(lds_hist, g2));
    hipLaunchKernelGGL(k, dim3(nb), dim3(DUP_T), lds_hist ? sizeof(uint32_t) * ntiles : 0, s, cam, P, geo, ranges,
                       tot, cursor, ntiles, keys, point_list, guard, (uint32_t)TILE_SORT_CAP, status, clk);
    return hipGetLastError();
}

// ------------------------------------------------------------- radix sort --
// Each workgroup owns SORT_TILE consecutive keys; wave w owns the w-th quarter
// in 8 slots of 64 lanes, so (wave, slot, lane) order == key order (stable).
__global__ void __launch_bounds__(SORT_THREADS)
radix_hist_kernel(const uint64_t* __restrict__ keys, uint32_t n, int shift, uint32_t* __restrict__ hist, int nsb) {
    __shared__ uint32_t wcnt[SORT_THREADS / 64][RADIX];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int k = tid; k < (SORT_THREADS / 64) * RADIX; k += SORT_THREADS) (&wcnt[0][0])[k] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * SORT_TILE + w * (SORT_TILE / 4);
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int s = 0; s < SORT_ITEMS; s++) {
        const uint32_t idx = base + s * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = valid ? (uint32_t)(keys[idx] >> shift) & (RADIX - 1) : 0u;
        const uint64_t m = wave_match8(d, valid);
        if (valid && (m & lt) == 0) wcnt[w][d] += (uint32_t)__popcll(m);
    }
    __syncthreads();
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < SORT_THREADS / 64; k++) c += wcnt[k][tid];
    hist[(size_t)tid * nsb + blockIdx.x] = c;
}

// Per-digit exclusive scan of the [digit][block] histogram rows: workgroup d
// scans row d in place and writes the digit total (no single-workgroup
// bottleneck over RADIX * nsb entries).
__global__ void __launch_bounds__(256) radix_rowscan_kernel(uint32_t* __restrict__ hist, int nsb,
                                                            uint32_t* __restrict__ digit_total) {
    __shared__ uint32_t wsums[4];
    __shared__ uint32_t s_carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t* row = hist + (size_t)blockIdx.x * nsb;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (int base = 0; base < nsb; base += 256) {
        const int i = base + tid;
        const uint32_t x = (i < nsb) ? row[i] : 0u;
        const uint32_t incl = wave_incl_scan(x);
        if (lane == 63) wsums[w] = incl;
        __syncthreads();
        uint32_t off = s_carry;
        for (int k = 0; k < w; k++) off += wsums[k];
        if (i < nsb) row[i] = off + incl - x;
        __syncthreads();
        if (tid == 255) s_carry = off + incl;
        __syncthreads();
    }
    if (tid == 0) digit_total[blockIdx.x] = s_carry;
}

__global__ void __launch_bounds__(SORT_THREADS)
radix_scatter_kernel(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin, uint64_t* __restrict__ kout,
                     uint32_t* __restrict__ vout, uint32_t n, int shift, const uint32_t* __restrict__ hist, int nsb,
                     const uint32_t* __restrict__ digit_total) {
    __shared__ uint32_t wcnt[SORT_THREADS / 64][RADIX];
    __shared__ uint32_t s_dsum[SORT_THREADS / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int k = tid; k < (SORT_THREADS / 64) * RADIX; k += SORT_THREADS) (&wcnt[0][0])[k] = 0;
    // exclusive scan of the 256 digit totals -> global base of each digit
    const uint32_t dt = digit_total[tid];
    const uint32_t dincl = wave_incl_scan(dt);
    if (lane == 63) s_dsum[w] = dincl;
    __syncthreads();
    uint32_t dbase = dincl - dt;
    for (int k = 0; k < w; k++) dbase += s_dsum[k];
    const uint32_t base = blockIdx.x * SORT_TILE + w * (SORT_TILE / 4);
    const uint64_t lt = (1ull << lane) - 1ull;
    uint64_t key[SORT_ITEMS];
    uint32_t val[SORT_ITEMS], rank[SORT_ITEMS], dig[SORT_ITEMS];
#pragma unroll
    for (int s = 0; s < SORT_ITEMS; s++) {
        const uint32_t idx = base + s * 64 + lane;
        const bool valid = idx < n;
        key[s] = valid ? kin[idx] : 0ull;
        val[s] = valid ? (vin ? vin[idx] : idx) : 0u;
        const uint32_t d = (uint32_t)(key[s] >> shift) & (RADIX - 1);
        dig[s] = d;
        const uint64_t m = wave_match8(d, valid);
        uint32_t prev = 0;
        if (valid) prev = wcnt[w][d];
        rank[s] = prev + (uint32_t)__popcll(m & lt);
        if (valid && (m & lt) == 0) wcnt[w][d] = prev + (uint32_t)__popcll(m);
    }
    __syncthreads();
    {
        const uint32_t c0 = wcnt[0][tid], c1 = wcnt[1][tid], c2 = wcnt[2][tid];
        const uint32_t g = dbase + hist[(size_t)tid * nsb + blockIdx.x];
        __syncthreads();
        wcnt[0][tid] = g;
        wcnt[1][tid] = g + c0;
        wcnt[2][tid] = g + c0 + c1;
        wcnt[3][tid] = g + c0 + c1 + c2;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SORT_ITEMS; s++) {
        const uint32_t idx = base + s * 64 + lane;
        if (idx < n) {
            const uint32_t pos = wcnt[w][dig[s]] + rank[s];
            kout[pos] = key[s];
            vout[pos] = val[s];
        }
    }
}

hipError_t launch_radix_sort(uint64_t* keys[2], uint32_t* vals[2], uint32_t* hist, uint32_t n, int nsb, int npass,
                             hipStream_t s) {
    uint32_t* digit_total = hist + (size_t)RADIX * nsb;
    for (int p = 0; p < npass; p++) {
        const int in = p & 1, out = in ^ 1;
        hipLaunchKernelGGL(radix_hist_kernel, dim3(nsb), dim3(SORT_THREADS), 0, s, keys[in], n, 8 * p, hist, nsb);
        hipLaunchKernelGGL(radix_rowscan_kernel, dim3(RADIX), dim3(256), 0, s, hist, nsb, digit_total);
        hipLaunchKernelGGL(radix_scatter_kernel, dim3(nsb), dim3(SORT_THREADS), 0, s, keys[in],
                           p == 0 ? (const uint32_t*)nullptr : vals[in], keys[out], vals[out], n, 8 * p, hist, nsb,
                           digit_total);
    }
    return hipGetLastError();
}

// ------------------------------------------------------- gather (fallback) --
// Fallback path only: Gaussian ids of the radix-sorted instances (values are
// unsorted instance indices).  Tile ranges already come from scan_counts_kernel.
__global__ void gather_ids_kernel(const uint32_t* __restrict__ vals, const uint32_t* __restrict__ gid,
                                  uint64_t* __restrict__ point_list, uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) point_list[k] = (PointEntry)gid[vals[k]];
}

hipError_t launch_gather_ids(const uint32_t* vals, const uint32_t* gid, uint64_t* point_list, uint32_t n,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_ids_kernel, dim3((n + 255) / 256), dim3(256), 0, s, vals, gid, point_list, n);
    return hipGetLastError();
}

// ----------------------------------------------------------- render (fwd) --
// Per 256-entry batch every Gaussian gets a 16-bit mask of the 4x4-pixel blocks
// its contribution ellipse reaches (block_mask); each 16-lane row (one block)
// then walks only its own compacted list, 4 entries per step (the four rows of
// a wave walk different lists in lockstep): the LDS reads and exp/alpha of the 4
// entries are independent (ILP), the transmittance chain is then applied in
// order with predicated (branch-free) updates.  The next batch's global
// gathers are issued before the current batch is rasterised.
// DUAL: a second colour set (colors2, e.g. SplaTAM's [z, 1, z^2]) is composited
// in the same pass -- same alpha / T / termination, so each output is bitwise
// the image a separate call would produce.
// L1 (with DUAL): the tracking loss epilogue of TrackL1 (gsr_common.h).
template <bool DUAL, bool L1 = false>
__global__ void __launch_bounds__(TILE_PIX, 5)
render_fwd_kernel(Camera cam, const uint2* __restrict__ ranges, PointEntry* __restrict__ point_list,
                  uint64_t* __restrict__ keys, const float4* __restrict__ rr, float* __restrict__ final_T, uint32_t* __restrict__ n_contrib,
                  float* __restrict__ out_color, float* __restrict__ out_color2, float* __restrict__ out_depth,
                  SpecGuard guard, unsigned long long* clk, TrackL1 l1) {
    static_assert(DUAL || !L1, "the tracking loss needs the depth / silhouette colour set");
    if (cam.gate.off()) return;
    kclock_begin(clk);
    RenderDiag dg;  // (diagnostics builds only, gsr_diag.h): phases 0 sort, 1 staging, 2 lists, 3 walk, 4 barrier,
    dg.begin();     // 5 epilogue
    if (guard.overflow()) {
        kclock_end(clk);
        return;
    }
    __shared__ __attribute__((aligned(16))) char smem[FwdShape<DUAL>::bytes];
    const int tile = sched_tile(cam);
    dg.tile(tile);
    const FwdPix f = fwd_tile<DUAL>(cam, tile, ranges, point_list, keys, rr, guard, smem, dg);
    float g[4];
    fwd_epilogue<DUAL, L1, true>(cam, tile, f, final_T, n_contrib, out_color, out_color2, out_depth, l1, g);
    dg.phase(5);
    dg.end();
    kclock_end(clk);
}

#if GSR_PHASE
extern "C" int gsr_diag_phase_fwd(unsigned long long* host) {  // copies and clears the phase cycles
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), sizeof(g_phase), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
#endif
#if GSR_WGTIME
extern "C" int gsr_diag_wgtime_fwd(unsigned long long* host, int n) {
    const size_t bytes = sizeof(unsigned long long) * 4 * (size_t)(n < GSR_WGTIME_MAX ? n : GSR_WGTIME_MAX);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wgtime), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

int track_l1_fused_scratch_floats(int ntiles) { return 2 * ntiles + ARRIVE_GROUPED_WORDS; }

hipError_t launch_render_fwd(const Camera& cam, const uint2* ranges, uint64_t* point_list,
                             uint64_t* keys, GeomPtrs geo,
                             const float* colors2, float* final_T, uint32_t* n_contrib, float* out_color,
                             float* out_color2, float* out_depth, SpecGuard guard, hipStream_t s,
                             unsigned long long* clk, const TrackL1* l1) {
    auto k = colors2 ? (l1 ? render_fwd_kernel<true, true> : render_fwd_kernel<true, false>)
                     : render_fwd_kernel<false, false>;
    hipLaunchKernelGGL(k, dim3(cam.gx * cam.gy), dim3(TILE_PIX), 0, s, cam, ranges, point_list, keys,
                       geo.rr, final_T,
                       n_contrib, out_color, out_color2, out_depth, guard, clk, l1 ? *l1 : TrackL1{});
    return hipGetLastError();
}

// ---------------------------------------------------------- geometry reuse --
// gsr_forward_reuse: the copied render records get this call's colours (preprocess writes the
// colours only for Gaussians that touch a tile: the same condition here, tiles[i] != 0)
__global__ void recolour_kernel(int P, const float* __restrict__ colors, float4* __restrict__ rr,
                                const uint32_t* __restrict__ tiles, Gate gate) {
    if (gate.off()) return;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P || tiles[i] == 0u) return;
    float4* q2 = rr + (size_t)RR_F4 * i + 2;
    const float4 old = *q2;
    *q2 = make_float4(colors[3 * i], colors[3 * i + 1], colors[3 * i + 2], old.w);
}
hipError_t launch_recolour(int P, const float* colors, GeomPtrs geo, hipStream_t s, Gate gate) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(recolour_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, colors, geo.rr, geo.tiles, gate);
    return hipGetLastError();
}
// gsr_forward_reuse_if_equal's copy of the previous call's state (runs only when the gate says "equal"): the
// geometry buffer up to its counters block plus counters[0..3] (num_rendered, prefiltered flag, longest list,
// sort cap: counters[4..7] stay this call's -- [5] holds the gate itself) and the radii; the render records'
// colour quarter (rr[i][2].xyz) of every Gaussian that touches a tile gets this call's colours on the way
// (recolour_kernel's condition and values, fused into the copy).  (The image and binning buffers are the
// previous call's, as in gsr_forward_reuse: the render writes the same final_T / n_contrib into them.)
// 16-B grid-stride streams (the geometry layout is 256-B aligned, the records at offset 0).
__global__ void __launch_bounds__(256) reuse_copy_kernel(Gate gate, const uint4* __restrict__ pg, uint4* __restrict__ g,
                                                         size_t ng16, const uint32_t* __restrict__ ptiles,
                                                         const float* __restrict__ colors, const int* __restrict__ prad,
                                                         int* __restrict__ rad, int P) {
    if (gate.off()) return;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nrr = (size_t)RR_F4 * P;
    for (size_t k = t0; k <= ng16; k += stride) {  // (k == ng16: counters[0..3])
        uint4 v = pg[k];
        if (k < nrr && (k % RR_F4) == 2) {
            const size_t i = k / RR_F4;
            if (ptiles[i] != 0u) {
                v.x = __float_as_uint(colors[3 * i]);
                v.y = __float_as_uint(colors[3 * i + 1]);
                v.z = __float_as_uint(colors[3 * i + 2]);
            }
        }
        g[k] = v;
    }
    for (size_t k = t0; k < (size_t)P; k += stride) rad[k] = prad[k];
}
hipError_t launch_reuse_copy(Gate gate, const void* prev_geom, void* geom, size_t geom_bytes, size_t tiles_offset,
                             const float* colors, const int* prev_radii, int* radii, int P, hipStream_t s) {
    if (geom_bytes & 15) return hipErrorInvalidValue;
    hipLaunchKernelGGL(reuse_copy_kernel, dim3(2048), dim3(256), 0, s, gate, (const uint4*)prev_geom, (uint4*)geom,
                       geom_bytes / 16, (const uint32_t*)((const char*)prev_geom + tiles_offset), colors, prev_radii,
                       radii, P);
    return hipGetLastError();
}
// *word = e when a[k] and b[k] differ bitwise anywhere (16-B loads where both arrays allow them)
__global__ void __launch_bounds__(256) epoch_mismatch_kernel(EqualPairs q, uint32_t* word, uint32_t e) {
    bool diff = false;
    const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x, stride = (long long)gridDim.x * blockDim.x;
    for (int k = 0; k < q.npairs; k++) {
        const float* a = q.a[k];
        const float* b = q.b[k];
        long long head = 0;
        if ((((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15u) == 0)) {
            const uint4* a4 = reinterpret_cast<const uint4*>(a);
            const uint4* b4 = reinterpret_cast<const uint4*>(b);
            const long long n4 = q.n[k] / 4;
            for (long long i = t0; i < n4; i += stride) {
                const uint4 x = a4[i], y = b4[i];
                diff = diff || x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w;
            }
            head = 4 * n4;
        }
        const uint32_t* au = reinterpret_cast<const uint32_t*>(a);
        const uint32_t* bu = reinterpret_cast<const uint32_t*>(b);
        for (long long i = head + t0; i < q.n[k]; i += stride) diff = diff || au[i] != bu[i];
    }
    if (__ballot(diff) != 0ull && __lane_id() == 0) atomicExch(word, e);
}
hipError_t launch_epoch_mismatch(const EqualPairs& q, uint32_t* word, uint32_t e, hipStream_t s) {
    hipLaunchKernelGGL(epoch_mismatch_kernel, dim3(1024), dim3(256), 0, s, q, word, e);
    return hipGetLastError();
}
// flag |= 1 when a[k][i] != b[k][i] bitwise for any pair k (grid-stride over the pairs' elements)
__global__ void bitwise_equal_kernel(EqualPairs q, int* flag) {
    bool diff = false;
    for (int k = 0; k < q.npairs; k++) {
        const uint32_t* a = reinterpret_cast<const uint32_t*>(q.a[k]);
        const uint32_t* b = reinterpret_cast<const uint32_t*>(q.b[k]);
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < q.n[k];
             i += (long long)gridDim.x * blockDim.x)
            diff = diff || a[i] != b[i];
    }
    if (__ballot(diff) != 0ull && __lane_id() == 0) atomicOr(flag, 1);
}
hipError_t launch_bitwise_equal(const EqualPairs& q, int* flag, hipStream_t s) {
    if (q.npairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(bitwise_equal_kernel, dim3(1024), dim3(256), 0, s, q, flag);
    return hipGetLastError();
}

// ----------------------------------------------------------- mark visible --
__global__ void mark_visible_kernel(int P, const float* __restrict__ means3D, const float* __restrict__ view,
                                    uint8_t* __restrict__ vis) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
    vis[i] = xform4x3(p, view).z > 0.001f ? 1 : 0;
}

hipError_t launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* vis, hipStream_t s) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, view, vis);
    return hipGetLastError();
}

}  // namespace gsr
