// gsr_backward.hip -- backward pipeline of the MI355X-native Gaussian rasterizer.
//
// power == 1 (the standard 3DGS backward; SplaTAM's tracking/mapping path):
//   render_bwd  (backward.cu:586-748 semantics) one 16x16 tile per workgroup,
//               back-to-front over LDS batches; each 16-lane row walks the list
//               of its 4x4-pixel block.  The per-pair 2D gradient terms are
//               summed across the row with a transposed DPP reduction, the 16
//               block partials are added through LDS in a fixed order, and ONE
//               plain 48-B record per (tile, Gaussian) instance is stored at
//               its unsorted position.
//               No global atomics at all: the reference issues ~25 float
//               atomics per contributing pair (backward.cu:1093-1137).
//   gauss_bwd   one lane per Gaussian: sums its instance records in a fixed
//               order (deterministic, bitwise reproducible) and applies the
//               per-Gaussian chain rule (backward.cu:144-274 cov2D,
//               412-475 cov3D, 480-530 projection, 20-139 SH).
#include <cstdlib>
#include <utility>

#include "gsr_chain.h"
#include "gsr_diag.h"
#include "gsr_glue_common.h"
#include "gsr_render_fwd.h"

#ifndef GSR_PK_XD
#define GSR_PK_XD 1  // the tile walk's e Tn and alpha Tn as one packed multiply
#endif
#ifndef GSR_POSE_TAIL
#define GSR_POSE_TAIL 2  // levels of the fused pose reduction's last-workgroup sum (1 or 2)
#endif

namespace gsr {

// Per-pair geometric terms (hx, hy, hx dx, hx dy, hy dy[, G dL/dalpha]) with
// h = G * dL/dG = (o * G) * dL/dalpha.
template <bool OPAC>
__device__ __forceinline__ void pair_geom(float* vk, float araw, float dLa, float G, v2f d) {
#if GSR_PK_XD
    if constexpr (OPAC) {  // (araw dLa, G dLa): one v_pk_mul_f32, the same two products
        const v2f ho = v2f{araw, G} * dLa;
        const v2f hv = ho.x * d;
        const v2f hh = hv.x * d;
        vk[0] = hv.x;
        vk[1] = hv.y;
        vk[2] = hh.x;
        vk[3] = hh.y;
        vk[4] = hv.y * d.y;
        vk[5] = ho.y;
        return;
    }
#endif
    const v2f hv = (araw * dLa) * d;  // (hx, hy)
    const v2f hh = hv.x * d;          // (hx dx, hx dy)
    vk[0] = hv.x;
    vk[1] = hv.y;
    vk[2] = hh.x;
    vk[3] = hh.y;
    vk[4] = hv.y * d.y;
    if (OPAC) vk[5] = G * dLa;
}
// Per-pair colour terms dch * dL/dpix (COL1: C1 = 3 channels, or 1 on a tile whose dL/dpix channels 1 and
// 2 are zero) and dch * dL/dpix2 (COL2, Q2 channels).
template <bool COL1, bool COL2, int Q2, int C1 = 3>
__device__ __forceinline__ void pair_colours(float* vk, float dch, v2f dp01, float dp2, float dq0, v2f dq01,
                                             float dq2) {
    if (COL1 && C1 == 1) {
        vk[0] = dch * dp01.x;
    } else if (COL1) {
        const v2f t = dch * dp01;
        vk[0] = t.x;
        vk[1] = t.y;
        vk[2] = dch * dp2;
    }
    float* v2 = vk + (COL1 ? C1 : 0);
    if (COL2 && Q2 == 1) {
        v2[0] = dch * dq0;
    } else if (COL2) {
        const v2f t = dch * dq01;
        v2[0] = t.x;
        v2[1] = t.y;
        v2[2] = dch * dq2;
    }
}
// Row totals of 4 entries x N values (entry-major) -> the LDS slots of this
// lane's entry: dst points at the entry's slot (+ the pass's value offset).
template <int N>
__device__ __forceinline__ void reduce_store(const float (&v)[4 * N], int lane, float* dst, bool store) {
    float r[RowReduce<N>::R];
    row_reduce<N>(v, r, lane);
    if (store && (lane & RowReduce<N>::WRITER_MASK) == 0) {
        float* p = dst + row_m0<N>(lane);
#pragma unroll
        for (int m = 0; m < RowReduce<N>::R; m++) p[m] = r[m];
    }
}

// Gaussians staged per batch: the per-row partial sums take 16 x batch x NV floats of LDS
// Entries staged per batch, and the batch's budget of per-(entry, block) LDS slots: each entry
// owns popcount(block mask) consecutive slots of NV floats (about 3 on average, at most 16), so a
// batch of BB entries is cut short when its masks need more than BS slots.
#ifndef GSR_BWD_BB
// batch of the variants with <= 6 sums (timing experiments may override); 144 and 160 entries (512 /
// 576 slots, still 5 waves/SIMD) measured 3-4 us slower on the config-3 tracking launch (r3 ab5)
#define GSR_BWD_BB 128
#endif
#ifndef GSR_BWD_WBB
// batch of the wide variants (> 6 sums): 96 measured faster than 64 (mapping render_bwd 362 -> 326 us) at 5
// waves/SIMD; 128 entries with a 384-slot budget (the 96-entry batch's s_acc; 2.7 blocks per entry on
// average) stay at 5 waves/SIMD and measured 3 % faster again (single-image full gradient 88 -> 85.5 us,
// config-4 dual 425 -> 410 us; profiles/r3_ab_render_bwd.txt); 448 slots drop the mapping variant to 4
#define GSR_BWD_WBB 128
#endif
template <int NV, int MOM = 0>
constexpr int bwd_batch() { return MOM ? 128 : (NV <= 6 ? GSR_BWD_BB : GSR_BWD_WBB); }
#ifndef GSR_BWD_WBS
#define GSR_BWD_WBS 384  // slot budget of the wide variants' batches
#endif
#ifndef GSR_BWD_BS
#define GSR_BWD_BS (4 * GSR_BWD_BB)  // slot budget of the batches of the variants with <= 6 sums
#endif
// the moment variants (backward_power == 2): 19 / 37 sums per slot; 256 / 128 slots keep 4 workgroups per CU
template <int NV, int MOM = 0>
constexpr int bwd_slots() { return MOM == 1 ? 256 : (MOM == 2 ? 128 : (NV <= 6 ? GSR_BWD_BS : GSR_BWD_WBS)); }

// DUAL: the pass also carries a second colour set (colors2, dL_dpix2) composited
// with the same alpha / T (one dual forward): the per-pair dL/dalpha is the sum
// of both renders'.  OPAC / COL1 / COL2: whether dL/dopacity, dL/dcolors and
// dL/dcolors2 are wanted; absent ones are neither formed nor reduced (tracking
// needs only the geometric sums and the depth colours).  Records always use the
// fixed 12-slot layout [hx, hy, hxx, hxy, hyy | G dL/dalpha | dch dp(3) | dch dq(3)].
// Q2: how many leading channels of dL_dpix2 may be non-zero (3, or 1 when the caller
// promises the rest are zero -- SplaTAM's tracking loss differentiates only the depth
// channel of the [depth, silhouette, depth^2] image).
//
// Per pixel the reference's back-to-front recurrence (backward.cu:966-1017)
// is carried on dot products with dL/dpixel: the colour accumulated behind the
// current Gaussian, accum_rec . dL/dpix, is one scalar A updated as
// A <- A + alpha (c . dL/dpix - A) after each contributing Gaussian (the
// reference's last_alpha / last_color / accum_rec update, one step earlier).
//
// Work split: each 16-lane row owns a 4x4-pixel block and walks its own list of
// the batch entries whose contribution ellipse reaches the block (block_mask),
// 4 entries per step; the per-pair products are summed over the row with the
// transposed in-row reduction (row_reduce) into a per-(block, entry) LDS slot,
// and after the batch one thread per entry adds its (at most 16) block slots
// in block order (deterministic) and stores ONE 48-B record per (tile,
// Gaussian) instance at its unsorted position.
// 5 workgroups per CU (<= 96 VGPRs): a 640x480 frame's 1200 tiles are all resident
// at once, so there is no second dispatch round behind the slowest tiles.
// MOM (backward_power == 2, gauss_bwd_mom_kernel): the pair's second moments instead of its values.
// The geometric terms are u = h (dx, dy, dx^2, dx dy, dy^2) (h = G dL/dG), so u_i u_j = h^2 dx^a dy^b
// with a + b in {2, 3, 4}: 12 distinct monomial moments instead of 15 products.  Layout:
//   [0, 12)  sum h^2 dx^a dy^b, monomial t: (2,0) (1,1) (0,2) | (3,0) (2,1) (1,2) (0,3) | (4,0) (3,1) (2,2) (1,3) (0,4)
//   12       sum (G dL/dalpha)^2
//   MOM 1 (colours precomputed, 16 sums): [13, 16) sum (dch dL/dpix_c)^2
//   MOM 2 (SH colours, 34 sums): [13, 19) sum dch^2 dL/dpix_c dL/dpix_d (c <= d, row-major),
//                                [19, 34) sum u_i dch dL/dpix_c (i-major)
template <bool DUAL, bool OPAC, bool COL1, bool COL2, int Q2, int MOM = 0, int C1 = 3>
constexpr int bwd_nv() { return MOM == 1 ? 16 : (MOM == 2 ? 34 : 5 + (OPAC ? 1 : 0) + (COL1 ? C1 : 0) + (COL2 ? Q2 : 0)); }
__host__ __device__ constexpr int mono_t(int a, int b) {  // monomial index of dx^a dy^b, a + b in {2, 3, 4}
    return a + b == 2 ? 2 - a : (a + b == 3 ? 3 + (3 - a) : 7 + (4 - a));
}
__host__ __device__ constexpr int u_a(int i) { return i == 0 ? 1 : (i == 2 ? 2 : (i == 3 ? 1 : 0)); }  // u_i ~ dx^a dy^b
__host__ __device__ constexpr int u_b(int i) { return i == 1 ? 1 : (i == 3 ? 1 : (i == 4 ? 2 : 0)); }
__host__ __device__ constexpr int ww_q(int c, int d) {  // MOM 2 index of the colour product (c, d), any order
    return c > d ? 13 + (d == 0 ? c : (d == 1 ? 2 + c : 5)) : 13 + (c == 0 ? d : (c == 1 ? 2 + d : 5));
}
static_assert(mono_t(2, 0) == 0 && mono_t(0, 2) == 2 && mono_t(0, 3) == 6 && mono_t(4, 0) == 7 && mono_t(0, 4) == 11, "");
static_assert(ww_q(0, 0) == 13 && ww_q(2, 1) == 17 && ww_q(2, 2) == 18, "");
// Per-entry quantities the moments are formed from
struct MomIn {
    float m20, m11, m02;  // h^2 dx^2, h^2 dx dy, h^2 dy^2
    float dx, dy, xx, xy, yy;
    float o2, c2;         // (G dL/dalpha)^2, dch^2
    float hc[3];          // h dch dL/dpix_c (MOM 2)
};
// moment Q of one entry (per-pixel constants: dp2[c] = dL/dpix_c^2, dpp[6] = the c <= d products)
template <int MOM, int Q>
__device__ __forceinline__ float mom_val(const MomIn& e, const float (&dp2)[3], const float (&dpp)[6]) {
    if constexpr (Q < 3) return Q == 0 ? e.m20 : (Q == 1 ? e.m11 : e.m02);
    else if constexpr (Q < 5) return e.m20 * (Q == 3 ? e.dx : e.dy);
    else if constexpr (Q < 7) return e.m02 * (Q == 5 ? e.dx : e.dy);
    else if constexpr (Q < 10) return e.m20 * (Q == 7 ? e.xx : (Q == 8 ? e.xy : e.yy));
    else if constexpr (Q < 12) return e.m02 * (Q == 10 ? e.xy : e.yy);
    else if constexpr (Q == 12) return e.o2;
    else if constexpr (MOM == 1) return e.c2 * dp2[Q - 13];
    else if constexpr (Q < 19) return e.c2 * dpp[Q - 13];
    else {
        constexpr int i = (Q - 19) / 3, c = (Q - 19) % 3;
        const float mono = i == 0 ? e.dx : (i == 1 ? e.dy : (i == 2 ? e.xx : (i == 3 ? e.xy : e.yy)));
        return e.hc[c] * mono;
    }
}
// One reduction pass over moments [Q0, Q0 + N) of the step's four entries.
template <int MOM, int Q0, int... Q>
__device__ __forceinline__ void mom_values(const MomIn (&e)[4], const float (&dp2)[3], const float (&dpp)[6], float* v,
                                           std::integer_sequence<int, Q...>) {
    constexpr int N = sizeof...(Q);
#pragma unroll
    for (int k = 0; k < 4; k++) ((v[N * k + Q] = mom_val<MOM, Q0 + Q>(e[k], dp2, dpp)), ...);
}
template <int MOM, int Q0, int N>
__device__ __forceinline__ void mom_pass(const MomIn (&e)[4], const float (&dp2)[3], const float (&dpp)[6], int lane,
                                         float* dst) {
    float v[4 * N];
    mom_values<MOM, Q0>(e, dp2, dpp, v, std::make_integer_sequence<int, N>{});
    reduce_store<N>(v, lane, dst + Q0, true);
}
// The moments as the symmetric 9 x 9 matrix of the base values b = (u0..u4, G dL/dalpha, dch dL/dpix_0..2)
// (MOM 1 forms no colour cross moments: those entries stay 0).
template <int MOM, int IJ>
struct MomSlot {  // (frontend-evaluated: every register-array index below is a compile-time constant)
    static constexpr int i = IJ / 9, j = IJ % 9;
    static constexpr int q = (i < 5 && j < 5) ? mono_t(u_a(i) + u_a(j), u_b(i) + u_b(j))
                             : (i == 5 && j == 5) ? 12
                             : (i >= 6 && j >= 6) ? (MOM == 1 ? (i == j ? 13 + (i - 6) : -1) : ww_q(i - 6, j - 6))
                             : (MOM == 2 && i < 5 && j >= 6) ? 19 + 3 * i + (j - 6)
                             : (MOM == 2 && j < 5 && i >= 6) ? 19 + 3 * j + (i - 6)
                                                             : -1;
};
template <int MOM, int... IJ>
__device__ __forceinline__ void mom_matrix(const float* S, float (&Sm)[9][9], std::integer_sequence<int, IJ...>) {
    ((Sm[MomSlot<MOM, IJ>::i][MomSlot<MOM, IJ>::j] = MomSlot<MOM, IJ>::q >= 0 ? S[MomSlot<MOM, IJ>::q >= 0 ? MomSlot<MOM, IJ>::q : 0] : 0.f), ...);
}
// 5 waves per SIMD (96 VGPRs; the wide variants reduce in two passes to fit), except
// the dual variants with a 3-channel second gradient (mapping-style), which spill
// at 96 VGPRs and run at 4
#ifndef GSR_BWD_WIDE_WAVES
#define GSR_BWD_WIDE_WAVES 5
#endif
#ifndef GSR_BWD_MAP_WAVES
#define GSR_BWD_MAP_WAVES 4
#endif
#ifndef GSR_BWD_SPLIT6
#define GSR_BWD_SPLIT6 1  // wide variants: the first reduction pass carries G dL/dalpha with the 5 geometric sums
// (6 + 6 instead of 5 + 7 sums for mapping: 84 instead of 96 DPP adds per step, render_bwd 312 -> 303 us at config 4)
#endif
#ifndef GSR_NT_STORES
#define GSR_NT_STORES 0  // render kernels' record / image stores as non-temporal (streaming) stores
#endif
#ifndef GSR_PACK_C
#define GSR_PACK_C 1  // DUAL, Q2 = 1: the second colour set's one channel staged in s_c.w (no s_d array)
#endif
template <bool DUAL, bool OPAC, bool COL1, bool COL2, int Q2, int MOM = 0>
constexpr int bwd_waves() {
    return MOM ? 4 : ((DUAL && Q2 == 3) ? GSR_BWD_MAP_WAVES : ((OPAC && COL1) ? GSR_BWD_WIDE_WAVES : 5));
}

// A tile backward's shape and LDS layout (carved from one byte array, so a kernel that also runs the
// forward of the same tile -- render_track_kernel -- can alias the two phases' LDS)
// C1 = 1: the single-image colour sums of a tile whose dL/dpix channels 1 and 2 are zero (SplaTAM's
// depth/silhouette render: its loss differentiates the depth channel only) -- one colour sum instead of
// three; the batch shape and the record layout stay those of the C1 = 3 variant (the two missing sums are
// stored as zeros), so both serve the same launch.
template <bool DUAL, bool OPAC, bool COL1, bool COL2, int Q2, int MOM, int C1 = 3>
struct BwdShape {
    static constexpr int NV = bwd_nv<DUAL, OPAC, COL1, COL2, Q2, MOM, C1>();
    static constexpr int NV3 = bwd_nv<DUAL, OPAC, COL1, COL2, Q2, MOM, 3>();
    static constexpr int BB = bwd_batch<NV3, MOM>(), BS = bwd_slots<NV3, MOM>();
    static constexpr int RS = (NV3 + 1) & ~1;  // record stride (floats)
    static constexpr int LS = BB + 4;          // row-list stride (u32)
    // entry BB is a dummy (opacity 0, never blends) that pads the row lists; its slot BS
    // absorbs the pad entries' (zero) sums
    static constexpr int SL = BB + 1;
    // PACKC: the dual render's second colour set needs only channel 0 (Q2 = 1): staged as s_c.w (the
    // tile-rect half s_c.w carried is consumed at staging), so a pair reads one colour float4, not two
    static constexpr bool PACKC = GSR_PACK_C && DUAL && Q2 == 1;
    static constexpr size_t o_a = 0, o_b = o_a + 16 * SL, o_c = o_b + 16 * SL, o_d = o_c + 16 * SL;
    static constexpr size_t o_acc = o_d + 16 * ((DUAL && !PACKC) ? SL : 1);
    static constexpr size_t o_list = o_acc + (4 * (BS + 1) * NV + 15) / 16 * 16;
    static constexpr size_t o_u = o_list + 4 * 16 * LS, o_mask = o_u + 4 * BB, o_base = o_mask + 2 * BB;
    static constexpr size_t o_rmax = (o_base + 2 * BB + 3) / 4 * 4;
    static constexpr size_t bytes = o_rmax + 64;
};

// One thread's pixel inputs of the tile backward: the forward's final transmittance and last
// contributor, dL/dpix of both colour sets
struct BwdPix {
    float T_final;
    uint32_t last;
    float dp0, dp1, dp2, dq0, dq1, dq2;
};

template <bool DUAL, bool OPAC, bool COL1, bool COL2, int Q2, int MOM, int C1 = 3>
__device__ __forceinline__ void bwd_tile(const Camera& cam, int tile, const BwdPix& pin,
                                         const uint2* __restrict__ ranges, const PointEntry* __restrict__ point_list,
                                         const float4* __restrict__ rr, const uint32_t* __restrict__ blocksums,
                                         float* __restrict__ inst, const BwdGuard& guard, char* smem,
                                         RenderDiag& dg) {
    static_assert(DUAL || !COL2, "COL2 needs the dual colour set");
    static_assert(!MOM || (!DUAL && OPAC && COL1), "the moment variants form every single-image gradient");
    static_assert(Q2 == 1 || Q2 == 3, "Q2 is 1 or 3 channels");
    static_assert(C1 == 3 || (C1 == 1 && COL1 && !DUAL && !MOM), "one colour sum: single-image colour variants only");
    using L = BwdShape<DUAL, OPAC, COL1, COL2, Q2, MOM, C1>;
    constexpr int NV = L::NV;
    constexpr int O_C1 = 5 + (OPAC ? 1 : 0);
    constexpr int BB = L::BB, BS = L::BS, RS = L::RS, LS = L::LS;
    constexpr bool PACKC = L::PACKC;
    float4* const s_a = reinterpret_cast<float4*>(smem + L::o_a);
    float4* const s_b = reinterpret_cast<float4*>(smem + L::o_b);
    float4* const s_c = reinterpret_cast<float4*>(smem + L::o_c);
    [[maybe_unused]] float4* const s_d = reinterpret_cast<float4*>(smem + L::o_d);
    uint32_t* const s_u = reinterpret_cast<uint32_t*>(smem + L::o_u);
    uint16_t* const s_mask = reinterpret_cast<uint16_t*>(smem + L::o_mask);
    uint16_t* const s_base = reinterpret_cast<uint16_t*>(smem + L::o_base);
    float* const s_acc = reinterpret_cast<float*>(smem + L::o_acc);
    uint32_t* const s_rmax = reinterpret_cast<uint32_t*>(smem + L::o_rmax);
    uint32_t* const s_list = reinterpret_cast<uint32_t*>(smem + L::o_list);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, row = (tid >> 4) & 3;
    const int tx = tile % cam.gx, ty = tile / cam.gx;
    const int px = tx * TILE_X + tile_px(tid);
    const int py = ty * TILE_Y + tile_py(tid);
    const float x0 = (float)(tx * TILE_X), y0 = (float)(ty * TILE_Y);
    const uint2 range = ranges[tile];
    const float T_final = pin.T_final;
    const uint32_t last = pin.last;
    const float dp0 = pin.dp0, dp1 = pin.dp1, dp2 = pin.dp2, dq0 = pin.dq0, dq1 = pin.dq1, dq2 = pin.dq2;
    // per-block (row) maximum of the pixels' last contributor: the forward's per-tile record (one uniform
    // 64-B load, no reduction over n_contrib before the first list entries can be fetched), else reduced here
    uint32_t bmax = 0;
    int rm[4];
    if (cam.rowmax) {
        const uint4* rp = reinterpret_cast<const uint4*>(cam.rowmax + 16 * tile);
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint4 q = rp[b];
            bmax = max(bmax, max(max(q.x, q.y), max(q.z, q.w)));
        }
        const uint4 qw = rp[w];  // the wave's four blocks (a second, cached 16-B load)
        rm[0] = (int)qw.x; rm[1] = (int)qw.y; rm[2] = (int)qw.z; rm[3] = (int)qw.w;
    } else {
        uint32_t rmax = last;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, o));
        if ((lane & 15) == 0) s_rmax[4 * w + row] = rmax;
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 16; b++) bmax = max(bmax, s_rmax[b]);
#pragma unroll
        for (int r = 0; r < 4; r++) rm[r] = (int)s_rmax[4 * w + r];
    }
    // Instances behind every pixel's last contributor receive zero gradient.
    for (uint32_t k = range.x + bmax + tid; k < range.y; k += TILE_PIX) {
        const uint32_t gk = pe_id(point_list[k]);
        const RenderRec r = load_rr(rr, gk);
        const uint32_t u = instance_slot(rr_rect(r), rr_offset(r, blocksums, gk, cam.pre_shift), tx, ty);
        float2* dst = reinterpret_cast<float2*>(inst + (size_t)RS * u);
#pragma unroll
        for (int m = 0; m < RS / 2; m++) dst[m] = make_float2(0.f, 0.f);
    }
    // background term of dL/dalpha, -T_final / (1 - alpha) * (bg . dL/dpix) (backward.cu:1014), folded
    // into the accumulator: with A' = A - Tbg / T (Tbg = -T_final bg.dL/dpix, T the transmittance in
    // front of the current Gaussian), dL/dalpha = T_n (c . dL/dpix - A') and A' follows A's own recurrence
    // A' <- A' + alpha (c . dL/dpix - A') (T_n = T / (1 - alpha)), from A'_0 = bg . dL/dpix: the colour
    // behind the last Gaussian is the background.  Bitwise the plain recurrence when bg = 0.
    float bg_dot = cam.bg[0] * dp0 + cam.bg[1] * dp1 + cam.bg[2] * dp2;
    if (DUAL) bg_dot += cam.bg[0] * dq0 + cam.bg[1] * dq1 + cam.bg[2] * dq2;
    const v2f pix = v2f{(float)px, (float)py};
    const v2f dp01 = v2f{dp0, dp1}, dq01 = v2f{dq0, dq1};
    const v2f dp2q0 = v2f{dp2, dq0};  // (PACKC) the colour dot's second packed pair
    // (MOM) per-pixel products of the colour gradient the colour moments need
    [[maybe_unused]] const float mdp2[3] = {dp0 * dp0, dp1 * dp1, dp2 * dp2};
    [[maybe_unused]] const float mdpp[6] = {dp0 * dp0, dp0 * dp1, dp0 * dp2, dp1 * dp1, dp1 * dp2, dp2 * dp2};
    float T = T_final, A = bg_dot;
    [[maybe_unused]] float ablate_sink = 0.f;  // (timing ablation 1)
    const int my_e = row_entry(lane);
    // Slots start zero; after every batch the used slots (those of the batch's entries, every slot a row
    // list can have written) are cleared, and the pad slot only ever receives zeros.
    constexpr bool kBulkClear = !OPAC;
    for (int q = tid; q < (BS + 1) * NV; q += TILE_PIX) s_acc[q] = 0.f;
    const uint32_t* my_list = s_list + (4 * w + row) * LS;
    if (tid == 0) {
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        s_a[BB] = z;
        s_b[BB] = z;
        s_c[BB] = z;
        if (DUAL && !PACKC) s_d[BB] = z;
    }
    // Batch staging, software-pipelined two batches deep: thread t < batch holds entry t's
    // render record (already in its LDS form) and block-sum word for the next batch, and the
    // sorted list entry for the batch after it, so neither dependent load (list entry ->
    // record) is waited on while a batch is rasterised; the instance slot is formed at staging.
    float4 pa = make_float4(0.f, 0.f, 0.f, 0.f), pb = pa, pc = pa, pd = pa;
    uint32_t pbs = 0, pm = 0, prh = 0;  // prh: tile-rect hi (q3.w) when q3 is not staged
    PointEntry pn = 0;
    auto fetch_entry = [&](int hi_) {
        if (tid < min(BB, hi_)) pn = point_list[range.x + (uint32_t)(hi_ - 1 - tid)];
    };
    auto fetch_rec = [&](int hi_) {
        if (tid < min(BB, hi_)) {
            const uint32_t gi = pe_id(pn);
            pm = pe_mask(pn);
            const RenderRec r = load_rr(rr, gi);
            pbs = blocksums[gi >> cam.pre_shift];
            pa = r.q0; pb = r.q1; pc = r.q2;
            if (DUAL && !PACKC) {
                pd = r.q3;
            } else {
                prh = __float_as_uint(r.q3.w);
                if (PACKC) pd.x = r.q3.x;
            }
        }
    };
    fetch_entry((int)bmax);
    fetch_rec((int)bmax);
    fetch_entry((int)bmax - BB);
    const uint32_t mean4 = sched_mean4(cam, guard.counters);
    const bool multi_round = sched_multi_round(cam);
    int hi_pf = (int)bmax;  // the batch start the staged registers hold
    dg.phase(0);
    for (int hi = (int)bmax; hi > 0;) {
        prio_by_remaining(hi, mean4, multi_round);
        if (hi != hi_pf) {  // the previous batch was cut by its slot budget: re-fetch (rare)
            fetch_entry(hi);
            fetch_rec(hi);
            fetch_entry(hi - BB);
        }
        const int cmax = min(BB, hi);
        int ts_ = tid;
        asm volatile("" : "+v"(ts_));  // staging addresses formed here, not hoisted across the batch loop
        if (ts_ < cmax) {
            s_u[ts_] = instance_slot(make_uint2(__float_as_uint(pc.w), (DUAL && !PACKC) ? __float_as_uint(pd.w) : prh),
                                     pbs + __float_as_uint(pb.w), tx, ty);
            s_a[ts_] = pa;
            s_b[ts_] = pb;
            s_c[ts_] = PACKC ? make_float4(pc.x, pc.y, pc.z, pd.x) : pc;
            if (DUAL && !PACKC) s_d[ts_] = pd;
            s_mask[ts_] = (uint16_t)pm;  // the instance's exact 4x4-block mask (sorted list entry)
        }
        __syncthreads();
        dg.phase(1);
        fetch_rec(hi - BB);        // records of the next batch (list entries loaded a batch ago)
        fetch_entry(hi - 2 * BB);  // list entries of the batch after it
        hi_pf = hi - BB;
        // entries j with pos = hi-1-j >= rmax lie behind every pixel of the block
        const int jmin[4] = {hi - rm[0], hi - rm[1], hi - rm[2], hi - rm[3]};
        // list words: (LDS byte offset of entry j's staged record, 16 j) | (byte offset of its slot) << 16
        static_assert(16 * BB < 65536 && (BS + 1) * NV * 4 < 65536, "list words hold 16-bit byte offsets");
        SlotLists sl = build_row_slot_lists(s_mask, s_base, cmax, BS, w, jmin, s_list + 4 * w * LS, LS,
                                            (uint32_t)(16 * BB) | ((uint32_t)(BS * NV * 4) << 16), 16u,
                                            (uint32_t)(NV * 4));
        if constexpr (kDupPhase == 3) {  // (VALU census only: the same lists again)
            asm volatile("" ::: "memory");
            sl = build_row_slot_lists(s_mask, s_base, cmax, BS, w, jmin, s_list + 4 * w * LS, LS,
                                      (uint32_t)(16 * BB) | ((uint32_t)(BS * NV * 4) << 16), 16u, (uint32_t)(NV * 4));
        }
        const int n = sl.len, cnt = sl.cnt;
        dg.phase(2);
        const int jlo16 = 16 * (hi - (int)last);  // pos = hi-1-j < last  <=>  j >= jlo  <=>  16 j >= 16 jlo
        for (int i = 0; i < n; i += 4) {
            // this lane's entry slot (the reduction's writer lanes): the high half of its entry's word
            const uint32_t soff = reinterpret_cast<const uint16_t*>(my_list + i + my_e)[1];
            // byte offsets 16 j of the step's entries in s_a / s_b / s_c / s_d: the low halves of the four
            // words, one ds_read_u16 each (zero-extended by the load: no v_and per entry on the VALU)
            int jb[4];
#pragma unroll
            for (int k = 0; k < 4; k++) jb[k] = (int)reinterpret_cast<const uint16_t*>(my_list + i + k)[0];
            auto rec = [&](const float4* arr, int k) {
                return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(arr) + jb[k]);
            };
            v2f d[4];
            float G[4], araw[4], alpha[4];
            bool ok[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float4 a = rec(s_a, k), b = rec(s_b, k);
                d[k] = pix_delta(a, pix);
                const float p2 = eval_p2(a, b, d[k]);                       // log2(e) * power
                // position in the tile list before the pixel's last contributor, power <= 0, alpha >= 1/255
                // (alpha = min(0.99, araw) >= 1/255 <=> araw >= 1/255); the pad entry has opacity 0.
                // Non-contributing pairs continue with alpha 0: T and A then pass through unchanged
                // (1 / (1 - 0) == 1 exactly).  Without the opacity sum the mask is applied to araw (a
                // masked pair's h = araw dL/dalpha is then 0, and G may even be inf there); with it,
                // G dL/dalpha needs a finite G and a masked dL/dalpha.
                G[k] = __builtin_amdgcn_exp2f(OPAC ? fminf(p2, 0.f) : p2);
                const float ar = b.y * G[k];
                ok[k] = jb[k] >= jlo16 && p2 <= 0.0f && ar >= 1.0f / 255.0f;
                araw[k] = (OPAC || ok[k]) ? ar : 0.f;
                alpha[k] = fminf(0.99f, araw[k]);
                if (OPAC) alpha[k] = ok[k] ? alpha[k] : 0.f;
            }
            {
                bool pad[4];
#pragma unroll
                for (int k = 0; k < 4; k++) pad[k] = jb[k] == 16 * BB;
                dg.step(pad, ok);
            }
            // (no wave-uniform skip of steps without a contributing pair: 0.04 % of steps, and the test
            // cost 2 VALU + a branch per step; config-4 dual 396 -> 387 us without it)
            // serial part (in list order): T and A, then dL/dalpha and dchannel/dcolor
            float dLa[4], dch[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float4 c = rec(s_c, k);
                float cd;
                if (DUAL && Q2 == 1 && PACKC) {  // (c.x, c.y) . dp01 + (c.z, c.w) . (dp2, dq0): pk_mul + pk_fma + add
                    const v2f t = __builtin_elementwise_fma(v2f{c.z, c.w}, dp2q0, v2f{c.x, c.y} * dp01);
                    cd = t.x + t.y;
                } else if (DUAL && Q2 == 1) {
                    const float c2x = rec(s_d, k).x;
                    const v2f t = v2f{c.x, c.y} * dp01;
                    cd = __builtin_fmaf(c.z, dp2, __builtin_fmaf(c2x, dq0, t.x + t.y));
                } else if (DUAL) {
                    const float4 c2 = rec(s_d, k);
                    const v2f t = v2f{c.x, c.y} * dp01 + v2f{c2.x, c2.y} * dq01;
                    cd = __builtin_fmaf(c.z, dp2, __builtin_fmaf(c2.z, dq2, t.x + t.y));
                } else if (C1 == 1) {  // dL/dpix channels 1, 2 zero on this tile: the same value (up to a zero's sign)
                    cd = c.x * dp0;
                } else {
                    const v2f t = v2f{c.x, c.y} * dp01;
                    cd = __builtin_fmaf(c.z, dp2, t.x + t.y);
                }
                const float inv = __builtin_amdgcn_rcpf(1.f - alpha[k]);   // v_rcp_f32 (~1 ulp)
                const float Tn = T * inv;                                   // T / (1 - alpha), backward.cu:978
                const float e = cd - A;
#if GSR_PK_XD
                const v2f xd = v2f{e, alpha[k]} * Tn;  // (e Tn, alpha Tn): one v_pk_mul_f32, the same two products
                const float x = xd.x;
                dch[k] = xd.y;                          // 0 when masked
#else
                const float x = e * Tn;
                dch[k] = alpha[k] * Tn;                 // 0 when masked
#endif
                dLa[k] = (OPAC && !ok[k]) ? 0.f : x;    // (without OPAC: h = araw dLa is 0 when masked)
                T = Tn;  // masked pairs: alpha = 0 and v_rcp_f32(1) == 1 exactly (tools/micro/rcp_one.hip)
                A = __builtin_fmaf(alpha[k], e, A);     // unchanged when masked
            }
            // Per pair: (hx, hy, hx*dx, hx*dy, hy*dy, G*dL/dalpha, dch*dL/dpix, dch*dL/dpix2) with
            // h = G * dL/dG = (o * G) * dL/dalpha.  gauss_bwd turns them into the reference's
            // per-pair quantities (backward.cu:1020-1038): dmean2D = -ddel * (Q [hx, hy]),
            // dconic = -0.5 * (hxx, hxy, hyy); both are linear in the sums (Q is per Gaussian).
            float* dst = reinterpret_cast<float*>(reinterpret_cast<char*>(s_acc) + soff);  // the (entry, block) slot
            if constexpr (MOM > 0) {  // backward_power == 2: the pair's second moments (gauss_bwd_mom_kernel)
                MomIn e[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
#if GSR_PK_XD
                    const v2f ho = v2f{araw[k], G[k]} * dLa[k];
                    const float h = ho.x, o = ho.y;
#else
                    const float h = araw[k] * dLa[k], o = G[k] * dLa[k];
#endif
                    const float hx = h * d[k].x, hy = h * d[k].y;
                    e[k].m20 = hx * hx;
                    e[k].m11 = hx * hy;
                    e[k].m02 = hy * hy;
                    e[k].dx = d[k].x;
                    e[k].dy = d[k].y;
                    e[k].xx = d[k].x * d[k].x;
                    e[k].xy = d[k].x * d[k].y;
                    e[k].yy = d[k].y * d[k].y;
                    e[k].o2 = o * o;
                    e[k].c2 = dch[k] * dch[k];
                    const float hc = h * dch[k];
                    e[k].hc[0] = hc * dp0;
                    e[k].hc[1] = hc * dp1;
                    e[k].hc[2] = hc * dp2;
                }
                // passes of 4 moments (the reduction's cost is per value: the pass size only sets how
                // many products are live at once)
                mom_pass<MOM, 0, 4>(e, mdp2, mdpp, lane, dst);
                mom_pass<MOM, 4, 4>(e, mdp2, mdpp, lane, dst);
                mom_pass<MOM, 8, 4>(e, mdp2, mdpp, lane, dst);
                if constexpr (MOM == 1) {
                    mom_pass<MOM, 12, 4>(e, mdp2, mdpp, lane, dst);
                } else {
                    mom_pass<MOM, 12, 4>(e, mdp2, mdpp, lane, dst);
                    mom_pass<MOM, 16, 4>(e, mdp2, mdpp, lane, dst);
                    mom_pass<MOM, 20, 4>(e, mdp2, mdpp, lane, dst);
                    mom_pass<MOM, 24, 5>(e, mdp2, mdpp, lane, dst);
                    mom_pass<MOM, 29, 5>(e, mdp2, mdpp, lane, dst);
                }
            } else if constexpr (NV <= 6) {  // one reduction over all values
                float v[4 * NV];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    pair_geom<OPAC>(v + NV * k, araw[k], dLa[k], G[k], d[k]);
                    pair_colours<COL1, COL2, Q2, C1>(v + NV * k + O_C1, dch[k], dp01, dp2, dq0, dq01, dq2);
                }
                if constexpr (kAblate == 1) {
#pragma unroll
                    for (int q = 0; q < 4 * NV; q++) ablate_sink += v[q];
                } else {
                    reduce_store<NV>(v, lane, dst, true);
                }
            } else {  // wide variants: geometric (+ opacity), then colour sums (register pressure)
                constexpr bool OP_A = OPAC && GSR_BWD_SPLIT6;
                constexpr int NA = 5 + (OP_A ? 1 : 0), NB = NV - NA;
                {
                    float v[4 * NA];
#pragma unroll
                    for (int k = 0; k < 4; k++) pair_geom<OP_A>(v + NA * k, araw[k], dLa[k], G[k], d[k]);
                    reduce_store<NA>(v, lane, dst, true);
                }
                {
                    float v[4 * NB];
                    constexpr int OB = (OPAC && !OP_A) ? 1 : 0;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (OB) v[NB * k] = G[k] * dLa[k];
                        pair_colours<COL1, COL2, Q2, C1>(v + NB * k + OB, dch[k], dp01, dp2, dq0, dq01, dq2);
                    }
                    reduce_store<NB>(v, lane, dst + NA, true);
                }
            }
        }
        dg.phase(3);
        __syncthreads();
        dg.phase(4);
        // Entry totals: TPE threads per entry, thread q of an entry owns values m = q, q + TPE, ...
        // and adds the entry's consecutive block slots in ascending block order (deterministic);
        // the TPE threads store adjacent floats of the packed record.
        constexpr int TPE = TILE_PIX / BB, NQ = (NV + TPE - 1) / TPE, NQR = (RS + TPE - 1) / TPE;
        int t_ = tid;
        asm volatile("" : "+v"(t_));  // addresses formed here, not hoisted across the batch loop (VGPRs)
        const int e = t_ / TPE, q = t_ % TPE;
        if (kAblate != 2 && e < cnt) {
            float c[NQ];
#pragma unroll
            for (int i = 0; i < NQ; i++) c[i] = 0.f;
            const int nb = __popc((uint32_t)s_mask[e]);
            float* src = s_acc + (int)s_base[e] * NV;
            for (int b = 0; b < nb; b++, src += NV) {
#pragma unroll
                for (int i = 0; i < NQ; i++)
                    if (q + TPE * i < NV) {
                        c[i] += src[q + TPE * i];
                        if constexpr (!kBulkClear) src[q + TPE * i] = 0.f;
                    }
            }
            float* dst = inst + (size_t)RS * s_u[e];  // packed record (RecLayout): the NV sums, zero pad
#pragma unroll
            for (int i = 0; i < NQR; i++)
                if (q + TPE * i < RS) {
                    // (streaming stores measured neutral for render_bwd and 3-9 us slower for the gauss_bwd that
                    // reads the records next: profiles/r4l_ab_nt.txt, r4m_ab_nt.txt)
                    const float val = i < NQ ? c[i] : 0.f;  // (C1 = 1: the two absent colour sums are zero)
                    if (GSR_NT_STORES) __builtin_nontemporal_store(val, &dst[q + TPE * i]);
                    else dst[q + TPE * i] = val;
                }
        }
        dg.phase(5);
        __syncthreads();
        // The batch's slots back to zero for the next batch's reduction: the used range [0, slots of entries
        // < cnt) as contiguous float4 stores (the next batch's staging barrier orders them before its walk).
        // Re-zeroing each slot right after reading it cost bank-conflicted scattered stores in the totals
        // (slot stride NV = 6 words: entries whose slot bases differ by 16 share banks).  Only in the lean
        // variants (no opacity gradient: the tracking render): the full-gradient ones are at their VGPR
        // bound, where the sweep's bookkeeping spilled (render_bwd<1,1,1,1,1,0>: 16 B of scratch, +10 us at
        // config 4), so they keep re-zeroing in the totals
        if constexpr (kBulkClear) {
            const int used = cnt > 0 ? (int)s_base[cnt - 1] + __popc((uint32_t)s_mask[cnt - 1]) : 0;
            float4* const a4 = reinterpret_cast<float4*>(s_acc);
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int q4 = tid; q4 < (used * NV + 3) / 4; q4 += TILE_PIX) a4[q4] = z;
        }
        dg.phase(6);
        dg.batch();
        hi -= cnt;
    }
    if (kAblate == 1 && ablate_sink == 1.2345f) inst[0] = ablate_sink;  // keeps the per-pair values alive
}

template <bool DUAL, bool OPAC, bool COL1, bool COL2, int Q2 = 3, int MOM = 0>
__global__ void __launch_bounds__(TILE_PIX, (bwd_waves<DUAL, OPAC, COL1, COL2, Q2, MOM>()))
render_bwd_kernel(Camera cam, const uint2* __restrict__ ranges, const PointEntry* __restrict__ point_list,
                  const float4* __restrict__ rr, const uint32_t* __restrict__ blocksums,
                  const float* __restrict__ final_T,
                  const uint32_t* __restrict__ n_contrib, const float* __restrict__ dL_dpix,
                  const float* __restrict__ dL_dpix2, float* __restrict__ inst, BwdGuard guard,
                  unsigned long long* clk) {
    kclock_begin(clk);
    RenderDiag dg;  // (diagnostics builds only, gsr_diag.h)
    dg.begin();
    if (guard.overflow()) {  // invalid forward state (static-mode overflow): touch nothing
        kclock_end(clk);
        return;
    }
    __shared__ __attribute__((aligned(16))) char smem[BwdShape<DUAL, OPAC, COL1, COL2, Q2, MOM>::bytes];
    const int tid = threadIdx.x;
    const int tile = sched_tile(cam), tx = tile % cam.gx, ty = tile / cam.gx;
    dg.tile(tile);
    const int px = tx * TILE_X + tile_px(tid);
    const int py = ty * TILE_Y + tile_py(tid);
    const bool inside = px < cam.W && py < cam.H;
    const int pid = py * cam.W + px;
    const int HW = cam.W * cam.H;
    BwdPix pin{0.f, 0u, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (inside) {
        pin.T_final = final_T[pid];
        pin.last = n_contrib[pid];
        pin.dp0 = dL_dpix[pid];
        pin.dp1 = dL_dpix[HW + pid];
        pin.dp2 = dL_dpix[2 * HW + pid];
        if (DUAL) {
            pin.dq0 = dL_dpix2[pid];
            if (Q2 == 3) {
                pin.dq1 = dL_dpix2[HW + pid];
                pin.dq2 = dL_dpix2[2 * HW + pid];
            }
        }
    }
    if constexpr (!DUAL && COL1 && MOM == 0) {
        // a tile whose incoming gradient has zero channels 1 and 2 everywhere (SplaTAM's depth/silhouette
        // render: get_loss differentiates only its depth channel, scripts/splatam.py:262-270) forms one colour
        // sum per pair instead of three; the others are exactly zero (records identical up to a zero's sign)
        if (!__syncthreads_or(pin.dp1 != 0.f || pin.dp2 != 0.f)) {
            bwd_tile<DUAL, OPAC, COL1, COL2, Q2, MOM, 1>(cam, tile, pin, ranges, point_list, rr, blocksums, inst, guard,
                                                         smem, dg);
            dg.end();
            kclock_end(clk);
            return;
        }
    }
    bwd_tile<DUAL, OPAC, COL1, COL2, Q2, MOM>(cam, tile, pin, ranges, point_list, rr, blocksums, inst, guard, smem, dg);
    dg.end();
    kclock_end(clk);
}

// The tracking iteration's render in one launch per tile (SplaTAM get_loss(tracking=True) with a static
// loss seed, scripts/splatam.py:220-353): the dual forward with the L1 loss epilogue, then -- in the same
// workgroup, its LDS reused -- the back-to-front walk of the depth-channel / geometric backward
// (render_bwd_kernel<true, false, false, true, 1>) from the pixel state still in registers.  The loss
// gradient is per pixel, so a tile's backward needs nothing from other tiles.  Saves the second launch
// (dispatch, drain, the end-of-kernel writeback), the backward's per-pixel reads (T, n_contrib, dL/dpix)
// and the forward's gradient-image stores.  Results are bitwise those of render_fwd + render_bwd.
constexpr size_t track_lds_bytes() {
    return FwdShape<true>::bytes > BwdShape<true, false, false, true, 1, 0>::bytes
               ? FwdShape<true>::bytes
               : BwdShape<true, false, false, true, 1, 0>::bytes;
}
// IMAGES = false: the images (and final_T / n_contrib / the block maxima) are not stored -- a separate
// instantiation, so that no store (and no wait the compiler places for one) is left in the code
template <bool IMAGES>
__global__ void __launch_bounds__(TILE_PIX, 5)
render_track_kernel(Camera cam, const uint2* __restrict__ ranges, PointEntry* __restrict__ point_list,
                    uint64_t* __restrict__ keys, const float4* __restrict__ rr, const uint32_t* __restrict__ blocksums,
                    float* __restrict__ final_T, uint32_t* __restrict__ n_contrib, float* __restrict__ out_color,
                    float* __restrict__ out_color2, float* __restrict__ out_depth, SpecGuard guard,
                    unsigned long long* clk, TrackL1 l1, float* __restrict__ inst) {
    kclock_begin(clk);
    RenderDiag dg;
    dg.begin();
    if (guard.overflow()) {
        kclock_end(clk);
        return;
    }
    __shared__ __attribute__((aligned(16))) char smem[track_lds_bytes()];
    if constexpr (!IMAGES) {  // (fwd_epilogue stores nothing for a null final_T)
        final_T = nullptr;
        cam.rowmax = nullptr;
    }
    const int tile = sched_tile(cam);
    dg.tile(tile);
    const FwdPix f = fwd_tile<true>(cam, tile, ranges, point_list, keys, rr, guard, smem, dg);
    float grad[4];
    // (the loss arrival stays here: moved after the backward it put the last workgroup's sum at the kernel's
    // end, within noise or 0.5 us slower: profiles/r4o_ab_l1_defer.txt)
    // STORE_GRADS = false: the gradient images are not formed here, and the C entry passes l1.dL_dim /
    // l1.dL_dds as NULL (a variant that stores them needs real image pointers from gsr_capi.hip)
    constexpr bool kStoreGrads = false;
    static_assert(!kStoreGrads, "render_track_kernel's callers pass no gradient images");
    fwd_epilogue<true, true, kStoreGrads>(cam, tile, f, final_T, n_contrib, out_color, out_color2, out_depth, l1,
                                          grad);
    __syncthreads();  // the forward's LDS (and its sorted point_list stores) before the backward reuses them
    const BwdPix pin{f.T, f.last16 >> 4, grad[0], grad[1], grad[2], grad[3], 0.f, 0.f};
    Camera cb = cam;
    cb.rowmax = nullptr;  // the block maxima from the registers
    bwd_tile<true, false, false, true, 1, 0>(cb, tile, pin, ranges, point_list, rr, blocksums, inst,
                                             BwdGuard{guard.counters, guard.cap_inst}, smem, dg);
    dg.end();
    kclock_end(clk);
}

int track_records_stride() { return BwdShape<true, false, false, true, 1, 0>::RS; }

hipError_t launch_render_track(const Camera& cam, const uint2* ranges, uint64_t* point_list, uint64_t* keys,
                               GeomPtrs geo, float* final_T, uint32_t* n_contrib, float* out_color,
                               float* out_color2, float* out_depth, SpecGuard guard, const TrackL1& l1, float* inst,
                               hipStream_t s, unsigned long long* clk) {
    auto k = final_T != nullptr ? render_track_kernel<true> : render_track_kernel<false>;
    hipLaunchKernelGGL(k, dim3(cam.gx * cam.gy), dim3(TILE_PIX), 0, s, cam, ranges, point_list,
                       keys, geo.rr, geo.blocksums, final_T, n_contrib, out_color, out_color2, out_depth, guard, clk,
                       l1, inst);
    return hipGetLastError();
}

template <bool DUAL, bool OPAC, bool COL1, bool COL2, int Q2 = 3>
static auto bwd_variant() { return render_bwd_kernel<DUAL, OPAC, COL1, COL2, Q2>; }

// The variant launch_render_bwd picks for (need, dual) and its record layout.
RecLayout bwd_rec_layout(unsigned need, bool dual) {
    const bool op = need & NEED_OPACITY, c1 = need & NEED_COLORS, c2 = dual && (need & NEED_COLORS2);
    const int q2 = (dual && (need & NEED_DL2_CH0_ONLY)) ? 1 : 3;
    RecLayout L;
    int nv = 5;
    L.o_op = op ? nv : -1;
    nv += op ? 1 : 0;
    L.o_c1 = c1 ? nv : -1;
    nv += c1 ? 3 : 0;
    L.o_c2 = c2 ? nv : -1;
    L.n_c2 = c2 ? q2 : 0;
    nv += L.n_c2;
    L.stride = (nv + 1) & ~1;
    return L;
}

hipError_t launch_render_bwd(const Camera& cam, const uint2* ranges, const uint64_t* point_list, GeomPtrs geo,
                             const float* final_T, const uint32_t* n_contrib, const float* dL_dpix,
                             const float* colors2, const float* dL_dpix2, unsigned need, float* inst,
                             BwdGuard guard, hipStream_t s, unsigned long long* clk) {
    const bool op = need & NEED_OPACITY, c1 = need & NEED_COLORS, c2 = colors2 && (need & NEED_COLORS2);
    const bool q1 = need & NEED_DL2_CH0_ONLY;
    auto k = bwd_variant<false, true, true, false>();
    if (!colors2) {
        k = op ? (c1 ? bwd_variant<false, 1, 1, 0>() : bwd_variant<false, 1, 0, 0>())
               : (c1 ? bwd_variant<false, 0, 1, 0>() : bwd_variant<false, 0, 0, 0>());
    } else if (q1 && !op && !c1) {  // SplaTAM tracking: depth-channel gradient only
        k = c2 ? bwd_variant<true, 0, 0, 1, 1>() : bwd_variant<true, 0, 0, 0, 1>();
    } else if (q1) {  // SplaTAM mapping: every Gaussian gradient, depth channel of the second image
        k = op ? (c1 ? (c2 ? bwd_variant<true, 1, 1, 1, 1>() : bwd_variant<true, 1, 1, 0, 1>())
                     : (c2 ? bwd_variant<true, 1, 0, 1, 1>() : bwd_variant<true, 1, 0, 0, 1>()))
               : (c2 ? bwd_variant<true, 0, 1, 1, 1>() : bwd_variant<true, 0, 1, 0, 1>());
    } else {
        k = op ? (c1 ? (c2 ? bwd_variant<true, 1, 1, 1>() : bwd_variant<true, 1, 1, 0>())
                     : (c2 ? bwd_variant<true, 1, 0, 1>() : bwd_variant<true, 1, 0, 0>()))
               : (c1 ? (c2 ? bwd_variant<true, 0, 1, 1>() : bwd_variant<true, 0, 1, 0>())
                     : (c2 ? bwd_variant<true, 0, 0, 1>() : bwd_variant<true, 0, 0, 0>()));
    }
    hipLaunchKernelGGL(k, dim3(cam.gx * cam.gy), dim3(TILE_PIX), 0, s, cam, ranges, point_list, geo.rr, geo.blocksums,
                       final_T, n_contrib, dL_dpix, dL_dpix2, inst, guard, clk);
    return hipGetLastError();
}

// SHL: per-lane SH chain (g.shs may be set).  Without it (colours precomputed, or SH handled by
// the staged sh_bwd_kernel) g.shs is NULL at compile time, and the 48-float dsh array and the SH
// chain drop out of the kernel (mapping variant: 142 -> fewer VGPRs, more waves per SIMD).
// at most 5 waves per SIMD: at 78-80 VGPRs the kernel would run 6, and the sixth wave measured slower for the
// mapping variant (1 M anisotropic Gaussians: 65.0 -> 64.0 us capped) and no faster for tracking
// (profiles/r5z_ab_gauss_bwd_waves.txt)
template <bool POSE, bool SHL>
__device__ __forceinline__ void gauss_bwd_body(Camera cam, GaussIn g, GeomPtrs geo, const int* __restrict__ radii,
                                               const float* __restrict__ inst, RecLayout rec, GradsOut out,
                                               BwdGuard guard, PoseFuse pf) {
    if constexpr (!SHL) {
        g.shs = nullptr;
        g.M = 0;
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (!POSE && i >= g.P) return;  // (POSE: every lane takes part in the workgroup sum)
    const bool live = i < g.P;
    const int nsh = g.shs ? (cam.sh_degree + 1) * (cam.sh_degree + 1) : 0;
    float g2[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float dcol2[3] = {0.f, 0.f, 0.f};
    float dmean[3] = {0.f, 0.f, 0.f}, dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, dscale[3] = {0.f, 0.f, 0.f},
          drot[4] = {0.f, 0.f, 0.f, 0.f};
    float dsh[48];
#pragma unroll
    for (int k = 0; k < 48; k++) dsh[k] = 0.f;
    // the Gaussian's geometry: recomputed from the world-frame map and the pre-step pose (tracking
    // forward that did not store its rendervars, PoseFuse::ls) or read from GaussIn
    GaussGeom gg;
    gg.m = make_float3(0.f, 0.f, 0.f);
    gg.s = make_float3(0.f, 0.f, 0.f);
    gg.q = make_float4(0.f, 0.f, 0.f, 0.f);
    // POSE: the frame's (pre-step) pose is workgroup-uniform: formed once by thread 0 (8 IEEE divisions and 2
    // square roots per lane otherwise) and read from LDS -- the same bits.  The Gaussian's own inputs (radius,
    // record range, the world-frame transform inputs) are loaded ahead of that barrier: loads issued after a
    // __syncthreads would wait for thread 0's pose chain (its loads and the make_pose arithmetic)
    const int rad = live ? radii[i] : 0;
    const bool xf_geom = POSE && pf.ls;
    TrackXf x;
    x.mw = pf.means_world; x.ur = pf.unnorm_rot; x.ls = pf.ls; x.scols = pf.scols;
    XfRaw xr{};
    if (xf_geom && live) xr = track_xform_load(x, i, false);
    uint32_t off = 0, cnt = 0, tl = 0xFFFFFFFFu;  // tl: live-tile mask (Camera::cull: culled slots are unwritten)
    if (POSE && live && rad > 0) {
        off = geo.offsets[i];
        cnt = geo.tiles[i];
        tl = reinterpret_cast<const uint32_t*>(geo.bin)[4 * (size_t)i + 3];
    }
    __shared__ Pose s_pose;
    if constexpr (POSE) {
        if (pf.ls || pf.scols != 1) {
            if (threadIdx.x == 0) s_pose = make_pose(pf.cam_q, pf.cam_t, pf.qs);
            __syncthreads();
        }
    }
    if (live && (POSE || rad > 0)) {  // (the pose sums need every live Gaussian's mean)
        if (xf_geom) {
            const Pose ps = s_pose;
            float m[3], sv[3];
            track_xform_geom_raw(xr, x.scols, ps, m, gg.q, sv);
            gg.m = make_float3(m[0], m[1], m[2]);
            gg.s = make_float3(sv[0], sv[1], sv[2]);
        } else {
            gg = load_geom(g, i);
        }
    }
    if (live && rad > 0 && !guard.overflow()) {  // overflow: zero gradients, no record reads
        if (!POSE) {
            off = geo.offsets[i];
            cnt = geo.tiles[i];
            tl = reinterpret_cast<const uint32_t*>(geo.bin)[4 * (size_t)i + 3];
        }
        // fixed-order sum of the Gaussian's instance records (deterministic)
        float acc[INST_REC_MAX];
#pragma unroll
        for (int m = 0; m < INST_REC_MAX; m++) acc[m] = 0.f;
        const int np = rec.stride / 2;
        // RU records' loads issued together (one memory round trip per RU instances instead of
        // per instance), then added in instance order: the same sums, bit for bit
        constexpr int RU = 4;
        for (uint32_t e0 = 0; e0 < cnt; e0 += RU) {
            float2 v[RU][INST_REC_MAX / 2];
#pragma unroll
            for (int k = 0; k < RU; k++) {
                const float2* r = reinterpret_cast<const float2*>(inst + (size_t)rec.stride * (off + e0 + k));
#pragma unroll
                for (int m = 0; m < INST_REC_MAX / 2; m++)
                    v[k][m] = (m < np && e0 + k < cnt && tile_live(tl, e0 + k)) ? r[m] : make_float2(0.f, 0.f);
            }
#pragma unroll
            for (int k = 0; k < RU; k++)
                if (e0 + k < cnt && tile_live(tl, e0 + k)) {  // (a culled slot's record would be +0: skipped exactly)
#pragma unroll
                    for (int m = 0; m < INST_REC_MAX / 2; m++)
                        if (m < np) {
                            acc[2 * m] += v[k][m].x;
                            acc[2 * m + 1] += v[k][m].y;
                        }
                }
        }
#pragma unroll
        for (int m = 0; m < 5; m++) g2[m] = acc[m];
#pragma unroll
        for (int m = 0; m < INST_REC_MAX; m++) {  // constant-index selects (no dynamic register indexing)
            if (m == rec.o_op) g2[5] = acc[m];
#pragma unroll
            for (int k = 0; k < 3; k++) {
                if (rec.o_c1 >= 0 && m == rec.o_c1 + k) g2[6 + k] = acc[m];
                if (rec.o_c2 >= 0 && k < rec.n_c2 && m == rec.o_c2 + k) dcol2[k] = acc[m];
            }
        }
        // instance records hold (hx, hy, hxx, hxy, hyy, dopacity, dcolor) sums (render_bwd_kernel);
        // the conic is recomputed exactly as preprocess computed it (the render record keeps
        // only its exp2-scaled form)
        float ca, cb, cc, c3[6];
        Proj pj;
        gaussian_conic(cam, g, gg, i, ca, cb, cc, &pj, c3);
        const float ddelx = (float)(0.5 * cam.W), ddely = (float)(0.5 * cam.H);  // backward.cu:935-936
        const float hx = g2[0], hy = g2[1];
        g2[0] = -(ca * hx + cb * hy) * ddelx;
        g2[1] = -(cc * hy + cb * hx) * ddely;
        g2[2] *= -0.5f;
        g2[3] *= -0.5f;
        g2[4] *= -0.5f;
        const unsigned clamped = g.shs ? geo.clamp[i] : 0u;  // (SH colour clamping; not stored without SH)
        gauss_chain(cam, g, gg, i, g2, clamped, dmean, dcov, dscale, drot, dsh, nsh, !POSE || pf.scols != 1, &pj, c3);
    }
    if constexpr (POSE) {
        // tracking: the pose sums of this Gaussian (track_transform_bwd_kernel's, gsr_glue.hip), then
        // one fixed-order workgroup sum, published; the last workgroup finishes the pose chain / Adam
        __shared__ float s_red[4 * POSE_PARTS];
        __shared__ float s_tot[POSE_PARTS];
        float v[POSE_PARTS];
#pragma unroll
        for (int k = 0; k < POSE_PARTS; k++) v[k] = 0.f;
        float c[4] = {0.f, 0.f, 0.f, 0.f};
        if (pf.scols != 1) {
            const Pose ps = s_pose;  // (c only: the same normalised quaternion)
#pragma unroll
            for (int k = 0; k < 4; k++) c[k] = ps.c[k];
        }
        if (live) {
            const float mci[3] = {gg.m.x, gg.m.y, gg.m.z};
            pose_partials_m(v, i, dmean, dcol2, pf.scols != 1 ? drot : nullptr, pf.means_world, pf.unnorm_rot, mci,
                            pf.w2c, c);
        }
        block_sum<POSE_PARTS>(v, s_red, s_tot);
        __syncthreads();
        if (threadIdx.x < POSE_PARTS) st_agent(pf.part + POSE_PARTS * blockIdx.x + threadIdx.x, s_tot[threadIdx.x]);
        if constexpr (kAblate == 3) return;  // timing ablation: no pose tail (invalid pose update)
#if GSR_POSE_TAIL == 1
        // One-level fixed-order sum: the last workgroup to arrive (grouped arrival counters) reads
        // all partials as one coalesced float stream (thread t: floats t, t + 256, ... = value
        // k = t % 16 of the partials t / 16, t / 16 + 16, ... in order, 40 loads in flight per round
        // trip), then adds the 16 classes of each value in order through LDS.  Three serial memory
        // round trips (publish, arrive, gather) instead of the two-level tail's six.
        {
            const int nb = gridDim.x;
            if (!last_block_arrive_grouped(reinterpret_cast<uint32_t*>(pf.part + POSE_PARTS * nb))) return;
            if constexpr (kAblate == 4) return;  // timing ablation: arrival only
            static_assert(256 % POSE_PARTS == 0, "a thread keeps one value index");
            constexpr int CH = 40;
            const int total = POSE_PARTS * nb;
            float acc = 0.f;
            for (int f0 = threadIdx.x; f0 < total; f0 += CH * 256) {
                float buf[CH];
#pragma unroll
                for (int u = 0; u < CH; u++) {
                    const int f = f0 + 256 * u;
                    buf[u] = f < total ? ld_agent(pf.part + f) : 0.f;
                }
#pragma unroll
                for (int u = 0; u < CH; u++) acc += buf[u];
            }
            __shared__ float s_cls[256];
            s_cls[threadIdx.x] = acc;
            __syncthreads();
            if (threadIdx.x < POSE_PARTS) {
                float t = 0.f;
#pragma unroll
                for (int c = 0; c < 256 / POSE_PARTS; c++) t += s_cls[threadIdx.x + POSE_PARTS * c];
                s_tot[threadIdx.x] = t;
            }
            __syncthreads();
            if (kAblate != 5 && threadIdx.x == 0) {  // (5: timing ablation, no pose_fin)
                const PoseAdam adam{pf.lr_q, pf.lr_t, pf.beta1, pf.beta2, (float)(1.0 - pf.beta1),
                                    (float)(1.0 - pf.beta2), (float)pf.eps, pf.adam_state, pf.cam_q, pf.cam_t,
                                    pf.guard, pf.cap, pf.loss, pf.best};
                pose_fin(s_tot, pf.cam_q, pf.qs, pf.dq, pf.dt, adam);
            }
            return;
        }
#endif
        // Two-level fixed-order sum of the ~1200 workgroup partials: the last workgroup of each
        // of the 16 arrival groups (b = g mod 16) adds its group's partials (one per thread)
        // and publishes the group sum; the last group then adds the 16 group sums.  (One
        // workgroup reading all partials serially cost ~18 us more than the separate pose kernel.)
        const int nb = gridDim.x;
        uint32_t* ctr = reinterpret_cast<uint32_t*>(pf.part + POSE_PARTS * nb);
        float* gsum = pf.part + POSE_PARTS * nb + ARRIVE_GROUPED_WORDS;
        __shared__ uint32_t s_flag;
        const uint32_t g = (uint32_t)blockIdx.x & 15u;
        const uint32_t ngroups = nb < 16 ? (uint32_t)nb : 16u;
        __builtin_amdgcn_s_waitcnt(0x0F70);  // s_waitcnt vmcnt(0): the partial stores have landed
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t gsize = (uint32_t)nb / 16u + (g < (uint32_t)nb % 16u ? 1u : 0u);
            uint32_t* gc = ctr + ARRIVE_STRIDE * (1 + g);
            const bool last = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1;
            if (last) __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_flag = last;
        }
        __syncthreads();
        if (!s_flag) return;
#pragma unroll
        for (int k = 0; k < POSE_PARTS; k++) v[k] = 0.f;
        for (int b = (int)g + 16 * threadIdx.x; b < nb; b += 16 * 256)
#pragma unroll
            for (int k = 0; k < POSE_PARTS; k++) v[k] += ld_agent(pf.part + POSE_PARTS * b + k);
        __syncthreads();
        block_sum<POSE_PARTS>(v, s_red, s_tot);
        __syncthreads();
        if (threadIdx.x < POSE_PARTS) st_agent(gsum + POSE_PARTS * g + threadIdx.x, s_tot[threadIdx.x]);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
        if (threadIdx.x == 0) {
            const bool last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
            if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_flag = last;
        }
        __syncthreads();
        if (!s_flag) return;
#pragma unroll
        for (int k = 0; k < POSE_PARTS; k++) v[k] = threadIdx.x < ngroups ? ld_agent(gsum + POSE_PARTS * threadIdx.x + k) : 0.f;
        __syncthreads();
        block_sum<POSE_PARTS>(v, s_red, s_tot);
        __syncthreads();
        if (threadIdx.x == 0) {
            const PoseAdam adam{pf.lr_q, pf.lr_t, pf.beta1, pf.beta2, (float)(1.0 - pf.beta1),
                                (float)(1.0 - pf.beta2), (float)pf.eps, pf.adam_state, pf.cam_q, pf.cam_t,
                                pf.guard, pf.cap, pf.loss, pf.best};
            pose_fin(s_tot, pf.cam_q, pf.qs, pf.dq, pf.dt, adam);
        }
        return;
    }
    if (out.dmeans2D) {
        out.dmeans2D[3 * i] = g2[0];
        out.dmeans2D[3 * i + 1] = g2[1];
        out.dmeans2D[3 * i + 2] = 0.f;
    }
    if (out.dcolors) {
        out.dcolors[3 * i] = g2[6];
        out.dcolors[3 * i + 1] = g2[7];
        out.dcolors[3 * i + 2] = g2[8];
    }
    if (out.dopacity) out.dopacity[i] = g2[5];
    if (out.dcolors2) {
        out.dcolors2[3 * i] = dcol2[0];
        out.dcolors2[3 * i + 1] = dcol2[1];
        out.dcolors2[3 * i + 2] = dcol2[2];
    }
#pragma unroll
    for (int k = 0; k < 3; k++) out.dmeans3D[3 * i + k] = dmean[k];
    if (out.dcov3D)
#pragma unroll
        for (int k = 0; k < 6; k++) out.dcov3D[6 * i + k] = dcov[k];
    if (out.dscales)
#pragma unroll
        for (int k = 0; k < 3; k++) out.dscales[3 * i + k] = dscale[k];
    if (out.drot)
#pragma unroll
        for (int k = 0; k < 4; k++) out.drot[4 * i + k] = drot[k];
    if (SHL && out.dsh && g.M > 0) {
        float* d = out.dsh + (size_t)3 * g.M * i;
#pragma unroll
        for (int k = 0; k < 48; k++)
            if (k < 3 * g.M) d[k] = (k < 3 * nsh) ? dsh[k] : 0.f;
        for (int k = 48; k < 3 * g.M; k++) d[k] = 0.f;
    }
}
template <bool POSE, bool SHL, bool CLK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 5)))
gauss_bwd_kernel(Camera cam, GaussIn g, GeomPtrs geo, const int* __restrict__ radii, const float* __restrict__ inst,
                 RecLayout rec, GradsOut out, BwdGuard guard, PoseFuse pf, unsigned long long* clk) {
    if constexpr (CLK) kclock_begin(clk);
    gauss_bwd_body<POSE, SHL>(cam, g, geo, radii, inst, rec, out, guard, pf);
    if constexpr (CLK) kclock_end(clk);
}

// workgroup partials, arrival counters, the 16 group sums
int pose_fuse_scratch_floats(int P) { return POSE_PARTS * ((P + 255) / 256) + ARRIVE_GROUPED_WORDS + 16 * POSE_PARTS; }

hipError_t launch_gauss_bwd(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii, const float* inst,
                            RecLayout rec, const GradsOut& out, BwdGuard guard, hipStream_t s, const PoseFuse* pose,
                            unsigned long long* clk) {
    if (g.P == 0) return hipSuccess;
    const bool shl = g.shs != nullptr;
    auto k = clk ? (pose ? (shl ? gauss_bwd_kernel<true, true, true> : gauss_bwd_kernel<true, false, true>)
                         : (shl ? gauss_bwd_kernel<false, true, true> : gauss_bwd_kernel<false, false, true>))
                 : (pose ? (shl ? gauss_bwd_kernel<true, true, false> : gauss_bwd_kernel<true, false, false>)
                         : (shl ? gauss_bwd_kernel<false, true, false> : gauss_bwd_kernel<false, false, false>));
    hipLaunchKernelGGL(k, dim3((g.P + 255) / 256), dim3(256), 0, s, cam, g, geo, radii, inst, rec, out, guard,
                       pose ? *pose : PoseFuse{}, clk);
    return hipGetLastError();
}

// ------------------------------------------------ backward_power == 2 --
// renderCUDAFused (backward.cu:850-1140) squares every per-pair output before summing it.  Every
// output of a pair is linear in the pair's base values b = (u, G dL/dalpha, dch dL/dpix) with a
// per-Gaussian coefficient row n (the chain, the conic and the NDC factor folded in), so
//   sum_p (n . b_p)^2 = n (sum_p b_p b_p^T) n^T:
// render_bwd forms the second moments sum_p b_p b_p^T (MOM layout, 16 or 34 sums per instance),
// and this kernel applies the quadratic forms once per Gaussian, in double.
hipError_t launch_render_bwd_moments(const Camera& cam, const uint2* ranges, const uint64_t* point_list, GeomPtrs geo,
                                     const float* final_T, const uint32_t* n_contrib, const float* dL_dpix, bool sh,
                                     float* inst, BwdGuard guard, hipStream_t s) {
    auto k = sh ? render_bwd_kernel<false, true, true, false, 3, 2> : render_bwd_kernel<false, true, true, false, 3, 1>;
    hipLaunchKernelGGL(k, dim3(cam.gx * cam.gy), dim3(TILE_PIX), 0, s, cam, ranges, point_list, geo.rr, geo.blocksums,
                       final_T, n_contrib, dL_dpix, nullptr, inst, guard, nullptr);
    return hipGetLastError();
}
int moments_record_floats(bool sh) { return sh ? 34 : 16; }

template <int MOM>
__global__ void __launch_bounds__(256)
gauss_bwd_mom_kernel(Camera cam, GaussIn g, GeomPtrs geo, const int* __restrict__ radii,
                     const float* __restrict__ inst, GradsOut out, BwdGuard guard) {
    constexpr int NV = MOM == 1 ? 16 : 34, RS = (NV + 1) & ~1;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.P) return;
    const int nsh = g.shs ? (cam.sh_degree + 1) * (cam.sh_degree + 1) : 0;
    float S[NV];
#pragma unroll
    for (int q = 0; q < NV; q++) S[q] = 0.f;
    const bool live = radii[i] > 0 && !guard.overflow();
    if (live) {  // fixed-order sum of the Gaussian's instance records (deterministic)
        const uint32_t off = geo.offsets[i], cnt = geo.tiles[i];
        const uint32_t tl = reinterpret_cast<const uint32_t*>(geo.bin)[4 * (size_t)i + 3];  // (Camera::cull)
        for (uint32_t e = 0; e < cnt; e++) {
            if (!tile_live(tl, e)) continue;
            const float2* r = reinterpret_cast<const float2*>(inst + (size_t)RS * (off + e));
            float2 v[RS / 2];
#pragma unroll
            for (int m = 0; m < RS / 2; m++) v[m] = r[m];
#pragma unroll
            for (int m = 0; m < NV / 2; m++) {
                S[2 * m] += v[m].x;
                S[2 * m + 1] += v[m].y;
            }
            if (NV % 2) S[NV - 1] += v[NV / 2].x;
        }
    }
    float Sm[9][9];
    mom_matrix<MOM>(S, Sm, std::make_integer_sequence<int, 81>{});
    float o_m2[2] = {0.f, 0.f}, o_mean[3] = {0.f, 0.f, 0.f}, o_cov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f},
          o_scale[3] = {0.f, 0.f, 0.f}, o_rot[4] = {0.f, 0.f, 0.f, 0.f}, ysq[16];
#pragma unroll
    for (int k = 0; k < 16; k++) ysq[k] = 0.f;
    unsigned clamped = 0u;
    // sum_ab n_a n_b Sm[a][b] over the geometric terms a, b in [A0, 5) and, with nw, the masked colours
    // (double: the terms of a quadratic form may cancel)
    auto qform = [&](const float (&n)[5], const float* nw, int A0) -> float {
        double acc = 0.0;
#pragma unroll
        for (int a = 0; a < 5; a++)
#pragma unroll
            for (int c = 0; c < 5; c++)
                if (a >= A0 && c >= A0) acc += (double)n[a] * (double)n[c] * (double)Sm[a][c];
        if (MOM == 2 && nw) {
#pragma unroll
            for (int a = 0; a < 5; a++)
#pragma unroll
                for (int c = 0; c < 3; c++) acc += 2.0 * (double)n[a] * (double)nw[c] * (double)Sm[a][6 + c];
#pragma unroll
            for (int c = 0; c < 3; c++)
#pragma unroll
                for (int e = 0; e < 3; e++) acc += (double)nw[c] * (double)nw[e] * (double)Sm[6 + c][6 + e];
        }
        return (float)acc;
    };
    if (live) {
        const GaussGeom gg = load_geom(g, i);
        float ca, cb, cc, c3[6];
        Proj pj;  // (with c3: reused by the unit chain evaluations below)
        gaussian_conic(cam, g, gg, i, ca, cb, cc, &pj, c3);
        const float ddx = (float)(0.5 * cam.W), ddy = (float)(0.5 * cam.H);  // backward.cu:935-936
        // chain input g2 = Lm u: dmean2D (NDC units) from (hx, hy), dconic = -u_conic / 2 (backward.cu:1020-1038)
        const float L0[2] = {-ca * ddx, -cb * ddx}, L1[2] = {-cb * ddy, -cc * ddy};
        {
            const float n0[5] = {L0[0], L0[1], 0.f, 0.f, 0.f}, n1[5] = {L1[0], L1[1], 0.f, 0.f, 0.f};
            o_m2[0] = qform(n0, nullptr, 0);
            o_m2[1] = qform(n1, nullptr, 0);
        }
        // coefficient rows n = (chain column) Lm, accumulated one unit chain input at a time
        float nm[3][5], nc[6][5], ns[3][5], nr[4][5], nw[3][3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
#pragma unroll
            for (int b = 0; b < 5; b++) nm[r][b] = 0.f;
#pragma unroll
            for (int c = 0; c < 3; c++) nw[r][c] = 0.f;
        }
#pragma unroll 1
        for (int kk = 0; kk < (MOM == 2 ? 8 : 5); kk++) {
            const int in = kk < 5 ? kk : kk + 1;
            float g2[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            g2[in] = 1.f;
            float dmean[3], dcov[6], dscale[3], drot[4], dsh[48];
            gauss_chain(cam, g, gg, i, g2, 0u, dmean, dcov, dscale, drot, dsh, nsh, true, &pj, c3);
            // (selects with constant indices: no dynamic register-array indexing)
#pragma unroll
            for (int b = 0; b < 5; b++) {
                const float lk = kk == 0 ? (b == 0 ? L0[0] : (b == 1 ? L0[1] : 0.f))
                                         : kk == 1 ? (b == 0 ? L1[0] : (b == 1 ? L1[1] : 0.f))
                                                   : (kk == b ? -0.5f : 0.f);
#pragma unroll
                for (int r = 0; r < 3; r++) nm[r][b] = __builtin_fmaf(dmean[r], lk, nm[r][b]);
                if (b >= 2) {  // cov3D / scale / rotation depend on the conic terms only
#pragma unroll
                    for (int r = 0; r < 6; r++) nc[r][b] = kk == b ? -0.5f * dcov[r] : (kk < 2 ? 0.f : nc[r][b]);
#pragma unroll
                    for (int r = 0; r < 3; r++) ns[r][b] = kk == b ? -0.5f * dscale[r] : (kk < 2 ? 0.f : ns[r][b]);
#pragma unroll
                    for (int r = 0; r < 4; r++) nr[r][b] = kk == b ? -0.5f * drot[r] : (kk < 2 ? 0.f : nr[r][b]);
                }
            }
            if (MOM == 2 && kk >= 5) {
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int r = 0; r < 3; r++) nw[r][c] = (kk - 5 == c) ? dmean[r] : nw[r][c];  // view-direction term
                if (kk == 5)
#pragma unroll
                    for (int k = 0; k < 16; k++) ysq[k] = k < nsh ? dsh[3 * k] * dsh[3 * k] : 0.f;
            }
        }
        clamped = g.shs ? geo.clamp[i] : 0u;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            float w3[3];
#pragma unroll
            for (int c = 0; c < 3; c++) w3[c] = ((clamped >> c) & 1u) ? 0.f : nw[r][c];
            o_mean[r] = qform(nm[r], w3, 0);
        }
#pragma unroll
        for (int r = 0; r < 6; r++) o_cov[r] = qform(nc[r], nullptr, 2);
        if (g.scales) {  // the reference forms no scale / rotation gradient from a precomputed cov3D
#pragma unroll
            for (int r = 0; r < 3; r++) o_scale[r] = qform(ns[r], nullptr, 2);
#pragma unroll
            for (int r = 0; r < 4; r++) o_rot[r] = qform(nr[r], nullptr, 2);
        }
    }
    if (out.dmeans2D) {
        out.dmeans2D[3 * i] = o_m2[0];
        out.dmeans2D[3 * i + 1] = o_m2[1];
        out.dmeans2D[3 * i + 2] = 0.f;
    }
    if (out.dcolors)
#pragma unroll
        for (int c = 0; c < 3; c++) out.dcolors[3 * i + c] = Sm[6 + c][6 + c];
    if (out.dopacity) out.dopacity[i] = Sm[5][5];
#pragma unroll
    for (int r = 0; r < 3; r++) out.dmeans3D[3 * i + r] = o_mean[r];
    if (out.dcov3D)
#pragma unroll
        for (int r = 0; r < 6; r++) out.dcov3D[6 * i + r] = o_cov[r];
    if (out.dscales)
#pragma unroll
        for (int r = 0; r < 3; r++) out.dscales[3 * i + r] = o_scale[r];
    if (out.drot)
#pragma unroll
        for (int r = 0; r < 4; r++) out.drot[4 * i + r] = o_rot[r];
    if (out.dsh && g.M > 0) {  // dsh[k][c] = Y_k dRGB_c per pair: Y_k^2 sum (dRGB_c)^2, 0 where the colour clamped
        float* d = out.dsh + (size_t)3 * g.M * i;
#pragma unroll
        for (int k = 0; k < 16; k++)
#pragma unroll
            for (int c = 0; c < 3; c++)
                if (k < g.M) d[3 * k + c] = !((clamped >> c) & 1u) ? ysq[k] * Sm[6 + c][6 + c] : 0.f;
        for (int k = 16; k < g.M; k++)
            for (int c = 0; c < 3; c++) d[3 * k + c] = 0.f;
    }
}

hipError_t launch_gauss_bwd_moments(const Camera& cam, const GaussIn& g, GeomPtrs geo, const int* radii,
                                    const float* inst, const GradsOut& out, BwdGuard guard, hipStream_t s) {
    if (g.P == 0) return hipSuccess;
    auto k = g.shs ? gauss_bwd_mom_kernel<2> : gauss_bwd_mom_kernel<1>;
    hipLaunchKernelGGL(k, dim3((g.P + 255) / 256), dim3(256), 0, s, cam, g, geo, radii, inst, out, guard);
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

#if GSR_STEPSTAT
extern "C" int gsr_diag_stepstat_bwd(unsigned long long* host) {  // copies and clears the counters
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stepstat), sizeof(g_stepstat), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stepstat), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
#endif
#if GSR_PHASE
extern "C" int gsr_diag_phase_bwd(unsigned long long* host) {  // copies and clears the phase cycles
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), sizeof(g_phase), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
#endif
#if GSR_WGTIME
extern "C" int gsr_diag_wgtime_bwd(unsigned long long* host, int n) {
    const size_t bytes = sizeof(unsigned long long) * 4 * (size_t)(n < GSR_WGTIME_MAX ? n : GSR_WGTIME_MAX);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wgtime), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace gsr
