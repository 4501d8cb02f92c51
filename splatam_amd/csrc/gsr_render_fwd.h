// gsr_render_fwd.h -- the tile forward of render_fwd_kernel as a device function (fwd_tile), with the
// per-tile sort it starts with: shared by render_fwd_kernel (gsr_forward.hip) and the tracking kernel
// that runs a tile's forward and backward in one workgroup (render_track_kernel, gsr_backward.hip).
#pragma once
#include "gsr_common.h"
#include "gsr_diag.h"

namespace gsr {

// Per-tile sort of the bucketed (depth bits << 32 | id) keys, done by render_fwd
// in its prologue (one workgroup per tile; no separate launch, no key round
// trip).  Keys are unique inside a tile, so the order is a total order and
// equals the reference's stable (tile, depth) radix order.
constexpr int TILE_SORT_THREADS = 256;
constexpr uint32_t TILE_SORT_REGS = 1024;  // longest list sorted in registers (256 threads x 4)

// Bitonic network over n = 256 * E keys (E per thread, blocked: thread t holds
// indices [t*E, t*E+E)).  Element i pairs with i ^ j, ascending iff (i & k) == 0.
// Partner in the same thread (j < E): register compare-exchange; in the same
// wave (j < 64 E): lane xor j/E, same slot; otherwise through LDS (3 of the 55
// stages for n = 1024).  The network is unrolled at compile time (template
// recursion over the stages), so every lane exchange is a fixed VALU permute:
// DPP quad_perm (xor 1, 2), DPP row shifts (xor 4), DPP row_ror (xor 8) and the
// gfx950 permlane16/32 swaps (xor 16, 32) -- no ds_bpermute, no loop control
// (the runtime-loop ds_bpermute version spent most of its time in SALU/branch
// overhead and LDS-permute latency: 32 us on the config-3 buckets,
// tools/micro/sort_bench.hip).  Lane mappings checked by tools/micro/lane_xor.hip.
#ifndef GSR_SORT_SWIZZLE
#define GSR_SORT_SWIZZLE 0  // lane exchanges of distance <= 16 by ds_swizzle (LDS pipe) instead of DPP / permlane (VALU):
                            // 779 static VALU fewer, bitwise the same order, the fused kernel unchanged (r8s_ab_sort_swizzle)
#endif
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x) {
    static_assert(M == 1 || M == 2 || M == 4 || M == 8 || M == 16 || M == 32, "lane xor distance");
    if constexpr (GSR_SORT_SWIZZLE && M <= 16) {
        // bit-mode swizzle inside each 32-lane half: lane' = (lane & 0x1F) ^ M
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (M << 10) | 0x1F);
    } else if constexpr (M == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (M == 4) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x104, 0xF, 0xF, false);  // row_shl:4 (l+4)
        const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xF, 0xF, false);  // row_shr:4 (l-4)
        return (__lane_id() & 4) ? dn : up;
    } else if constexpr (M == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (M == 16) {
        const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (__lane_id() & 16) ? p[0] : p[1];
    } else {
        const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (__lane_id() & 32) ? p[0] : p[1];
    }
}
template <int M>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v) {
    return ((uint64_t)lane_xor<M>((uint32_t)(v >> 32)) << 32) | lane_xor<M>((uint32_t)v);
}

template <int E, int J>
__device__ __forceinline__ void bitonic_reg_stage(uint64_t (&v)[E], uint32_t base, uint32_t k) {
#pragma unroll
    for (int e = 0; e < E; e++) {
        if (e & J) continue;
        const bool up = ((base + (uint32_t)e) & k) == 0;
        const uint64_t a = v[e], b = v[e + J];
        const bool sw = (b < a) == up;  // one 64-bit compare, then two selects per word
        v[e] = sw ? b : a;
        v[e + J] = sw ? a : b;
    }
}

// keep the smaller of (mine, partner) iff keep_min: one 64-bit compare + 2 selects
__device__ __forceinline__ uint64_t bitonic_pick(uint64_t v, uint64_t o, bool keep_min) {
    return ((o < v) == keep_min) ? o : v;
}

// stage (k = 2^LK, j = 2^LJ) of the network, then the rest of the network
template <int E, int LK, int LJ>
__device__ __forceinline__ void bitonic_net(uint64_t (&v)[E], uint32_t base, uint64_t* sk) {
    constexpr uint32_t k = 1u << LK, j = 1u << LJ;
    if constexpr (j >= (uint32_t)E) {
        // j >= E, so k > j covers only thread-index bits: direction and side are the
        // same for all E slots of a thread
        const bool up = (base & k) == 0, keep_min = ((base & j) == 0) == up;
        if constexpr (j >= 64u * E) {  // partner in another wave
#pragma unroll
            for (int e = 0; e < E; e++) sk[base + e] = v[e];
            __syncthreads();
#pragma unroll
            for (int e = 0; e < E; e++) v[e] = bitonic_pick(v[e], sk[(base + e) ^ j], keep_min);
            __syncthreads();
        } else {  // partner lane ^ j/E, same slot
#pragma unroll
            for (int e = 0; e < E; e++) v[e] = bitonic_pick(v[e], lane_xor64<(int)(j / E)>(v[e]), keep_min);
        }
    } else {  // partner in this thread
        bitonic_reg_stage<E, (int)j>(v, base, k);
    }
    constexpr int LOGN = E == 1 ? 8 : E == 2 ? 9 : 10;
    if constexpr (LJ > 0) bitonic_net<E, LK, LJ - 1>(v, base, sk);
    else if constexpr (LK < LOGN) bitonic_net<E, LK + 1, LK>(v, base, sk);
}

template <int E, typename Emit>
__device__ void tile_sort_regs(const uint64_t* __restrict__ src, uint32_t cnt, Emit emit, uint64_t* sk) {
    static_assert(E == 1 || E == 2 || E == 4, "256 x E keys");
    const uint32_t base = threadIdx.x * E;
    uint64_t v[E];
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = base + e < cnt ? src[base + e] : ~0ull;
    bitonic_net<E, 1, 0>(v, base, sk);
#pragma unroll
    for (int e = 0; e < E; e++)  // (a padding key can only land here through a network bug: emit id 0, never
        if (base + e < cnt) emit(base + e, v[e] == ~0ull ? 0u : (uint32_t)v[e]);  // an out-of-range id)
}

// Sorts one tile's bucket src[0, cnt) (cnt <= TILE_SORT_CAP) into dst as Gaussian
// ids (render_fwd adds the block mask in the high half when it stages an entry).
// Every thread of the workgroup calls it (cnt is workgroup-uniform); sk: LDS for
// TILE_SORT_REGS keys (the network's cross-wave stages, the rank searches).
//   cnt <= 512:  one register network of 256 or 512 keys, ids emitted directly.
//   otherwise:   the bucket is cut into chunks of TILE_SORT_REGS keys, each sorted by
//                the 256 x 4 register network; a single chunk is emitted directly,
//                several are written back in place (the keys are scratch once sorted)
//                and every key's final position is its index in its own chunk plus,
//                for every other chunk (staged in LDS), the number of that chunk's
//                keys below it -- exact, as the keys are unique in a tile.
// The result equals a stable (tile, depth) radix order (ids break depth ties).
#ifndef GSR_FWD_PAIR25
#define GSR_FWD_PAIR25 1  // dual forward walk: channels 2 and 5 blended by one v_pk_fma (0: two v_fmac)
#endif
#ifndef GSR_FWD_DONE_EXIT
#define GSR_FWD_DONE_EXIT 1  // forward walk: done lanes exit the loop (0: a wave-uniform ballot test per step)
#endif
#ifndef GSR_FWD_ABLATE
#define GSR_FWD_ABLATE 0  // timing ablations (tools/gpu_round.sh ab=; results invalid except 5, 6): 1 no per-tile
                          // sort, 2 no walk, 4 no tracking-loss epilogue, 5 bounding-box block masks, 6 no block
                          // masks, 7 masks of an earlier launch read back, 8 no image stores.  0 in every real build
#endif
#if GSR_FWD_ABLATE == 7
static __device__ uint16_t g_fab_mask[1u << 23];
#endif
__device__ __forceinline__ void tile_sort_bucket(uint64_t* __restrict__ src, uint32_t cnt,
                                                 PointEntry* __restrict__ dst, uint64_t* sk) {
    auto emit = [&](uint32_t i, uint32_t gi) { dst[i] = (PointEntry)gi; };
    if (GSR_FWD_ABLATE == 1) {  // timing only: the bucket copied unsorted (wrong order)
        for (uint32_t i = threadIdx.x; i < cnt; i += TILE_SORT_THREADS) emit(i, (uint32_t)src[i]);
        return;
    }
    if (cnt <= 1) {
        if (cnt == 1 && threadIdx.x == 0) emit(0, (uint32_t)src[0]);
        return;
    }
    if (cnt <= 256) {
        tile_sort_regs<1>(src, cnt, emit, sk);
        return;
    }
    if (cnt <= 512) {
        tile_sort_regs<2>(src, cnt, emit, sk);
        return;
    }
    const uint32_t nch = (cnt + TILE_SORT_REGS - 1) / TILE_SORT_REGS;
    const uint32_t base = threadIdx.x * 4;
    for (uint32_t c = 0; c < nch; c++) {  // one network instance for every chunk
        const uint32_t c0 = c * TILE_SORT_REGS, len = min(TILE_SORT_REGS, cnt - c0);
        uint64_t v[4];
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = base + e < len ? src[c0 + base + e] : ~0ull;
        bitonic_net<4, 1, 0>(v, base, sk);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            if (base + e >= len) continue;
            if (nch == 1) emit(base + e, v[e] == ~0ull ? 0u : (uint32_t)v[e]);  // (never an out-of-range id)
            else src[c0 + base + e] = v[e];
        }
    }
    if (nch == 1) return;
    __syncthreads();  // the sorted chunks (global) are visible to the workgroup
    for (uint32_t c = 0; c < nch; c++) {
        const uint32_t c0 = c * TILE_SORT_REGS, len = min(TILE_SORT_REGS, cnt - c0);
        uint64_t v[4];
        uint32_t pos[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            v[e] = base + e < len ? src[c0 + base + e] : ~0ull;
            pos[e] = base + e;
        }
        for (uint32_t c2 = 0; c2 < nch; c2++) {
            if (c2 == c) continue;
            const uint32_t d0 = c2 * TILE_SORT_REGS, dlen = min(TILE_SORT_REGS, cnt - d0);
            __syncthreads();  // sk is free
            for (uint32_t i = threadIdx.x; i < dlen; i += TILE_SORT_THREADS) sk[i] = src[d0 + i];
            __syncthreads();
#pragma unroll
            for (int e = 0; e < 4; e++) {  // keys of chunk c2 below v[e]: branch-free lower bound
                uint32_t lo = 0;
#pragma unroll
                for (uint32_t st = TILE_SORT_REGS; st > 0; st >>= 1)
                    if (lo + st <= dlen && sk[lo + st - 1] < v[e]) lo += st;
                pos[e] += lo;
            }
        }
#pragma unroll
        for (int e = 0; e < 4; e++)
            if (base + e < len) emit(pos[e], (uint32_t)v[e]);
    }
    __syncthreads();  // sk (aliased by the caller) is free again
}

// One tile's forward LDS (carved from one byte array: render_track_kernel aliases it with the backward's)
template <bool DUAL>
struct FwdShape {
    static constexpr int LS = RENDER_BATCH + 4;  // row-list stride (u16)
    static constexpr size_t o_ab = 0, o_c = o_ab + 2 * 16 * (RENDER_BATCH + 1), o_d = o_c + 16 * (RENDER_BATCH + 1);
    static constexpr size_t o_list = o_d + 16 * (DUAL ? RENDER_BATCH + 1 : 1);
    static constexpr size_t o_mask = o_list + 2 * 16 * LS;
    static constexpr size_t bytes = o_mask + 2 * RENDER_BATCH;
    static_assert(2 * 16 * (RENDER_BATCH + 1) >= TILE_SORT_REGS * sizeof(uint64_t) && TILE_SORT_THREADS == TILE_PIX,
                  "tile sort (256 x 4 keys) LDS aliases s_a / s_b");
};

// One thread's pixel after the tile forward
struct FwdPix {
    float T, C2, C5, D;
    v2f C01, C34;
    uint32_t last16;  // 16 x n_contrib
};

// The tile forward (sort, staging, row lists, front-to-back walk) up to the epilogue
template <bool DUAL>
__device__ __forceinline__ FwdPix fwd_tile(const Camera& cam, int tile, const uint2* __restrict__ ranges,
                                           PointEntry* __restrict__ point_list, uint64_t* __restrict__ keys,
                                           const float4* __restrict__ rr, const SpecGuard& guard, char* smem,
                                           RenderDiag& dg) {
    using L = FwdShape<DUAL>;
    constexpr int LS = L::LS;
    // entry RENDER_BATCH is a dummy (opacity 0, never blends) that pads the row lists
    // s_a and s_b share one array: before the first batch it is the tile sort's LDS
    float4* const s_ab = reinterpret_cast<float4*>(smem + L::o_ab);
    float4* const s_a = s_ab;
    float4* const s_b = s_ab + RENDER_BATCH + 1;
    float4* const s_c = reinterpret_cast<float4*>(smem + L::o_c);
    [[maybe_unused]] float4* const s_d = reinterpret_cast<float4*>(smem + L::o_d);
    uint16_t* const s_mask = reinterpret_cast<uint16_t*>(smem + L::o_mask);
    uint16_t* const s_list = reinterpret_cast<uint16_t*>(smem + L::o_list);
    const int tid = threadIdx.x, w = tid >> 6, row = (tid >> 4) & 3;
    const int tx = tile % cam.gx, ty = tile / cam.gx;
    const int px = tx * TILE_X + tile_px(tid);
    const int py = ty * TILE_Y + tile_py(tid);
    const float x0 = (float)(tx * TILE_X), y0 = (float)(ty * TILE_Y);
    const bool inside = px < cam.W && py < cam.H;
    const v2f pix = v2f{(float)px, (float)py};
    const uint2 range = ranges[tile];
    bool done = !inside;
    float T = 1.f, C2 = 0.f, D = 15.0f;  // forward.cu:308 median-depth default
    float C5 = 0.f;
    v2f C01 = v2f{0.f, 0.f}, C34 = v2f{0.f, 0.f};  // channel pairs: one v_pk_fma_f32 per pair and Gaussian
    uint32_t last16 = 0;  // 16 x n_contrib
    float4 pa = make_float4(0.f, 0.f, 0.f, 0.f), pb = pa, pc = pa, pd = pa;
    uint32_t pg = 0, pgn = 0;  // the staged entry's Gaussian id, the id of the entry a batch later
    if (keys != nullptr) {
        // the tile's bucket is sorted here; the sorted ids land in point_list and are read
        // back below by this same workgroup (guard: every list is <= TILE_SORT_CAP)
        tile_sort_bucket(keys + range.x, range.y - range.x, point_list + range.x,
                         reinterpret_cast<uint64_t*>(s_ab));
        __syncthreads();
        if constexpr (kDupPhase == 1) {  // (VALU census only: the same sort again, same result)
            tile_sort_bucket(keys + range.x, range.y - range.x, point_list + range.x,
                             reinterpret_cast<uint64_t*>(s_ab));
            __syncthreads();
        }
    }
    if (tid == 0) {
        s_a[RENDER_BATCH] = pa;
        s_b[RENDER_BATCH] = pa;
        s_c[RENDER_BATCH] = pa;
        if (DUAL) s_d[RENDER_BATCH] = pa;
    }
    // Batch staging pipelined two deep: the sorted id of an entry is loaded a batch before its
    // render record, and the record's block mask is formed at staging, so no dependent load is
    // waited on while a batch is rasterised.
    auto fetch_id = [&](uint32_t s0) {
        if (s0 + tid < range.y) pgn = pe_id(point_list[s0 + tid]);
    };
    auto fetch_rec = [&](uint32_t s0) {
        if (s0 + tid < range.y) {
            pg = pgn;
            const RenderRec r = load_rr(rr, pg);
            pa = r.q0; pb = r.q1; pc = r.q2;
            if (DUAL) pd = r.q3;
        }
    };
    fetch_id(range.x);
    fetch_rec(range.x);
    fetch_id(range.x + RENDER_BATCH);
    const uint32_t mean4 = sched_mean4(cam, guard.counters);
    const bool multi_round = sched_multi_round(cam);
    dg.phase(0);
    for (uint32_t start = range.x; start < range.y; start += RENDER_BATCH) {
        prio_by_remaining((int)(range.y - start), mean4, multi_round);
        if (__syncthreads_and(done)) break;  // forward.cu:314-316
        const int cnt = (int)min((uint32_t)RENDER_BATCH, range.y - start);
        PointEntry ent = 0;
        if (tid < cnt) {
            float xs = x0, ys = y0;
            asm volatile("" : "+v"(xs), "+v"(ys));  // block bounds formed here, not hoisted (VGPRs)
            // (GSR_FWD_ABLATE 5: the bounding-box mask; 6: every block -- timing ablations)
            uint32_t pm = GSR_FWD_ABLATE == 5 ? block_mask(pa, pb, xs, ys)
                        : GSR_FWD_ABLATE == 6 ? 0xFFFFu : 0u;
#if GSR_FWD_ABLATE == 7
            // timing only: the exact masks of an earlier launch read back by sorted position (the bound of
            // forming them outside this kernel; valid only while the same frame is rendered again)
            pm = g_fab_mask[start + tid];
            if (pm == 0u) {
                pm = block_mask_exact(pa, pb, xs, ys);
                g_fab_mask[start + tid] = (uint16_t)pm;
            }
#else
            if (GSR_FWD_ABLATE != 5 && GSR_FWD_ABLATE != 6) pm = block_mask_exact(pa, pb, xs, ys);
#endif
            s_a[tid] = pa;
            s_b[tid] = pb;
            // (DUAL: the second set's third channel rides in s_c.w -- the walk blends channels (0, 1), (2, 5)
            // and (3, 4) as three pairs -- and the rect half it replaces is not read after staging)
            s_c[tid] = (DUAL && GSR_FWD_PAIR25) ? make_float4(pc.x, pc.y, pc.z, pd.z) : pc;
            if (DUAL) s_d[tid] = pd;
            s_mask[tid] = (uint16_t)pm;
            ent = ((PointEntry)pm << 32) | pg;  // the mask, for render_bwd (stored below)
        }
        __syncthreads();
        dg.phase(1);
        fetch_rec(start + RENDER_BATCH);      // records of the next batch (ids loaded a batch ago)
        fetch_id(start + 2 * RENDER_BATCH);   // ids of the batch after it
        // the entry's store after those loads: a load issued behind a store waits for the store too
        // (vmcnt counts both), so the other order put this store's latency in front of every gather
        if (tid < cnt) point_list[start + tid] = ent;
        const int jmin0[4] = {0, 0, 0, 0};
        // list entries: LDS byte offsets 16 j of the staged records (the walk loads them with ds_read_u16)
        static_assert(16 * RENDER_BATCH < 65536, "16-bit byte offsets");
        int n = build_row_lists(s_mask, cnt, w, jmin0, s_list + 4 * w * LS, LS, (uint16_t)(16 * RENDER_BATCH), 16u);
        if constexpr (kDupPhase == 2) {  // (VALU census only: the same lists again)
            asm volatile("" ::: "memory");
            n = build_row_lists(s_mask, cnt, w, jmin0, s_list + 4 * w * LS, LS, (uint16_t)(16 * RENDER_BATCH), 16u);
        }
        const uint16_t* my_list = s_list + (4 * w + row) * LS;
        const uint32_t pos16 = 16u * (start - range.x) + 16u;  // 16 (position of entry 0 + 1)
        dg.phase(2);
        for (int i = 0; i < (GSR_FWD_ABLATE == 2 ? 0 : n); i += 4) {
            // a lane whose pixel is done leaves the walk (the wave's loop ends when every lane has: exec-mask
            // bookkeeping on the scalar unit -- a __ballot(!done) test cost 2 VALU per step)
            if (GSR_FWD_DONE_EXIT ? done : __ballot(!done) == 0ull) break;
            int jb[4];  // byte offsets 16 j, one ds_read_u16 each (no unpacking on the VALU; volatile keeps
#pragma unroll  // the four adjacent u16 loads from being merged into one b64 load + 4 VALU unpacks)
            for (int k = 0; k < 4; k++)
                jb[k] = (int)((const volatile __attribute__((address_space(3))) uint16_t*)my_list)[i + k];
            auto rec = [&](const float4* arr, int k) {
                return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(arr) + jb[k]);
            };
            float alpha[4], depth[4];
            bool ok[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float4 a = rec(s_a, k), b = rec(s_b, k);
                const float p2 = eval_p2(a, b, pix_delta(a, pix));           // log2(e) * power
                // (no clamp of p2: a pair with p2 > 0 -- exp2 up to inf, alpha then 0.99 -- is excluded by ok[k],
                // as forward.cu:342 skips it; a NaN p2 fails p2 <= 0 too)
                alpha[k] = fminf(0.99f, b.y * __builtin_amdgcn_exp2f(p2));
                depth[k] = b.z;
                ok[k] = p2 <= 0.0f && alpha[k] >= 1.0f / 255.0f;  // the pad entry has alpha 0
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                // (no per-entry wave-uniform skip when no lane blends: nearly every entry has a blending
                // lane in one of the four rows, and the test cost a branch + 2 VALU per entry: 63.6 ->
                // 61.8 us without it at config 3)
                const bool okk = ok[k] && !done;
                const float test_T = T * (1.f - alpha[k]);
                const bool term = okk && test_T < 0.0001f;
                done = done || term;
                const bool blend = okk && !term;
                const float4 c = rec(s_c, k);
                float4 c2;
                if (DUAL) c2 = rec(s_d, k);
                if (blend) {
                    const float wgt = alpha[k] * T;
                    C01 = __builtin_elementwise_fma(v2f{c.x, c.y}, v2f{wgt, wgt}, C01);
                    if (DUAL && GSR_FWD_PAIR25) {  // the same fused products per channel, two per instruction
                        const v2f c25 = __builtin_elementwise_fma(v2f{c.z, c.w}, v2f{wgt, wgt}, v2f{C2, C5});
                        C2 = c25.x;
                        C5 = c25.y;
                        C34 = __builtin_elementwise_fma(v2f{c2.x, c2.y}, v2f{wgt, wgt}, C34);
                    } else {
                        C2 += c.z * wgt;
                        if (DUAL) {
                            C34 = __builtin_elementwise_fma(v2f{c2.x, c2.y}, v2f{wgt, wgt}, C34);
                            C5 += c2.z * wgt;
                        }
                    }
                    if (T > 0.5f && test_T < 0.5f) D = depth[k];  // median depth (forward.cu:368-372)
                    T = test_T;
                    last16 = pos16 + (uint32_t)jb[k];              // 16 x entries visited up to the last blend
                }
            }
        }
        dg.phase(3);
        __syncthreads();
        dg.phase(4);
        dg.batch();
    }
    return FwdPix{T, C2, C5, D, C01, C34, last16};
}


#ifndef GSR_NT_STORES
#define GSR_NT_STORES 0  // render kernels' record / image stores as non-temporal (streaming) stores
#endif
#ifndef GSR_L1_CH
#define GSR_L1_CH 8  // tracking-loss epilogue: partials in flight per round trip of the last workgroup
#endif

// The tile forward's epilogue: per-block n_contrib maxima (cam.rowmax), the images, and with L1 the
// tracking loss -- its per-pixel gradients (dL/dim_0..2, dL/ddepth) returned in grad and stored into
// l1.dL_dim / l1.dL_dds when STORE_GRADS, the workgroup's loss partials published and summed by the
// last workgroup.
// The tracking loss from the workgroups' published partials: the last workgroup to arrive adds them in
// tile order and writes l1.loss (every thread of every workgroup calls it, after its partial store)
__device__ __forceinline__ void l1_finish(const TrackL1& l1) {
    if constexpr (kAblate == 6) return;  // timing ablation: no loss arrival / sum (loss invalid)
    __shared__ float s_fin[16];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, row4 = lane >> 4;
    const int nb = gridDim.x * gridDim.y;
    if (last_block_arrive_grouped(reinterpret_cast<uint32_t*>(l1.part + 2 * nb))) {
        float v[4] = {0.f, 0.f, 0.f, 0.f}, r[1];
        {
            float v2[2] = {0.f, 0.f};
            gather_partials<2, GSR_L1_CH>(l1.part, 2, nb, tid, TILE_PIX, v2);
            v[0] = v2[0];
            v[1] = v2[1];
        }
        wave_reduce_n<4>(v, r);
        if ((lane & 15) == 0) s_fin[w * 4 + row4] = r[0];
        __syncthreads();
        if (tid == 0) {
            const float s0 = (s_fin[0] + s_fin[4]) + (s_fin[8] + s_fin[12]);
            const float s1 = (s_fin[1] + s_fin[5]) + (s_fin[9] + s_fin[13]);
            l1.loss[0] = l1.w_im * s0 + l1.w_depth * s1;
        }
    }
}

// L1_FINISH: the arrival / last-workgroup sum right here (render_fwd_kernel); false: the caller calls
// l1_finish later (render_track_kernel, after the tile's backward: no atomic round trip between its phases)
template <bool DUAL, bool L1, bool STORE_GRADS, bool L1_FINISH = true>
__device__ __forceinline__ void fwd_epilogue(const Camera& cam, int tile, const FwdPix& f, float* __restrict__ final_T,
                                             uint32_t* __restrict__ n_contrib, float* __restrict__ out_color,
                                             float* __restrict__ out_color2, float* __restrict__ out_depth,
                                             const TrackL1& l1, float (&grad)[4]) {
    const int tid = threadIdx.x, w = tid >> 6, row = (tid >> 4) & 3;
    const int tx = tile % cam.gx, ty = tile / cam.gx;
    const int px = tx * TILE_X + tile_px(tid);
    const int py = ty * TILE_Y + tile_py(tid);
    const bool inside = px < cam.W && py < cam.H;
    const float T = f.T, C2 = f.C2, C5 = f.C5, D = f.D;
    const float C0 = f.C01.x, C1 = f.C01.y, C3 = f.C34.x, C4 = f.C34.y;
    const uint32_t last16 = f.last16;
    (void)C3; (void)C4; (void)C5;
#pragma unroll
    for (int c = 0; c < 4; c++) grad[c] = 0.f;
    if (cam.rowmax) {  // per-block maximum of n_contrib for render_bwd (ImgLayout::rowmax)
        uint32_t rmax = last16 >> 4;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, o));
        if ((tid & 15) == 0) cam.rowmax[16 * tile + 4 * w + row] = rmax;
    }
    // the loss epilogue's inputs are loaded before the image stores: a load issued after a store
    // also waits for the store's completion (vmcnt counts both)
    float l1_seed = 0.f, l1_gd = 0.f, l1_gi[3] = {0.f, 0.f, 0.f};
    if constexpr (L1 && GSR_FWD_ABLATE != 4) {
        if (inside) {
            const int pid = py * cam.W + px;
            const int HW = cam.W * cam.H;
            l1_seed = l1.seed[0];
            l1_gd = l1.gt_depth[pid];
#pragma unroll
            for (int c = 0; c < 3; c++) l1_gi[c] = l1.gt_im[c * HW + pid];
        }
    }
    if (inside && final_T != nullptr && (GSR_FWD_ABLATE != 8 || T == 1.2345f)) {  // (ablation 8: no image stores)
        const int pid = py * cam.W + px;
        const int HW = cam.W * cam.H;
        auto st = [](float* p, float v) {
            if (GSR_NT_STORES) __builtin_nontemporal_store(v, p);
            else *p = v;
        };
        st(final_T + pid, T);
        if (GSR_NT_STORES) __builtin_nontemporal_store(last16 >> 4, n_contrib + pid);
        else n_contrib[pid] = last16 >> 4;
        st(out_color + pid, C0 + T * cam.bg[0]);
        st(out_color + HW + pid, C1 + T * cam.bg[1]);
        st(out_color + 2 * HW + pid, C2 + T * cam.bg[2]);
        st(out_depth + pid, D);
        if (DUAL) {
            st(out_color2 + pid, C3 + T * cam.bg[0]);
            st(out_color2 + HW + pid, C4 + T * cam.bg[1]);
            st(out_color2 + 2 * HW + pid, C5 + T * cam.bg[2]);
        }
    }
    if constexpr (L1 && GSR_FWD_ABLATE != 4) {
        // get_loss(tracking=True) on this pixel (gsr_glue.hip track_l1_kernel, same expressions on the
        // values just written): mask = gt_depth > 0 & !isnan(depth) & !isnan(depth_sq - depth^2) &
        // silhouette > thres; sums of |gt - x| over the mask; dL/dx = -sgn(gt - x) * w * dL/dloss
        __shared__ float s_red[4 * 4];
        __shared__ float s_tot[4];
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (inside) {
            const int pid = py * cam.W + px;
            const int HW = cam.W * cam.H;
            const float g = l1_seed;
            const float im[3] = {C0 + T * cam.bg[0], C1 + T * cam.bg[1], C2 + T * cam.bg[2]};
            const float d = C3 + T * cam.bg[0], sil = C4 + T * cam.bg[1], dsq = C5 + T * cam.bg[2];
            const float gd = l1_gd;
            const float unc = dsq - d * d;
            const bool m = gd > 0.f && !isnan(d) && !isnan(unc) && sil > l1.sil_thres;
            const float gi[3] = {l1_gi[0], l1_gi[1], l1_gi[2]};
            if (m) {
                v[0] = fabsf(gi[0] - im[0]) + fabsf(gi[1] - im[1]) + fabsf(gi[2] - im[2]);
                v[1] = fabsf(gd - d);
            }
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const float x = gi[c] - im[c];
                grad[c] = m ? (g * l1.w_im) * (x > 0.f ? -1.f : (x < 0.f ? 1.f : 0.f)) : 0.f;
            }
            const float xd = gd - d;
            grad[3] = m ? (g * l1.w_depth) * (xd > 0.f ? -1.f : (xd < 0.f ? 1.f : 0.f)) : 0.f;
            if (STORE_GRADS) {
#pragma unroll
                for (int c = 0; c < 3; c++) l1.dL_dim[c * HW + pid] = grad[c];
                l1.dL_dds[pid] = grad[3];
                l1.dL_dds[HW + pid] = 0.f;
                l1.dL_dds[2 * HW + pid] = 0.f;
            }
        }
        // fixed-order workgroup sums, published; the last workgroup adds them in tile order
        float r[1];
        wave_reduce_n<4>(v, r);
        const int lane = tid & 63, row4 = lane >> 4;
        if ((lane & 15) == 0) s_red[w * 4 + row4] = r[0];
        __syncthreads();
        if (tid < 4) s_tot[tid] = (s_red[tid] + s_red[4 + tid]) + (s_red[8 + tid] + s_red[12 + tid]);
        __syncthreads();
        if (tid < 2) st_agent(l1.part + 2 * tile + tid, s_tot[tid]);
        if (L1_FINISH) l1_finish(l1);
    }
}

}  // namespace gsr
