// gsr_diag.h -- diagnostics hooks of the render kernels, compiled out of every real build.
//
// The kernels call the hooks of one RenderDiag object at their phase boundaries; each hook is an empty
// inline function unless its diagnostics build switch is set (the build_variant libraries that
// tools/stepstat.py, tools/phase_bwd.py and tools/wgtime.py load through GSR_LIB):
//   GSR_STEPSTAT  render_bwd step statistics: [wave-steps, wave-steps with a contributing pair,
//                 contributing (lane, entry) pairs, pad (lane, entry) slots, batches x waves,
//                 listed (row, entry) items, listed items with no contributing pixel]
//   GSR_PHASE     per-wave s_memtime cycles per render_bwd phase: [0] prologue, [1] batch staging + barrier,
//                 [2] row / slot list build, [3] row walk, [4] barrier after the walk, [5] entry totals +
//                 record stores, [6] barrier after the totals, [7] batches x waves
//   GSR_WGTIME    per-workgroup [start, end, HW_ID, XCC_ID] of the render kernels (gsr_common.h)
// GSR_ABLATE / GSR_FWD_ABLATE (timing ablations, results invalid) are compile-time constants read through
// kAblate / kFwdAblate.
#pragma once
#include "gsr_common.h"

#ifndef GSR_STEPSTAT
#define GSR_STEPSTAT 0
#endif
#ifndef GSR_PHASE
#define GSR_PHASE 0
#endif
#ifndef GSR_ABLATE
#define GSR_ABLATE 0  // render_bwd / gauss_bwd timing ablations (1 no row reduction, 2 no entry totals, 3-5 pose tail,
                      // 6 no tracking-loss arrival / sum)
#endif

namespace gsr {

constexpr int kAblate = GSR_ABLATE;
#ifndef GSR_DUP_PHASE
#define GSR_DUP_PHASE 0  // VALU census by SQ counters (tools/gpu_round.sh sqab=): one render phase run twice (1 the
                         // tile sort, 2 the forward row lists, 3 the backward slot lists); results unchanged
#endif
constexpr int kDupPhase = GSR_DUP_PHASE;
GSR_WGTIME_TABLE  // (GSR_WGTIME builds: this translation unit's per-workgroup timeline table)

#if GSR_STEPSTAT
static __device__ unsigned long long g_stepstat[8];
#endif
#if GSR_PHASE
static __device__ unsigned long long g_phase[8];
#endif

struct RenderDiag {
#if GSR_PHASE
    unsigned long long t = 0, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
#if GSR_STEPSTAT
    unsigned long long steps = 0, csteps = 0, ok = 0, pads = 0, batches = 0, items = 0, dead = 0;
#endif
    __device__ __forceinline__ void begin() {
        GSR_WGTIME_MARK(false);
#if GSR_PHASE
        t = __builtin_amdgcn_s_memtime();
#endif
    }
    // the workgroup's tile (GSR_WGTIME: stored beside its timeline)
    __device__ __forceinline__ void tile(int t) {
#if GSR_WGTIME
        const unsigned b_ = blockIdx.y * gridDim.x + blockIdx.x;
        if (threadIdx.x == 0 && b_ < GSR_WGTIME_MAX)
            g_wgtime[b_][3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) | ((unsigned long long)t << 32);
#else
        (void)t;
#endif
    }
    // end of phase k (GSR_PHASE); k == 7 counts a batch
    __device__ __forceinline__ void phase(int k) {
#if GSR_PHASE
        const unsigned long long n = __builtin_amdgcn_s_memtime();
        acc[k] += n - t;
        t = n;
#else
        (void)k;
#endif
    }
    __device__ __forceinline__ void batch() {
#if GSR_PHASE
        acc[7]++;
#endif
#if GSR_STEPSTAT
        batches++;
#endif
    }
    // one walk step of four entries: pad[k] = the lane's entry k is the row list's pad, okk[k] = the pair
    // contributes
    __device__ __forceinline__ void step(const bool (&pad)[4], const bool (&okk)[4]) {
#if GSR_STEPSTAT
        steps++;
        bool any = false;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            pads += __popcll(__ballot(pad[k]));
            ok += __popcll(__ballot(okk[k]));
            any = any || okk[k];
            const uint64_t okb = __ballot(okk[k]), padb = __ballot(pad[k]);
#pragma unroll
            for (int r = 0; r < 4; r++) {  // (row, entry) items: listed, and listed with no contributing pixel
                const bool listed = ((padb >> (16 * r)) & 0xFFFFull) == 0ull;
                items += listed;
                dead += listed && ((okb >> (16 * r)) & 0xFFFFull) == 0ull;
            }
        }
        csteps += __ballot(any) != 0ull;
#else
        (void)pad;
        (void)okk;
#endif
    }
    __device__ __forceinline__ void end() {
#if GSR_PHASE
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < 8; k++) atomicAdd(&g_phase[k], acc[k]);
#endif
#if GSR_STEPSTAT
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&g_stepstat[0], steps);
            atomicAdd(&g_stepstat[1], csteps);
            atomicAdd(&g_stepstat[2], ok);
            atomicAdd(&g_stepstat[3], pads);
            atomicAdd(&g_stepstat[4], batches);
            atomicAdd(&g_stepstat[5], items);
            atomicAdd(&g_stepstat[6], dead);
        }
#endif
        GSR_WGTIME_MARK(true);
    }
};

}  // namespace gsr
