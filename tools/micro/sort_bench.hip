// Microbenchmark of the per-tile sort on config-3-shaped buckets (1200 tiles x ~564
// random (depth, id) keys), against an empty kernel with the same grid and LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#include "gsr_common.h"

namespace gsr {
hipError_t launch_tile_sort(int ntiles, const uint2* ranges, const uint64_t* keys, uint64_t* point_list,
                            SpecGuard guard, hipStream_t s);
}

__global__ void __launch_bounds__(256) empty_kernel(const uint2* r, uint64_t* out) {
    __shared__ uint64_t sk[4096];
    sk[threadIdx.x] = r[blockIdx.x].x;
    __syncthreads();
    if (threadIdx.x == 0 && sk[255] == 0xdeadbeef) out[0] = 1;
}

int main() {
    const int T = 1200;
    std::vector<uint2> ranges(T);
    std::vector<uint64_t> keys;
    srand(3);
    for (int t = 0; t < T; t++) {
        int c = 480 + rand() % 200;
        ranges[t] = make_uint2((uint32_t)keys.size(), (uint32_t)(keys.size() + c));
        for (int i = 0; i < c; i++) keys.push_back(((uint64_t)(0x3f000000u + rand() % 0x800000) << 32) | (uint64_t)(rand() % 300000));
    }
    uint2* dr; uint64_t *dk, *dp; uint32_t* dc;
    (void)hipMalloc(&dr, sizeof(uint2) * T);
    (void)hipMalloc(&dk, 8 * keys.size());
    (void)hipMalloc(&dp, 8 * keys.size());
    (void)hipMalloc(&dc, 16);
    (void)hipMemcpy(dr, ranges.data(), sizeof(uint2) * T, hipMemcpyHostToDevice);
    (void)hipMemcpy(dk, keys.data(), 8 * keys.size(), hipMemcpyHostToDevice);
    (void)hipMemset(dc, 0, 16);
    gsr::SpecGuard g{dc, 0xffffffffu, 0xffffffffu};
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    for (int variant = 0; variant < 2; variant++) {
        float best = 1e9;
        for (int rep = 0; rep < 20; rep++) {
            (void)hipEventRecord(a);
            if (variant == 0) (void)gsr::launch_tile_sort(T, dr, dk, dp, g, 0);
            else hipLaunchKernelGGL(empty_kernel, dim3(T), dim3(256), 0, 0, dr, dp);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms; (void)hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
        }
        printf("%s: %.2f us\n", variant == 0 ? "tile_sort" : "empty (same grid, 32KB LDS)", best * 1000);
    }
    // check: every tile's ids in (depth, id) order of its keys
    std::vector<uint64_t> pl(keys.size());
    (void)hipMemcpy(pl.data(), dp, 8 * keys.size(), hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (int t = 0; t < T; t++) {
        std::vector<uint64_t> k(keys.begin() + ranges[t].x, keys.begin() + ranges[t].y);
        std::sort(k.begin(), k.end());
        for (size_t i = 0; i < k.size(); i++) bad += (uint32_t)pl[ranges[t].x + i] != (uint32_t)k[i];
    }
    printf("done %zu keys, %zu misplaced\n", keys.size(), bad);
    return bad != 0;
}
