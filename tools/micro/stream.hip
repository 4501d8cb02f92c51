// STREAM-style HBM bandwidth on the box ("confirm [8 TB/s] with a STREAM-style copy").
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro/stream.hip -o tools/micro/stream
// Prints one JSON line: copy / scale / add / triad GB/s (best of 20 timed launches after 3 warm-ups,
// hipEvents), counting each kernel's algorithmic bytes (copy, scale: 2 x 8 B... per element of float4:
// read + write; add, triad: 2 reads + 1 write), over 1 GiB arrays (far beyond the 256 MB of L2 + MALL).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

// grid-stride float4 streams, 4 float4 per thread per iteration (loads issued before the stores)
__global__ void __launch_bounds__(256) k_copy(const float4* __restrict__ a, float4* __restrict__ c, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c[i] = a[i];
}
__global__ void __launch_bounds__(256) k_scale(const float4* __restrict__ a, float4* __restrict__ c, float s,
                                                size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 v = a[i];
        c[i] = make_float4(s * v.x, s * v.y, s * v.z, s * v.w);
    }
}
__global__ void __launch_bounds__(256) k_add(const float4* __restrict__ a, const float4* __restrict__ b,
                                              float4* __restrict__ c, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 x = a[i], y = b[i];
        c[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
    }
}
__global__ void __launch_bounds__(256) k_triad(const float4* __restrict__ a, const float4* __restrict__ b,
                                                float4* __restrict__ c, float s, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 x = a[i], y = b[i];
        c[i] = make_float4(x.x + s * y.x, x.y + s * y.y, x.z + s * y.z, x.w + s * y.w);
    }
}

int main() {
    const size_t bytes = (size_t)1 << 30, n = bytes / sizeof(float4);
    float4 *a, *b, *c;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&c, bytes));
    CHECK(hipMemset(a, 0, bytes));
    CHECK(hipMemset(b, 0, bytes));
    CHECK(hipMemset(c, 0, bytes));
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char* names[4] = {"copy", "scale", "add", "triad"};
    const double traffic[4] = {2.0 * bytes, 2.0 * bytes, 3.0 * bytes, 3.0 * bytes};
    double best[4] = {0, 0, 0, 0};
    const int grids[3] = {cus * 8, cus * 16, cus * 32};
    int best_grid[4] = {0, 0, 0, 0};
    for (int gi = 0; gi < 3; gi++) {
        const dim3 grid(grids[gi]), block(256);
        for (int k = 0; k < 4; k++) {
            auto launch = [&]() {
                if (k == 0) hipLaunchKernelGGL(k_copy, grid, block, 0, 0, a, c, n);
                if (k == 1) hipLaunchKernelGGL(k_scale, grid, block, 0, 0, a, c, 3.0f, n);
                if (k == 2) hipLaunchKernelGGL(k_add, grid, block, 0, 0, a, b, c, n);
                if (k == 3) hipLaunchKernelGGL(k_triad, grid, block, 0, 0, a, b, c, 3.0f, n);
            };
            for (int w = 0; w < 3; w++) launch();
            CHECK(hipDeviceSynchronize());
            for (int r = 0; r < 20; r++) {
                CHECK(hipEventRecord(e0, 0));
                launch();
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms = 0.f;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                const double gbs = traffic[k] / (ms * 1e-3) / 1e9;
                if (gbs > best[k]) {
                    best[k] = gbs;
                    best_grid[k] = grids[gi];
                }
            }
        }
    }
    printf("{\"array_bytes\": %zu, \"cus\": %d", bytes, cus);
    for (int k = 0; k < 4; k++) printf(", \"%s_gbs\": %.1f, \"%s_grid\": %d", names[k], best[k], names[k], best_grid[k]);
    printf("}\n");
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(c));
    return 0;
}
