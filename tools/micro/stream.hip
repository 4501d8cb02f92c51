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
// one-shot block tiles: every thread issues U float4 loads (strided by the block size, so each load
// instruction covers 1 KiB contiguous per wave... 4 KiB per block) before its U stores; NT: nontemporal
// loads/stores (streaming data that is never re-read)
typedef float f4v __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_copy_tile(const float4* __restrict__ a4, float4* __restrict__ c4, size_t n) {
    const f4v* __restrict__ a = reinterpret_cast<const f4v*>(a4);
    f4v* __restrict__ c = reinterpret_cast<f4v*>(c4);
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f4v v[U];
#pragma unroll
    for (int j = 0; j < U; j++) {
        const size_t i = base + (size_t)j * 256;
        if (i < n) v[j] = NT ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int j = 0; j < U; j++) {
        const size_t i = base + (size_t)j * 256;
        if (i < n) {
            if (NT)
                __builtin_nontemporal_store(v[j], c + i);
            else
                c[i] = v[j];
        }
    }
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
    // the block-tile copies (U float4 per thread, plain or nontemporal): the best of them is copy_tile_gbs
    const char* tnames[6] = {"u4", "u8", "u16", "u4nt", "u8nt", "u16nt"};
    double tbest[6] = {0, 0, 0, 0, 0, 0};
    for (int v = 0; v < 6; v++) {
        const int U = (v % 3 == 0) ? 4 : (v % 3 == 1) ? 8 : 16;
        const dim3 grid((unsigned)((n + 256 * U - 1) / (256 * U))), block(256);
        auto launch = [&]() {
            switch (v) {
                case 0: hipLaunchKernelGGL((k_copy_tile<4, false>), grid, block, 0, 0, a, c, n); break;
                case 1: hipLaunchKernelGGL((k_copy_tile<8, false>), grid, block, 0, 0, a, c, n); break;
                case 2: hipLaunchKernelGGL((k_copy_tile<16, false>), grid, block, 0, 0, a, c, n); break;
                case 3: hipLaunchKernelGGL((k_copy_tile<4, true>), grid, block, 0, 0, a, c, n); break;
                case 4: hipLaunchKernelGGL((k_copy_tile<8, true>), grid, block, 0, 0, a, c, n); break;
                default: hipLaunchKernelGGL((k_copy_tile<16, true>), grid, block, 0, 0, a, c, n); break;
            }
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
            const double gbs = 2.0 * bytes / (ms * 1e-3) / 1e9;
            if (gbs > tbest[v]) tbest[v] = gbs;
        }
    }
    int tb = 0;
    for (int v = 1; v < 6; v++)
        if (tbest[v] > tbest[tb]) tb = v;
    printf("{\"array_bytes\": %zu, \"cus\": %d, \"copy_tile_gbs\": %.1f, \"copy_tile_form\": \"%s\"", bytes, cus,
           tbest[tb], tnames[tb]);
    for (int v = 0; v < 6; v++) printf(", \"copy_tile_%s_gbs\": %.1f", tnames[v], tbest[v]);
    for (int k = 0; k < 4; k++) printf(", \"%s_gbs\": %.1f, \"%s_grid\": %d", names[k], best[k], names[k], best_grid[k]);
    printf("}\n");
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(c));
    return 0;
}
