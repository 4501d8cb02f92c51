// LDS read throughput of the render kernels' access shapes: ds_read_b128 (and b32) issued back to back by
// W waves per SIMD, addresses (a) one per wave (all 64 lanes the same), (b) one per 16-lane row (4 per wave:
// the per-row lists' entry records), (c) 64 consecutive 16-B slots.  Reports LDS bytes delivered to lanes
// per CU cycle-equivalent (ns) from the kernel's wall time.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/lds_bcast.hip -o tools/micro/lds_bcast
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 2048;

template <int MODE, bool B128>
__global__ void __launch_bounds__(256) lds_kernel(float* out, int salt) {
    __shared__ float4 s[1024];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 1024; i += 256) s[i] = make_float4(i, i + 1, i + 2, i + 3);
    __syncthreads();
    int idx = MODE == 0 ? 0 : MODE == 1 ? (lane >> 4) * 7 : lane;
    idx += salt;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int a = (idx + 64 * k + it) & 1023;
            if (B128) {
                const float4 v = s[a];
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            } else {
                acc.x += reinterpret_cast<const float*>(s)[a];
            }
        }
    }
    out[blockIdx.x * 256 + tid] = acc.x + acc.y + acc.z + acc.w;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * cus * 8);
    const char* mode[3] = {"one address per wave", "one address per 16-lane row", "64 consecutive slots"};
    for (int b = 0; b < 2; b++)
        for (int m = 0; m < 3; m++)
            for (int w = 1; w <= 8; w *= 2) {  // workgroups of 4 waves per CU = waves per SIMD
                auto k = b ? (m == 0 ? lds_kernel<0, true> : m == 1 ? lds_kernel<1, true> : lds_kernel<2, true>)
                           : (m == 0 ? lds_kernel<0, false> : m == 1 ? lds_kernel<1, false> : lds_kernel<2, false>);
                hipLaunchKernelGGL(k, dim3(cus * w), dim3(256), 0, 0, out, 0);
                hipEvent_t e0, e1;
                hipEventCreate(&e0);
                hipEventCreate(&e1);
                hipEventRecord(e0);
                hipLaunchKernelGGL(k, dim3(cus * w), dim3(256), 0, 0, out, 0);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0.f;
                hipEventElapsedTime(&ms, e0, e1);
                const double reads_per_cu = 4.0 * w * ITERS * 8;  // wave-instructions per CU
                const double ns = ms * 1e6;
                printf("%s %-30s waves/SIMD %d: %.2f ns per wave-instruction per CU, %.1f B/ns per CU delivered\n",
                       b ? "b128" : "b32 ", mode[m], w, ns / reads_per_cu, reads_per_cu * 64 * (b ? 16 : 4) / ns);
            }
    return 0;
}
