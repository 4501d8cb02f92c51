// Microbenchmark: 677k global atomicAdds (2.26 per thread, like the binning
// counters) onto A distinct addresses (stride S u32), returning vs not.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_atomic(const uint32_t* __restrict__ tgt, int n, uint32_t* ctr, int stride, int ret,
                         uint32_t* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t acc = 0;
    for (int r = 0; r < 2; r++) {  // 2 atomics per thread (~2.26 in the rasterizer)
        uint32_t t = tgt[2 * i + r];
        if (ret) acc += atomicAdd(&ctr[t * stride], 1u);
        else atomicAdd(&ctr[t * stride], 1u);
    }
    if (ret) out[i] = acc;
}

int main() {
    const int n = 340000;  // threads -> 680k atomics
    std::vector<uint32_t> h(2 * n);
    uint32_t *dt, *dc, *dout;
    hipMalloc(&dt, 8 * n);
    hipMalloc(&dc, 4 * 16 * 64 * 10000);
    hipMalloc(&dout, 4 * n);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int addrs[] = {1200, 9600, 76800};
    int strides[] = {1, 16, 32, 64};
    for (int A : addrs) {
        srand(1);
        for (auto& x : h) x = rand() % A;
        hipMemcpy(dt, h.data(), 8 * n, hipMemcpyHostToDevice);
        for (int S : strides) {
            if ((size_t)A * S > 16u * 64 * 10000) continue;
            for (int ret = 0; ret < 2; ret++) {
                float best = 1e9;
                for (int rep = 0; rep < 5; rep++) {
                    hipMemsetAsync(dc, 0, 4 * (size_t)A * S);
                    hipEventRecord(a);
                    hipLaunchKernelGGL(k_atomic, dim3((n + 255) / 256), dim3(256), 0, 0, dt, n, dc, S, ret, dout);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                    float ms;
                    hipEventElapsedTime(&ms, a, b);
                    if (ms < best) best = ms;
                }
                printf("addrs %6d stride %3d %s: %8.2f us\n", A, S, ret ? "returning" : "no-return", best * 1000);
            }
        }
    }
    return 0;
}
