// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of the
// render kernels (MI355X_MICROARCH.md: "other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern").  Each kernel moves a known number of bytes
// through a table far larger than the 256 MiB Infinity Cache, each line touched once:
//   stream16   coalesced 16 B / lane reads                  (the guide's reference pattern)
//   gather64   one 64-B record (4 x float4) per lane at permuted record indices (render records)
//   scatter24  one 24-B record (3 x float2) per lane at permuted slots (tracking instance records)
//   scatter40  one 40-B record (5 x float2) per lane at permuted slots (mapping instance records)
//   stream4    the 4-B permutation reads alone (subtracted from the permuted kernels)
//   gather24   24-B records at permuted slots (gauss_bwd-style record reads, contiguous per lane)
// Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); the known
// byte counts are printed.  Build: hipcc -O3 --offload-arch=gfx950 traffic_calib.hip -o traffic_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void stream16(const float4* __restrict__ a, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = a[i];
    if (v.x == 1.2345f) out[0] = v.y;
}
__global__ void gather64(const float4* __restrict__ rec, const uint32_t* __restrict__ perm, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4* r = rec + 4 * (size_t)perm[i];
    const float4 a = r[0], b = r[1], c = r[2], d = r[3];
    const float s = a.x + b.y + c.z + d.w;
    if (s == 1.2345f) out[0] = s;
}
__global__ void stream4(const uint32_t* __restrict__ perm, int n, float* out) {  // the permutation reads alone
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (perm[i] == 0xFFFFFFFFu) out[0] = 1.f;
}
template <int NF2>
__global__ void scatter_rec(float2* __restrict__ dst, const uint32_t* __restrict__ perm, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float2* d = dst + (size_t)NF2 * perm[i];
#pragma unroll
    for (int m = 0; m < NF2; m++) d[m] = make_float2((float)i, (float)m);
}
template <int NF2>
__global__ void gather_rec(const float2* __restrict__ src, const uint32_t* __restrict__ perm, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2* s = src + (size_t)NF2 * perm[i];
    float acc = 0.f;
#pragma unroll
    for (int m = 0; m < NF2; m++) acc += s[m].x + s[m].y;
    if (acc == 1.2345f) out[0] = acc;
}

int main() {
    const int n = 8 << 20;  // 8 Mi records: 512 MiB of 64-B records, 192 / 320 MiB of 24 / 40-B records
    std::vector<uint32_t> p(n);
    for (int i = 0; i < n; i++) p[i] = (uint32_t)i;
    srand(1);
    for (int i = n - 1; i > 0; i--) {
        const int j = (int)(((unsigned long long)rand() * RAND_MAX + rand()) % (unsigned long long)(i + 1));
        const uint32_t t = p[i];
        p[i] = p[j];
        p[j] = t;
    }
    uint32_t* perm;
    float4* big;
    float* out;
    const size_t big_bytes = (size_t)64 * n;
    hipMalloc(&perm, sizeof(uint32_t) * n);
    hipMalloc(&big, big_bytes);
    hipMalloc(&out, 64);
    hipMemcpy(perm, p.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice);
    hipMemset(big, 0, big_bytes);
    const int tb = 256, nb = (n + tb - 1) / tb;
    // stream16 over the whole 512 MiB table as float4 (4 per 64-B record)
    hipLaunchKernelGGL(stream16, dim3(4 * nb), dim3(tb), 0, 0, big, 4 * n, out);
    hipLaunchKernelGGL(stream4, dim3(nb), dim3(tb), 0, 0, perm, n, out);
    hipLaunchKernelGGL(gather64, dim3(nb), dim3(tb), 0, 0, big, perm, n, out);
    hipLaunchKernelGGL((scatter_rec<3>), dim3(nb), dim3(tb), 0, 0, (float2*)big, perm, n);
    hipLaunchKernelGGL((scatter_rec<5>), dim3(nb), dim3(tb), 0, 0, (float2*)big, perm, n);
    hipLaunchKernelGGL((gather_rec<3>), dim3(nb), dim3(tb), 0, 0, (const float2*)big, perm, n, out);
    hipDeviceSynchronize();
    printf("{\"records\": %d, \"stream16_bytes\": %zu, \"gather64_bytes\": %zu, \"scatter24_bytes\": %zu, "
           "\"scatter40_bytes\": %zu, \"gather24_bytes\": %zu, \"perm_bytes\": %zu}\n",
           n, big_bytes, (size_t)64 * n, (size_t)24 * n, (size_t)40 * n, (size_t)24 * n, sizeof(uint32_t) * (size_t)n);
    return 0;
}
