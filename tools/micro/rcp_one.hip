// Does v_rcp_f32(1.0f) return exactly 1.0f?  (render_bwd's T update T * rcp(1 - alpha) with alpha = 0
// for non-contributing pairs keeps T unchanged without a select only if it does.)
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/rcp_one.hip -o tools/micro/rcp_one
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void rcp_kernel(const float* in, float* out) {
    const int i = threadIdx.x;
    out[i] = __builtin_amdgcn_rcpf(1.f - in[i]);
}

int main() {
    float h_in[64], h_out[64];
    for (int i = 0; i < 64; i++) h_in[i] = 0.f;
    h_in[1] = -0.f;
    float *d_in, *d_out;
    hipMalloc(&d_in, sizeof(h_in));
    hipMalloc(&d_out, sizeof(h_out));
    hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(rcp_kernel, dim3(1), dim3(64), 0, 0, d_in, d_out);
    hipMemcpy(h_out, d_out, sizeof(h_out), hipMemcpyDeviceToHost);
    unsigned b0, b1;
    memcpy(&b0, &h_out[0], 4);
    memcpy(&b1, &h_out[1], 4);
    printf("rcp(1 - 0) bits 0x%08x, rcp(1 - (-0)) bits 0x%08x, exact one: %s\n", b0, b1,
           (b0 == 0x3f800000u && b1 == 0x3f800000u) ? "yes" : "no");
    return 0;
}
