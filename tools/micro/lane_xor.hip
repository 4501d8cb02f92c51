// Checks the DPP / permlane-swap forms of a lane-xor exchange against __shfl_xor
// (which lowers to ds_bpermute) for every xor distance used by the tile sort.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/lane_xor.hip -o /tmp/lane_xor
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned* out) {
    const unsigned lane = threadIdx.x, x = lane;
    unsigned c[9];
    c[0] = __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    c[1] = __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    c[2] = __builtin_amdgcn_mov_dpp(x, 0x104, 0xF, 0xF, false);  // row_shl:4
    c[3] = __builtin_amdgcn_mov_dpp(x, 0x114, 0xF, 0xF, false);  // row_shr:4
    c[4] = __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false);  // row_ror:8
    auto p16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    auto p32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    c[5] = p16[0]; c[6] = p16[1]; c[7] = p32[0]; c[8] = p32[1];
    for (int k = 0; k < 9; k++) out[k * 64 + lane] = c[k];
}

int main() {
    unsigned* d;
    hipMalloc(&d, 9 * 64 * 4);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    unsigned h[9 * 64];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[9] = {"qp1032", "qp2301", "row_shl4", "row_shr4", "row_ror8", "p16[0]", "p16[1]", "p32[0]",
                            "p32[1]"};
    for (int k = 0; k < 9; k++) {
        printf("%-9s", names[k]);
        for (int l = 0; l < 64; l++) printf(" %2u", h[k * 64 + l]);
        printf("\n");
    }
    return 0;
}
