// VALU issue rate on one SIMD as a function of the waves sharing it (the question behind the render
// kernels' bound: how many cycles does a wave64 VALU instruction occupy the 32-lane SIMD when 1..6 waves
// interleave).  Every CU gets W 256-thread workgroups (W waves per SIMD); each wave runs a long stream of
// a given instruction mix on 8 independent accumulator chains (no memory traffic), timed per wave with
// s_memtime (shader clock).  cycles per instruction per SIMD = (wave cycles / instructions) / W.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/micro/valu_rate.hip -o tools/micro/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

template <int MIX>
__global__ void __launch_bounds__(256) valu_kernel(float* out, unsigned long long* cyc, float seed) {
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = seed * (threadIdx.x + k);
    const float b = seed * 1.0001f, c = seed * 0.9999f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (MIX == 0) {  // plain fma
                a[k] = __builtin_fmaf(a[k], b, c);
            } else if (MIX == 1) {  // fma + a DPP add (the row reduction's form)
                a[k] = __builtin_fmaf(a[k], b, c);
                a[k] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a[k]), 0x128, 0xF, 0xF, true));
            } else if (MIX == 2) {  // fma + select (v_cndmask)
                a[k] = __builtin_fmaf(a[k], b, c);
                a[k] = a[k] > c ? a[k] : b;
            } else if (MIX == 3) {  // fma + exp (transcendental)
                a[k] = __builtin_fmaf(a[k], b, c);
                a[k] = __builtin_amdgcn_exp2f(a[k]);
            } else if (MIX >= 4) {  // fma, then (after the unrolled fmas) a lane-half swap per pair + add/sub
                a[k] = __builtin_fmaf(a[k], b, c);
            }
        }
        if (MIX >= 4) {  // v_permlane32_swap (MIX 4) / v_permlane16_swap (MIX 5): one per two chains
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const auto r = MIX == 4 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(a[k]), __float_as_uint(a[k + 1]), false, false)
                                        : __builtin_amdgcn_permlane16_swap(__float_as_uint(a[k]), __float_as_uint(a[k + 1]), false, false);
                a[k] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
                a[k + 1] = __uint_as_float(r[0]) - __uint_as_float(r[1]);
            }
        }
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; k++) s += a[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int maxw = 6;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, sizeof(float) * 256 * cus * maxw);
    hipMalloc(&cyc, sizeof(unsigned long long) * 4 * cus * maxw);
    const char* names[6] = {"fma", "fma+dpp_add", "fma+cndmask", "fma+exp", "fma+pl32swap", "fma+pl16swap"};
    const int per_iter[6] = {8, 16, 24, 16, 20, 20};  // VALU instructions per loop iteration (checked in the ISA, -fno-slp-vectorize)
    for (int mix = 0; mix < 6; mix++) {
        for (int w = 1; w <= maxw; w++) {
            const int blocks = cus * w;
            auto k = mix == 0 ? valu_kernel<0> : mix == 1 ? valu_kernel<1> : mix == 2 ? valu_kernel<2> : mix == 3 ? valu_kernel<3> : mix == 4 ? valu_kernel<4> : valu_kernel<5>;
            hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0f);  // warm-up
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long* h = new unsigned long long[4 * blocks];
            hipMemcpy(h, cyc, sizeof(unsigned long long) * 4 * blocks, hipMemcpyDeviceToHost);
            double mean = 0;
            for (int i = 0; i < 4 * blocks; i++) mean += (double)h[i];
            mean /= 4 * blocks;
            delete[] h;
            const double insts = (double)ITERS * per_iter[mix];
            // every SIMD holds w waves for the whole run: wall instructions per SIMD = w * insts
            const double sec = ms * 1e-3;
            printf("%-12s waves/SIMD %d: %.2f cycles/instr per wave (s_memtime), %.2f cycles/instr per SIMD; "
                   "kernel %.1f us, SIMD issue rate %.3f instr/ns\n",
                   names[mix], w, mean / insts, mean / insts / w, ms * 1e3, w * insts / (sec * 1e9));
        }
    }
    return 0;
}
