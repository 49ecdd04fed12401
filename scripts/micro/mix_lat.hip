// Dependent-chain latency of v_fma_mix_f32 (f16 operand from an SGPR half) vs v_fma_f32, and of a mix -> v_max3
// pair: one chain per lane, one wave per SIMD, so each instruction waits for its predecessor's result.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int FORM>
__global__ __launch_bounds__(64) void k(const int* __restrict__ sp, float* out, unsigned long long* cyc, int iters) {
    const int w = sp[0];
    float a = threadIdx.x, c = 0.5f;
    const float b = 1.0001f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#define STEP                                                                                                  \
    if constexpr (FORM == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "s"(w), "v"(b));             \
    else if constexpr (FORM == 1) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(a) : "s"(w), "v"(b)); \
    else if constexpr (FORM == 2) asm volatile("v_fma_f32 %0, %1, %2, %0\n\tv_max3_f32 %0, %0, %3, %3" : "+v"(a) : "s"(w), "v"(b), "v"(c)); \
    else asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]\n\tv_max3_f32 %0, %0, %3, %3" : "+v"(a) : "s"(w), "v"(b), "v"(c));
        STEP STEP STEP STEP STEP STEP STEP STEP
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    int* sp;
    float* out;
    unsigned long long* cyc;
    (void)hipMalloc(&sp, 4);
    int h = 0x3c003c00;
    (void)hipMemcpy(sp, &h, 4, hipMemcpyHostToDevice);
    const int blocks = 1024;
    (void)hipMalloc(&out, 4 * 64 * blocks);
    (void)hipMalloc(&cyc, 8 * blocks);
    static unsigned long long hc[1024];
    const char* names[4] = {"v_fma_f32 chain", "v_fma_mix_f32 chain", "v_fma_f32 -> v_max3 chain (per pair)",
                            "v_fma_mix_f32 -> v_max3 chain (per pair)"};
    for (int f = 0; f < 4; ++f)
        for (int rep = 0; rep < 2; ++rep) {
            const int iters = 1024;
            if (f == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, sp, out, cyc, iters);
            if (f == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, sp, out, cyc, iters);
            if (f == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, sp, out, cyc, iters);
            if (f == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(64), 0, 0, sp, out, cyc, iters);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(hc, cyc, 8 * blocks, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < blocks; ++i) s += hc[i];
            if (rep == 1) printf("%-45s %.2f s_memtime ticks per step\n", names[f], s / blocks / (8.0 * iters));
        }
    return 0;
}
