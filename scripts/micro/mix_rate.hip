// VALU issue rate of v_fma_mix_f32 (f16 operand from an SGPR half) vs v_fma_f32 (f32 SGPR operand), the two forms of
// the render kernel's box-plane evaluation: 8 independent chains per lane, 256 iterations, one wave per SIMD or four.
// usage: ./mix_rate   (prints cycles per wave-instruction for each form and occupancy)
#include <hip/hip_runtime.h>
#include <cstdio>

template <int FORM>
__global__ __launch_bounds__(256) void k(const int* __restrict__ sp, float* out, unsigned long long* cyc, int iters) {
    const int w = sp[0];  // scalar
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float b = 1.0001f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#define STEP(x)                                                                                                     \
    if constexpr (FORM == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "s"(w), "v"(b));                  \
    else if constexpr (FORM == 1) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "s"(w), "v"(b)); \
    else asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(x) : "s"(w), "v"(b));
        STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    int* sp;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&sp, 4);
    int h = 0x3c003c00;
    hipMemcpy(sp, &h, 4, hipMemcpyHostToDevice);
    const int blocks = 256 * 4;
    hipMalloc(&out, 4 * 256 * blocks * 4);
    hipMalloc(&cyc, 8 * blocks * 4);
    unsigned long long hc[4096];
    const char* names[3] = {"v_fma_f32 (SGPR f32)", "v_fma_mix_f32 (SGPR f16 lo)", "v_fma_mix_f32 (SGPR f16 hi)"};
    for (int wpb : {64, 256}) {  // 1 wave per workgroup / 4 waves per workgroup
        for (int f = 0; f < 3; ++f) {
            for (int rep = 0; rep < 2; ++rep) {
                const int iters = 512;
                hipEvent_t e0, e1;
                hipEventCreate(&e0);
                hipEventCreate(&e1);
                hipEventRecord(e0);
                if (f == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(wpb), 0, 0, sp, out, cyc, iters);
                if (f == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(wpb), 0, 0, sp, out, cyc, iters);
                if (f == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(wpb), 0, 0, sp, out, cyc, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                hipMemcpy(hc, cyc, 8 * blocks, hipMemcpyDeviceToHost);
                double s = 0;
                for (int i = 0; i < blocks; ++i) s += hc[i];
                const double instr = 8.0 * iters;
                // s_memtime counts at a fixed 100 MHz-class clock on gfx9? report raw ticks and the event time
                if (rep == 1)
                    printf("%-30s wave/WG %d: %.3f ms, %.2f memtime ticks per instr per wave, %.1f G wave-instr/s\n",
                           names[f], wpb / 64, ms, s / blocks / instr, blocks * (wpb / 64) * instr / (ms * 1e-3) / 1e9);
            }
        }
    }
    return 0;
}
