// Probe: which (XCC_ID, HW_ID) keys do one-wave workgroups run on?  Prints the distinct keys and counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void k(unsigned* out) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = hw; out[2 * blockIdx.x + 1] = xcc; }
}
int main() {
    const int n = 8192;
    unsigned* d; (void)hipMalloc(&d, 8 * n);
    hipLaunchKernelGGL(k, dim3(n), dim3(64), 0, 0, d);
    std::vector<unsigned> h(2 * n);
    (void)hipMemcpy(h.data(), d, 8 * n, hipMemcpyDeviceToHost);
    std::map<unsigned, int> keys;
    std::map<unsigned, int> xccs;
    for (int i = 0; i < n; ++i) {
        unsigned hw = h[2 * i], x = h[2 * i + 1];
        unsigned key = ((x & 0xF) << 16) | ((hw >> 8) & 0xFFFF);
        keys[key]++; xccs[x]++;
        if (i < 24) printf("block %d hw %08x xcc %08x cu %u sh %u se %u\n", i, hw, x, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7);
    }
    printf("distinct (xcc, hw[23:8]) keys: %zu\n", keys.size());
    printf("distinct xcc values: %zu\n", xccs.size());
    std::map<unsigned, int> cus;
    for (auto& kv : keys) cus[(kv.first & 0xF0000) | (kv.first & 0xFF)]++;
    printf("distinct (xcc, se, sh, cu): %zu\n", cus.size());
    int shown = 0;
    for (auto& kv : cus) { if (shown++ < 40) printf("  xcc %u se %u sh %u cu %u\n", kv.first >> 16, (kv.first >> 5) & 7, (kv.first >> 4) & 1, kv.first & 15); }
    return 0;
}
