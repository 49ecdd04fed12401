// Microbenchmark (round 4, dispatch-order study): cost of device-scope atomics on one address and on distinct
// addresses, from lane 0 of each one-wave workgroup, dependent chains of K operations.  Vector atomics only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_same(unsigned* ctr, int k, unsigned* sink) {
    if (threadIdx.x != 0) return;
    unsigned v = 0;
    for (int i = 0; i < k; ++i) v += atomicAdd(ctr, 1u + (v & 0u));
    sink[blockIdx.x] = v;
}
__global__ void k_distinct(unsigned* ctr, int k, unsigned* sink) {
    if (threadIdx.x != 0) return;
    unsigned v = 0;
    for (int i = 0; i < k; ++i) v += atomicAdd(ctr + 64u * blockIdx.x, 1u + (v & 0u));
    sink[blockIdx.x] = v;
}
__global__ void k_same_wg(unsigned* ctr, int k, unsigned* sink) {
    if (threadIdx.x != 0) return;
    unsigned v = 0;
    for (int i = 0; i < k; ++i)
        v += __hip_atomic_fetch_add(ctr + 64u * (blockIdx.x % 8u), 1u + (v & 0u), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
    sink[blockIdx.x] = v;
}
__global__ void k_same8(unsigned* ctr, int k, unsigned* sink) {
    if (threadIdx.x != 0) return;
    unsigned v = 0;
    for (int i = 0; i < k; ++i) v += atomicAdd(ctr + 64u * (blockIdx.x % 8u), 1u + (v & 0u));
    sink[blockIdx.x] = v;
}

// dependent chains: each atomic's address depends on the previous result (latency, not throughput)
__global__ void k_chain_rmw(unsigned* ctr, int k, unsigned* sink) {
    if (threadIdx.x != 0) return;
    unsigned v = 0;
    for (int i = 0; i < k; ++i) v = atomicAdd(ctr + 64u * blockIdx.x + (v & 1u), 0u);
    sink[blockIdx.x] = v;
}
__global__ void k_chain_load(unsigned* ctr, int k, unsigned* sink) {
    if (threadIdx.x != 0) return;
    unsigned v = 0;
    for (int i = 0; i < k; ++i)
        v = __hip_atomic_load(ctr + 64u * blockIdx.x + (v & 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sink[blockIdx.x] = v;
}
__global__ void k_chain_plain(unsigned* ctr, int k, unsigned* sink) {
    if (threadIdx.x != 0) return;
    unsigned v = 0;
    for (int i = 0; i < k; ++i) v = ((volatile unsigned*)ctr)[64u * blockIdx.x + (v & 1u)];
    sink[blockIdx.x] = v;
}

int main() {
    unsigned *ctr, *sink;
    const int nb = 32400;
    hipMalloc(&ctr, 64 * 4 * nb);
    hipMalloc(&sink, 4 * nb);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct K { const char* name; void (*f)(unsigned*, int, unsigned*); };
    K ks[] = {{"same", k_same}, {"distinct", k_distinct}, {"same8_agent", k_same8}, {"same8_wg_scope", k_same_wg}};
    {
        K cs[] = {{"chain_rmw", k_chain_rmw}, {"chain_agent_load", k_chain_load}, {"chain_volatile", k_chain_plain}};
        for (auto& kk : cs) {
            const int k = 64;
            float best = 1e9f;
            for (int rep = 0; rep < 4; ++rep) {
                hipMemset(ctr, 0, 64 * 4 * nb);
                hipEventRecord(a);
                hipLaunchKernelGGL(kk.f, dim3(256), dim3(64), 0, 0, ctr, k, sink);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            printf("%-16s 256 waves, chains of %d: %8.3f ms  (%6.0f ns per dependent op)\n", kk.name, k, best,
                   best * 1e6 / k);
        }
    }
    for (auto& kk : ks) {
        for (int k : {1, 4, 16}) {
            float best = 1e9f;
            for (int rep = 0; rep < 4; ++rep) {
                hipMemset(ctr, 0, 64 * 4 * nb);
                hipEventRecord(a);
                hipLaunchKernelGGL(kk.f, dim3(nb), dim3(64), 0, 0, ctr, k, sink);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
            }
            unsigned h[8 * 64];
            hipMemcpy(h, ctr, sizeof(h), hipMemcpyDeviceToHost);
            unsigned tot = 0;
            for (int q = 0; q < 8; ++q) tot += h[64 * q];
            printf("%-16s k=%2d  %8.3f ms  (%6.1f ns per op over %d ops)  counter(s) %u expected %d\n", kk.name, k, best,
                   best * 1e6 / ((double)nb * k), nb * k, (kk.f == k_distinct) ? h[0] : (kk.f == k_same ? h[0] : tot),
                   (kk.f == k_distinct) ? k : nb * k);
        }
    }
    return 0;
}
