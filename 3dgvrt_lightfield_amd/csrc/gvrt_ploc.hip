// gvrt_ploc.hip — PLOC binary BVH builder (parallel locally-ordered clustering).
//
// Meister & Bittner, "Parallel Locally-Ordered Clustering for Bounding Volume Hierarchy
// Construction", IEEE TVCG 2018.  Starting from the proxies in Morton order (gvrt_lbvh.hip steps
// 1-4), every iteration
//   1. finds each cluster's nearest neighbour among the R clusters on either side in Morton order,
//      distance = surface area of the union box (LDS-staged window, one thread per cluster),
//   2. merges mutual nearest neighbours into a new binary node (the lower index keeps the merged
//      cluster, the higher one drops out),
//   3. compacts the surviving clusters (hipcub scan), keeping Morton order,
// until one cluster (the root) is left.  The agglomerative merges give lower-SAH trees than the
// Karras LBVH (fewer node visits per ray); the output is the same binary BvhNode layout (child
// boxes inline), with parent links for the depth census and the 4-wide collapse.
#include <hipcub/hipcub.hpp>

#include "gvrt_internal.h"

using namespace gvrt;

namespace {

constexpr int PLOC_R = 16;   // search radius
constexpr int PLOC_B = 256;  // clusters per block

__device__ inline float half_area6(const float* a, const float* b) {
    const float ex = fmaxf(a[3], b[3]) - fminf(a[0], b[0]);
    const float ey = fmaxf(a[4], b[4]) - fminf(a[1], b[1]);
    const float ez = fmaxf(a[5], b[5]) - fminf(a[2], b[2]);
    return ex * ey + ey * ez + ez * ex;
}

// 1. nearest neighbour within +-R in cluster order; ties -> the lower index (symmetric distance, so
// the mutual-pair test below is consistent)
__global__ __launch_bounds__(PLOC_B) void k_ploc_nn(uint32_t n, const float* __restrict__ boxes, int32_t* __restrict__ nn) {
    __shared__ float sb[(PLOC_B + 2 * PLOC_R) * 6];
    const int64_t base = (int64_t)blockIdx.x * PLOC_B - PLOC_R;
    for (int t = threadIdx.x; t < (PLOC_B + 2 * PLOC_R) * 6; t += PLOC_B) {
        const int64_t j = base + t / 6;
        sb[t] = (j >= 0 && j < (int64_t)n) ? boxes[6 * j + t % 6] : 0.0f;
    }
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * PLOC_B + threadIdx.x;
    if (i >= (int64_t)n) return;
    const float* bi = sb + 6 * (threadIdx.x + PLOC_R);
    float best = INFINITY;
    int32_t bj = -1;
    for (int d = -PLOC_R; d <= PLOC_R; ++d) {
        const int64_t j = i + d;
        if (d == 0 || j < 0 || j >= (int64_t)n) continue;
        const float a = half_area6(bi, sb + 6 * (threadIdx.x + PLOC_R + d));
        if (a < best) {  // strict: scanning upward, a tie keeps the lower index
            best = a;
            bj = (int32_t)j;
        }
    }
    nn[i] = bj;
}

// 2. merge mutual pairs; keep[i] = 1 for every cluster that survives (merged or untouched)
__global__ __launch_bounds__(256) void k_ploc_merge(uint32_t n, const int32_t* __restrict__ nn, float* __restrict__ boxes,
                                                    int32_t* __restrict__ refs, BvhNode* __restrict__ bin,
                                                    uint32_t* __restrict__ counter, int32_t* __restrict__ leaf_parent,
                                                    int32_t* __restrict__ node_parent, uint32_t* __restrict__ keep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n) return;
    const int32_t j = nn[i];
    const bool mutual = j >= 0 && nn[j] == (int32_t)i;
    if (!mutual) {
        keep[i] = 1u;
        return;
    }
    if (j < i) {
        keep[i] = 0u;  // the partner (lower index) builds the node
        return;
    }
    const uint32_t id = atomicAdd(counter, 1u);
    BvhNode nd;
    float* f = reinterpret_cast<float*>(&nd);
    float u[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const float a = boxes[6 * i + k], b = boxes[6 * (int64_t)j + k];
        f[k] = a;
        f[6 + k] = b;
        u[k] = k < 3 ? fminf(a, b) : fmaxf(a, b);
    }
    int32_t ri = refs[i], rj = refs[j];
    // split axis (for the render kernel's child order): the axis of the largest centroid separation,
    // with c0 on its lower side
    float cs[3];
    for (int k = 0; k < 3; ++k) cs[k] = (f[6 + k] + f[9 + k]) - (f[k] + f[3 + k]);
    const uint32_t ax = fabsf(cs[0]) >= fabsf(cs[1]) && fabsf(cs[0]) >= fabsf(cs[2]) ? 0u : (fabsf(cs[1]) >= fabsf(cs[2]) ? 1u : 2u);
    if (cs[ax] < 0.0f) {
        for (int k = 0; k < 6; ++k) {
            const float t = f[k];
            f[k] = f[6 + k];
            f[6 + k] = t;
        }
        const int32_t t = ri;
        ri = rj;
        rj = t;
    }
    nd.c0 = ri;
    nd.c1 = rj;
    nd.pad0 = ax;
    nd.pad1 = 0;
    bin[id] = nd;
    if (ri < 0) leaf_parent[~ri] = (int32_t)id;
    else node_parent[ri] = (int32_t)id;
    if (rj < 0) leaf_parent[~rj] = (int32_t)id;
    else node_parent[rj] = (int32_t)id;
#pragma unroll
    for (int k = 0; k < 6; ++k) boxes[6 * i + k] = u[k];
    refs[i] = (int32_t)id;
    keep[i] = 1u;
}

// 3. order-preserving compaction of the surviving clusters
__global__ __launch_bounds__(256) void k_ploc_compact(uint32_t n, const uint32_t* __restrict__ keep,
                                                      const uint32_t* __restrict__ pos, const float* __restrict__ boxes,
                                                      const int32_t* __restrict__ refs, float* __restrict__ boxes2,
                                                      int32_t* __restrict__ refs2) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n || !keep[i]) return;
    const uint32_t p = pos[i];
#pragma unroll
    for (int k = 0; k < 6; ++k) boxes2[6 * (int64_t)p + k] = boxes[6 * i + k];
    refs2[p] = refs[i];
}

__global__ __launch_bounds__(256) void k_ploc_init(uint32_t m, const float* __restrict__ leaf_boxes, float* __restrict__ boxes,
                                                   int32_t* __restrict__ refs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)m) return;
#pragma unroll
    for (int k = 0; k < 6; ++k) boxes[6 * i + k] = leaf_boxes[6 * i + k];
    refs[i] = ~(int32_t)i;
}

}  // namespace

// Builds the binary tree over m >= 2 leaves (leaf j = record j, boxes in leaf order) into bin
// (m - 1 nodes); fills leaf_parent / node_parent (root's parent -1) and returns the root index.
gvrt_status gvrt_ploc_build(gvrt_context* c, uint32_t m, const float* leaf_boxes, BvhNode* bin, int32_t* leaf_parent,
                            int32_t* node_parent, int32_t* root, uint32_t* iterations) {
    gvrt_status s = GVRT_OK;
    float *b0 = nullptr, *b1 = nullptr;
    int32_t *r0 = nullptr, *r1 = nullptr, *nn = nullptr;
    uint32_t *keep = nullptr, *pos = nullptr, *counter = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    auto cleanup = [&]() {
        gvrt_dfree(c, (void**)&b0);
        gvrt_dfree(c, (void**)&b1);
        gvrt_dfree(c, (void**)&r0);
        gvrt_dfree(c, (void**)&r1);
        gvrt_dfree(c, (void**)&nn);
        gvrt_dfree(c, (void**)&keep);
        gvrt_dfree(c, (void**)&pos);
        gvrt_dfree(c, (void**)&counter);
        gvrt_dfree(c, &tmp);
    };
#define TRY(x)                      \
    do {                            \
        if ((s = (x)) != GVRT_OK) { \
            cleanup();              \
            return s;               \
        }                           \
    } while (0)
#define TRYH(x, what)                           \
    do {                                        \
        hipError_t _e = (x);                    \
        if (_e != hipSuccess) {                 \
            cleanup();                          \
            return gvrt_hip_check(c, _e, what); \
        }                                       \
    } while (0)
    TRY(gvrt_dalloc(c, (void**)&b0, 24ull * m));
    TRY(gvrt_dalloc(c, (void**)&b1, 24ull * m));
    TRY(gvrt_dalloc(c, (void**)&r0, 4ull * m));
    TRY(gvrt_dalloc(c, (void**)&r1, 4ull * m));
    TRY(gvrt_dalloc(c, (void**)&nn, 4ull * m));
    TRY(gvrt_dalloc(c, (void**)&keep, 4ull * (m + 1)));
    TRY(gvrt_dalloc(c, (void**)&pos, 4ull * (m + 1)));
    TRY(gvrt_dalloc(c, (void**)&counter, 4));
    TRYH(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, keep, pos, (int)(m + 1), c->stream), "scan size");
    TRY(gvrt_dalloc(c, &tmp, tmp_bytes ? tmp_bytes : 16));
    TRYH(hipMemsetAsync(counter, 0, 4, c->stream), "memset");
    hipLaunchKernelGGL(k_ploc_init, dim3((m + 255) / 256), dim3(256), 0, c->stream, m, leaf_boxes, b0, r0);
    uint32_t n = m, it = 0;
    while (n > 1) {
        const unsigned g = (n + 255) / 256;
        hipLaunchKernelGGL(k_ploc_nn, dim3((n + PLOC_B - 1) / PLOC_B), dim3(PLOC_B), 0, c->stream, n, b0, nn);
        hipLaunchKernelGGL(k_ploc_merge, dim3(g), dim3(256), 0, c->stream, n, nn, b0, r0, bin, counter, leaf_parent,
                           node_parent, keep);
        TRYH(hipMemsetAsync(keep + n, 0, 4, c->stream), "memset");
        size_t tb = tmp_bytes;
        TRYH(hipcub::DeviceScan::ExclusiveSum(tmp, tb, keep, pos, (int)(n + 1), c->stream), "scan");
        hipLaunchKernelGGL(k_ploc_compact, dim3(g), dim3(256), 0, c->stream, n, keep, pos, b0, r0, b1, r1);
        TRYH(hipGetLastError(), "ploc");
        uint32_t nn_host = 0;
        TRYH(hipMemcpyAsync(&nn_host, pos + n, 4, hipMemcpyDeviceToHost, c->stream), "n");
        TRYH(hipStreamSynchronize(c->stream), "sync");
        if (nn_host == 0 || nn_host >= n) {  // every iteration merges at least the globally closest pair
            cleanup();
            return gvrt_fail(c, GVRT_ERR_STATE, "PLOC made no progress");
        }
        n = nn_host;
        std::swap(b0, b1);
        std::swap(r0, r1);
        ++it;
    }
    int32_t rt = 0;
    TRYH(hipMemcpyAsync(&rt, r0, 4, hipMemcpyDeviceToHost, c->stream), "root");
    TRYH(hipStreamSynchronize(c->stream), "sync");
    const int32_t minus1 = -1;
    TRYH(hipMemcpyAsync(node_parent + rt, &minus1, 4, hipMemcpyHostToDevice, c->stream), "root parent");
    TRYH(hipStreamSynchronize(c->stream), "sync");
    *root = rt;
    *iterations = it;
    cleanup();
#undef TRY
#undef TRYH
    return GVRT_OK;
}
