// gvrt_nodes.hip — the compact 64-B node format of the FAST render kernel (gvrt_device.h Bvh4C) and the leaf
// renumbering it needs.
//
// The reference traverses the driver's BLAS built with PREFER_FAST_TRACE (VulkanFullRT.cpp:575-674, :621); here the
// 4-wide tree of any builder (gvrt_lbvh.hip, gvrt_sah.hip) is re-encoded at half the size: a visit is one
// s_load_dwordx16 into 16 SGPRs instead of two into 32.
//
// Leaf renumbering: in a node's slot order its leaf children are interleaved with subtrees, so their leaf ids are not
// consecutive.  After every build the leaves are renumbered in breadth-first node order (node i's leaf children get
// ids base[i], base[i] + 1, ... in slot order, base = exclusive scan of the per-node leaf counts); the per-leaf arrays
// (records, SH, leaf -> compaction index, split pieces) and the binary tree's leaf links follow the permutation.  A
// leaf id names the same particle (or piece) everywhere, and the k-buffer orders crossings by t, never by id, so no
// image changes.
#include <hipcub/hipcub.hpp>

#include "gvrt_internal.h"

using namespace gvrt;

namespace {

__device__ inline uint32_t leaf_slots(const Bvh4Node& n) {
    const uint32_t valid = n.nchild >= 32 ? 0xFFFFFFFFu : ((1u << n.nchild) - 1u);
    return valid & ~n.pad[1] & ((1u << BVH_W) - 1u);
}

__global__ __launch_bounds__(256) void k_leaf_slot_count(uint64_t n, const Bvh4Node* __restrict__ nodes,
                                                         uint32_t* __restrict__ cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    cnt[i] = i < n ? (uint32_t)__popc(leaf_slots(nodes[i])) : 0u;  // cnt[n] = 0: the scan's last entry is the total
}

__global__ __launch_bounds__(256) void k_leaf_renumber(uint64_t n, Bvh4Node* __restrict__ nodes,
                                                       const uint32_t* __restrict__ base, uint64_t m,
                                                       uint32_t* __restrict__ new2old, uint32_t* __restrict__ old2new,
                                                       uint32_t* __restrict__ fail) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Bvh4Node nd = nodes[i];
    const uint32_t ls = leaf_slots(nd);
    uint32_t r = base[i];
    for (int k = 0; k < BVH_W; ++k) {
        if (!((ls >> k) & 1u)) continue;
        const uint32_t old = (uint32_t)~nd.child[k];
        if (nd.child[k] >= 0 || old >= m || r >= m) {
            atomicOr(fail, 1u);
            return;
        }
        new2old[r] = old;
        old2new[old] = r;
        nodes[i].child[k] = ~(int32_t)r;
        ++r;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_gather(uint64_t n, const uint32_t* __restrict__ idx, uint32_t per,
                                                const T* __restrict__ src, T* __restrict__ dst) {
    // dst element i of each leaf l = i / per: src element idx[l] * per + i % per
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * per) return;
    const uint64_t l = i / per, j = i % per;
    dst[i] = src[(uint64_t)idx[l] * per + j];
}

__global__ __launch_bounds__(256) void k_remap_binary(uint64_t ni, BvhNode* __restrict__ bin,
                                                      const uint32_t* __restrict__ old2new) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ni) return;
    if (bin[i].c0 < 0) bin[i].c0 = ~(int32_t)old2new[(uint32_t)~bin[i].c0];
    if (bin[i].c1 < 0) bin[i].c1 = ~(int32_t)old2new[(uint32_t)~bin[i].c1];
}

// ---- f16 with directed rounding (the conversion runs once per build; double keeps lo - O exact)
__device__ inline double h2d(uint16_t h) { return (double)__builtin_bit_cast(_Float16, h); }
__device__ inline uint16_t h_next_up(uint16_t h) {
    if (h == 0x8000u) return 0x0001u;                  // -0 -> smallest positive
    return (h & 0x8000u) ? (uint16_t)(h - 1u) : (uint16_t)(h + 1u);
}
__device__ inline uint16_t h_next_down(uint16_t h) {
    if (h == 0x0000u) return 0x8001u;
    return (h & 0x8000u) ? (uint16_t)(h + 1u) : (uint16_t)(h - 1u);
}
__device__ inline uint16_t h_round(double x, bool up) {
    uint16_t h = __builtin_bit_cast(uint16_t, (_Float16)(float)x);
    if (up) {
        while (h2d(h) < x) h = h_next_up(h);
    } else {
        while (h2d(h) > x) h = h_next_down(h);
    }
    return h;
}
constexpr double F16_MAX = 65504.0;
constexpr double F16_MIN_NORMAL = 6.103515625e-05;  // 2^-14: offsets are kept out of the subnormal range

__global__ __launch_bounds__(256) void k_compact_nodes(uint64_t n, const Bvh4Node* __restrict__ src,
                                                       Bvh4C* __restrict__ dst, uint32_t* __restrict__ fail) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Bvh4Node nd = src[i];
    const uint32_t valid = (1u << min(nd.nchild, (uint32_t)BVH_W)) - 1u;
    const uint32_t inner = nd.pad[1] & valid, leafm = valid & ~inner;
    bool live[BVH_W];
    for (int k = 0; k < BVH_W; ++k) live[k] = ((valid >> k) & 1u) && !(nd.box[k][0] > 1e37f);  // empty / dropped
    // origin: per axis the largest f16 <= every live child's lo
    uint16_t oh[3];
    double od[3];
    bool bad = false;
    for (int a = 0; a < 3; ++a) {
        double mn = INFINITY;
        for (int k = 0; k < BVH_W; ++k)
            if (live[k]) mn = fmin(mn, (double)nd.box[k][2 * a]);
        if (mn == INFINITY) mn = 0.0;
        bad = bad || !(mn >= -F16_MAX && mn <= F16_MAX);
        oh[a] = bad ? 0 : h_round(mn, false);
        od[a] = h2d(oh[a]);
    }
    uint32_t plane[BVH_W][3];
    for (int k = 0; k < BVH_W; ++k)
        for (int a = 0; a < 3; ++a) {
            if (!live[k]) {
                plane[k][a] = F16_INF2;
                continue;
            }
            // offsets rounded outward by one more f16 step than the rounding needs (the margin of the render kernel's
            // FMA-form plane evaluation); lo - O >= 0 by construction
            const double lo = (double)nd.box[k][2 * a] - od[a], hi = (double)nd.box[k][2 * a + 1] - od[a];
            bad = bad || !(lo >= 0.0) || !(hi >= lo) || hi > 0.5 * F16_MAX;
            uint16_t hl = h_round(lo, false), hh = h_round(hi, true);
            hl = hl == 0 ? hl : h_next_down(hl);
            hh = h_next_up(hh);
            if (h2d(hl) < F16_MIN_NORMAL) hl = 0;                     // no subnormal offsets
            if (h2d(hh) < F16_MIN_NORMAL) hh = 0x0400u;                // 2^-14
            plane[k][a] = (uint32_t)hl | ((uint32_t)hh << 16);
        }
    // links: inner children consecutive node ids, leaf children consecutive leaf ids (gvrt_renumber_leaves)
    uint32_t ibase = 0, lbase = 0, ri = 0, rl = 0;
    for (int k = 0; k < BVH_W; ++k) {
        if ((inner >> k) & 1u) {
            if (ri == 0) ibase = (uint32_t)nd.child[k];
            bad = bad || nd.child[k] < 0 || (uint32_t)nd.child[k] != ibase + ri;
            ++ri;
        } else if ((leafm >> k) & 1u) {
            if (rl == 0) lbase = (uint32_t)~nd.child[k];
            bad = bad || nd.child[k] >= 0 || (uint32_t)~nd.child[k] != lbase + rl;
            ++rl;
        }
    }
    if (inner == 0) ibase = nd.pad[2];  // all-leaf node: the acceptance widening D (0 in proxy-box nodes)
    if (bad) atomicOr(fail, 1u);
    const uint32_t meta = inner | (leafm << 4) | ((nd.pad[0] & 3u) << 8);
    // copy 0: (lo, hi); copy 1 + o: octant o, (hi, lo) on every axis whose bit is set in o (rays along -axis)
    for (uint32_t cpy = 0; cpy < 9; ++cpy) {
        Bvh4C c;
        const uint32_t o = cpy == 0 ? 0u : cpy - 1;
        for (int k = 0; k < BVH_W; ++k)
            for (int a = 0; a < 3; ++a) {
                const uint32_t w = plane[k][a];
                c.plane[3 * k + a] = ((o >> a) & 1u) ? ((w >> 16) | (w << 16)) : w;
            }
        c.oxy = (uint32_t)oh[0] | ((uint32_t)oh[1] << 16);
        c.ozm = (uint32_t)oh[2] | (meta << 16);
        c.ibase = ibase;
        c.lbase = lbase;
        dst[cpy * n + i] = c;
    }
}

}  // namespace

gvrt_status gvrt_renumber_leaves(gvrt_context* c) {
    const uint64_t n = c->n_nodes4, m = c->n_leaves;
    if (!n || !m || !c->d_nodes4) return GVRT_OK;
    if (m >= (1ull << 31)) return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "too many leaves to renumber");
    uint32_t *cnt = nullptr, *base = nullptr, *n2o = nullptr, *o2n = nullptr, *fail = nullptr;
    void* tmp = nullptr;
    void* nw = nullptr;
    gvrt_status s = GVRT_OK;
    auto cleanup = [&]() {
        gvrt_dfree(c, (void**)&cnt);
        gvrt_dfree(c, (void**)&base);
        gvrt_dfree(c, (void**)&n2o);
        gvrt_dfree(c, (void**)&o2n);
        gvrt_dfree(c, (void**)&fail);
        gvrt_dfree(c, &tmp);
        gvrt_dfree(c, &nw);
    };
#define TRY(x)                      \
    do {                            \
        if ((s = (x)) != GVRT_OK) { \
            cleanup();              \
            return s;               \
        }                           \
    } while (0)
#define TRYH(x, what)                         \
    do {                                      \
        hipError_t _e = (x);                  \
        if (_e != hipSuccess) {               \
            cleanup();                        \
            return gvrt_hip_check(c, _e, what); \
        }                                     \
    } while (0)
    TRY(gvrt_dalloc(c, (void**)&cnt, 4 * (n + 1)));
    TRY(gvrt_dalloc(c, (void**)&base, 4 * (n + 1)));
    TRY(gvrt_dalloc(c, (void**)&n2o, 4 * m));
    TRY(gvrt_dalloc(c, (void**)&o2n, 4 * m));
    TRY(gvrt_dalloc(c, (void**)&fail, 4));
    TRYH(hipMemsetAsync(fail, 0, 4, c->stream), "memset");
    hipLaunchKernelGGL(k_leaf_slot_count, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, c->stream, n,
                       c->d_nodes4, cnt);
    size_t tb = 0;
    TRYH(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, base, (int)(n + 1), c->stream), "scan size");
    TRY(gvrt_dalloc(c, &tmp, tb ? tb : 16));
    TRYH(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, base, (int)(n + 1), c->stream), "scan");
    uint32_t total = 0;
    TRYH(hipMemcpyAsync(&total, base + n, 4, hipMemcpyDeviceToHost, c->stream), "total");
    TRYH(hipStreamSynchronize(c->stream), "sync");
    if (total != m) {
        cleanup();
        return gvrt_fail(c, GVRT_ERR_HIP, "leaf renumbering: the 4-wide tree does not hold every leaf once");
    }
    hipLaunchKernelGGL(k_leaf_renumber, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, n, c->d_nodes4,
                       base, m, n2o, o2n, fail);
    uint32_t hf = 0;
    TRYH(hipMemcpyAsync(&hf, fail, 4, hipMemcpyDeviceToHost, c->stream), "fail");
    TRYH(hipStreamSynchronize(c->stream), "sync");
    if (hf) {
        cleanup();
        return gvrt_fail(c, GVRT_ERR_HIP, "leaf renumbering: a leaf link out of range");
    }
    // per-leaf arrays through the permutation (new leaf l reads old leaf n2o[l])
    auto permute = [&](void** arr, uint64_t bytes_per_leaf) -> gvrt_status {
        if (!*arr) return GVRT_OK;
        gvrt_status st = gvrt_dalloc(c, &nw, bytes_per_leaf * m);
        if (st) return st;
        const uint64_t per = bytes_per_leaf / 16 ? bytes_per_leaf / 16 : 1;
        const uint64_t tot = m * per;
        if (bytes_per_leaf % 16 == 0)
            hipLaunchKernelGGL(k_gather<uint4>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, c->stream, m, n2o,
                               (uint32_t)per, (const uint4*)*arr, (uint4*)nw);
        else
            hipLaunchKernelGGL(k_gather<uint32_t>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, c->stream, m, n2o,
                               1u, (const uint32_t*)*arr, (uint32_t*)nw);
        gvrt_dfree(c, arr);
        *arr = nw;
        nw = nullptr;
        return GVRT_OK;
    };
    TRY(permute((void**)&c->d_recs, sizeof(RenderRec)));
    TRY(permute((void**)&c->d_sh, 192));
    TRY(permute((void**)&c->d_leaf_src, 4));
    TRY(permute((void**)&c->d_leaf_aux, 16));
    if (c->d_nodes && m > 1)
        hipLaunchKernelGGL(k_remap_binary, dim3((unsigned)((m - 1 + 255) / 256)), dim3(256), 0, c->stream, m - 1,
                           c->d_nodes, o2n);
    TRYH(hipGetLastError(), "renumber");
    TRYH(hipStreamSynchronize(c->stream), "sync");
    cleanup();
#undef TRY
#undef TRYH
    return GVRT_OK;
}

gvrt_status gvrt_launch_compact_nodes(gvrt_context* c, const Bvh4Node* src, Bvh4C** dst) {
    // (an existing array has this build's size: the acceptance refit rewrites it in stream order, after its readers)
    const uint64_t n = c->n_nodes4;
    if (!n || !src || !c->opt[GVRT_OPT_COMPACT_NODES]) {
        gvrt_dfree(c, (void**)dst);
        return GVRT_OK;
    }
    // render-kernel addressing: 32-bit byte offsets within a copy
    if (n >= (1ull << 26)) return GVRT_OK;
    if (!*dst && !gvrt_dalloc_optional(c, (void**)dst, 9 * n * sizeof(Bvh4C))) return GVRT_OK;
    uint32_t* fail = nullptr;
    gvrt_status s = gvrt_dalloc(c, (void**)&fail, 4);
    if (s) {
        gvrt_dfree(c, (void**)dst);
        return s;
    }
    uint32_t hf = 0;
    hipError_t e = hipMemsetAsync(fail, 0, 4, c->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_compact_nodes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, n, src, *dst,
                           fail);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&hf, fail, 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    gvrt_dfree(c, (void**)&fail);
    if (e != hipSuccess) {
        gvrt_dfree(c, (void**)dst);
        return gvrt_hip_check(c, e, "compact nodes");
    }
    if (hf) gvrt_dfree(c, (void**)dst);  // a box beyond the f16 range (or links not consecutive): 128-B nodes
    return GVRT_OK;
}
