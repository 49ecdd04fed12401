// gvrt_wide.hip — 64-wide node copies for the tile-beam traversal (handle option GVRT_OPT_WIDE_NODES; experiment of
// VERDICT r03 #3).
//
// The packet traversal of the 4-wide tree spends ~40 % of a wave's time on a chain of ~170 dependent scalar node
// fetches per wave.  Here a wide node is the 3-level subtree below a 4-wide node: its up-to-64 descendants at
// relative depth 3 (inner) or above (leaves) become its children, one per lane.  A wave then tests all children of a
// node at once, lane-parallel, against the interval bound of its 64 rays (the ranges of 1/d over the tile, the wave's
// t range), and walks the hit children in visiting order: inner ones one level down, leaves through the exact
// per-lane leaf test of k_render.  The tree is ~4x shallower and a node visit is one coalesced vector fetch.
//
// Children are stored in the visiting order of the packet kernel (each 4-wide node's children in split order,
// reversed when the ray runs along -axis on the node's split axis), so there are 8 copies, one per ray-direction
// octant; a wave reads the copy of its first active ray.  Leaf children carry their acceptance box and D (the
// largest distance along the ray between an admitted crossing and the box, k_accept_leaf) when the handle's FAST
// launches use acceptance boxes: per child, since each lane tests its own child.
#include <algorithm>
#include <cstring>
#include <vector>

#include "gvrt_internal.h"

using namespace gvrt;

namespace {

// one leaf's acceptance box and D for the launch's thresholds (the per-leaf form of k_accept_leaf): out[8] = box
// [lx, hx, ly, hy, lz, hz], D, flag (0: proxy box kept, 1: acceptance box, 2: never accepted: drop)
__global__ __launch_bounds__(256) void k_leaf_accept(uint64_t m, const RenderRec* __restrict__ recs, float min_response,
                                                     float alpha_min, float kmin, uint32_t kopts, float kdeg,
                                                     float pad_abs, float* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const RenderRec r = recs[i];
    float* o = out + 8 * i;
    const float rho = r.density;
    o[7] = 0.0f;
    if (rho != rho || !(rho > 0.0f)) return;  // NaN density is accepted everywhere; non-positive: keep the proxy
    const float mm = fmaxf(min_response, alpha_min / rho);
    if (!(rho > alpha_min) || !(mm < 1.0f) || !(alpha_min < 0.99f)) {
        o[7] = 2.0f;
        return;
    }
    constexpr float ICO_CIRCUM = 1.2584086f;
    const float re = powf(logf(mm) / KERNEL_S, 0.25f) * 1.01f;
    const float sx = 1.0f / r.isx, sy = 1.0f / r.isy, sz = 1.0f / r.isz;
    const float hx = re * sqrtf(r.c0x * r.c0x * sx * sx + r.c0y * r.c0y * sy * sy + r.c0z * r.c0z * sz * sz);
    const float hy = re * sqrtf(r.c1x * r.c1x * sx * sx + r.c1y * r.c1y * sy * sy + r.c1z * r.c1z * sz * sz);
    const float hz = re * sqrtf(r.c2x * r.c2x * sx * sx + r.c2y * r.c2y * sy * sy + r.c2z * r.c2z * sz * sz);
    const float c3[3] = {r.px, r.py, r.pz}, h3[3] = {hx, hy, hz};
    for (int ax = 0; ax < 3; ++ax) {
        const float lo = c3[ax] - h3[ax] * 1.0001f, hi = c3[ax] + h3[ax] * 1.0001f;
        const float pad = 1e-5f * (hi - lo) + 1e-6f * fabsf(c3[ax]) + pad_abs + 1e-30f;
        o[2 * ax] = lo - pad;
        o[2 * ax + 1] = hi + pad;
    }
    const float rc = ICO_CIRCUM * 1.001f * kernel_scale(rho, kmin, kopts, kdeg);
    const float gap = sqrtf(fmaxf(rc * rc - re * re, 0.0f));
    o[6] = gap * fmaxf(sx, fmaxf(sy, sz)) * 1.01f + 4.0f * pad_abs;
    o[7] = 1.0f;
}

}  // namespace

gvrt_status gvrt_build_wide(gvrt_context* c, bool accept, float min_response, float alpha_min) {
    c->wide_ok = false;
    const uint64_t n4 = c->n_nodes4;
    if (!n4 || !c->d_nodes4 || c->split_cells) return GVRT_OK;
    std::vector<Bvh4Node> nd(n4);
    GVRT_HIP(c, hipMemcpyAsync(nd.data(), c->d_nodes4, n4 * sizeof(Bvh4Node), hipMemcpyDeviceToHost, c->stream));
    std::vector<float> lacc;
    if (accept) {
        float* d = nullptr;
        gvrt_status s;
        if ((s = gvrt_dalloc(c, (void**)&d, 32 * c->n_leaves))) return s;
        hipLaunchKernelGGL(k_leaf_accept, dim3((unsigned)((c->n_leaves + 255) / 256)), dim3(256), 0, c->stream,
                           c->n_leaves, c->d_recs, min_response, alpha_min, c->enc.kernel_min_response, c->enc.opts,
                           c->enc.degree, c->box_pad_abs, d);
        lacc.resize(8 * c->n_leaves);
        const hipError_t e = hipMemcpyAsync(lacc.data(), d, 32 * c->n_leaves, hipMemcpyDeviceToHost, c->stream);
        const hipError_t e2 = hipStreamSynchronize(c->stream);
        gvrt_dfree(c, (void**)&d);
        GVRT_HIP(c, e);
        GVRT_HIP(c, e2);
    } else {
        GVRT_HIP(c, hipStreamSynchronize(c->stream));
    }
    // wide roots: the 4-wide root and every 4-wide node three levels below a wide root
    std::vector<int32_t> wid(n4, -1);
    std::vector<int32_t> roots{0};
    wid[0] = 0;
    std::vector<uint32_t> depth{0};  // wide depth of each root (the traversal's level count bound)
    uint32_t maxdepth = 0;
    std::vector<WideChild> out;  // [octant][node][64]
    // first pass: collect the roots breadth-first (octant-independent)
    for (size_t q = 0; q < roots.size(); ++q) {
        std::vector<std::pair<int32_t, int>> st{{roots[q], 1}};
        while (!st.empty()) {
            auto [x, dep] = st.back();
            st.pop_back();
            const Bvh4Node& n = nd[x];
            for (uint32_t k = 0; k < BVH_W; ++k) {
                if (n.box[k][0] > 1e37f || n.child[k] < 0) continue;
                const int32_t ch = n.child[k];
                if (dep == 3) {
                    if (wid[ch] < 0) {
                        wid[ch] = (int32_t)roots.size();
                        roots.push_back(ch);
                        depth.push_back(depth[q] + 1);
                        maxdepth = std::max(maxdepth, depth[q] + 1);
                    }
                } else {
                    st.push_back({ch, dep + 1});
                }
            }
        }
    }
    if (maxdepth + 1 > WIDE_LEVELS) return GVRT_OK;  // deeper than the kernel's per-level LDS buffers: not used
    const uint64_t nw = roots.size();
    out.assign(8 * nw * WIDE_W, WideChild{});
    for (auto& w : out) {
        w.n[0] = w.n[1] = w.n[2] = EMPTY_BOX;
        w.f[0] = w.f[1] = w.f[2] = -EMPTY_BOX;
        w.link = WIDE_EMPTY;
        w.d = 0.0f;
    }
    for (uint32_t o = 0; o < 8; ++o) {
        for (uint64_t q = 0; q < nw; ++q) {
            WideChild* dst = &out[((uint64_t)o * nw + q) * WIDE_W];
            int cnt = 0;
            // depth-first expansion in the packet kernel's visiting order for octant o
            auto emit = [&](const Bvh4Node& n, uint32_t k, int32_t link) {
                WideChild& w = dst[cnt++];
                float b[6];
                for (int j = 0; j < 6; ++j) b[j] = n.box[k][j];
                if (link < 0 && accept) {
                    const float* la = &lacc[8 * (uint64_t)(~link)];
                    if (la[7] == 2.0f) {  // never accepted: dropped
                        --cnt;
                        return;
                    }
                    if (la[7] == 1.0f) {
                        for (int j = 0; j < 6; ++j) b[j] = la[j];
                        w.d = la[6];
                    }
                }
                for (int ax = 0; ax < 3; ++ax) {
                    const bool neg = (o >> ax) & 1u;
                    w.n[ax] = neg ? b[2 * ax + 1] : b[2 * ax];
                    w.f[ax] = neg ? b[2 * ax] : b[2 * ax + 1];
                }
                w.link = link;
            };
            struct Frame {
                int32_t x;
                int dep;
            };
            // recursive expansion as an explicit ordered walk
            std::vector<Frame> st;
            auto expand = [&](auto&& self, int32_t x, int dep) -> void {
                const Bvh4Node& n = nd[x];
                const bool rev = (o >> n.pad[0]) & 1u;
                for (uint32_t kk = 0; kk < BVH_W; ++kk) {
                    const uint32_t k = rev ? BVH_W - 1 - kk : kk;
                    if (n.box[k][0] > 1e37f) continue;
                    const int32_t ch = n.child[k];
                    if (ch < 0) emit(n, k, ch);
                    else if (dep == 3) emit(n, k, wid[ch]);
                    else self(self, ch, dep + 1);
                }
            };
            expand(expand, roots[q], 1);
        }
    }
    if (!c->d_wide || c->wide_cap < out.size()) {
        gvrt_dfree(c, (void**)&c->d_wide);
        c->wide_cap = 0;
        if (!gvrt_dalloc_optional(c, (void**)&c->d_wide, out.size() * sizeof(WideChild))) return GVRT_OK;
        c->wide_cap = out.size();
    }
    GVRT_HIP(c, hipMemcpyAsync(c->d_wide, out.data(), out.size() * sizeof(WideChild), hipMemcpyHostToDevice, c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    c->n_wide = nw;
    c->wide_depth = maxdepth + 1;
    c->wide_accept = accept;
    c->wide_key[0] = min_response;
    c->wide_key[1] = alpha_min;
    c->wide_ok = true;
    return GVRT_OK;
}
