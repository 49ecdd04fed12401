// gvrt_sah.hip — the static-scene quality build on gfx950: binned-SAH binary BVH + surface-area-optimal
// 4-wide collapse, both on the device (gvrt_accel_params.builder = 2, collapse = 1).
//
// The counterpart of the reference's BLAS built once with PREFER_FAST_TRACE
// (projects/VulkanFullRT/VulkanFullRT.cpp:575-674, flag at :621): the driver builds it on the GPU, and
// so does this file.  The algorithm is host_sah_build / host_dp_collapse of gvrt_lbvh.hip (builder = 3,
// kept as the checker) restated for the device with the same arithmetic, so both produce the same
// tree node for node (tests/test_gpu_sah.py):
//   * per range [b, e) of Morton-ordered leaves: centroid bounds, 32 bins per axis (bin =
//     min(31, (int)((c - lo) * (32 / extent)))), split of least SA(L)·n(L) + SA(R)·n(R) (first in
//     axis-major, bin order on ties), stable partition; equal centroids halve the range;
//   * node ids by range: [b, e) is node id, its left child id + 1, its right child id + |left|;
//   * DP over the binary tree (Ylitie et al. 2017) and the breadth-first 4-wide layout.
// Float min / max are exact in any order, and every area / cost is evaluated with contraction off in
// the host's operation order, so the decisions agree bit for bit.
//
// Mapping to CDNA4.  Level-synchronous, top down:
//   * ranges above LARGE proxies: chunks of CHUNK proxies, one 256-thread workgroup each; centroid
//     bounds and bins reduced in LDS (ordered-uint min / max atomics), merged into the range's global
//     bins with one atomic per bin value; one wave evaluates the 96 candidate splits (prefix / suffix
//     unions by shuffles across 32 lanes); a two-pass stable partition (per-chunk left counts, then
//     ballot ranks) writes the other index buffer;
//   * ranges of 2..LARGE proxies: one wave per range, everything in one launch per level (bins in the
//     wave's LDS, the same split evaluation, ballot-rank stable partition), queued ranges in device
//     arrays, no host round trip inside a level.
// Collapse: one thread per leaf climbs to the root with an arrival counter per node (the second child
// to arrive evaluates the node's DP row), then one launch pair + one scan per 4-wide level lays the
// nodes out breadth-first.
#include <hipcub/hipcub.hpp>

#include <vector>

#include "gvrt_internal.h"

using namespace gvrt;

namespace {

constexpr int NB = 32;              // bins per axis (host_sah_build's default GVRT_SAH_BINS)
constexpr uint32_t LARGE = 4096;    // ranges above this go through the chunked multi-workgroup path
constexpr uint32_t TINY = 64;      // ranges of at most this many proxies: the whole subtree in one wave
constexpr uint32_t CHUNK = 4096;    // proxies per workgroup in the chunked path
constexpr int SMALL_WAVES = 4;      // waves per workgroup of the per-range kernel

__device__ inline uint32_t f2o(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float o2f(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u); }
constexpr uint32_t ORD_MIN_ID = 0xFFFFFFFFu;  // identity of an ordered-uint min (above f2o(+inf))
constexpr uint32_t ORD_MAX_ID = 0u;

// Box::area of host_sah_build (empty box: 0)
__device__ inline float sah_area(const float* lo, const float* hi) {
#pragma clang fp contract(off)
    if (!(hi[0] >= lo[0])) return 0.0f;
    const float ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
    return ex * ey + ey * ez + ez * ex;
}
__device__ inline float sah_cost(float al, uint32_t nl, float ar, uint32_t nr) {
#pragma clang fp contract(off)
    return al * (float)nl + ar * (float)nr;
}
// bin of centroid coordinate c on an axis with lower bound lo and scale sc = NB / extent
__device__ inline int sah_bin(float c, float lo, float sc) {
    const int k = (int)((c - lo) * sc);
    return k < NB - 1 ? k : NB - 1;
}
__device__ inline float centroid(const float* __restrict__ boxes, uint32_t p, int a) {
    return 0.5f * (boxes[6ull * p + a] + boxes[6ull * p + 3 + a]);
}

struct Bins {  // ordered-uint bounds per (axis, bin), counts
    uint32_t lo[3][NB][3];
    uint32_t hi[3][NB][3];
    uint32_t n[3][NB];
};
constexpr int BIN_WORDS = sizeof(Bins) / 4;  // 672

struct LgRange {  // chunked path, per range: centroid bounds then bins
    uint32_t cb[6];
    uint32_t pad[2];
    Bins bins;
};

struct Task {
    uint32_t b, e, node, db;  // db = depth << 1 | index buffer holding the range
};

struct Split {
    int axis, k;  // k = -1: no split (halve)
    uint32_t nl;
    float lb[6], rb[6];  // lo xyz, hi xyz
};

// Per-axis scale, or 0 when the axis cannot be binned (host: ext <= 0 or NB / ext not finite)
__device__ inline void axis_scales(const float* cl, const float* ch, float* sc) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float ext = ch[a] - cl[a];
        const float s = ext > 0.0f ? (float)NB / ext : 0.0f;
        sc[a] = (ext > 0.0f && s < INFINITY) ? s : 0.0f;
    }
}

// Split evaluation by one wave over a range's bins (any address space).  Lane l handles (axis l >> 5,
// bin l & 31) in the first pass and (axis 2, bin l) in the second; the left side of split k is the
// inclusive prefix union of bins 0..k, the right side the suffix union of k + 1..31.  Chosen: the least
// cost, the first in (axis, bin) order on ties — host_sah_build's strict `cost < best_cost` sweep.
template <typename BinsT>
__device__ inline Split sah_eval(const BinsT& B, const float* sc) {
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    Split s;
    s.axis = -1;
    s.k = -1;
    s.nl = 0;
    float best = INFINITY;
    for (int pass = 0; pass < 2; ++pass) {
        const int a = pass == 0 ? (lane >> 5) : 2;
        const int k = lane & 31;
        const bool on = (pass == 0 || lane < 32) && sc[a] > 0.0f;
        float lo[3], hi[3];
        uint32_t n = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            lo[j] = on ? o2f(B.lo[a][k][j]) : INFINITY;
            hi[j] = on ? o2f(B.hi[a][k][j]) : -INFINITY;
        }
        if (on) n = B.n[a][k];
        // inclusive prefix (left) and suffix unions within the 32-lane half
        float pl[3], ph[3], sl[3], sh[3];
        uint32_t pn = n, sn = n;
#pragma unroll
        for (int j = 0; j < 3; ++j) pl[j] = sl[j] = lo[j], ph[j] = sh[j] = hi[j];
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) {
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const float ul = __shfl_up(pl[j], off, 32), uh = __shfl_up(ph[j], off, 32);
                const float dl = __shfl_down(sl[j], off, 32), dh = __shfl_down(sh[j], off, 32);
                if (k >= off) pl[j] = fminf(pl[j], ul), ph[j] = fmaxf(ph[j], uh);
                if (k + off < 32) sl[j] = fminf(sl[j], dl), sh[j] = fmaxf(sh[j], dh);
            }
            const uint32_t un = __shfl_up(pn, off, 32), dn = __shfl_down(sn, off, 32);
            if (k >= off) pn += un;
            if (k + off < 32) sn += dn;
        }
        float rl[3], rh[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) rl[j] = __shfl_down(sl[j], 1, 32), rh[j] = __shfl_down(sh[j], 1, 32);
        const uint32_t rn = __shfl_down(sn, 1, 32);
        float cost = INFINITY;
        const bool cand0 = on && k < NB - 1 && pn > 0 && rn > 0;
        if (cand0) cost = sah_cost(sah_area(pl, ph), pn, sah_area(rl, rh), rn);
        const bool cand = cand0 && cost < INFINITY;
        // wave minimum of the candidates' costs, then the first lane holding it
        float mc = cand ? cost : INFINITY;
        for (int off = 32; off > 0; off >>= 1) mc = fminf(mc, __shfl_xor(mc, off));
        const uint64_t bal = __ballot(cand && cost == mc);
        if (bal && mc < best) {  // a later pass wins only with a strictly lower cost
            const int src = __builtin_ctzll(bal);
            best = mc;
            s.axis = pass == 0 ? (src >> 5) : 2;
            s.k = src & 31;
            s.nl = __shfl(pn, src);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                s.lb[j] = __shfl(pl[j], src);
                s.lb[3 + j] = __shfl(ph[j], src);
                s.rb[j] = __shfl(rl[j], src);
                s.rb[3 + j] = __shfl(rh[j], src);
            }
        }
    }
    return s;
}

// Box union of boxes[idx[i]] for i in [b, e) by one wave (the halving fallback), uniform result
__device__ inline void wave_box_union(const float* __restrict__ boxes, const uint32_t* __restrict__ idx, uint32_t b,
                                      uint32_t e, float* out) {
    const int lane = threadIdx.x & 63;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = b + lane; i < e; i += 64) {
        const uint32_t p = idx[i];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], boxes[6ull * p + a]);
            hi[a] = fmaxf(hi[a], boxes[6ull * p + 3 + a]);
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        for (int off = 32; off > 0; off >>= 1) {
            lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
            hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
        }
        out[a] = lo[a];
        out[3 + a] = hi[a];
    }
}

struct BuildOut {
    BvhNode* nodes;
    uint32_t* maxd;   // max binary leaf depth (root at depth 1)
    Task* mid_q;      // log of ranges of TINY+1..LARGE proxies (one segment per level), appended at *mid_n
    uint32_t* mid_n;
    Task* tiny_q;     // ranges of 2..TINY proxies (whole subtrees, one wave each)
    uint32_t* tiny_n;
    Task* large_q;    // ranges above LARGE (next level of the chunked path)
    uint32_t* large_n;
    uint32_t dmax;    // depth budget (SAH_DEPTH_MAX or gvrt_accel_params.depth_budget)
};

// Write node t.node with split s (mid = left end) and queue its children; lane 0 writes.  first_l /
// first_r: the first proxy of each side after the partition (the leaf of a one-proxy side).
__device__ inline void emit_node(const Task& t, const Split& s, uint32_t mid, uint32_t first_l, uint32_t first_r,
                                 const BuildOut& o) {
    const int lane = threadIdx.x & 63;
    if (lane != 0) return;
    const uint32_t depth = t.db >> 1, buf = t.db & 1u;
    const uint32_t L = mid - t.b;
    BvhNode nd;
    nd.l0x = s.lb[0], nd.l0y = s.lb[1], nd.l0z = s.lb[2];
    nd.h0x = s.lb[3], nd.h0y = s.lb[4], nd.h0z = s.lb[5];
    nd.l1x = s.rb[0], nd.l1y = s.rb[1], nd.l1z = s.rb[2];
    nd.h1x = s.rb[3], nd.h1y = s.rb[4], nd.h1z = s.rb[5];
    nd.pad0 = (uint32_t)(s.axis < 0 ? 0 : s.axis);
    nd.pad1 = 0;
    const uint32_t cdb = (depth + 1) << 1 | (buf ^ 1u);  // children's ranges live in the other buffer
    auto child = [&](uint32_t b, uint32_t e, uint32_t id, uint32_t leaf) -> int32_t {
        const uint32_t n = e - b;
        if (n == 1) {
            atomicMax(o.maxd, depth + 1);
            return ~(int32_t)leaf;
        }
        const Task ct{b, e, id, cdb};
        if (n > LARGE) o.large_q[atomicAdd(o.large_n, 1u)] = ct;
        else if (n > TINY) o.mid_q[atomicAdd(o.mid_n, 1u)] = ct;
        else o.tiny_q[atomicAdd(o.tiny_n, 1u)] = ct;
        return (int32_t)id;
    };
    nd.c0 = child(t.b, mid, t.node + 1, first_l);
    nd.c1 = child(mid, t.e, t.node + L, first_r);
    o.nodes[t.node] = nd;
}

// ---------------- ranges of TINY+1..LARGE proxies: one wave per range, one launch per level.  The level's
// ranges are log[se[0] .. se[1]); children of this size are appended at se[2] (the next segment).
__global__ __launch_bounds__(64 * SMALL_WAVES) void k_sah_mid(const Task* __restrict__ log, uint32_t* se,
                                                             uint32_t* __restrict__ idx0, uint32_t* __restrict__ idx1,
                                                             const float* __restrict__ boxes, BuildOut o) {
    __shared__ Bins sb[SMALL_WAVES];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    Bins& B = sb[w];
    const uint32_t q0 = se[0], q1 = se[1];
    o.mid_q = const_cast<Task*>(log);
    o.mid_n = se + 2;
    const uint32_t nw = gridDim.x * SMALL_WAVES;
    for (uint32_t ti = q0 + blockIdx.x * SMALL_WAVES + w; ti < q1; ti += nw) {
        const Task t = log[ti];
        const uint32_t* __restrict__ src = (t.db & 1u) ? idx1 : idx0;
        uint32_t* __restrict__ dst = (t.db & 1u) ? idx0 : idx1;
        const uint32_t n = t.e - t.b;
        // centroid bounds
        float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = t.b + lane; i < t.e; i += 64) {
            const uint32_t p = src[i];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float c = centroid(boxes, p, a);
                cl[a] = fminf(cl[a], c);
                ch[a] = fmaxf(ch[a], c);
            }
        }
#pragma unroll
        for (int a = 0; a < 3; ++a)
            for (int off = 32; off > 0; off >>= 1) {
                cl[a] = fminf(cl[a], __shfl_xor(cl[a], off));
                ch[a] = fmaxf(ch[a], __shfl_xor(ch[a], off));
            }
        float sc[3];
        axis_scales(cl, ch, sc);
        Split s;
        s.axis = -1;
        s.k = -1;
        if (sc[0] > 0.0f || sc[1] > 0.0f || sc[2] > 0.0f) {
            uint32_t* bw = reinterpret_cast<uint32_t*>(&B);
            for (int j = lane; j < BIN_WORDS; j += 64) bw[j] = j < 2 * 3 * NB * 3 ? (j < 3 * NB * 3 ? ORD_MIN_ID : ORD_MAX_ID) : 0u;
            for (uint32_t i = t.b + lane; i < t.e; i += 64) {
                const uint32_t p = src[i];
                float bl[3], bh[3];
#pragma unroll
                for (int a = 0; a < 3; ++a) bl[a] = boxes[6ull * p + a], bh[a] = boxes[6ull * p + 3 + a];
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    if (!(sc[a] > 0.0f)) continue;
                    const int k = sah_bin(0.5f * (bl[a] + bh[a]), cl[a], sc[a]);
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        atomicMin(&B.lo[a][k][j], f2o(bl[j]));
                        atomicMax(&B.hi[a][k][j], f2o(bh[j]));
                    }
                    atomicAdd(&B.n[a][k], 1u);
                }
            }
            s = sah_eval(B, sc);
            // depth budget (SAH_DEPTH_MAX): a split whose larger side could not finish in budget halves instead
            if (s.k >= 0 && !sah_split_in_budget(t.db >> 1, s.nl, n - s.nl, o.dmax)) s.axis = -1, s.k = -1;
        }
        uint32_t mid, first_l = 0xFFFFFFFFu, first_r = 0xFFFFFFFFu;
        if (s.k >= 0) {
            mid = t.b + s.nl;
            // stable partition: ballot ranks, left side from b, right side from mid
            uint32_t lb = t.b, rb = mid;
            const uint64_t below = (1ull << lane) - 1ull;
            for (uint32_t i0 = t.b; i0 < t.e; i0 += 64) {
                const uint32_t i = i0 + lane;
                const bool v = i < t.e;
                const uint32_t p = v ? src[i] : 0u;
                const bool left = v && sah_bin(centroid(boxes, p, s.axis), cl[s.axis], sc[s.axis]) <= s.k;
                const uint64_t bl = __ballot(left), br = __ballot(v && !left);
                if (left) dst[lb + __popcll(bl & below)] = p;
                else if (v) dst[rb + __popcll(br & below)] = p;
                if (first_l == 0xFFFFFFFFu && bl) first_l = __shfl(p, (int)__builtin_ctzll(bl));
                if (first_r == 0xFFFFFFFFu && br) first_r = __shfl(p, (int)__builtin_ctzll(br));
                lb += __popcll(bl);
                rb += __popcll(br);
            }
        } else {
            // every centroid equal, or the depth budget: halve the range, boxes of the halves
            mid = t.b + n / 2;
            for (uint32_t i = t.b + lane; i < t.e; i += 64) dst[i] = src[i];
            wave_box_union(boxes, src, t.b, mid, s.lb);
            wave_box_union(boxes, src, mid, t.e, s.rb);
            first_l = src[t.b];
            first_r = src[mid];
        }
        emit_node(t, s, mid, first_l, first_r, o);
    }
}

// host_dp_collapse's DP row of a node from its children's rows (leaves: 0) and its union-box area
__device__ inline float4 dp_row(float area, const float* f0, const float* f1) {
#pragma clang fp contract(off)
    float best4 = INFINITY;
    for (int j = 1; j < 4; ++j) best4 = fminf(best4, f0[j - 1] + f1[3 - j]);
    float r[4];
    r[0] = area + best4;
    for (int k = 2; k <= 4; ++k) {
        float b = r[k - 2];
        for (int j = 1; j < k; ++j) b = fminf(b, f0[j - 1] + f1[k - j - 1]);
        r[k - 1] = b;
    }
    return make_float4(r[0], r[1], r[2], r[3]);
}
// host_area of the union of a binary node's two child boxes
__device__ inline float union_area(const float* lb, const float* rb) {
#pragma clang fp contract(off)
    const float ex = fmaxf(lb[3], rb[3]) - fminf(lb[0], rb[0]);
    const float ey = fmaxf(lb[4], rb[4]) - fminf(lb[1], rb[1]);
    const float ez = fmaxf(lb[5], rb[5]) - fminf(lb[2], rb[2]);
    return ex * ey + ey * ez + ez * ex;
}

// ---------------- ranges of 2..TINY proxies: the whole subtree in one wave (lane i holds the range's i-th
// proxy: index and box in registers), splits taken depth first from a small LDS stack, the data moved by
// ds_permute after each partition; then the subtree's DP rows bottom-up (reverse pre-order).
__global__ __launch_bounds__(64 * SMALL_WAVES) void k_sah_tiny(const Task* __restrict__ q, const uint32_t* __restrict__ qn,
                                                              const uint32_t* __restrict__ idx0, const uint32_t* __restrict__ idx1,
                                                              const float* __restrict__ boxes, BvhNode* __restrict__ nodes,
                                                              float4* __restrict__ F, uint32_t* __restrict__ maxd,
                                                              uint32_t dmax) {
    __shared__ Bins sb[SMALL_WAVES];
    __shared__ uint32_t s_rng[SMALL_WAVES][TINY];  // stack: lb | le << 8 | local node id << 16
    __shared__ uint32_t s_dep[SMALL_WAVES][TINY];
    __shared__ int32_t s_kid[SMALL_WAVES][TINY][2];
    __shared__ float s_ua[SMALL_WAVES][TINY];
    __shared__ uint32_t s_ord[SMALL_WAVES][TINY];
    __shared__ float4 s_F[SMALL_WAVES][TINY];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    Bins& B = sb[w];
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t n_tasks = *qn;
    const uint32_t nw = gridDim.x * SMALL_WAVES;
    for (uint32_t ti = blockIdx.x * SMALL_WAVES + w; ti < n_tasks; ti += nw) {
        const Task t = q[ti];
        const uint32_t* __restrict__ src = (t.db & 1u) ? idx1 : idx0;
        const uint32_t n = t.e - t.b;
        const uint32_t root = t.node;
        uint32_t pid = 0;
        float bx[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if ((uint32_t)lane < n) {
            pid = src[t.b + lane];
#pragma unroll
            for (int j = 0; j < 6; ++j) bx[j] = boxes[6ull * pid + j];
        }
        uint32_t wmaxd = 0, cnt = 0;
        int sp = 1;
        if (lane == 0) s_rng[w][0] = n << 8, s_dep[w][0] = t.db >> 1;
        while (sp > 0) {
            --sp;
            const uint32_t rg = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_rng[w][sp]);
            const uint32_t dep = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_dep[w][sp]);
            const uint32_t lb = rg & 0xFFu, le = (rg >> 8) & 0xFFu, lid = rg >> 16;
            const uint32_t nn = le - lb;
            const bool act = (uint32_t)lane >= lb && (uint32_t)lane < le;
            float cen[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) cen[a] = 0.5f * (bx[a] + bx[3 + a]);
            float cl[3], ch[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                cl[a] = act ? cen[a] : INFINITY;
                ch[a] = act ? cen[a] : -INFINITY;
                for (int off = 32; off > 0; off >>= 1) {
                    cl[a] = fminf(cl[a], __shfl_xor(cl[a], off));
                    ch[a] = fmaxf(ch[a], __shfl_xor(ch[a], off));
                }
            }
            float sc[3];
            axis_scales(cl, ch, sc);
            Split s;
            s.axis = -1;
            s.k = -1;
            s.nl = 0;
            bool left = false;
            if (nn == 2) {
                // two proxies: every candidate split separates them at the same cost, so the first
                // binnable axis wins and the lower centroid goes left (bins 0 and 31 of that axis)
                for (int a = 2; a >= 0; --a)
                    if (sc[a] > 0.0f) s.axis = a;
                if (s.axis >= 0) {
                    s.k = 0;
                    s.nl = 1;
                    const float c0 = __shfl(cen[s.axis], (int)lb), c1 = __shfl(cen[s.axis], (int)lb + 1);
                    left = (uint32_t)lane == (c0 < c1 ? lb : lb + 1);
                    const int ll = c0 < c1 ? (int)lb : (int)lb + 1, rl = c0 < c1 ? (int)lb + 1 : (int)lb;
#pragma unroll
                    for (int j = 0; j < 6; ++j) s.lb[j] = __shfl(bx[j], ll), s.rb[j] = __shfl(bx[j], rl);
                }
            } else if (sc[0] > 0.0f || sc[1] > 0.0f || sc[2] > 0.0f) {
                uint32_t* bw = reinterpret_cast<uint32_t*>(&B);
                for (int j = lane; j < BIN_WORDS; j += 64)
                    bw[j] = j < 2 * 3 * NB * 3 ? (j < 3 * NB * 3 ? ORD_MIN_ID : ORD_MAX_ID) : 0u;
                if (act) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        if (!(sc[a] > 0.0f)) continue;
                        const int k = sah_bin(cen[a], cl[a], sc[a]);
#pragma unroll
                        for (int j = 0; j < 3; ++j) {
                            atomicMin(&B.lo[a][k][j], f2o(bx[j]));
                            atomicMax(&B.hi[a][k][j], f2o(bx[3 + j]));
                        }
                        atomicAdd(&B.n[a][k], 1u);
                    }
                }
                s = sah_eval(B, sc);
                if (s.k >= 0 && !sah_split_in_budget(dep, s.nl, nn - s.nl, dmax)) s.axis = -1, s.k = -1;  // depth budget
                if (s.k >= 0) left = act && sah_bin(cen[s.axis], cl[s.axis], sc[s.axis]) <= s.k;
            }
            uint32_t mid;
            if (s.k >= 0) {
                mid = lb + s.nl;
                const uint64_t bl = __ballot(left), br = __ballot(act && !left);
                const uint32_t dest = left ? lb + __popcll(bl & below) : (act ? mid + __popcll(br & below) : (uint32_t)lane);
                const int addr = (int)(dest * 4);
                pid = (uint32_t)__builtin_amdgcn_ds_permute(addr, (int)pid);
#pragma unroll
                for (int j = 0; j < 6; ++j) bx[j] = __int_as_float(__builtin_amdgcn_ds_permute(addr, __float_as_int(bx[j])));
            } else {
                // equal centroids: halve, boxes of the halves
                mid = lb + nn / 2;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    float a0 = act && (uint32_t)lane < mid ? bx[j] : INFINITY, a1 = act && (uint32_t)lane < mid ? bx[3 + j] : -INFINITY;
                    float b0 = act && (uint32_t)lane >= mid ? bx[j] : INFINITY, b1 = act && (uint32_t)lane >= mid ? bx[3 + j] : -INFINITY;
                    for (int off = 32; off > 0; off >>= 1) {
                        a0 = fminf(a0, __shfl_xor(a0, off));
                        a1 = fmaxf(a1, __shfl_xor(a1, off));
                        b0 = fminf(b0, __shfl_xor(b0, off));
                        b1 = fmaxf(b1, __shfl_xor(b1, off));
                    }
                    s.lb[j] = a0, s.lb[3 + j] = a1, s.rb[j] = b0, s.rb[3 + j] = b1;
                }
            }
            const uint32_t L = mid - lb, R = le - mid;
            const int32_t c0 = L == 1 ? ~(int32_t)__shfl(pid, (int)lb) : (int32_t)(root + lid + 1);
            const int32_t c1 = R == 1 ? ~(int32_t)__shfl(pid, (int)mid) : (int32_t)(root + lid + L);
            if (lane < 16) {  // the node's 16 words, one per lane
                uint32_t v = 0u;
#pragma unroll
                for (int j = 0; j < 6; ++j) {  // static indices (a dynamic one puts the boxes in scratch)
                    if (lane == j) v = __float_as_uint(s.lb[j]);
                    if (lane == 6 + j) v = __float_as_uint(s.rb[j]);
                }
                if (lane < 12) {
                } else if (lane == 12) v = (uint32_t)c0;
                else if (lane == 13) v = (uint32_t)c1;
                else if (lane == 14) v = (uint32_t)(s.axis < 0 ? 0 : s.axis);
                else v = 0u;
                reinterpret_cast<uint32_t*>(nodes + root + lid)[lane] = v;
            }
            if (F) {
                if (lane == 0) {
                    s_kid[w][lid][0] = c0;
                    s_kid[w][lid][1] = c1;
                    s_ua[w][lid] = union_area(s.lb, s.rb);
                    s_ord[w][cnt] = lid;
                }
                ++cnt;
            }
            if (L == 1 || R == 1) wmaxd = dep + 1 > wmaxd ? dep + 1 : wmaxd;
            if (lane == 0) {
                if (R > 1) s_rng[w][sp] = mid | le << 8 | (lid + L) << 16, s_dep[w][sp] = dep + 1;
                if (L > 1) s_rng[w][sp + (R > 1 ? 1 : 0)] = lb | mid << 8 | (lid + 1) << 16, s_dep[w][sp + (R > 1 ? 1 : 0)] = dep + 1;
            }
            sp += (R > 1 ? 1 : 0) + (L > 1 ? 1 : 0);
        }
        if (F) {
            for (int i = (int)cnt - 1; i >= 0; --i) {
                const uint32_t lid = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_ord[w][i]);
                const int32_t k0 = s_kid[w][lid][0], k1 = s_kid[w][lid][1];
                float f0[4] = {0.f, 0.f, 0.f, 0.f}, f1[4] = {0.f, 0.f, 0.f, 0.f};
                if (k0 >= 0) {
                    const float4 v = s_F[w][k0 - root];
                    f0[0] = v.x, f0[1] = v.y, f0[2] = v.z, f0[3] = v.w;
                }
                if (k1 >= 0) {
                    const float4 v = s_F[w][k1 - root];
                    f1[0] = v.x, f1[1] = v.y, f1[2] = v.z, f1[3] = v.w;
                }
                const float4 r = dp_row(s_ua[w][lid], f0, f1);
                if (lane == 0) s_F[w][lid] = r;
            }
            if ((uint32_t)lane + 1 < n) F[root + lane] = s_F[w][lane];
        }
        if (lane == 0) atomicMax(maxd, wmaxd);
    }
}

// ---------------- ranges above LARGE: chunked, one workgroup per CHUNK proxies
struct Chunk {
    uint32_t task;  // index into the level's range list
    uint32_t b, e;  // proxy positions of this chunk
    uint32_t first; // index of the range's first chunk (left counts of earlier chunks are summed from it)
};

__global__ __launch_bounds__(256) void k_lg_init(LgRange* __restrict__ r, uint32_t nr) {
    const uint32_t i = blockIdx.x;
    if (i >= nr) return;
    uint32_t* w = reinterpret_cast<uint32_t*>(&r[i]);
    for (int j = threadIdx.x; j < (int)(sizeof(LgRange) / 4); j += 256) {
        uint32_t v;
        if (j < 3) v = ORD_MIN_ID;
        else if (j < 8) v = ORD_MAX_ID;
        else {
            const int k = j - 8;
            v = k < 3 * NB * 3 ? ORD_MIN_ID : (k < 2 * 3 * NB * 3 ? ORD_MAX_ID : 0u);
        }
        w[j] = v;
    }
}

__device__ inline void block_minmax6(float* lo, float* hi, float (*red)[6]) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int a = 0; a < 3; ++a)
        for (int off = 32; off > 0; off >>= 1) {
            lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
            hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
        }
    if (lane == 0)
        for (int a = 0; a < 3; ++a) red[w][a] = lo[a], red[w][3 + a] = hi[a];
    __syncthreads();
    for (int a = 0; a < 3; ++a) {
        lo[a] = fminf(fminf(red[0][a], red[1][a]), fminf(red[2][a], red[3][a]));
        hi[a] = fmaxf(fmaxf(red[0][3 + a], red[1][3 + a]), fmaxf(red[2][3 + a], red[3][3 + a]));
    }
}

__global__ __launch_bounds__(256) void k_lg_cbounds(const Chunk* __restrict__ ch, const Task* __restrict__ tasks,
                                                    const uint32_t* __restrict__ idx0, const uint32_t* __restrict__ idx1,
                                                    const float* __restrict__ boxes, LgRange* __restrict__ r) {
    __shared__ float red[4][6];
    const Chunk c = ch[blockIdx.x];
    const uint32_t* __restrict__ src = (tasks[c.task].db & 1u) ? idx1 : idx0;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = c.b + threadIdx.x; i < c.e; i += 256) {
        const uint32_t p = src[i];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = centroid(boxes, p, a);
            lo[a] = fminf(lo[a], v);
            hi[a] = fmaxf(hi[a], v);
        }
    }
    block_minmax6(lo, hi, red);
    if (threadIdx.x < 3) atomicMin(&r[c.task].cb[threadIdx.x], f2o(lo[threadIdx.x]));
    else if (threadIdx.x < 6) atomicMax(&r[c.task].cb[threadIdx.x], f2o(hi[threadIdx.x - 3]));
}

__device__ inline void range_scales(const LgRange& r, float* cl, float* sc) {
    float ch[3];
    for (int a = 0; a < 3; ++a) cl[a] = o2f(r.cb[a]), ch[a] = o2f(r.cb[3 + a]);
    axis_scales(cl, ch, sc);
}

__global__ __launch_bounds__(256) void k_lg_bin(const Chunk* __restrict__ ch, const Task* __restrict__ tasks,
                                                const uint32_t* __restrict__ idx0, const uint32_t* __restrict__ idx1,
                                                const float* __restrict__ boxes, LgRange* __restrict__ r) {
    __shared__ Bins B;
    const Chunk c = ch[blockIdx.x];
    const uint32_t* __restrict__ src = (tasks[c.task].db & 1u) ? idx1 : idx0;
    float cl[3], sc[3];
    range_scales(r[c.task], cl, sc);
    uint32_t* bw = reinterpret_cast<uint32_t*>(&B);
    for (int j = threadIdx.x; j < BIN_WORDS; j += 256) bw[j] = j < 2 * 3 * NB * 3 ? (j < 3 * NB * 3 ? ORD_MIN_ID : ORD_MAX_ID) : 0u;
    __syncthreads();
    for (uint32_t i = c.b + threadIdx.x; i < c.e; i += 256) {
        const uint32_t p = src[i];
        float bl[3], bh[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) bl[a] = boxes[6ull * p + a], bh[a] = boxes[6ull * p + 3 + a];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (!(sc[a] > 0.0f)) continue;
            const int k = sah_bin(0.5f * (bl[a] + bh[a]), cl[a], sc[a]);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                atomicMin(&B.lo[a][k][j], f2o(bl[j]));
                atomicMax(&B.hi[a][k][j], f2o(bh[j]));
            }
            atomicAdd(&B.n[a][k], 1u);
        }
    }
    __syncthreads();
    uint32_t* gw = reinterpret_cast<uint32_t*>(&r[c.task].bins);
    for (int j = threadIdx.x; j < BIN_WORDS; j += 256) {
        const uint32_t v = bw[j];
        if (j < 3 * NB * 3) { if (v != ORD_MIN_ID) atomicMin(gw + j, v); }
        else if (j < 2 * 3 * NB * 3) { if (v != ORD_MAX_ID) atomicMax(gw + j, v); }
        else if (v) atomicAdd(gw + j, v);
    }
}

// one wave per range: the split decision
struct Decision {
    Split s;
    uint32_t mid;
};
__global__ __launch_bounds__(64) void k_lg_eval(const Task* __restrict__ tasks, const LgRange* __restrict__ r,
                                                Decision* __restrict__ dec, uint32_t dmax) {
    const uint32_t t = blockIdx.x;
    float cl[3], sc[3];
    range_scales(r[t], cl, sc);
    Split s;
    s.axis = -1;
    s.k = -1;
    s.nl = 0;
    if (sc[0] > 0.0f || sc[1] > 0.0f || sc[2] > 0.0f) s = sah_eval(r[t].bins, sc);
    const Task tk = tasks[t];
    // depth budget (SAH_DEPTH_MAX): halve the range instead of a split whose larger side could not finish in budget
    if (s.k >= 0 && !sah_split_in_budget(tk.db >> 1, s.nl, (tk.e - tk.b) - s.nl, dmax)) s.axis = -1, s.k = -1;
    if ((threadIdx.x & 63) == 0) {
        Decision d;
        d.s = s;
        d.mid = s.k >= 0 ? tk.b + s.nl : tk.b + (tk.e - tk.b) / 2;
        dec[t] = d;
    }
}

__device__ inline bool lg_left(const Decision& d, const LgRange& r, const float* __restrict__ boxes, uint32_t p,
                               uint32_t pos) {
    if (d.s.k < 0) return pos < d.mid;
    float cl[3], sc[3];
    range_scales(r, cl, sc);
    const int a = d.s.axis;
    return sah_bin(centroid(boxes, p, a), cl[a], sc[a]) <= d.s.k;
}

__global__ __launch_bounds__(256) void k_lg_count(const Chunk* __restrict__ ch, const Task* __restrict__ tasks,
                                                  const uint32_t* __restrict__ idx0, const uint32_t* __restrict__ idx1,
                                                  const float* __restrict__ boxes, const LgRange* __restrict__ r,
                                                  const Decision* __restrict__ dec, uint32_t* __restrict__ nleft) {
    __shared__ uint32_t red[4];
    const Chunk c = ch[blockIdx.x];
    const uint32_t* __restrict__ src = (tasks[c.task].db & 1u) ? idx1 : idx0;
    const Decision d = dec[c.task];
    uint32_t cnt = 0;
    for (uint32_t i = c.b + threadIdx.x; i < c.e; i += 256) cnt += lg_left(d, r[c.task], boxes, src[i], i) ? 1u : 0u;
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) nleft[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void k_lg_scatter(const Chunk* __restrict__ ch, const Task* __restrict__ tasks,
                                                    uint32_t* __restrict__ idx0, uint32_t* __restrict__ idx1,
                                                    const float* __restrict__ boxes, const LgRange* __restrict__ r,
                                                    const Decision* __restrict__ dec, const uint32_t* __restrict__ nleft) {
    __shared__ uint32_t wl[4], wr[4];
    __shared__ uint32_t base_s[2];
    const Chunk c = ch[blockIdx.x];
    const Task t = tasks[c.task];
    const uint32_t* __restrict__ src = (t.db & 1u) ? idx1 : idx0;
    uint32_t* __restrict__ dst = (t.db & 1u) ? idx0 : idx1;
    const Decision d = dec[c.task];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        uint32_t before = 0;  // left proxies in earlier chunks of this range
        for (uint32_t k = c.first; k < blockIdx.x; ++k) before += nleft[k];
        base_s[0] = t.b + before;
        base_s[1] = d.mid + (c.b - t.b) - before;
    }
    __syncthreads();
    uint32_t lb = base_s[0], rb = base_s[1];
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint32_t i0 = c.b; i0 < c.e; i0 += 256) {
        const uint32_t i = i0 + threadIdx.x;
        const bool v = i < c.e;
        const uint32_t p = v ? src[i] : 0u;
        const bool left = v && lg_left(d, r[c.task], boxes, p, i);
        const uint64_t bl = __ballot(left), br = __ballot(v && !left);
        if (lane == 0) wl[w] = __popcll(bl), wr[w] = __popcll(br);
        __syncthreads();
        uint32_t ol = 0, orr = 0, tl = 0, tr = 0;
        for (int k = 0; k < 4; ++k) {
            if (k < w) ol += wl[k], orr += wr[k];
            tl += wl[k];
            tr += wr[k];
        }
        if (left) dst[lb + ol + __popcll(bl & below)] = p;
        else if (v) dst[rb + orr + __popcll(br & below)] = p;
        lb += tl;
        rb += tr;
        __syncthreads();
    }
}

// one wave per range: node + children (after the partition, so a one-proxy child names its leaf)
__global__ __launch_bounds__(64) void k_lg_finish(const Task* __restrict__ tasks, const Decision* __restrict__ dec,
                                                  const uint32_t* __restrict__ idx0, const uint32_t* __restrict__ idx1,
                                                  const float* __restrict__ boxes, BuildOut o) {
    const Task t = tasks[blockIdx.x];
    const uint32_t* __restrict__ dst = (t.db & 1u) ? idx0 : idx1;
    Decision d = dec[blockIdx.x];
    if (d.s.k < 0) {
        wave_box_union(boxes, dst, t.b, d.mid, d.s.lb);
        wave_box_union(boxes, dst, d.mid, t.e, d.s.rb);
    }
    emit_node(t, d.s, d.mid, dst[t.b], dst[d.mid], o);
}

// ---------------- surface-area-optimal collapse
// DP rows F[n][k-1] (k = 1..4) of the binary nodes built by the level kernels: one launch per logged
// level, deepest first (every child was built, and so logged, after its parent), one thread per node.
// The tiny subtrees computed their own rows.
__device__ inline float rowv(const float4* __restrict__ F, int32_t x, int k) {
    if (x < 0) return 0.0f;
    return reinterpret_cast<const float*>(F + x)[k - 1];
}

__global__ __launch_bounds__(256) void k_dp_seg(const Task* __restrict__ log, const uint32_t* __restrict__ se,
                                                const BvhNode* __restrict__ bn, float4* __restrict__ F) {
    const uint32_t q0 = se[0], q1 = se[1];
    for (uint32_t i = q0 + blockIdx.x * blockDim.x + threadIdx.x; i < q1; i += gridDim.x * blockDim.x) {
        const uint32_t x = log[i].node;
        const BvhNode n = bn[x];
        const float* nb = reinterpret_cast<const float*>(&n);
        float f0[4] = {0.f, 0.f, 0.f, 0.f}, f1[4] = {0.f, 0.f, 0.f, 0.f};
        if (n.c0 >= 0) {
            const float4 v = F[n.c0];
            f0[0] = v.x, f0[1] = v.y, f0[2] = v.z, f0[3] = v.w;
        }
        if (n.c1 >= 0) {
            const float4 v = F[n.c1];
            f1[0] = v.x, f1[1] = v.y, f1[2] = v.z, f1[3] = v.w;
        }
        F[x] = dp_row(union_area(nb, nb + 6), f0, f1);
    }
}

struct Piece {
    int32_t ref;
    float box[6];  // lo xyz, hi xyz
};

// The pieces of the 4-wide node opened at binary node x: host_dp_collapse's `expand` (children
// in depth-first, left-first order), iteratively
__device__ inline int dp_pieces(const BvhNode* __restrict__ bn, const float4* __restrict__ F, int32_t x, Piece* out) {
#pragma clang fp contract(off)
    struct Item {
        int32_t x;
        int k;
        float box[6];
    };
    Item st[4];
    int sp = 0, np = 0;
    auto push_children = [&](int32_t y, int k) {  // split y's k pieces between its children
        const BvhNode n = bn[y];
        const float* nb = reinterpret_cast<const float*>(&n);
        int bj = 1;
        float bv = INFINITY;
        for (int j = 1; j < k; ++j) {
            const float v = rowv(F, n.c0, j) + rowv(F, n.c1, k - j);
            if (v < bv) bv = v, bj = j;
        }
        Item a, b;
        a.x = n.c0, a.k = bj;
        b.x = n.c1, b.k = k - bj;
        for (int q = 0; q < 6; ++q) a.box[q] = nb[q], b.box[q] = nb[6 + q];
        st[sp++] = b;  // right pushed first: the left is expanded first
        st[sp++] = a;
    };
    push_children(x, 4);
    while (sp > 0) {
        Item it = st[--sp];
        while (it.x >= 0 && it.k > 1 && rowv(F, it.x, it.k) == rowv(F, it.x, it.k - 1)) --it.k;
        if (it.x < 0 || it.k == 1) {
            out[np].ref = it.x;
            for (int q = 0; q < 6; ++q) out[np].box[q] = it.box[q];
            ++np;
        } else {
            push_children(it.x, it.k);
        }
    }
    return np;
}

__global__ __launch_bounds__(256) void k_dp_count(uint32_t n, const int32_t* __restrict__ queue, const BvhNode* __restrict__ bn,
                                                  const float4* __restrict__ F, uint32_t* __restrict__ cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    if (i == n) { cnt[i] = 0; return; }
    Piece ps[4];
    const int np = dp_pieces(bn, F, queue[i], ps);
    uint32_t c = 0;
    for (int j = 0; j < np; ++j) c += ps[j].ref >= 0 ? 1u : 0u;
    cnt[i] = c;
}

__global__ __launch_bounds__(256) void k_dp_emit(uint32_t n, uint32_t base, const int32_t* __restrict__ queue_in,
                                                 int32_t* __restrict__ queue_out, const BvhNode* __restrict__ bn,
                                                 const float4* __restrict__ F, const uint32_t* __restrict__ off,
                                                 Bvh4Node* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t x = queue_in[i];
    Piece ps[4];
    const int np = dp_pieces(bn, F, x, ps);
    Bvh4Node o;
    uint32_t imask = 0, q = off[i];
    for (int j = 0; j < BVH_W; ++j) {
        if (j < np) {
            int32_t r = ps[j].ref;
            if (r >= 0) {
                queue_out[q] = r;
                r = (int32_t)(base + n + q);  // breadth-first id: after this level's n nodes
                ++q;
                imask |= 1u << j;
            }
            const float* b = ps[j].box;
            o.box[j][0] = b[0], o.box[j][1] = b[3];
            o.box[j][2] = b[1], o.box[j][3] = b[4];
            o.box[j][4] = b[2], o.box[j][5] = b[5];
            o.child[j] = r;
        } else {
            for (int k = 0; k < 6; ++k) o.box[j][k] = EMPTY_BOX;
            o.child[j] = 0;
        }
    }
    o.nchild = (uint32_t)np;
    o.pad[0] = bn[x].pad0;
    o.pad[1] = imask;
    o.pad[2] = 0;
    out[base + i] = o;
}

template <typename T>
struct DevBuf {
    gvrt_context* c;
    T* p = nullptr;
    explicit DevBuf(gvrt_context* c_) : c(c_) {}
    ~DevBuf() { gvrt_dfree(c, (void**)&p); }
    gvrt_status alloc(uint64_t n) { return gvrt_dalloc(c, (void**)&p, sizeof(T) * (n ? n : 1)); }
};

}  // namespace

#define SAH_TRY(x)                            \
    do {                                      \
        const gvrt_status _s = (x);           \
        if (_s != GVRT_OK) return _s;         \
    } while (0)

// Binary binned-SAH tree over m >= 2 Morton-ordered leaf boxes into nodes[0 .. m-2] (root 0) and its
// max binary leaf depth; with out4 != null also the surface-area-optimal 4-wide collapse into out4
// (*n4 nodes, *depth4 levels).
gvrt_status gvrt_sah_build_device(gvrt_context* c, uint64_t m, const float* lboxes, BvhNode* nodes, Bvh4Node* out4,
                                  uint32_t* depth_out, uint64_t* n4_out, uint32_t* depth4_out, uint32_t dmax) {
    if (m < 2) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "device SAH build needs two or more leaves");
    if (m > 0x7FFFFFFFull) return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "device SAH build: too many leaves");
    const bool dp = out4 != nullptr;
    const uint64_t ni = m - 1;
    DevBuf<uint32_t> idx0(c), idx1(c), ctl(c), nleft(c), ends(c), lends(c);
    DevBuf<Task> midq(c), tinyq(c), lq(c), llog(c);
    DevBuf<Chunk> chunks(c);
    DevBuf<LgRange> lr(c);
    DevBuf<Decision> dec(c);
    DevBuf<float4> F(c);
    const uint64_t lcap = m / LARGE + 2;
    const uint64_t ccap = m / CHUNK + lcap + 2;
    SAH_TRY(idx0.alloc(m));
    SAH_TRY(idx1.alloc(m));
    SAH_TRY(midq.alloc(m));          // every mid range is one internal node
    SAH_TRY(ends.alloc(m + 4));      // mid level segment ends (a level holds >= 1 range)
    SAH_TRY(tinyq.alloc(m / 2 + 2));
    SAH_TRY(lq.alloc(2 * lcap));
    SAH_TRY(ctl.alloc(8));           // [0] tiny count, [2] large count, [3] max depth
    SAH_TRY(chunks.alloc(ccap));
    SAH_TRY(nleft.alloc(ccap));
    SAH_TRY(lr.alloc(lcap));
    SAH_TRY(dec.alloc(lcap));
    if (dp) SAH_TRY(F.alloc(ni));
    hipStream_t st = c->stream;
    {
        std::vector<uint32_t> h(m);
        for (uint64_t i = 0; i < m; ++i) h[i] = (uint32_t)i;
        GVRT_HIP(c, hipMemcpyAsync(idx0.p, h.data(), 4 * m, hipMemcpyHostToDevice, st));
        GVRT_HIP(c, hipMemsetAsync(ctl.p, 0, 32, st));
        GVRT_HIP(c, hipMemsetAsync(ends.p, 0, 8, st));
        const Task root{0u, (uint32_t)m, 0u, 1u << 1};
        const uint32_t one = 1;
        if (m <= TINY) {
            GVRT_HIP(c, hipMemcpyAsync(tinyq.p, &root, sizeof(Task), hipMemcpyHostToDevice, st));
            GVRT_HIP(c, hipMemcpyAsync(ctl.p + 0, &one, 4, hipMemcpyHostToDevice, st));
        } else if (m <= LARGE) {
            GVRT_HIP(c, hipMemcpyAsync(midq.p, &root, sizeof(Task), hipMemcpyHostToDevice, st));
            GVRT_HIP(c, hipMemcpyAsync(ends.p + 1, &one, 4, hipMemcpyHostToDevice, st));
        }
        GVRT_HIP(c, hipStreamSynchronize(st));
    }
    BuildOut o{nodes, ctl.p + 3, midq.p, ends.p + 1, tinyq.p, ctl.p + 0, nullptr, ctl.p + 2, dmax};
    // ---- chunked levels: host-side list of the level's large ranges (a handful per level), logged for the DP
    std::vector<Task> lt = m > LARGE ? std::vector<Task>{Task{0u, (uint32_t)m, 0u, 1u << 1}} : std::vector<Task>{};
    std::vector<Task> hlog;
    std::vector<uint32_t> hends{0};
    Task* lcur = lq.p;
    Task* lnext = lq.p + lcap;
    while (!lt.empty()) {
        const uint32_t nr = (uint32_t)lt.size();
        hlog.insert(hlog.end(), lt.begin(), lt.end());
        hends.push_back((uint32_t)hlog.size());
        std::vector<Chunk> hc;
        for (uint32_t t = 0; t < nr; ++t) {
            const uint32_t first = (uint32_t)hc.size();
            for (uint32_t b = lt[t].b; b < lt[t].e; b += CHUNK) hc.push_back(Chunk{t, b, std::min(lt[t].e, b + CHUNK), first});
        }
        const uint32_t nc = (uint32_t)hc.size();
        if (nc > ccap || nr > lcap) return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "device SAH build: chunk list overflow");
        GVRT_HIP(c, hipMemcpyAsync(chunks.p, hc.data(), sizeof(Chunk) * nc, hipMemcpyHostToDevice, st));
        GVRT_HIP(c, hipMemcpyAsync(lcur, lt.data(), sizeof(Task) * nr, hipMemcpyHostToDevice, st));
        GVRT_HIP(c, hipMemsetAsync(ctl.p + 2, 0, 4, st));
        hipLaunchKernelGGL(k_lg_init, dim3(nr), dim3(256), 0, st, lr.p, nr);
        hipLaunchKernelGGL(k_lg_cbounds, dim3(nc), dim3(256), 0, st, chunks.p, lcur, idx0.p, idx1.p, lboxes, lr.p);
        hipLaunchKernelGGL(k_lg_bin, dim3(nc), dim3(256), 0, st, chunks.p, lcur, idx0.p, idx1.p, lboxes, lr.p);
        hipLaunchKernelGGL(k_lg_eval, dim3(nr), dim3(64), 0, st, lcur, lr.p, dec.p, dmax);
        hipLaunchKernelGGL(k_lg_count, dim3(nc), dim3(256), 0, st, chunks.p, lcur, idx0.p, idx1.p, lboxes, lr.p, dec.p,
                           nleft.p);
        hipLaunchKernelGGL(k_lg_scatter, dim3(nc), dim3(256), 0, st, chunks.p, lcur, idx0.p, idx1.p, lboxes, lr.p, dec.p,
                           nleft.p);
        o.large_q = lnext;
        hipLaunchKernelGGL(k_lg_finish, dim3(nr), dim3(64), 0, st, lcur, dec.p, idx0.p, idx1.p, lboxes, o);
        GVRT_HIP(c, hipGetLastError());
        uint32_t nn = 0;
        GVRT_HIP(c, hipMemcpyAsync(&nn, ctl.p + 2, 4, hipMemcpyDeviceToHost, st));
        GVRT_HIP(c, hipStreamSynchronize(st));
        lt.resize(nn);
        if (nn) GVRT_HIP(c, hipMemcpyAsync(lt.data(), lnext, sizeof(Task) * nn, hipMemcpyDeviceToHost, st));
        GVRT_HIP(c, hipStreamSynchronize(st));
        std::swap(lcur, lnext);
    }
    // ---- mid levels: level L is midq[ends[L] .. ends[L+1]); it appends the next level at ends[L+2]
    // (seeded with ends[L+1]).  The host looks for an empty level every few launches.
    const unsigned grid = 2048;
    uint64_t nlev = 0;
    bool done = false;
    for (uint64_t lv = 0; lv + 2 < m + 4; ++lv) {
        GVRT_HIP(c, hipMemcpyAsync(ends.p + lv + 2, ends.p + lv + 1, 4, hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(k_sah_mid, dim3(grid), dim3(64 * SMALL_WAVES), 0, st, midq.p, ends.p + lv, idx0.p, idx1.p,
                           lboxes, o);
        GVRT_HIP(c, hipGetLastError());
        nlev = lv + 1;
        if ((lv & 3) == 3 || lv == 0) {
            uint32_t e2[2] = {0, 0};
            GVRT_HIP(c, hipMemcpyAsync(e2, ends.p + lv + 1, 8, hipMemcpyDeviceToHost, st));
            GVRT_HIP(c, hipStreamSynchronize(st));
            if (e2[0] == e2[1]) { done = true; break; }  // level lv + 1 is empty
        }
    }
    if (!done) return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "device SAH build did not finish");
    // ---- tiny subtrees (with their DP rows)
    hipLaunchKernelGGL(k_sah_tiny, dim3(grid), dim3(64 * SMALL_WAVES), 0, st, tinyq.p, ctl.p + 0, idx0.p, idx1.p,
                       lboxes, nodes, dp ? F.p : nullptr, ctl.p + 3, dmax);
    GVRT_HIP(c, hipGetLastError());
    GVRT_HIP(c, hipMemcpyAsync(depth_out, ctl.p + 3, 4, hipMemcpyDeviceToHost, st));
    if (!dp) {
        GVRT_HIP(c, hipStreamSynchronize(st));
        return GVRT_OK;
    }
    // ---- DP rows of the mid and large nodes, deepest logged level first
    for (uint64_t lv = nlev; lv-- > 0;)
        hipLaunchKernelGGL(k_dp_seg, dim3(256), dim3(256), 0, st, midq.p, ends.p + lv, nodes, F.p);
    if (!hlog.empty()) {
        SAH_TRY(llog.alloc(hlog.size()));
        SAH_TRY(lends.alloc(hends.size()));
        GVRT_HIP(c, hipMemcpyAsync(llog.p, hlog.data(), sizeof(Task) * hlog.size(), hipMemcpyHostToDevice, st));
        GVRT_HIP(c, hipMemcpyAsync(lends.p, hends.data(), 4 * hends.size(), hipMemcpyHostToDevice, st));
        for (size_t lv = hends.size() - 1; lv-- > 0;)
            hipLaunchKernelGGL(k_dp_seg, dim3(256), dim3(256), 0, st, llog.p, lends.p + lv, nodes, F.p);
    }
    GVRT_HIP(c, hipGetLastError());
    // ---- breadth-first 4-wide layout: per level, piece counts, a scan, then the nodes
    DevBuf<uint32_t> cnt(c), off(c);
    DevBuf<int32_t> q0(c), q1(c);
    DevBuf<uint8_t> tmp(c);
    SAH_TRY(cnt.alloc(ni + 1));
    SAH_TRY(off.alloc(ni + 1));
    SAH_TRY(q0.alloc(ni));
    SAH_TRY(q1.alloc(ni));
    size_t tb = 0;
    GVRT_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt.p, off.p, (int)(ni + 1), st));
    SAH_TRY(tmp.alloc(tb ? tb : 16));
    const int32_t root = 0;
    GVRT_HIP(c, hipMemcpyAsync(q0.p, &root, 4, hipMemcpyHostToDevice, st));
    uint32_t n = 1, base = 0, levels = 0;
    int32_t* qin = q0.p;
    int32_t* qout = q1.p;
    while (n) {
        if (base + n > ni) return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "4-wide collapse overflow");
        const unsigned g = (unsigned)((n + 1 + 255) / 256);
        hipLaunchKernelGGL(k_dp_count, dim3(g), dim3(256), 0, st, n, qin, nodes, F.p, cnt.p);
        GVRT_HIP(c, hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, cnt.p, off.p, (int)(n + 1), st));
        hipLaunchKernelGGL(k_dp_emit, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, base, qin, qout, nodes, F.p,
                           off.p, out4);
        GVRT_HIP(c, hipGetLastError());
        uint32_t next = 0;
        GVRT_HIP(c, hipMemcpyAsync(&next, off.p + n, 4, hipMemcpyDeviceToHost, st));
        GVRT_HIP(c, hipStreamSynchronize(st));
        base += n;
        n = next;
        ++levels;
        std::swap(qin, qout);
    }
    *n4_out = base;
    *depth4_out = levels;
    return GVRT_OK;
}
