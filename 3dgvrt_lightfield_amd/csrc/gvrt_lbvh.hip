// gvrt_lbvh.hip — linear BVH over the enclosing proxies, built on gfx950.
//
// Replaces the driver BLAS/TLAS builds of VulkanFullRT::createBottomLevelAccelerationStructure3DGRT
// and createTopLevelAccelerationStructure3DGRT (VulkanFullRT.cpp:575-787).  The reference builds
// a BLAS over the 20 triangles of every proxy (20N primitives, Q4); here one leaf is one proxy
// (the render kernel clips the ray against the analytic icosahedron), so the tree has M leaves.
//
//   1. centroid bounds        (block reduction + ordered-uint atomics)
//   2. 63-bit Morton codes    (21 bits per axis)
//   3. stable radix sort      (rocPRIM via hipcub, keys 63 bits, values = compaction index)
//   4. permute records        (render records, SH, boxes into leaf order: leaf j = record j)
//   5. Karras 2012 hierarchy  (one thread per internal node; index tie-break for equal codes)
//   6. child boxes            (range-union sparse table over the leaf boxes, written by the hierarchy pass)
//   7. depth census           (guards the render kernel's fixed LDS stack)
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "gvrt_internal.h"

using namespace gvrt;

namespace {

__device__ inline uint32_t f2ord(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float ord2f(uint32_t u) {
    const uint32_t b = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
#ifdef __HIP_DEVICE_COMPILE__
    return __uint_as_float(b);
#else
    float f;
    memcpy(&f, &b, 4);
    return f;
#endif
}

// bounds of the box centroids (CENTROID) or of the boxes themselves, pass 1: one partial per block
// (block reduce in LDS, no contended atomics)
template <bool CENTROID>
__global__ __launch_bounds__(256) void k_bounds(uint64_t m, const float* __restrict__ boxes, float* __restrict__ part) {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float bl = boxes[6 * i + k], bh = boxes[6 * i + 3 + k];
            const float c = 0.5f * (bl + bh);
            lo[k] = fminf(lo[k], CENTROID ? c : bl);
            hi[k] = fmaxf(hi[k], CENTROID ? c : bh);
        }
    }
    __shared__ float red[4][6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        for (int off = 32; off > 0; off >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], off));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], off));
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            red[w][k] = lo[k];
            red[w][3 + k] = hi[k];
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        float v = red[0][k];
        for (int j = 1; j < 4; ++j) v = k < 3 ? fminf(v, red[j][k]) : fmaxf(v, red[j][k]);
        part[6 * blockIdx.x + k] = v;
    }
}

// pass 2: one block folds the partials into the ordered-uint bounds k_morton reads
__global__ __launch_bounds__(256) void k_bounds_final(uint32_t nparts, const float* __restrict__ part,
                                                      uint32_t* __restrict__ out) {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            lo[k] = fminf(lo[k], part[6 * i + k]);
            hi[k] = fmaxf(hi[k], part[6 * i + 3 + k]);
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        for (int off = 32; off > 0; off >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], off));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], off));
        }
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            atomicMin(out + k, f2ord(lo[k]));
            atomicMax(out + 3 + k, f2ord(hi[k]));
        }
    }
}

// spread the low 21 bits of v to every third bit of a 64-bit word
__device__ inline uint64_t expand21(uint64_t v) {
    v &= 0x1FFFFFull;
    v = (v | (v << 32)) & 0x1F00000000FFFFull;
    v = (v | (v << 16)) & 0x1F0000FF0000FFull;
    v = (v | (v << 8)) & 0x100F00F00F00F00Full;
    v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
    v = (v | (v << 2)) & 0x1249249249249249ull;
    return v;
}

// 63-bit Morton codes (21 bits per axis): at 1 M proxies a 30-bit grid leaves many equal codes in the
// dense object region, whose order (by index) is spatially arbitrary
__global__ __launch_bounds__(256) void k_morton(uint64_t m, const float* __restrict__ boxes, const uint32_t* __restrict__ bnd,
                                                uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint64_t code = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float lo = ord2f(bnd[k]), hi = ord2f(bnd[3 + k]);
        const float c = 0.5f * (boxes[6 * i + k] + boxes[6 * i + 3 + k]);
        const float ext = hi - lo;
        float u = ext > 0.0f ? (c - lo) / ext : 0.5f;
        u = fminf(fmaxf(u * 2097152.0f, 0.0f), 2097151.0f);
        code |= expand21((uint64_t)u) << (2 - k);
    }
    keys[i] = code;
    vals[i] = (uint32_t)i;
}

// Leaf order: leaf j takes sorted item perm[j] (a proxy, or a split piece whose proxy is psrc[.]).
// Records and SH are copied per leaf, pieces included: the k-buffer payload is the leaf index, so the
// composite, the origin record copies and the acceptance boxes read per-leaf arrays with or without split.
__global__ __launch_bounds__(256) void k_permute(uint64_t m, const uint32_t* __restrict__ perm, const RenderRec* __restrict__ rin,
                                                 const float* __restrict__ shin, const float* __restrict__ bin,
                                                 const uint4* __restrict__ paux, RenderRec* __restrict__ rout,
                                                 float* __restrict__ shout, float* __restrict__ bout,
                                                 uint32_t* __restrict__ leaf_src, uint4* __restrict__ aux) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t t = perm[j];
    const uint4 pa = paux ? paux[t] : make_uint4(t, 0xFFFFFFFFu, 0u, 0u);
    const uint32_t s = pa.x;
    rout[j] = rin[s];
    if (shout) {
        const float4* si = reinterpret_cast<const float4*>(shin + 48ull * s);
        float4* so = reinterpret_cast<float4*>(shout + 48ull * j);
#pragma unroll
        for (int k = 0; k < 12; ++k) so[k] = si[k];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) bout[6 * j + k] = bin[6ull * t + k];
    leaf_src[j] = s;
    if (aux) aux[j] = pa;
}

// ---- SplitBLAS analogue (SplitBLAS.cpp:91-186): proxies split into grid-cell pieces
struct Grid {
    float mn[3];
    float inv;   // 1 / cell size
    float size;  // cell size
    uint32_t n[3];
};
__device__ inline int grid_cell(const Grid& g, int a, float x) {
    const int i = (int)floorf((x - g.mn[a]) * g.inv);
    return i < 0 ? 0 : (i >= (int)g.n[a] ? (int)g.n[a] - 1 : i);
}

// A proxy is split when its box overlaps at least min_span cells along one axis (min_span <= 2: every proxy that
// overlaps more than one cell, the reference's rule); a smaller one stays one piece that admits every crossing.
__device__ inline bool piece_single(const int lo[3], const int hi[3], uint32_t min_span) {
    int span = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) span = max(span, hi[a] - lo[a] + 1);
    return span < (int)(min_span > 2u ? min_span : 2u);
}

__global__ __launch_bounds__(256) void k_piece_count(uint64_t m, const float* __restrict__ boxes, Grid g,
                                                     uint32_t min_span, uint64_t* __restrict__ cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > m) return;
    if (i == m) {
        cnt[i] = 0;
        return;
    }
    int lo[3], hi[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = grid_cell(g, a, boxes[6 * i + a]);
        hi[a] = grid_cell(g, a, boxes[6 * i + 3 + a]);
    }
    uint64_t c = 1;
    if (!piece_single(lo, hi, min_span))
#pragma unroll
        for (int a = 0; a < 3; ++a) c *= (uint64_t)(hi[a] - lo[a] + 1);
    cnt[i] = c;
}

__device__ inline uint32_t pack_cell(int x, int y, int z) { return (uint32_t)x | ((uint32_t)y << 10) | ((uint32_t)z << 20); }

// One piece per overlapped cell: box = proxy box clipped to the cell, padded so that a crossing point
// the render kernel assigns to the cell is inside it.  aux = {proxy, cell, proxy's lowest cell,
// highest cell} (cells packed 10 bits per axis); the render kernel admits a crossing in the piece
// whose cell holds the crossing point (clamped to the proxy's cell range), so every crossing of the
// proxy is taken exactly once — the analogue of the reference's triangle clipping, where a ray
// crosses a clipped triangle only inside its cell.  A proxy inside one cell keeps its box and cell
// "any" (0xFFFFFFFF: no point test).
__global__ __launch_bounds__(256) void k_piece_emit(uint64_t m, const float* __restrict__ boxes, Grid g,
                                                    uint32_t min_span, float pad_abs, const uint64_t* __restrict__ off,
                                                    float* __restrict__ pbox, uint4* __restrict__ paux) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int lo[3], hi[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = grid_cell(g, a, boxes[6 * i + a]);
        hi[a] = grid_cell(g, a, boxes[6 * i + 3 + a]);
    }
    uint64_t p = off[i];
    const bool single = piece_single(lo, hi, min_span);
    if (single) {  // one piece: the proxy's own box, every crossing admitted
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            pbox[6 * p + a] = boxes[6 * i + a];
            pbox[6 * p + 3 + a] = boxes[6 * i + 3 + a];
        }
        paux[p] = make_uint4((uint32_t)i, 0xFFFFFFFFu, 0u, 0u);
        return;
    }
    const uint32_t plo = pack_cell(lo[0], lo[1], lo[2]), phi = pack_cell(hi[0], hi[1], hi[2]);
    for (int iz = lo[2]; iz <= hi[2]; ++iz)
        for (int iy = lo[1]; iy <= hi[1]; ++iy)
            for (int ix = lo[0]; ix <= hi[0]; ++ix, ++p) {
                const int ci[3] = {ix, iy, iz};
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const float bl = boxes[6 * i + a], bh = boxes[6 * i + 3 + a];
                    const float cl = g.mn[a] + (float)ci[a] * g.size, ch = g.mn[a] + (float)(ci[a] + 1) * g.size;
                    // (+ the proxy boxes' absolute padding, so a cell face covers the render kernel's plane
                    // rounding as a proxy face does: RenderArgs::box_exact)
                    const float pad = 1e-5f * g.size + 1e-6f * fmaxf(fabsf(cl), fabsf(ch)) + pad_abs;
                    pbox[6 * p + a] = fmaxf(bl, cl - pad);
                    pbox[6 * p + 3 + a] = fminf(bh, ch + pad);
                }
                paux[p] = make_uint4((uint32_t)i, pack_cell(ix, iy, iz), plo, phi);
            }
}

// Split builds: bit 4 + k of pad[1] marks leaf child k as a piece with a cell (its crossings need the cell test,
// gvrt_render.hip GVRT_LEAF); the render kernel loads a leaf's aux record only for those, so the proxies a split
// leaves whole cost what they cost without split
__global__ __launch_bounds__(256) void k_mark_pieces(uint64_t n, Bvh4Node* __restrict__ nodes,
                                                     const uint4* __restrict__ aux) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < BVH_W; ++k) {
        const int32_t ch = nodes[i].child[k];
        if (nodes[i].box[k][0] > 1e37f || ch >= 0) continue;  // empty slot or inner child
        if (aux[~ch].y != 0xFFFFFFFFu) bits |= 16u << k;
    }
    nodes[i].pad[1] = (nodes[i].pad[1] & 0xFu) | bits;
}

// Range-union sparse table over the leaf boxes (leaf order): level k holds, for every i, the union of
// leaves [i, i + 2^k).  The box of any leaf range [l, r] is then the union of two level-k entries
// (k = floor(log2(r - l + 1))) — min / max are exact and order-free, so the result is bit-identical
// to a bottom-up refit, without the refit's per-level cross-XCD atomics.
__global__ __launch_bounds__(256) void k_sparse_level(uint64_t m, uint64_t half, const float* __restrict__ prev,
                                                      float* __restrict__ cur) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i + 2 * half > m) return;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const float a = prev[6 * i + k], b = prev[6 * (i + half) + k];
        cur[6 * i + k] = k < 3 ? fminf(a, b) : fmaxf(a, b);
    }
}

__device__ inline void range_box(const float* const* __restrict__ lv, int64_t l, int64_t r, float* out) {
    const uint64_t len = (uint64_t)(r - l + 1);
    const int k = 63 - __clzll(len);
    const float* a = lv[k] + 6 * l;
    const float* b = lv[k] + 6 * (r - ((int64_t)1 << k) + 1);
#pragma unroll
    for (int j = 0; j < 6; ++j) out[j] = j < 3 ? fminf(a[j], b[j]) : fmaxf(a[j], b[j]);
}

__device__ inline int delta(const uint64_t* __restrict__ codes, int64_t m, int64_t i, int64_t j) {
    if (j < 0 || j >= m) return -1;
    const uint64_t a = codes[i], b = codes[j];
    if (a == b) return 64 + __clz((uint32_t)(i ^ j));
    return __clzll(a ^ b);
}

// Karras, "Maximizing Parallelism in the Construction of BVHs, Octrees, and k-d Trees", HPG 2012.
__global__ __launch_bounds__(256) void k_karras(int64_t m, const uint64_t* __restrict__ codes, BvhNode* __restrict__ nodes,
                                                int32_t* __restrict__ leaf_parent, int32_t* __restrict__ node_parent,
                                                const float* const* __restrict__ levels) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m - 1) return;
    const int d = (delta(codes, m, i, i + 1) - delta(codes, m, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(codes, m, i, i - d);
    int64_t lmax = 2;
    while (delta(codes, m, i, i + lmax * d) > dmin) lmax <<= 1;
    int64_t l = 0;
    for (int64_t t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(codes, m, i, i + (l + t) * d) > dmin) l += t;
    const int64_t j = i + l * d;
    const int dnode = delta(codes, m, i, j);
    int64_t s = 0;
    int64_t t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(codes, m, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int64_t gamma = i + s * d + (d < 0 ? -1 : 0);
    const int64_t lo = i < j ? i : j, hi = i < j ? j : i;
    int32_t c0, c1;
    if (lo == gamma) {
        c0 = ~(int32_t)gamma;
        leaf_parent[gamma] = (int32_t)i;
    } else {
        c0 = (int32_t)gamma;
        node_parent[gamma] = (int32_t)i;
    }
    if (hi == gamma + 1) {
        c1 = ~(int32_t)(gamma + 1);
        leaf_parent[gamma + 1] = (int32_t)i;
    } else {
        c1 = (int32_t)(gamma + 1);
        node_parent[gamma + 1] = (int32_t)i;
    }
    nodes[i].c0 = c0;
    nodes[i].c1 = c1;
    // child boxes straight from the leaf ranges [lo, gamma] and [gamma + 1, hi]
    float b0[6], b1[6];
    range_box(levels, lo, gamma, b0);
    range_box(levels, gamma + 1, hi, b1);
    float* nf = reinterpret_cast<float*>(nodes + i);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        nf[k] = b0[k];
        nf[6 + k] = b1[k];
    }
    // split axis: the first Morton bit where the range differs (bit 3b+2 = x, 3b+1 = y, 3b = z); c0 is the
    // lower side, so the render kernel can order children by the ray's direction on this axis
    const int p = 63 - dnode;
    nodes[i].pad0 = dnode >= 64 ? 0u : (uint32_t)(2 - p % 3);
    nodes[i].pad1 = 0;
    if (i == 0) node_parent[0] = -1;
}

__device__ inline void put_slot(Bvh4Node& o, int k, const float* b, int32_t ref) {
    o.box[k][0] = b[0]; o.box[k][1] = b[3];  // x: lo, hi
    o.box[k][2] = b[1]; o.box[k][3] = b[4];  // y
    o.box[k][4] = b[2]; o.box[k][5] = b[5];  // z
    o.child[k] = ref;
}

__device__ inline float half_area(const float* b) {
    const float ex = b[3] - b[0], ey = b[4] - b[1], ez = b[5] - b[2];
    return ex * ey + ey * ez + ez * ex;
}

// Greedy surface-area collapse, one 4-wide level per launch: a 4-wide node starts from its binary
// root's two children and opens the internal child with the largest surface area until it holds four;
// its internal children become next-level 4-wide nodes.  Ids are allocated per level: level L holds
// ids [base_L, base_L + cnt[L]) with base_L = cnt[0] + ... + cnt[L-1], and level L allocates its
// children as base_{L+1} + atomicAdd(&cnt[L+1], 1) — every count a launch reads is final (its level
// was filled by the previous launch), so no bookkeeping launch runs between levels.  The binary depth
// of every slot rides along (bdep), giving the max leaf depth without a separate leaf-to-root walk.
// ctl = {max 4-wide level, max binary leaf depth}.
__global__ __launch_bounds__(256) void k_collapse_level(const BvhNode* __restrict__ bin, int32_t* __restrict__ src4,
                                                        uint32_t* __restrict__ bdep, uint32_t* __restrict__ cnt,
                                                        uint32_t* __restrict__ ctl, uint32_t level,
                                                        Bvh4Node* __restrict__ out) {
    uint32_t begin = 0;
    for (uint32_t l = 0; l < level; ++l) begin += cnt[l];
    const uint32_t end = begin + cnt[level];
    const uint64_t i = (uint64_t)begin + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // (no early return: the whole wave takes part in the id allocation below)
    const bool live = i < end;
    const BvhNode n = bin[live ? src4[i] : 0];
    const uint32_t d0 = live ? bdep[i] : 0u;  // binary depth of this 4-wide node's binary root (root = 1)
    int32_t ref[BVH_W];
    uint32_t rd[BVH_W];
    float box[BVH_W][6];
    const float* nb = reinterpret_cast<const float*>(&n);
    ref[0] = n.c0;
    ref[1] = n.c1;
    rd[0] = rd[1] = d0 + 1;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        box[0][k] = nb[k];
        box[1][k] = nb[6 + k];
    }
    int cnt_s = 2;
    while (live && cnt_s < BVH_W) {
        int best = -1;
        float ba = -1.0f;
        for (int j = 0; j < cnt_s; ++j) {
            if (ref[j] >= 0) {
                const float ar = half_area(box[j]);
                if (ar > ba) {
                    ba = ar;
                    best = j;
                }
            }
        }
        if (best < 0) break;
        const BvhNode g = bin[ref[best]];
        const float* gb = reinterpret_cast<const float*>(&g);
        const uint32_t gd = rd[best] + 1;
        for (int j = cnt_s; j > best + 1; --j) {  // keep the children in order (c0 before c1)
            ref[j] = ref[j - 1];
            rd[j] = rd[j - 1];
            for (int k = 0; k < 6; ++k) box[j][k] = box[j - 1][k];
        }
        ref[best] = g.c0;
        ref[best + 1] = g.c1;
        rd[best] = rd[best + 1] = gd;
        for (int k = 0; k < 6; ++k) {
            box[best][k] = gb[k];
            box[best + 1][k] = gb[6 + k];
        }
        ++cnt_s;
    }
    // next-level ids: one atomic per block (device atomics on one word serialise, ~11 ns each on MI355X:
    // one per node, then one per wave, cost tens of microseconds per wide level), lanes offset by an exclusive
    // prefix sum of their internal-child counts within the block
    uint32_t nin = 0;
    if (live)
        for (int j = 0; j < cnt_s; ++j) nin += ref[j] >= 0 ? 1u : 0u;
    const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
    uint32_t incl = nin;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, off, 64);
        if (lane >= off) incl += v;
    }
    // the deepest binary leaf below this lane's node
    uint32_t ld = 0;
    if (live)
        for (int j = 0; j < cnt_s; ++j) ld = ref[j] < 0 ? max(ld, rd[j]) : ld;
    for (int off = 32; off > 0; off >>= 1) ld = max(ld, (uint32_t)__shfl_xor((int)ld, off, 64));
    __shared__ uint32_t s_wt[4], s_ld[4], s_base;
    if (lane == 63) s_wt[wave] = incl;
    if (lane == 0) s_ld[wave] = ld;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t tot = s_wt[0] + s_wt[1] + s_wt[2] + s_wt[3];
        const uint32_t bld = max(max(s_ld[0], s_ld[1]), max(s_ld[2], s_ld[3]));
        s_base = tot ? atomicAdd(cnt + level + 1, tot) : 0u;
        if (tot) atomicMax(ctl + 0, level + 1);  // this level made next-level nodes
        if (bld) atomicMax(ctl + 1, bld);
    }
    __syncthreads();
    uint32_t wbase = s_base;
    for (int w = 0; w < wave; ++w) wbase += s_wt[w];
    if (!live) return;
    uint32_t next_id = end + wbase + (incl - nin);  // level + 1 starts right after this level
    Bvh4Node o;
    uint32_t imask = 0;
    for (int j = 0; j < cnt_s; ++j) {
        int32_t r = ref[j];
        if (r >= 0) {
            const uint32_t id = next_id++;
            src4[id] = r;
            bdep[id] = rd[j];
            r = (int32_t)id;
            imask |= 1u << j;
        }
        put_slot(o, j, box[j], r);
    }
    const float eb[6] = {EMPTY_BOX, EMPTY_BOX, EMPTY_BOX, EMPTY_BOX, EMPTY_BOX, EMPTY_BOX};
    o.nchild = (uint32_t)cnt_s;
    for (int j = cnt_s; j < BVH_W; ++j) put_slot(o, j, eb, 0);
    o.pad[0] = n.pad0;  // split axis of the binary root (children are in its in-order)
    o.pad[1] = imask;   // children that are 4-wide nodes
    o.pad[2] = 0;
    out[i] = o;
}

}  // namespace

// Surface-area-optimal 4-wide collapse (dynamic programming over the binary tree, after Ylitie, Karras
// and Laine, "Efficient Incoherent Ray Traversal on GPUs Through Compressed Wide BVHs", HPG 2017 §4),
// gvrt_accel_params.collapse = 1 on the host (builders 0, 1, 3).  With one proxy per leaf the leaf term of the SAH is the same
// for every collapse, so the DP minimises the summed surface area of the 4-wide nodes:
//   F(leaf, k) = 0;  F(n, 1) = C(n) = SA(n) + min_j F(c0, j) + F(c1, 4 - j);
//   F(n, k) = min(F(n, k - 1), min_j F(c0, j) + F(c1, k - j))   (k = 2..4)
// and the tree is rebuilt top-down, breadth-first, children in the binary in-order (split-axis order).
static float host_area(const float* b) {
    const float ex = b[3] - b[0], ey = b[4] - b[1], ez = b[5] - b[2];
    return ex * ey + ey * ez + ez * ex;
}

// Binned-SAH binary BVH on the host (builder = 3, the checker of the device build): the trace-quality build of a
// static scene, the counterpart of the reference's BLAS built once with
// VK_BUILD_ACCELERATION_STRUCTURE_PREFER_FAST_TRACE_BIT_KHR (VulkanFullRT.cpp:575-787).  Top-down over
// the Morton-ordered leaf boxes: per range, 32 centroid bins on each axis, the split of least
// SA(left)·n(left) + SA(right)·n(right); an undecidable range (equal centroids) splits at its middle.
// Nodes are written depth-first from the root (id 0) in the BvhNode layout the collapse reads: child 0 on
// the lower side of the recorded split axis, leaves as ~(leaf index).
// keep != null: the tree stays on the host for the host-side collapse (no upload / download round trip)
static gvrt_status host_sah_build(gvrt_context* c, uint64_t m, const float* d_lboxes, int32_t* root,
                                  std::vector<BvhNode>* keep, uint32_t dmax) {
    std::vector<float> bx(6 * m);
    GVRT_HIP(c, hipMemcpyAsync(bx.data(), d_lboxes, 24 * m, hipMemcpyDeviceToHost, c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    std::vector<uint32_t> idx(m);
    std::vector<float> cen(3 * m);
    for (uint64_t i = 0; i < m; ++i) {
        idx[i] = (uint32_t)i;
        for (int a = 0; a < 3; ++a) cen[3 * i + a] = 0.5f * (bx[6 * i + a] + bx[6 * i + 3 + a]);
    }
    struct Box {
        float lo[3], hi[3];
        void reset() {
            for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
        }
        void grow(const float* b) {
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b[a]); hi[a] = std::max(hi[a], b[3 + a]); }
        }
        void grow(const Box& b) {
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], b.lo[a]); hi[a] = std::max(hi[a], b.hi[a]); }
        }
        float area() const {
            if (!(hi[0] >= lo[0])) return 0.0f;
            const float ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
            return ex * ey + ey * ez + ez * ex;
        }
    };
    // 32 bins per axis, as the device build (gvrt_sah.hip); 64 / 128 bins or an exact sweep over the sorted
    // centroids for small ranges measured within noise
    constexpr int NB = 32, NBMAX = NB;
    // ids by range: the node of [b, e) is id, its left subtree (L leaves) takes ids id + 1 .. id + L - 1
    // and the right child is id + L — independent of the order ranges are processed in, so subtrees
    // build on several threads with the same result
    std::vector<BvhNode> nodes(m - 1);
    struct Task { uint32_t b, e, node, d; };  // d: binary depth of the range's node (root 1)
    auto split = [&](const Task& t, Task* kids, int& nk) {
        uint32_t mid = t.b + (t.e - t.b) / 2;
        int axis = 0;
        float cl[3] = {INFINITY, INFINITY, INFINITY}, ch[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = t.b; i < t.e; ++i)
            for (int a = 0; a < 3; ++a) {
                cl[a] = std::min(cl[a], cen[3 * idx[i] + a]);
                ch[a] = std::max(ch[a], cen[3 * idx[i] + a]);
            }
        int best_axis = -1, best_split = 0;
        uint32_t best_nl = 0;
        float best_cost = INFINITY;
        for (int a = 0; a < 3; ++a) {
            const float ext = ch[a] - cl[a];
            if (!(ext > 0.0f)) continue;
            const float sc = NB / ext;
            if (!(sc < INFINITY)) continue;  // extent too small to bin
            Box bb[NBMAX];
            uint32_t bn[NBMAX] = {};
            for (int k = 0; k < NB; ++k) bb[k].reset();
            for (uint32_t i = t.b; i < t.e; ++i) {
                const int k = std::min(NB - 1, (int)((cen[3 * idx[i] + a] - cl[a]) * sc));
                bb[k].grow(&bx[6ull * idx[i]]);
                ++bn[k];
            }
            float rarea[NBMAX];
            uint32_t rcnt[NBMAX];
            Box acc;
            acc.reset();
            uint32_t n = 0;
            for (int k = NB - 1; k > 0; --k) {
                acc.grow(bb[k]);
                n += bn[k];
                rarea[k] = acc.area();
                rcnt[k] = n;
            }
            acc.reset();
            n = 0;
            for (int k = 0; k < NB - 1; ++k) {  // split between bins k and k + 1
                acc.grow(bb[k]);
                n += bn[k];
                if (n == 0 || rcnt[k + 1] == 0) continue;
                const float cost = acc.area() * (float)n + rarea[k + 1] * (float)rcnt[k + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_split = k;
                    best_nl = n;
                }
            }
        }
        // depth budget (SAH_DEPTH_MAX, as the device build): halve instead of a split whose larger side could not
        // finish in budget
        if (best_axis >= 0 && !sah_split_in_budget(t.d, best_nl, (t.e - t.b) - best_nl, dmax)) best_axis = -1;
        if (best_axis >= 0) {
            axis = best_axis;
            const float sc = NB / (ch[axis] - cl[axis]);
            // stable: the device build (gvrt_sah.hip) partitions by a prefix count and must agree
            const auto it = std::stable_partition(idx.begin() + t.b, idx.begin() + t.e, [&](uint32_t p) {
                return std::min(NB - 1, (int)((cen[3 * p + axis] - cl[axis]) * sc)) <= best_split;
            });
            mid = (uint32_t)(it - idx.begin());
        }  // else every centroid equal, or the depth budget: halve the range
        Box lb, rb;
        lb.reset();
        rb.reset();
        for (uint32_t i = t.b; i < mid; ++i) lb.grow(&bx[6ull * idx[i]]);
        for (uint32_t i = mid; i < t.e; ++i) rb.grow(&bx[6ull * idx[i]]);
        BvhNode& nd = nodes[t.node];
        float* nf = reinterpret_cast<float*>(&nd);
        for (int a = 0; a < 3; ++a) {
            nf[a] = lb.lo[a];
            nf[3 + a] = lb.hi[a];
            nf[6 + a] = rb.lo[a];
            nf[9 + a] = rb.hi[a];
        }
        const uint32_t L = mid - t.b;
        nk = 0;
        if (L == 1) nd.c0 = ~(int32_t)idx[t.b];
        else { nd.c0 = (int32_t)(t.node + 1); kids[nk++] = {t.b, mid, t.node + 1, t.d + 1}; }
        if (t.e - mid == 1) nd.c1 = ~(int32_t)idx[mid];
        else { nd.c1 = (int32_t)(t.node + L); kids[nk++] = {mid, t.e, t.node + L, t.d + 1}; }
        nd.pad0 = (uint32_t)axis;
        nd.pad1 = 0;
    };
    auto subtree = [&](Task root) {
        std::vector<Task> st{root};
        Task kids[2];
        int nk = 0;
        while (!st.empty()) {
            const Task t = st.back();
            st.pop_back();
            split(t, kids, nk);
            for (int k = 0; k < nk; ++k) st.push_back(kids[k]);
        }
    };
    // the top of the tree breadth-first on this thread until there is work for every thread, then the
    // subtrees on a small pool
    const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<Task> front{{0u, (uint32_t)m, 0u, 1u}}, next;
    while (!front.empty() && front.size() < 4 * nth) {
        next.clear();
        for (const Task& t : front) {
            if (t.e - t.b < 4096) { next.push_back(t); continue; }
            Task kids[2];
            int nk = 0;
            split(t, kids, nk);
            for (int k = 0; k < nk; ++k) next.push_back(kids[k]);
        }
        if (next.size() == front.size()) { front.swap(next); break; }  // only small ranges left
        front.swap(next);
    }
    std::atomic<size_t> cursor{0};
    std::vector<std::thread> pool;
    for (unsigned w = 0; w < nth; ++w)
        pool.emplace_back([&]() {
            for (size_t i; (i = cursor.fetch_add(1)) < front.size();) subtree(front[i]);
        });
    for (auto& th : pool) th.join();
    *root = 0;
    // the binary tree also goes to the device (gvrt_read_accel compares it with the device build's)
    GVRT_HIP(c, hipMemcpyAsync(c->d_nodes, nodes.data(), sizeof(BvhNode) * nodes.size(), hipMemcpyHostToDevice,
                               c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    if (keep) keep->swap(nodes);
    return GVRT_OK;
}

static gvrt_status host_dp_collapse(gvrt_context* c, int32_t root, uint64_t m, std::vector<BvhNode>* host_tree,
                                    uint32_t* depth_out,
                                    uint32_t* depth4_out, uint64_t* n4_out) {
    const uint64_t ni = m - 1;
    std::vector<BvhNode> bn;
    if (host_tree && host_tree->size() == ni) {
        bn.swap(*host_tree);
    } else {
        bn.resize(ni);
        GVRT_HIP(c, hipMemcpyAsync(bn.data(), c->d_nodes, sizeof(BvhNode) * ni, hipMemcpyDeviceToHost, c->stream));
    }
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    // F[n][k-1], k = 1..4, bottom-up by an explicit post-order walk
    std::vector<float> F(4 * ni, 0.0f);
    auto f = [&](int32_t x, int k) -> float { return x < 0 ? 0.0f : F[4 * (uint64_t)x + (k - 1)]; };
    std::vector<std::pair<int32_t, uint32_t>> st;  // (node, binary depth)
    std::vector<uint8_t> seen(ni, 0);
    uint32_t maxd = 0;
    st.push_back({root, 1});
    while (!st.empty()) {
        const auto [x, dx] = st.back();
        const BvhNode& n = bn[x];
        if (!seen[x]) {
            seen[x] = 1;
            if (n.c0 >= 0) st.push_back({n.c0, dx + 1}); else maxd = std::max(maxd, dx + 1);
            if (n.c1 >= 0) st.push_back({n.c1, dx + 1}); else maxd = std::max(maxd, dx + 1);
            continue;
        }
        st.pop_back();
        const float* nb = reinterpret_cast<const float*>(&n);
        float ub[6];
        for (int k = 0; k < 3; ++k) {
            ub[k] = std::min(nb[k], nb[6 + k]);
            ub[3 + k] = std::max(nb[3 + k], nb[9 + k]);
        }
        float best4 = INFINITY;
        for (int j = 1; j < 4; ++j) best4 = std::min(best4, f(n.c0, j) + f(n.c1, 4 - j));
        float* Fx = &F[4 * (uint64_t)x];
        Fx[0] = host_area(ub) + best4;
        for (int k = 2; k <= 4; ++k) {
            float b = Fx[k - 2];
            for (int j = 1; j < k; ++j) b = std::min(b, f(n.c0, j) + f(n.c1, k - j));
            Fx[k - 1] = b;
        }
    }
    // frontier of node x (box bx) in at most k pieces
    struct Piece { int32_t ref; float box[6]; };
    std::function<void(int32_t, const float*, int, std::vector<Piece>&)> expand =
        [&](int32_t x, const float* bx, int k, std::vector<Piece>& out) {
            if (x < 0 || k == 1) {
                Piece p;
                p.ref = x;
                std::memcpy(p.box, bx, 24);
                out.push_back(p);
                return;
            }
            if (F[4 * (uint64_t)x + (k - 1)] == F[4 * (uint64_t)x + (k - 2)]) {
                expand(x, bx, k - 1, out);
                return;
            }
            const BvhNode& n = bn[x];
            const float* nb = reinterpret_cast<const float*>(&n);
            int bj = 1;
            float bv = INFINITY;
            for (int j = 1; j < k; ++j) {
                const float v = f(n.c0, j) + f(n.c1, k - j);
                if (v < bv) bv = v, bj = j;
            }
            expand(n.c0, nb, bj, out);
            expand(n.c1, nb + 6, k - bj, out);
        };
    std::vector<Bvh4Node> outn;
    outn.reserve(ni);
    std::vector<int32_t> queue{root};
    std::vector<uint32_t> qlev{0};
    uint32_t maxlev = 0;
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const int32_t x = queue[qi];
        const BvhNode& n = bn[x];
        const float* nb = reinterpret_cast<const float*>(&n);
        int bj = 1;
        float bv = INFINITY;
        for (int j = 1; j < 4; ++j) {
            const float v = f(n.c0, j) + f(n.c1, 4 - j);
            if (v < bv) bv = v, bj = j;
        }
        std::vector<Piece> ps;
        expand(n.c0, nb, bj, ps);
        expand(n.c1, nb + 6, 4 - bj, ps);
        Bvh4Node o{};
        uint32_t imask = 0;
        for (size_t j = 0; j < ps.size(); ++j) {
            int32_t r = ps[j].ref;
            if (r >= 0) {
                r = (int32_t)queue.size();
                queue.push_back(ps[j].ref);
                qlev.push_back(qlev[qi] + 1);
                maxlev = std::max(maxlev, qlev[qi] + 1);
                imask |= 1u << j;
            }
            const float* b = ps[j].box;
            o.box[j][0] = b[0]; o.box[j][1] = b[3];
            o.box[j][2] = b[1]; o.box[j][3] = b[4];
            o.box[j][4] = b[2]; o.box[j][5] = b[5];
            o.child[j] = r;
        }
        for (size_t j = ps.size(); j < (size_t)BVH_W; ++j) {
            for (int k = 0; k < 6; ++k) o.box[j][k] = EMPTY_BOX;
            o.child[j] = 0;
        }
        o.nchild = (uint32_t)ps.size();
        o.pad[0] = n.pad0;
        o.pad[1] = imask;
        o.pad[2] = 0;
        outn.push_back(o);
    }
    GVRT_HIP(c, hipMemcpyAsync(c->d_nodes4, outn.data(), sizeof(Bvh4Node) * outn.size(), hipMemcpyHostToDevice,
                               c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    *depth_out = maxd;
    *depth4_out = maxlev + 1;
    *n4_out = outn.size();
    return GVRT_OK;
}


gvrt_status gvrt_launch_build_accel(gvrt_context* c, const gvrt_accel_params& ap) {
    const int64_t mp = (int64_t)c->m;  // proxies (survivors)
    gvrt_dfree(c, (void**)&c->d_recs);
    gvrt_dfree(c, (void**)&c->d_sh);
    gvrt_dfree(c, (void**)&c->d_nodes);
    gvrt_dfree(c, (void**)&c->d_nodes4);
    gvrt_dfree(c, (void**)&c->d_leaf_src);
    gvrt_dfree(c, (void**)&c->d_leaf_aux);
    c->n_nodes4 = 0;
    c->n_leaves = 0;
    c->split_cells = 0;
    c->accel = false;
    c->depth = 0;
    if (mp == 0) {
        c->accel = true;
        c->stats.bvh_nodes = 0;
        c->stats.bvh_leaves = 0;
        c->stats.bvh_depth = 0;
        c->stats.bvh_depth4 = 0;
        c->stats.bvh_builder = ap.builder;
        c->stats.bvh_depth4_rebuilt = 0;
        return GVRT_OK;
    }
    if (mp > 0x7FFFFFFFll) return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "more than 2^31-1 survivors");
    gvrt_status s;

    // scratch
    uint32_t *bnd = nullptr, *vals = nullptr, *vals2 = nullptr, *dep = nullptr;
    float *stab = nullptr, *bpart = nullptr;
    float** dlv = nullptr;
    uint64_t *keys = nullptr, *keys2 = nullptr;
    int32_t *lpar = nullptr, *npar = nullptr;
    float* lboxes = nullptr;
    void* tmp = nullptr;
    float* pbox = nullptr;  // split pieces
    uint4* paux = nullptr;
    uint64_t *pcnt = nullptr, *poff = nullptr;
    void* ptmp = nullptr;
    auto cleanup = [&]() {
        gvrt_dfree(c, (void**)&bnd);
        gvrt_dfree(c, (void**)&keys);
        gvrt_dfree(c, (void**)&vals);
        gvrt_dfree(c, (void**)&keys2);
        gvrt_dfree(c, (void**)&vals2);
        gvrt_dfree(c, (void**)&stab);
        gvrt_dfree(c, (void**)&dlv);
        gvrt_dfree(c, (void**)&bpart);
        gvrt_dfree(c, (void**)&dep);
        gvrt_dfree(c, (void**)&lpar);
        gvrt_dfree(c, (void**)&npar);
        gvrt_dfree(c, (void**)&lboxes);
        gvrt_dfree(c, &tmp);
        gvrt_dfree(c, (void**)&pbox);
        gvrt_dfree(c, (void**)&paux);
        gvrt_dfree(c, (void**)&pcnt);
        gvrt_dfree(c, (void**)&poff);
        gvrt_dfree(c, &ptmp);
    };
#define TRY(x)                   \
    do {                         \
        if ((s = (x)) != GVRT_OK) { \
            cleanup();           \
            return s;            \
        }                        \
    } while (0)
#define TRYH(x, what)                                   \
    do {                                                \
        hipError_t _e = (x);                            \
        if (_e != hipSuccess) {                         \
            cleanup();                                  \
            return gvrt_hip_check(c, _e, what);         \
        }                                               \
    } while (0)

    // ---- optional split into grid-cell pieces (SplitBLAS analogue): the BVH leaves become pieces
    int64_t m = mp;  // leaves
    const float* boxes_in = c->d_boxes_c;
    if (ap.split_cells > 0) {
        const unsigned pb = (unsigned)((mp + 255) / 256), prb = pb < 1024 ? pb : 1024;
        TRY(gvrt_dalloc(c, (void**)&bnd, 32));
        TRY(gvrt_dalloc(c, (void**)&bpart, 24ull * prb));
        const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
        TRYH(hipMemcpyAsync(bnd, init, 24, hipMemcpyHostToDevice, c->stream), "bounds init");
        hipLaunchKernelGGL(k_bounds<false>, dim3(prb), dim3(256), 0, c->stream, (uint64_t)mp, c->d_boxes_c, bpart);
        hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(256), 0, c->stream, prb, bpart, bnd);
        uint32_t hb[6];
        TRYH(hipMemcpyAsync(hb, bnd, 24, hipMemcpyDeviceToHost, c->stream), "scene box");
        TRYH(hipStreamSynchronize(c->stream), "sync");
        // grid of SplitBLAS.cpp:103-112: SCENE_EPSILON 1e-4 margins, N cells on the longest axis
        Grid g{};
        float size[3], maxs = 0.0f;
        for (int a = 0; a < 3; ++a) {
            g.mn[a] = ord2f(hb[a]) - 1e-4f;
            size[a] = (ord2f(hb[3 + a]) + 1e-4f) - g.mn[a];
            maxs = size[a] > maxs ? size[a] : maxs;
        }
        g.size = maxs / (float)ap.split_cells;
        g.inv = 1.0f / g.size;
        for (int a = 0; a < 3; ++a)
            g.n[a] = size[a] == maxs ? ap.split_cells : (uint32_t)(size[a] / g.size) + 1u;
        TRY(gvrt_dalloc(c, (void**)&pcnt, 8ull * (mp + 1)));
        TRY(gvrt_dalloc(c, (void**)&poff, 8ull * (mp + 1)));
        hipLaunchKernelGGL(k_piece_count, dim3((unsigned)((mp + 1 + 255) / 256)), dim3(256), 0, c->stream, (uint64_t)mp,
                           c->d_boxes_c, g, ap.split_min_span, pcnt);
        size_t pt = 0;
        TRYH(hipcub::DeviceScan::ExclusiveSum(nullptr, pt, pcnt, poff, (int)(mp + 1), c->stream), "scan size");
        TRY(gvrt_dalloc(c, &ptmp, pt ? pt : 16));
        TRYH(hipcub::DeviceScan::ExclusiveSum(ptmp, pt, pcnt, poff, (int)(mp + 1), c->stream), "scan");
        uint64_t np = 0;
        TRYH(hipMemcpyAsync(&np, poff + mp, 8, hipMemcpyDeviceToHost, c->stream), "pieces");
        TRYH(hipStreamSynchronize(c->stream), "sync");
        if (np == 0 || np > (1ull << 27)) {  // (memory: ~300 B of build scratch per piece)
            cleanup();
            return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "split produced an unsupported number of pieces");
        }
        // no proxy split (every one inside one cell, or below split_min_span): the unsplit build, no cell tests
        if (np != (uint64_t)mp) {
            m = np;
            TRY(gvrt_dalloc(c, (void**)&pbox, 24ull * m));
            TRY(gvrt_dalloc(c, (void**)&paux, 16ull * m));
            hipLaunchKernelGGL(k_piece_emit, dim3(pb), dim3(256), 0, c->stream, (uint64_t)mp, c->d_boxes_c, g,
                               ap.split_min_span, c->box_pad_abs, poff, pbox, paux);
            TRYH(hipGetLastError(), "k_piece_emit");
            boxes_in = pbox;
            c->split_cells = ap.split_cells;
            for (int a = 0; a < 3; ++a) {
                c->grid_min[a] = g.mn[a];
                c->grid_n[a] = g.n[a];
            }
            c->grid_inv = g.inv;
        }
        gvrt_dfree(c, (void**)&bnd);
        gvrt_dfree(c, (void**)&bpart);
    }
    c->n_leaves = (uint64_t)m;

    const int64_t ninternal = m > 1 ? m - 1 : 1;
    TRY(gvrt_dalloc(c, (void**)&c->d_recs, sizeof(RenderRec) * m));
    TRY(gvrt_dalloc(c, (void**)&c->d_sh, 192ull * m));
    if (c->split_cells) TRY(gvrt_dalloc(c, (void**)&c->d_leaf_aux, 16ull * m));
    TRY(gvrt_dalloc(c, (void**)&c->d_nodes, sizeof(BvhNode) * ninternal));
    TRY(gvrt_dalloc(c, (void**)&c->d_leaf_src, 4ull * m));

    TRY(gvrt_dalloc(c, (void**)&bnd, 32));
    TRY(gvrt_dalloc(c, (void**)&keys, 8ull * m));
    TRY(gvrt_dalloc(c, (void**)&vals, 4ull * m));
    TRY(gvrt_dalloc(c, (void**)&keys2, 8ull * m));
    TRY(gvrt_dalloc(c, (void**)&vals2, 4ull * m));
    // sparse-table levels 1 .. L-1 (level 0 = the leaf boxes themselves)
    int nlev = 1;
    while (((uint64_t)1 << nlev) <= (uint64_t)m) ++nlev;
    std::vector<const float*> hlv(nlev, nullptr);
    if (nlev > 1) TRY(gvrt_dalloc(c, (void**)&stab, 24ull * m * (nlev - 1)));
    TRY(gvrt_dalloc(c, (void**)&dlv, sizeof(float*) * nlev));
    TRY(gvrt_dalloc(c, (void**)&dep, 4 * (8 + 128)));  // collapse control + per-level counts
    TRY(gvrt_dalloc(c, (void**)&lpar, 4ull * m));
    TRY(gvrt_dalloc(c, (void**)&npar, 4ull * ninternal));
    TRY(gvrt_dalloc(c, (void**)&lboxes, 24ull * m));

    const unsigned blocks = (unsigned)((m + 255) / 256);
    const unsigned rblocks = blocks < 1024 ? blocks : 1024;
    TRY(gvrt_dalloc(c, (void**)&bpart, 24ull * rblocks));

    size_t tmp_bytes = 0;
    TRYH(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys2, vals, vals2, (int)m, 0, 63, c->stream),
         "SortPairs size");
    TRY(gvrt_dalloc(c, &tmp, tmp_bytes ? tmp_bytes : 16));
    // the 4-wide nodes: upper bound of one per binary node (allocated before the timed region)
    if (m > 1) TRY(gvrt_dalloc(c, (void**)&c->d_nodes4, sizeof(Bvh4Node) * (m - 1)));

    TRYH(hipEventRecord(c->ev0, c->stream), "event");
    const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
    TRYH(hipMemcpyAsync(bnd, init, 24, hipMemcpyHostToDevice, c->stream), "bounds init");
    hipLaunchKernelGGL(k_bounds<true>, dim3(rblocks), dim3(256), 0, c->stream, (uint64_t)m, boxes_in, bpart);
    hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(256), 0, c->stream, rblocks, bpart, bnd);
    hipLaunchKernelGGL(k_morton, dim3(blocks), dim3(256), 0, c->stream, (uint64_t)m, boxes_in, bnd, keys, vals);
    TRYH(hipGetLastError(), "k_morton");
    TRYH(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys2, vals, vals2, (int)m, 0, 63, c->stream),
         "SortPairs");
    hipLaunchKernelGGL(k_permute, dim3(blocks), dim3(256), 0, c->stream, (uint64_t)m, vals2, c->d_recs_c, c->d_sh48,
                       boxes_in, paux, c->d_recs, c->d_sh, lboxes, c->d_leaf_src,
                       reinterpret_cast<uint4*>(c->d_leaf_aux));
    TRYH(hipGetLastError(), "k_permute");
    if (m == 1) {
        // single proxy: one 4-wide root with one leaf slot
        Bvh4Node root{};
        float hb[6];
        TRYH(hipMemcpyAsync(hb, lboxes, 24, hipMemcpyDeviceToHost, c->stream), "leaf box");
        TRYH(hipStreamSynchronize(c->stream), "sync");
        for (int k = 0; k < BVH_W; ++k) {
            const float* b = k == 0 ? hb : nullptr;
            for (int a = 0; a < 3; ++a) {
                root.box[k][2 * a] = b ? b[a] : EMPTY_BOX;
                root.box[k][2 * a + 1] = b ? b[3 + a] : EMPTY_BOX;
            }
            root.child[k] = k == 0 ? ~0 : 0;
        }
        root.nchild = 1;
        root.pad[0] = root.pad[1] = root.pad[2] = 0;
        TRY(gvrt_dalloc(c, (void**)&c->d_nodes4, sizeof(Bvh4Node)));
        TRYH(hipMemcpyAsync(c->d_nodes4, &root, sizeof(root), hipMemcpyHostToDevice, c->stream), "root");
        c->n_nodes4 = 1;
        c->depth = 1;
        c->depth4 = 1;
    } else {
        TRYH(hipMemsetAsync(dep, 0, 4, c->stream), "memset");
        const bool ploc = ap.builder == 1;  // PLOC: measured 3 % slower to render (more visits), see DESIGN.md
        // binned SAH: on the device (builder 2), or the same algorithm on the host (builder 3: the device
        // build's checker, tests/test_gpu_sah.py)
        const bool sah_host = !ploc && ap.builder == 3;
        const bool sah_dev = !ploc && !sah_host && ap.builder == 2;
        const bool dp = ap.collapse == 1;
        std::vector<BvhNode> htree;  // SAH tree kept on the host for the DP collapse
        // the SAH builds' depth budget (gvrt_accel_params.depth_budget: 0 = SAH_DEPTH_MAX); one the leaves cannot
        // meet (1 + ceil(log2 m) levels are needed) is refused
        const uint32_t dmax = ap.depth_budget ? ap.depth_budget : SAH_DEPTH_MAX;
        if ((sah_host || sah_dev) && 1u + ceil_log2((uint32_t)m) > dmax)
            TRY(gvrt_fail(c, GVRT_ERR_INVALID_ARG, "depth_budget below 1 + ceil(log2(leaves))"));
        int32_t root = 0;
        uint32_t sah_depth = 0, sah_d4 = 0;
        uint64_t sah_n4 = 0;
        if (ploc) {
            uint32_t iters = 0;
            TRY(gvrt_ploc_build(c, (uint32_t)m, lboxes, c->d_nodes, lpar, npar, &root, &iters));
        } else if (sah_host) {
            TRY(host_sah_build(c, (uint64_t)m, lboxes, &root, dp ? &htree : nullptr, dmax));
        } else if (sah_dev) {
            TRY(gvrt_sah_build_device(c, (uint64_t)m, lboxes, c->d_nodes, dp ? c->d_nodes4 : nullptr, &sah_depth,
                                      &sah_n4, &sah_d4, dmax));
        } else {
            // leaf-range union table, then the hierarchy with its child boxes in one pass (no refit)
            hlv[0] = lboxes;
            for (int k = 1; k < nlev; ++k) {
                hlv[k] = stab + 6ull * m * (k - 1);
                const uint64_t half = (uint64_t)1 << (k - 1);
                const uint64_t cnt = (uint64_t)m - 2 * half + 1;
                hipLaunchKernelGGL(k_sparse_level, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, c->stream,
                                   (uint64_t)m, half, hlv[k - 1], const_cast<float*>(hlv[k]));
            }
            TRYH(hipMemcpyAsync(dlv, hlv.data(), sizeof(float*) * nlev, hipMemcpyHostToDevice, c->stream), "levels");
            const unsigned iblocks = (unsigned)((m - 1 + 255) / 256);
            hipLaunchKernelGGL(k_karras, dim3(iblocks), dim3(256), 0, c->stream, m, keys2, c->d_nodes, lpar, npar,
                               (const float* const*)dlv);
        }
        const int64_t ni = m - 1;
        TRYH(hipGetLastError(), "k_karras");
        if (dp && sah_dev) {  // collapsed by gvrt_sah_build_device
            c->depth = sah_depth;
            c->depth4 = sah_d4;
            c->n_nodes4 = sah_n4;
        } else if (dp) {
            uint32_t d2 = 0, d4 = 0;
            uint64_t n4 = 0;
            TRY(host_dp_collapse(c, root, m, &htree, &d2, &d4, &n4));
            c->depth = d2;
            c->depth4 = d4;
            c->n_nodes4 = n4;
        } else {
            // ---- greedy surface-area collapse, level by level (upper bound: one 4-wide node per binary node)
            int32_t* src4 = lpar;                                  // lpar (m entries) is free after the hierarchy
            uint32_t* bdep = reinterpret_cast<uint32_t*>(keys);    // the sort keys are free too (8m bytes)
            uint32_t* cnt = dep + 8;                               // per-level counts (MAX_LEVELS)
            uint32_t* ctl = dep;                                   // {max 4-wide level, max binary leaf depth}
            constexpr uint32_t MAX_LEVELS = 120;
            TRYH(hipMemsetAsync(dep, 0, 4 * (8 + MAX_LEVELS + 1), c->stream), "ctl");
            const uint32_t one = 1u;
            TRYH(hipMemcpyAsync(cnt, &one, 4, hipMemcpyHostToDevice, c->stream), "cnt0");
            TRYH(hipMemcpyAsync(src4, &root, 4, hipMemcpyHostToDevice, c->stream), "src4");
            TRYH(hipMemcpyAsync(bdep, &one, 4, hipMemcpyHostToDevice, c->stream), "bdep");
            // launches in chunks of 8 levels; after each chunk the count of the next level says whether
            // the tree goes deeper (one small readback per chunk instead of a depth census)
            uint64_t width = 1;
            uint32_t lv = 0;
            while (lv < MAX_LEVELS) {
                const uint32_t stop = std::min(lv + 8, MAX_LEVELS);
                for (; lv < stop; ++lv) {
                    const uint64_t w = width < (uint64_t)ni ? width : (uint64_t)ni;
                    hipLaunchKernelGGL(k_collapse_level, dim3((unsigned)((w + 255) / 256)), dim3(256), 0, c->stream,
                                       c->d_nodes, src4, bdep, cnt, ctl, lv, c->d_nodes4);
                    width = width * BVH_W < (uint64_t)ni ? width * BVH_W : (uint64_t)ni;
                }
                uint32_t pending = 0;
                TRYH(hipMemcpyAsync(&pending, cnt + lv, 4, hipMemcpyDeviceToHost, c->stream), "cnt");
                TRYH(hipStreamSynchronize(c->stream), "sync");
                if (pending == 0) break;
            }
            TRYH(hipGetLastError(), "k_collapse_level");
            if (lv >= MAX_LEVELS) TRY(gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "4-wide collapse deeper than 120 levels"));
            uint32_t hc[2];
            std::vector<uint32_t> hcnt(MAX_LEVELS);
            TRYH(hipMemcpyAsync(hc, ctl, 8, hipMemcpyDeviceToHost, c->stream), "ctl");
            TRYH(hipMemcpyAsync(hcnt.data(), cnt, 4 * MAX_LEVELS, hipMemcpyDeviceToHost, c->stream), "cnt");
            TRYH(hipStreamSynchronize(c->stream), "sync");
            uint32_t total = 0;
            for (uint32_t v : hcnt) total += v;
            c->depth = hc[1];
            c->depth4 = hc[0] + 1;
            c->n_nodes4 = total;
        }
    }
    if (c->split_cells && c->n_nodes4 && c->d_leaf_aux) {
        hipLaunchKernelGGL(k_mark_pieces, dim3((unsigned)((c->n_nodes4 + 255) / 256)), dim3(256), 0, c->stream,
                           (uint64_t)c->n_nodes4, c->d_nodes4, reinterpret_cast<const uint4*>(c->d_leaf_aux));
        TRYH(hipGetLastError(), "k_mark_pieces");
    }
    TRYH(hipEventRecord(c->ev1, c->stream), "event");
    TRYH(hipStreamSynchronize(c->stream), "sync");
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
    c->stats.accel_ms = ms;
    cleanup();
#undef TRY
#undef TRYH
    // the traversal pushes at most BVH_W - 1 entries per level.  The SAH builds (2, 3) keep the depth budget by
    // construction (SAH_DEPTH_MAX); an LBVH or PLOC tree too deep for the stack (clustered, multi-scale geometry) is
    // rebuilt by the device SAH build with the same collapse and split options instead of refusing the scene
    if ((BVH_W - 1) * c->depth4 + 2 > (uint32_t)STACK_DEPTH) {
        if (ap.builder == 0 || ap.builder == 1) {
            gvrt_accel_params q = ap;
            q.builder = 2;
            const uint32_t d4 = c->depth4;
            const gvrt_status s2 = gvrt_launch_build_accel(c, q);
            c->stats.bvh_depth4_rebuilt = d4;
            return s2;
        }
        return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "BVH deeper than the render kernel's traversal stack");
    }
    c->stats.bvh_nodes = c->n_nodes4;
    c->stats.bvh_leaves = c->n_leaves;
    c->stats.bvh_depth = c->depth;
    c->stats.bvh_depth4 = c->depth4;
    c->stats.bvh_builder = ap.builder;
    c->stats.bvh_depth4_rebuilt = 0;
    c->accel = true;
    return GVRT_OK;
}
