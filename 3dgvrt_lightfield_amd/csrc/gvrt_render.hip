// gvrt_render.hip — Particle Rendering pass on gfx950.
//
// Replaces the per-pixel ray-march of shaders/glsl/VulkanFullRT/particleRendering.comp:117-191
// (ray query), raygen.rgen:303-383 + anyhit.rahit:40-71 (RT pipeline) and
// raygenGaussianLightField.rgen:114-202 (multi-camera light field), and the driver's BVH
// traversal behind traceRayEXT / rayQueryProceedEXT.
//
// Mapping to CDNA4: one wave64 = one 8x8 pixel tile (one lane per ray), four tiles per
// 256-thread workgroup.  Traversal is wave-uniform (packet traversal): node and leaf records
// are addressed by a wave-uniform index and fetched with scalar loads (one s_load_dwordx16 per
// 64-B node / record), every lane clips its own ray against both child boxes, and a ballot
// decides which children the packet descends into; the far child goes on a per-wave LDS stack.
// Leaves are clipped against the analytic icosahedron (10 antipodal slab pairs in the kernel
// frame), which yields the same two crossings (entry and exit face, Q1) as the reference's
// 20-triangle proxy.  Each lane keeps a 16-slot register k-buffer (compareAndSwapHitPayloadValue
// chain, anyhit.rahit:29-71); a full buffer shrinks that lane's culling distance as the
// driver's tmax does.  After each traversal round every lane composites its hits front to back
// (processHit, gaussianfunctions.glsl:153-229) with the SH basis of its ray direction
// precomputed once per ray (the reference's scalar basis factors, same summation order).
//
// Modes: LITERAL = every crossing enters the k-buffer, rounds exactly as the reference
// (16 per trace, `last` advanced by rejected hits too).  FAST = only accepted crossings enter the
// k-buffer; with an exclusive tmin the composited sequence, and therefore the image, is the
// same (rejected crossings only ever advanced `last`), while far fewer rounds are needed.
#include "gvrt_internal.h"

using namespace gvrt;

namespace {

// 3dgs.glsl:34-49
constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f, SH_C2_2 = 0.31539156525252005f,
                SH_C2_3 = -1.0925484305920792f, SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f, SH_C3_1 = 2.890611442640554f, SH_C3_2 = -0.4570457994644658f,
                SH_C3_3 = 0.3731763325901154f, SH_C3_4 = -0.4570457994644658f, SH_C3_5 = 1.445305721320277f,
                SH_C3_6 = -0.5900435899266435f;

__device__ inline bool box_hit(float lx, float ly, float lz, float hx, float hy, float hz, f3 o, f3 inv, float t0,
                               float t1, float& tenter) {
    const float ax = (lx - o.x) * inv.x, bx = (hx - o.x) * inv.x;
    const float ay = (ly - o.y) * inv.y, by = (hy - o.y) * inv.y;
    const float az = (lz - o.z) * inv.z, bz = (hz - o.z) * inv.z;
    const float tn = fmaxf(fmaxf(t0, fminf(ax, bx)), fmaxf(fminf(ay, by), fminf(az, bz)));
    const float tf = fminf(fminf(t1, fmaxf(ax, bx)), fminf(fmaxf(ay, by), fmaxf(az, bz)));
    tenter = tn;
    // culling only: a relative slack so rounding can never drop a crossing
    return tn <= tf + 2e-6f * fabsf(tf);
}

template <int K>
__device__ inline void kb_insert(float t, uint32_t id, float al, float (&kt)[K], uint32_t (&kid)[K], float (&ka)[K]) {
    if (!(t < kt[K - 1])) return;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const bool sw = t < kt[i];
        const float tt = kt[i];
        const uint32_t ti = kid[i];
        const float ta = ka[i];
        kt[i] = sw ? t : tt;
        kid[i] = sw ? id : ti;
        ka[i] = sw ? al : ta;
        t = sw ? tt : t;
        id = sw ? ti : id;
        al = sw ? ta : al;
    }
}

__device__ inline uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ inline int32_t unii(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <bool LITERAL, bool ADAPTIVE>
__global__ __launch_bounds__(256) void k_render(RenderArgs a) {
    __shared__ int32_t s_stack[4][STACK_DEPTH];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const uint64_t tile_idx = (uint64_t)blockIdx.x * 4 + wid;
    if (tile_idx >= a.ntiles) return;  // wave-uniform
    uint32_t cam, tx, ty;
    if (a.tiles) {
        const uint32_t t = a.tiles[tile_idx];
        cam = t >> 24;
        ty = (t >> 12) & 0xFFFu;
        tx = t & 0xFFFu;
    } else {
        const uint64_t per = (uint64_t)a.tiles_x * a.tiles_y;
        cam = (uint32_t)(tile_idx / per);
        const uint32_t rem = (uint32_t)(tile_idx % per);
        ty = rem / a.tiles_x;
        tx = rem % a.tiles_x;
    }
    cam = uni(cam);
    const uint32_t px = tx * 8 + (lane & 7), py = ty * 8 + (lane >> 3);
    const bool valid = px < a.width && py < a.height && cam < a.ncams;

    // ---- ray generation (particleRendering.comp:123-129, raygen.rgen:116-121)
    const float* V = a.view_inv + 16 * (cam < a.ncams ? cam : 0);
    const float u = ((float)px + a.pixel_offset) / (float)a.width;
    const float v = ((float)py + a.pixel_offset) / (float)a.height;
    const float nx = u * 2.0f - 1.0f, ny = v * 2.0f - 1.0f;
    const f3 o = mk3(V[12], V[13], V[14]);
    float tg[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) tg[r] = a.proj_inv[r] * nx + a.proj_inv[4 + r] * ny + a.proj_inv[8 + r] + a.proj_inv[12 + r];
    float wv[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) wv[r] = V[r] * tg[0] + V[4 + r] * tg[1] + V[8 + r] * tg[2];
    const float wl = sqrtf(wv[0] * wv[0] + wv[1] * wv[1] + wv[2] * wv[2]);
    const f3 d = mk3(wv[0] / wl, wv[1] / wl, wv[2] / wl);

    // traversal reciprocal (zero components clamped; culling only)
    const float dxs = fabsf(d.x) < 1e-12f ? copysignf(1e-12f, d.x) : d.x;
    const float dys = fabsf(d.y) < 1e-12f ? copysignf(1e-12f, d.y) : d.y;
    const float dzs = fabsf(d.z) < 1e-12f ? copysignf(1e-12f, d.z) : d.z;
    const f3 inv = mk3(1.0f / dxs, 1.0f / dys, 1.0f / dzs);

    // SH basis of the ray direction: the scalar factors of radianceFromSpH
    // (gaussianfunctions.glsl:122-151), signs folded, zero past sph_eval_degree.
    float shb[16];
    {
        const float x = d.x, y = d.y, z = d.z;
        const uint32_t deg = a.sph_deg;
        shb[0] = SH_C0;
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        shb[1] = deg > 0 ? -(SH_C1 * y) : 0.f;
        shb[2] = deg > 0 ? SH_C1 * z : 0.f;
        shb[3] = deg > 0 ? -(SH_C1 * x) : 0.f;
        shb[4] = deg > 1 ? SH_C2_0 * xy : 0.f;
        shb[5] = deg > 1 ? SH_C2_1 * yz : 0.f;
        shb[6] = deg > 1 ? SH_C2_2 * (2.0f * zz - xx - yy) : 0.f;
        shb[7] = deg > 1 ? SH_C2_3 * xz : 0.f;
        shb[8] = deg > 1 ? SH_C2_4 * (xx - yy) : 0.f;
        shb[9] = deg > 2 ? SH_C3_0 * y * (3.0f * xx - yy) : 0.f;
        shb[10] = deg > 2 ? SH_C3_1 * xy * z : 0.f;
        shb[11] = deg > 2 ? SH_C3_2 * y * (4.0f * zz - xx - yy) : 0.f;
        shb[12] = deg > 2 ? SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) : 0.f;
        shb[13] = deg > 2 ? SH_C3_4 * x * (4.0f * zz - xx - yy) : 0.f;
        shb[14] = deg > 2 ? SH_C3_5 * z * (xx - yy) : 0.f;
        shb[15] = deg > 2 ? SH_C3_6 * x * (xx - 3.0f * yy) : 0.f;
    }

    // intersectAABB (gaussianfunctions.glsl:8-16, Q12)
    float tminb, tmaxb;
    {
        const float ddx = fmaxf(d.x, 1e-6f), ddy = fmaxf(d.y, 1e-6f), ddz = fmaxf(d.z, 1e-6f);
        const float t0x = (a.aabb[0] - o.x) / ddx, t0y = (a.aabb[1] - o.y) / ddy, t0z = (a.aabb[2] - o.z) / ddz;
        const float t1x = (a.aabb[3] - o.x) / ddx, t1y = (a.aabb[4] - o.y) / ddy, t1z = (a.aabb[5] - o.z) / ddz;
        tminb = fmaxf(0.0f, fmaxf(fminf(t0x, t1x), fmaxf(fminf(t0y, t1y), fminf(t0z, t1z))));
        tmaxb = fminf(fmaxf(t0x, t1x), fminf(fmaxf(t0y, t1y), fmaxf(t0z, t1z)));
    }
    float last = fmaxf(0.0f, tminb - EPS_T);
    float T = 1.0f, cr = 0.0f, cg = 0.0f, cb = 0.0f, calpha = a.alpha_init;
    uint32_t nacc = 0, nproc = 0, rounds = 0;
    bool active = valid && a.nrecs > 0 && (last <= tmaxb) && (T > a.min_transmittance);

    float kt[K_HITS];
    uint32_t kid[K_HITS];
    float ka[K_HITS];
    int32_t* stack = s_stack[wid];

    while (__ballot(active)) {
        if (active && a.max_rounds && rounds >= a.max_rounds) active = false;
        if (active) ++rounds;
        const float tlo = last + EPS_T;
        const float thi = tmaxb + EPS_T;
#pragma unroll
        for (int i = 0; i < K_HITS; ++i) {
            kt[i] = INF_DIST;
            kid[i] = INVALID_ID;
            ka[i] = 0.0f;
        }

        // ---------------- trace(): packet traversal of the LBVH
        int sp = 0;
        int32_t node = 0;
        while (true) {
            const BvhNode nd = a.nodes[node];
            const float tc = fminf(thi, kt[K_HITS - 1]);
            float e0, e1;
            const bool h0 = active && box_hit(nd.l0x, nd.l0y, nd.l0z, nd.h0x, nd.h0y, nd.h0z, o, inv, tlo, tc, e0);
            const bool h1 = active && box_hit(nd.l1x, nd.l1y, nd.l1z, nd.h1x, nd.h1y, nd.h1z, o, inv, tlo, tc, e1);
            uint64_t b0 = __ballot(h0), b1 = __ballot(h1);
            const int32_t c0 = unii(nd.c0), c1 = unii(nd.c1);
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                const int32_t cc = side ? c1 : c0;
                const uint64_t bb = side ? b1 : b0;
                const bool hh = side ? h1 : h0;
                if (bb && cc < 0 && !(side == 1 && a.root_is_leaf)) {
                    const uint32_t gi = uni((uint32_t)(~cc));
                    if (hh) {
                        // ---- leaf: analytic icosahedron clip + response (processHit's math)
                        const RenderRec rec = a.recs[gi];
                        const f3 dxo = o - mk3(rec.px, rec.py, rec.pz);
                        const f3 ok = mk3(rec.c0x * dxo.x + rec.c1x * dxo.y + rec.c2x * dxo.z,
                                          rec.c0y * dxo.x + rec.c1y * dxo.y + rec.c2y * dxo.z,
                                          rec.c0z * dxo.x + rec.c1z * dxo.y + rec.c2z * dxo.z) *
                                      mk3(rec.isx, rec.isy, rec.isz);
                        const f3 dk = mk3(rec.c0x * d.x + rec.c1x * d.y + rec.c2x * d.z,
                                          rec.c0y * d.x + rec.c1y * d.y + rec.c2y * d.z,
                                          rec.c0z * d.x + rec.c1z * d.y + rec.c2z * d.z) *
                                      mk3(rec.isx, rec.isy, rec.isz);
                        const float hk =
                            ADAPTIVE ? kernel_scale(rec.density, a.kmin, a.kopts, a.kdeg) * SQRT3 : a.kernel_h;
                        float tn = -INFINITY, tf = INFINITY;
#define GVRT_SLAB(AX, AY, AZ)                                      \
    {                                                              \
        const float sa = (AX) * ok.x + (AY) * ok.y + (AZ) * ok.z;  \
        const float sb = (AX) * dk.x + (AY) * dk.y + (AZ) * dk.z;  \
        const float ib = 1.0f / sb;                                \
        const float t1 = (-hk - sa) * ib, t2 = (hk - sa) * ib;     \
        tn = fmaxf(tn, fminf(t1, t2));                             \
        tf = fminf(tf, fmaxf(t1, t2));                             \
    }
                        GVRT_SLAB(1.f, 1.f, 1.f)
                        GVRT_SLAB(1.f, 1.f, -1.f)
                        GVRT_SLAB(1.f, -1.f, 1.f)
                        GVRT_SLAB(-1.f, 1.f, 1.f)
                        GVRT_SLAB(0.f, PHI, IPHI)
                        GVRT_SLAB(0.f, PHI, -IPHI)
                        GVRT_SLAB(IPHI, 0.f, PHI)
                        GVRT_SLAB(-IPHI, 0.f, PHI)
                        GVRT_SLAB(PHI, IPHI, 0.f)
                        GVRT_SLAB(PHI, -IPHI, 0.f)
#undef GVRT_SLAB
                        if (tn <= tf) {
                            // particleResponse / alpha (gaussianfunctions.glsl:186-200)
                            const float l2 = dk.x * dk.x + dk.y * dk.y + dk.z * dk.z;
                            const f3 grd = l2 > 0.0f ? dk * (1.0f / sqrtf(l2)) : dk;
                            const f3 gc = cross3(grd, ok);
                            const float gd = gc.x * gc.x + gc.y * gc.y + gc.z * gc.z;
                            const float gres = expf(KERNEL_S * gd * gd);
                            const float galpha = fminf(0.99f, gres * rec.density);
                            const bool acc = (gres > a.min_response) && (galpha > a.alpha_min);
                            if (LITERAL || acc) {
                                const float al = acc ? galpha : -1.0f;
                                const bool in0 = (a.tmin_inclusive ? tn >= tlo : tn > tlo) && tn <= thi;
                                const bool in1 = (a.tmin_inclusive ? tf >= tlo : tf > tlo) && tf <= thi;
                                if (in0) kb_insert<K_HITS>(tn, gi, al, kt, kid, ka);
                                if (in1) kb_insert<K_HITS>(tf, gi, al, kt, kid, ka);
                            }
                        }
                    }
                    if (side == 0) b0 = 0;
                    else b1 = 0;
                }
            }
            if (b0 && b1) {
                const uint64_t both = __ballot(h0 && h1);
                const uint64_t pref0 = __ballot(h0 && h1 && e0 <= e1);
                const bool first0 = 2 * __popcll(pref0) >= __popcll(both);
                const int32_t near = first0 ? c0 : c1, far = first0 ? c1 : c0;
                stack[sp] = far;
                ++sp;
                node = near;
            } else if (b0) {
                node = c0;
            } else if (b1) {
                node = c1;
            } else {
                if (sp == 0) break;
                --sp;
                node = unii(stack[sp]);
            }
        }

        // ---------------- process k hits (particleRendering.comp:153-187)
        if (active) {
            if (kid[0] == INVALID_ID) {
                active = false;
            } else {
#pragma unroll
                for (int i = 0; i < K_HITS; ++i) {
                    if (kid[i] != INVALID_ID && T > a.min_transmittance) {
                        ++nproc;
                        if (ka[i] > 0.0f) {
                            const float weight = ka[i] * T;
                            const float4* s4 = reinterpret_cast<const float4*>(a.sh + 48ull * kid[i]);
                            float rr = 0.f, rg = 0.f, rb = 0.f;
                            // 16 coefficients x rgb = 12 float4
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const float4 v0 = s4[3 * q], v1 = s4[3 * q + 1], v2 = s4[3 * q + 2];
                                // coefficients 4q..4q+3: (v0.xyz) (v0.w v1.xy) (v1.zw v2.x) (v2.yzw)
                                rr += shb[4 * q] * v0.x; rg += shb[4 * q] * v0.y; rb += shb[4 * q] * v0.z;
                                rr += shb[4 * q + 1] * v0.w; rg += shb[4 * q + 1] * v1.x; rb += shb[4 * q + 1] * v1.y;
                                rr += shb[4 * q + 2] * v1.z; rg += shb[4 * q + 2] * v1.w; rb += shb[4 * q + 2] * v2.x;
                                rr += shb[4 * q + 3] * v2.y; rg += shb[4 * q + 3] * v2.z; rb += shb[4 * q + 3] * v2.w;
                            }
                            rr = fmaxf(rr + 0.5f, 0.0f);
                            rg = fmaxf(rg + 0.5f, 0.0f);
                            rb = fmaxf(rb + 0.5f, 0.0f);
                            cr += rr * weight;
                            cg += rg * weight;
                            cb += rb * weight;
                            calpha += 1.0f;
                            T *= (1.0f - ka[i]);
                            ++nacc;
                        }
                        last = fmaxf(last, kt[i]);
                    }
                }
                active = (last <= tmaxb) && (T > a.min_transmittance);
            }
        }
    }

    // ---------------- outputs
    if (valid) {
        const uint64_t pix = ((uint64_t)cam * a.height + py) * a.width + px;
        const uint64_t oi = a.packed ? tile_idx * 64 + lane : pix;
        if (a.rgba32f) reinterpret_cast<float4*>(a.rgba32f)[oi] = make_float4(cr, cg, cb, calpha);
        if (a.rgba8) {
            auto q8 = [](float f) -> uint32_t { return (uint32_t)(fminf(fmaxf(f, 0.0f), 1.0f) * 255.0f + 0.5f); };
            reinterpret_cast<uint32_t*>(a.rgba8)[oi] = q8(cr) | (q8(cg) << 8) | (q8(cb) << 16) | (q8(calpha) << 24);
        }
        if (a.hit_counts) a.hit_counts[oi] = nacc;
        if (a.ray_dirs) {
            const uint64_t di = a.ray_dirs_layout == 1
                                    ? ((uint64_t)cam * a.width * a.height + (uint64_t)px * a.height + py)
                                    : pix;
            reinterpret_cast<float4*>(a.ray_dirs)[di] = make_float4(d.x, d.y, d.z, 0.0f);
        }
    } else if (a.packed) {
        const uint64_t oi = tile_idx * 64 + lane;
        if (a.rgba32f) reinterpret_cast<float4*>(a.rgba32f)[oi] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.rgba8) reinterpret_cast<uint32_t*>(a.rgba8)[oi] = 0u;
        if (a.hit_counts) a.hit_counts[oi] = 0u;
    }
    if (a.stats) {
        unsigned long long s0 = nproc, s1 = nacc, s2 = rounds;
        for (int off = 32; off > 0; off >>= 1) {
            s0 += __shfl_xor(s0, off);
            s1 += __shfl_xor(s1, off);
            s2 += __shfl_xor(s2, off);
        }
        if (lane == 0) {
            atomicAdd(a.stats + 0, s0);
            atomicAdd(a.stats + 1, s1);
            atomicAdd(a.stats + 2, s2);
        }
    }
}

__global__ __launch_bounds__(256) void k_unpack(const uint32_t* __restrict__ packed, const uint32_t* __restrict__ tiles,
                                                uint64_t ntiles, uint32_t width, uint32_t height,
                                                uint32_t* __restrict__ frame) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ntiles * 64) return;
    const uint32_t t = tiles[i >> 6];
    const uint32_t lane = (uint32_t)(i & 63);
    const uint32_t cam = t >> 24, ty = (t >> 12) & 0xFFFu, tx = t & 0xFFFu;
    const uint32_t px = tx * 8 + (lane & 7), py = ty * 8 + (lane >> 3);
    if (px >= width || py >= height) return;
    frame[((uint64_t)cam * height + py) * width + px] = packed[i];
}

}  // namespace

gvrt_status gvrt_launch_render_mode(gvrt_context* c, const RenderArgs& a, uint64_t nwaves, bool literal) {
    const uint64_t blocks = (nwaves + 3) / 4;
    if (blocks == 0) return GVRT_OK;
    const bool adaptive = (a.kopts & 1u) != 0;
    if (literal) {
        if (adaptive) hipLaunchKernelGGL((k_render<true, true>), dim3((unsigned)blocks), dim3(256), 0, c->stream, a);
        else hipLaunchKernelGGL((k_render<true, false>), dim3((unsigned)blocks), dim3(256), 0, c->stream, a);
    } else {
        if (adaptive) hipLaunchKernelGGL((k_render<false, true>), dim3((unsigned)blocks), dim3(256), 0, c->stream, a);
        else hipLaunchKernelGGL((k_render<false, false>), dim3((unsigned)blocks), dim3(256), 0, c->stream, a);
    }
    GVRT_HIP(c, hipGetLastError());
    return GVRT_OK;
}

gvrt_status gvrt_launch_unpack(gvrt_context* c, const void* packed, const uint32_t* tiles, uint64_t ntiles,
                               uint32_t width, uint32_t height, void* frame) {
    const uint64_t n = ntiles * 64;
    if (!n) return GVRT_OK;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream,
                       (const uint32_t*)packed, tiles, ntiles, width, height, (uint32_t*)frame);
    GVRT_HIP(c, hipGetLastError());
    return GVRT_OK;
}
