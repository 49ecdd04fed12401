// gvrt_enclose.hip — Gaussian Enclosing pass on gfx950.
//
// Replaces shaders/glsl/VulkanFullRT/particlePrimitives.comp (dispatched by
// VulkanFullRT::computeGaussianEnclosingIcosaHedron, VulkanFullRT.cpp:1503-1514).
// One thread per Gaussian.  The reference compacts survivors with an atomicAdd whose
// order is nondeterministic (Q3, and the counter is never zeroed); here compaction is a
// flag pass + exclusive scan + emit pass, so saveIdx = rank among survivors in input order.
//
// Bytes per Gaussian (roofline): reads 236 B of SoA splat data (+ the filter's
// neighbour re-reads, L2-resident), writes 48 B density + 192 B SH + 64 B render record +
// 24 B proxy box (+ 144 B vertices + 240 B indices when emit_triangles).
#include <hipcub/hipcub.hpp>

#include "gvrt_internal.h"

using namespace gvrt;

namespace {

constexpr uint32_t SPEC_DIM = 45;  // SPECULAR_DIMENSION, 3dgs.glsl:14

// particlePrimitives.comp:120-140 — abnormal particle filter on one Gaussian's f_dc and the 45 f_rest
// floats starting at its own (s[45..] are the next particles', Q5: the reference reads them for i >= 15;
// the device buffer carries 90 zero floats past the end, so the last two particles read 0.0 there).
__device__ inline bool survives(float a0, float a1, float a2, const float* s) {
    const float albedoStrength = sqrtf(a0 * a0 + a1 * a1 + a2 * a2);
    float specularStrength = 0.0f, maxSpecular = 0.0f, minSpecular = 1e10f;
#pragma unroll 4
    for (uint32_t i = 1; i < SPEC_DIM; i++) {
        const float x = s[3 * i], y = s[3 * i + 1], z = s[3 * i + 2];
        specularStrength += sqrtf(x * x + y * y + z * z);
        maxSpecular = fmaxf(maxSpecular, specularStrength);
        minSpecular = fminf(minSpecular, specularStrength);
    }
    if (albedoStrength > 3.0f) return false;
    if (maxSpecular / (minSpecular + 1e-5f) > 150.0f) return false;
    return true;
}

// One block = 256 Gaussians.  The block's f_rest span (256 x 45 floats plus the 90 the Q5 neighbour reads
// reach into) is staged in LDS with coalesced float4 loads; each thread then walks its own 45 floats
// there (stride 45 words: odd, so the 64 lanes hit distinct banks).  Per-thread global reads at a 180-B
// stride touched a different cache line in every lane of every load instruction.
constexpr uint32_t FB = 256;                        // Gaussians per block
constexpr uint32_t FSPAN = FB * SPEC_DIM + 2 * SPEC_DIM;  // staged floats (multiple of 4: 11610 -> pad)
constexpr uint32_t FSPAN4 = (FSPAN + 3) / 4;

__global__ __launch_bounds__(256) void k_enclose_flags(uint64_t n, const float* __restrict__ fdc,
                                                       const float* __restrict__ frest,
                                                       uint32_t* __restrict__ flags) {
    __shared__ float4 s_fr4[FSPAN4];
    const uint64_t g0 = (uint64_t)blockIdx.x * FB;
    // frest holds 45 n + 90 floats (zero tail) and g0 * 45 * 4 B is 16-B aligned (g0 is a multiple of 256)
    const uint64_t avail = (n - g0) * SPEC_DIM + 2 * SPEC_DIM;  // floats readable from this block's start
    const float4* src4 = reinterpret_cast<const float4*>(frest + g0 * SPEC_DIM);
    float* s_fr = reinterpret_cast<float*>(s_fr4);
    for (uint32_t i = threadIdx.x; i < FSPAN4; i += blockDim.x) {
        if (4ull * i + 3 < avail) {
            s_fr4[i] = src4[i];
        } else {
            for (uint32_t k = 0; k < 4; ++k) s_fr[4 * i + k] = 4ull * i + k < avail ? frest[g0 * SPEC_DIM + 4 * i + k] : 0.0f;
        }
    }
    __syncthreads();
    const uint64_t g = g0 + threadIdx.x;
    if (g >= n) return;
    const bool ok = survives(fdc[3 * g], fdc[3 * g + 1], fdc[3 * g + 2], s_fr + threadIdx.x * SPEC_DIM);
    flags[g] = ok ? 1u : 0u;
}

// SH records [f_dc, f_rest] in compaction order (particlePrimitives.comp:207-214): consecutive threads write
// consecutive float4s and read consecutive floats of one Gaussian (the 48-float rows of consecutive survivors
// come from nearly consecutive sources).
__global__ __launch_bounds__(256) void k_enclose_sh(const uint32_t* __restrict__ count, const uint32_t* __restrict__ src,
                                                    const float* __restrict__ fdc, const float* __restrict__ frest,
                                                    float* __restrict__ sh48) {
    // one thread per output float4 (12 per survivor): aligned 16-B stores, and the 4 input floats of a thread are
    // consecutive in the survivor's f_dc / f_rest row, so a wave's reads stay row-contiguous
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= 12ull * *count) return;  // grid sized for n; the survivor count is scan[n]
    const uint64_t sidx = q / 12;
    const uint32_t c0 = 4 * (uint32_t)(q - 12 * sidx);
    const uint64_t g = src[sidx];
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t c = c0 + k;
        v[k] = c < 3 ? fdc[3 * g + c] : frest[g * SPEC_DIM + (c - 3)];
    }
    reinterpret_cast<float4*>(sh48)[q] = make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __constant__ float c_icosa[12][3] = {
    {-1, PHI, 0}, {1, PHI, 0},  {0, 1, -PHI},  {-PHI, 0, -1}, {-PHI, 0, 1}, {0, 1, PHI},
    {PHI, 0, 1},  {0, -1, PHI}, {-1, -PHI, 0}, {0, -1, -PHI}, {PHI, 0, -1}, {1, -PHI, 0}};
__device__ __constant__ uint32_t c_tri[20][3] = {
    {0, 1, 2},  {0, 2, 3},  {0, 3, 4},   {0, 4, 5},  {0, 5, 1},  {6, 1, 5},  {6, 5, 7},
    {6, 7, 11}, {6, 11, 10}, {6, 10, 1}, {8, 4, 3},  {8, 3, 9},  {8, 9, 11}, {8, 11, 7},
    {8, 7, 4},  {9, 3, 2},  {9, 2, 10},  {9, 10, 11}, {5, 4, 7},  {1, 10, 2}};

struct EncloseArgs {
    uint64_t n;
    const float* pos;
    const float* rot;
    const float* scl;
    const float* opa;
    const float* fdc;
    const float* frest;
    const uint32_t* flags;
    const uint32_t* scan;
    float kmin;
    uint32_t opts;
    float degree;
    float* density12;
    float* sh48;
    float* verts;
    uint32_t* tris;
    uint32_t* src;
    RenderRec* recs;
    float* boxes;
    const uint32_t* absmax;  // bits of the largest finite |position component| (k_pos_absmax)
};

// Largest finite |position component| of the splats (float bits: non-negative floats order as their bits).
// The proxy boxes get an absolute padding of 2^-18 x this bound: it covers the rounding of the render
// kernel's FMA-form box planes for ray origins within 4x the bound, so that kernel needs no per-box slack.
// One atomic per block: device atomics on one word serialise (~11 ns each on MI355X), so the
// 8192 per-wave atomics of the first version cost 97 us at 1 M; the grid is capped at 1024 blocks.
__global__ __launch_bounds__(256) void k_pos_absmax(uint64_t n3, const float* __restrict__ pos,
                                                    uint32_t* __restrict__ out) {
    __shared__ float s_m[4];
    float m = 0.0f;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
#pragma unroll 4
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n3; i += stride) {
        const float v = fabsf(pos[i]);
        if (v <= 3.0e38f) m = fmaxf(m, v);  // NaN / inf positions do not set the bound
    }
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(out, __float_as_uint(fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]))));
}

// particlePrimitives.comp:142-214
__global__ __launch_bounds__(256) void k_enclose_emit(EncloseArgs a) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.n || !a.flags[g]) return;
    const uint32_t saveIdx = a.scan[g];
    a.src[saveIdx] = (uint32_t)g;

    float q[4] = {a.rot[4 * g], a.rot[4 * g + 1], a.rot[4 * g + 2], a.rot[4 * g + 3]};
    const float qn = 1.0f / sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] *= qn;
    q[1] *= qn;
    q[2] *= qn;
    q[3] *= qn;
    const float w = q[0], x = q[1], y = q[2], z = q[3];
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, xz = x * z, yz = y * z;
    const float wx = w * x, wy = w * y, wz = w * z;
    // quaternionWXYZToMatrixTranspose (utils.glsl:36-56): columns of the world rotation R
    const f3 r0 = mk3(1.0f - 2.0f * (yy + zz), 2.0f * (xy + wz), 2.0f * (xz - wy));
    const f3 r1 = mk3(2.0f * (xy - wz), 1.0f - 2.0f * (xx + zz), 2.0f * (yz + wx));
    const f3 r2 = mk3(2.0f * (xz + wy), 2.0f * (yz - wx), 1.0f - 2.0f * (xx + yy));
    const f3 scl = mk3(expf(a.scl[3 * g]), expf(a.scl[3 * g + 1]), expf(a.scl[3 * g + 2]));
    const f3 trans = mk3(a.pos[3 * g], a.pos[3 * g + 1], a.pos[3 * g + 2]);
    const float density = 1.0f / (1.0f + expf(-a.opa[g]));  // sigmoid :107-110
    const float ks = kernel_scale(density, a.kmin, a.opts, a.degree);
    const f3 kscl = scl * (ks * ICOSA_VRT_SCALE);

    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const f3 v = mk3(c_icosa[i][0] * kscl.x, c_icosa[i][1] * kscl.y, c_icosa[i][2] * kscl.z);
        const f3 vert = r0 * v.x + r1 * v.y + r2 * v.z + trans;
        lo[0] = fminf(lo[0], vert.x);
        lo[1] = fminf(lo[1], vert.y);
        lo[2] = fminf(lo[2], vert.z);
        hi[0] = fmaxf(hi[0], vert.x);
        hi[1] = fmaxf(hi[1], vert.y);
        hi[2] = fmaxf(hi[2], vert.z);
        if (a.verts) {
            float* vp = a.verts + 36ull * saveIdx + 3 * i;
            vp[0] = vert.x;
            vp[1] = vert.y;
            vp[2] = vert.z;
        }
    }
    if (a.tris) {
        uint32_t* tp = a.tris + 60ull * saveIdx;
#pragma unroll
        for (int i = 0; i < 20; ++i)
            for (int k = 0; k < 3; ++k) tp[3 * i + k] = c_tri[i][k] + 12u * saveIdx;
    }
    // Proxy AABB, padded so the analytic icosahedron of the render kernel (exact planes) is
    // always inside the box built from the rounded vertices.
    float* bx = a.boxes + 6ull * saveIdx;
    const float pad_abs = ldexpf(__uint_as_float(*a.absmax), -18);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float c = 0.5f * (lo[k] + hi[k]);
        const float pad = 1e-5f * (hi[k] - lo[k]) + 1e-6f * fabsf(c) + pad_abs + 1e-30f;
        bx[k] = lo[k] - pad;
        bx[3 + k] = hi[k] + pad;
    }

    // density record (std140 ParticleDensity, 3dgs.glsl:56-62), particlePrimitives.comp:187-205
    float4* dr = reinterpret_cast<float4*>(a.density12 + 12ull * saveIdx);
    dr[0] = make_float4(trans.x, trans.y, trans.z, density);
    dr[1] = make_float4(q[0], q[1], q[2], q[3]);
    dr[2] = make_float4(scl.x, scl.y, scl.z, 0.0f);

    // (SH record: k_enclose_sh, coalesced, after this pass)

    // render record: what processHit derives per hit from the density record
    // (fetchParticleDensity + quaternionWXYZToMatrix, gaussianfunctions.glsl:89-101, utils.glsl:13-34)
    RenderRec rr;
    rr.px = trans.x;
    rr.py = trans.y;
    rr.pz = trans.z;
    rr.density = density;
    rr.c0x = 1.0f - 2.0f * (yy + zz);
    rr.c0y = 2.0f * (xy - wz);
    rr.c0z = 2.0f * (xz + wy);
    rr.c1x = 2.0f * (xy + wz);
    rr.c1y = 1.0f - 2.0f * (xx + zz);
    rr.c1z = 2.0f * (yz - wx);
    rr.c2x = 2.0f * (xz - wy);
    rr.c2y = 2.0f * (yz + wx);
    rr.c2z = 1.0f - 2.0f * (xx + yy);
    rr.isx = 1.0f / scl.x;
    rr.isy = 1.0f / scl.y;
    rr.isz = 1.0f / scl.z;
    a.recs[saveIdx] = rr;
}

}  // namespace

gvrt_status gvrt_launch_enclose(gvrt_context* c, const gvrt_enclosing_params* p, uint64_t* m_out) {
    const uint64_t n = c->n;
    // capacity for n survivors
    if (c->cap < n || !c->d_density12) {
        gvrt_dfree(c, (void**)&c->d_density12);
        gvrt_dfree(c, (void**)&c->d_sh48);
        gvrt_dfree(c, (void**)&c->d_src);
        gvrt_dfree(c, (void**)&c->d_recs_c);
        gvrt_dfree(c, (void**)&c->d_boxes_c);
        gvrt_dfree(c, (void**)&c->d_flags);
        gvrt_dfree(c, (void**)&c->d_scan);
        const uint64_t nn = n ? n : 1;
        gvrt_status s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_density12, 48 * nn))) return s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_sh48, 192 * nn))) return s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_src, 4 * nn))) return s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_recs_c, sizeof(RenderRec) * nn))) return s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_boxes_c, 24 * nn))) return s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_flags, 4 * (nn + 1)))) return s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_scan, 4 * (nn + 1)))) return s;
        c->cap = nn;
    }
    if (!c->d_absmax) {
        gvrt_status s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_absmax, 4))) return s;
    }
    gvrt_dfree(c, (void**)&c->d_verts);
    gvrt_dfree(c, (void**)&c->d_tris);
    if (p->emit_triangles && n) {
        gvrt_status s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_verts, 144 * n))) return s;
        if ((s = gvrt_dalloc(c, (void**)&c->d_tris, 240 * n))) return s;
    }
    if (n == 0) {
        *m_out = 0;
        c->box_pad_abs = 0.0f;
        return GVRT_OK;
    }
    const unsigned blocks = (unsigned)((n + 255) / 256);
    GVRT_HIP(c, hipEventRecord(c->ev0, c->stream));
    hipLaunchKernelGGL(k_enclose_flags, dim3(blocks), dim3(256), 0, c->stream, n, c->d_fdc, c->d_frest,
                       c->d_flags);
    GVRT_HIP(c, hipGetLastError());
    // exclusive scan over n+1 flags (flags[n] = 0) so scan[n] is the survivor count
    GVRT_HIP(c, hipMemsetAsync(c->d_flags + n, 0, 4, c->stream));
    size_t tmp_bytes = 0;
    GVRT_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, c->d_flags, c->d_scan, (int)(n + 1), c->stream));
    void* tmp = nullptr;
    gvrt_status s;
    if ((s = gvrt_dalloc(c, &tmp, tmp_bytes ? tmp_bytes : 16))) return s;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, c->d_flags, c->d_scan, (int)(n + 1), c->stream);
    if (e != hipSuccess) {
        gvrt_dfree(c, &tmp);
        return gvrt_hip_check(c, e, "DeviceScan::ExclusiveSum");
    }
    // scene position bound for the absolute box padding (read by k_enclose_emit on the device)
    uint32_t* d_absmax = c->d_absmax;
    GVRT_HIP(c, hipMemsetAsync(d_absmax, 0, 4, c->stream));
    {
        const uint64_t n3 = 3 * n;
        const unsigned rb = (unsigned)std::min<uint64_t>((n3 + 255) / 256, 1024);
        hipLaunchKernelGGL(k_pos_absmax, dim3(rb), dim3(256), 0, c->stream, n3, c->d_pos, d_absmax);
        e = hipGetLastError();
        if (e != hipSuccess) {
            gvrt_dfree(c, &tmp);
            return gvrt_hip_check(c, e, "k_pos_absmax");
        }
    }
    EncloseArgs a;
    a.n = n;
    a.pos = c->d_pos;
    a.rot = c->d_rot;
    a.scl = c->d_scl;
    a.opa = c->d_opa;
    a.fdc = c->d_fdc;
    a.frest = c->d_frest;
    a.flags = c->d_flags;
    a.scan = c->d_scan;
    a.kmin = p->kernel_min_response;
    a.opts = p->opts;
    a.degree = p->degree;
    a.density12 = c->d_density12;
    a.sh48 = c->d_sh48;
    a.verts = c->d_verts;
    a.tris = c->d_tris;
    a.src = c->d_src;
    a.recs = c->d_recs_c;
    a.boxes = c->d_boxes_c;
    a.absmax = d_absmax;
    hipLaunchKernelGGL(k_enclose_emit, dim3(blocks), dim3(256), 0, c->stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) {
        gvrt_dfree(c, &tmp);
        return gvrt_hip_check(c, e, "k_enclose_emit");
    }
    {
        const uint64_t nq = 12ull * n;
        hipLaunchKernelGGL(k_enclose_sh, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, c->stream, c->d_scan + n,
                           c->d_src, c->d_fdc, c->d_frest, c->d_sh48);
        e = hipGetLastError();
        if (e != hipSuccess) {
            gvrt_dfree(c, &tmp);
            return gvrt_hip_check(c, e, "k_enclose_sh");
        }
    }
    GVRT_HIP(c, hipEventRecord(c->ev1, c->stream));
    uint32_t count = 0, absmax = 0;
    GVRT_HIP(c, hipMemcpyAsync(&count, c->d_scan + n, 4, hipMemcpyDeviceToHost, c->stream));
    GVRT_HIP(c, hipMemcpyAsync(&absmax, d_absmax, 4, hipMemcpyDeviceToHost, c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    float r;
    std::memcpy(&r, &absmax, 4);
    c->box_pad_abs = std::ldexp(r, -18);
    gvrt_dfree(c, &tmp);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
    c->stats.enclose_ms = ms;
    *m_out = count;
    return GVRT_OK;
}
