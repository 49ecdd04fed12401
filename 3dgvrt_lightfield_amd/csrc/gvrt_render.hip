// gvrt_render.hip — Particle Rendering pass on gfx950.
//
// Replaces the per-pixel ray-march of shaders/glsl/VulkanFullRT/particleRendering.comp:117-191
// (ray query), raygen.rgen:113-193 + anyhit.rahit:40-71 (RT pipeline) and
// raygenGaussianLightField.rgen:114-202 (multi-camera light field), and the driver's BVH
// traversal behind traceRayEXT / rayQueryProceedEXT.
//
// Mapping to CDNA4: one wave64 = one 8x8 pixel tile (one lane per ray), one wave per
// workgroup, 4 waves per SIMD.  Workgroups take tiles in the order of a tile list: costliest first by the
// previous launch's per-tile cost classes, each class dealt to the 8 XCDs in contiguous chunks
// (k_tile_order); the first launch of a frame size walks 8x4-tile supertiles.  Traversal is wave-uniform
// (packet traversal) over the 4-wide BVH: node and leaf-record addresses are wave-uniform, so both are
// fetched with scalar loads (two s_load_dwordx16 per 128-B node, one per 64-B record).  A wave whose active
// rays share one direction octant reads the octant copy of the nodes, whose planes are stored in (near, far)
// order for that octant.  Every lane clips its own ray against the four child boxes and ballots decide
// which children the packet descends into; children are visited in the node's stored (split) order,
// forward or backward by the sign of the first lane's direction on the split axis, and the farther ones go
// on a 128-entry per-wave LDS stack.  Leaves are tested response first (an accepted crossing passes inside
// the proxy's inscribed sphere), then clipped against the analytic icosahedron (10 antipodal slab pairs in
// the kernel frame), which yields the same two crossings (entry and exit face, Q1) as the reference's
// 20-triangle proxy.  Each lane keeps a register k-buffer (FAST: 32 slots of {t, record id << 8 | q},
// q a conservative optical-depth code that drives the termination cull; LITERAL: the reference's 16 slots
// of every crossing, anyhit.rahit:29-71).  After each traversal round every lane composites its slots front
// to back (processHit, gaussianfunctions.glsl:153-229) with the SH basis of its ray direction precomputed
// once per ray in LDS.
//
// Modes: LITERAL = every crossing enters the k-buffer, rounds exactly as the reference
// (16 per trace, `last` advanced by rejected hits too).  FAST = only accepted crossings enter the
// k-buffer; with an exclusive tmin the composited sequence, and therefore the image, is the
// same (rejected crossings only ever advanced `last`), while far fewer rounds are needed.
#include <hip/hip_ext.h>

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

static_assert(BVH_W == 4, "the render kernel traverses 4-wide nodes");

// Composite tuning (same-box A/B): the first SH_EARLY of a hit's 12 SH float4 loads are summed
// before the accept branch (round 2: issued with the record's, -1.5 %; the ROCm 7.2 compiler sinks them into the
// branch again, and forcing 3 or 6 of them out with an asm anchor measured +0.5-1 % in round 4); a FAST K = 24
// buffer is composited in groups of COMP_GROUP slots (static register indices, one buffer shift per group).
constexpr int SH_EARLY = 6;
constexpr int COMP_GROUP = 6;

// Slab test in FMA form t = lo * inv - o * inv (one v_fma per plane).  Culling only: the proxy boxes are
// padded (gvrt_enclose.hip), so a crossing is never dropped.
template <bool SLACK>
__device__ inline bool box_hit(float lx, float ly, float lz, float hx, float hy, float hz, f3 oinv, f3 inv,
                               float t0, float t1) {
    const float ax = fmaf(lx, inv.x, -oinv.x), bx = fmaf(hx, inv.x, -oinv.x);
    const float ay = fmaf(ly, inv.y, -oinv.y), by = fmaf(hy, inv.y, -oinv.y);
    const float az = fmaf(lz, inv.z, -oinv.z), bz = fmaf(hz, inv.z, -oinv.z);
    const float tn = fmaxf(fmaxf(t0, fminf(ax, bx)), fmaxf(fminf(ay, by), fminf(az, bz)));
    const float tf = fminf(fminf(t1, fmaxf(ax, bx)), fminf(fmaxf(ay, by), fmaxf(az, bz)));
    // SLACK: a relative slack on the exit distance absorbs the plane rounding.  Without it the
    // absolute box padding of gvrt_enclose.hip (2^-18 x the scene's position bound) covers the rounding
    // of these FMA-form planes, (2|lo| + 3|o|) * 2^-24 per plane in world units, as long as the ray
    // origin lies within 4x that bound (render_impl chooses the variant per launch).
    if constexpr (SLACK) return tn <= tf + 2e-6f * fabsf(tf);
    else return tn <= tf;
}

// Slab test on planes stored in (near, far) order for the ray's octant (octant copies of the nodes): the
// same plane values as box_hit's, and its min / max pairs are the near / far planes, so no pair is needed
template <bool SLACK>
__device__ inline bool box_hit_nf(float nx, float ny, float nz, float fx, float fy, float fz, f3 oinv, f3 inv, float t0,
                                  float t1) {
    const float an = fmaf(nx, inv.x, -oinv.x), af = fmaf(fx, inv.x, -oinv.x);
    const float bn = fmaf(ny, inv.y, -oinv.y), bf = fmaf(fy, inv.y, -oinv.y);
    const float cn = fmaf(nz, inv.z, -oinv.z), cf = fmaf(fz, inv.z, -oinv.z);
    const float tn = fmaxf(fmaxf(t0, an), fmaxf(bn, cn));
    const float tf = fminf(fminf(t1, af), fminf(bf, cf));
    if constexpr (SLACK) return tn <= tf + 2e-6f * fabsf(tf);
    else return tn <= tf;
}

// Insert two crossings of one proxy (a.t <= b.t, either may be INF_DIST) in one pass.  Per slot the
// same strict-< rule as compareAndSwapHitPayloadValue (ties keep the earlier arrival first).
template <int K>
__device__ inline void kb_insert2(float ta, float tb, uint32_t id, float al, float (&kt)[K], uint32_t (&kid)[K],
                                  float (&ka)[K]) {
    float pt0 = ta, pt1 = tb;
    uint32_t pi0 = id, pi1 = id;
    float pa0 = al, pa1 = al;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const bool c0 = pt0 < kt[i];
        const float st = kt[i];
        const uint32_t si = kid[i];
        const float sa = ka[i];
        kt[i] = c0 ? pt0 : st;
        kid[i] = c0 ? pi0 : si;
        ka[i] = c0 ? pa0 : sa;
        const float xt = c0 ? st : pt0;  // displaced (larger) of slot / pending 0
        const uint32_t xi = c0 ? si : pi0;
        const float xa = c0 ? sa : pa0;
        const bool c1 = pt1 < xt;
        pt0 = c1 ? pt1 : xt;
        pi0 = c1 ? pi1 : xi;
        pa0 = c1 ? pa1 : xa;
        pt1 = c1 ? xt : pt1;
        pi1 = c1 ? xi : pi1;
        pa1 = c1 ? xa : pa1;
    }
}

// Packed FAST k-buffer: slot payload = (record id << 8) | q, q = floor(-log2(1 - alpha) * QSCALE)
// clamped to [0, 255] (alpha <= 0.99 so the exact code is <= 255).  q only drives the termination
// cull: its running sum never exceeds the exact optical depth, so the cull stays conservative; the
// composite recomputes alpha from the record as processHit does (gaussianfunctions.glsl:186-200).
constexpr float QSCALE = 38.3837f;  // 255 / log2(100), slightly low so q(0.99) <= 255
constexpr uint32_t PK_EMPTY = 0xFFFFFFFFu;

__device__ inline uint32_t alpha_code(float alpha) {
    const float q = -__log2f(1.0f - alpha) * QSCALE - 0.02f;  // margin covers v_log_f32 error
    return (uint32_t)fminf(fmaxf(q, 0.0f), 255.0f);
}

// As kb_insert2, with one 32-bit payload per slot (t, then payload; same strict-< rule).  The chain
// runs in groups of 8 slots (4 when K is not a multiple of 8), and a group is skipped when no inserting
// lane has its pending crossing below the group's last slot: the pending pair stays sorted (pt0 <= pt1),
// so such a group would not change.  With front-to-back traversal most crossings land near the end of
// the buffer.  An 8-slot group is one asm block whose slot registers are updated in place ("+v"): left to
// the compiler, the updated slots of a group landed in fresh registers and the join with the group-skip
// path copied the whole buffer back (~40 v_mov per executed group for 80 useful VALU).  Per slot: 2 v_cmp
// (to SGPR pairs) + 8 v_cndmask, ordered so that every mask is read at least two instructions after the
// v_cmp that writes it (the gfx950 VALU-SGPR-write -> lane-mask-read hazard).
#define KB_S_HEAD(T, P)                                      \
    "v_cndmask_b32_e64 %[xt], %[pt0], " T ", %[m0]\n\t"      \
    "v_cmp_lt_f32_e64 %[m1], %[pt1], %[xt]\n\t"              \
    "v_cndmask_b32_e64 %[xp], %[pp0], " P ", %[m0]\n\t"      \
    "v_cndmask_b32_e64 " T ", " T ", %[pt0], %[m0]\n\t"      \
    "v_cndmask_b32_e64 " P ", " P ", %[pp0], %[m0]\n\t"      \
    "v_cndmask_b32_e64 %[pt0], %[xt], %[pt1], %[m1]\n\t"
#define KB_S_TAIL                                             \
    "v_cndmask_b32_e64 %[pp0], %[xp], %[pp1], %[m1]\n\t"     \
    "v_cndmask_b32_e64 %[pt1], %[pt1], %[xt], %[m1]\n\t"     \
    "v_cndmask_b32_e64 %[pp1], %[pp1], %[xp], %[m1]\n\t"
#define KB_S(T, P, TN) KB_S_HEAD(T, P) "v_cmp_lt_f32_e64 %[m0], %[pt0], " TN "\n\t" KB_S_TAIL
#define KB_S_LAST(T, P) KB_S_HEAD(T, P) KB_S_TAIL

// one 8-slot group of kb_insert2p, slots g..g+7 of kt / kp updated in place
__device__ inline void kb_group8(float& t0, float& t1, float& t2, float& t3, float& t4, float& t5, float& t6, float& t7,
                                 uint32_t& p0, uint32_t& p1, uint32_t& p2, uint32_t& p3, uint32_t& p4, uint32_t& p5,
                                 uint32_t& p6, uint32_t& p7, float& pt0, uint32_t& pp0, float& pt1, uint32_t& pp1) {
    float xt;
    uint32_t xp;
    uint64_t m0, m1;
    asm("v_cmp_lt_f32_e64 %[m0], %[pt0], %[t0]\n\t"
        "s_nop 1\n\t"
        KB_S("%[t0]", "%[p0]", "%[t1]") KB_S("%[t1]", "%[p1]", "%[t2]") KB_S("%[t2]", "%[p2]", "%[t3]")
        KB_S("%[t3]", "%[p3]", "%[t4]") KB_S("%[t4]", "%[p4]", "%[t5]") KB_S("%[t5]", "%[p5]", "%[t6]")
        KB_S("%[t6]", "%[p6]", "%[t7]") KB_S_LAST("%[t7]", "%[p7]")
        : [t0] "+v"(t0), [t1] "+v"(t1), [t2] "+v"(t2), [t3] "+v"(t3), [t4] "+v"(t4), [t5] "+v"(t5), [t6] "+v"(t6),
          [t7] "+v"(t7), [p0] "+v"(p0), [p1] "+v"(p1), [p2] "+v"(p2), [p3] "+v"(p3), [p4] "+v"(p4), [p5] "+v"(p5),
          [p6] "+v"(p6), [p7] "+v"(p7), [pt0] "+v"(pt0), [pp0] "+v"(pp0), [pt1] "+v"(pt1), [pp1] "+v"(pp1),
          [xt] "=&v"(xt), [xp] "=&v"(xp), [m0] "=&s"(m0), [m1] "=&s"(m1));
}

template <int K>
__device__ inline void kb_insert2p(float ta, float tb, uint32_t pk, float (&kt)[K], uint32_t (&kp)[K]) {
    constexpr int G = (K % 8 == 0) ? 8 : 4;
    static_assert(K % G == 0, "whole groups");
    float pt0 = ta, pt1 = tb;
    uint32_t pp0 = pk, pp1 = pk;
#pragma unroll
    for (int g = 0; g < K; g += G) {
        if (__builtin_amdgcn_ballot_w64(pt0 < kt[g + G - 1])) {
            if constexpr (G == 8) {
                kb_group8(kt[g], kt[g + 1], kt[g + 2], kt[g + 3], kt[g + 4], kt[g + 5], kt[g + 6], kt[g + 7], kp[g],
                          kp[g + 1], kp[g + 2], kp[g + 3], kp[g + 4], kp[g + 5], kp[g + 6], kp[g + 7], pt0, pp0, pt1,
                          pp1);
                continue;
            }
#pragma unroll
            for (int i = g; i < g + G; ++i) {
                const bool c0 = pt0 < kt[i];
                const float st = kt[i];
                const uint32_t sp = kp[i];
                kt[i] = c0 ? pt0 : st;
                kp[i] = c0 ? pp0 : sp;
                const float xt = c0 ? st : pt0;
                const uint32_t xp = c0 ? sp : pp0;
                const bool c1 = pt1 < xt;
                pt0 = c1 ? pt1 : xt;
                pp0 = c1 ? pp1 : xp;
                pt1 = c1 ? xt : pt1;
                pp1 = c1 ? xp : pp1;
            }
        }
    }
}

// Kernel-frame ray of one particle (gaussianfunctions.glsl:186-191): ok = S^-1 R^T (o - p), dk = S^-1 R^T d.
// Written with explicit fmaf and contraction off: the insert-time and composite-time evaluations of
// kernel_frame / particle_alpha must round identically, and the backend otherwise fuses mul+add pairs
// differently at each inlined site (SLP-packed v_pk_fma_f32 at one, scalar mul/sub at the other).
__device__ inline f3 kernel_org(const RenderRec& rec, f3 o) {
#pragma clang fp contract(off)
    const float ex = o.x - rec.px, ey = o.y - rec.py, ez = o.z - rec.pz;
    return mk3(fmaf(rec.c2x, ez, fmaf(rec.c1x, ey, rec.c0x * ex)) * rec.isx,
               fmaf(rec.c2y, ez, fmaf(rec.c1y, ey, rec.c0y * ex)) * rec.isy,
               fmaf(rec.c2z, ez, fmaf(rec.c1z, ey, rec.c0z * ex)) * rec.isz);
}
__device__ inline f3 kernel_dir(const RenderRec& rec, f3 d) {
#pragma clang fp contract(off)
    return mk3(fmaf(rec.c2x, d.z, fmaf(rec.c1x, d.y, rec.c0x * d.x)) * rec.isx,
               fmaf(rec.c2y, d.z, fmaf(rec.c1y, d.y, rec.c0y * d.x)) * rec.isy,
               fmaf(rec.c2z, d.z, fmaf(rec.c1z, d.y, rec.c0z * d.x)) * rec.isz);
}
// OKREC: the launch's records carry the kernel-frame origin ok in place of the position (k_rec_origin
// wrote it for this launch's single camera origin, with kernel_org: the same bits as computing it here)
__device__ inline float to_vgpr(float x) {  // a scalar-loaded record field copied to a VGPR: not kept live in
    float r;                                  // SGPRs past the leaf test (that spilled SGPRs)
    asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}
// SREC: rec was fetched by scalar loads (leaf visits), else per lane (composite)
template <bool OKREC, bool SREC = false>
__device__ inline void kernel_frame(const RenderRec& rec, f3 o, f3 d, f3& ok, f3& dk) {
    if constexpr (OKREC && SREC) ok = mk3(to_vgpr(rec.px), to_vgpr(rec.py), to_vgpr(rec.pz));
    else if constexpr (OKREC) ok = mk3(rec.px, rec.py, rec.pz);
    else ok = kernel_org(rec, o);
    dk = kernel_dir(rec, d);
}

__device__ inline float len2(f3 v) {
#pragma clang fp contract(off)
    return fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x));
}

// particleResponse + alpha + the accept test (gaussianfunctions.glsl:192-200); one definition so the
// insert-time and composite-time evaluations are the same arithmetic (v_rsq / v_exp: parity unchanged)
__device__ inline bool particle_alpha(f3 ok, f3 dk, float l2, float density, float min_response, float alpha_min,
                                      float& galpha) {
#pragma clang fp contract(off)
    const float rl = l2 > 0.0f ? __builtin_amdgcn_rsqf(l2) : 1.0f;
    const float gx = dk.x * rl, gy = dk.y * rl, gz = dk.z * rl;
    const float cx = fmaf(gy, ok.z, -(gz * ok.y));
    const float cy = fmaf(gz, ok.x, -(gx * ok.z));
    const float cz = fmaf(gx, ok.y, -(gy * ok.x));
    const float gd = fmaf(cz, cz, fmaf(cy, cy, cx * cx));
    const float gres = __expf((KERNEL_S * gd) * gd);
    galpha = fminf(0.99f, gres * density);
    return (gres > min_response) && (galpha > alpha_min);
}

// Cell of the crossing point o + t d (grid of gvrt_lbvh.hip's k_piece_emit), each axis clamped to
// the proxy's cell range [lo, hi] so that every crossing maps to one of the proxy's pieces; packed 10
// bits per axis.  Every piece of a proxy evaluates the same expression on the same record, so a
// crossing is admitted by exactly one piece.
__device__ inline uint32_t crossing_cell(f3 o, f3 d, float t, const RenderArgs& a, uint32_t lo, uint32_t hi) {
    const float p[3] = {fmaf(t, d.x, o.x), fmaf(t, d.y, o.y), fmaf(t, d.z, o.z)};
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int l = (int)((lo >> (10 * k)) & 1023u), h = (int)((hi >> (10 * k)) & 1023u);
        const int i = (int)floorf((p[k] - a.grid_min[k]) * a.grid_inv);
        c |= (uint32_t)(i < l ? l : (i > h ? h : i)) << (10 * k);
    }
    return c;
}

// Entry / exit distance of a ray through the icosahedron proxy (kernel frame, inradius hk / sqrt(3) *
// sqrt(3) = kS): the 20 faces lie on 10 antipodal slab pairs |n . x| <= hk with the normals below
// (particlePrimitives.comp:76-79 vertices; their face planes).  Per slab the crossing interval is
// centre m = -(n . ok) / (n . dk) +- hk / |n . dk|; the reciprocal is clamped to +-1e30 so a ray
// parallel to a slab gives an unbounded interval when inside it and an empty one when outside.
__device__ inline void ico_clip(f3 ok, f3 dk, float hk, float& tn, float& tf) {
    float lo = -INFINITY, hi = INFINITY;
    // one slab at a time (short live ranges: this runs with the whole k-buffer in registers)
    auto slab = [&](float sa, float sb) {
        const float ib = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(sb), -1e30f, 1e30f);
        const float h = hk * fabsf(ib);
        lo = fmaxf(lo, fmaf(-sa, ib, -h));
        hi = fminf(hi, fmaf(-sa, ib, h));
    };
    {
        const float pxy = ok.x + ok.y, qxy = dk.x + dk.y;
        slab(pxy + ok.z, qxy + dk.z);
        slab(pxy - ok.z, qxy - dk.z);
    }
    {
        const float mxy = ok.x - ok.y, nxy = dk.x - dk.y;
        slab(mxy + ok.z, nxy + dk.z);
        slab(ok.z - mxy, dk.z - nxy);
    }
    {
        const float py = PHI * ok.y, qy = PHI * dk.y;
        slab(fmaf(IPHI, ok.z, py), fmaf(IPHI, dk.z, qy));
        slab(fmaf(-IPHI, ok.z, py), fmaf(-IPHI, dk.z, qy));
    }
    {
        const float pz = PHI * ok.z, qz = PHI * dk.z;
        slab(fmaf(IPHI, ok.x, pz), fmaf(IPHI, dk.x, qz));
        slab(fmaf(-IPHI, ok.x, pz), fmaf(-IPHI, dk.x, qz));
    }
    {
        const float px = PHI * ok.x, qx = PHI * dk.x;
        slab(fmaf(IPHI, ok.y, px), fmaf(IPHI, dk.y, qx));
        slab(fmaf(-IPHI, ok.y, px), fmaf(-IPHI, dk.y, qx));
    }
    tn = lo;
    tf = hi;
}

// arr[k] for a wave-uniform k: a select chain (s_cmp / s_cselect) over the four values.  A macro, not a
// function taking the array by reference: that form pushed the arrays to scratch (+55 % time).
template <typename T>
__device__ inline T sel4(T a0, T a1, T a2, T a3, uint32_t k) {  // values, not an array: stays s_cselect
    const T lo = (k & 1u) ? a1 : a0, hi = (k & 1u) ? a3 : a2;
    return (k & 2u) ? hi : lo;
}
#define GVRT_PICK(a, k) sel4((a)[0], (a)[1], (a)[2], (a)[3], (uint32_t)(k))

// Node fetch.  The compiler split a 128-B node into dwordx16 + dwordx8 + dwordx4 + dword loads with
// lgkmcnt waits between them (three dependent scalar round trips per node visit); the asm issues the two
// s_load_dwordx16 back to back and waits once.  The node's 32-bit byte offset rides in the loads' SGPR
// offset field (one shift instead of 64-bit pointer arithmetic per visit); so does a record's.
typedef int32_t sv16 __attribute__((ext_vector_type(16)));
struct NodeS {
    sv16 a, b;  // dwords 0..15, 16..31 of a Bvh4Node
    __device__ int32_t w(int i) const { return i < 16 ? a[i] : b[i - 16]; }
    __device__ float f(int i) const { return __int_as_float(w(i)); }
};
__device__ inline NodeS load_node_at(const Bvh4Node* __restrict__ base, int32_t idx) {
    NodeS n;
    const uint32_t off = (uint32_t)idx << 7;
    asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx16 %1, %2, %3 offset:0x40\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(n.a), "=&s"(n.b)
                 : "s"(base), "s"(off));
    return n;
}
__device__ inline RenderRec load_rec_at(const RenderRec* __restrict__ base, int32_t idx) {
    sv16 v;
    const uint32_t off = (uint32_t)idx << 6;
    asm volatile("s_load_dwordx16 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(base), "s"(off));
    return __builtin_bit_cast(RenderRec, v);
}
// ADAPTIVE: the record and its leaf's icosahedron half-width (k_leaf_hk) in one round trip
__device__ inline RenderRec load_rec_hk_at(const RenderRec* __restrict__ base, const float* __restrict__ hkbase,
                                           int32_t idx, float& hk) {
    sv16 v;
    float h;
    const uint32_t off = (uint32_t)idx << 6, off4 = (uint32_t)idx << 2;
    asm volatile("s_load_dwordx16 %0, %2, %4\n\ts_load_dword %1, %3, %5\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(v), "=&s"(h)
                 : "s"(base), "s"(hkbase), "s"(off), "s"(off4));
    hk = h;
    return __builtin_bit_cast(RenderRec, v);
}
#define NODE_BOX(nd, k, j) (nd).f(6 * (k) + (j))
#define NODE_CHILD(nd, k) (nd).w(24 + (k))
#define NODE_PAD(nd, j) (nd).w(29 + (j))

// lane id recomputed at the point of use (asm volatile: not merged with the kernel-entry value, so no
// register holds it through the traversal)
__device__ inline int lane_now() {
    int r;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
    return r;
}

// bit if the lane mask is non-empty, on the SALU (left to the compiler one of the four went through a
// v_cndmask + v_readfirstlane round trip on every node visit)
__device__ inline uint32_t nz_bit(uint64_t m, uint32_t bit) {
    uint32_t r;
    asm("s_cmp_lg_u64 %1, 0\n\ts_cselect_b32 %0, %2, 0" : "=s"(r) : "s"(m), "s"(bit) : "scc");
    return r;
}

// The lane index laundered at each LDS access inside the loops (FAST kernels): the loop-invariant per-array
// addresses (array base + lane * size) are then not hoisted into VGPRs of their own (one per array, one of
// which was spilled to scratch); each access recomputes the shift and folds the base into the DS offset.
__device__ inline int launder_lane(int l) {
    asm volatile("" : "+v"(l));
    return l;
}
__device__ inline uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

__device__ inline int32_t unii(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Dispatch geometry.  One wave per workgroup: a finished wave's slot and LDS go to the next tile at once
// (5.5 % / 4.4 % / 3.2 % faster than 2 x 2-tile workgroups on bicycle / dense / garden).  Without a tile
// list, workgroups walk ST_W x ST_H supertiles of tiles in row-major order (0.9 / 2.0 / 1.8 % faster than
// row-major tiles).  4 waves per SIMD (<= 128 VGPRs) measured fastest, ahead of 3 (no spills) and 5 (heavy
// spills or a smaller k-buffer).
// One leaf (record li) for the lanes in bk: response, icosahedron clip, k-buffer insertion.  A macro (as a lambda
// capturing the k-buffer by reference the kernel spilled 8 B per lane); round 4's wide-node traversal expanded it
// too (commit f850e68).
#define GVRT_LEAF(LI_, BK_, PIECE_)                                                                                \
    {                                                                                                              \
        const int32_t li = (LI_);                                                                                  \
        const uint64_t bk = (BK_);                                                                                 \
        float hk_leaf = 0.0f;                                                                                      \
        const RenderRec rec =                                                                                      \
            ADAPTIVE ? load_rec_hk_at(recw, a.leaf_hk, unii(li), hk_leaf) : load_rec_at(recw, unii(li));           \
                                                                                                                   \
        /* split (SplitBLAS analogue): the piece's proxy id and cell; cell == ~0u admits every crossing */         \
        uint4 pa = make_uint4((uint32_t)li, 0xFFFFFFFFu, 0u, 0u);                                                  \
        if (PIECE_) pa = aux_[li]; /* a split piece (node mark): its cell */                                       \
        {                                                                                                          \
            const uint32_t gi = (uint32_t)li; /* payload: the leaf (per-leaf records and SH, pieces too) */      \
            wadd(W_LEAVES, 1);                                                                                     \
            if (__builtin_amdgcn_inverse_ballot_w64(bk)) {  /* exec &= bk: no per-lane bit test */                 \
                ladd(L_LEAVES);                                                                                    \
                /* ---- leaf: response (processHit's math) + analytic icosahedron clip */                          \
                f3 ok, dk;                                                                                         \
                kernel_frame<OKREC, true>(rec, o, d, ok, dk);                                                      \
                /* Conservative pre-reject: gres > hitMinGaussianResponse needs the squared line */                \
                /* distance gd = |dk x ok|^2 / |dk|^2 below sqrt(ln(minResponse)/S) (a.gpre carries a */           \
                /* 1e-3 margin), so most proxies are rejected without the sqrt / exp below. */                     \
                const float l2 = len2(dk);                                                                         \
                const f3 cu = cross3(dk, ok);                                                                      \
                const bool maybe = (cu.x * cu.x + cu.y * cu.y + cu.z * cu.z) < a.gpre * l2;                        \
                bool acc = false;                                                                                  \
                float galpha = 0.0f;                                                                               \
                if (maybe) acc = particle_alpha(ok, dk, l2, rec.density, a.min_response, a.alpha_min, galpha);     \
                if (LITERAL || acc) {                                                                              \
                    /* (adaptive: sqrt(3) kernelScale(density) of the leaf, precomputed by k_leaf_hk with the */   \
                    /* same kernel_scale arithmetic) */                                                            \
                    const float hk = ADAPTIVE ? hk_leaf : a.kernel_h;                                              \
                    float tn, tf;                                                                                  \
                    ico_clip(ok, dk, hk, tn, tf);                                                                  \
                    if (tn <= tf) {                                                                                \
                        const float al = acc ? galpha : -1.0f;                                                     \
                        /* (an inclusive tmin exists only in LITERAL mode: the API refuses it otherwise) */        \
                        const bool incl = LITERAL && a.tmin_inclusive;                                             \
                        bool in0 = (incl ? tn >= tlo : tn > tlo) & (tn <= thi);                                    \
                        bool in1 = (incl ? tf >= tlo : tf > tlo) & (tf <= thi);                                    \
                        if (uni(pa.y) != 0xFFFFFFFFu) {                                                            \
                            in0 = in0 && crossing_cell(o, d, tn, a, pa.z, pa.w) == pa.y;                           \
                            in1 = in1 && crossing_cell(o, d, tf, a, pa.z, pa.w) == pa.y;                           \
                        }                                                                                          \
                        /* (bitwise &: short-circuit && became exec-mask branches around these selects) */         \
                        const bool c0 = in0 & (tn < tcut), c1 = in1 & (tf < tcut);                                 \
                        const float ta = c0 ? tn : (c1 ? tf : INF_DIST);                                           \
                        const float tb = (c0 & c1) ? tf : INF_DIST;  /* tn <= tf: in0 & in1 & tf < tcut */         \
                        if (ta < kt[KB - 1]) {                                                                     \
                          if constexpr (PACK) {                                                                    \
                            const uint32_t q = alpha_code(galpha);                                                 \
                            kb_insert2p<KB>(ta, tb, (gi << 8) | q, kt, kid);                                       \
                            /* termination cull on the q codes (see kb_insert2p): the first slot */                \
                            /* whose running sum reaches qneed is the last one composited; no */                   \
                            /* slot can reach it while the inserted total is still below */                        \
                            qtot += tb < INF_DIST ? 2 * q : q;                                                     \
                            if (__builtin_amdgcn_ballot_w64(qtot >= qneed)) TERM_WALK                             \
                          } else {                                                                                 \
                            kb_insert2<KB>(ta, tb, gi, al, kt, kid, ka);                                           \
                            /* Termination-aware cull distance: walking the sorted slots with the */               \
                            /* composite's T update, the first slot after which T <= minTransmittance */           \
                            /* is the last one that can ever be composited (the loop ends there), so */            \
                            /* nothing farther is needed.  The 1e-4 margin keeps the bound */                      \
                            /* conservative against ulp differences from the composite's arithmetic. */            \
                            float Tp = s_T[LL], tt = INF_DIST;                                                     \
                            const float term_cut = a.min_transmittance * 0.9999f;                                  \
                _Pragma("unroll")                                                                                  \
                            for (int i = 0; i < KB; ++i) {                                                         \
                                const bool acc_i = kid[i] != INVALID_ID && ka[i] > 0.0f;                           \
                                Tp = acc_i ? Tp * (1.0f - ka[i]) : Tp;                                             \
                                tt = (tt == INF_DIST && acc_i && Tp < term_cut) ? kt[i] : tt;                      \
                            }                                                                                      \
                            tcut = fminf(tcut, tt);                                                                \
                          }                                                                                        \
                        }                                                                                          \
                    }                                                                                              \
                }                                                                                                  \
            }                                                                                                      \
        }                                                                                                          \
    }

// Termination walk (kb_insert2p's cull): the first slot whose running q sum reaches qneed bounds what can still be
// composited.  3 VALU per slot: g = (qneed - running sum) x 2^100 as a float (exact: integers below 2^24 times a power of
// two), one v_cvt_f32_ubyte0 + one FMA per slot; med3(kt, g, tt) keeps tt while g > 0 (g >= 2^100 > any t) and takes
// min(kt, tt) once g <= 0, so with kt ascending tt ends at the first slot whose sum reaches qneed -- the compare /
// select / min form's result with a quarter fewer instructions (qneed above KB x 255 can never be reached and is
// clamped to 8191, which keeps that while KB x 255 < 8191: K <= 32, asserted).  Same-box: dense -1.2 %, bicycle -0.3 %
// (profiles/r05/ab/ab_walk_branchfree.log)
#define TERM_WALK                                                                           \
    {                                                                                       \
        static_assert(KB * 255 < 8191, "the qneed clamp must stay above any reachable q sum"); \
        float g = (float)(qneed < 8191u ? qneed : 8191u) * 0x1p100f;                         \
        float tt = INF_DIST;                                                                \
        _Pragma("unroll") for (int i = 0; i < KB; ++i) {                                    \
            g = fmaf((float)(kid[i] & 0xFFu), -0x1p100f, g);                                \
            tt = __builtin_amdgcn_fmed3f(kt[i], g, tt);                                     \
        }                                                                                   \
        tcut = fminf(tcut, tt);                                                             \
    }

constexpr uint32_t ST_W = 8, ST_H = 4;
constexpr int RENDER_MIN_WAVES = 4;

template <bool LITERAL, bool ADAPTIVE, int KB, bool STATS, bool PACK, bool SLACK, bool OKREC, bool OKCAM = false>
__global__ __launch_bounds__(64, RENDER_MIN_WAVES) void k_render(const RenderArgs a, const Bvh4Node* __restrict__ nodes_,
                                                                 const RenderRec* __restrict__ recs_,
                                                                 const RenderRec* __restrict__ crecs_,
                                                                 const uint4* __restrict__ aux_,
                                                                 const float* __restrict__ sh_,
                                                                 const float* __restrict__ view_inv_,
                                                                 const uint32_t* __restrict__ tiles_,
                                                                 uint8_t* __restrict__ rgba8_,
                                                                 float* __restrict__ rgba32f_,
                                                                 float* __restrict__ ray_dirs_,
                                                                 uint32_t* __restrict__ hit_counts_,
                                                                 unsigned long long* __restrict__ stats_) {
    // SH basis of each lane's ray direction, chunk-major so one ds_read_b128 per chunk is
    // conflict-free (16 KB per block; occupancy is VGPR-bound, not LDS-bound)
    __shared__ float4 s_basis[4][64];
    // composite state (rgb, alpha accumulator) and transmittance, parked in LDS during traversal so
    // their VGPRs go to the k-buffer (2 x KB registers)
    __shared__ float4 s_acc[64];
    __shared__ float s_T[64];
    __shared__ float s_last[64];  // `last` and the AABB exit: round-boundary state, not needed in traversal
    __shared__ float s_tmax[64];
    __shared__ uint32_t s_pxy[64];  // px | py << 16, parked for the output stage (not live in VGPRs)
    __shared__ unsigned long long s_t0;  // wave start (s_memtime), for the per-tile cost class
    __shared__ int32_t s_stack[STACK_DEPTH];
    // STATS: the counters live in LDS, not registers (kept in registers they spilled 76-80 B per lane, so the
    // diagnostic build had another register allocation than the shipped kernel): per wave [node visits, leaf visits,
    // node / leaf / composite cycles, dead node visits, rounds, node visits after round 1], per lane [processed
    // crossings, rounds, leaf tests]; every lane of the wave writes the same value to a wave counter
    __shared__ unsigned long long s_wst[STATS ? 8 : 1];
    __shared__ unsigned long long s_tph[STATS ? 3 : 1];  // STATS: s_memtime at the start of the node / leaf phase, wave
    __shared__ uint32_t s_lst[STATS ? 3 : 1][64];
    // lane from mbcnt (no register input)
    const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
#define LL (PACK ? launder_lane(lane) : lane)  // FAST kernels only: LITERAL spilled more with it
    // the round-boundary state (s_last, s_tmax): the unpacked kernels recompute the lane there (v_mbcnt) -- a
    // kernel-lifetime LDS address hoisted for them was the 8-24 B/lane of scratch of the K = 16 instantiations
#define LLB (PACK ? launder_lane(lane) : lane_now())
    // tile-list position: the cost-ordered permutation of the list, or the workgroup's own
    const uint64_t tile_idx = a.perm ? (uint64_t)a.perm[blockIdx.x] : (uint64_t)blockIdx.x;
    uint32_t cam, tx, ty;
    if (tiles_) {
        if (tile_idx >= a.ntiles) return;  // wave-uniform
        const uint32_t t = tiles_[tile_idx];
        cam = t >> 24;
        ty = (t >> 12) & 0xFFFu;
        tx = t & 0xFFFu;
    } else {
        // tiles in row-major order of ST_W x ST_H supertiles (row-major inside), per camera
        const uint32_t sx_n = (a.tiles_x + ST_W - 1) / ST_W, sy_n = (a.tiles_y + ST_H - 1) / ST_H;
        const uint64_t per = (uint64_t)sx_n * sy_n * (ST_W * ST_H);
        const uint64_t bid = blockIdx.x;
        cam = (uint32_t)(bid / per);
        const uint32_t rem = (uint32_t)(bid % per);
        const uint32_t st = rem / (ST_W * ST_H), in = rem % (ST_W * ST_H);
        ty = (st / sx_n) * ST_H + in / ST_W;
        tx = (st % sx_n) * ST_W + in % ST_W;
        if (tx >= a.tiles_x || ty >= a.tiles_y) return;  // wave-uniform: tile outside the frame
    }
    cam = uni(cam);
    // OKCAM: a multi-origin launch whose records carry each camera's kernel-frame origins, one copy per camera
    const RenderRec* __restrict__ recw = OKCAM ? recs_ + (uint64_t)cam * a.recs_cam_stride : recs_;
    const RenderRec* __restrict__ crecw = OKCAM ? crecs_ + (uint64_t)cam * a.recs_cam_stride : crecs_;
    const uint32_t px = tx * 8 + (lane & 7), py = ty * 8 + (lane >> 3);
    const bool valid = px < a.width && py < a.height && cam < a.ncams;

    // ---- ray generation (particleRendering.comp:123-129, raygen.rgen:116-121)
    const float* V = view_inv_ + 16 * (cam < a.ncams ? cam : 0);
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
    const f3 oinv = o * inv;
    // direction signs of the wave's first ray (bit a: negative on axis a): child visiting order
    const uint32_t rsign = uni((inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u));
    // intersectAABB (gaussianfunctions.glsl:8-16, Q12)
    float tminb, tmaxb;
    {
        const float ddx = fmaxf(d.x, 1e-6f), ddy = fmaxf(d.y, 1e-6f), ddz = fmaxf(d.z, 1e-6f);
        const float t0x = (a.aabb[0] - o.x) / ddx, t0y = (a.aabb[1] - o.y) / ddy, t0z = (a.aabb[2] - o.z) / ddz;
        const float t1x = (a.aabb[3] - o.x) / ddx, t1y = (a.aabb[4] - o.y) / ddy, t1z = (a.aabb[5] - o.z) / ddz;
        tminb = fmaxf(0.0f, fmaxf(fminf(t0x, t1x), fmaxf(fminf(t0y, t1y), fminf(t0z, t1z))));
        tmaxb = fminf(fmaxf(t0x, t1x), fminf(fmaxf(t0y, t1y), fmaxf(t0z, t1z)));
    }
    // minTransmittance x 0.9999 (v_mul by the constant, as the compiler forms it), formed where it is used: a
    // kernel-lifetime copy in a VGPR was spilled to scratch (asm volatile: not hoisted out of the loops)
    auto term_cut_now = [&]() {
        float r, k;
        asm volatile("v_mov_b32 %1, 0x3f7ff972\n\tv_mul_f32 %0, %2, %1" : "=v"(r), "=&v"(k) : "s"(a.min_transmittance));
        return r;
    };
    s_last[lane] = fmaxf(0.0f, tminb - EPS_T);
    s_tmax[lane] = tmaxb;
    s_acc[lane] = make_float4(0.0f, 0.0f, 0.0f, a.alpha_init);
    s_T[lane] = 1.0f;
    s_pxy[lane] = px | py << 16;
    if (a.tile_bucket) s_t0 = __builtin_amdgcn_s_memtime();
    // counters: the STATS instantiation keeps them in LDS (s_wst, s_lst); LITERAL keeps its round count (max_rounds)
    // in a register.  The accepted-hit count is recovered exactly from the alpha accumulator (RQ/RT alpha =
    // alpha_init + #accepted, Q10)
    uint32_t rounds = 0;
    enum { W_NODES, W_LEAVES, C_NODE, C_LEAF, C_COMP, W_DEAD, W_ROUNDS, W_LATE };
    enum { L_NPROC, L_ROUNDS, L_LEAVES };
    auto wadd = [&](int k, unsigned long long x) {  // wave counter += x (every lane writes the same sum)
        if constexpr (STATS) s_wst[k] = s_wst[k] + x;
    };
    auto ladd = [&](int k) {  // this lane's counter += 1
        if constexpr (STATS) {
            const int l = lane_now();
            s_lst[k][l] = s_lst[k][l] + 1u;
        }
    };
    if constexpr (STATS) {
        if (lane < 8) s_wst[lane] = 0ull;
        s_lst[0][lane] = s_lst[1][lane] = s_lst[2][lane] = 0u;
    }
    if constexpr (STATS) s_tph[2] = __builtin_amdgcn_s_memtime();
    bool active = valid && a.nrecs > 0 && (fmaxf(0.0f, tminb - EPS_T) <= tmaxb) && (1.0f > a.min_transmittance);
    // a wave whose active rays share one direction octant reads that octant's node copy (planes in near / far
    // order, box_hit_nf); waves straddling an axis sign (a few tiles on the lines where a direction component
    // changes sign) read the plain nodes
    bool octw = false;
    const Bvh4Node* __restrict__ nbase = nodes_;
    if (a.nodes8) {
        const uint32_t oct = (inv.x < 0.0f ? 1u : 0u) | (inv.y < 0.0f ? 2u : 0u) | (inv.z < 0.0f ? 4u : 0u);
        const uint64_t am = __builtin_amdgcn_ballot_w64(active);
        const uint32_t oct0 = (uint32_t)__builtin_amdgcn_readlane((int)oct, am ? (int)__builtin_ctzll(am) : 0);
        octw = __builtin_amdgcn_ballot_w64(active && oct != oct0) == 0;
        if (octw) nbase = a.nodes8 + a.nodes8_stride * oct0;
    }

    static_assert(!(LITERAL && PACK), "LITERAL keeps rejected crossings: unpacked k-buffer");
    float kt[KB];
    uint32_t kid[KB];       // record id, or the packed payload (id << 8 | q) when PACK
    float ka[PACK ? 1 : KB];  // alpha per slot (unpacked only; < 0 = rejected crossing in LITERAL)
    // Per-wave traversal stack in LDS
    int32_t* stack = s_stack;
    int sp = 0;
    auto push = [&](int32_t v) { stack[sp++] = v; };
    auto pop = [&]() -> int32_t { return unii(stack[--sp]); };
    {
        // radianceFromSpH basis factors (gaussianfunctions.glsl:122-151), signs folded, zero past
        // sph_eval_degree; computed once per ray and kept in LDS (not registers) through the traversal
        const float x = d.x, y = d.y, z = d.z;
        const uint32_t deg = a.sph_deg;
        const float xx = x * x, yy = y * y, zz = z * z;
        s_basis[0][lane] = make_float4(SH_C0, deg > 0 ? -(SH_C1 * y) : 0.f, deg > 0 ? SH_C1 * z : 0.f,
                                       deg > 0 ? -(SH_C1 * x) : 0.f);
        s_basis[1][lane] = make_float4(deg > 1 ? SH_C2_0 * (x * y) : 0.f, deg > 1 ? SH_C2_1 * (y * z) : 0.f,
                                       deg > 1 ? SH_C2_2 * (2.0f * zz - xx - yy) : 0.f,
                                       deg > 1 ? SH_C2_3 * (x * z) : 0.f);
        s_basis[2][lane] = make_float4(deg > 1 ? SH_C2_4 * (xx - yy) : 0.f,
                                       deg > 2 ? SH_C3_0 * y * (3.0f * xx - yy) : 0.f,
                                       deg > 2 ? SH_C3_1 * (x * y) * z : 0.f,
                                       deg > 2 ? SH_C3_2 * y * (4.0f * zz - xx - yy) : 0.f);
        s_basis[3][lane] = make_float4(deg > 2 ? SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) : 0.f,
                                       deg > 2 ? SH_C3_4 * x * (4.0f * zz - xx - yy) : 0.f,
                                       deg > 2 ? SH_C3_5 * z * (xx - yy) : 0.f,
                                       deg > 2 ? SH_C3_6 * x * (xx - 3.0f * yy) : 0.f);
    }

    while (__ballot(active)) {
        if constexpr (LITERAL) {
            if (active && a.max_rounds && rounds >= a.max_rounds) active = false;
        }
        if constexpr (LITERAL) {
            if (active) ++rounds;
        }
        if constexpr (STATS) {
            if (active) ladd(L_ROUNDS);
        }
        // (an inactive lane gets tlo = INF_DIST, so no box test of it can hit and the ballots need no AND with
        // the active mask)
        const float tlo = active ? s_last[LLB] + EPS_T : INF_DIST;
        const float thi = s_tmax[LLB] + EPS_T;
#pragma unroll
        for (int i = 0; i < KB; ++i) {
            kt[i] = INF_DIST;
            kid[i] = PACK ? PK_EMPTY : INVALID_ID;  // same all-ones value
            if constexpr (!PACK) ka[i] = 0.0f;  // never read for an empty slot, but keeps the register set defined
        }
        // PACK: optical-depth budget of this round in q units; a slot whose running q sum reaches it
        // drives T below minTransmittance (q sums never exceed the exact depth; +0.5 q of margin)
        uint32_t qneed = 0;
        if constexpr (PACK) {
            const float Tr = s_T[LL];
            const float term_cut = term_cut_now();
            const float need = Tr > term_cut ? __log2f(Tr / term_cut) * QSCALE + 0.5f : 0.0f;
            qneed = (uint32_t)fminf(ceilf(need), 4.0e9f);
        }
        uint32_t qtot = 0;  // PACK: sum of the q codes inserted this round (>= the buffer's sum)

        // ---------------- trace(): packet traversal of the 4-wide BVH
        float tcut = INF_DIST;  // termination-aware cull distance of this lane (see the leaf insert)
        sp = 0;
        int32_t cur = 0;  // node index (wave-uniform); the node is fetched at the top of each visit so its
                          // 32 SGPRs are not loop-carried
        wadd(W_ROUNDS, 1);
        while (true) {
            if constexpr (STATS) {
                wadd(W_NODES, 1);
                wadd(W_LATE, s_wst[W_ROUNDS] > 1 ? 1u : 0u);
                s_tph[0] = __builtin_amdgcn_s_memtime();  // the node phase includes the fetch
            }
            const NodeS nd = load_node_at(nbase, unii(cur));  // whole node: 2x s_load_dwordx16
            float tc = fminf(fminf(thi, kt[KB - 1]), tcut);
            float tl = tlo;
            if constexpr (PACK) {
                // acceptance-box nodes (FAST): the leaf children's boxes bound each particle's acceptance ellipsoid,
                // which lies within the node's D (pad[2]) of an admitted crossing along the ray, so the range is
                // widened by D; nodes with inner children and the proxy-box nodes carry D = 0
                const float dn = __int_as_float(unii(NODE_PAD(nd, 2)));
                tl = tlo - dn;
                tc = tc + dn;
            }
            uint64_t bal[BVH_W];
            if (octw) {
                // (an opaque copy of 1/d: otherwise the first child's plane FMAs, common to both tests, are hoisted
                // above the branch and every min / max input after it gets a canonicalising v_max)
                f3 iv = inv;
                asm("" : "+v"(iv.x), "+v"(iv.y), "+v"(iv.z));
#pragma unroll
                for (int k = 0; k < BVH_W; ++k)
                    bal[k] = __builtin_amdgcn_ballot_w64(
                        box_hit_nf<SLACK>(NODE_BOX(nd, k, 0), NODE_BOX(nd, k, 2), NODE_BOX(nd, k, 4), NODE_BOX(nd, k, 1),
                                          NODE_BOX(nd, k, 3), NODE_BOX(nd, k, 5), oinv, iv, tl, tc));
            } else {
#pragma unroll
                for (int k = 0; k < BVH_W; ++k)  // compare results straight to SGPR masks
                    bal[k] = __builtin_amdgcn_ballot_w64(
                        box_hit<SLACK>(NODE_BOX(nd, k, 0), NODE_BOX(nd, k, 2), NODE_BOX(nd, k, 4), NODE_BOX(nd, k, 1),
                                       NODE_BOX(nd, k, 3), NODE_BOX(nd, k, 5), oinv, inv, tl, tc));
            }
            int32_t ch[BVH_W];
#pragma unroll
            for (int k = 0; k < BVH_W; ++k) ch[k] = unii(NODE_CHILD(nd, k));
            // ---- children in the node's stored order (in-order of the binary split), forward when the
            // first lane's ray points along +axis, else backward: a handful of SALU ops per node
            // (sorting the hit children by the first hitting lane's entry distance cost ~100 SALU per node and
            // visited more nodes: 2.79 vs 2.18 ms)
            uint32_t hm = 0;
#pragma unroll
            for (int k = 0; k < BVH_W; ++k) hm |= nz_bit(bal[k], 1u << k);
            if constexpr (STATS) wadd(W_DEAD, hm == 0 ? 1u : 0u);
            const uint32_t inner = uni(NODE_PAD(nd, 1));
            uint32_t leafmask = hm & ~inner;
            uint32_t im = hm & inner;
            int32_t next = -1;
            if (im) {
                const bool rev = (rsign >> uni(NODE_PAD(nd, 0))) & 1u;
                const int first = rev ? 31 - __clz(im) : __ffs(im) - 1;
                next = GVRT_PICK(ch, first);
                im &= ~(1u << first);
                while (im) {  // the next child in visiting order ends on top
                    const int k = rev ? __ffs(im) - 1 : 31 - __clz(im);
                    push(GVRT_PICK(ch, k));
                    im &= ~(1u << k);
                }
            } else if (sp > 0) {
                next = pop();
            }
            if constexpr (STATS) {
                const uint64_t t = __builtin_amdgcn_s_memtime();
                wadd(C_NODE, t - s_tph[0]);
                s_tph[1] = t;
            }
            // ---- leaves of this node (the k-buffer orders them); one rolled loop = one insertion site
#pragma unroll 1
            while (leafmask) {
                const int k = __builtin_ctz(leafmask);
                leafmask &= leafmask - 1;
                // leaf slot, lanes whose ray hits its box, and whether it is a split piece (pad[1] bit 4 + k)
                GVRT_LEAF(~GVRT_PICK(ch, k), GVRT_PICK(bal, k), (inner >> (4 + k)) & 1u)
            }
            if constexpr (STATS) wadd(C_LEAF, __builtin_amdgcn_s_memtime() - s_tph[1]);
            if (next < 0) break;
            cur = next;  // uniform by construction; readfirstlane at the load lets the compiler see it
        }

        // ---------------- process k hits (particleRendering.comp:153-187)
        [[maybe_unused]] const uint64_t t_comp0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
        if (active) {
            if (kid[0] == INVALID_ID) {
                active = false;
            } else {
                float T = s_T[LL];
                float4 acc = s_acc[LL];
                float last = s_last[LLB];
                // FAST: a buffer that did not fill holds every admitted crossing of (tlo, thi] (nothing was
                // culled by kt[K-1]; what tcut culled lies past the slot where T drops below
                // minTransmittance).  Once they are composited nothing is left, so the next round that
                // the reference's loop would trace (and find empty) is skipped.
                const bool full = LITERAL || kid[KB - 1] != INVALID_ID;
                // Slots in groups of CUN (static indices inside a group, so no per-hit register shift);
                // the buffer shifts down by CUN between groups.  Per lane: stop at the first empty slot
                // or once T <= minTransmittance (slots are sorted with the empty ones last, T only falls).
                bool go = true;
                // groups of 6 at K = 24 (fewer shifts), else 4 (K = 32: 8 spills, 6 measured even)
                constexpr int CUN = (PACK && KB == 24) ? COMP_GROUP : 4;
#pragma unroll 1
                for (int base = 0; base < KB; base += CUN) {
#pragma unroll
                    for (int j = 0; j < CUN; ++j) {
                        go = go && kid[j] != INVALID_ID && T > a.min_transmittance;
                        if (!go) continue;
                        ladd(L_NPROC);
                        uint32_t hid;
                        float halpha;
                        bool hacc;
                        hid = PACK ? (kid[j] >> 8) : kid[j];
                        // the SH address needs only the id: all 12 loads in one batch, one memory round trip
                        // instead of one per dependent chunk (see SH_EARLY for where the compiler issues them);
                        // K = 32 loads the second half after the first (48 VGPRs of SH spilled the buffer)
                        constexpr int SH_FIRST = (PACK && KB > 24) ? 6 : 12;
                        static_assert(SH_FIRST >= SH_EARLY && SH_FIRST % 3 == 0, "the early chunks are loaded first");
                        float4 shv[12];
                        const float4* s4 = reinterpret_cast<const float4*>(sh_ + 48ull * hid);
#pragma unroll
                        for (int q = 0; q < SH_FIRST; ++q) shv[q] = s4[q];
                        if constexpr (PACK) {
                            // processHit re-evaluates the response of the hit particle (per-lane record load)
                            const RenderRec rec = crecw[hid];
                            f3 ok, dk;
                            kernel_frame<OKREC>(rec, o, d, ok, dk);
                            const float l2 = len2(dk);
                            hacc = particle_alpha(ok, dk, l2, rec.density, a.min_response, a.alpha_min, halpha);
                        } else {
                            halpha = ka[j];
                            hacc = ka[j] > 0.0f;
                        }
                        float er = 0.f, eg = 0.f, eb = 0.f;  // SH terms of the first SH_EARLY / 3 chunks
                        if constexpr (PACK) {
#pragma unroll
                            for (int q = 0; q < SH_EARLY / 3; ++q) {
                                const float4 v0 = shv[3 * q], v1 = shv[3 * q + 1], v2 = shv[3 * q + 2];
                                const float4 bq = s_basis[q][LL];
                                er += bq.x * v0.x; eg += bq.x * v0.y; eb += bq.x * v0.z;
                                er += bq.y * v0.w; eg += bq.y * v1.x; eb += bq.y * v1.y;
                                er += bq.z * v1.z; eg += bq.z * v1.w; eb += bq.z * v2.x;
                                er += bq.w * v2.y; eg += bq.w * v2.z; eb += bq.w * v2.w;
                            }
                        }
                        if (hacc) {
                            if constexpr (SH_FIRST < 12) {
                                asm volatile("" ::: "memory");
#pragma unroll
                                for (int q = SH_FIRST; q < 12; ++q) shv[q] = s4[q];
                            }
                            const float weight = halpha * T;
                            float rr = er, rg = eg, rb = eb;
#pragma unroll
                            for (int q = PACK ? SH_EARLY / 3 : 0; q < 4; ++q) {
                                const float4 v0 = shv[3 * q], v1 = shv[3 * q + 1], v2 = shv[3 * q + 2];
                                const float4 bq = s_basis[q][LL];
                                const float b0 = bq.x, b1 = bq.y, b2 = bq.z, b3 = bq.w;
                                // coefficients 4q..4q+3: (v0.xyz) (v0.w v1.xy) (v1.zw v2.x) (v2.yzw)
                                rr += b0 * v0.x; rg += b0 * v0.y; rb += b0 * v0.z;
                                rr += b1 * v0.w; rg += b1 * v1.x; rb += b1 * v1.y;
                                rr += b2 * v1.z; rg += b2 * v1.w; rb += b2 * v2.x;
                                rr += b3 * v2.y; rg += b3 * v2.z; rb += b3 * v2.w;
                            }
                            rr = fmaxf(rr + 0.5f, 0.0f);
                            rg = fmaxf(rg + 0.5f, 0.0f);
                            rb = fmaxf(rb + 0.5f, 0.0f);
                            acc.x += rr * weight;
                            acc.y += rg * weight;
                            acc.z += rb * weight;
                            acc.w += 1.0f;
                            T *= (1.0f - halpha);
                        }
                        last = fmaxf(last, kt[j]);
                    }
                    if (!__builtin_amdgcn_ballot_w64(go) || base + CUN >= KB) break;
#pragma unroll
                    for (int i = 0; i < KB - CUN; ++i) {
                        kt[i] = kt[i + CUN];
                        kid[i] = kid[i + CUN];
                        if constexpr (!PACK) ka[i] = ka[i + CUN];
                    }
#pragma unroll
                    for (int i = KB - CUN; i < KB; ++i) kid[i] = INVALID_ID;
                }
                active = full && (last <= s_tmax[LLB]) && (T > a.min_transmittance);
                s_last[LLB] = last;
                s_T[LL] = T;
                s_acc[LL] = acc;
            }
        }
        if constexpr (STATS) wadd(C_COMP, __builtin_amdgcn_s_memtime() - t_comp0);
    }
#undef LL
#undef LLB

    // ---------------- outputs (pixel coordinates and lane recomputed: kept live through the traversal
    // they were spilled to scratch)
    const int olane = lane_now();
    const float4 acc = s_acc[olane];
    const float cr = acc.x, cg = acc.y, cb = acc.z, calpha = acc.w;
    const uint32_t pxy = s_pxy[olane];
    const uint32_t opx = pxy & 0xFFFFu, opy = pxy >> 16;
    const bool ovalid = opx < a.width && opy < a.height && cam < a.ncams;
    const uint64_t otile = a.perm ? (uint64_t)a.perm[blockIdx.x] : (uint64_t)blockIdx.x;
    if (ovalid) {
        const uint64_t pix = ((uint64_t)cam * a.height + opy) * a.width + opx;
        const uint64_t oi = a.packed ? otile * 64 + olane : pix;
        if (rgba32f_) reinterpret_cast<float4*>(rgba32f_)[oi] = make_float4(cr, cg, cb, calpha);
        if (rgba8_) {
            auto q8 = [](float f) -> uint32_t { return (uint32_t)(fminf(fmaxf(f, 0.0f), 1.0f) * 255.0f + 0.5f); };
            reinterpret_cast<uint32_t*>(rgba8_)[oi] = q8(cr) | (q8(cg) << 8) | (q8(cb) << 16) | (q8(calpha) << 24);
        }
        if (hit_counts_) hit_counts_[oi] = (uint32_t)(calpha - a.alpha_init);
        if (ray_dirs_) {
            const uint64_t di = a.ray_dirs_layout == 1
                                    ? ((uint64_t)cam * a.width * a.height + (uint64_t)opx * a.height + opy)
                                    : pix;
            reinterpret_cast<float4*>(ray_dirs_)[di] = make_float4(d.x, d.y, d.z, 0.0f);
        }
    } else if (a.packed) {
        const uint64_t oi = otile * 64 + olane;
        if (rgba32f_) reinterpret_cast<float4*>(rgba32f_)[oi] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (rgba8_) reinterpret_cast<uint32_t*>(rgba8_)[oi] = 0u;
        if (hit_counts_) hit_counts_[oi] = 0u;
    }
    if (a.tile_bucket && olane == 0) {
        // this tile's cost class, 4 per octave of its cycles, at its tile-list position (vector store and
        // atomic from lane 0)
        const uint64_t cyc = __builtin_amdgcn_s_memtime() - s_t0;
        const float lc = (float)TILE_CPO * (__log2f((float)cyc + 1.0f) - 10.0f);  // 1 k cycles: class 0
        const uint32_t b = (uint32_t)fminf(fmaxf(lc, 0.0f), (float)(TILE_BUCKETS - 1));
        a.tile_bucket[otile] = (uint8_t)b;
        atomicAdd(a.tile_hist + b, 1u);
    }
    if constexpr (STATS) {
        unsigned long long s0 = s_lst[L_NPROC][olane], s1 = ovalid ? (uint32_t)(calpha - a.alpha_init) : 0u,
                           s2 = s_lst[L_ROUNDS][olane], s5 = s_lst[L_LEAVES][olane];
        for (int off = 32; off > 0; off >>= 1) {
            s0 += __shfl_xor(s0, off);
            s1 += __shfl_xor(s1, off);
            s2 += __shfl_xor(s2, off);
            s5 += __shfl_xor(s5, off);
        }
        if (olane == 0) {
            atomicAdd(stats_ + 0, s0);
            atomicAdd(stats_ + 1, s1);
            atomicAdd(stats_ + 2, s2);
            atomicAdd(stats_ + 3, s_wst[W_NODES]);
            atomicAdd(stats_ + 4, s_wst[W_LEAVES]);
            atomicAdd(stats_ + 5, s5);
            atomicAdd(stats_ + 6, s_wst[C_NODE]);
            atomicAdd(stats_ + 7, s_wst[C_LEAF]);
            atomicAdd(stats_ + 8, s_wst[C_COMP]);
            atomicAdd(stats_ + 9, (unsigned long long)(__builtin_amdgcn_s_memtime() - s_tph[2]));
            atomicAdd(stats_ + 10, s_wst[W_DEAD]);
            atomicAdd(stats_ + 11, s_wst[W_ROUNDS]);
            atomicAdd(stats_ + 12, s_wst[W_LATE]);
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

gvrt_status gvrt_launch_render_mode(gvrt_context* c, const RenderArgs& a, uint64_t nwaves, bool literal,
                                     hipEvent_t ev_start, hipEvent_t ev_stop) {
    uint64_t blocks = nwaves;
    if (!a.tiles)
        blocks = (uint64_t)((a.tiles_x + ST_W - 1) / ST_W) * ((a.tiles_y + ST_H - 1) / ST_H) * (ST_W * ST_H) * a.ncams;
    if (nwaves == 0 || blocks == 0) {
        GVRT_HIP(c, hipEventRecord(ev_start, c->stream));
        GVRT_HIP(c, hipEventRecord(ev_stop, c->stream));
        return GVRT_OK;
    }
    if (blocks > 0x7FFFFFFFull) return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "too many tiles");
    const bool adaptive = (a.kopts & 1u) != 0;
    const dim3 g((unsigned)blocks), b(64);
    // every pointer is its own __restrict__ argument: the uniform node / record loads can then be
    // proven unclobbered by the output stores and are emitted as scalar (s_load) loads
#define KARGS a.nodes, a.recs, a.crecs, a.aux, a.sh, a.view_inv, a.tiles, a.rgba8, a.rgba32f, a.ray_dirs, a.hit_counts, a.stats
    // the kernel-time events ride on the dispatch itself (hipExtLaunchKernelGGL): no separate event packets
    // between one frame's render and the next launch
#define GVRT_LAUNCH_SOC(L, A, K, P, S, O, C)                                                                    \
    do {                                                                                                        \
        if (a.stats)                                                                                            \
            hipExtLaunchKernelGGL((k_render<L, A, K, true, P, S, O, C>), g, b, 0, c->stream, ev_start, ev_stop, 0u, \
                                  a, KARGS);                                                                    \
        else                                                                                                    \
            hipExtLaunchKernelGGL((k_render<L, A, K, false, P, S, O, C>), g, b, 0, c->stream, ev_start, ev_stop,   \
                                  0u, a, KARGS);                                                                \
    } while (0)
#define GVRT_LAUNCH_SO(L, A, K, P, S, O) GVRT_LAUNCH_SOC(L, A, K, P, S, O, false)
#define GVRT_LAUNCH(L, A, K, P) GVRT_LAUNCH_SO(L, A, K, P, true, false)
    // FAST packed kernels also come without the per-child box slack, used when the absolute box padding
    // covers the plane rounding for this launch's cameras (RenderArgs::box_exact, set by render_impl)
#define GVRT_LAUNCH_F(K)                                                                             \
    do {                                                                                             \
        if (a.box_exact) GVRT_LAUNCH_SO(false, false, K, true, false, false);                        \
        else GVRT_LAUNCH_SO(false, false, K, true, true, false);                                     \
    } while (0)
    // packed payload needs record ids below 2^24 - 1 (id << 8 | q, all-ones = empty slot); the handle
    // option GVRT_OPT_PACKED_KBUFFER = 0 forces the unpacked path, which larger scenes take, for testing
    const bool pack = a.nrecs < 0xFFFFFFu && c->opt[GVRT_OPT_PACKED_KBUFFER] != 0;
    if (literal) {  // the reference's 16-slot k-buffer (MAX_HIT_PER_TRACE)
        if (adaptive) GVRT_LAUNCH(true, true, K_HITS, false);
        else GVRT_LAUNCH(true, false, K_HITS, false);
    } else if (!pack) {
        if (adaptive) GVRT_LAUNCH(false, true, K_HITS, false);
        else GVRT_LAUNCH(false, false, K_HITS, false);
    } else if (adaptive) {
        GVRT_LAUNCH(false, true, K_FAST_DEFAULT, true);  // adaptive leaves at the default depth (round 6)
    } else {
        // FAST: the k-buffer depth sets the number of traversal rounds; it can also move rays whose tie or threshold
        // decisions the oracle flags (a round boundary falls elsewhere), so the 24 -> 32 default change altered
        // a few flagged garden and dense rgba8 pixels (tests/test_gpu_frame_digest.py)
        switch (a.kfast) {
            case 8: GVRT_LAUNCH_F(8); break;
            case 12: GVRT_LAUNCH_F(12); break;
            case 16: GVRT_LAUNCH_F(16); break;
            case 20: GVRT_LAUNCH_F(20); break;
            case 24: GVRT_LAUNCH_F(24); break;
            default:
                // the default depth also reads kernel-frame origins from the records when render_impl
                // prepared them for a single-origin launch (RenderArgs::okrec)
                // (one record copy per camera for a multi-origin launch: RenderArgs::recs_cam_stride)
                if (a.okrec && a.recs_cam_stride) {
                    if (a.box_exact) GVRT_LAUNCH_SOC(false, false, K_FAST_DEFAULT, true, false, true, true);
                    else GVRT_LAUNCH_SOC(false, false, K_FAST_DEFAULT, true, true, true, true);
                } else if (a.okrec && a.box_exact) GVRT_LAUNCH_SO(false, false, K_FAST_DEFAULT, true, false, true);
                else if (a.okrec) GVRT_LAUNCH_SO(false, false, K_FAST_DEFAULT, true, true, true);
                else GVRT_LAUNCH_F(K_FAST_DEFAULT);
                break;
        }
    }
#undef GVRT_LAUNCH
#undef GVRT_LAUNCH_F
#undef GVRT_LAUNCH_SO
#undef GVRT_LAUNCH_SOC
#undef KARGS
    GVRT_HIP(c, hipGetLastError());
    return GVRT_OK;
}

// The next launch's dispatch order (a permutation of tile-list positions) from this launch's cost classes,
// costliest class first.  Class counts and
// fill cursors are double-buffered by launch parity: the render kernel of launch k counts into hist[k & 1],
// this kernel turns them into class starts (every block computes the 64-entry prefix), places each tile at
// start + cursor (ranks within a block by LDS atomics, one global atomic per class per block) and clears the
// other parity's arrays for launch k + 1.  Order within a class is arbitrary (it
// changes only which wave renders a tile when).
__global__ __launch_bounds__(256) void k_tile_order(uint32_t n, const uint8_t* __restrict__ bucket,
                                                    uint32_t* __restrict__ hist,
                                                    uint32_t* __restrict__ fill, uint32_t* __restrict__ hist_next,
                                                    uint32_t* __restrict__ fill_next, uint32_t* __restrict__ order,
                                                    uint32_t xcd) {
    __shared__ uint32_t base[TILE_BUCKETS];
    __shared__ uint32_t total;
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int b = TILE_BUCKETS - 1; b >= 0; --b) {
            base[b] = acc;
            acc += hist[b];
        }
        total = acc;
    }
    if (blockIdx.x == 0 && threadIdx.x < TILE_BUCKETS) {
        hist_next[threadIdx.x] = 0u;
        fill_next[threadIdx.x] = 0u;
    }
    __syncthreads();
    // block-level: ranks within the block's classes by LDS atomics, then one global cursor add per class
    __shared__ uint32_t cnt[TILE_BUCKETS], off[TILE_BUCKETS];
    if (threadIdx.x < TILE_BUCKETS) cnt[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (total != n) {  // counts not from one complete launch (never expected): the plain order, every tile once
        if (i < n) order[i] = i;
        return;
    }
    const uint32_t b = i < n ? bucket[i] : 0u;
    const uint32_t r = i < n ? atomicAdd(&cnt[b], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < TILE_BUCKETS && cnt[threadIdx.x]) off[threadIdx.x] = atomicAdd(fill + threadIdx.x, cnt[threadIdx.x]);
    __syncthreads();
    if (i < n) {
        uint32_t pos = base[b] + off[b] + r;
        if (xcd && pos < n) {
            // XCD-aware: workgroup w runs on XCD w % 8, so deal the class's ranks q to the XCDs in
            // contiguous chunks (nearby tiles share BVH nodes and records in one XCD's L2): the class
            // occupies workgroups [s, s + nc); XCD offset u = (w - s) % 8 holds cnt(u) of them.
            const uint32_t s0 = base[b], nc = hist[b], q = pos - s0;
            const uint32_t a8 = nc / 8, r8 = nc % 8;
            uint32_t u, j;
            if (q < r8 * (a8 + 1)) {
                u = q / (a8 + 1);
                j = q % (a8 + 1);
            } else {
                const uint32_t q2 = q - r8 * (a8 + 1);
                u = r8 + q2 / a8;
                j = q2 % a8;
            }
            pos = s0 + u + 8 * j;
        }
        if (pos < n) order[pos] = i;
    }
}

// Moving camera: the previous frame's cost of a screen tile predicts the cost of the tiles around it in this
// frame.  The classes are spread by a max filter of radius R tiles (R from the camera motion, render_impl) before
// ordering, so that a costly region that moved by up to R tiles still starts early (a stale exact order put the
// costly tiles of the moved view last: 2.04 ms vs 1.58 unordered at 2 deg per frame).
// k_tile_scatter: the classes of the tile list into a screen grid (one byte per tile); k_tile_dilate: per list
// position the largest class within R tiles, with the class counts for k_tile_order.
__global__ __launch_bounds__(256) void k_tile_scatter(uint32_t n, const uint32_t* __restrict__ codes,
                                                      const uint8_t* __restrict__ bucket, uint32_t tiles_x,
                                                      uint32_t tiles_y, uint8_t* __restrict__ grid,
                                                      uint32_t* __restrict__ hist_dilated) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    // the dilated class counts k_tile_dilate adds into (the previous launch's k_tile_order has read them)
    if (i < TILE_BUCKETS) hist_dilated[i] = 0u;
    if (i >= n) return;
    const uint32_t t = codes[i];
    grid[((uint64_t)(t >> 24) * tiles_y + ((t >> 12) & 0xFFFu)) * tiles_x + (t & 0xFFFu)] = bucket[i];
}
__global__ __launch_bounds__(256) void k_tile_dilate(uint32_t n, const uint32_t* __restrict__ codes,
                                                     const uint8_t* __restrict__ grid, uint32_t tiles_x,
                                                     uint32_t tiles_y, int radius, uint8_t* __restrict__ out,
                                                     uint32_t* __restrict__ hist) {
    // class counts per block in LDS, one global add per class per block (per-tile global atomics on 64 counters
    // serialised: 0.27 ms per frame)
    __shared__ uint32_t cnt[TILE_BUCKETS];
    if (threadIdx.x < TILE_BUCKETS) cnt[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
    const uint32_t t = codes[i];
    const int tx = (int)(t & 0xFFFu), ty = (int)((t >> 12) & 0xFFFu);
    const uint8_t* g = grid + (uint64_t)(t >> 24) * tiles_y * tiles_x;
    const int x0 = max(0, tx - radius), x1 = min((int)tiles_x - 1, tx + radius);
    const int y0 = max(0, ty - radius), y1 = min((int)tiles_y - 1, ty + radius);
    uint32_t m = 0;
    for (int y = y0; y <= y1; ++y)
        for (int x = x0; x <= x1; ++x) m = max(m, (uint32_t)g[(uint64_t)y * tiles_x + x]);
    m = min(m, (uint32_t)(TILE_BUCKETS - 1));  // cnt[] / k_tile_order's classes are TILE_BUCKETS wide
    out[i] = (uint8_t)m;
    atomicAdd(&cnt[m], 1u);
    }
    __syncthreads();
    if (threadIdx.x < TILE_BUCKETS && cnt[threadIdx.x]) atomicAdd(hist + threadIdx.x, cnt[threadIdx.x]);
}

gvrt_status gvrt_launch_tile_order(gvrt_context* c, const uint32_t* codes, int radius) {
    const uint32_t p = c->ord_parity;
    uint32_t* h = c->d_thist;  // [hist 0, hist 1, fill 0, fill 1, dilated hist] x TILE_BUCKETS
    const uint32_t n = (uint32_t)c->ord_n;
    // XCD-aware dealing of each cost class (GVRT_OPT_TILE_XCD = 0: off): -2 to -4 % kernel time
    const uint32_t xcd = c->opt[GVRT_OPT_TILE_XCD] != 0;
    const uint8_t* bucket = c->d_tbucket;
    uint32_t* hist = h + TILE_BUCKETS * p;
    if (radius > 0 && codes) {
        const uint64_t cells = (uint64_t)c->ord_tx * c->ord_ty * c->ord_nc;
        // the handle's own full-frame list (d_tcode: every tile exactly once) writes every grid cell; a caller's
        // list may be partial or repeat tiles, so the cells it does not write are cleared to class 0 first
        if (codes != c->d_tcode || n < cells) GVRT_HIP(c, hipMemsetAsync(c->d_tgrid, 0, cells, c->stream));
        hipLaunchKernelGGL(k_tile_scatter, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, codes, c->d_tbucket,
                           c->ord_tx, c->ord_ty, c->d_tgrid, h + 4 * TILE_BUCKETS);
        hipLaunchKernelGGL(k_tile_dilate, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, codes, c->d_tgrid,
                           c->ord_tx, c->ord_ty, radius, c->d_tbucket2, h + 4 * TILE_BUCKETS);
        bucket = c->d_tbucket2;
        hist = h + 4 * TILE_BUCKETS;
    }
    hipLaunchKernelGGL(k_tile_order, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, bucket,
                       hist, h + TILE_BUCKETS * (2 + p), h + TILE_BUCKETS * (1 - p),
                       h + TILE_BUCKETS * (3 - p), c->d_order, xcd);
    GVRT_HIP(c, hipGetLastError());
    c->ord_parity = 1 - p;
    c->ord_ready = true;
    return GVRT_OK;
}

// Record copies for FAST launches: each leaf record with its position replaced by its kernel-frame origin
// ok = S^-1 R^T (o - p) of the launch camera (kernel_org, the arithmetic the render kernel would otherwise do per
// leaf visit and per composited hit).  d_recs keeps the positions.
// (cam_dst: the camera ring slot this launch's render reads, written from the kernel argument: a moving camera then
// needs no separate host-to-device copy in the stream)
__global__ __launch_bounds__(256) void k_rec_origin(uint64_t m, const RenderRec* __restrict__ src, RenderRec* dst,
                                                    float ox, float oy, float oz, float* __restrict__ cam_dst,
                                                    const CamArg cam, uint32_t pos_only) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (cam_dst && i < 16) cam_dst[i] = cam.v[i];
    if (i >= m) return;
    RenderRec r = src[i];
    const f3 ok = kernel_org(r, mk3(ox, oy, oz));
    if (pos_only) {  // the copy's other fields already equal src's: 12 of the 64 bytes written
        dst[i].px = ok.x;
        dst[i].py = ok.y;
        dst[i].pz = ok.z;
        return;
    }
    r.px = ok.x;
    r.py = ok.y;
    r.pz = ok.z;
    dst[i] = r;
}

// Adaptive enclosing (opts & 1): each leaf's icosahedron half-width sqrt(3) kernelScale(density) -- what the leaf
// test computed per visit before (powf / logf: 36 B of scratch per lane in the render kernel)
__global__ __launch_bounds__(256) void k_leaf_hk(uint64_t m, const RenderRec* __restrict__ recs, float kmin,
                                                 uint32_t kopts, float kdeg, float* __restrict__ hk) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    hk[i] = kernel_scale(recs[i].density, kmin, kopts, kdeg) * SQRT3;
}

gvrt_status gvrt_launch_leaf_hk(gvrt_context* c) {
    const uint64_t m = c->n_leaves;
    if (!m) return GVRT_OK;
    hipLaunchKernelGGL(k_leaf_hk, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, c->stream, m, c->d_recs,
                       c->enc.kernel_min_response, c->enc.opts, c->enc.degree, c->d_leaf_hk);
    GVRT_HIP(c, hipGetLastError());
    return GVRT_OK;
}

// Multi-origin launches (a light-field rig): one record copy per camera, copy c holding camera c's origins
__global__ __launch_bounds__(256) void k_rec_origin_cams(uint64_t m, uint32_t ncams, const RenderRec* __restrict__ src,
                                                         RenderRec* dst, const float* __restrict__ view_inv) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const RenderRec r = src[i];
    for (uint32_t c = 0; c < ncams; ++c) {
        const float* v = view_inv + 16 * c;
        const f3 ok = kernel_org(r, mk3(v[12], v[13], v[14]));
        RenderRec w = r;
        w.px = ok.x;
        w.py = ok.y;
        w.pz = ok.z;
        dst[(uint64_t)c * m + i] = w;
    }
}

gvrt_status gvrt_launch_rec_cams(gvrt_context* c, uint32_t ncams, const float* d_view_inv, RenderRec* dst) {
    const uint64_t m = c->n_leaves;
    if (!m) return GVRT_OK;
    hipLaunchKernelGGL(k_rec_origin_cams, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, c->stream, m, ncams,
                       c->d_recs, dst, d_view_inv);
    GVRT_HIP(c, hipGetLastError());
    return GVRT_OK;
}

gvrt_status gvrt_launch_rec_origin(gvrt_context* c, const float* o, RenderRec* dst, hipStream_t stream,
                                   float* cam_dst, const float* cam, bool pos_only) {
    const uint64_t m = c->n_leaves;
    if (!m) return GVRT_OK;
    CamArg ca;
    CamArg ca0 = {};
    ca = ca0;
    if (cam_dst)
        for (int k = 0; k < 16; ++k) ca.v[k] = cam[k];
    hipLaunchKernelGGL(k_rec_origin, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, m, c->d_recs, dst,
                       o[0], o[1], o[2], cam_dst, ca, pos_only ? 1u : 0u);
    GVRT_HIP(c, hipGetLastError());
    return GVRT_OK;
}

// The 8 octant copies of the 4-wide nodes: copy o stores, for every axis a with bit a of o set (rays along
// -a), each child box's (hi, lo) in the (lo, hi) slots, so a wave of octant o finds its near planes in the lo
// slots.  Empty slots hold EMPTY_BOX in all six and stay unhittable; children and flags are copied unchanged.
__global__ __launch_bounds__(256) void k_node_octants(uint64_t n, const Bvh4Node* __restrict__ src,
                                                      Bvh4Node* __restrict__ dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 8 * n) return;
    const uint32_t o = (uint32_t)(i / n);
    Bvh4Node nd = src[i % n];
#pragma unroll
    for (int k = 0; k < BVH_W; ++k)
#pragma unroll
        for (int ax = 0; ax < 3; ++ax)
            if ((o >> ax) & 1u) {
                const float lo = nd.box[k][2 * ax];
                nd.box[k][2 * ax] = nd.box[k][2 * ax + 1];
                nd.box[k][2 * ax + 1] = lo;
            }
    dst[i] = nd;
}

gvrt_status gvrt_launch_node_octants(gvrt_context* c) {
    const uint64_t n = c->n_nodes4;
    if (!n || !c->d_nodes4) return GVRT_OK;
    // 8 x the node array (0.46 GB at 1 M Gaussians); when it does not fit, waves read the plain nodes
    if (!gvrt_dalloc_optional(c, (void**)&c->d_nodes4x8, 8 * n * sizeof(Bvh4Node))) return GVRT_OK;
    hipLaunchKernelGGL(k_node_octants, dim3((unsigned)((8 * n + 255) / 256)), dim3(256), 0, c->stream, n, c->d_nodes4,
                       c->d_nodes4x8);
    GVRT_HIP(c, hipGetLastError());
    return GVRT_OK;
}

// ---- Acceptance boxes (FAST launches, handle option GVRT_OPT_ACCEPT_BOXES).
// In FAST mode only accepted crossings enter the k-buffer, and a crossing of particle P is accepted only if
// gres > hitMinGaussianResponse and min(0.99, gres * density) > alphaMinThreshold (gaussianfunctions.glsl:192-200),
// i.e. gres > m = max(min_response, alpha_min / density), with gres = exp(S d^4) and d the distance of the ray's
// line from P's centre in the kernel frame.  So the line passes through the ball E = {|x_k| <= r}, r^4 = ln(m) / S.
// The proxy's AABB is larger (the icosahedron's circumradius is Rc = 1.258 kS, r <= kS when min_response is the
// enclosing pass's kernel response, and r shrinks with density).  In this copy of the nodes the leaves of every
// all-leaf node get the boxes of E, and particles that can never be accepted (density <= alpha_min) are dropped
// everywhere.  The admitted crossing (entry or exit face, in (tlo, tc]) lies on the proxy and, along the line, at
// most sqrt(Rc^2 - r^2) (kernel frame) from E's chord, i.e. D = s_max sqrt(Rc^2 - r^2) in t, so an all-leaf node's
// children are tested over [tlo - D, tc + D], D the largest of its leaves' (pad[2]; 0 elsewhere and in the
// proxy-box nodes).  Nodes with inner children keep their proxy boxes: one D per node would widen the inner
// children's range too (every node on E boxes refit upwards, or a per-child D, measured slower: DESIGN.md §4).
// Which crossings are admitted does not change, only which leaves a wave visits.  A split piece (SplitBLAS
// analogue) admits only the crossings in its own box, so its acceptance box is E's box clipped to the piece's box
// grown by the leaf's own D (the line's point in E lies within D of such a crossing); a piece E cannot reach is dropped.
constexpr float ICO_CIRCUM = 1.2584086f;  // icosahedron circumradius / inradius
__device__ inline bool slot_empty(const Bvh4Node& n, int k) { return n.box[k][0] > 1e37f; }
__device__ inline void set_empty(Bvh4Node& n, int k) {
#pragma unroll
    for (int j = 0; j < 6; ++j) n.box[k][j] = EMPTY_BOX;
}

struct AcceptArgs {
    float min_response, alpha_min, kmin, kdeg, pad_abs;
    uint32_t kopts;
    uint32_t split;  // leaves are split pieces (gvrt_accel_params.split_cells)
};

__global__ __launch_bounds__(256) void k_accept_leaf(uint64_t n, const Bvh4Node* __restrict__ src,
                                                     const RenderRec* __restrict__ recs, AcceptArgs p,
                                                     Bvh4Node* __restrict__ dst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Bvh4Node nd = src[i];
    float dmax = 0.0f;
    // a node with inner children keeps its leaves' proxy boxes (D = 0 would not cover the acceptance boxes, and a
    // D > 0 would widen the inner children's range too); only never-accepted leaves are dropped there
    const bool all_leaves = (nd.pad[1] & 0xFu) == 0u;
#pragma unroll
    for (int k = 0; k < BVH_W; ++k) {
        if (slot_empty(nd, k) || nd.child[k] >= 0) continue;
        const RenderRec r = recs[~nd.child[k]];
        const float rho = r.density;
        // a NaN density keeps its proxy box: the render's min(0.99, gres * NaN) is 0.99, i.e. accepted
        if (rho != rho) continue;
        // (alpha_min >= 0.99: galpha = min(0.99, .) never exceeds it)
        const float m = fmaxf(p.min_response, p.alpha_min / rho);  // > 0 (render_impl: min_response or alpha_min > 0)
        if (!(rho > p.alpha_min) || !(m < 1.0f) || !(p.alpha_min < 0.99f)) {
            set_empty(nd, k);
            continue;
        }
        // (a non-positive density with a negative alpha_min is accepted outside a shell, not inside a ball:
        // sigmoid-activated densities are positive, but such a leaf keeps its proxy box)
        if (!all_leaves || !(rho > 0.0f)) continue;
        const float re = powf(logf(m) / KERNEL_S, 0.25f) * 1.01f;  // 1 % margin on r
        const float sx = 1.0f / r.isx, sy = 1.0f / r.isy, sz = 1.0f / r.isz;
        // world = p + R diag(s) x_k; row i of R diag(s) = (c_i.x sx, c_i.y sy, c_i.z sz) (kernel_org's columns)
        const float hx = re * sqrtf(r.c0x * r.c0x * sx * sx + r.c0y * r.c0y * sy * sy + r.c0z * r.c0z * sz * sz);
        const float hy = re * sqrtf(r.c1x * r.c1x * sx * sx + r.c1y * r.c1y * sy * sy + r.c1z * r.c1z * sz * sz);
        const float hz = re * sqrtf(r.c2x * r.c2x * sx * sx + r.c2y * r.c2y * sy * sy + r.c2z * r.c2z * sz * sz);
        const float c3[3] = {r.px, r.py, r.pz}, h3[3] = {hx, hy, hz};
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
            // the proxy boxes' padding (gvrt_enclose.hip), so the render kernel's plane rounding is covered alike
            const float lo = c3[ax] - h3[ax] * 1.0001f, hi = c3[ax] + h3[ax] * 1.0001f;
            const float pad = 1e-5f * (hi - lo) + 1e-6f * fabsf(c3[ax]) + p.pad_abs + 1e-30f;
            nd.box[k][2 * ax] = lo - pad;
            nd.box[k][2 * ax + 1] = hi + pad;
        }
        // the icosahedron the render kernel clips against: inradius kS (kernel_scale with the enclosing options)
        const float rc = ICO_CIRCUM * 1.001f * kernel_scale(rho, p.kmin, p.kopts, p.kdeg);
        const float gap = sqrtf(fmaxf(rc * rc - re * re, 0.0f));
        const float dk = gap * fmaxf(sx, fmaxf(sy, sz)) * 1.01f + 4.0f * p.pad_abs;
        if (p.split) {
            // a piece admits only the crossings whose point lies in its box (the proxy's box clipped to its cell):
            // the line's point in E lies within dk of such a crossing, so E's box meets the piece's box grown by dk
            // (+ its own padding); a piece whose cell E cannot reach that way never admits an accepted crossing
            bool empty = false;
            const Bvh4Node& sn = src[i];
#pragma unroll
            for (int ax = 0; ax < 3; ++ax) {
                const float plo = sn.box[k][2 * ax], phi = sn.box[k][2 * ax + 1];
                const float pad = 1e-5f * (phi - plo + 2.0f * dk) + 1e-6f * fmaxf(fabsf(plo), fabsf(phi)) + p.pad_abs;
                const float lo = fmaxf(nd.box[k][2 * ax], plo - dk - pad);
                const float hi = fminf(nd.box[k][2 * ax + 1], phi + dk + pad);
                nd.box[k][2 * ax] = lo;
                nd.box[k][2 * ax + 1] = hi;
                empty = empty || !(lo <= hi);
            }
            if (empty) {
                set_empty(nd, k);
                continue;
            }
        }
        dmax = fmaxf(dmax, dk);
    }
    nd.pad[2] = __float_as_uint(dmax);
    dst[i] = nd;
}

gvrt_status gvrt_launch_accept_nodes(gvrt_context* c, float min_response, float alpha_min) {
    const uint64_t n = c->n_nodes4;
    c->accept_ok = false;
    if (!n || !c->d_nodes4) return GVRT_OK;
    if (!c->d_nodes4e) {
        // without the memory FAST launches keep the proxy-box nodes (no retry until the next build)
        if (c->accept_nomem) return GVRT_OK;
        if (!gvrt_dalloc_optional(c, (void**)&c->d_nodes4e, n * sizeof(Bvh4Node))) {
            c->accept_nomem = true;
            return GVRT_OK;
        }
        // octant copies: without them (no memory) the octant waves read the plain acceptance nodes
        (void)gvrt_dalloc_optional(c, (void**)&c->d_nodes4ex8, 8 * n * sizeof(Bvh4Node));
    }
    AcceptArgs p;
    p.min_response = min_response;
    p.alpha_min = alpha_min;
    p.kmin = c->enc.kernel_min_response;
    p.kdeg = c->enc.degree;
    p.kopts = c->enc.opts;
    p.pad_abs = c->box_pad_abs;
    p.split = c->split_cells ? 1u : 0u;
    hipLaunchKernelGGL(k_accept_leaf, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, n, c->d_nodes4,
                       c->d_recs, p, c->d_nodes4e);
    if (c->d_nodes4ex8)
        hipLaunchKernelGGL(k_node_octants, dim3((unsigned)((8 * n + 255) / 256)), dim3(256), 0, c->stream, n,
                           c->d_nodes4e, c->d_nodes4ex8);
    GVRT_HIP(c, hipGetLastError());
    c->accept_key[0] = min_response;
    c->accept_key[1] = alpha_min;
    c->accept_ok = true;
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
