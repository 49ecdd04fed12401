// ============================================================================
// gvrt_oracle.cpp — CPU ORACLE for the Gaussian ray-traced Particle Rendering
// path of wlckslxh/3DGVRT_lightfield.
//
//   *** TEST INFRASTRUCTURE ONLY ***
//   Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may
//   load this library, and only as the checker / CPU baseline.  The product
//   (3dgvrt_lightfield_amd/libgvrt.so) never links, loads or calls it.
//
// What it restates (reference paths relative to /root/reference):
//   * Gaussian Enclosing pass   shaders/glsl/VulkanFullRT/particlePrimitives.comp:81-215
//       (kernelScale :81-105, sigmoid :107-110, filter :120-140, compaction :142,
//        icosahedron :153-185, density record :187-205, SH record :207-214)
//   * utils                     shaders/glsl/base/utils.glsl:8-56
//   * math / constants          shaders/glsl/base/3dgs.glsl:13-71
//   * processHit & friends      shaders/glsl/base/gaussianfunctions.glsl:8-229
//   * ray-march round loop      shaders/glsl/VulkanFullRT/particleRendering.comp:117-191 (RQ)
//                               shaders/glsl/VulkanFullRT/raygen.rgen:113-193 (RT)
//                               shaders/glsl/VulkanFullRT/raygenGaussianLightField.rgen:114-202 (LF)
//   * k-buffer any-hit          shaders/glsl/VulkanFullRT/anyhit.rahit:29-71,
//                               particleRendering.comp:63-115
//   * acceleration structure    projects/VulkanFullRT/VulkanFullRT.cpp:575-787: a BLAS over the
//       20 triangles of every proxy, non-opaque, instance FACING_CULL_DISABLE (both faces hit).
//       The driver's traversal is replaced here by a CPU BVH + watertight ray/triangle test
//       (Woop, Benthin & Wald 2013), i.e. a restatement of the published algorithm; the
//       driver's internal ordering of equal-t candidates is not observable.
//
// Parity status: no golden vector produced by the reference exists
// for this path (its only end-to-end PNGs need an absent asset), so the render
// restatement is pinned by analytic known-answer tests (tests/test_oracle_kat.py) and by the
// reference's own PLY loader compiled from source (oracle/_ref, row 1).  Traversal-level parity
// with the NVIDIA driver is "parity unpinned" (SURVEY §8c).
//
// Semantic switches (SURVEY §8a quirk index):
//   pixel_offset 0 (RQ, default) / 0.5 (RT, LF)                      Q11
//   alpha_init   0 (RQ, default) / 1 (RT, LF)                        Q10
//   tmin_inclusive 0 (default, see DESIGN.md: an inclusive tmin would make every ray whose
//                  farthest crossing is rejected loop forever) / 1   Q13
//   proxy_mode   0 literal 20-triangle soup, 1 analytic icosahedron (10 slab pairs)
//   drop_rejected 0 literal k-buffer / 1 only accepted crossings enter the k-buffer
//                 (identical image when tmin is exclusive; used to prove the HIP fast path)
// ============================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct V3 {
    float x, y, z;
};
inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
inline V3 operator*(float s, V3 a) { return v3(a.x * s, a.y * s, a.z * s); }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
inline float length(V3 a) { return std::sqrt(dot(a, a)); }
inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// GLSL mat3 is column-major: c[0], c[1], c[2] are columns; M*v = c0*v.x + c1*v.y + c2*v.z.
struct M3 {
    V3 c[3];
};
inline V3 mul(const M3& m, V3 v) { return m.c[0] * v.x + m.c[1] * v.y + m.c[2] * v.z; }

// utils.glsl:8-11
inline V3 safeNormalize(V3 v) {
    const float l = v.x * v.x + v.y * v.y + v.z * v.z;
    return l > 0.0f ? (v * (1.0f / std::sqrt(l))) : v;
}

// utils.glsl:13-34 (returns the TRANSPOSE of the standard rotation: SURVEY §8a row 11)
inline M3 quaternionWXYZToMatrix(const float q[4]) {
    const float w = q[0], x = q[1], y = q[2], z = q[3];
    const float xx = x * x, yy = y * y, zz = z * z;
    const float xy = x * y, xz = x * z, yz = y * z;
    const float wx = w * x, wy = w * y, wz = w * z;
    M3 m;
    m.c[0] = v3(1.0f - 2.0f * (yy + zz), 2.0f * (xy - wz), 2.0f * (xz + wy));
    m.c[1] = v3(2.0f * (xy + wz), 1.0f - 2.0f * (xx + zz), 2.0f * (yz - wx));
    m.c[2] = v3(2.0f * (xz - wy), 2.0f * (yz + wx), 1.0f - 2.0f * (xx + yy));
    return m;
}

// utils.glsl:36-56 (the standard rotation R; world = R * local)
inline M3 quaternionWXYZToMatrixTranspose(const float q[4]) {
    const float w = q[0], x = q[1], y = q[2], z = q[3];
    const float xx = x * x, yy = y * y, zz = z * z;
    const float xy = x * y, xz = x * z, yz = y * z;
    const float wx = w * x, wy = w * y, wz = w * z;
    M3 m;
    m.c[0] = v3(1.0f - 2.0f * (yy + zz), 2.0f * (xy + wz), 2.0f * (xz - wy));
    m.c[1] = v3(2.0f * (xy - wz), 1.0f - 2.0f * (xx + zz), 2.0f * (yz + wx));
    m.c[2] = v3(2.0f * (xz + wy), 2.0f * (yz - wx), 1.0f - 2.0f * (xx + yy));
    return m;
}

// ---------------------------------------------------------------- constants (3dgs.glsl)
const float EPS_T = 1e-9f;                       // 3dgs.glsl:13
const uint32_t MAX_HIT_PER_TRACE = 16;           // 3dgs.glsl:15
const uint32_t INVALID_PARTICLE_ID = 0xFFFFFFFFu; // 3dgs.glsl:26
const float INFINITE_DISTANCE = 1e20f;           // 3dgs.glsl:27
const uint32_t SPECULAR_DIMENSION = 45;          // 3dgs.glsl:14
const float SH_C0 = 0.28209479177387814f;        // 3dgs.glsl:34-49
const float SH_C1 = 0.4886025119029199f;
const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                        -1.0925484305920792f, 0.5462742152960396f};
const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                        0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                        -0.5900435899266435f};

// particlePrimitives.comp:74-79
const float goldenRatio = 1.618033988749895f;
const float icosaEdge = 1.323169076499215f;
const float icosaVrtScale = 0.5f * icosaEdge;
const V3 icosaHedronVrt[12] = {
    {-1, goldenRatio, 0}, {1, goldenRatio, 0},  {0, 1, -goldenRatio},  {-goldenRatio, 0, -1},
    {-goldenRatio, 0, 1}, {0, 1, goldenRatio},  {goldenRatio, 0, 1},   {0, -1, goldenRatio},
    {-1, -goldenRatio, 0}, {0, -1, -goldenRatio}, {goldenRatio, 0, -1}, {1, -goldenRatio, 0}};
const uint32_t icosaHedronTri[20][3] = {
    {0, 1, 2},  {0, 2, 3},  {0, 3, 4},  {0, 4, 5},  {0, 5, 1},  {6, 1, 5},  {6, 5, 7},
    {6, 7, 11}, {6, 11, 10}, {6, 10, 1}, {8, 4, 3},  {8, 3, 9},  {8, 9, 11}, {8, 11, 7},
    {8, 7, 4},  {9, 3, 2},  {9, 2, 10}, {9, 10, 11}, {5, 4, 7},  {1, 10, 2}};

// particlePrimitives.comp:81-105
float kernelScale(float density, float modulatedMinResponse, uint32_t opts, float kernelDegree) {
    const float responseModulation = (opts & 1u) != 0 ? density : 1.0f;
    const float minResponse = std::min(modulatedMinResponse / responseModulation, 0.97f);
    if (kernelDegree < 0) {
        const float k = std::fabs(kernelDegree);
        const float s = 1.0f / std::pow(3.0f, k);
        const float ks = std::pow((1.f / (std::log(minResponse) - 1.f) + 1.f) / s, 1.f / k);
        return ks;
    }
    if (kernelDegree == 0) {
        return ((1.0f - minResponse) / 3.0f) / -0.329630334487f;
    }
    const float b = kernelDegree;
    const float a = -4.5f / std::pow(3.0f, b);
    return std::pow(std::log(minResponse) / a, 1.0f / b);
}

// particlePrimitives.comp:107-110
inline float sigmoid(float x) { return 1.0f / (1.0f + std::exp(-x)); }

// gaussianfunctions.glsl:18-57, PARTICLE_KERNEL_DEGREE = 4 (3dgs.glsl:22)
inline float particleResponse(float grayDist) {
    const float s = -0.0555555555556f;
    return std::exp(s * grayDist * grayDist);
}

// gaussianfunctions.glsl:8-16 (Q12: max(dir, 1e-6) leaves negative components unconstrained)
inline void intersectAABB(const float aabb[6], V3 o, V3 d, float& tmin, float& tmax) {
    const V3 dd = v3(std::max(d.x, 1e-6f), std::max(d.y, 1e-6f), std::max(d.z, 1e-6f));
    const V3 t0 = v3((aabb[0] - o.x) / dd.x, (aabb[1] - o.y) / dd.y, (aabb[2] - o.z) / dd.z);
    const V3 t1 = v3((aabb[3] - o.x) / dd.x, (aabb[4] - o.y) / dd.y, (aabb[5] - o.z) / dd.z);
    const V3 tM = v3(std::max(t0.x, t1.x), std::max(t0.y, t1.y), std::max(t0.z, t1.z));
    const V3 tm = v3(std::min(t0.x, t1.x), std::min(t0.y, t1.y), std::min(t0.z, t1.z));
    tmin = std::max(0.0f, std::max(tm.x, std::max(tm.y, tm.z)));
    tmax = std::min(tM.x, std::min(tM.y, tM.z));
}

// gaussianfunctions.glsl:122-151
V3 radianceFromSpH(uint32_t deg, const V3 c[16], V3 rdir, bool clamped) {
    V3 rad = SH_C0 * c[0];
    if (deg > 0) {
        const float x = rdir.x, y = rdir.y, z = rdir.z;
        rad = rad - SH_C1 * y * c[1] + SH_C1 * z * c[2] - SH_C1 * x * c[3];
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            rad = rad + SH_C2[0] * xy * c[4] + SH_C2[1] * yz * c[5] +
                  SH_C2[2] * (2.0f * zz - xx - yy) * c[6] + SH_C2[3] * xz * c[7] +
                  SH_C2[4] * (xx - yy) * c[8];
            if (deg > 2) {
                rad = rad + SH_C3[0] * y * (3.0f * xx - yy) * c[9] + SH_C3[1] * xy * z * c[10] +
                      SH_C3[2] * y * (4.0f * zz - xx - yy) * c[11] +
                      SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * c[12] +
                      SH_C3[4] * x * (4.0f * zz - xx - yy) * c[13] +
                      SH_C3[5] * z * (xx - yy) * c[14] + SH_C3[6] * x * (xx - 3.0f * yy) * c[15];
            }
        }
    }
    rad = rad + v3(0.5f, 0.5f, 0.5f);
    return clamped ? v3(std::max(rad.x, 0.0f), std::max(rad.y, 0.0f), std::max(rad.z, 0.0f)) : rad;
}

struct Scene {
    const float* verts;    // 36*M  (particlePrimitives.comp:162-167)
    const uint32_t* tris;  // 60*M  (particlePrimitives.comp:179-185)
    const float* density;  // 12*M  std140 ParticleDensity (3dgs.glsl:56-62)
    const float* sh;       // 48*M  (particlePrimitives.comp:207-214)
    uint32_t M;
    std::vector<float> kS;  // per-particle kernel scale (analytic proxy only)
};

// gaussianfunctions.glsl:153-229 processHit (SURFEL_PRIMITIVE false, ENABLE_NORMALS false)
// cond (parity accounting only): the relative change of gres per ulp of rounding in the ray or the kernel-frame
// origin.  The line's distance from the centre, |gcrod| = |grd x gro|, is a difference of products of size |gro|,
// so one ulp moves it by ~ |gro| 2^-24, and ln gres = S grayDist^2 = S |gcrod|^4 moves by 4 |ln gres| times its
// relative change: cond = 4 |ln gres| |gro| / |gcrod| 2^-24.  A particle far away in kernel units (|gro| of
// several hundred: small and distant) makes the response ill-conditioned, and two float evaluations of it (the
// GPU's v_rsq / FMA order, this CPU's) can then differ by more than the fixed THR_EPS.
struct HitEval {
    float gres, galpha;
    float cond = 0.0f;
    // the same for a rounding of the world-space ray (its direction moves by up to ~3 ulps between evaluations): an
    // error of |o - p| 2^-24 in world units reaches the kernel frame amplified by up to 1 / s_min, which exceeds |gro|
    // for an anisotropic particle seen along a long axis (parity accounting of values, FLAG_VALUE_EPS)
    float vcond = 0.0f;
};
constexpr float ULP = 5.9604645e-8f;  // 2^-24

// Parity accounting only (oracle_params::perturb_ulps, tests/test_oracle_kat.py): "another float evaluation" of the
// same ray -- the ray direction and each particle's kernel-frame origin and direction moved by a pseudo-random
// whole number of ulps in [-g_jig_ulps, g_jig_ulps], seeded by (ray, particle) so that every evaluation of one
// crossing (clip, insert-time and composite-time response) sees the same perturbation, as on the GPU.
thread_local uint32_t g_jig_ulps = 0;
thread_local uint64_t g_jig_ray = 0;
inline uint64_t mix64(uint64_t h) {
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return h;
}
inline float jigf(float x, uint64_t& h) {
    h = mix64(h + 0x9E3779B97F4A7C15ull);
    const int32_t k = (int32_t)(h % (2 * g_jig_ulps + 1)) - (int32_t)g_jig_ulps;
    for (int32_t i = 0; i < std::abs(k); ++i) x = std::nextafter(x, k > 0 ? INFINITY : -INFINITY);
    return x;
}
inline V3 jig3(V3 v, uint64_t& h) {
    if (!g_jig_ulps) return v;
    const float x = jigf(v.x, h), y = jigf(v.y, h), z = jigf(v.z, h);
    return v3(x, y, z);
}
inline uint64_t jig_seed(uint32_t idx) { return mix64(g_jig_ray * 0x100000001B3ull + idx + 1); }
inline float responseCond(float grayDist, float gro_len) {
    // |ln gres| = |S| grayDist^2 and |gcrod| = sqrt(grayDist)
    if (!(grayDist > 0.0f)) return 0.0f;
    return 4.0f * 0.0555555555556f * grayDist * std::sqrt(grayDist) * gro_len * ULP;
}
inline HitEval evalResponse(const Scene& s, uint32_t idx, V3 o, V3 d) {
    const float* rec = s.density + 12ull * idx;  // fetchParticleDensity :89-101
    const V3 pos = v3(rec[0], rec[1], rec[2]);
    const float dens = rec[3];
    const M3 R = quaternionWXYZToMatrix(rec + 4);
    const V3 scl = v3(rec[8], rec[9], rec[10]);
    const V3 giscl = v3(1 / scl.x, 1 / scl.y, 1 / scl.z);
    const V3 gposc = o - pos;
    const V3 gposcr = mul(R, gposc);
    uint64_t jh = jig_seed(idx);
    const V3 gro = jig3(giscl * gposcr, jh);
    const V3 rayDirR = mul(R, d);
    const V3 grdu = jig3(giscl * rayDirR, jh);
    const V3 grd = safeNormalize(grdu);
    const V3 gcrod = cross(grd, gro);
    const float grayDist = dot(gcrod, gcrod);
    HitEval h;
    h.gres = particleResponse(grayDist);
    h.galpha = std::min(0.99f, h.gres * dens);
    h.cond = responseCond(grayDist, length(gro));
    h.vcond = responseCond(grayDist, std::max(length(gro), length(gposc) * std::max(giscl.x, std::max(giscl.y, giscl.z))));
    return h;
}

struct RayState {
    float T;
    float rad[4];
    float depth;
};

// flip (parity accounting, marchRay's alternatives): the accept test taken the other way
bool processHit(const Scene& s, V3 o, V3 d, uint32_t idx, float minKernelDensity, float minAlpha,
                uint32_t sphEvalDegree, RayState& st, HitEval* eval = nullptr, float* radmax = nullptr,
                bool flip = false) {
    const float* rec = s.density + 12ull * idx;
    const V3 pos = v3(rec[0], rec[1], rec[2]);
    const float dens = rec[3];
    const M3 R = quaternionWXYZToMatrix(rec + 4);
    const V3 scl = v3(rec[8], rec[9], rec[10]);
    const V3 giscl = v3(1 / scl.x, 1 / scl.y, 1 / scl.z);
    const V3 gposc = o - pos;
    const V3 gposcr = mul(R, gposc);
    uint64_t jh = jig_seed(idx);
    const V3 gro = jig3(giscl * gposcr, jh);
    const V3 rayDirR = mul(R, d);
    const V3 grdu = jig3(giscl * rayDirR, jh);
    const V3 grd = safeNormalize(grdu);
    const V3 gcrod = cross(grd, gro);
    const float grayDist = dot(gcrod, gcrod);
    const float gres = particleResponse(grayDist);
    const float galpha = std::min(0.99f, gres * dens);
    const bool acceptHit = flip != ((gres > minKernelDensity) && (galpha > minAlpha));
    if (eval)
        *eval = HitEval{gres, galpha, responseCond(grayDist, length(gro)),
                        responseCond(grayDist, std::max(length(gro), length(gposc) * std::max(giscl.x, std::max(giscl.y, giscl.z))))};
    if (acceptHit) {
        const float weight = galpha * st.T;
        const V3 grds = scl * grd * dot(grd, -1.0f * gro);
        const float hitT = std::sqrt(dot(grds, grds));
        V3 c[16];
        const float* shp = s.sh + 48ull * idx;  // fetchParticleSphCoefficients :104-115
        for (int i = 0; i < 16; ++i) c[i] = v3(shp[3 * i], shp[3 * i + 1], shp[3 * i + 2]);
        const V3 grad = radianceFromSpH(sphEvalDegree, c, d, true);
        if (radmax) *radmax = std::max(*radmax, std::max(grad.x, std::max(grad.y, grad.z)));
        st.rad[0] += grad.x * weight;
        st.rad[1] += grad.y * weight;
        st.rad[2] += grad.z * weight;
        st.rad[3] += 1.0f;  // Q10: alpha counts accepted hits
        st.T *= (1 - galpha);
        st.depth += hitT * weight;
    }
    return acceptHit;
}

// largest colour channel of particle idx's radiance along d (parity accounting: the colour a flipped decision moves)
float radianceMax(const Scene& s, uint32_t idx, V3 d, uint32_t sphEvalDegree) {
    V3 c[16];
    const float* shp = s.sh + 48ull * idx;
    for (int i = 0; i < 16; ++i) c[i] = v3(shp[3 * i], shp[3 * i + 1], shp[3 * i + 2]);
    const V3 r = radianceFromSpH(sphEvalDegree, c, d, true);
    return std::max(r.x, std::max(r.y, r.z));
}

// Thresholds of the parity accounting (oracle/oracle.py THR_EPS, PAIR_EPS, BOUND_EPS must equal these:
// oracle_flag_eps, tests/test_oracle_kat.py)
constexpr float FLAG_THR_EPS = 1e-4f, FLAG_PAIR_EPS = 2e-6f, FLAG_BOUND_EPS = 1e-5f;
// Ill-conditioned values (round 6): an accepted crossing whose response is ill-conditioned (a particle far away in
// kernel units: a tiny Gaussian seen from afar, whose response depends on the ray to ~|gro| ulps) moves the colour by
// about 2 T a c x its relative change even when no decision is near a threshold.  Per accepted crossing j, v_j = 2 T_j
// a_j vcond_j c (one ulp of its inputs, HitEval::vcond: the world-space ray's rounding amplified by |o - p| / s_min
// where that exceeds |gro|, an anisotropic particle seen along a long axis, randomised sweep case 77; c the ray's
// largest radiance channel): a ray whose largest v_j exceeds
// FLAG_VALUE_EPS (colour units, half the 1e-4 comparison tolerance) is flagged, and its value bound vb =
// FLAG_VALUE_ULPS x sum_j v_j joins its flip bound.  (Calibrated: an ordinary crossing of the stand-ins has v_j ~ 2e-5,
// and the GPU's unflagged rays stay within 4.3e-5 of the oracle on 47 M rays; a 1e-4-scale Gaussian 1.8 units away
// has v_j ~ 3e-4.)
constexpr float FLAG_VALUE_EPS = 5e-5f, FLAG_VALUE_ULPS = 2.0f;
// Conditioning-aware margins (unflagged rays beyond 1e-4 were all threshold or pair decisions of
// ill-conditioned crossings).  A decision is flagged when it lies within its fixed epsilon or within FLAG_COND_ULPS
// ulps of rounding of its inputs, whichever is larger: a response threshold within FLAG_COND_ULPS x cond (HitEval),
// the transmittance within the summed relative error of its factors, two crossings' t within FLAG_COND_ULPS x the
// sum of their t conditioning (Hit::kt).  Two independent float evaluations of the same crossing (the GPU's and this
// one) differ by up to ~3 cond (measured, scripts/parity_outliers.py), and the ray direction itself by up to 3 ulps.
// (the default; oracle_params::flag_cond_ulps overrides it per call, 0 giving round 3's fixed margins)
constexpr float FLAG_COND_ULPS = 6.0f;
// margin columns stay comparable to the fixed epsilons: a distance r against an uncertainty max(eps, u) is stored as
// r * eps / max(eps, u), so "r < max(eps, u)" reads "stored < eps" (oracle.ambiguous is unchanged)
inline float normMargin(float r, float eps, float unc) { return r * eps / std::max(eps, unc); }

// ---------------------------------------------------------------- CPU BVH over proxies
struct BNode {
    float lo[3], hi[3];
    uint32_t left;   // internal: index of left child (right = left+1); leaf: first item
    uint32_t count;  // 0 = internal
};

struct Bvh {
    std::vector<BNode> nodes;
    std::vector<uint32_t> items;
};

void buildBvh(const std::vector<float>& boxes /*6 per item*/, uint32_t n, Bvh& b) {
    b.items.resize(n);
    for (uint32_t i = 0; i < n; ++i) b.items[i] = i;
    b.nodes.clear();
    b.nodes.reserve(2 * n + 1);
    struct Task {
        uint32_t node, begin, end;
    };
    std::vector<Task> stack;
    b.nodes.push_back(BNode{});
    stack.push_back({0, 0, n});
    std::vector<float> cen(3ull * n);
    for (uint32_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) cen[3ull * i + k] = 0.5f * (boxes[6ull * i + k] + boxes[6ull * i + 3 + k]);
    while (!stack.empty()) {
        Task t = stack.back();
        stack.pop_back();
        BNode nd;
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = INFINITY;
            nd.hi[k] = -INFINITY;
        }
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i = t.begin; i < t.end; ++i) {
            const uint32_t it = b.items[i];
            for (int k = 0; k < 3; ++k) {
                nd.lo[k] = std::min(nd.lo[k], boxes[6ull * it + k]);
                nd.hi[k] = std::max(nd.hi[k], boxes[6ull * it + 3 + k]);
                clo[k] = std::min(clo[k], cen[3ull * it + k]);
                chi[k] = std::max(chi[k], cen[3ull * it + k]);
            }
        }
        const uint32_t cnt = t.end - t.begin;
        if (cnt <= 4) {
            nd.left = t.begin;
            nd.count = cnt;
            b.nodes[t.node] = nd;
            continue;
        }
        // Split: binned surface-area heuristic (16 centroid bins per axis), falling back to the centroid median of
        // the longest axis when no bin boundary separates the items.  A median split alone made the oracle ~50x
        // slower per ray on a scene with heavy-tailed sizes (scene.trained_standin): large and small proxies mixed in
        // every subtree.  Culling only: any tree finds the same crossings (ties aside, which the margins flag).
        int axis = 0;
        float ext = chi[0] - clo[0];
        for (int k = 1; k < 3; ++k)
            if (chi[k] - clo[k] > ext) {
                ext = chi[k] - clo[k];
                axis = k;
            }
        constexpr int NBIN = 16;
        auto area = [](const float* lo, const float* hi) {
            if (!(hi[0] >= lo[0])) return 0.0f;
            const float ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
            return ex * ey + ey * ez + ez * ex;
        };
        int best_axis = -1, best_k = 0;
        float best_cost = INFINITY;
        for (int a = 0; a < 3; ++a) {
            const float ea = chi[a] - clo[a];
            if (!(ea > 0.0f) || !(NBIN / ea < INFINITY)) continue;
            const float sc = NBIN / ea;
            float blo[NBIN][3], bhi[NBIN][3];
            uint32_t bn[NBIN] = {};
            for (int q = 0; q < NBIN; ++q)
                for (int k = 0; k < 3; ++k) blo[q][k] = INFINITY, bhi[q][k] = -INFINITY;
            for (uint32_t i = t.begin; i < t.end; ++i) {
                const uint32_t it = b.items[i];
                const int q = std::min(NBIN - 1, (int)((cen[3ull * it + a] - clo[a]) * sc));
                ++bn[q];
                for (int k = 0; k < 3; ++k) {
                    blo[q][k] = std::min(blo[q][k], boxes[6ull * it + k]);
                    bhi[q][k] = std::max(bhi[q][k], boxes[6ull * it + 3 + k]);
                }
            }
            float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            float rarea[NBIN];
            uint32_t rcnt[NBIN], n = 0;
            for (int q = NBIN - 1; q > 0; --q) {
                for (int k = 0; k < 3; ++k) rlo[k] = std::min(rlo[k], blo[q][k]), rhi[k] = std::max(rhi[k], bhi[q][k]);
                n += bn[q];
                rarea[q] = area(rlo, rhi);
                rcnt[q] = n;
            }
            float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            n = 0;
            for (int q = 0; q < NBIN - 1; ++q) {
                for (int k = 0; k < 3; ++k) llo[k] = std::min(llo[k], blo[q][k]), lhi[k] = std::max(lhi[k], bhi[q][k]);
                n += bn[q];
                if (n == 0 || rcnt[q + 1] == 0) continue;
                const float cost = area(llo, lhi) * (float)n + rarea[q + 1] * (float)rcnt[q + 1];
                if (cost < best_cost) best_cost = cost, best_axis = a, best_k = q;
            }
        }
        uint32_t mid;
        if (best_axis >= 0) {
            const float sc = NBIN / (chi[best_axis] - clo[best_axis]);
            const float lo_a = clo[best_axis];
            mid = (uint32_t)(std::partition(b.items.begin() + t.begin, b.items.begin() + t.end,
                                            [&](uint32_t it) {
                                                return std::min(NBIN - 1, (int)((cen[3ull * it + best_axis] - lo_a) *
                                                                                sc)) <= best_k;
                                            }) -
                             b.items.begin());
        } else {
            mid = t.begin + cnt / 2;
            std::nth_element(b.items.begin() + t.begin, b.items.begin() + mid, b.items.begin() + t.end,
                             [&](uint32_t a, uint32_t c) {
                                 const float ca = cen[3ull * a + axis], cc = cen[3ull * c + axis];
                                 return ca < cc || (ca == cc && a < c);
                             });
        }
        nd.left = (uint32_t)b.nodes.size();
        nd.count = 0;
        b.nodes[t.node] = nd;
        b.nodes.push_back(BNode{});
        b.nodes.push_back(BNode{});
        stack.push_back({nd.left, t.begin, mid});
        stack.push_back({nd.left + 1, mid, t.end});
    }
}

// conservative slab test against [t0, t1]
inline bool boxHit(const BNode& n, V3 o, V3 inv, float t0, float t1, float* tenter = nullptr) {
    float tn = t0, tf = t1;
    for (int k = 0; k < 3; ++k) {
        const float ok = comp(o, k), ik = comp(inv, k);
        float a = (n.lo[k] - ok) * ik, b = (n.hi[k] - ok) * ik;
        if (std::isnan(a)) a = -INFINITY;
        if (std::isnan(b)) b = INFINITY;
        if (a > b) std::swap(a, b);
        // widen by a relative epsilon: this is culling only, it must never lose a crossing
        const float pad = 1e-5f * (std::fabs(a) + std::fabs(b)) + 1e-12f;
        tn = std::max(tn, a - pad);
        tf = std::min(tf, b + pad);
    }
    if (tenter) *tenter = tn;
    return tn <= tf;
}

// Watertight ray/triangle intersection (Woop, Benthin, Wald, JCGT 2013), no culling (Q1).
inline bool rayTri(V3 org, V3 dir, int kx, int ky, int kz, float Sx, float Sy, float Sz, V3 p0,
                   V3 p1, V3 p2, float& tOut) {
    const V3 A = p0 - org, B = p1 - org, C = p2 - org;
    const float Ax = comp(A, kx) - Sx * comp(A, kz), Ay = comp(A, ky) - Sy * comp(A, kz);
    const float Bx = comp(B, kx) - Sx * comp(B, kz), By = comp(B, ky) - Sy * comp(B, kz);
    const float Cx = comp(C, kx) - Sx * comp(C, kz), Cy = comp(C, ky) - Sy * comp(C, kz);
    float U = Cx * By - Cy * Bx, V = Ax * Cy - Ay * Cx, W = Bx * Ay - By * Ax;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        U = (float)((double)Cx * By - (double)Cy * Bx);
        V = (float)((double)Ax * Cy - (double)Ay * Cx);
        W = (float)((double)Bx * Ay - (double)By * Ax);
    }
    const float det = U + V + W;
    if (det == 0.0f) return false;
    // Shared-edge ownership: a ray exactly on an edge must hit one of the two triangles sharing it,
    // not both (watertight hardware semantics).  The sign given to a zero edge function is
    // antisymmetric in the edge direction, and a consistently wound mesh traverses a shared edge in
    // opposite directions, so exactly one triangle owns it.
    auto own = [](float e, float ex, float ey) -> float {
        if (e != 0.0f) return e;
        return (ey > 0.0f || (ey == 0.0f && ex > 0.0f)) ? 1.0f : -1.0f;
    };
    const float Us = own(U, Cx - Bx, Cy - By);  // edge B->C
    const float Vs = own(V, Ax - Cx, Ay - Cy);  // edge C->A
    const float Ws = own(W, Bx - Ax, By - Ay);  // edge A->B
    if ((Us < 0.0f || Vs < 0.0f || Ws < 0.0f) && (Us > 0.0f || Vs > 0.0f || Ws > 0.0f)) return false;
    const float Az = Sz * comp(A, kz), Bz = Sz * comp(B, kz), Cz = Sz * comp(C, kz);
    const float T = U * Az + V * Bz + W * Cz;
    tOut = T / det;
    return true;
}

// Analytic proxy: the icosahedron of particlePrimitives.comp:153-167 in the kernel frame
// x_k = (1/scl) * (R^T (x - p)) is the canonical icosahedron scaled by kS, whose 20 faces are
// 10 antipodal plane pairs n_j . x = +-sqrt(3) kS (n_j = dual dodecahedron directions).
const float IPHI = 0.618033988749895f;
const float PHI = 1.618033988749895f;
const V3 SLAB_N[10] = {{1, 1, 1},     {1, 1, -1},     {1, -1, 1},    {-1, 1, 1},  {0, PHI, IPHI},
                       {0, PHI, -IPHI}, {IPHI, 0, PHI}, {-IPHI, 0, PHI}, {PHI, IPHI, 0}, {PHI, -IPHI, 0}};
const float SQRT3 = 1.7320508075688772f;

// kin / kout (parity accounting): the relative t uncertainty per ulp of the entry / exit crossing.  With
// t = (+-h - n.ok) / (n.dk), one ulp of rounding in ok, dk or the ray moves t by ~ (|n||ok| + |t||n||dk|) 2^-24 /
// |n.dk|: about 2^-24 / cos(theta) relative, theta the angle between the ray and the face it crosses, which grows
// without bound for a face crossed at grazing incidence.
inline bool icosaCross(const Scene& s, uint32_t idx, V3 o, V3 d, float& tin, float& tout, float* kin = nullptr,
                       float* kout = nullptr) {
    const float* rec = s.density + 12ull * idx;
    const V3 pos = v3(rec[0], rec[1], rec[2]);
    const M3 R = quaternionWXYZToMatrix(rec + 4);
    const V3 giscl = v3(1 / rec[8], 1 / rec[9], 1 / rec[10]);
    uint64_t jh = jig_seed(idx);
    const V3 ok = jig3(giscl * mul(R, o - pos), jh);
    const V3 dk = jig3(giscl * mul(R, d), jh);
    const float h = s.kS[idx] * SQRT3;
    float tn = -INFINITY, tf = INFINITY;
    int jn = -1, jf = -1;
    for (int j = 0; j < 10; ++j) {
        const float a = dot(SLAB_N[j], ok), b = dot(SLAB_N[j], dk);
        const float ib = 1.0f / b;
        const float t1 = (-h - a) * ib, t2 = (h - a) * ib;
        const float lo = std::fmin(t1, t2), hi = std::fmax(t1, t2);
        if (lo > tn) jn = j;
        if (hi < tf) jf = j;
        tn = std::fmax(tn, lo);
        tf = std::fmin(tf, hi);
    }
    tin = tn;
    tout = tf;
    if (kin && kout) {
        const float okl = length(ok), dkl = length(dk);
        auto kap = [&](int j, float t) {
            if (j < 0) return 0.0f;
            const float nl = length(SLAB_N[j]), b = std::fabs(dot(SLAB_N[j], dk));
            if (!(b > 0.0f) || !(std::fabs(t) > 0.0f)) return 1.0f;
            return std::min(1.0f, nl * (okl + std::fabs(t) * dkl) / (b * std::fabs(t)) * ULP);
        };
        *kin = kap(jn, tn);
        *kout = kap(jf, tf);
    }
    return tn <= tf;
}

}  // namespace

// =============================================================================== C API
extern "C" {

typedef struct {
    float aabb[6];
    float min_transmittance;
    float hit_min_gaussian_response;
    uint32_t sph_eval_degree;
    float alpha_min;
    float pixel_offset;
    float alpha_init;
    uint32_t tmin_inclusive;
    uint32_t proxy_mode;     // 0 triangles, 1 analytic
    uint32_t drop_rejected;  // 0 literal, 1 accepted-only k-buffer
    uint32_t max_rounds;     // 0 = unlimited
    uint32_t ray_dirs_layout;  // 0 [cam][y][x], 1 light-field [cam][x][y]
    // enclosing params (analytic proxy size)
    float kernel_min_response;
    uint32_t kernel_opts;
    float kernel_degree;
    // parity accounting only (tests/test_oracle_kat.py): every ray's origin and direction components moved by a
    // pseudo-random whole number of ulps in [-perturb_ulps, perturb_ulps] (seeded by the ray index), the size of the
    // differences between two float evaluations of the ray (the GPU's ray generation differs by up to 3 ulps)
    uint32_t perturb_ulps;
    float flag_cond_ulps;  // conditioning factor of the margins (FLAG_COND_ULPS; 0: the fixed epsilons alone)
} oracle_params;

int oracle_version(void) { return 4; }

// the parity accounting's flag thresholds (oracle.py THR_EPS, PAIR_EPS, BOUND_EPS)
void oracle_value_eps(float* out1) { out1[0] = FLAG_VALUE_EPS; }

void oracle_flag_eps(float* out4) {
    out4[0] = FLAG_THR_EPS;
    out4[1] = FLAG_PAIR_EPS;
    out4[2] = FLAG_BOUND_EPS;
    out4[3] = FLAG_COND_ULPS;
}

// particlePrimitives.comp:112-215, with deterministic compaction (saveIdx = rank among
// survivors in input order; the reference's atomicAdd order is nondeterministic, Q3) and
// out-of-bounds specular reads (Q5) returning 0.0.
int oracle_enclose(const float* gPos, const float* gRot, const float* gScl, const float* gDns,
                   const float* featuresAlbedo, const float* featuresSpecular, uint32_t gNum,
                   float kernelMinResponse, uint32_t opts, float degree, float* gPrimVrt,
                   uint32_t* gPrimTri, float* writeParticleDensity,
                   float* writeParticleSphCoefficient, uint32_t* particleCounts,
                   uint32_t* srcIndex) {
    uint32_t counter = 0;
    const uint64_t specLen = (uint64_t)gNum * SPECULAR_DIMENSION;
    for (uint32_t globalIdx = 0; globalIdx < gNum; ++globalIdx) {
        const uint32_t sPosIdx = globalIdx * 3, sRotIdx = globalIdx * 4, sSclIdx = globalIdx * 3;
        const V3 albedo = v3(featuresAlbedo[globalIdx * 3], featuresAlbedo[globalIdx * 3 + 1],
                             featuresAlbedo[globalIdx * 3 + 2]);
        const float albedoStrength = length(albedo);
        float specularStrength = 0.0f, maxSpecular = 0.0f, minSpecular = 1e10f;
        for (uint32_t i = 1; i < SPECULAR_DIMENSION; i++) {
            float c3[3];
            for (int k = 0; k < 3; ++k) {
                const uint64_t off = (uint64_t)globalIdx * SPECULAR_DIMENSION + 3 * i + k;
                c3[k] = off < specLen ? featuresSpecular[off] : 0.0f;  // Q5
            }
            specularStrength += length(v3(c3[0], c3[1], c3[2]));
            maxSpecular = std::max(maxSpecular, specularStrength);
            minSpecular = std::min(minSpecular, specularStrength);
        }
        if (albedoStrength > 3.0f) continue;
        if (maxSpecular / (minSpecular + 1e-5f) > 150.0f) continue;

        const uint32_t saveIdx = counter++;
        if (srcIndex) srcIndex[saveIdx] = globalIdx;
        const uint32_t sVertIdx = 12 * saveIdx * 3;
        const uint32_t sTriIdx = 20 * saveIdx * 3;
        float q[4] = {gRot[sRotIdx], gRot[sRotIdx + 1], gRot[sRotIdx + 2], gRot[sRotIdx + 3]};
        const float qn = 1.0f / std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int k = 0; k < 4; ++k) q[k] *= qn;
        const M3 rot = quaternionWXYZToMatrixTranspose(q);
        const V3 scl = v3(std::exp(gScl[sSclIdx]), std::exp(gScl[sSclIdx + 1]), std::exp(gScl[sSclIdx + 2]));
        const V3 trans = v3(gPos[sPosIdx], gPos[sPosIdx + 1], gPos[sPosIdx + 2]);
        const float density = sigmoid(gDns[globalIdx]);
        const V3 kscl = kernelScale(density, kernelMinResponse, opts, degree) * scl * icosaVrtScale;
        if (gPrimVrt) {
            for (int i = 0; i < 12; ++i) {
                const V3 vert = mul(rot, icosaHedronVrt[i] * kscl) + trans;
                gPrimVrt[sVertIdx + i * 3] = vert.x;
                gPrimVrt[sVertIdx + i * 3 + 1] = vert.y;
                gPrimVrt[sVertIdx + i * 3 + 2] = vert.z;
            }
        }
        if (gPrimTri) {
            for (int i = 0; i < 20; ++i)
                for (int k = 0; k < 3; ++k) gPrimTri[sTriIdx + i * 3 + k] = icosaHedronTri[i][k] + 12 * saveIdx;
        }
        float* dr = writeParticleDensity + 12ull * saveIdx;
        dr[0] = gPos[globalIdx * 3];
        dr[1] = gPos[globalIdx * 3 + 1];
        dr[2] = gPos[globalIdx * 3 + 2];
        dr[3] = density;
        dr[4] = q[0];
        dr[5] = q[1];
        dr[6] = q[2];
        dr[7] = q[3];
        dr[8] = scl.x;
        dr[9] = scl.y;
        dr[10] = scl.z;
        dr[11] = 0.0f;
        float* sr = writeParticleSphCoefficient + 48ull * saveIdx;
        for (uint32_t i = 0; i < 3; i++) sr[i] = featuresAlbedo[globalIdx * 3 + i];
        for (uint32_t i = 0; i < SPECULAR_DIMENSION; i++)
            sr[3 + i] = featuresSpecular[(uint64_t)globalIdx * SPECULAR_DIMENSION + i];
    }
    *particleCounts = counter;
    return 0;
}

// Ray generation (particleRendering.comp:123-129 / raygen.rgen:116-121): column-major mats.
static void genRay(const float* viewInv, const float* projInv, uint32_t x, uint32_t y, uint32_t W,
                   uint32_t H, float off, V3& o, V3& d) {
    const float u = ((float)x + off) / (float)W;
    const float v = ((float)y + off) / (float)H;
    const float nx = u * 2.0f - 1.0f, ny = v * 2.0f - 1.0f;
    o = v3(viewInv[12], viewInv[13], viewInv[14]);
    float t[4];
    for (int r = 0; r < 4; ++r)
        t[r] = projInv[0 * 4 + r] * nx + projInv[1 * 4 + r] * ny + projInv[2 * 4 + r] * 1.0f +
               projInv[3 * 4 + r] * 1.0f;
    float w[3];
    for (int r = 0; r < 3; ++r)
        w[r] = viewInv[0 * 4 + r] * t[0] + viewInv[1 * 4 + r] * t[1] + viewInv[2 * 4 + r] * t[2];
    const float l = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    d = v3(w[0] / l, w[1] / l, w[2] / l);
}

struct Hit {
    uint32_t id;
    float t;
    float kt = 0.0f;   // parity accounting: relative change of t per ulp of rounding (icosaCross); 0 for triangles
    uint8_t face = 0;  // which crossing of the proxy: 0 entry, 1 exit (triangle soup: 0)
};

// debugging aid: when set (single-threaded trace of one ray), every processed crossing is appended as
// {id, t, gres, galpha, T after, accepted, round}
static thread_local std::vector<float>* g_trace = nullptr;

// ---- Alternative outcomes of flagged decisions (parity accounting only).  Every decision the margins
// flag can go the other way under another float evaluation of the ray (the GPU's).  The march records, for each
// flagged decision, the variants that other outcome can take (one decision may have several: a near-tied pair may
// swap or, tied bitwise at a round boundary of the other evaluation, lose either crossing to the exclusive tmin, Q13),
// each a change to one crossing or one particle:
//   VAR_ACCEPT  the particle's accept test (response vs hitMinGaussianResponse, alpha vs alphaMin) inverted, for every
//               crossing of it (gaussianfunctions.glsl:192-200; both faces share the response);
//   VAR_TERM    the transmittance test after crossing (id, face): mode 0 the ray stops there (T <= minTransmittance),
//               mode 1 it goes on until its next accepted crossing (particleRendering.comp:153-187);
//   VAR_SET_T   crossing (id, face) found at t instead (a near tie resolved the other way: it moves just past its
//               neighbour, or to `last`);
//   VAR_DROP    crossing (id, face) dropped (its t tied bitwise with `last` at a round boundary, Q13);
//   VAR_GRAZE   the proxy's crossing pair toggled (a grazing ray: crossed or not is a few-ulp decision).
// A re-march with a set of variants applied (Forced) gives that alternative's colour.
enum : uint8_t { VAR_ACCEPT = 1, VAR_TERM = 2, VAR_SET_T = 3, VAR_DROP = 4, VAR_GRAZE = 5 };
struct Variant {
    uint8_t kind, face, mode;
    uint32_t id;
    float t;
    uint32_t group;  // the flagged decision it belongs to (variants of one decision are exclusive)
};
struct Forced {
    const Variant* v = nullptr;
    int n = 0;
    bool accept_flip(uint32_t id) const {
        bool f = false;
        for (int i = 0; i < n; ++i) f ^= v[i].kind == VAR_ACCEPT && v[i].id == id;
        return f;
    }
    bool graze(uint32_t id) const {
        for (int i = 0; i < n; ++i)
            if (v[i].kind == VAR_GRAZE && v[i].id == id) return true;
        return false;
    }
    // the crossing's t in this alternative; false: dropped
    bool crossing(uint32_t id, uint8_t face, float& t) const {
        for (int i = 0; i < n; ++i) {
            if (v[i].id != id || v[i].face != face) continue;
            if (v[i].kind == VAR_DROP) return false;
            if (v[i].kind == VAR_SET_T) t = v[i].t;
        }
        return true;
    }
    int term(uint32_t id, uint8_t face) const {  // -1: none, else the mode
        for (int i = 0; i < n; ++i)
            if (v[i].kind == VAR_TERM && v[i].id == id && v[i].face == face) return v[i].mode;
        return -1;
    }
};

struct OracleScene {
    Scene s;
    Bvh bvh;
    uint32_t proxy_mode;
};

struct RayOut {
    float rgba[4];
    float depth;
    uint32_t stats[3];
    float margin[4];
    float vbound;  // the ray's value bound (FLAG_VALUE_EPS), with want_margin
};

}  // extern "C"

// The per-ray ray-march: particleRendering.comp:117-191 (RQ) / raygen.rgen:113-193 (RT).
// out.stats = {processed crossings (X_r), accepted (A_r), rounds}.
// out.margin (want_margin; parity accounting, not part of the reference algorithm): how
// close the ray came to a decision that a few-ulp different float evaluation (GPU exp / rsqrt / rcp,
// FMA contraction) could take the other way.  Columns 0-2 are normalised to their fixed epsilon: a distance r
// against the decision's uncertainty max(eps, flag_cond_ulps x its conditioning) is stored as r x eps /
// max(eps, uncertainty) (normMargin), so "stored < eps" means "within the uncertainty".
//   [0] relative distance to a threshold: |gres/hitMin - 1| and |galpha/alphaMin - 1| of every processed
//       crossing, |T/minTransmittance - 1| after every accepted one;
//   [1] relative t gap |t_i - t_j| / |t_i| between consecutive accepted crossings (their composite
//       order);
//   [2] relative t gap at a boundary: the first crossing of a round (if accepted) against the last one of
//       the round before, the last slot of a full buffer against the nearest crossing left out (one of the
//       two accepted), the crossing that ends the ray (T <= minTransmittance) against its successor (if that
//       one would be accepted), a ray grazing a proxy
//       whose crossings would be accepted (relative chord |tout - tin| / |t|), and 0 for a crossing
//       dropped because its t tied bitwise with `last` (the exclusive-tmin round boundary, Q13);
//   [3] flip bound: an upper bound on |d rgb| that the decisions flagged by [0..2] (below FLAG_*_EPS) can cause
//       if a different float evaluation takes them the other way.  Every flagged decision can at worst add or drop
//       one crossing j (a threshold flip; a pair within PAIR_EPS that ties bitwise and straddles a round boundary
//       of the other evaluation, where the exclusive tmin drops one of the two, Q13; a boundary tie), which moves
//       the colour by at most 2 T_j a_j c (its own term, and the rescaling of everything behind it) plus the
//       crossings a moved termination point adds or removes, at most minTransmittance / (1 - a_j) x c.  The bound is
//       the sum over the ray's flagged crossings (both of a flagged pair) of 2 T_j a_j, plus minTransmittance / (1 -
//       the largest such a_j), times c, the largest radiance channel of every crossing composited or flagged on the
//       ray.  0 for a ray with no flagged decision.
// F (alternatives): the flagged decisions' variants to apply; rec: where the flagged decisions' variants are recorded
// (with want_margin).
static void marchRay(const OracleScene& os, const oracle_params* P, V3 o, V3 d, bool want_margin, const Forced* F,
                     std::vector<Variant>* rec, RayOut& out) {
    const Scene& s = os.s;
    const Bvh& bvh = os.bvh;
    const float* verts = s.verts;
    const uint32_t* tris = s.tris;
    const float CU = P->flag_cond_ulps >= 0.0f ? P->flag_cond_ulps : FLAG_COND_ULPS;
    const V3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    RayState st;
    st.T = 1.0f;
    st.rad[0] = st.rad[1] = st.rad[2] = 0.0f;
    st.rad[3] = P->alpha_init;
    st.depth = 0.0f;
    uint32_t nproc = 0, nacc = 0, rounds = 0;
    float tminb, tmaxb;
    intersectAABB(P->aabb, o, d, tminb, tmaxb);
    float last = std::max(0.0f, tminb - EPS_T);
    Hit kb[MAX_HIT_PER_TRACE];
    float m_thr = INFINITY, m_t = INFINITY, m_b = INFINITY, prev_t = NAN, prev_acc_t = NAN;
    // t conditioning of the previous processed / accepted crossing, and the relative uncertainty of T (the summed
    // relative errors of its factors 1 - alpha_j: alpha_j / (1 - alpha_j) x FLAG_COND_ULPS x cond_j, plus one
    // rounding per factor)
    float prev_kt = 0.0f, prev_acc_kt = 0.0f, t_unc = 0.0f;
    // flip bound (margin[3]): summed T x alpha of the flagged decisions, the largest radiance channel
    // involved, and the previous accepted crossing's T before it and alpha (pair swaps)
    float fw = 0.0f, fc = 0.0f, famax = 0.0f, prev_acc_T = 0.0f, prev_acc_a = 0.0f;
    float vsum = 0.0f, vmax = 0.0f;  // sum and largest of 2 T_j a_j cond_j over accepted crossings (FLAG_VALUE_EPS)
    bool flagged = false;
    uint32_t prev_id_acc = INVALID_PARTICLE_ID;
    uint8_t prev_face = 0, prev_acc_face = 0;
    uint32_t group = 0;  // flagged decisions recorded so far (rec)
    // a crossing `id` that a flagged decision may add or drop, with T before it and its alpha
    auto flag = [&](float T, float alpha, uint32_t id) {
        flagged = true;
        fw += 2.0f * T * alpha;
        famax = std::max(famax, alpha);
        if (id != INVALID_PARTICLE_ID) fc = std::max(fc, radianceMax(s, id, d, P->sph_eval_degree));
    };
    // the variants of one flagged decision (rec)
    auto record = [&](std::initializer_list<Variant> vs) {
        if (!rec) return;
        for (Variant v : vs) {
            v.group = group;
            rec->push_back(v);
        }
        ++group;
    };
    // the alternative's accept test of particle id
    auto acceptOf = [&](uint32_t id, bool a) { return F && F->accept_flip(id) ? !a : a; };
    // the ray is composited on while T > minTransmittance; an alternative may stop it after a crossing, or carry it
    // past one up to its next accepted crossing
    bool forced_stop = false, forced_go = false;
    auto alive = [&]() { return !forced_stop && (forced_go || st.T > P->min_transmittance); };
    bool round_start = false;
    uint32_t prev_id = INVALID_PARTICLE_ID;
    std::vector<uint32_t> last_ids;  // ids processed with t == last (tie detection, margin)
    std::vector<uint8_t> last_faces;  // and which crossing of each
    std::vector<uint32_t> stack;
    stack.reserve(128);
    while (last <= tmaxb && alive()) {
        if (P->max_rounds && rounds >= P->max_rounds) break;
        ++rounds;
        const float tmin = last + EPS_T, tmax = tmaxb + EPS_T;
        const float T_round = st.T;
        for (uint32_t i = 0; i < MAX_HIT_PER_TRACE; ++i) kb[i] = Hit{INVALID_PARTICLE_ID, INFINITE_DISTANCE};
        Hit h_out{INVALID_PARTICLE_ID, INFINITE_DISTANCE};  // nearest crossing left out of a full buffer
        // ---- trace(): driver traversal + any-hit (anyhit.rahit:40-71)
        auto anyhit = [&](uint32_t pid, float t, float kt, uint8_t face) {
            if (F && !F->crossing(pid, face, t)) return;
            const bool inRange = (P->tmin_inclusive ? t >= tmin : t > tmin) && t <= tmax;
            if (!inRange) {
                if (want_margin && t == last && t <= tmax &&
                    std::find(last_ids.begin(), last_ids.end(), pid) == last_ids.end()) {
                    m_b = 0.0f;  // dropped only because its t ties with the last processed crossing
                    const HitEval he = evalResponse(s, pid, o, d);
                    if (he.gres > P->hit_min_gaussian_response && he.galpha > P->alpha_min) {
                        flag(T_round, he.galpha, pid);
                        // the other evaluation finds it just past `last`, or took it in the previous round in place
                        // of the crossing that set `last` (tied: arrival order), which is then the one dropped
                        if (!last_ids.empty())
                            record({Variant{VAR_SET_T, face, 0, pid, std::nextafter(last, INFINITY), 0},
                                    Variant{VAR_SET_T, face, 0, pid, std::nextafter(last, -INFINITY), 0},
                                    Variant{VAR_DROP, last_faces.back(), 0, last_ids.back(), 0.0f, 0}});
                        else
                            record({Variant{VAR_SET_T, face, 0, pid, std::nextafter(last, INFINITY), 0}});
                    }
                }
                return;
            }
            if (P->drop_rejected) {
                const HitEval he = evalResponse(s, pid, o, d);
                if (!acceptOf(pid, he.gres > P->hit_min_gaussian_response && he.galpha > P->alpha_min)) return;
            }
            Hit hit{pid, t, kt, face};
            if (hit.t < kb[MAX_HIT_PER_TRACE - 1].t) {
                for (uint32_t i = 0; i < MAX_HIT_PER_TRACE; ++i) {  // compareAndSwapHitPayloadValue
                    if (hit.t < kb[i].t) std::swap(hit, kb[i]);
                }
            }
            // margin: the nearest crossing left out of (or pushed out of) the full buffer
            if (hit.id != INVALID_PARTICLE_ID && hit.t < h_out.t) h_out = hit;
        };
        stack.clear();
        stack.push_back(0);
        while (!stack.empty()) {
            const uint32_t ni = stack.back();
            stack.pop_back();
            const BNode& nd = bvh.nodes[ni];
            const float tcull = kb[MAX_HIT_PER_TRACE - 1].t < INFINITE_DISTANCE
                                    ? std::min(tmax, kb[MAX_HIT_PER_TRACE - 1].t)
                                    : tmax;
            if (!boxHit(nd, o, inv, tmin, tcull)) continue;
            if (nd.count == 0) {
                // front-to-back: pop the nearer child first (culling only; results unchanged)
                float e0 = INFINITY, e1 = INFINITY;
                const bool h0 = boxHit(bvh.nodes[nd.left], o, inv, tmin, tcull, &e0);
                const bool h1 = boxHit(bvh.nodes[nd.left + 1], o, inv, tmin, tcull, &e1);
                if (h0 && h1) {
                    stack.push_back(e0 <= e1 ? nd.left + 1 : nd.left);
                    stack.push_back(e0 <= e1 ? nd.left : nd.left + 1);
                } else if (h0) {
                    stack.push_back(nd.left);
                } else if (h1) {
                    stack.push_back(nd.left + 1);
                }
                continue;
            }
            for (uint32_t k = 0; k < nd.count; ++k) {
                const uint32_t g = bvh.items[nd.left + k];
                if (P->proxy_mode == 1) {
                    float tin, tout, kin = 0.0f, kout = 0.0f;
                    bool crossed = icosaCross(s, g, o, d, tin, tout, &kin, &kout);
                    const float geps = std::max(FLAG_BOUND_EPS, CU * (kin + kout));
                    if (want_margin && std::fabs(tout - tin) < geps * std::max(std::fabs(tin), std::fabs(tout))) {
                        // grazing the proxy: whether it is crossed at all is a few-ulp decision; it
                        // matters when its crossings would be composited
                        const HitEval he = evalResponse(s, g, o, d);
                        if (he.gres > P->hit_min_gaussian_response && he.galpha > P->alpha_min) {
                            const float gg = std::fabs(tout - tin) / std::max(std::fabs(tin), 1e-30f);
                            m_b = std::min(m_b, normMargin(gg, FLAG_BOUND_EPS, geps));
                            if (gg < geps) {  // both crossings of the proxy
                                flag(T_round, he.galpha, g);
                                flag(T_round, he.galpha, g);
                                record({Variant{VAR_GRAZE, 0, 0, g, 0.0f, 0}});
                            }
                        }
                    }
                    if (F && F->graze(g)) {  // the other evaluation crosses it, or misses it
                        if (crossed) {
                            crossed = false;
                        } else if (std::fabs(tout - tin) < geps * std::max(std::fabs(tin), std::fabs(tout))) {
                            crossed = true;
                            const float a = std::min(tin, tout), b = std::max(tin, tout);
                            tin = a;
                            tout = b;
                        }
                    }
                    if (crossed) {
                        anyhit(g, tin, kin, 0);
                        anyhit(g, tout, kout, 1);
                    }
                } else {
                    // watertight setup
                    int kz = 0;
                    float ax = std::fabs(d.x), ay = std::fabs(d.y), az = std::fabs(d.z);
                    if (ay > ax && ay >= az) kz = 1;
                    else if (az > ax && az > ay) kz = 2;
                    int kx = (kz + 1) % 3, ky = (kx + 1) % 3;
                    if (comp(d, kz) < 0.0f) std::swap(kx, ky);
                    const float Sx = comp(d, kx) / comp(d, kz), Sy = comp(d, ky) / comp(d, kz),
                                Sz = 1.0f / comp(d, kz);
                    for (uint32_t t = 0; t < 20; ++t) {
                        const uint32_t* tr = tris + 60ull * g + 3 * t;
                        const V3 p0 = v3(verts[3ull * tr[0]], verts[3ull * tr[0] + 1], verts[3ull * tr[0] + 2]);
                        const V3 p1 = v3(verts[3ull * tr[1]], verts[3ull * tr[1] + 1], verts[3ull * tr[1] + 2]);
                        const V3 p2 = v3(verts[3ull * tr[2]], verts[3ull * tr[2] + 1], verts[3ull * tr[2] + 2]);
                        float th;
                        if (rayTri(o, d, kx, ky, kz, Sx, Sy, Sz, p0, p1, p2, th))
                            anyhit((20 * g + t) / 20, th, 0.0f, 0);  // Q2: particle id = primitive / 20
                    }
                }
            }
        }
        if (kb[0].id == INVALID_PARTICLE_ID) break;
        auto gap = [](float a, float b) { return std::fabs(a - b) / std::max(std::fabs(a), 1e-30f); };
        // margin: a crossing tied with the buffer's last slot may or may not make this round,
        // depending on arrival order
        auto accepted = [&](uint32_t id) {
            const HitEval he = evalResponse(s, id, o, d);
            return he.gres > P->hit_min_gaussian_response && he.galpha > P->alpha_min;
        };
        // (which of two tied crossings makes the round changes the image only if one of them is accepted)
        // (the uncertainty of a gap between two crossings: the larger of the fixed epsilon and their summed
        // t conditioning)
        auto teps = [CU](float eps, const Hit& a, const Hit& b) { return std::max(eps, CU * (a.kt + b.kt)); };
        const Hit& k15 = kb[MAX_HIT_PER_TRACE - 1];
        if (want_margin && k15.id != INVALID_PARTICLE_ID && h_out.id != INVALID_PARTICLE_ID &&
            gap(k15.t, h_out.t) < teps(FLAG_BOUND_EPS, k15, h_out) && (accepted(k15.id) || accepted(h_out.id))) {
            const float gg = gap(k15.t, h_out.t);
            const float ge = teps(FLAG_BOUND_EPS, k15, h_out);
            m_b = std::min(m_b, normMargin(gg, FLAG_BOUND_EPS, ge));
            if (gg < ge) {
                flag(T_round, evalResponse(s, k15.id, o, d).galpha, k15.id);
                flag(T_round, evalResponse(s, h_out.id, o, d).galpha, h_out.id);
                // the other evaluation takes the crossing left out into this round instead; tied, the one that
                // arrives second is found again at `last` in the next round and dropped (exclusive tmin, Q13)
                record({Variant{VAR_SET_T, h_out.face, 0, h_out.id, std::nextafter(k15.t, -INFINITY), 0},
                        Variant{VAR_DROP, k15.face, 0, k15.id, 0.0f, 0},
                        Variant{VAR_DROP, h_out.face, 0, h_out.id, 0.0f, 0}});
            }
        }
        round_start = true;
        // ---- process k hits
        for (uint32_t i = 0; i < MAX_HIT_PER_TRACE; ++i) {
            const Hit h = kb[i];
            if (h.id != INVALID_PARTICLE_ID && alive()) {
                HitEval ev{0.0f, 0.0f};
                const float T_before = st.T;
                const bool acc = processHit(s, o, d, h.id, P->hit_min_gaussian_response, P->alpha_min,
                                            P->sph_eval_degree, st, &ev, want_margin ? &fc : nullptr,
                                            F && F->accept_flip(h.id));
                if (acc && forced_go) forced_go = false;  // carried past the stop to this crossing: it is the last
                if (acc && F) {
                    const int tm = F->term(h.id, h.face);
                    if (tm == 0) forced_stop = true;
                    if (tm == 1 && !(st.T > P->min_transmittance)) forced_go = true;
                }
                if (g_trace)
                    g_trace->insert(g_trace->end(), {(float)h.id, h.t, ev.gres, ev.galpha, st.T, acc ? 1.0f : 0.0f,
                                                     (float)rounds});
                if (want_margin) {
                    const float r0 = std::fabs(ev.gres / P->hit_min_gaussian_response - 1.0f);
                    const float r1 = std::fabs(ev.galpha / P->alpha_min - 1.0f);
                    // both thresholds see gres's relative error (galpha = gres x density below the 0.99 clamp)
                    const float re = std::max(FLAG_THR_EPS, CU * ev.cond);
                    m_thr = std::min(m_thr, normMargin(std::min(r0, r1), FLAG_THR_EPS, re));
                    if (r0 < re || r1 < re) {
                        flag(T_before, ev.galpha, h.id);
                        record({Variant{VAR_ACCEPT, 0, 0, h.id, 0.0f, 0}});
                    }
                    if (acc) {
                        if (ev.galpha < 0.99f) {
                            t_unc += ev.galpha / (1.0f - ev.galpha) * CU * ev.cond + (CU > 0.0f ? 2.0f * ULP : 0.0f);
                            const float vj = 2.0f * T_before * ev.galpha * ev.vcond;
                            vsum += vj;
                            vmax = std::max(vmax, vj);
                        }
                        const float r2 = std::fabs(st.T / P->min_transmittance - 1.0f);
                        const float te = std::max(FLAG_THR_EPS, t_unc);
                        m_thr = std::min(m_thr, normMargin(r2, FLAG_THR_EPS, te));
                        if (r2 < te) {  // the ray may go on (or stop before this crossing)
                            const Hit nx = i + 1 < MAX_HIT_PER_TRACE ? kb[i + 1] : h_out;
                            flag(T_before, ev.galpha, h.id);
                            flag(st.T, 1.0f, nx.id);
                            record({Variant{VAR_TERM, h.face, (uint8_t)(st.T > P->min_transmittance ? 0 : 1), h.id,
                                            0.0f, 0}});
                        }
                    }
                    // (an inclusive tmin re-finds the same crossing: not an ordering question)
                    const bool refound = h.id == prev_id && h.t == prev_t;
                    if (acc && round_start && prev_t == prev_t && !refound) {
                        const float gg = gap(h.t, prev_t);
                        const float ge = std::max(FLAG_BOUND_EPS, CU * (h.kt + prev_kt));
                        m_b = std::min(m_b, normMargin(gg, FLAG_BOUND_EPS, ge));
                        if (gg < ge) {
                            flag(T_before, ev.galpha, h.id);
                            // tied with `last` in the other evaluation: one of the two lost to the exclusive tmin
                            record({Variant{VAR_DROP, h.face, 0, h.id, 0.0f, 0},
                                    Variant{VAR_DROP, prev_face, 0, prev_id, 0.0f, 0}});
                        }
                    }
                    if (acc && prev_acc_t == prev_acc_t && !refound) {
                        const float gg = gap(h.t, prev_acc_t);
                        const float ge = std::max(FLAG_PAIR_EPS, CU * (h.kt + prev_acc_kt));
                        m_t = std::min(m_t, normMargin(gg, FLAG_PAIR_EPS, ge));
                        if (gg < ge) {  // may swap, or tie and lose one at a round boundary
                            flag(prev_acc_T, prev_acc_a, prev_id_acc);
                            flag(T_before, ev.galpha, h.id);
                            record({Variant{VAR_SET_T, h.face, 0, h.id, std::nextafter(prev_acc_t, -INFINITY), 0},
                                    Variant{VAR_DROP, h.face, 0, h.id, 0.0f, 0},
                                    Variant{VAR_DROP, prev_acc_face, 0, prev_id_acc, 0.0f, 0}});
                        }
                    }
                    round_start = false;
                    prev_t = h.t;
                    prev_kt = h.kt;
                    prev_id = h.id;
                    prev_face = h.face;
                    if (acc) {
                        prev_acc_t = h.t;
                        prev_acc_kt = h.kt;
                        prev_acc_T = T_before;
                        prev_acc_a = ev.galpha;
                        prev_id_acc = h.id;
                        prev_acc_face = h.face;
                    }
                    if (h.t > last) last_ids.clear(), last_faces.clear();
                    if (h.t >= last) last_ids.push_back(h.id), last_faces.push_back(h.face);
                    // the crossing that ends the ray against its successor: a tie decides which of
                    // the two is composited
                    // (only an accepted successor changes the image by coming first)
                    if (acc && !(st.T > P->min_transmittance)) {
                        const Hit nx = i + 1 < MAX_HIT_PER_TRACE && kb[i + 1].id != INVALID_PARTICLE_ID ? kb[i + 1]
                                                                                                      : h_out;
                        if (nx.id != INVALID_PARTICLE_ID && gap(h.t, nx.t) < teps(FLAG_BOUND_EPS, h, nx) &&
                            accepted(nx.id)) {
                            const float gg = gap(h.t, nx.t);
                            const float ge = teps(FLAG_BOUND_EPS, h, nx);
                            m_b = std::min(m_b, normMargin(gg, FLAG_BOUND_EPS, ge));
                            if (gg < ge) {
                                flag(T_before, ev.galpha, h.id);
                                flag(T_before, evalResponse(s, nx.id, o, d).galpha, nx.id);
                                // the successor comes first; or, tied bitwise with it, the successor takes the last
                                // slot of a full buffer of the other evaluation (FAST: 32 accepted), the round ends
                                // there and this crossing is lost to the exclusive tmin (Q13)
                                record({Variant{VAR_SET_T, nx.face, 0, nx.id, std::nextafter(h.t, -INFINITY), 0},
                                        Variant{VAR_DROP, h.face, 0, h.id, 0.0f, 0}});
                            }
                        }
                    }
                }
                last = std::max(last, h.t);
                ++nproc;
                nacc += acc ? 1 : 0;
            }
        }
    }
    for (int k = 0; k < 4; ++k) out.rgba[k] = st.rad[k];
    out.depth = st.depth;
    out.stats[0] = nproc;
    out.stats[1] = nacc;
    out.stats[2] = rounds;
    const float vb = FLAG_VALUE_ULPS * vsum * fc;
    const bool vflag = want_margin && vmax * fc > FLAG_VALUE_EPS;
    out.vbound = vb;
    out.margin[0] = vflag ? 0.0f : m_thr;  // an ill-conditioned value: flagged like a decision on its threshold
    out.margin[1] = m_t;
    out.margin[2] = m_b;
    out.margin[3] = (flagged ? (fw + P->min_transmittance / std::max(1.0f - famax, 0.01f)) * fc : 0.0f) +
                    (flagged || vflag ? vb : 0.0f);
}

// ray r of a launch: its origin and direction (with the parity accounting's perturbation, if any)
static void rayOf(const oracle_params* P, const float* viewInverse, const float* projInverse, uint32_t W, uint32_t H,
                  uint64_t r, V3& o, V3& d, uint32_t* cam_out = nullptr, uint32_t* px_out = nullptr,
                  uint32_t* py_out = nullptr) {
    const uint32_t cam = (uint32_t)(r / ((uint64_t)W * H));
    const uint32_t rem = (uint32_t)(r % ((uint64_t)W * H));
    const uint32_t py = rem / W, px = rem % W;
    genRay(viewInverse + 16ull * cam, projInverse, px, py, W, H, P->pixel_offset, o, d);
    g_jig_ulps = P->perturb_ulps;
    g_jig_ray = r;
    if (g_jig_ulps) {
        uint64_t hh = mix64(r + 0x1234567ull);
        d = jig3(d, hh);
    }
    if (cam_out) *cam_out = cam;
    if (px_out) *px_out = px;
    if (py_out) *py_out = py;
}

extern "C" {

// Acceleration structure of the oracle (the driver BLAS/TLAS build is not restated; any
// correct BVH yields the same k-nearest sets).  Input arrays must outlive the scene.
void* oracle_scene_create(const float* verts, const uint32_t* tris, const float* density, const float* sh,
                          uint32_t M, uint32_t proxy_mode, float kernel_min_response, uint32_t kernel_opts,
                          float kernel_degree) {
    if (!density || !sh) return nullptr;
    if (proxy_mode == 0 && (!verts || !tris)) return nullptr;
    OracleScene* os = new OracleScene{Scene{verts, tris, density, sh, M, {}}, Bvh{}, proxy_mode};
    Scene& s = os->s;
    oracle_params kp{};
    kp.kernel_min_response = kernel_min_response;
    kp.kernel_opts = kernel_opts;
    kp.kernel_degree = kernel_degree;
    kp.proxy_mode = proxy_mode;
    const oracle_params* P = &kp;
    // proxy boxes
    std::vector<float> boxes(6ull * M);
    if (P->proxy_mode == 1) {
        s.kS.resize(M);
        for (uint32_t i = 0; i < M; ++i) {
            const float* rec = density + 12ull * i;
            s.kS[i] = kernelScale(rec[3], P->kernel_min_response, P->kernel_opts, P->kernel_degree);
            // world AABB of the canonical icosahedron (circumradius 1.2584 * kS in kernel frame):
            // |R * diag(scl) * x|_k <= sum_j |R_kj| scl_j * rc
            float qn[4] = {rec[4], rec[5], rec[6], rec[7]};
            const M3 Rw = quaternionWXYZToMatrixTranspose(qn);
            const float rc = s.kS[i] * icosaVrtScale * std::sqrt(1.0f + goldenRatio * goldenRatio) * 1.0001f;
            for (int k = 0; k < 3; ++k) {
                const float e = (std::fabs(comp(Rw.c[0], k)) * rec[8] + std::fabs(comp(Rw.c[1], k)) * rec[9] +
                                 std::fabs(comp(Rw.c[2], k)) * rec[10]) * rc;
                boxes[6ull * i + k] = rec[k] - e;
                boxes[6ull * i + 3 + k] = rec[k] + e;
            }
        }
    } else {
        for (uint32_t i = 0; i < M; ++i) {
            float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int t = 0; t < 20; ++t)
                for (int c = 0; c < 3; ++c) {
                    const uint32_t vi = tris[60ull * i + 3 * t + c];
                    for (int k = 0; k < 3; ++k) {
                        lo[k] = std::min(lo[k], verts[3ull * vi + k]);
                        hi[k] = std::max(hi[k], verts[3ull * vi + k]);
                    }
                }
            for (int k = 0; k < 3; ++k) {
                boxes[6ull * i + k] = lo[k];
                boxes[6ull * i + 3 + k] = hi[k];
            }
        }
    }
    buildBvh(boxes, M, os->bvh);
    return os;
}

void oracle_scene_destroy(void* h) { delete static_cast<OracleScene*>(h); }

int oracle_scene_render(void* h, const oracle_params* P, const float* viewInverse, const float* projInverse,
                        uint32_t W, uint32_t H, uint32_t ncams, const uint64_t* subset, uint64_t nsubset,
                        float* out_rgba, float* out_depth, float* out_ray_dirs, uint32_t* out_stats,
                        float* out_margin, int nthreads) {
    OracleScene* os = static_cast<OracleScene*>(h);
    if (!os || !P || !viewInverse || !projInverse || !out_rgba) return -1;
    if (P->proxy_mode != os->proxy_mode) return -2;
    const uint64_t nrays_full = (uint64_t)W * H * ncams;
    const uint64_t nwork = subset ? nsubset : nrays_full;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64)
#endif
    for (int64_t w = 0; w < (int64_t)nwork; ++w) {
        const uint64_t r = subset ? subset[w] : (uint64_t)w;
        V3 o, d;
        uint32_t cam, px, py;
        rayOf(P, viewInverse, projInverse, W, H, r, o, d, &cam, &px, &py);
        if (out_ray_dirs) {
            uint64_t di = P->ray_dirs_layout == 1 ? ((uint64_t)cam * W * H + (uint64_t)px * H + py) : r;
            if (subset) di = w;
            out_ray_dirs[4 * di] = d.x;
            out_ray_dirs[4 * di + 1] = d.y;
            out_ray_dirs[4 * di + 2] = d.z;
            out_ray_dirs[4 * di + 3] = 0.0f;
        }
        RayOut ro;
        marchRay(*os, P, o, d, out_margin != nullptr, nullptr, nullptr, ro);
        const uint64_t oi = subset ? (uint64_t)w : r;
        for (int k = 0; k < 4; ++k) out_rgba[4 * oi + k] = ro.rgba[k];
        if (out_depth) out_depth[oi] = ro.depth;
        if (out_stats)
            for (int k = 0; k < 3; ++k) out_stats[3 * oi + k] = ro.stats[k];
        if (out_margin)
            for (int k = 0; k < 4; ++k) out_margin[4 * oi + k] = ro.margin[k];
    }
    return 0;
}

// Explaining a ray's flagged decisions (parity accounting): the ray re-marched with its flagged
// decisions taken the other way.  For each ray rays[k] the march records every flagged decision's variants
// (Variant); the alternatives are the base march, each single variant, then each pair of variants of two different
// decisions (at most max_pairs pairs), tried in that order until one lies within tol of target[3k .. 3k+2] (max
// |d rgb|, less the alternative's own value bound, FLAG_VALUE_EPS).  out[5k ..]: {the distance of the best
// alternative, its kind (0 base, 1 single, 2 pair), the number of variants, the number of decisions, its value
// bound}.  alt_rgba (optional, 4 floats per ray): that alternative's colour.
int oracle_scene_explain(void* h, const oracle_params* P, const float* viewInverse, const float* projInverse,
                         uint32_t W, uint32_t H, uint32_t ncams, const uint64_t* rays, uint64_t n, const float* target,
                         float tol, uint32_t max_pairs, float* out, float* alt_rgba, int nthreads) {
    OracleScene* os = static_cast<OracleScene*>(h);
    if (!os || !P || !viewInverse || !projInverse || !rays || !target || !out) return -1;
    if (P->proxy_mode != os->proxy_mode) return -2;
    (void)ncams;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t k = 0; k < (int64_t)n; ++k) {
        V3 o, d;
        rayOf(P, viewInverse, projInverse, W, H, rays[k], o, d);
        std::vector<Variant> vars;
        RayOut base;
        marchRay(*os, P, o, d, true, nullptr, &vars, base);
        const float* tg = target + 3 * k;
        // an alternative explains the target exactly when it lies within tol; failing that, within tol plus the
        // alternative's own value bound (the colour its ill-conditioned responses may move, FLAG_VALUE_EPS).  The search
        // runs until an exact alternative is found (single variants, then pairs) and reports it; otherwise the one
        // whose excess over its value bound is smallest
        auto dist = [&](const RayOut& ro) {
            float m = 0.0f;
            for (int c = 0; c < 3; ++c) m = std::max(m, std::fabs(ro.rgba[c] - tg[c]));
            return m;
        };
        float best_exact = dist(base), best_rel = dist(base) - base.vbound;
        int kind_exact = 0, kind_rel = 0;
        RayOut exact_out = base, rel_out = base;
        uint32_t ngroups = vars.empty() ? 0u : vars.back().group + 1u;
        auto consider = [&](const Variant* v, int nv, int knd) {
            Forced F;
            F.v = v;
            F.n = nv;
            RayOut ro;
            marchRay(*os, P, o, d, true, &F, nullptr, ro);
            const float dd = dist(ro);
            if (dd < best_exact) {
                best_exact = dd;
                kind_exact = knd;
                exact_out = ro;
            }
            if (dd - ro.vbound < best_rel) {
                best_rel = dd - ro.vbound;
                kind_rel = knd;
                rel_out = ro;
            }
        };
        for (size_t i = 0; i < vars.size() && best_exact > tol; ++i) consider(&vars[i], 1, 1);
        uint32_t pairs = 0;
        for (size_t i = 0; i < vars.size() && best_exact > tol && pairs < max_pairs; ++i)
            for (size_t j = i + 1; j < vars.size() && best_exact > tol && pairs < max_pairs; ++j) {
                if (vars[i].group == vars[j].group) continue;
                const Variant two[2] = {vars[i], vars[j]};
                consider(two, 2, 2);
                ++pairs;
            }
        const bool exact = best_exact <= tol;
        const RayOut& best_out = exact ? exact_out : rel_out;
        const int kind = exact ? kind_exact : kind_rel;
        out[5 * k] = dist(best_out);
        out[5 * k + 1] = (float)kind;
        out[5 * k + 2] = (float)vars.size();
        out[5 * k + 3] = (float)ngroups;
        out[5 * k + 4] = best_out.vbound;
        if (alt_rgba)
            for (int c = 0; c < 4; ++c) alt_rgba[4 * k + c] = best_out.rgba[c];
    }
    return 0;
}

int oracle_render(const float* verts, const uint32_t* tris, const float* density, const float* sh,
                  uint32_t M, const oracle_params* P, const float* viewInverse,
                  const float* projInverse, uint32_t W, uint32_t H, uint32_t ncams,
                  const uint64_t* subset, uint64_t nsubset, float* out_rgba, float* out_depth,
                  float* out_ray_dirs, uint32_t* out_stats, float* out_margin, int nthreads) {
    if (!P) return -1;
    void* h = oracle_scene_create(verts, tris, density, sh, M, P->proxy_mode, P->kernel_min_response,
                                  P->kernel_opts, P->kernel_degree);
    if (!h) return -1;
    const int rc = oracle_scene_render(h, P, viewInverse, projInverse, W, H, ncams, subset, nsubset, out_rgba,
                                       out_depth, out_ray_dirs, out_stats, out_margin, nthreads);
    oracle_scene_destroy(h);
    return rc;
}

// Processed-crossing trace of one ray (debugging): 7 floats per crossing (see g_trace); returns the count.
int oracle_scene_trace(void* h, const oracle_params* P, const float* viewInverse, const float* projInverse,
                       uint32_t W, uint32_t H, uint32_t ncams, uint64_t ray, float* out, int maxn) {
    std::vector<float> tr;
    g_trace = &tr;
    float rgba[4];
    const int rc = oracle_scene_render(h, P, viewInverse, projInverse, W, H, ncams, &ray, 1, rgba, nullptr, nullptr,
                                       nullptr, nullptr, 1);
    g_trace = nullptr;
    if (rc) return rc;
    const int n = (int)(tr.size() / 7);
    std::memcpy(out, tr.data(), sizeof(float) * 7 * std::min(n, maxn));
    return n;
}

// Single-Gaussian response helper for known-answer tests.
int oracle_eval_response(const float* density_rec, const float* o, const float* d, float* gres,
                         float* galpha) {
    Scene s{nullptr, nullptr, density_rec, nullptr, 1, {}};
    const HitEval h = evalResponse(s, 0, v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]));
    *gres = h.gres;
    *galpha = h.galpha;
    return 0;
}

float oracle_kernel_scale(float density, float minResponse, uint32_t opts, float degree) {
    return kernelScale(density, minResponse, opts, degree);
}

int oracle_radiance_from_sh(uint32_t deg, const float* sh48, const float* dir, float* out3) {
    V3 c[16];
    for (int i = 0; i < 16; ++i) c[i] = v3(sh48[3 * i], sh48[3 * i + 1], sh48[3 * i + 2]);
    const V3 r = radianceFromSpH(deg, c, v3(dir[0], dir[1], dir[2]), true);
    out3[0] = r.x;
    out3[1] = r.y;
    out3[2] = r.z;
    return 0;
}

}  // extern "C"
