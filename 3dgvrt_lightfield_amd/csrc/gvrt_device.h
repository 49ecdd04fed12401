// gvrt_device.h — device-side records and math shared by the gfx950 kernels.
//
// HBM layout (per survivor, BVH-leaf order after gvrt_build_accel):
//   RenderRec  64 B   everything processHit needs except SH: position, activated density,
//                     R = quaternionWXYZToMatrix(q) (utils.glsl:13-34, i.e. R^T of the
//                     world rotation) as three GLSL columns, 1/scale.  One s_load_dwordx16.
//   SH         192 B  [f_dc.rgb, f_rest 45] (particlePrimitives.comp:207-214), read only for
//                     accepted crossings (fetchParticleSphCoefficients, gaussianfunctions.glsl:104-115)
//   BvhNode    64 B   two child AABBs inline + child links (LBVH, Karras 2012)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gvrt {

constexpr float EPS_T = 1e-9f;                        // 3dgs.glsl:13
constexpr int K_HITS = 16;                            // MAX_HIT_PER_TRACE, 3dgs.glsl:15
constexpr int K_FAST_DEFAULT = 32;                    // FAST k-buffer depth (fewer rounds; same image)
constexpr uint32_t INVALID_ID = 0xFFFFFFFFu;          // 3dgs.glsl:26
constexpr float INF_DIST = 1e20f;                     // 3dgs.glsl:27
constexpr float KERNEL_S = -0.0555555555556f;         // degree-4 response, gaussianfunctions.glsl:31-35
constexpr float PHI = 1.618033988749895f;             // particlePrimitives.comp:77
constexpr float IPHI = 0.618033988749895f;
constexpr float ICOSA_VRT_SCALE = 0.5f * 1.323169076499215f;  // particlePrimitives.comp:78-79
constexpr float SQRT3 = 1.7320508075688772f;
constexpr int STACK_DEPTH = 128;                      // per-wave LDS traversal stack
// Depth budget of the SAH builds (device gvrt_sah.hip and its host checker): max binary leaf depth, root at depth 1.
// A range of n proxies at depth d keeps d + ceil(log2 n) <= SAH_DEPTH_MAX: a SAH split whose larger side would break
// it halves the (Morton-ordered) range instead, which keeps it.  So the binary tree, and with it the 4-wide tree
// (every 4-wide level descends at least one binary level), stays within the traversal stack at any M and any
// geometry.  Trees of the stand-in scenes are 30-33 deep: the budget never fires there, their builds are unchanged.
constexpr uint32_t SAH_DEPTH_MAX = 43;
static_assert((4 - 1) * (SAH_DEPTH_MAX - 1) + 2 <= (uint32_t)STACK_DEPTH, "the 4-wide depth bound fits the stack");
__host__ __device__ inline uint32_t ceil_log2(uint32_t n) { return n <= 1 ? 0u : 32u - (uint32_t)__builtin_clz(n - 1u); }
// a split of a range at depth d into sides of nl and nr proxies keeps the budget dmax (<= SAH_DEPTH_MAX;
// gvrt_accel_params.depth_budget tightens it for tests)
__host__ __device__ inline bool sah_split_in_budget(uint32_t d, uint32_t nl, uint32_t nr, uint32_t dmax) {
    return d + 1u + ceil_log2(nl > nr ? nl : nr) <= dmax;
}
constexpr int TILE_CPO = 4;                           // cost classes per octave of the cost-ordered dispatch
constexpr int TILE_BUCKETS = 16 * TILE_CPO;           // classes: 1 k .. 64 M cycles

struct alignas(16) RenderRec {
    float px, py, pz, density;
    float c0x, c0y, c0z, c1x;  // GLSL mat3 columns of quaternionWXYZToMatrix(q)
    float c1y, c1z, c2x, c2y;
    float c2z, isx, isy, isz;  // giscl = 1/scale
};
static_assert(sizeof(RenderRec) == 64, "RenderRec must be 64 B");

struct alignas(16) BvhNode {
    float l0x, l0y, l0z, h0x;
    float h0y, h0z, l1x, l1y;
    float l1z, h1x, h1y, h1z;
    int32_t c0, c1;  // >= 0 internal node index; < 0 leaf ~index (record index)
    uint32_t pad0, pad1;  // pad0: split axis (c0 on the lower side)
};
static_assert(sizeof(BvhNode) == 64, "BvhNode must be 64 B");

// 4-wide node collapsed from the binary LBVH (every 4-wide node is a binary subtree opened greedily
// by surface area).  Per child the box is stored as (lo.x, hi.x, lo.y, hi.y, lo.z, hi.z): two scalar
// loads bring the whole node, and each axis' (lo, hi) is an aligned SGPR pair, so one v_pk_fma_f32
// gives both plane distances.  Empty slots hold a far point box that no ray can hit.
constexpr int BVH_W = 4;  // children per node (8-wide nodes: 24 % fewer node visits, 18 % more leaf visits, slower)
constexpr float EMPTY_BOX = 3e37f;
struct alignas(16) Bvh4Node {  // (name kept from the 4-wide layout; BVH_W children)
    float box[BVH_W][6];   // [child][lx, hx, ly, hy, lz, hz]
    int32_t child[BVH_W];  // >= 0: node index; < 0: leaf ~record index
    uint32_t nchild;
    uint32_t pad[3];       // [0] split axis of the children's order (0 x, 1 y, 2 z), [1] internal-child mask (bits
                           // 0-3) | split-piece leaf mask << 4 (leaves with a cell test), [2] acceptance widening D
};
static_assert(sizeof(Bvh4Node) == 28 * BVH_W + 16, "node layout: 128 B (4-wide) / 240 B (8-wide)");


struct f3 {
    float x, y, z;
};
__host__ __device__ inline f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
__host__ __device__ inline f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
__host__ __device__ inline f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
__host__ __device__ inline f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
__host__ __device__ inline f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
__host__ __device__ inline float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ inline f3 cross3(f3 a, f3 b) {
    return mk3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}

// Render-kernel launch arguments (one struct, passed by value).
struct CamArg {  // one camera matrix as a by-value kernel argument
    float v[16];
};

struct RenderArgs {
    const RenderRec* __restrict__ recs;  // leaf order (one per BVH leaf)
    const RenderRec* __restrict__ crecs; // by k-buffer id: = recs, or the compaction order when split
    const float* __restrict__ sh;        // 48 f32 per k-buffer id
    const uint4* __restrict__ aux;       // split: per leaf {proxy, cell, cell range lo, hi}; else null
    const Bvh4Node* __restrict__ nodes;
    const float* __restrict__ view_inv;  // 16 per camera, column-major
    const uint32_t* __restrict__ tiles;  // packed (cam<<24 | ty<<12 | tx) or null
    float proj_inv[16];
    float aabb[6];
    float min_transmittance;
    float min_response;
    float alpha_min;
    float pixel_offset;
    float alpha_init;
    float kernel_h;      // sqrt(3) * kernelScale (uniform when opts has no adaptive clamping)
    float gpre;          // pre-reject bound on the squared line distance: sqrt(ln(min_response)/S) * 1.001
    float kmin;          // enclosing kernelMinResponse (adaptive clamping recomputes kS per particle)
    float kdeg;
    uint32_t kopts;
    uint32_t sph_deg;
    uint32_t width, height, ncams;
    uint32_t tiles_x, tiles_y;
    uint64_t ntiles;
    uint32_t nrecs;
    uint32_t tmin_inclusive;
    uint32_t max_rounds;
    uint32_t ray_dirs_layout;
    uint32_t packed;
    uint32_t kfast;  // FAST-mode k-buffer depth (8, 12, 16, 24)
    uint32_t okrec;      // records hold kernel-frame origins for this launch's camera origin(s)
    uint64_t recs_cam_stride;  // okrec with several origins: camera c reads the record copy at recs + c x stride
    const Bvh4Node* nodes8;  // the 4-wide nodes in 8 copies, copy o with each axis a of o's bits stored (hi, lo):
    uint64_t nodes8_stride;  // a wave whose rays share octant o reads (near, far) planes in place (nodes per copy)
    uint32_t box_exact;  // box padding covers the plane rounding for these cameras: no per-child slack
    float grid_min[3];  // split grid (SplitBLAS analogue): origin and 1 / cell size
    float grid_inv;
    uint8_t* rgba8;
    float* rgba32f;
    float* ray_dirs;
    uint32_t* hit_counts;
    unsigned long long* stats;  // [crossings, accepted, rounds] or null
    const uint32_t* perm;       // dispatch order: workgroup -> tile-list position (cost-ordered), or null
    uint8_t* tile_bucket;       // per tile-list position: log-scale cost class of its wave, or null
    uint32_t* tile_hist;        // tiles per cost class (TILE_BUCKETS), for the next frame's order
    const float* leaf_hk;       // adaptive enclosing (opts & 1): sqrt(3) x kernelScale(density) per leaf, else null
};

// kernelScale, particlePrimitives.comp:81-105
__host__ __device__ inline float kernel_scale(float density, float modulatedMinResponse, uint32_t opts,
                                              float kernelDegree) {
    const float responseModulation = (opts & 1u) != 0 ? density : 1.0f;
    const float minResponse = fminf(modulatedMinResponse / responseModulation, 0.97f);
    if (kernelDegree < 0) {
        const float k = fabsf(kernelDegree);
        const float s = 1.0f / powf(3.0f, k);
        return powf((1.f / (logf(minResponse) - 1.f) + 1.f) / s, 1.f / k);
    }
    if (kernelDegree == 0) return ((1.0f - minResponse) / 3.0f) / -0.329630334487f;
    const float b = kernelDegree;
    const float a = -4.5f / powf(3.0f, b);
    return powf(logf(minResponse) / a, 1.0f / b);
}

}  // namespace gvrt
