/*
 * gvrt.h — C-ABI of the MI355X-native Gaussian ray tracer (libgvrt.so).
 *
 * This is the drop-in boundary for the Particle Rendering hot path of
 * wlckslxh/3DGVRT_lightfield (reference snapshot 2025-08-24).  Each entry point names the
 * reference interface it replaces (paths relative to the reference root).  Plain C types
 * only: pointers, sizes and POD structs; no HIP or torch types cross this boundary.
 *
 * Threading: a handle is bound to one HIP device and one HIP stream and is not thread-safe.
 * Different handles (one per GPU) may be driven from different threads or processes.
 * Errors: every call returns a gvrt_status; nothing aborts.  gvrt_last_error() gives text.
 */
#ifndef GVRT_H_
#define GVRT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GVRT_ABI_VERSION 2

typedef int32_t gvrt_status;
#define GVRT_OK 0
#define GVRT_ERR_INVALID_ARG (-1)
#define GVRT_ERR_OOM (-2)
#define GVRT_ERR_HIP (-3)
#define GVRT_ERR_STATE (-4)
#define GVRT_ERR_NO_DEVICE (-5)
#define GVRT_ERR_IO (-6)
#define GVRT_ERR_UNSUPPORTED (-7)
#define GVRT_ERR_RCCL (-8) /* a collective of the multi-GPU frame exchange failed (host/gvrt_host.h GvrtApp) */

typedef struct gvrt_context* gvrt_handle;

/* Host SoA splat arrays, laid out exactly as vk3DGRT::SplatSet
 * (base/Vulkan3DGRTModel.h:16-28): f_rest already reordered to coefficient-major RGB
 * (base/Vulkan3DGRTModel.cpp:62-77), rotation stored w,x,y,z. */
typedef struct {
    uint64_t n;
    const float* positions; /* 3n  x,y,z */
    const float* f_dc;      /* 3n  f_dc_0..2 */
    const float* f_rest;    /* 45n coefficient-major interleaved RGB */
    const float* opacity;   /* n   raw logit */
    const float* scale;     /* 3n  raw log-scale */
    const float* rotation;  /* 4n  raw quaternion w,x,y,z */
} gvrt_splats;

/* GaussianEnclosingUniformData (base/VulkanUtils.h:63-68); host defaults from
 * projects/VulkanFullRT/VulkanFullRT.cpp:1353-1356. */
typedef struct {
    float kernel_min_response; /* 0.0113 */
    uint32_t opts;             /* MOGRenderOpts bit 0 = adaptive kernel clamping; default 0 */
    float degree;              /* 4 */
    uint32_t emit_triangles;   /* 1: also keep the 36n vertex / 60n index proxy soup */
} gvrt_enclosing_params;

/* Render parameters: UniformDataStatic (base/VulkanUtils.h:50-61), the GLSL constants of
 * shaders/glsl/base/3dgs.glsl:13-22 and the variant switches of SURVEY §8a (Q10, Q11, Q13). */
typedef struct {
    float aabb[6];                   /* minX,minY,minZ,maxX,maxY,maxZ = +-100 */
    float min_transmittance;         /* 0.001 */
    float hit_min_gaussian_response; /* 0.0113 */
    uint32_t sph_eval_degree;        /* 3 */
    float alpha_min;                 /* 1/255 (ALPHA_MIN_THRESHOLD) */
    float pixel_offset;              /* 0 = ray-query compute variant (default), 0.5 = RT pipeline / LF */
    float alpha_init;                /* 0 = ray-query variant (default), 1 = RT pipeline / LF */
    uint32_t tmin_inclusive;         /* 0 (default); 1 only with mode LITERAL and max_rounds > 0 */
    uint32_t mode;                   /* GVRT_MODE_FAST (default) or GVRT_MODE_LITERAL */
    uint32_t max_rounds;             /* 0 = unlimited */
    uint32_t ray_dirs_layout;        /* 0: [cam][y][x]; 1: light-field [cam][x][y] (raygenGaussianLightField.rgen:129) */
    uint32_t kbuffer_depth;          /* FAST only: 0 = default (32); 8, 12, 16, 20, 24 or 32 slots per ray.  Sets
                                        the number of traversal rounds; rays whose tie or threshold decisions the
                                        oracle flags can move with it (the 24 -> 32 default change altered a few
                                        such garden and dense rgba8 pixels) */
    uint32_t reserved[4];
} gvrt_render_params;

#define GVRT_MODE_FAST 0u    /* only accepted crossings enter the k-buffer (same image) */
#define GVRT_MODE_LITERAL 1u /* every crossing enters the 16-slot k-buffer, rounds as the reference */

/* One 8x8 pixel tile of camera `cam` (tile coordinates, not pixels). */
typedef struct {
    uint16_t tx, ty;
    uint16_t cam, pad;
} gvrt_tile;

/* Output surfaces.  Any pointer may be NULL.  Pointers are device pointers when
 * device_ptrs = 1, else host pointers (the library stages them). */
typedef struct {
    void* rgba8;        /* uint8  [cam][H][W][4]  (R8G8B8A8_UNORM storage image) */
    float* rgba32f;     /* float  [cam][H][W][4]  (the pre-quantisation rayRadiance) */
    float* ray_dirs;    /* float4 per ray, layout per params.ray_dirs_layout */
    uint32_t* hit_counts; /* accepted hits per ray (ENABLE_HIT_COUNTS, raygen.rgen:187-189) */
    uint32_t device_ptrs;
    uint32_t packed;      /* 1: outputs are tile-packed in tile-list order (64 px per tile, row-major in tile) */
} gvrt_image;

typedef struct {
    uint64_t n_input;      /* N */
    uint64_t n_survivors;  /* M (ParticleCounts) */
    uint64_t bvh_nodes;    /* internal nodes */
    uint32_t bvh_depth;    /* max leaf depth of the binary tree (root 1) */
    uint32_t bvh_depth4;   /* levels of the 4-wide tree the render kernel traverses */
    uint64_t rays;         /* last render */
    uint64_t crossings;    /* processed crossings (X), last render; only with stats enabled */
    uint64_t accepted;     /* accepted crossings (A) */
    uint64_t rounds;       /* sum over rays of k-buffer rounds */
    float enclose_ms;
    float accel_ms;
    float render_ms;       /* device time of the last render kernel (HIP events on the handle's stream) */
    float pad1;
    uint64_t device_bytes; /* bytes of device memory held by the handle */
    uint64_t wave_node_visits;  /* traversal diagnostics of the last render (stats enabled): */
    uint64_t wave_leaf_visits;  /*   BVH nodes / leaves visited per wave, summed over waves,  */
    uint64_t lane_leaf_tests;   /*   and ray-proxy clip tests summed over lanes               */
    uint64_t phase_cycles[4];   /* s_memtime cycles summed over waves (stats enabled): node visits,
                                   leaf tests + k-buffer insertion, compositing, whole kernel */
    uint64_t wave_dead_visits;  /* node visits in which no lane hit any child box */
    uint64_t bvh_leaves;        /* BVH leaves: the survivors, or their grid-cell pieces when split */
    uint64_t wave_rounds;       /* traversal rounds summed over waves (stats enabled) */
    uint64_t wave_late_node_visits; /* node visits in the second and later rounds of a wave */
    uint32_t bvh_builder;       /* the builder that made the tree: the requested one, or 2 (device SAH) when an
                                   LBVH / PLOC tree was too deep for the traversal stack */
    uint32_t bvh_depth4_rebuilt; /* 4-wide levels of that too-deep tree (0: the requested builder's tree was kept) */
} gvrt_stats;

/* --------------------------------------------------------------------------------------- */
int gvrt_abi_version(void);
const char* gvrt_build_info(void);

void gvrt_default_enclosing_params(gvrt_enclosing_params* p);
void gvrt_default_render_params(gvrt_render_params* p);

/* VulkanRTBase::initVulkan device pick + VulkanFullRT ctor (base/VulkanRTBase.cpp:1361-1432). */
gvrt_status gvrt_create(int device, gvrt_handle* out);
/* VulkanFullRT::~VulkanFullRT (projects/VulkanFullRT/VulkanFullRT.cpp:209-259). */
gvrt_status gvrt_destroy(gvrt_handle h);
const char* gvrt_last_error(gvrt_handle h);
gvrt_status gvrt_device_count(int* count);

/* vk3DGRT::Model::allocateAttributeBuffers (base/Vulkan3DGRTModel.cpp:163-222):
 * copies the six SoA arrays to device memory. */
gvrt_status gvrt_load_splats(gvrt_handle h, const gvrt_splats* s);

/* VulkanFullRT::computeGaussianEnclosingIcosaHedron (VulkanFullRT.cpp:1503-1514) dispatching
 * particlePrimitives.comp; writes the survivor count (ParticleCounts) to *m. */
gvrt_status gvrt_build_enclosing(gvrt_handle h, const gvrt_enclosing_params* p, uint64_t* m);

/* Read back the enclosing outputs in compaction order (saveIdx): density records 12 f32
 * (std140 ParticleDensity), SH records 48 f32, and when emit_triangles was set the
 * 36 f32 vertex / 60 u32 index proxy soup; src_index[i] = input index of survivor i.
 * Any pointer may be NULL; host pointers; arrays sized for m survivors. */
gvrt_status gvrt_read_enclosing(gvrt_handle h, float* density12, float* sh48, float* verts36,
                                uint32_t* tris60, uint32_t* src_index);

/* Acceleration-structure options.  split_cells > 0 is the SplitBLAS analogue (SPLIT_BLAS,
 * base/Define.h:45-47; projects/VulkanFullRT/SplitBLAS.cpp:91-186): a grid of split_cells cells on
 * the scene's longest axis (the reference uses NUMBER_OF_CELLS_PER_LONGEST_AXIS = 10), every proxy
 * split into one piece per grid cell its box overlaps, each piece admitting only the crossings whose
 * point lies in its cell (so every crossing is found exactly once).  split_cells <= 1023 (0: no
 * split).  builder: 0 Karras LBVH, 1 PLOC, 2 binned SAH on the device (the PREFER_FAST_TRACE-style
 * quality build of a static scene, VulkanFullRT.cpp:621), 3 the same binned SAH on the host (the
 * device build's checker: identical trees).  collapse: 0 greedy surface-area 4-wide collapse on the
 * device, 1 surface-area-optimal collapse (dynamic programming; on the device with builder 2, on
 * the host otherwise).  Every build fits the render kernel's traversal stack, whatever the geometry:
 * the SAH builds keep a binary depth budget by construction (a split whose larger side could not
 * finish within it halves the Morton-ordered range instead), and an LBVH or PLOC tree too deep for the
 * stack is rebuilt by the device SAH build (the Vulkan driver's BVH never refuses a scene either).
 * depth_budget: 0 = the default budget (43 binary levels, i.e. at most 42 4-wide levels); smaller values
 * (>= 1 + ceil(log2 survivors)) tighten it for tests of the budget path.  split_min_span (with
 * split_cells): a proxy is split only when its box overlaps at least this many cells along one axis,
 * smaller ones stay whole (one piece admitting every crossing); 0-2 = every proxy that overlaps more
 * than one cell (the reference's rule), at most 1023.  A split that splits no proxy is the unsplit
 * build (gvrt_stats.bvh_leaves = survivors).  Pieces keep every per-leaf path of the unsplit tree
 * (acceptance boxes, kernel-frame origin records, exact boxes); a leaf that is a piece costs one more
 * 16-B load per visit. */
typedef struct {
    uint32_t split_cells;
    uint32_t builder;
    uint32_t collapse;
    uint32_t depth_budget;
    uint32_t split_min_span;
    uint32_t reserved[3];
} gvrt_accel_params;

void gvrt_default_accel_params(gvrt_accel_params* p);

/* createBottomLevel/TopLevelAccelerationStructure3DGRT (VulkanFullRT.cpp:575-787):
 * BVH over the proxies (Morton codes, radix sort, Karras hierarchy, 4-wide collapse). */
gvrt_status gvrt_build_accel(gvrt_handle h);
gvrt_status gvrt_build_accel_ex(gvrt_handle h, const gvrt_accel_params* p);

/* Copy the acceleration structure to host memory (parity checks of the builders, like inspecting a
 * serialized VkAccelerationStructure).  which = 0: the binary tree (n_leaves - 1 nodes of 64 B:
 * child 0 box, child 1 box, c0, c1, split axis, 0); which = 1: the 4-wide tree the render kernel
 * traverses (128 B per node); which = 2: adaptive enclosing only, each leaf's icosahedron half-width
 * sqrt(3) kernelScale(density) as the build wrote it for the render kernel (4 B per leaf).  *count receives
 * the element count; at most cap elements are written (out may be NULL to query the count). */
gvrt_status gvrt_read_accel(gvrt_handle h, int which, void* out, uint64_t cap, uint64_t* count);

/* Particle Rendering pass: buildCommandBuffer (VulkanFullRT.cpp:1185-1244) dispatching
 * raygen/anyhit (RT) or particleRendering.comp (RQ), and the light-field launch
 * computeGaussianLightField (VulkanFullRT.cpp:1900-1976) when ncams > 1.
 * view_inverse: ncams column-major 4x4 (UniformDataDynamic.viewInverse per camera);
 * proj_inverse: one column-major 4x4.  tiles/ntiles: optional 8x8 tile list (multi-GPU
 * split); NULL renders every tile of every camera.  Synchronous. */
gvrt_status gvrt_render(gvrt_handle h, const gvrt_render_params* p, const float* view_inverse,
                        const float* proj_inverse, uint32_t width, uint32_t height,
                        uint32_t ncams, const gvrt_tile* tiles, uint64_t ntiles,
                        const gvrt_image* out);

/* Asynchronous variant of gvrt_render (SURVEY §8b "an async variant plus gvrt_sync"): queues the
 * launch on the handle's stream and returns; outputs must be device pointers and stats off.  Frames
 * queued back to back run without a host round trip between them (the reference's per-frame
 * vkQueueSubmit + fence, VulkanRTBase.cpp:983-1059).  gvrt_sync waits for every queued launch and sets
 * stats.render_ms to their mean kernel time.  A queue of 1024 launches waits for them before queueing
 * the next (bounded event pool). */
gvrt_status gvrt_render_async(gvrt_handle h, const gvrt_render_params* p, const float* view_inverse,
                              const float* proj_inverse, uint32_t width, uint32_t height,
                              uint32_t ncams, const gvrt_tile* tiles, uint64_t ntiles,
                              const gvrt_image* out);
gvrt_status gvrt_sync(gvrt_handle h);

/* Launch on the caller's HIP stream (a hipStream_t; NULL: the handle's own stream again), as a BLAS
 * handle's set-stream does: the caller's work on that stream is then ordered with the renders without a
 * host round trip or a cross-stream event.  The multi-GPU frame exchange renders on the stream its
 * gathers are posted from (the reference chains its per-frame submits with semaphores,
 * VulkanRTBase.cpp:983-1059).  Waits for the work queued on the previous stream first; the stream must
 * outlive its use by the handle.  The handle's own stream is non-blocking: work on the legacy NULL
 * stream is not ordered with it, so a caller that posts its work there cannot share it this way. */
gvrt_status gvrt_set_stream(gvrt_handle h, void* stream);

/* Device identity for the benchmark report: the VkPhysicalDeviceProperties fields vks::Benchmark
 * prints and writes to fps.txt (deviceName, driverVersion; base/benchmark.hpp:23,67-70,85). */
typedef struct {
    char device_name[256];
    uint32_t driver_version;  /* hipDriverGetVersion */
    uint32_t compute_units;
    uint64_t total_memory;    /* bytes of device memory */
    char arch_name[64];       /* e.g. "gfx950:sramecc+:xnack-" */
} gvrt_device_properties;
gvrt_status gvrt_get_device_properties(int device, gvrt_device_properties* out);

/* Device buffers held by a handle, i.e. vk3DGRT::Model::Attributes::storageBuffer
 * (base/Vulkan3DGRTModel.h:43-48, filled by allocateAttributeBuffers, Vulkan3DGRTModel.cpp:163-222)
 * and the Gaussian Enclosing outputs bound to the render pass (ParticleDensity / SH storage buffers,
 * VulkanFullRT.cpp:1045-1062).  Device pointers, valid until the next load / build / destroy on the
 * handle; NULL where the stage has not run (vertices / indices also need emit_triangles). */
typedef struct {
    uint64_t n;                       /* splats loaded */
    const float* positions;           /* 3n  */
    const float* rotations;           /* 4n  */
    const float* scales;              /* 3n  */
    const float* densities;           /* n   raw opacity */
    const float* features_albedo;     /* 3n  f_dc */
    const float* features_specular;   /* 45n f_rest (coefficient-major) */
    uint64_t m;                       /* survivors of the enclosing pass */
    const float* vertices;            /* 36m proxy vertices */
    const uint32_t* indices;          /* 60m proxy triangle indices */
    const float* particle_density;    /* 12m std140 ParticleDensity records */
    const float* particle_sph;        /* 48m SH records */
} gvrt_device_buffers;
gvrt_status gvrt_get_device_buffers(gvrt_handle h, gvrt_device_buffers* out);

/* Per-handle tuning switches: the measured-best defaults; each exists so that a same-box
 * A/B can turn one choice off.  None of them changes an image.  Values are 0 or 1 except where stated. */
#define GVRT_OPT_TILE_ORDER 0u      /* 1 (default): tiles dispatched costliest first by the previous launch's
                                       per-tile costs; 0: supertile order */
#define GVRT_OPT_TILE_XCD 1u        /* 1 (default): each cost class dealt to the 8 XCDs in contiguous chunks */
#define GVRT_OPT_OCTANT_NODES 2u    /* 1 (default): waves read the octant copy of the nodes (8x node memory) */
#define GVRT_OPT_RECORD_ORIGINS 3u  /* 1 (default): FAST launches read copies of the leaf records holding each
                                       camera's kernel-frame origins, written by one pass per camera origin (kept
                                       while the origins stay the same; up to 16 cameras per launch) */
#define GVRT_OPT_BOX_SLACK 4u       /* 0 (default): per-child exit slack only when the box padding does not
                                       cover the plane rounding for the launch's cameras; 1: always */
#define GVRT_OPT_PACKED_KBUFFER 5u  /* 1 (default): packed FAST k-buffer when record ids fit 24 bits; 0: the
                                       unpacked FAST kernel that larger scenes take */
#define GVRT_OPT_ORDER_SPREAD 6u    /* 0..8 (default 0): the least radius, in tiles, by which the previous launch's
                                       tile costs are spread (max filter) before ordering; the camera's motion sets
                                       it otherwise (0 for a static camera) */
#define GVRT_OPT_ACCEPT_BOXES 7u   /* 1 (default): FAST launches traverse a copy of the 4-wide nodes in which the
                                       leaves of all-leaf nodes have the boxes of their acceptance ellipsoids (for
                                       the launch's hit_min_gaussian_response / alpha_min) and particles that can
                                       never be accepted are dropped; 0: the proxy boxes */
#define GVRT_OPT_OPTIONAL_MEM_MB 8u /* 0 (default): no limit; N > 0: the optional speed-up copies (octant and
                                       acceptance node copies, record-origin copies) are allocated only while the
                                       handle's device memory stays within N MiB; a copy that does not fit (or
                                       whose hipMalloc fails) is left out and launches run without it */
#define GVRT_OPT_COUNT 9u
gvrt_status gvrt_set_option(gvrt_handle h, uint32_t option, int64_t value);
gvrt_status gvrt_get_option(gvrt_handle h, uint32_t option, int64_t* value);

/* Enable per-render statistics (crossings/accepted/rounds; costs one atomic per wave). */
gvrt_status gvrt_set_stats(gvrt_handle h, int enable);
gvrt_status gvrt_get_stats(gvrt_handle h, gvrt_stats* s);

/* Scatter a tile-packed rgba8 buffer (gathered from ranks) into a full frame [ncams][H][W][4]; device
 * ptrs.  Every tile must lie inside the frame (tx < ceil(W/8), ty < ceil(H/8), cam < ncams), else
 * GVRT_ERR_INVALID_ARG and nothing is written.  Runs on the handle's stream behind any queued
 * gvrt_render_async launches: synchronous when none are queued, else it completes by gvrt_sync. */
gvrt_status gvrt_unpack_tiles_rgba8(gvrt_handle h, const void* packed, const gvrt_tile* tiles,
                                    uint64_t ntiles, uint32_t width, uint32_t height, uint32_t ncams,
                                    void* frame);

/* Per-tile cost classes of the last cost-ordered launch (GVRT_OPT_TILE_ORDER): class c means the tile's wave
 * ran about 2^(c/4) x 1024 cycles (0..63).  A full-frame launch fills out[(cam * ceil(H/8) + ty) * ceil(W/8) + tx];
 * a caller tile list fills out[i] for list entry i.  n must be that tile count.  Waits for queued launches.
 * GVRT_ERR_STATE when no ordered launch has run at this size.  The multi-GPU tile split uses it to cut the
 * frame into parts of equal cost; the reference has no equivalent (one GPU, one dispatch). */
gvrt_status gvrt_read_tile_costs(gvrt_handle h, uint8_t* out, uint64_t n);

/* --------------------------------------------------------------------------------------- */
/* Host-side loader: vk3DGRT::PLYLoader::loadPLYModel (base/Vulkan3DGRTModel.cpp:7-125).
 * Allocates host arrays owned by the returned object; free with gvrt_ply_free. */
typedef struct {
    uint64_t n;
    float* positions;
    float* f_dc;
    float* f_rest;
    float* opacity;
    float* scale;
    float* rotation;
} gvrt_splat_buffers;

gvrt_status gvrt_ply_load(const char* path, gvrt_splat_buffers* out);
void gvrt_ply_free(gvrt_splat_buffers* b);
/* Write a binary little-endian 3DGS PLY (inverse of the loader; f_rest written channel-major). */
gvrt_status gvrt_ply_save(const char* path, const gvrt_splats* s);

#ifdef __cplusplus
}
#endif
#endif /* GVRT_H_ */
