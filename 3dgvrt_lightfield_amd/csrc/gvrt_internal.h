// gvrt_internal.h — the handle behind gvrt.h and the launchers each .hip file provides.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gvrt.h"
#include "gvrt_device.h"

struct gvrt_context {
    int device = -1;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;  // created with the handle; stream is it unless gvrt_set_stream chose another
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    uint64_t device_bytes = 0;
    std::unordered_map<void*, uint64_t> allocs;

    // splat inputs (Model::allocateAttributeBuffers, Vulkan3DGRTModel.cpp:163-222)
    uint64_t n = 0;
    float* d_pos = nullptr;    // 3n
    float* d_rot = nullptr;    // 4n
    float* d_scl = nullptr;    // 3n
    float* d_opa = nullptr;    // n
    float* d_fdc = nullptr;    // 3n
    float* d_frest = nullptr;  // 45n + 90 zero pad (Q5 out-of-bounds reads read 0)

    // enclosing outputs, compaction order (saveIdx)
    bool enclosed = false;
    gvrt_enclosing_params enc{};
    uint64_t m = 0;
    uint64_t cap = 0;
    float* d_density12 = nullptr;
    float* d_sh48 = nullptr;
    float* d_verts = nullptr;
    uint32_t* d_tris = nullptr;
    uint32_t* d_src = nullptr;
    gvrt::RenderRec* d_recs_c = nullptr;
    float* d_boxes_c = nullptr;  // 6 per survivor
    uint32_t* d_absmax = nullptr;  // k_pos_absmax result (float bits)
    float box_pad_abs = 0.0f;      // absolute proxy-box padding of the last enclose: 2^-18 x max |position|
    uint32_t* d_flags = nullptr;
    uint32_t* d_scan = nullptr;

    // acceleration structure, leaf order
    bool accel = false;
    gvrt::RenderRec* d_recs = nullptr;
    float* d_sh = nullptr;
    gvrt::BvhNode* d_nodes = nullptr;   // binary LBVH (kept for diagnostics)
    gvrt::Bvh4Node* d_nodes4 = nullptr; // 4-wide collapse traversed by the render kernel
    uint64_t n_nodes4 = 0;
    gvrt::Bvh4Node* d_nodes4x8 = nullptr;  // 8 octant copies of d_nodes4 (planes in near / far order)
    uint32_t* d_leaf_src = nullptr;  // leaf -> compaction index
    // FAST launches: the 4-wide nodes with acceptance boxes (gvrt_launch_accept_nodes), plain and in 8 octant
    // copies, for the acceptance thresholds in accept_key (refit when a launch brings other thresholds)
    gvrt::Bvh4Node* d_nodes4e = nullptr;
    gvrt::Bvh4Node* d_nodes4ex8 = nullptr;
    float accept_key[2] = {0.0f, 0.0f};
    bool accept_ok = false;
    bool accept_nomem = false;  // the acceptance copy did not fit (until the next build)
    // Single-origin FAST launches read one of two copies of the leaf records whose positions are replaced by the
    // launch camera's kernel-frame origin (k_rec_origin, in stream order); d_recs itself always keeps the
    // positions, so no other reader has to restore anything.  Two copies: a camera that comes back to the
    // previous origin (alternating views) finds its copy still written.
    gvrt::RenderRec* d_okrecs[2] = {nullptr, nullptr};
    uint64_t okrecs_n = 0;
    float okrecs_origin[2][3] = {{0, 0, 0}, {0, 0, 0}};
    bool okrecs_valid[2] = {false, false};
    bool okrecs_full[2] = {false, false};  // every field but the origin equals d_recs (a pass may write 12 B)
    int okrecs_cur = 0;
    bool okrecs_nomem = false;  // the copies did not fit (until the next build): launches read d_recs
    // multi-origin launches (light-field rigs): one record copy per camera with that camera's kernel-frame origins,
    // kept while the set of origins is unchanged
    gvrt::RenderRec* d_recs_cams = nullptr;
    uint64_t recs_cams_bytes = 0;
    std::vector<float> recs_cams_origins;
    bool recs_cams_ok = false;
    bool recs_cams_nomem = false;  // the per-camera copies did not fit (until the next build)
    // adaptive enclosing (opts & 1): each leaf's icosahedron half-width sqrt(3) kernelScale(density), once per build
    // (the render kernel computing it per leaf visit spilled 36 B per lane)
    float* d_leaf_hk = nullptr;
    bool leaf_hk_ok = false;
    uint64_t n_leaves = 0;           // BVH leaves: the survivors, or their split pieces
    uint32_t* d_leaf_aux = nullptr;  // split: per leaf {proxy, cell, proxy's cell range lo, hi} (uint4); else null
    uint32_t split_cells = 0;        // grid cells on the longest axis (0: no split)
    float grid_min[3] = {0, 0, 0};
    float grid_inv = 0.0f;           // 1 / cell size
    uint32_t grid_n[3] = {0, 0, 0};
    uint32_t depth = 0;   // binary LBVH depth
    uint32_t depth4 = 0;  // 4-wide levels (bounds the traversal stack: 3 pushes per level)

    // per-render scratch
    bool stats_on = false;
    unsigned long long* d_stats = nullptr;
    uint32_t* d_tiles = nullptr;
    uint64_t tiles_cap = 0;
    // camera matrices: a ring of CAM_RING slots in device memory, filled from a pinned host mirror, so that a
    // camera that changes every frame (a moving camera) is uploaded without waiting for the queued frames
    static constexpr uint32_t CAM_RING = 16;
    float* d_viewinv = nullptr;      // CAM_RING slots of cam_stride floats
    float* h_viewinv_pin = nullptr;  // pinned host mirror of the ring (the source of the stream-ordered uploads)
    uint64_t cam_stride = 0;         // floats per slot (16 x the largest camera count so far)
    uint32_t cam_slot = 0;           // the slot holding the current cameras
    bool cam_valid = false;          // cam_slot holds h_viewinv
    hipEvent_t cam_ev[CAM_RING] = {};  // recorded after the last launch that read each slot
    bool cam_ev_live[CAM_RING] = {};
    std::vector<float> h_viewinv;    // the cameras in cam_slot
    std::vector<uint32_t> h_tiles; // host copy of what d_tiles holds (uploaded only when the list changes)
    bool tiles_valid = false;      // d_tiles holds h_tiles
    // gvrt_unpack_tiles_rgba8's lists (own buffers: queued renders may read d_tiles): one per rank part of a
    // split frame, so that assembling a static split uploads nothing per frame
    struct TileListBuf {
        std::vector<uint32_t> host;
        uint32_t* dev = nullptr;
        uint64_t cap = 0;
        bool valid = false;
        uint64_t used = 0;  // last use (LRU)
    };
    std::vector<TileListBuf> unpack_lists;
    uint64_t unpack_calls = 0;
    std::vector<hipEvent_t> async_ev;  // event pairs of queued gvrt_render_async launches
    uint32_t async_pending = 0;
    double async_ms_sum = 0.0;         // kernel times of async launches drained before the next gvrt_sync
    uint64_t async_drained = 0;
    // cost-ordered dispatch: the previous launch's per-tile cost classes, tiles ordered costliest first
    uint64_t ord_key = 0;            // width | height << 16 | ncams << 32 (| 1 << 63: full frame) of the arrays below
    std::vector<uint32_t> ord_list;  // the caller's tile list the order belongs to (empty: full frame)
    uint64_t ord_n = 0;              // tiles
    bool ord_ready = false;          // d_order holds an order for ord_key / ord_list
    uint8_t* d_tbucket = nullptr;    // per tile-list position: cost class of the last launch
    uint32_t* d_thist = nullptr;     // [class counts, fill cursors] x launch parity (gvrt_render.hip)
    uint32_t ord_parity = 0;         // parity of the next launch
    uint32_t* d_tcode = nullptr;     // full frames: the tile list (cam << 24 | ty << 12 | tx), supertile order
    uint32_t* d_order = nullptr;     // dispatch order: tile-list positions, costliest class first
    uint8_t* d_tgrid = nullptr;      // moving camera: the classes on a screen grid (tiles_x x tiles_y x ncams)
    uint8_t* d_tbucket2 = nullptr;   // moving camera: the classes spread by the motion radius
    uint32_t ord_tx = 0, ord_ty = 0, ord_nc = 0;  // grid of the order arrays
    float ord_prev_vi[16] = {};      // camera 0 of the previous ordered launch (motion radius)
    bool ord_prev_valid = false;
    std::vector<uint32_t> h_tcode;   // host source of d_tcode (kept alive for its stream-ordered upload)
    void* d_stage = nullptr;  // staging for host outputs
    uint64_t stage_cap = 0;

    gvrt_stats stats{};
    // per-handle tuning switches (gvrt_set_option), measured-best defaults
    int64_t opt[GVRT_OPT_COUNT] = {1, 1, 1, 1, 0, 1, 0, 1, 0};
};

gvrt_status gvrt_fail(gvrt_context* c, gvrt_status code, const std::string& msg);
gvrt_status gvrt_hip_check(gvrt_context* c, hipError_t e, const char* what);
gvrt_status gvrt_dalloc(gvrt_context* c, void** p, uint64_t bytes);
void gvrt_dfree(gvrt_context* c, void** p);
// An optional speed-up copy (octant nodes, acceptance nodes, record-origin copies): false, with no error left on the
// handle, when it does not fit (hipMalloc fails, or the handle's device bytes would exceed GVRT_OPT_OPTIONAL_MEM_MB);
// the caller then runs without the copy
bool gvrt_dalloc_optional(gvrt_context* c, void** p, uint64_t bytes);

#define GVRT_HIP(ctx, expr)                                         \
    do {                                                            \
        hipError_t _e = (expr);                                     \
        if (_e != hipSuccess) return gvrt_hip_check(ctx, _e, #expr); \
    } while (0)

// gvrt_enclose.hip
gvrt_status gvrt_launch_enclose(gvrt_context* c, const gvrt_enclosing_params* p, uint64_t* m);
// gvrt_lbvh.hip
gvrt_status gvrt_launch_build_accel(gvrt_context* c, const gvrt_accel_params& p);
gvrt_status gvrt_ploc_build(gvrt_context* c, uint32_t m, const float* leaf_boxes, gvrt::BvhNode* bin,
                            int32_t* leaf_parent, int32_t* node_parent, int32_t* root, uint32_t* iterations);
// gvrt_sah.hip (the quality build on the device: binned SAH + SAH-optimal collapse)
gvrt_status gvrt_sah_build_device(gvrt_context* c, uint64_t m, const float* lboxes, gvrt::BvhNode* nodes,
                                  gvrt::Bvh4Node* out4, uint32_t* depth_out, uint64_t* n4_out, uint32_t* depth4_out,
                                  uint32_t dmax);
// gvrt_render.hip
// the render launch; ev_start / ev_stop are recorded at the kernel's start and end (its kernel time)
gvrt_status gvrt_launch_render_mode(gvrt_context* c, const gvrt::RenderArgs& a, uint64_t nwaves, bool literal,
                                    hipEvent_t ev_start, hipEvent_t ev_stop);
// codes: the tile list the order is over (cam << 24 | ty << 12 | tx); radius > 0: classes spread by a max filter
gvrt_status gvrt_launch_tile_order(gvrt_context* c, const uint32_t* codes, int radius);
// record preparation: op 0 save leaf positions, 1 write kernel-frame origins for o, 2 restore positions
// k_rec_origin: dst = d_recs with each position replaced by the kernel-frame origin of o, on `stream`; with cam_dst
// it also writes the 16 floats at cam into cam_dst (the launch's camera slot); pos_only: dst already holds the
// other fields of every record (only the three origin floats are written)
gvrt_status gvrt_launch_rec_origin(gvrt_context* c, const float* o, gvrt::RenderRec* dst, hipStream_t stream,
                                   float* cam_dst = nullptr, const float* cam = nullptr, bool pos_only = false);
// multi-origin launches: per-camera record copies (dst = ncams x n_leaves records) for the cameras at d_view_inv
gvrt_status gvrt_launch_rec_cams(gvrt_context* c, uint32_t ncams, const float* d_view_inv, gvrt::RenderRec* dst);
// adaptive enclosing: d_leaf_hk from the leaf records (k_leaf_hk)
gvrt_status gvrt_launch_leaf_hk(gvrt_context* c);
// the 8 octant copies of the 4-wide nodes (d_nodes4x8)
gvrt_status gvrt_launch_node_octants(gvrt_context* c);
// FAST launches: d_nodes4e (+ octant copies d_nodes4ex8) with acceptance boxes for these thresholds
gvrt_status gvrt_launch_accept_nodes(gvrt_context* c, float min_response, float alpha_min);
gvrt_status gvrt_launch_unpack(gvrt_context* c, const void* packed, const uint32_t* tiles,
                               uint64_t ntiles, uint32_t width, uint32_t height, void* frame);
