// gvrt_api.hip — the C-ABI of include/gvrt.h: handle lifetime, device memory, launches.
//
// The library owns all device memory (splats, proxies, LBVH, scratch); callers own host
// arrays (copied during the call) and output surfaces.  No pointer is retained after a call.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "gvrt_internal.h"

using namespace gvrt;

static thread_local std::string g_global_err;

gvrt_status gvrt_fail(gvrt_context* c, gvrt_status code, const std::string& msg) {
    if (c) c->err = msg;
    else g_global_err = msg;
    return code;
}

gvrt_status gvrt_hip_check(gvrt_context* c, hipError_t e, const char* what) {
    if (e == hipSuccess) return GVRT_OK;
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return gvrt_fail(c, e == hipErrorOutOfMemory ? GVRT_ERR_OOM : GVRT_ERR_HIP, m);
}

gvrt_status gvrt_dalloc(gvrt_context* c, void** p, uint64_t bytes) {
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        *p = nullptr;
        (void)hipGetLastError();
        return gvrt_hip_check(c, e, "hipMalloc");
    }
    c->allocs[*p] = bytes;
    c->device_bytes += bytes;
    return GVRT_OK;
}

bool gvrt_dalloc_optional(gvrt_context* c, void** p, uint64_t bytes) {
    *p = nullptr;
    const int64_t cap_mb = c->opt[GVRT_OPT_OPTIONAL_MEM_MB];
    if (cap_mb > 0 && c->device_bytes + bytes > ((uint64_t)cap_mb << 20)) return false;
    if (gvrt_dalloc(c, p, bytes) != GVRT_OK) {
        *p = nullptr;
        c->err.clear();
        return false;
    }
    return true;
}

void gvrt_dfree(gvrt_context* c, void** p) {
    if (!*p) return;
    auto it = c->allocs.find(*p);
    if (it != c->allocs.end()) {
        c->device_bytes -= it->second;
        c->allocs.erase(it);
    }
    (void)hipFree(*p);
    *p = nullptr;
}

extern "C" {

int gvrt_abi_version(void) { return GVRT_ABI_VERSION; }

const char* gvrt_build_info(void) {
    return "gvrt " "abi2 gfx950 hip" " (" __DATE__ " " __TIME__ ")";
}

void gvrt_default_enclosing_params(gvrt_enclosing_params* p) {
    if (!p) return;
    p->kernel_min_response = 0.0113f;  // VulkanFullRT.cpp:1354
    p->opts = 0;                       // MOGRenderNone, VulkanFullRT.cpp:1355
    p->degree = 4.0f;                  // VulkanFullRT.cpp:1356
    p->emit_triangles = 0;
}

void gvrt_default_render_params(gvrt_render_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    const float aabb[6] = {-100.f, -100.f, -100.f, 100.f, 100.f, 100.f};  // VulkanUtils.h:53
    std::memcpy(p->aabb, aabb, sizeof(aabb));
    p->min_transmittance = 0.001f;          // VulkanUtils.h:54
    p->hit_min_gaussian_response = 0.0113f;  // VulkanUtils.h:55
    p->sph_eval_degree = 3;                  // VulkanUtils.h:56
    p->alpha_min = 0.0039215686275f;         // 3dgs.glsl:16
    p->pixel_offset = 0.0f;                  // RQ variant (particleRendering.comp:124)
    p->alpha_init = 0.0f;                    // RQ variant (particleRendering.comp:132)
    p->tmin_inclusive = 0;
    p->mode = GVRT_MODE_FAST;
    p->max_rounds = 0;
    p->ray_dirs_layout = 0;
}

gvrt_status gvrt_device_count(int* count) {
    if (!count) return gvrt_fail(nullptr, GVRT_ERR_INVALID_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *count = 0;
        return GVRT_OK;
    }
    *count = n;
    return GVRT_OK;
}

gvrt_status gvrt_create(int device, gvrt_handle* out) {
    if (!out) return gvrt_fail(nullptr, GVRT_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return gvrt_fail(nullptr, GVRT_ERR_NO_DEVICE, "no HIP device available");
    }
    if (device < 0 || device >= n) return gvrt_fail(nullptr, GVRT_ERR_INVALID_ARG, "device index out of range");
    gvrt_context* c = new (std::nothrow) gvrt_context();
    if (!c) return gvrt_fail(nullptr, GVRT_ERR_OOM, "host allocation failed");
    c->device = device;
    e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    c->stream = c->own_stream;
    if (e == hipSuccess) e = hipEventCreate(&c->ev0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev1);
    if (e != hipSuccess) {
        gvrt_status s = gvrt_hip_check(nullptr, e, "gvrt_create");
        delete c;
        return s;
    }
    if (gvrt_dalloc(c, (void**)&c->d_stats, 128) != GVRT_OK) {
        delete c;
        return gvrt_fail(nullptr, GVRT_ERR_OOM, "stats alloc");
    }
    *out = c;
    return GVRT_OK;
}

gvrt_status gvrt_destroy(gvrt_handle c) {
    if (!c) return GVRT_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    std::vector<void*> ptrs;
    for (auto& kv : c->allocs) ptrs.push_back(kv.first);
    for (void* p : ptrs) (void)hipFree(p);
    c->allocs.clear();
    for (hipEvent_t e : c->async_ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->cam_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->h_viewinv_pin) (void)hipHostFree(c->h_viewinv_pin);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return GVRT_OK;
}

const char* gvrt_last_error(gvrt_handle c) { return c ? c->err.c_str() : g_global_err.c_str(); }

gvrt_status gvrt_load_splats(gvrt_handle c, const gvrt_splats* s) {
    if (!c || !s) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL argument");
    if (s->n && (!s->positions || !s->f_dc || !s->f_rest || !s->opacity || !s->scale || !s->rotation))
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL splat array");
    if (s->n > 0xFFFFFFFFull) return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "more than 2^32-1 splats");
    GVRT_HIP(c, hipSetDevice(c->device));
    gvrt_dfree(c, (void**)&c->d_pos);
    gvrt_dfree(c, (void**)&c->d_rot);
    gvrt_dfree(c, (void**)&c->d_scl);
    gvrt_dfree(c, (void**)&c->d_opa);
    gvrt_dfree(c, (void**)&c->d_fdc);
    gvrt_dfree(c, (void**)&c->d_frest);
    c->enclosed = false;
    c->accel = false;
    c->m = 0;
    c->n = 0;  // the handle holds no splats until every buffer below exists
    c->stats.n_input = 0;
    const uint64_t n = s->n;
    gvrt_status st = GVRT_OK;
    float** bufs[6] = {&c->d_pos, &c->d_rot, &c->d_scl, &c->d_opa, &c->d_fdc, &c->d_frest};
    const uint64_t bytes[6] = {12 * n, 16 * n, 12 * n, 4 * n, 12 * n, 180 * n + 360};
    for (int i = 0; i < 6 && st == GVRT_OK; ++i) st = gvrt_dalloc(c, (void**)bufs[i], bytes[i]);
    if (st != GVRT_OK) {  // no half-loaded state: a later build sees "not loaded", never a short buffer
        std::string msg = c->err;
        for (float** b : bufs) gvrt_dfree(c, (void**)b);
        return gvrt_fail(c, st, msg);
    }
    if (n) {
        GVRT_HIP(c, hipMemcpyAsync(c->d_pos, s->positions, 12 * n, hipMemcpyHostToDevice, c->stream));
        GVRT_HIP(c, hipMemcpyAsync(c->d_rot, s->rotation, 16 * n, hipMemcpyHostToDevice, c->stream));
        GVRT_HIP(c, hipMemcpyAsync(c->d_scl, s->scale, 12 * n, hipMemcpyHostToDevice, c->stream));
        GVRT_HIP(c, hipMemcpyAsync(c->d_opa, s->opacity, 4 * n, hipMemcpyHostToDevice, c->stream));
        GVRT_HIP(c, hipMemcpyAsync(c->d_fdc, s->f_dc, 12 * n, hipMemcpyHostToDevice, c->stream));
        GVRT_HIP(c, hipMemcpyAsync(c->d_frest, s->f_rest, 180 * n, hipMemcpyHostToDevice, c->stream));
    }
    GVRT_HIP(c, hipMemsetAsync(reinterpret_cast<char*>(c->d_frest) + 180 * n, 0, 360, c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    c->n = n;
    c->stats.n_input = n;
    return GVRT_OK;
}

gvrt_status gvrt_build_enclosing(gvrt_handle c, const gvrt_enclosing_params* p, uint64_t* m) {
    if (!c) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL handle");
    gvrt_enclosing_params def;
    gvrt_default_enclosing_params(&def);
    if (!p) p = &def;
    if (!c->d_pos || !c->d_rot || !c->d_scl || !c->d_opa || !c->d_fdc || !c->d_frest)
        return gvrt_fail(c, GVRT_ERR_STATE, "gvrt_load_splats has not been called");
    GVRT_HIP(c, hipSetDevice(c->device));
    uint64_t mm = 0;
    gvrt_status s = gvrt_launch_enclose(c, p, &mm);
    if (s) return s;
    c->enc = *p;
    c->m = mm;
    c->enclosed = true;
    c->accel = false;
    c->stats.n_survivors = mm;
    if (m) *m = mm;
    return GVRT_OK;
}

gvrt_status gvrt_read_enclosing(gvrt_handle c, float* density12, float* sh48, float* verts36, uint32_t* tris60,
                                uint32_t* src_index) {
    if (!c) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL handle");
    if (!c->enclosed) return gvrt_fail(c, GVRT_ERR_STATE, "enclosing pass has not run");
    GVRT_HIP(c, hipSetDevice(c->device));
    const uint64_t m = c->m;
    if ((verts36 || tris60) && !c->enc.emit_triangles)
        return gvrt_fail(c, GVRT_ERR_STATE, "triangles requested but emit_triangles was 0");
    if (m) {
        if (density12) GVRT_HIP(c, hipMemcpyAsync(density12, c->d_density12, 48 * m, hipMemcpyDeviceToHost, c->stream));
        if (sh48) GVRT_HIP(c, hipMemcpyAsync(sh48, c->d_sh48, 192 * m, hipMemcpyDeviceToHost, c->stream));
        if (verts36) GVRT_HIP(c, hipMemcpyAsync(verts36, c->d_verts, 144 * m, hipMemcpyDeviceToHost, c->stream));
        if (tris60) GVRT_HIP(c, hipMemcpyAsync(tris60, c->d_tris, 240 * m, hipMemcpyDeviceToHost, c->stream));
        if (src_index) GVRT_HIP(c, hipMemcpyAsync(src_index, c->d_src, 4 * m, hipMemcpyDeviceToHost, c->stream));
    }
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    return GVRT_OK;
}

void gvrt_default_accel_params(gvrt_accel_params* p) {
    if (!p) return;
    *p = gvrt_accel_params{};
}

gvrt_status gvrt_build_accel_ex(gvrt_handle c, const gvrt_accel_params* p) {
    if (!c) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL handle");
    if (!c->enclosed) return gvrt_fail(c, GVRT_ERR_STATE, "gvrt_build_enclosing has not been called");
    gvrt_accel_params d;
    gvrt_default_accel_params(&d);
    if (!p) p = &d;
    if (p->split_cells > 1023) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "split_cells must be <= 1023");
    if (p->builder > 3)
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG,
                         "builder must be 0 (LBVH), 1 (PLOC), 2 (binned SAH, device) or 3 (binned SAH, host)");
    if (p->collapse > 1) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "collapse must be 0 (greedy) or 1 (SAH-optimal DP)");
    if (p->split_min_span > 1023)
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "split_min_span must be at most 1023");
    if (p->depth_budget > gvrt::SAH_DEPTH_MAX)
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "depth_budget must be 0 (default) or at most 43");
    GVRT_HIP(c, hipSetDevice(c->device));
    c->okrecs_valid[0] = c->okrecs_valid[1] = false;
    c->okrecs_full[0] = c->okrecs_full[1] = false;
    c->recs_cams_ok = false;
    c->okrecs_nomem = c->recs_cams_nomem = false;
    c->leaf_hk_ok = false;
    gvrt_dfree(c, (void**)&c->d_leaf_hk);
    gvrt_dfree(c, (void**)&c->d_nodes4x8);
    gvrt_dfree(c, (void**)&c->d_nodes4e);
    gvrt_dfree(c, (void**)&c->d_nodes4ex8);
    c->accept_ok = false;
    c->accept_nomem = false;
    gvrt_status s = gvrt_launch_build_accel(c, *p);
    if (s) return s;
    if ((s = gvrt_launch_node_octants(c))) return s;
    // adaptive enclosing: each leaf's icosahedron half-width, a required array allocated with the build (a render
    // never allocates it, so a handle that builds also renders without a new out-of-memory point)
    if ((c->enc.opts & 1u) && c->n_leaves) {
        if ((s = gvrt_dalloc(c, (void**)&c->d_leaf_hk, 4 * c->n_leaves))) return s;
        if ((s = gvrt_launch_leaf_hk(c))) return s;
        c->leaf_hk_ok = true;
    }
    return GVRT_OK;
}

gvrt_status gvrt_build_accel(gvrt_handle c) { return gvrt_build_accel_ex(c, nullptr); }

gvrt_status gvrt_get_device_properties(int device, gvrt_device_properties* out) {
    if (!out) return gvrt_fail(nullptr, GVRT_ERR_INVALID_ARG, "out is NULL");
    std::memset(out, 0, sizeof(*out));
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return gvrt_fail(nullptr, GVRT_ERR_NO_DEVICE, "no HIP device available");
    }
    if (device < 0 || device >= n) return gvrt_fail(nullptr, GVRT_ERR_INVALID_ARG, "device index out of range");
    hipDeviceProp_t prop{};
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return gvrt_hip_check(nullptr, e, "hipGetDeviceProperties");
    std::snprintf(out->device_name, sizeof(out->device_name), "%s", prop.name);
    std::snprintf(out->arch_name, sizeof(out->arch_name), "%s", prop.gcnArchName);
    out->compute_units = (uint32_t)prop.multiProcessorCount;
    out->total_memory = (uint64_t)prop.totalGlobalMem;
    int drv = 0;
    if (hipDriverGetVersion(&drv) == hipSuccess) out->driver_version = (uint32_t)drv;
    return GVRT_OK;
}

gvrt_status gvrt_read_accel(gvrt_handle c, int which, void* out, uint64_t cap, uint64_t* count) {
    if (!c || !count) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL argument");
    if (which < 0 || which > 2)
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "which must be 0 (binary), 1 (4-wide) or 2 (leaf half-widths)");
    if (!c->accel) return gvrt_fail(c, GVRT_ERR_STATE, "gvrt_build_accel has not been called");
    const uint64_t n = which == 0   ? (c->n_leaves > 1 ? c->n_leaves - 1 : 0)
                       : which == 1 ? c->n_nodes4
                                    : (c->leaf_hk_ok ? c->n_leaves : 0);
    const void* src = which == 0 ? (const void*)c->d_nodes : which == 1 ? (const void*)c->d_nodes4 : (const void*)c->d_leaf_hk;
    const uint64_t sz = which == 0 ? sizeof(gvrt::BvhNode) : which == 1 ? sizeof(gvrt::Bvh4Node) : sizeof(float);
    *count = n;
    if (!out || !n) return GVRT_OK;
    if (!src) return gvrt_fail(c, GVRT_ERR_STATE, "tree not kept by this build");
    GVRT_HIP(c, hipSetDevice(c->device));
    GVRT_HIP(c, hipMemcpyAsync(out, src, sz * (cap < n ? cap : n), hipMemcpyDeviceToHost, c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    return GVRT_OK;
}

gvrt_status gvrt_get_device_buffers(gvrt_handle c, gvrt_device_buffers* out) {
    if (!c || !out) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL argument");
    std::memset(out, 0, sizeof(*out));
    out->n = c->n;
    out->positions = c->d_pos;
    out->rotations = c->d_rot;
    out->scales = c->d_scl;
    out->densities = c->d_opa;
    out->features_albedo = c->d_fdc;
    out->features_specular = c->d_frest;
    if (c->enclosed) {
        out->m = c->m;
        out->particle_density = c->d_density12;
        out->particle_sph = c->d_sh48;
        if (c->enc.emit_triangles) {
            out->vertices = c->d_verts;
            out->indices = c->d_tris;
        }
    }
    return GVRT_OK;
}

gvrt_status gvrt_set_option(gvrt_handle c, uint32_t option, int64_t value) {
    if (!c) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL handle");
    if (option >= GVRT_OPT_COUNT) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "unknown option");
    const int64_t vmax = option == GVRT_OPT_ORDER_SPREAD ? 8 : (option == GVRT_OPT_OPTIONAL_MEM_MB ? (1ll << 40) : 1);
    if (value < 0 || value > vmax)
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG,
                         option == GVRT_OPT_ORDER_SPREAD       ? "order spread is 0..8 tiles"
                         : option == GVRT_OPT_OPTIONAL_MEM_MB ? "optional memory limit is 0..2^40 MiB"
                                                              : "option values are 0 or 1");
    if (c->opt[option] == value) return GVRT_OK;
    GVRT_HIP(c, hipSetDevice(c->device));
    if (c->async_pending) GVRT_HIP(c, hipStreamSynchronize(c->stream));  // queued launches used the old value
    c->opt[option] = value;
    if (option == GVRT_OPT_TILE_ORDER || option == GVRT_OPT_TILE_XCD) c->ord_key = 0;  // the order starts over
    return GVRT_OK;
}

gvrt_status gvrt_get_option(gvrt_handle c, uint32_t option, int64_t* value) {
    if (!c || !value) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL argument");
    if (option >= GVRT_OPT_COUNT) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "unknown option");
    *value = c->opt[option];
    return GVRT_OK;
}

static gvrt_status finish_async(gvrt_context* c);

gvrt_status gvrt_read_tile_costs(gvrt_handle c, uint8_t* out, uint64_t n) {
    if (!c || !out) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL argument");
    if (!c->d_tbucket || c->ord_key == 0 || !c->ord_ready)
        return gvrt_fail(c, GVRT_ERR_STATE, "no cost-ordered launch has run");
    if (n != c->ord_n) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "n is not the tile count of the last ordered launch");
    GVRT_HIP(c, hipSetDevice(c->device));
    if (c->async_pending || c->async_drained) {
        gvrt_status s = finish_async(c);
        if (s) return s;
    }
    std::vector<uint8_t> cls(n);
    GVRT_HIP(c, hipMemcpyAsync(cls.data(), c->d_tbucket, n, hipMemcpyDeviceToHost, c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    if (c->ord_list.empty() && c->h_tcode.size() == n) {
        // full frame: list position i holds tile h_tcode[i] (cam << 24 | ty << 12 | tx)
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t t = c->h_tcode[i];
            const uint64_t cam = t >> 24, ty = (t >> 12) & 0xFFFu, tx = t & 0xFFFu;
            out[(cam * c->ord_ty + ty) * c->ord_tx + tx] = cls[i];
        }
    } else {
        std::memcpy(out, cls.data(), n);
    }
    return GVRT_OK;
}

gvrt_status gvrt_set_stats(gvrt_handle c, int enable) {
    if (!c) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL handle");
    c->stats_on = enable != 0;
    return GVRT_OK;
}

gvrt_status gvrt_get_stats(gvrt_handle c, gvrt_stats* s) {
    if (!c || !s) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL argument");
    c->stats.device_bytes = c->device_bytes;
    *s = c->stats;
    return GVRT_OK;
}

static gvrt_status ensure(gvrt_context* c, void** p, uint64_t* cap, uint64_t bytes) {
    if (*cap >= bytes && *p) return GVRT_OK;
    gvrt_dfree(c, p);
    *cap = 0;
    gvrt_status s = gvrt_dalloc(c, p, bytes);
    if (s) return s;
    *cap = bytes;
    return GVRT_OK;
}

// Stream-ordered completion of the async launches queued so far: their kernel times (HIP events) are
// folded into a running sum, and the event pairs are free for reuse.
static gvrt_status drain_async(gvrt_context* c) {
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    for (uint32_t k = 0; k < c->async_pending; ++k) {
        float ms = 0.f;
        GVRT_HIP(c, hipEventElapsedTime(&ms, c->async_ev[2 * k], c->async_ev[2 * k + 1]));
        c->async_ms_sum += ms;
    }
    c->async_drained += c->async_pending;
    c->async_pending = 0;
    return GVRT_OK;
}

// gvrt_sync: every async launch since the previous sync completed; stats.render_ms = their mean kernel time
static gvrt_status finish_async(gvrt_context* c) {
    gvrt_status s;
    if ((s = drain_async(c))) return s;
    if (c->async_drained) c->stats.render_ms = (float)(c->async_ms_sum / (double)c->async_drained);
    c->async_ms_sum = 0.0;
    c->async_drained = 0;
    return GVRT_OK;
}

// a queue deeper than this many launches waits for the queued ones first (bounds the event pool)
constexpr uint32_t MAX_ASYNC_PENDING = 1024;

// Encode a caller tile list (cam << 24 | ty << 12 | tx) and upload it only when it differs from what the
// device buffer already holds: a static split (the multi-GPU tile list) then costs no host round trip per
// frame, so frames queue back to back.  A changed list waits for queued launches first (they may read the
// buffer, and the host copy is the source of the pageable upload).
static gvrt_status upload_tile_list(gvrt_context* c, const gvrt_tile* tiles, uint64_t ntiles, uint32_t tiles_x,
                                    uint32_t tiles_y, uint32_t ncams, std::vector<uint32_t>& host, uint32_t** dev,
                                    uint64_t* cap, bool& valid) {
    std::vector<uint32_t> tl(ntiles);
    for (uint64_t i = 0; i < ntiles; ++i) {
        if (tiles[i].tx >= tiles_x || tiles[i].ty >= tiles_y || tiles[i].cam >= ncams)
            return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "tile outside the image");
        tl[i] = ((uint32_t)tiles[i].cam << 24) | ((uint32_t)tiles[i].ty << 12) | tiles[i].tx;
    }
    if (valid && tl == host) return GVRT_OK;
    if (c->async_pending) GVRT_HIP(c, hipStreamSynchronize(c->stream));
    valid = false;
    host.swap(tl);
    gvrt_status s;
    if ((s = ensure(c, (void**)dev, cap, 4 * (ntiles ? ntiles : 1)))) return s;
    if (ntiles) GVRT_HIP(c, hipMemcpyAsync(*dev, host.data(), 4 * ntiles, hipMemcpyHostToDevice, c->stream));
    valid = true;
    return GVRT_OK;
}

// Cost-ordered dispatch.  A tile's render time varies ~4x across the frame (scene depth complexity), and
// with the default row-major supertile order the costly tiles that start last set a tail of ~27 % over a
// perfectly balanced schedule (list-scheduling model on measured per-tile cycles).  Each
// launch records every tile's cost class (log2 of its wave's cycles, 4 classes per octave); one small
// kernel after it orders the tiles costliest class first, and the next launch of the same frame size
// dispatches them in that order.  The order changes only which wave renders a tile when, never a pixel.
// GVRT_OPT_TILE_ORDER = 0 turns it off.

// Arrays of the order for a launch of n tile-list entries: kept while the frame size and the tile list stay
// the same (list == null: a full frame, whose list is every tile in supertile order), reset otherwise.
static gvrt_status ensure_tile_order(gvrt_context* c, uint32_t tiles_x, uint32_t tiles_y, uint32_t ncams,
                                     const std::vector<uint32_t>* list) {
    const uint64_t key = (uint64_t)tiles_x | ((uint64_t)tiles_y << 16) | ((uint64_t)ncams << 32) |
                         (list ? 0ull : (1ull << 63));
    if (c->ord_key == key && c->d_tbucket && (!list || *list == c->ord_list)) return GVRT_OK;
    GVRT_HIP(c, hipStreamSynchronize(c->stream));  // queued launches may still read the old arrays (and
                                                    // the previous list's upload may still read h_tcode)
    gvrt_dfree(c, (void**)&c->d_tbucket);
    gvrt_dfree(c, (void**)&c->d_tbucket2);
    gvrt_dfree(c, (void**)&c->d_tgrid);
    gvrt_dfree(c, (void**)&c->d_thist);
    gvrt_dfree(c, (void**)&c->d_tcode);
    gvrt_dfree(c, (void**)&c->d_order);
    c->ord_ready = false;
    c->ord_key = 0;
    c->ord_list.clear();
    const uint64_t n = list ? list->size() : (uint64_t)tiles_x * tiles_y * ncams;
    if (n == 0) return GVRT_OK;
    gvrt_status s;
    if ((s = gvrt_dalloc(c, (void**)&c->d_tbucket, n))) return s;
    if ((s = gvrt_dalloc(c, (void**)&c->d_tbucket2, n))) return s;
    if ((s = gvrt_dalloc(c, (void**)&c->d_tgrid, (uint64_t)tiles_x * tiles_y * ncams))) return s;
    if ((s = gvrt_dalloc(c, (void**)&c->d_thist, 4 * 5 * TILE_BUCKETS))) return s;
    if ((s = gvrt_dalloc(c, (void**)&c->d_order, 4 * n))) return s;
    if (!list) {
        // the full frame as a tile list in the render kernel's supertile order (its first launch's order)
        if ((s = gvrt_dalloc(c, (void**)&c->d_tcode, 4 * n))) return s;
        std::vector<uint32_t>& code = c->h_tcode;  // kept: the source of the stream-ordered upload below
        code.clear();
        code.reserve(n);
        const uint32_t STW = 8, STH = 4;  // as GVRT_ST_W / GVRT_ST_H of gvrt_render.hip
        for (uint32_t cam = 0; cam < ncams; ++cam)
            for (uint32_t sy = 0; sy < tiles_y; sy += STH)
                for (uint32_t sx = 0; sx < tiles_x; sx += STW)
                    for (uint32_t ty = sy; ty < std::min(sy + STH, tiles_y); ++ty)
                        for (uint32_t tx = sx; tx < std::min(sx + STW, tiles_x); ++tx)
                            code.push_back((cam << 24) | (ty << 12) | tx);
        GVRT_HIP(c, hipMemcpyAsync(c->d_tcode, code.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
    } else {
        c->ord_list = *list;
    }
    GVRT_HIP(c, hipMemsetAsync(c->d_thist, 0, 4 * 5 * TILE_BUCKETS, c->stream));
    c->ord_tx = tiles_x;
    c->ord_ty = tiles_y;
    c->ord_nc = ncams;
    c->ord_prev_valid = false;
    c->ord_parity = 0;
    c->ord_n = n;
    c->ord_key = key;
    return GVRT_OK;
}

// Tiles a screen point may move between two launches (camera 0 of each): the angle between the cameras' axes
// plus the translation seen at the eye's distance to the origin, in pixels
// (H / (2 tan(fovy / 2)) per radian, tan(fovy / 2) = |projInverse[1][1]|), over the 8-pixel tile.  Only a
// scheduling hint (the order never changes a pixel): 0 for a static camera.
static int motion_radius(const float* prev, const float* cur, const float* proj_inv, uint32_t height) {
    float ang = 0.0f;
    for (int k = 0; k < 3; ++k) {
        const float* a = prev + 4 * k;
        const float* b = cur + 4 * k;
        const float na = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        const float nb = std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
        if (!(na > 0.0f) || !(nb > 0.0f)) return 0;
        const float cs = std::min(1.0f, std::max(-1.0f, (a[0] * b[0] + a[1] * b[1] + a[2] * b[2]) / (na * nb)));
        ang = std::max(ang, std::acos(cs));
    }
    const float dx = cur[12] - prev[12], dy = cur[13] - prev[13], dz = cur[14] - prev[14];
    const float dist = std::sqrt(cur[12] * cur[12] + cur[13] * cur[13] + cur[14] * cur[14]);
    const float trans = std::sqrt(dx * dx + dy * dy + dz * dz) / std::max(dist, 1e-3f);
    const float th = std::fabs(proj_inv[5]);
    if (!(th > 0.0f)) return 0;
    const float px = (ang + trans) * (float)height / (2.0f * th);
    if (!(px == px)) return 0;
    return (int)std::min(std::ceil(px / 8.0f), 64.0f);
}

// The camera ring sized for ncams cameras per slot (regrown, after the queued frames, when a launch has more).
static gvrt_status ensure_cameras(gvrt_context* c, uint32_t ncams) {
    if (c->cam_stride >= 16ull * ncams && c->d_viewinv) return GVRT_OK;
    GVRT_HIP(c, hipStreamSynchronize(c->stream));  // queued frames read the old ring
    gvrt_dfree(c, (void**)&c->d_viewinv);
    if (c->h_viewinv_pin) {
        (void)hipHostFree(c->h_viewinv_pin);
        c->h_viewinv_pin = nullptr;
    }
    c->cam_stride = 0;
    c->cam_valid = false;
    for (uint32_t i = 0; i < gvrt_context::CAM_RING; ++i) {
        if (!c->cam_ev[i]) GVRT_HIP(c, hipEventCreateWithFlags(&c->cam_ev[i], hipEventDisableTiming));
        c->cam_ev_live[i] = false;
    }
    const uint64_t stride = 16ull * std::max<uint32_t>(ncams, 4);
    gvrt_status s;
    if ((s = gvrt_dalloc(c, (void**)&c->d_viewinv, 4 * stride * gvrt_context::CAM_RING))) return s;
    GVRT_HIP(c, hipHostMalloc((void**)&c->h_viewinv_pin, 4 * stride * gvrt_context::CAM_RING, hipHostMallocDefault));
    c->cam_stride = stride;
    return GVRT_OK;
}

static gvrt_status render_impl(gvrt_handle c, const gvrt_render_params* p, const float* view_inverse,
                               const float* proj_inverse, uint32_t width, uint32_t height, uint32_t ncams,
                               const gvrt_tile* tiles, uint64_t ntiles, const gvrt_image* out, bool async) {
    if (!c) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL handle");
    if (async && out && !out->device_ptrs)
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "gvrt_render_async needs device output pointers");
    if (async && c->stats_on) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "stats need the synchronous gvrt_render");
    if (!view_inverse || !proj_inverse || !out) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL argument");
    if (width == 0 || height == 0 || ncams == 0) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "empty image");
    if (width > 32768 || height > 32768 || ncams > 255)
        return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "image larger than 32768^2 or more than 255 cameras");
    if (!c->accel) return gvrt_fail(c, GVRT_ERR_STATE, "gvrt_build_accel has not been called");
    gvrt_render_params def;
    gvrt_default_render_params(&def);
    if (!p) p = &def;
    if (p->mode > GVRT_MODE_LITERAL) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "unknown mode");
    if (p->tmin_inclusive && (p->mode != GVRT_MODE_LITERAL || p->max_rounds == 0))
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG,
                         "tmin_inclusive needs mode LITERAL and max_rounds > 0 (an inclusive tmin re-finds the last "
                         "hit every round and never terminates when it is rejected)");
    if (out->packed && !tiles) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "packed output needs a tile list");
    if (out->packed && out->ray_dirs) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "ray_dirs cannot be packed");
    GVRT_HIP(c, hipSetDevice(c->device));

    const uint32_t tiles_x = (width + 7) / 8, tiles_y = (height + 7) / 8;
    const uint64_t total_tiles = (uint64_t)tiles_x * tiles_y * ncams;
    gvrt_status s;
    RenderArgs a;
    std::memset(&a, 0, sizeof(a));
    a.recs = c->d_recs;
    // split: the k-buffer holds proxy (compaction) ids, shared by the proxy's pieces
    a.crecs = c->d_recs;
    a.sh = c->d_sh;
    a.aux = reinterpret_cast<const uint4*>(c->d_leaf_aux);
    for (int k = 0; k < 3; ++k) a.grid_min[k] = c->grid_min[k];
    a.grid_inv = c->grid_inv;
    a.nodes = c->d_nodes4;
    a.nodes8 = c->opt[GVRT_OPT_OCTANT_NODES] ? c->d_nodes4x8 : nullptr;
    a.nodes8_stride = c->n_nodes4;
    // k-buffer payloads are leaf indices (split pieces included): the packed buffer's 24-bit ids bound the leaves
    a.nrecs = (uint32_t)std::max<uint64_t>(c->m, c->n_leaves);
    // the render kernel addresses leaf records (64 B) and 4-wide nodes (128 B) by 32-bit byte offsets
    if (c->n_leaves >= (1ull << 26) || c->n_nodes4 >= (1ull << 25))
        return gvrt_fail(c, GVRT_ERR_UNSUPPORTED, "more than 2^26 BVH leaves or 2^25 nodes (32-bit record offsets)");
    // cameras: uploaded only when they changed, into the next slot of the device ring, so that a moving camera
    // costs no host round trip per frame.  The outgoing slot's event is recorded when the camera changes (after
    // every queued launch that read it), so a static camera records none; a slot's event is waited for only when
    // the ring comes round to it with its readers still queued (CAM_RING camera changes deep)
    if ((s = ensure_cameras(c, ncams))) return s;
    float* cam_pending = nullptr;  // one camera's ring slot still to be written
    struct CamGuard {  // a return before the slot is written: the next launch uploads the camera again
        gvrt_context* c;
        float* const* p;
        ~CamGuard() {
            if (*p) c->cam_valid = false;
        }
    } cam_guard{c, &cam_pending};
    if (!c->cam_valid || c->h_viewinv.size() != 16ull * ncams ||
        std::memcmp(c->h_viewinv.data(), view_inverse, 64ull * ncams) != 0) {
        if (c->cam_valid) {
            GVRT_HIP(c, hipEventRecord(c->cam_ev[c->cam_slot], c->stream));
            c->cam_ev_live[c->cam_slot] = true;
        }
        const uint32_t slot = (c->cam_slot + 1) % gvrt_context::CAM_RING;
        if (c->cam_ev_live[slot]) GVRT_HIP(c, hipEventSynchronize(c->cam_ev[slot]));
        if (ncams == 1) {
            // written by this launch's k_rec_origin pass when it has one (a moving camera), else copied below
            cam_pending = c->d_viewinv + slot * c->cam_stride;
        } else {
            float* src = c->h_viewinv_pin + slot * c->cam_stride;
            std::memcpy(src, view_inverse, 64ull * ncams);
            GVRT_HIP(c, hipMemcpyAsync(c->d_viewinv + slot * c->cam_stride, src, 64ull * ncams,
                                       hipMemcpyHostToDevice, c->stream));
        }
        c->h_viewinv.assign(view_inverse, view_inverse + 16ull * ncams);
        c->cam_slot = slot;
        c->cam_valid = true;
    }
    a.view_inv = c->d_viewinv + c->cam_slot * c->cam_stride;
    std::memcpy(a.proj_inv, proj_inverse, 64);
    std::memcpy(a.aabb, p->aabb, 24);
    a.min_transmittance = p->min_transmittance;
    a.min_response = p->hit_min_gaussian_response;
    a.alpha_min = p->alpha_min;
    a.pixel_offset = p->pixel_offset;
    a.alpha_init = p->alpha_init;
    a.kmin = c->enc.kernel_min_response;
    a.kdeg = c->enc.degree;
    a.kopts = c->enc.opts;
    a.kernel_h = kernel_scale(1.0f, a.kmin, a.kopts & ~1u, a.kdeg) * SQRT3;
    a.sph_deg = p->sph_eval_degree;
    // gres > r  <=>  gd^2 < ln(r)/S (S < 0); r <= 0 accepts everything, r >= 1 nothing
    {
        const double r = p->hit_min_gaussian_response;
        a.gpre = r <= 0.0 ? INFINITY : (r >= 1.0 ? 0.0f : (float)(std::sqrt(std::log(r) / (double)KERNEL_S) * 1.001));
    }
    a.width = width;
    a.height = height;
    a.ncams = ncams;
    a.tiles_x = tiles_x;
    a.tiles_y = tiles_y;
    a.tmin_inclusive = p->tmin_inclusive;
    a.max_rounds = p->max_rounds;
    a.ray_dirs_layout = p->ray_dirs_layout;
    a.packed = out->packed;
    // no per-child box slack when the absolute box padding covers the plane rounding for every camera of
    // the launch (|origin component| <= 4 x the scene's position bound; split pieces keep the slack)
    {
        float omax = 0.0f;
        for (uint32_t i = 0; i < ncams; ++i)
            for (int k = 12; k < 15; ++k) omax = std::max(omax, std::fabs(view_inverse[16ull * i + k]));
        a.box_exact = c->opt[GVRT_OPT_BOX_SLACK] == 0 && c->box_pad_abs > 0.0f &&
                      std::ldexp(omax, -20) <= c->box_pad_abs;  // also false for a NaN origin
    }
    a.kfast = p->kbuffer_depth ? p->kbuffer_depth : (uint32_t)K_FAST_DEFAULT;
    // adaptive enclosing: the per-leaf icosahedron half-widths, written with the build (gvrt_build_accel_ex)
    if ((c->enc.opts & 1u) && c->n_leaves) {
        if (!c->leaf_hk_ok) return gvrt_fail(c, GVRT_ERR_STATE, "adaptive enclosing without per-leaf half-widths");
        a.leaf_hk = c->d_leaf_hk;
    }
    // FAST launches traverse the acceptance-box nodes (gvrt_launch_accept_nodes), refit when the acceptance
    // thresholds change; LITERAL launches keep every crossing and so the proxy boxes.  A negative alphaMin keeps the
    // proxy boxes too: a particle of density rho <= alphaMin < 0 is then accepted in a shell (min(0.99, gres rho) >
    // alphaMin for small gres), not inside a ball, so neither its acceptance ball nor its drop would be exact
    if (p->mode == GVRT_MODE_FAST && c->opt[GVRT_OPT_ACCEPT_BOXES] && p->alpha_min >= 0.0f &&
        (p->hit_min_gaussian_response > 0.0f || p->alpha_min > 0.0f) && a.nrecs < 0xFFFFFFu &&
        c->opt[GVRT_OPT_PACKED_KBUFFER]) {
        if (!c->accept_ok || c->accept_key[0] != p->hit_min_gaussian_response || c->accept_key[1] != p->alpha_min)
            if ((s = gvrt_launch_accept_nodes(c, p->hit_min_gaussian_response, p->alpha_min))) return s;
        if (c->accept_ok) {
            a.nodes = c->d_nodes4e;
            a.nodes8 = c->opt[GVRT_OPT_OCTANT_NODES] ? c->d_nodes4ex8 : nullptr;
        }
    }
    // Single-origin FAST launches at the default depth read each leaf's kernel-frame origin ok from its record:
    // one pass per launch writes ok = S^-1 R^T (o - p) in place of the position (k_rec_origin), instead of
    // every leaf visit and composited hit of every wave recomputing it.  Other launches get the positions back.
    {
        bool one_origin = true;
        for (uint32_t i = 1; i < ncams && one_origin; ++i)
            one_origin = std::memcmp(view_inverse + 16ull * i + 12, view_inverse + 12, 12) == 0;
        const bool adaptive = (c->enc.opts & 1u) != 0;
        const bool okbase = c->opt[GVRT_OPT_RECORD_ORIGINS] && p->mode == GVRT_MODE_FAST &&
                            a.kfast == (uint32_t)K_FAST_DEFAULT && !adaptive && a.nrecs < 0xFFFFFFu &&
                            c->opt[GVRT_OPT_PACKED_KBUFFER] && c->n_leaves;
        a.okrec = okbase && one_origin;
        const uint64_t cams_bytes = (uint64_t)ncams * c->n_leaves * sizeof(RenderRec);
        // (the copies are an optional speed-up: one that does not fit leaves the launch on d_recs, okrec = 0, until
        // the next build)
        bool cams_ready = false;
        if (okbase && !one_origin && ncams <= 16 && cams_bytes <= (8ull << 30) && !c->recs_cams_nomem) {
            // several origins (a light-field rig): one record copy per camera, written when the set of origins
            // changes (a static rig: once), and camera c's waves read copy c (RenderArgs::recs_cam_stride)
            std::vector<float> org(3ull * ncams);
            for (uint32_t i = 0; i < ncams; ++i)
                for (int k = 0; k < 3; ++k) org[3ull * i + k] = view_inverse[16ull * i + 12 + k];
            cams_ready = c->recs_cams_ok && c->recs_cams_origins == org;
            if (!cams_ready) {
                if (c->recs_cams_bytes < cams_bytes) {
                    if (c->d_recs_cams) GVRT_HIP(c, hipStreamSynchronize(c->stream));  // queued launches read it
                    gvrt_dfree(c, (void**)&c->d_recs_cams);
                    c->recs_cams_bytes = 0;
                    c->recs_cams_ok = false;
                    if (gvrt_dalloc_optional(c, (void**)&c->d_recs_cams, cams_bytes)) c->recs_cams_bytes = cams_bytes;
                    else c->recs_cams_nomem = true;
                }
                if (!c->recs_cams_nomem) {
                    if ((s = gvrt_launch_rec_cams(c, ncams, a.view_inv, c->d_recs_cams))) return s;
                    c->recs_cams_origins = org;
                    c->recs_cams_ok = true;
                    cams_ready = true;
                }
            }
        }
        if (a.okrec && !c->okrecs_nomem && (c->okrecs_n != c->n_leaves || !c->d_okrecs[0])) {
            GVRT_HIP(c, hipStreamSynchronize(c->stream));
            for (int j = 0; j < 2; ++j) {
                gvrt_dfree(c, (void**)&c->d_okrecs[j]);
                c->okrecs_valid[j] = false;
                c->okrecs_full[j] = false;
            }
            c->okrecs_n = 0;
            bool ok = true;
            for (int j = 0; j < 2 && ok; ++j)
                ok = gvrt_dalloc_optional(c, (void**)&c->d_okrecs[j], c->n_leaves * sizeof(RenderRec));
            if (ok) {
                c->okrecs_n = c->n_leaves;
            } else {
                for (int j = 0; j < 2; ++j) gvrt_dfree(c, (void**)&c->d_okrecs[j]);
                c->okrecs_nomem = true;
            }
        }
        if (c->okrecs_nomem) a.okrec = 0;
        if (cams_ready) {
            a.okrec = 1;
            a.recs = c->d_recs_cams;
            a.crecs = c->d_recs_cams;
            a.recs_cam_stride = c->n_leaves;
        } else if (a.okrec) {
            // a copy already holding this origin's kernel-frame origins (a static camera, the frames of one view,
            // or a camera coming back): no pass
            int k = -1;
            for (int j = 0; j < 2; ++j)
                if (c->okrecs_valid[j] && c->okrecs_n == c->n_leaves &&
                    std::memcmp(c->okrecs_origin[j], view_inverse + 12, 12) == 0)
                    k = j;
            if (k < 0) {
                // the copy not used by the latest launch, rewritten in stream order (after its queued readers);
                // a side stream overlapping the pass with the previous frame measured slower
                k = c->okrecs_valid[c->okrecs_cur] ? 1 - c->okrecs_cur : c->okrecs_cur;
                if ((s = gvrt_launch_rec_origin(c, view_inverse + 12, c->d_okrecs[k], c->stream, cam_pending,
                                                view_inverse, c->okrecs_full[k])))
                    return s;
                cam_pending = nullptr;
                c->okrecs_full[k] = true;
                std::memcpy(c->okrecs_origin[k], view_inverse + 12, 12);
                c->okrecs_valid[k] = true;
            }
            c->okrecs_cur = k;
            a.recs = c->d_okrecs[k];
            a.crecs = c->d_okrecs[k];
        }
    }
    if (cam_pending) {
        float* src = c->h_viewinv_pin + (uint64_t)(cam_pending - c->d_viewinv);
        std::memcpy(src, view_inverse, 64);
        GVRT_HIP(c, hipMemcpyAsync(cam_pending, src, 64, hipMemcpyHostToDevice, c->stream));
        cam_pending = nullptr;
    }
    if (a.kfast != 8 && a.kfast != 12 && a.kfast != 16 && a.kfast != 20 && a.kfast != 24 && a.kfast != 32)
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "kbuffer_depth must be 0, 8, 12, 16, 20, 24 or 32");
    uint64_t nwork = total_tiles;
    if (tiles) {
        if ((s = upload_tile_list(c, tiles, ntiles, tiles_x, tiles_y, ncams, c->h_tiles, &c->d_tiles, &c->tiles_cap,
                                  c->tiles_valid)))
            return s;
        a.tiles = c->d_tiles;
        nwork = ntiles;
    }
    // cost-ordered dispatch: full frames and caller tile lists alike (the kernel renders list position
    // perm[i] in workgroup i; outputs stay where the list puts them)
    const bool ordered = c->opt[GVRT_OPT_TILE_ORDER] != 0 && nwork > 0;
    int ord_radius = 0;  // moving camera: spread of the previous launch's tile costs (motion_radius)
    if (ordered) {
        if ((s = ensure_tile_order(c, tiles_x, tiles_y, ncams, tiles ? &c->h_tiles : nullptr))) return s;
        if (c->ord_prev_valid) ord_radius = motion_radius(c->ord_prev_vi, view_inverse, proj_inverse, height);
        ord_radius = std::max(ord_radius, (int)c->opt[GVRT_OPT_ORDER_SPREAD]);
        std::memcpy(c->ord_prev_vi, view_inverse, 64);
        c->ord_prev_valid = true;
        if (!tiles) a.tiles = c->d_tcode;
        a.tile_bucket = c->d_tbucket;
        a.tile_hist = c->d_thist + TILE_BUCKETS * c->ord_parity;
        // a camera that moved by more than 12 tiles in one frame: the previous costs say little, supertile order
        if (c->ord_ready && ord_radius <= 12) a.perm = c->d_order;
    }
    a.ntiles = nwork;
    const uint64_t npix = out->packed ? nwork * 64 : (uint64_t)width * height * ncams;

    // outputs: device pointers used directly; host pointers staged
    const uint64_t b8 = out->rgba8 ? 4 * npix : 0;
    const uint64_t b32 = out->rgba32f ? 16 * npix : 0;
    const uint64_t bdir = out->ray_dirs ? 16ull * width * height * ncams : 0;
    const uint64_t bhc = out->hit_counts ? 4 * npix : 0;
    if (out->device_ptrs) {
        a.rgba8 = (uint8_t*)out->rgba8;
        a.rgba32f = out->rgba32f;
        a.ray_dirs = out->ray_dirs;
        a.hit_counts = out->hit_counts;
    } else {
        const uint64_t total = b8 + b32 + bdir + bhc;
        if ((s = ensure(c, &c->d_stage, &c->stage_cap, total ? total : 16))) return s;
        char* base = (char*)c->d_stage;
        uint64_t off = 0;
        if (b32) { a.rgba32f = (float*)(base + off); off += b32; }
        if (bdir) { a.ray_dirs = (float*)(base + off); off += bdir; }
        if (bhc) { a.hit_counts = (uint32_t*)(base + off); off += bhc; }
        if (b8) { a.rgba8 = (uint8_t*)(base + off); off += b8; }
        if (!out->packed && tiles) {
            // pixels outside the tile list keep zeros
            GVRT_HIP(c, hipMemsetAsync(base, 0, total, c->stream));
        }
    }
    if (c->stats_on) {
        GVRT_HIP(c, hipMemsetAsync(c->d_stats, 0, 104, c->stream));
        a.stats = c->d_stats;
    }
    if (async) {
        // one event pair per queued launch, reused after every drain
        if (c->async_pending >= MAX_ASYNC_PENDING && (s = drain_async(c))) return s;
        if (2 * (c->async_pending + 1) > c->async_ev.size()) {
            for (int k = 0; k < 2; ++k) {
                hipEvent_t e = nullptr;
                GVRT_HIP(c, hipEventCreate(&e));
                c->async_ev.push_back(e);
            }
        }
        hipEvent_t e0 = c->async_ev[2 * c->async_pending], e1 = c->async_ev[2 * c->async_pending + 1];
        if ((s = gvrt_launch_render_mode(c, a, nwork, p->mode == GVRT_MODE_LITERAL, e0, e1))) return s;
        if (ordered && (s = gvrt_launch_tile_order(c, a.tiles, std::min(ord_radius, 8)))) return s;
        ++c->async_pending;
        c->stats.rays = (tiles || out->packed) ? nwork * 64 : total_tiles * 64;
        return GVRT_OK;
    }
    if ((c->async_pending || c->async_drained) && (s = finish_async(c))) return s;
    if ((s = gvrt_launch_render_mode(c, a, nwork, p->mode == GVRT_MODE_LITERAL, c->ev0, c->ev1))) return s;
    if (ordered && (s = gvrt_launch_tile_order(c, a.tiles, std::min(ord_radius, 8)))) return s;
    if (!out->device_ptrs) {
        if (b32) GVRT_HIP(c, hipMemcpyAsync(out->rgba32f, a.rgba32f, b32, hipMemcpyDeviceToHost, c->stream));
        if (bdir) GVRT_HIP(c, hipMemcpyAsync(out->ray_dirs, a.ray_dirs, bdir, hipMemcpyDeviceToHost, c->stream));
        if (bhc) GVRT_HIP(c, hipMemcpyAsync(out->hit_counts, a.hit_counts, bhc, hipMemcpyDeviceToHost, c->stream));
        if (b8) GVRT_HIP(c, hipMemcpyAsync(out->rgba8, a.rgba8, b8, hipMemcpyDeviceToHost, c->stream));
    }
    unsigned long long hs[13] = {};
    if (c->stats_on) GVRT_HIP(c, hipMemcpyAsync(hs, c->d_stats, 104, hipMemcpyDeviceToHost, c->stream));
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    float ms = 0.f;
    GVRT_HIP(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->stats.render_ms = ms;
    c->stats.rays = nwork * 64;
    c->stats.crossings = hs[0];
    c->stats.accepted = hs[1];
    c->stats.rounds = hs[2];
    c->stats.wave_node_visits = hs[3];
    c->stats.wave_leaf_visits = hs[4];
    c->stats.lane_leaf_tests = hs[5];
    for (int k = 0; k < 4; ++k) c->stats.phase_cycles[k] = hs[6 + k];
    c->stats.wave_dead_visits = hs[10];
    c->stats.wave_rounds = hs[11];
    c->stats.wave_late_node_visits = hs[12];
    return GVRT_OK;
}

gvrt_status gvrt_render(gvrt_handle c, const gvrt_render_params* p, const float* view_inverse,
                        const float* proj_inverse, uint32_t width, uint32_t height, uint32_t ncams,
                        const gvrt_tile* tiles, uint64_t ntiles, const gvrt_image* out) {
    return render_impl(c, p, view_inverse, proj_inverse, width, height, ncams, tiles, ntiles, out, false);
}

gvrt_status gvrt_render_async(gvrt_handle c, const gvrt_render_params* p, const float* view_inverse,
                              const float* proj_inverse, uint32_t width, uint32_t height, uint32_t ncams,
                              const gvrt_tile* tiles, uint64_t ntiles, const gvrt_image* out) {
    return render_impl(c, p, view_inverse, proj_inverse, width, height, ncams, tiles, ntiles, out, true);
}

gvrt_status gvrt_sync(gvrt_handle c) {
    if (!c) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL handle");
    GVRT_HIP(c, hipSetDevice(c->device));
    return finish_async(c);
}

gvrt_status gvrt_set_stream(gvrt_handle c, void* stream) {
    if (!c) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL handle");
    GVRT_HIP(c, hipSetDevice(c->device));
    gvrt_status s;
    if (c->async_pending && (s = drain_async(c))) return s;  // their kernel times stay counted for gvrt_sync
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    c->stream = stream ? reinterpret_cast<hipStream_t>(stream) : c->own_stream;
    return GVRT_OK;
}

gvrt_status gvrt_unpack_tiles_rgba8(gvrt_handle c, const void* packed, const gvrt_tile* tiles, uint64_t ntiles,
                                    uint32_t width, uint32_t height, uint32_t ncams, void* frame) {
    if (!c || !packed || !tiles || !frame) return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "NULL argument");
    if (width == 0 || height == 0 || width > 32768 || height > 32768 || ncams == 0 || ncams > 255)
        return gvrt_fail(c, GVRT_ERR_INVALID_ARG, "frame must be 1..32768 pixels per side, 1..255 cameras");
    const uint32_t tiles_x = (width + 7) / 8, tiles_y = (height + 7) / 8;
    GVRT_HIP(c, hipSetDevice(c->device));
    gvrt_status s;
    // the cached list equal to this one, else the least recently used of up to UNPACK_LISTS buffers
    constexpr size_t UNPACK_LISTS = 16;
    auto& L = c->unpack_lists;
    size_t pick = L.size();
    for (size_t i = 0; i < L.size(); ++i)
        if (L[i].valid && L[i].host.size() == ntiles) {
            bool same = true;
            for (uint64_t j = 0; j < ntiles && same; ++j)
                same = L[i].host[j] == (((uint32_t)tiles[j].cam << 24) | ((uint32_t)tiles[j].ty << 12) | tiles[j].tx);
            if (same) {
                pick = i;
                break;
            }
        }
    if (pick == L.size()) {
        if (L.size() < UNPACK_LISTS) {
            L.emplace_back();
        } else {
            pick = 0;
            for (size_t i = 1; i < L.size(); ++i)
                if (L[i].used < L[pick].used) pick = i;
        }
    }
    gvrt_context::TileListBuf& b = L[pick];
    b.used = ++c->unpack_calls;
    if ((s = upload_tile_list(c, tiles, ntiles, tiles_x, tiles_y, ncams, b.host, &b.dev, &b.cap, b.valid))) return s;
    if ((s = gvrt_launch_unpack(c, packed, b.dev, ntiles, width, height, frame))) return s;
    // behind queued renders (gvrt_render_async) the unpack is queued too and completes by gvrt_sync
    if (c->async_pending) return GVRT_OK;
    GVRT_HIP(c, hipStreamSynchronize(c->stream));
    return GVRT_OK;
}

}  // extern "C"
