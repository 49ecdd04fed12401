// gvrt_rccl.cpp — RcclBackend: the RCCL / HIP / libgvrt implementation of SplitBackend (gvrt_rccl.h), and the
// communicator rendezvous.
#include "gvrt_rccl.h"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <thread>

namespace gvrt_host {

gvrt_status rccl_rendezvous(const std::string& path, int rank, ncclUniqueId* id, std::string* err, double timeout_s) {
    if (rank == 0) {
        const ncclResult_t r = ncclGetUniqueId(id);
        if (r != ncclSuccess) {
            *err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
            return GVRT_ERR_RCCL;
        }
        const std::string tmp = path + ".tmp";
        {
            std::ofstream f(tmp, std::ios::binary);
            f.write(reinterpret_cast<const char*>(id), sizeof(*id));
            if (!f) {
                *err = "cannot write " + tmp;
                return GVRT_ERR_IO;
            }
        }
        if (std::rename(tmp.c_str(), path.c_str()) != 0) {
            *err = "cannot rename " + tmp;
            return GVRT_ERR_IO;
        }
        return GVRT_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    while (true) {
        std::ifstream f(path, std::ios::binary);
        if (f && f.read(reinterpret_cast<char*>(id), sizeof(*id)) && f.gcount() == (std::streamsize)sizeof(*id))
            return GVRT_OK;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
            *err = "no RCCL id at " + path + " after " + std::to_string(timeout_s) + " s";
            return GVRT_ERR_RCCL;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}

#define STREAM (static_cast<hipStream_t>(stream_))

RcclBackend::RcclBackend(GvrtApp& app, int rank, int world, const ncclUniqueId& id)
    : app_(app), rank_(rank), world_(world), id_(id) {}

RcclBackend::~RcclBackend() {
    (void)hipSetDevice(app_.device.ordinal);
    if (stream_) (void)hipStreamSynchronize(STREAM);
    if (bound_ && app_.handle()) (void)gvrt_set_stream(app_.handle(), nullptr);
    if (comm_) (void)ncclCommDestroy(comm_);
    if (stream_) (void)hipStreamDestroy(STREAM);
}

bool RcclBackend::nccl(ncclResult_t r, const char* what, std::string* err) {
    if (r == ncclSuccess) return true;
    if (err) *err = std::string(what) + ": " + ncclGetErrorString(r);
    return false;
}

gvrt_status RcclBackend::init(bool* comm_ok, std::string* err) {
    *comm_ok = false;
    if (hipSetDevice(app_.device.ordinal) != hipSuccess) {
        *err = "hipSetDevice";
        return GVRT_ERR_HIP;
    }
    if (!nccl(ncclCommInitRank(&comm_, world_, id_, rank_), "ncclCommInitRank", err)) {
        comm_ = nullptr;
        return GVRT_ERR_RCCL;
    }
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        // the collectives need a stream: without one this rank cannot take part
        *err = "hipStreamCreateWithFlags";
        abort();
        return GVRT_ERR_HIP;
    }
    stream_ = s;
    *comm_ok = true;
    // the handle renders (and unpacks) on the exchange's stream: render -> send/recv -> scatter in stream order
    if (gvrt_set_stream(app_.handle(), stream_) != GVRT_OK) {
        *err = std::string("gvrt_set_stream: ") + gvrt_last_error(app_.handle());
        return GVRT_ERR_HIP;
    }
    bound_ = true;
    return GVRT_OK;
}

bool RcclBackend::alloc(void** p, size_t bytes) {
    if (hipMalloc(p, bytes) == hipSuccess) return true;
    *p = nullptr;
    return false;
}
void RcclBackend::release(void* p) { (void)hipFree(p); }
bool RcclBackend::upload(void* dst, const void* src, size_t n) {
    return hipMemcpy(dst, src, n, hipMemcpyHostToDevice) == hipSuccess;
}
bool RcclBackend::download(void* dst, const void* src, size_t n) {
    return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) == hipSuccess;
}
bool RcclBackend::fill(void* dst, int value, size_t n) { return hipMemset(dst, value, n) == hipSuccess; }

bool RcclBackend::allreduce_max_i32(int32_t* d, std::string* err) {
    return nccl(ncclAllReduce(d, d, 1, ncclInt32, ncclMax, comm_, STREAM), "ncclAllReduce", err);
}
bool RcclBackend::broadcast(void* d, size_t bytes, int root, std::string* err) {
    return nccl(ncclBroadcast(d, d, bytes, ncclUint8, root, comm_, STREAM), "ncclBroadcast", err);
}
bool RcclBackend::group_start(std::string* err) { return nccl(ncclGroupStart(), "ncclGroupStart", err); }
bool RcclBackend::group_end(std::string* err) { return nccl(ncclGroupEnd(), "ncclGroupEnd", err); }
bool RcclBackend::send(const void* p, size_t bytes, int peer, std::string* err) {
    return nccl(ncclSend(p, bytes, ncclUint8, peer, comm_, STREAM), "ncclSend", err);
}
bool RcclBackend::recv(void* p, size_t bytes, int peer, std::string* err) {
    return nccl(ncclRecv(p, bytes, ncclUint8, peer, comm_, STREAM), "ncclRecv", err);
}

void RcclBackend::abort() {
    if (comm_) {
        (void)ncclCommAbort(comm_);
        comm_ = nullptr;
    }
}

bool RcclBackend::async_error(std::string* err) {
    if (!comm_) return false;
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &ae) != ncclSuccess) return false;
    if (ae == ncclSuccess || ae == ncclInProgress) return false;
    *err = ncclGetErrorString(ae);
    return true;
}

int RcclBackend::query(std::string* err) {
    const hipError_t q = hipStreamQuery(STREAM);
    if (q == hipSuccess) return 1;
    if (q == hipErrorNotReady) return 0;
    *err = hipGetErrorString(q);
    return -1;
}

void RcclBackend::drain() {
    if (stream_) (void)hipStreamSynchronize(STREAM);
}

bool RcclBackend::render_tiles(const gvrt_tile* tiles, size_t n, uint32_t width, uint32_t height, void* packed,
                               std::string* err) {
    gvrt_handle h = app_.handle();
    gvrt_image img{packed, nullptr, nullptr, nullptr, 1, 1};
    if (gvrt_render_async(h, &app_.params, app_.uniformDataDynamic.viewInverse.data(),
                          app_.uniformDataDynamic.projInverse.data(), width, height, 1, tiles, n, &img) == GVRT_OK)
        return true;
    *err = std::string("gvrt_render_async: ") + gvrt_last_error(h);
    return false;
}

bool RcclBackend::render_views(const float* view_inv, uint32_t nviews, const float* proj_inv, uint32_t width,
                               uint32_t height, void* out, std::string* err) {
    gvrt_handle h = app_.handle();
    gvrt_image img{out, nullptr, nullptr, nullptr, 1, 0};
    if (gvrt_render_async(h, &app_.params, view_inv, proj_inv, width, height, nviews, nullptr, 0, &img) == GVRT_OK)
        return true;
    *err = std::string("gvrt_render_async: ") + gvrt_last_error(h);
    return false;
}

bool RcclBackend::tile_costs(uint32_t width, uint32_t height, void* scratch, uint8_t* classes, size_t n,
                             std::string* err) {
    // the full frame twice: the second launch is cost-ordered and records every tile's class again
    gvrt_handle h = app_.handle();
    gvrt_image img{scratch, nullptr, nullptr, nullptr, 1, 0};
    for (int k = 0; k < 2; ++k)
        if (gvrt_render_async(h, &app_.params, app_.uniformDataDynamic.viewInverse.data(),
                              app_.uniformDataDynamic.projInverse.data(), width, height, 1, nullptr, 0, &img) != GVRT_OK ||
            gvrt_sync(h) != GVRT_OK) {
            *err = std::string("render: ") + gvrt_last_error(h);
            return false;
        }
    if (gvrt_read_tile_costs(h, classes, n) != GVRT_OK) {
        *err = std::string("gvrt_read_tile_costs: ") + gvrt_last_error(h);
        return false;
    }
    return true;
}

bool RcclBackend::view_cost(const float* view_inv, const float* proj_inv, uint32_t width, uint32_t height,
                            void* scratch, double* ms, std::string* err) {
    gvrt_handle h = app_.handle();
    gvrt_image img{scratch, nullptr, nullptr, nullptr, 1, 0};
    for (int k = 0; k < 2; ++k)
        if (gvrt_render_async(h, &app_.params, view_inv, proj_inv, width, height, 1, nullptr, 0, &img) != GVRT_OK ||
            gvrt_sync(h) != GVRT_OK) {
            *err = std::string("render: ") + gvrt_last_error(h);
            return false;
        }
    *ms = app_.stats().render_ms;
    return true;
}

bool RcclBackend::unpack(const void* part, const gvrt_tile* tiles, size_t n, uint32_t width, uint32_t height,
                         void* frame, std::string* err) {
    gvrt_handle h = app_.handle();
    if (gvrt_unpack_tiles_rgba8(h, part, tiles, n, width, height, 1, frame) == GVRT_OK) return true;
    *err = std::string("gvrt_unpack_tiles_rgba8: ") + gvrt_last_error(h);
    return false;
}

bool RcclBackend::sync_renders(std::string* err) {
    gvrt_handle h = app_.handle();
    if (gvrt_sync(h) == GVRT_OK) return true;
    *err = std::string("gvrt_sync: ") + gvrt_last_error(h);
    return false;
}

double RcclBackend::last_kernel_ms() { return app_.stats().render_ms; }

#undef STREAM

std::vector<float> RcclSplitFrame::flat(const std::vector<gm::mat4>* rig) {
    std::vector<float> out;
    if (rig)
        for (const gm::mat4& m : *rig) out.insert(out.end(), m.data(), m.data() + 16);
    return out;
}

RcclSplitFrame::RcclSplitFrame(GvrtApp& app, int rank, int world, const ncclUniqueId& id, uint32_t width,
                               uint32_t height, Layout layout, const std::vector<gm::mat4>* rig,
                               const gm::mat4* rig_proj_inv)
    : SplitFrame(std::unique_ptr<SplitBackend>(new RcclBackend(app, rank, world, id)), rank, world, width, height,
                 layout, flat(rig), rig_proj_inv ? rig_proj_inv->data() : nullptr) {}

}  // namespace gvrt_host
