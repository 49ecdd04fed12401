// gvrt_rccl.cpp — SplitFrame: the one-process-per-GPU tile split of a frame with an RCCL gather to rank 0
// (gvrt_rccl.h).
#include "gvrt_rccl.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <thread>

namespace gvrt_host {

std::vector<gvrt_tile> rank_tiles(uint32_t width, uint32_t height, uint32_t ncams, int rank, int world,
                                  uint32_t block) {
    // renderer.tiles_for_rank: blocks of block x block tiles in row-major order per camera, block k to rank k % world
    const uint32_t tx_n = (width + 7) / 8, ty_n = (height + 7) / 8;
    const uint32_t bx_n = (tx_n + block - 1) / block, by_n = (ty_n + block - 1) / block;
    std::vector<gvrt_tile> out;
    uint64_t k = 0;
    for (uint32_t c = 0; c < ncams; ++c)
        for (uint32_t by = 0; by < by_n; ++by)
            for (uint32_t bx = 0; bx < bx_n; ++bx, ++k) {
                if ((int)(k % (uint64_t)world) != rank) continue;
                for (uint32_t ty = by * block; ty < std::min((by + 1) * block, ty_n); ++ty)
                    for (uint32_t tx = bx * block; tx < std::min((bx + 1) * block, tx_n); ++tx)
                        out.push_back(gvrt_tile{(uint16_t)tx, (uint16_t)ty, (uint16_t)c, 0});
            }
    return out;
}

std::vector<std::vector<gvrt_tile>> band_tiles(uint32_t width, uint32_t height, int world, const uint8_t* classes,
                                               uint32_t block) {
    // dist.band_tiles: prefix sums of the weights in block order, cut k at the first position whose prefix reaches
    // k/world of the total (numpy searchsorted, side left)
    static const double quarter[4] = {1.0, 1.189207115002721, 1.4142135623730951, 1.681792830507429};
    const std::vector<gvrt_tile> order = rank_tiles(width, height, 1, 0, 1, block);
    const uint32_t tx_n = (width + 7) / 8;
    const size_t n = order.size();
    std::vector<double> cum(n + 1, 0.0);
    for (size_t i = 0; i < n; ++i) {
        double w = 1.0;
        if (classes) {
            const uint32_t c = classes[(size_t)order[i].ty * tx_n + order[i].tx];
            w = std::ldexp(quarter[c & 3u], (int)(c >> 2));
        }
        cum[i + 1] = cum[i] + w;
    }
    std::vector<size_t> cuts(world + 1, 0);
    cuts[world] = n;
    for (int k = 1; k < world; ++k) {
        const double target = cum[n] * k / world;
        cuts[k] = std::min(n, (size_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin()));
        cuts[k] = std::max(cuts[k], cuts[k - 1]);
    }
    std::vector<std::vector<gvrt_tile>> out(world);
    for (int r = 0; r < world; ++r) out[r].assign(order.begin() + cuts[r], order.begin() + cuts[r + 1]);
    return out;
}

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

gvrt_status SplitFrame::fail(gvrt_status s, const std::string& m) {
    if (st_ == GVRT_OK) {
        st_ = s;
        err_ = m;
    }
    return s;
}

gvrt_status SplitFrame::rccl(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return GVRT_OK;
    return fail(GVRT_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

gvrt_status SplitFrame::cost_classes(std::vector<uint8_t>* classes) {
    gvrt_handle h = app_.handle();
    const uint64_t n = (uint64_t)((width_ + 7) / 8) * ((height_ + 7) / 8);
    classes->assign(n, 0);
    uint8_t* d = nullptr;
    if (hipMalloc(&d, std::max<uint64_t>(n, (uint64_t)4 * width_ * height_)) != hipSuccess)
        return fail(GVRT_ERR_OOM, "cost-class buffer");
    gvrt_status s = GVRT_OK;
    if (rank_ == 0) {
        // the full frame twice: the second launch is cost-ordered and records every tile's class again
        gvrt_image img{d, nullptr, nullptr, nullptr, 1, 0};
        for (int k = 0; k < 2 && s == GVRT_OK; ++k)
            if (gvrt_render_async(h, &app_.params, app_.uniformDataDynamic.viewInverse.data(),
                                  app_.uniformDataDynamic.projInverse.data(), width_, height_, 1, nullptr, 0,
                                  &img) != GVRT_OK ||
                gvrt_sync(h) != GVRT_OK)
                s = fail(GVRT_ERR_HIP, std::string("calibration render: ") + gvrt_last_error(h));
        if (s == GVRT_OK && gvrt_read_tile_costs(h, classes->data(), n) != GVRT_OK)
            s = fail(GVRT_ERR_HIP, std::string("gvrt_read_tile_costs: ") + gvrt_last_error(h));
        if (s == GVRT_OK && hipMemcpy(d, classes->data(), n, hipMemcpyHostToDevice) != hipSuccess)
            s = fail(GVRT_ERR_HIP, "class upload");
    }
    // one broadcast at set-up (not per frame): every rank cuts the same bands from the same classes
    if (s == GVRT_OK) s = rccl(ncclBroadcast(d, d, n, ncclUint8, 0, comm_, stream_), "ncclBroadcast");
    if (s == GVRT_OK && hipStreamSynchronize(stream_) != hipSuccess) s = fail(GVRT_ERR_HIP, "broadcast sync");
    if (s == GVRT_OK && hipMemcpy(classes->data(), d, n, hipMemcpyDeviceToHost) != hipSuccess)
        s = fail(GVRT_ERR_HIP, "class readback");
    (void)hipFree(d);
    return s;
}

SplitFrame::SplitFrame(GvrtApp& app, int rank, int world, const ncclUniqueId& id, uint32_t width, uint32_t height,
                       Layout layout)
    : app_(app), rank_(rank), world_(world), width_(width), height_(height) {
    if (world < 1 || rank < 0 || rank >= world) {
        fail(GVRT_ERR_INVALID_ARG, "rank must be in [0, world)");
        return;
    }
    if (hipSetDevice(app.device.ordinal) != hipSuccess) {
        fail(GVRT_ERR_HIP, "hipSetDevice");
        return;
    }
    if (rccl(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank")) return;
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
        fail(GVRT_ERR_HIP, "hipStreamCreateWithFlags");
        return;
    }
    // the handle renders (and unpacks) on the exchange's stream: render -> send/recv -> scatter in stream order
    if (gvrt_set_stream(app.handle(), stream_) != GVRT_OK) {
        fail(GVRT_ERR_HIP, std::string("gvrt_set_stream: ") + gvrt_last_error(app.handle()));
        return;
    }
    if (layout == COST_BANDS) {
        std::vector<uint8_t> classes;
        if (cost_classes(&classes) != GVRT_OK) return;
        all_tiles_ = band_tiles(width, height, world, classes.data());
    } else {
        for (int r = 0; r < world; ++r) all_tiles_.push_back(rank_tiles(width, height, 1, r, world));
    }
    tiles_ = all_tiles_[rank];
    if (hipMalloc(&d_part_, std::max<size_t>(16, (size_t)tiles_.size() * 256)) != hipSuccess) {
        d_part_ = nullptr;
        fail(GVRT_ERR_OOM, "part buffer");
        return;
    }
    if (rank == 0) {
        d_recv_.assign(world, nullptr);
        for (int r = 0; r < world; ++r)
            if (hipMalloc(&d_recv_[r], std::max<size_t>(16, (size_t)all_tiles_[r].size() * 256)) != hipSuccess) {
                d_recv_[r] = nullptr;
                fail(GVRT_ERR_OOM, "receive buffer");
                return;
            }
    }
}

SplitFrame::~SplitFrame() {
    (void)hipSetDevice(app_.device.ordinal);
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (app_.handle()) (void)gvrt_set_stream(app_.handle(), nullptr);
    for (void* p : d_recv_)
        if (p) (void)hipFree(p);
    if (d_part_) (void)hipFree(d_part_);
    if (comm_) (void)ncclCommDestroy(comm_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

gvrt_status SplitFrame::draw(void* frame) {
    if (st_ != GVRT_OK) return st_;
    if (rank_ == 0 && !frame) return fail(GVRT_ERR_INVALID_ARG, "rank 0 needs a frame");
    gvrt_handle h = app_.handle();
    // this rank's tiles, tile-packed, queued on the stream (gvrt_render_async: no host wait)
    gvrt_image img{d_part_, nullptr, nullptr, nullptr, 1, 1};
    if (gvrt_render_async(h, &app_.params, app_.uniformDataDynamic.viewInverse.data(),
                          app_.uniformDataDynamic.projInverse.data(), width_, height_, 1, tiles_.data(), tiles_.size(),
                          &img) != GVRT_OK)
        return fail(GVRT_ERR_HIP, std::string("gvrt_render_async: ") + gvrt_last_error(h));
    // the exchange: every rank's part to rank 0, one group (rank 0 also sends its own part to itself)
    if (rccl(ncclGroupStart(), "ncclGroupStart")) return st_;
    if (rccl(ncclSend(d_part_, tiles_.size() * 256, ncclUint8, 0, comm_, stream_), "ncclSend")) return st_;
    if (rank_ == 0)
        for (int r = 0; r < world_; ++r)
            if (rccl(ncclRecv(d_recv_[r], all_tiles_[r].size() * 256, ncclUint8, r, comm_, stream_), "ncclRecv"))
                return st_;
    if (rccl(ncclGroupEnd(), "ncclGroupEnd")) return st_;
    // rank 0: scatter every part into the frame, behind the receives on the same stream
    if (rank_ == 0)
        for (int r = 0; r < world_; ++r)
            if (gvrt_unpack_tiles_rgba8(h, d_recv_[r], all_tiles_[r].data(), all_tiles_[r].size(), width_, height_, 1,
                                        frame) != GVRT_OK)
                return fail(GVRT_ERR_HIP, std::string("gvrt_unpack_tiles_rgba8: ") + gvrt_last_error(h));
    return GVRT_OK;
}

gvrt_status SplitFrame::sync() {
    if (st_ != GVRT_OK) return st_;
    if (gvrt_sync(app_.handle()) != GVRT_OK)
        return fail(GVRT_ERR_HIP, std::string("gvrt_sync: ") + gvrt_last_error(app_.handle()));
    ncclResult_t async_err = ncclSuccess;
    if (rccl(ncclCommGetAsyncError(comm_, &async_err), "ncclCommGetAsyncError")) return st_;
    if (rccl(async_err, "RCCL async error")) return st_;
    return GVRT_OK;
}

double SplitFrame::lastKernelMs() const { return app_.stats().render_ms; }

}  // namespace gvrt_host
