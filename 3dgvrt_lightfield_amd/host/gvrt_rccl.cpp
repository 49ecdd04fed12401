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

std::vector<std::vector<uint32_t>> balanced_views(const std::vector<double>& costs, int world) {
    // dist.balanced_views: longest-processing-time list scheduling with a count bound
    const size_t n = costs.size();
    std::vector<size_t> cap(world);
    for (int r = 0; r < world; ++r) cap[r] = n / world + ((size_t)r < n % world ? 1 : 0);
    std::vector<double> load(world, 0.0);
    std::vector<std::vector<uint32_t>> out(world);
    std::vector<uint32_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return costs[a] > costs[b] || (costs[a] == costs[b] && a < b);  // sorted by (-cost, index)
    });
    for (uint32_t v : order) {
        int best = -1;
        for (int r = 0; r < world; ++r)
            if (out[r].size() < cap[r] && (best < 0 || load[r] < load[best])) best = r;  // ties: lower rank
        out[best].push_back(v);
        load[best] += costs[v];
    }
    for (auto& g : out) std::sort(g.begin(), g.end());
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

gvrt_status SplitFrame::group_failed() {
    // an RCCL call between ncclGroupStart and ncclGroupEnd failed: close the group, then abort (the peers' matching
    // calls never complete; their bounded waits time out)
    (void)ncclGroupEnd();
    abort_comm();
    return st_;
}

gvrt_status SplitFrame::wait(const char* what) {
    // hipStreamSynchronize would wait forever for a collective whose peer never entered it (a rank that failed before
    // the call, or aborted its communicator: ncclCommAbort does not notify peers over P2P / SHM links).  Poll the
    // stream and the communicator's asynchronous error against a deadline instead; a timeout or an error aborts the
    // communicator, which makes its queued kernels exit.
    const auto t0 = std::chrono::steady_clock::now();
    auto sleep = std::chrono::microseconds(20);
    while (true) {
        const hipError_t q = hipStreamQuery(stream_);
        if (q == hipSuccess) return GVRT_OK;
        if (q != hipErrorNotReady) {
            fail(GVRT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(q));
            abort_comm();
            return st_;
        }
        if (comm_) {
            ncclResult_t ae = ncclSuccess;
            if (ncclCommGetAsyncError(comm_, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                fail(GVRT_ERR_RCCL, std::string(what) + ": RCCL async error: " + ncclGetErrorString(ae));
                abort_comm();
                return st_;
            }
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_) {
            fail(GVRT_ERR_RCCL, std::string(what) + ": no progress within " + std::to_string(timeout_s_) +
                                    " s (a peer did not take part in the exchange)");
            abort_comm();
            return st_;
        }
        std::this_thread::sleep_for(sleep);
        sleep = std::min(sleep * 2, std::chrono::microseconds(2000));
    }
}

gvrt_status SplitFrame::agree(gvrt_status local) {
    // every rank enters this all-reduce (max of the status magnitudes) before anything rank-specific, so a set-up
    // failure on one rank is every rank's failure and nobody waits in a later collective
    int32_t* d = nullptr;
    if (hipMalloc(&d, sizeof(int32_t)) != hipSuccess) {
        abort_comm();  // cannot take part: the peers' all-reduce errors out
        return fail(GVRT_ERR_OOM, "status word");
    }
    const int32_t mine = -(int32_t)local;  // statuses are <= 0
    gvrt_status s = GVRT_OK;
    if (hipMemcpy(d, &mine, sizeof(mine), hipMemcpyHostToDevice) != hipSuccess) s = fail(GVRT_ERR_HIP, "status upload");
    // (a failed upload still enters the all-reduce: the word then holds garbage, which can only look worse)
    if (rccl(ncclAllReduce(d, d, 1, ncclInt32, ncclMax, comm_, stream_), "ncclAllReduce")) {
        (void)hipFree(d);
        return st_;
    }
    int32_t all = 0;
    if (wait("agree") != GVRT_OK) {
        (void)hipFree(d);
        return st_;
    }
    if (hipMemcpy(&all, d, sizeof(all), hipMemcpyDeviceToHost) != hipSuccess) s = fail(GVRT_ERR_HIP, "status readback");
    (void)hipFree(d);
    if (s == GVRT_OK && all != 0) s = fail((gvrt_status)(-all), local != GVRT_OK ? err_ : "set-up failed on another rank");
    return s == GVRT_OK ? GVRT_OK : st_;
}

void SplitFrame::abort_comm() {
    if (comm_) {
        (void)ncclCommAbort(comm_);
        comm_ = nullptr;
    }
}

gvrt_status SplitFrame::cost_classes(std::vector<uint8_t>* classes) {
    gvrt_handle h = app_.handle();
    const uint64_t n = (uint64_t)((width_ + 7) / 8) * ((height_ + 7) / 8);
    classes->assign(n, 0);
    // broadcast payload: one status byte (0: rank 0 measured the classes) then the classes
    uint8_t* d = nullptr;
    gvrt_status local = GVRT_OK;
    if (hipMalloc(&d, std::max<uint64_t>(n + 1, (uint64_t)4 * width_ * height_)) != hipSuccess) {
        d = nullptr;
        local = fail(GVRT_ERR_OOM, "cost-class buffer");
    }
    if (agree(local) != GVRT_OK) {
        if (d) (void)hipFree(d);
        return st_;
    }
    std::string why;
    if (rank_ == 0) {
        // the full frame twice: the second launch is cost-ordered and records every tile's class again
        gvrt_image img{d, nullptr, nullptr, nullptr, 1, 0};
        bool ok = true;
        for (int k = 0; k < 2 && ok; ++k)
            ok = gvrt_render_async(h, &app_.params, app_.uniformDataDynamic.viewInverse.data(),
                                   app_.uniformDataDynamic.projInverse.data(), width_, height_, 1, nullptr, 0,
                                   &img) == GVRT_OK &&
                 gvrt_sync(h) == GVRT_OK;
        if (!ok) why = std::string("calibration render: ") + gvrt_last_error(h);
        if (ok && gvrt_read_tile_costs(h, classes->data(), n) != GVRT_OK) {
            ok = false;
            why = std::string("gvrt_read_tile_costs: ") + gvrt_last_error(h);
        }
        std::vector<uint8_t> msg(n + 1, 0);
        msg[0] = ok ? 0 : 1;
        if (ok) std::copy(classes->begin(), classes->end(), msg.begin() + 1);
        if (hipMemcpy(d, msg.data(), n + 1, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipMemset(d, 1, 1);  // best effort: the peers learn of the failure from the status byte
            if (ok) why = "class upload";
        }
    }
    // one broadcast at set-up (not per frame), entered by every rank whatever rank 0's calibration gave: every rank
    // cuts the same bands from the same classes, or learns that there are none
    if (rccl(ncclBroadcast(d, d, n + 1, ncclUint8, 0, comm_, stream_), "ncclBroadcast")) {
        (void)hipFree(d);
        return st_;
    }
    std::vector<uint8_t> msg(n + 1, 1);
    gvrt_status s = wait("class broadcast");
    if (s == GVRT_OK && hipMemcpy(msg.data(), d, n + 1, hipMemcpyDeviceToHost) != hipSuccess)
        s = fail(GVRT_ERR_HIP, "class readback");
    (void)hipFree(d);
    if (s == GVRT_OK && msg[0] != 0)
        s = fail(GVRT_ERR_STATE, "tile-cost calibration failed on rank 0" + (why.empty() ? std::string() : ": " + why));
    if (s == GVRT_OK) std::copy(msg.begin() + 1, msg.end(), classes->begin());
    return s;
}

gvrt_status SplitFrame::view_costs_bcast(std::vector<double>* costs) {
    gvrt_handle h = app_.handle();
    const size_t nv = rig_.size();
    costs->assign(nv, 0.0);
    // broadcast payload: a status word (0.0: rank 0 timed every view) then one kernel time per view
    double* d = nullptr;
    void* img_buf = nullptr;
    gvrt_status local = GVRT_OK;
    if (hipMalloc(&d, sizeof(double) * (nv + 1)) != hipSuccess) {
        d = nullptr;
        local = fail(GVRT_ERR_OOM, "view-cost buffer");
    }
    if (local == GVRT_OK && rank_ == 0 && hipMalloc(&img_buf, (size_t)4 * width_ * height_) != hipSuccess) {
        img_buf = nullptr;
        local = fail(GVRT_ERR_OOM, "calibration frame");
    }
    if (agree(local) != GVRT_OK) {
        if (d) (void)hipFree(d);
        if (img_buf) (void)hipFree(img_buf);
        return st_;
    }
    std::string why;
    if (rank_ == 0) {
        // each view alone, twice: the second launch is cost-ordered (bench.py view_cost_calibration)
        std::vector<double> msg(nv + 1, 0.0);
        gvrt_image img{img_buf, nullptr, nullptr, nullptr, 1, 0};
        bool ok = true;
        for (size_t v = 0; v < nv && ok; ++v) {
            for (int k = 0; k < 2 && ok; ++k)
                ok = gvrt_render_async(h, &app_.params, rig_[v].data(), rig_proj_.data(), width_, height_, 1, nullptr, 0,
                                       &img) == GVRT_OK &&
                     gvrt_sync(h) == GVRT_OK;
            if (ok) msg[v + 1] = app_.stats().render_ms;
        }
        if (!ok) why = std::string("calibration render: ") + gvrt_last_error(h);
        msg[0] = ok ? 0.0 : 1.0;
        if (hipMemcpy(d, msg.data(), sizeof(double) * (nv + 1), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipMemset(d, 0xFF, sizeof(double));  // best effort: a NaN status word reads as a failure
            if (ok) why = "cost upload";
        }
        (void)hipFree(img_buf);
    }
    if (rccl(ncclBroadcast(d, d, nv + 1, ncclFloat64, 0, comm_, stream_), "ncclBroadcast")) {
        (void)hipFree(d);
        return st_;
    }
    std::vector<double> msg(nv + 1, 1.0);
    gvrt_status s = wait("cost broadcast");
    if (s == GVRT_OK && hipMemcpy(msg.data(), d, sizeof(double) * (nv + 1), hipMemcpyDeviceToHost) != hipSuccess)
        s = fail(GVRT_ERR_HIP, "cost readback");
    (void)hipFree(d);
    if (s == GVRT_OK && !(msg[0] == 0.0))
        s = fail(GVRT_ERR_STATE, "view-cost calibration failed on rank 0" + (why.empty() ? std::string() : ": " + why));
    if (s == GVRT_OK) std::copy(msg.begin() + 1, msg.end(), costs->begin());
    return s;
}

SplitFrame::SplitFrame(GvrtApp& app, int rank, int world, const ncclUniqueId& id, uint32_t width, uint32_t height,
                       Layout layout, const std::vector<gm::mat4>* rig, const gm::mat4* rig_proj_inv)
    : app_(app), rank_(rank), world_(world), width_(width), height_(height), layout_(layout) {
    if (world < 1 || rank < 0 || rank >= world) {
        fail(GVRT_ERR_INVALID_ARG, "rank must be in [0, world)");
        return;
    }
    // (argument errors are the same on every rank: refused before the communicator exists)
    if (layout == VIEWS && (!rig || !rig_proj_inv || rig->empty() || rig->size() > 255)) {
        fail(GVRT_ERR_INVALID_ARG, "the VIEWS layout needs a rig of 1..255 views and its projection inverse");
        return;
    }
    if (hipSetDevice(app.device.ordinal) != hipSuccess) {
        fail(GVRT_ERR_HIP, "hipSetDevice");
        return;
    }
    if (rccl(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank")) return;
    // from here on every failure is agreed on (agree) or travels in a broadcast's status word: no rank leaves a
    // collective its peers have entered
    gvrt_status local = GVRT_OK;
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
        // the collectives below need a stream: without one this rank cannot take part
        fail(GVRT_ERR_HIP, "hipStreamCreateWithFlags");
        stream_ = nullptr;
        abort_comm();
        return;
    }
    // the handle renders (and unpacks) on the exchange's stream: render -> send/recv -> scatter in stream order
    if (gvrt_set_stream(app.handle(), stream_) != GVRT_OK)
        local = fail(GVRT_ERR_HIP, std::string("gvrt_set_stream: ") + gvrt_last_error(app.handle()));
    if (agree(local) != GVRT_OK) return;
    size_t part_bytes = 0;
    if (layout == VIEWS) {
        rig_ = *rig;
        rig_proj_ = *rig_proj_inv;
        if (view_costs_bcast(&view_costs_) != GVRT_OK) return;
        views_ = balanced_views(view_costs_, world);
        for (uint32_t v : views_[rank])
            my_vi_.insert(my_vi_.end(), rig_[v].data(), rig_[v].data() + 16);
        part_bytes = (size_t)views_[rank].size() * 4 * width * height;
    } else {
        if (layout == COST_BANDS) {
            std::vector<uint8_t> classes;
            if (cost_classes(&classes) != GVRT_OK) return;
            all_tiles_ = band_tiles(width, height, world, classes.data());
        } else {
            for (int r = 0; r < world; ++r) all_tiles_.push_back(rank_tiles(width, height, 1, r, world));
        }
        tiles_ = all_tiles_[rank];
        part_bytes = (size_t)tiles_.size() * 256;
    }
    if (hipMalloc(&d_part_, std::max<size_t>(16, part_bytes)) != hipSuccess) {
        d_part_ = nullptr;
        local = fail(GVRT_ERR_OOM, "part buffer");
    }
    if (local == GVRT_OK && rank == 0 && layout != VIEWS) {
        d_recv_.assign(world, nullptr);
        for (int r = 0; r < world && local == GVRT_OK; ++r)
            if (hipMalloc(&d_recv_[r], std::max<size_t>(16, (size_t)all_tiles_[r].size() * 256)) != hipSuccess) {
                d_recv_[r] = nullptr;
                local = fail(GVRT_ERR_OOM, "receive buffer");
            }
    }
    agree(local);
}

SplitFrame::~SplitFrame() {
    (void)hipSetDevice(app_.device.ordinal);
    if (stream_) {
        // (bounded: a peer that never entered a queued exchange leaves it pending; the wait then aborts the
        // communicator, whose kernels exit, and the synchronize below returns)
        if (comm_) (void)wait("teardown");
        (void)hipStreamSynchronize(stream_);
    }
    if (app_.handle() && stream_) (void)gvrt_set_stream(app_.handle(), nullptr);
    for (void* p : d_recv_)
        if (p) (void)hipFree(p);
    if (d_part_) (void)hipFree(d_part_);
    if (comm_) (void)ncclCommDestroy(comm_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

gvrt_status SplitFrame::draw(void* frame) {
    if (st_ != GVRT_OK) {
        abort_comm();  // a rank that cannot take part any more: its peers' exchange errors out instead of waiting
        return st_;
    }
    if (rank_ == 0 && !frame) {
        // refused before the exchange: the peers are told through the aborted communicator
        fail(GVRT_ERR_INVALID_ARG, "rank 0 needs a frame");
        abort_comm();
        return st_;
    }
    gvrt_handle h = app_.handle();
    const size_t view_bytes = (size_t)4 * width_ * height_;
    // this rank's part, queued on the stream (gvrt_render_async: no host wait): its tiles tile-packed, or its views
    // in one batched launch ([view][H][W][4])
    gvrt_status local = GVRT_OK;
    gvrt_image img{d_part_, nullptr, nullptr, nullptr, 1, layout_ == VIEWS ? 0u : 1u};
    gvrt_status rs;
    if (layout_ == VIEWS)
        rs = views_[rank_].empty() ? GVRT_OK
                                   : gvrt_render_async(h, &app_.params, my_vi_.data(), rig_proj_.data(), width_, height_,
                                                       (uint32_t)views_[rank_].size(), nullptr, 0, &img);
    else
        rs = gvrt_render_async(h, &app_.params, app_.uniformDataDynamic.viewInverse.data(),
                               app_.uniformDataDynamic.projInverse.data(), width_, height_, 1, tiles_.data(),
                               tiles_.size(), &img);
    if (rs != GVRT_OK) local = fail(GVRT_ERR_HIP, std::string("gvrt_render_async: ") + gvrt_last_error(h));
    // the exchange, entered even after a failed render (the part then holds a stale frame): every rank's part to
    // rank 0 in one group, exact sizes (rank 0 also sends its own part to itself); views land in their frame slots
    if (rccl(ncclGroupStart(), "ncclGroupStart")) {
        abort_comm();
        return st_;
    }
    if (layout_ == VIEWS) {
        for (size_t i = 0; i < views_[rank_].size(); ++i)
            if (rccl(ncclSend((uint8_t*)d_part_ + i * view_bytes, view_bytes, ncclUint8, 0, comm_, stream_), "ncclSend"))
                return group_failed();
        if (rank_ == 0)
            for (int r = 0; r < world_; ++r)
                for (uint32_t v : views_[r])
                    if (rccl(ncclRecv((uint8_t*)frame + v * view_bytes, view_bytes, ncclUint8, r, comm_, stream_),
                             "ncclRecv"))
                        return group_failed();
    } else {
        if (rccl(ncclSend(d_part_, tiles_.size() * 256, ncclUint8, 0, comm_, stream_), "ncclSend"))
            return group_failed();
        if (rank_ == 0)
            for (int r = 0; r < world_; ++r)
                if (rccl(ncclRecv(d_recv_[r], all_tiles_[r].size() * 256, ncclUint8, r, comm_, stream_), "ncclRecv"))
                    return group_failed();
    }
    if (rccl(ncclGroupEnd(), "ncclGroupEnd")) {
        abort_comm();
        return st_;
    }
    if (local != GVRT_OK) {
        // this frame's exchange is queued: drain it (bounded) so the peers' matching receives / sends complete, then
        // abort; a peer that reaches its next exchange learns of it through its own bounded wait
        const std::string keep = err_;
        st_ = GVRT_OK;
        (void)wait("failed frame's exchange");
        st_ = local;
        err_ = keep;
        abort_comm();
        return st_;
    }
    // rank 0, tile layouts: scatter every part into the frame, behind the receives on the same stream
    if (rank_ == 0 && layout_ != VIEWS)
        for (int r = 0; r < world_; ++r)
            if (gvrt_unpack_tiles_rgba8(h, d_recv_[r], all_tiles_[r].data(), all_tiles_[r].size(), width_, height_, 1,
                                        frame) != GVRT_OK) {
                fail(GVRT_ERR_HIP, std::string("gvrt_unpack_tiles_rgba8: ") + gvrt_last_error(h));
                abort_comm();
                return st_;
            }
    return GVRT_OK;
}

gvrt_status SplitFrame::sync() {
    if (st_ != GVRT_OK) return st_;
    if (wait("sync") != GVRT_OK) return st_;  // bounded: the queued frames' exchanges include the peers
    if (gvrt_sync(app_.handle()) != GVRT_OK)
        return fail(GVRT_ERR_HIP, std::string("gvrt_sync: ") + gvrt_last_error(app_.handle()));
    ncclResult_t async_err = ncclSuccess;
    if (rccl(ncclCommGetAsyncError(comm_, &async_err), "ncclCommGetAsyncError")) return st_;
    if (rccl(async_err, "RCCL async error")) return st_;
    return GVRT_OK;
}

double SplitFrame::lastKernelMs() const { return app_.stats().render_ms; }

}  // namespace gvrt_host
