// gvrt_split.cpp — SplitFrame over a SplitBackend (gvrt_split.h); no HIP or RCCL here (gvrt_rccl.cpp has those).
#include "gvrt_split.h"

#include <algorithm>
#include <chrono>
#include <cmath>
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

gvrt_status SplitFrame::fail(gvrt_status s, const std::string& m) {
    if (st_ == GVRT_OK) {
        st_ = s;
        err_ = m;
    }
    return s;
}

gvrt_status SplitFrame::comm_fail(const std::string& what, const std::string& err) {
    return fail(GVRT_ERR_RCCL, what + ": " + err);
}

gvrt_status SplitFrame::group_failed() {
    // a call between group start and end failed: close the group, then abort (the peers' matching calls never
    // complete; their bounded waits time out)
    std::string ignore;
    (void)be_->group_end(&ignore);
    be_->abort();
    return st_;
}

gvrt_status SplitFrame::wait(const char* what) {
    // an unbounded stream synchronize would wait forever for a collective whose peer never entered it (a rank that
    // failed before the call, or aborted its communicator: an abort does not notify peers over P2P / SHM links).
    // Poll the stream and the communicator's asynchronous error against a deadline instead; a timeout or an error
    // aborts the communicator, which makes its queued operations end.
    const auto t0 = std::chrono::steady_clock::now();
    auto sleep = std::chrono::microseconds(20);
    std::string e;
    while (true) {
        const int q = be_->query(&e);
        if (q == 1) return GVRT_OK;
        if (q < 0) {
            fail(GVRT_ERR_HIP, std::string(what) + ": " + e);
            be_->abort();
            return st_;
        }
        if (be_->has_comm() && be_->async_error(&e)) {
            comm_fail(std::string(what) + ": async error", e);
            be_->abort();
            return st_;
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s_) {
            fail(GVRT_ERR_RCCL, std::string(what) + ": no progress within " + std::to_string(timeout_s_) +
                                    " s (a peer did not take part in the exchange)");
            be_->abort();
            return st_;
        }
        std::this_thread::sleep_for(sleep);
        sleep = std::min(sleep * 2, std::chrono::microseconds(2000));
    }
}

gvrt_status SplitFrame::agree(gvrt_status local) {
    // every rank enters this all-reduce (max of the status magnitudes) before anything rank-specific, so a set-up
    // failure on one rank is every rank's failure and nobody waits in a later collective
    void* d = nullptr;
    if (!be_->alloc(&d, sizeof(int32_t))) {
        be_->abort();  // cannot take part: the peers' all-reduce ends in their bounded wait
        return fail(GVRT_ERR_OOM, "status word");
    }
    const int32_t mine = -(int32_t)local;  // statuses are <= 0
    gvrt_status s = GVRT_OK;
    if (!be_->upload(d, &mine, sizeof(mine))) s = fail(GVRT_ERR_HIP, "status upload");
    // (a failed upload still enters the all-reduce: the word then holds garbage, which can only look worse)
    std::string e;
    if (!be_->allreduce_max_i32(static_cast<int32_t*>(d), &e)) {
        comm_fail("all-reduce", e);
        be_->release(d);
        return st_;
    }
    int32_t all = 0;
    if (wait("agree") != GVRT_OK) {
        be_->release(d);
        return st_;
    }
    if (!be_->download(&all, d, sizeof(all))) s = fail(GVRT_ERR_HIP, "status readback");
    be_->release(d);
    if (s == GVRT_OK && all != 0) s = fail((gvrt_status)(-all), local != GVRT_OK ? err_ : "set-up failed on another rank");
    return s == GVRT_OK ? GVRT_OK : st_;
}

gvrt_status SplitFrame::cost_classes(std::vector<uint8_t>* classes) {
    const uint64_t n = (uint64_t)((width_ + 7) / 8) * ((height_ + 7) / 8);
    classes->assign(n, 0);
    // broadcast payload: one status byte (0: rank 0 measured the classes) then the classes; the same buffer is
    // rank 0's calibration frame
    void* d = nullptr;
    gvrt_status local = GVRT_OK;
    if (!be_->alloc(&d, std::max<uint64_t>(n + 1, (uint64_t)4 * width_ * height_))) {
        d = nullptr;
        local = fail(GVRT_ERR_OOM, "cost-class buffer");
    }
    if (agree(local) != GVRT_OK) {
        if (d) be_->release(d);
        return st_;
    }
    std::string why;
    if (rank_ == 0) {
        std::string e;
        const bool ok = be_->tile_costs(width_, height_, d, classes->data(), n, &e);
        if (!ok) why = "calibration: " + e;
        std::vector<uint8_t> msg(n + 1, 0);
        msg[0] = ok ? 0 : 1;
        if (ok) std::copy(classes->begin(), classes->end(), msg.begin() + 1);
        if (!be_->upload(d, msg.data(), n + 1)) {
            (void)be_->fill(d, 1, 1);  // best effort: the peers learn of the failure from the status byte
            if (ok) why = "class upload";
        }
    }
    // one broadcast at set-up (not per frame), entered by every rank whatever rank 0's calibration gave: every rank
    // cuts the same bands from the same classes, or learns that there are none
    std::string e;
    if (!be_->broadcast(d, n + 1, 0, &e)) {
        comm_fail("broadcast", e);
        be_->release(d);
        return st_;
    }
    std::vector<uint8_t> msg(n + 1, 1);
    gvrt_status s = wait("class broadcast");
    if (s == GVRT_OK && !be_->download(msg.data(), d, n + 1)) s = fail(GVRT_ERR_HIP, "class readback");
    be_->release(d);
    if (s == GVRT_OK && msg[0] != 0)
        s = fail(GVRT_ERR_STATE, "tile-cost calibration failed on rank 0" + (why.empty() ? std::string() : ": " + why));
    if (s == GVRT_OK) std::copy(msg.begin() + 1, msg.end(), classes->begin());
    return s;
}

gvrt_status SplitFrame::view_costs_bcast(std::vector<double>* costs) {
    const size_t nv = rig_.size() / 16;
    costs->assign(nv, 0.0);
    // broadcast payload: a status word (0.0: rank 0 timed every view) then one kernel time per view
    void* d = nullptr;
    void* img = nullptr;
    gvrt_status local = GVRT_OK;
    if (!be_->alloc(&d, sizeof(double) * (nv + 1))) {
        d = nullptr;
        local = fail(GVRT_ERR_OOM, "view-cost buffer");
    }
    if (local == GVRT_OK && rank_ == 0 && !be_->alloc(&img, (size_t)4 * width_ * height_)) {
        img = nullptr;
        local = fail(GVRT_ERR_OOM, "calibration frame");
    }
    if (agree(local) != GVRT_OK) {
        if (d) be_->release(d);
        if (img) be_->release(img);
        return st_;
    }
    std::string why;
    if (rank_ == 0) {
        // each view alone, twice: the second launch is cost-ordered (bench.py view_cost_calibration)
        std::vector<double> msg(nv + 1, 0.0);
        bool ok = true;
        for (size_t v = 0; v < nv && ok; ++v) {
            std::string e;
            ok = be_->view_cost(rig_.data() + 16 * v, rig_proj_, width_, height_, img, &msg[v + 1], &e);
            if (!ok) why = "calibration: " + e;
        }
        msg[0] = ok ? 0.0 : 1.0;
        if (!be_->upload(d, msg.data(), sizeof(double) * (nv + 1))) {
            (void)be_->fill(d, 0xFF, sizeof(double));  // best effort: a NaN status word reads as a failure
            if (ok) why = "cost upload";
        }
        be_->release(img);
    }
    std::string e;
    if (!be_->broadcast(d, sizeof(double) * (nv + 1), 0, &e)) {
        comm_fail("broadcast", e);
        be_->release(d);
        return st_;
    }
    std::vector<double> msg(nv + 1, 1.0);
    gvrt_status s = wait("cost broadcast");
    if (s == GVRT_OK && !be_->download(msg.data(), d, sizeof(double) * (nv + 1))) s = fail(GVRT_ERR_HIP, "cost readback");
    be_->release(d);
    if (s == GVRT_OK && !(msg[0] == 0.0))
        s = fail(GVRT_ERR_STATE, "view-cost calibration failed on rank 0" + (why.empty() ? std::string() : ": " + why));
    if (s == GVRT_OK) std::copy(msg.begin() + 1, msg.end(), costs->begin());
    return s;
}

SplitFrame::SplitFrame(std::unique_ptr<SplitBackend> backend, int rank, int world, uint32_t width, uint32_t height,
                       Layout layout, const std::vector<float>& rig, const float* rig_proj_inv)
    : be_(std::move(backend)), rank_(rank), world_(world), width_(width), height_(height), layout_(layout) {
    // (argument errors are the same on every rank: refused before the communicator exists)
    if (!be_) {
        fail(GVRT_ERR_INVALID_ARG, "no backend");
        return;
    }
    if (world < 1 || rank < 0 || rank >= world) {
        fail(GVRT_ERR_INVALID_ARG, "rank must be in [0, world)");
        return;
    }
    if (layout == VIEWS && (!rig_proj_inv || rig.empty() || rig.size() % 16 || rig.size() / 16 > 255)) {
        fail(GVRT_ERR_INVALID_ARG, "the VIEWS layout needs a rig of 1..255 views and its projection inverse");
        return;
    }
    bool comm_ok = false;
    std::string e;
    const gvrt_status init = be_->init(&comm_ok, &e);
    if (!comm_ok) {  // no communicator: nothing to agree through (the peers' set-up waits end in their bound)
        fail(init != GVRT_OK ? init : GVRT_ERR_RCCL, "set-up: " + e);
        return;
    }
    // from here on every failure is agreed on (agree) or travels in a broadcast's status word: no rank leaves a
    // collective its peers have entered
    gvrt_status local = init != GVRT_OK ? fail(init, "set-up: " + e) : GVRT_OK;
    if (agree(local) != GVRT_OK) return;
    size_t part_bytes = 0;
    if (layout == VIEWS) {
        rig_ = rig;
        std::copy(rig_proj_inv, rig_proj_inv + 16, rig_proj_);
        if (view_costs_bcast(&view_costs_) != GVRT_OK) return;
        views_ = balanced_views(view_costs_, world);
        for (uint32_t v : views_[rank]) my_vi_.insert(my_vi_.end(), rig_.begin() + 16 * v, rig_.begin() + 16 * v + 16);
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
    if (!be_->alloc(&d_part_, std::max<size_t>(16, part_bytes))) {
        d_part_ = nullptr;
        local = fail(GVRT_ERR_OOM, "part buffer");
    }
    if (local == GVRT_OK && rank == 0 && layout != VIEWS) {
        d_recv_.assign(world, nullptr);
        for (int r = 0; r < world && local == GVRT_OK; ++r)
            if (!be_->alloc(&d_recv_[r], std::max<size_t>(16, (size_t)all_tiles_[r].size() * 256))) {
                d_recv_[r] = nullptr;
                local = fail(GVRT_ERR_OOM, "receive buffer");
            }
    }
    agree(local);
}

SplitFrame::~SplitFrame() {
    if (!be_) return;
    // (bounded: a peer that never entered a queued exchange leaves it pending; the wait then aborts the
    // communicator, whose operations end, and the drain below returns)
    if (be_->has_comm()) (void)wait("teardown");
    be_->drain();
    for (void* p : d_recv_)
        if (p) be_->release(p);
    if (d_part_) be_->release(d_part_);
    be_.reset();
}

gvrt_status SplitFrame::draw(void* frame) {
    if (st_ != GVRT_OK) {
        be_->abort();  // a rank that cannot take part any more: its peers' exchange ends in their bounded waits
        return st_;
    }
    if (rank_ == 0 && !frame) {
        // refused before the exchange: the peers are told through the aborted communicator
        fail(GVRT_ERR_INVALID_ARG, "rank 0 needs a frame");
        be_->abort();
        return st_;
    }
    // the previous frame first (bounded), so that no host wait of the render call below sits behind an exchange
    // whose peer is gone
    if (!pipelined_ && wait("previous frame") != GVRT_OK) return st_;
    const size_t view_bytes = (size_t)4 * width_ * height_;
    // this rank's part, queued on the stream: its tiles tile-packed, or its views in one batched launch
    gvrt_status local = GVRT_OK;
    std::string e;
    bool rs = true;
    if (layout_ == VIEWS)
        rs = views_[rank_].empty() || be_->render_views(my_vi_.data(), (uint32_t)views_[rank_].size(), rig_proj_,
                                                        width_, height_, d_part_, &e);
    else
        rs = be_->render_tiles(tiles_.data(), tiles_.size(), width_, height_, d_part_, &e);
    if (!rs) local = fail(GVRT_ERR_HIP, "render: " + e);
    // the exchange, entered even after a failed render (the part then holds a stale frame): every rank's part to
    // rank 0 in one group, exact sizes (rank 0 also sends its own part to itself); views land in their frame slots
    if (!be_->group_start(&e)) {
        comm_fail("group start", e);
        be_->abort();
        return st_;
    }
    if (layout_ == VIEWS) {
        for (size_t i = 0; i < views_[rank_].size(); ++i)
            if (!be_->send((uint8_t*)d_part_ + i * view_bytes, view_bytes, 0, &e)) {
                comm_fail("send", e);
                return group_failed();
            }
        if (rank_ == 0)
            for (int r = 0; r < world_; ++r)
                for (uint32_t v : views_[r])
                    if (!be_->recv((uint8_t*)frame + v * view_bytes, view_bytes, r, &e)) {
                        comm_fail("recv", e);
                        return group_failed();
                    }
    } else {
        if (!be_->send(d_part_, tiles_.size() * 256, 0, &e)) {
            comm_fail("send", e);
            return group_failed();
        }
        if (rank_ == 0)
            for (int r = 0; r < world_; ++r)
                if (!be_->recv(d_recv_[r], all_tiles_[r].size() * 256, r, &e)) {
                    comm_fail("recv", e);
                    return group_failed();
                }
    }
    if (!be_->group_end(&e)) {
        comm_fail("group end", e);
        be_->abort();
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
        be_->abort();
        return st_;
    }
    // rank 0, tile layouts: scatter every part into the frame, behind the receives on the same stream
    if (rank_ == 0 && layout_ != VIEWS)
        for (int r = 0; r < world_; ++r)
            if (!be_->unpack(d_recv_[r], all_tiles_[r].data(), all_tiles_[r].size(), width_, height_, frame, &e)) {
                fail(GVRT_ERR_HIP, "unpack: " + e);
                be_->abort();
                return st_;
            }
    return GVRT_OK;
}

gvrt_status SplitFrame::sync() {
    if (st_ != GVRT_OK) return st_;
    if (wait("sync") != GVRT_OK) return st_;  // bounded: the queued frames' exchanges include the peers
    std::string e;
    if (!be_->sync_renders(&e)) return fail(GVRT_ERR_HIP, "render sync: " + e);
    if (be_->async_error(&e)) return comm_fail("async error", e);
    return GVRT_OK;
}

double SplitFrame::lastKernelMs() const { return be_ ? be_->last_kernel_ms() : 0.0; }

}  // namespace gvrt_host
