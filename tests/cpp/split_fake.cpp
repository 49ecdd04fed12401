// SplitFrame (host/gvrt_split.h) with real peers on the CPU: an in-process SplitBackend whose ranks are threads
// (VERDICT r05 #5).  The fake keeps RCCL's semantics that SplitFrame's failure handling relies on:
//   * every rank's operations are queued on its own in-order stream; a collective finishes when every rank has
//     posted it, a send when its receiver has posted the matching receive (and the reverse), in per-channel order;
//   * abort() ends the rank's queued operations and takes its communicator away, without telling the peers (as
//     ncclCommAbort over P2P / SHM links), so a peer's matching operation stays pending until its bounded wait;
//   * renders are deterministic pixel codes, so rank 0's assembled frame can be checked pixel for pixel.
// Failures are injected per rank: a failed allocation at set-up, a rank that stops mid-run, a failed send inside a
// frame's group, a failed render.  Usage: split_fake <scenario> <world>; prints one JSON line and exits 0 (the test,
// tests/test_host_cpp.py, checks the statuses and runs the binary under a hard wall limit).
#include <algorithm>
#include <atomic>
#include <climits>
#include <functional>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "gvrt_split.h"

using gvrt_host::SplitBackend;
using gvrt_host::SplitFrame;

namespace {

uint32_t pixel_code(uint32_t x, uint32_t y, uint32_t v) { return (x * 73856093u) ^ (y * 19349663u) ^ (v * 83492791u) ^ 1u; }

struct Inject {
    int fail_alloc = -1;       // the n-th alloc of this rank fails (0-based)
    int stop_after = -1;       // the rank's thread returns after this many frames (a rank that stops mid-run)
    int fail_send_frame = -1;  // send() fails in this frame (an error inside the group)
    int fail_render_frame = -1;
};

struct World {
    int n;
    std::mutex mu;
    // collectives: seq -> {posted by ranks, inputs}
    struct Coll {
        int kind = 0;  // 1 all-reduce max i32, 2 broadcast
        size_t bytes = 0;
        int root = 0;
        std::map<int, std::vector<uint8_t>> in;
    };
    std::map<uint64_t, Coll> coll;
    // point to point: (src, dst, seq) -> the sent bytes; posted receives
    std::map<std::tuple<int, int, uint64_t>, std::vector<uint8_t>> sent;
    std::set<std::tuple<int, int, uint64_t>> recv_posted;
    explicit World(int n_) : n(n_) {}
};

class FakeBackend : public SplitBackend {
  public:
    FakeBackend(World& w, int rank, Inject inj) : w_(w), rank_(rank), inj_(inj), send_seq_(w.n, 0), recv_seq_(w.n, 0) {}
    ~FakeBackend() override {
        for (void* p : live_) std::free(p);
    }
    int frame = 0;  // set by the driver before each draw (failure injection)

    gvrt_status init(bool* comm_ok, std::string* err) override {
        (void)err;
        *comm_ok = true;
        comm_ = true;
        return GVRT_OK;
    }
    bool alloc(void** p, size_t bytes) override {
        if (n_alloc_++ == inj_.fail_alloc) {
            *p = nullptr;
            return false;
        }
        *p = std::calloc(bytes, 1);
        live_.insert(*p);
        return *p != nullptr;
    }
    void release(void* p) override {
        live_.erase(p);
        std::free(p);
    }
    bool upload(void* dst, const void* src, size_t n) override { return std::memcpy(dst, src, n), true; }
    bool download(void* dst, const void* src, size_t n) override { return std::memcpy(dst, src, n), true; }
    bool fill(void* dst, int value, size_t n) override { return std::memset(dst, value, n), true; }

    bool allreduce_max_i32(int32_t* d, std::string* err) override { return coll(1, d, 4, 0, err); }
    bool broadcast(void* d, size_t bytes, int root, std::string* err) override { return coll(2, d, bytes, root, err); }
    bool group_start(std::string* err) override { return alive(err); }
    bool group_end(std::string* err) override { return alive(err); }
    bool send(const void* p, size_t bytes, int peer, std::string* err) override {
        if (!alive(err)) return false;
        if (frame == inj_.fail_send_frame) {
            *err = "injected send failure";
            return false;
        }
        std::lock_guard<std::mutex> g(w_.mu);
        const auto key = std::make_tuple(rank_, peer, send_seq_[peer]++);
        w_.sent[key].assign((const uint8_t*)p, (const uint8_t*)p + bytes);
        ops_.push_back(Op{Op::SEND, key, nullptr, 0, 0, {}});
        return true;
    }
    bool recv(void* p, size_t bytes, int peer, std::string* err) override {
        if (!alive(err)) return false;
        std::lock_guard<std::mutex> g(w_.mu);
        const auto key = std::make_tuple(peer, rank_, recv_seq_[peer]++);
        w_.recv_posted.insert(key);
        ops_.push_back(Op{Op::RECV, key, p, bytes, 0, {}});
        return true;
    }
    bool has_comm() const override { return comm_; }
    void abort() override {
        std::lock_guard<std::mutex> g(w_.mu);
        comm_ = false;
        ops_.clear();  // its queued operations end; the peers are not told
    }
    bool async_error(std::string* err) override {
        (void)err;
        return false;
    }
    int query(std::string* err) override {
        (void)err;
        std::lock_guard<std::mutex> g(w_.mu);
        while (!ops_.empty()) {
            Op& o = ops_.front();
            if (o.kind == Op::SEND) {
                const auto& k = o.key;
                if (!w_.recv_posted.count(k)) return 0;
            } else if (o.kind == Op::RECV) {
                auto it = w_.sent.find(o.key);
                if (it == w_.sent.end()) return 0;
                std::memcpy(o.dst, it->second.data(), std::min(o.bytes, it->second.size()));
            } else if (o.kind == Op::COLL) {
                auto& c = w_.coll[o.seq];
                if ((int)c.in.size() < w_.n) return 0;
                if (c.kind == 1) {
                    int32_t m = INT32_MIN;
                    for (auto& kv : c.in) {
                        int32_t v;
                        std::memcpy(&v, kv.second.data(), 4);
                        m = std::max(m, v);
                    }
                    std::memcpy(o.dst, &m, 4);
                } else {
                    std::memcpy(o.dst, c.in[c.root].data(), c.bytes);
                }
            } else if (o.kind == Op::LOCAL) {
                o.fn(o);
            }
            ops_.erase(ops_.begin());
        }
        return 1;
    }
    void drain() override {
        // teardown after the bounded wait: whatever is still queued waits on a peer that is gone
        std::lock_guard<std::mutex> g(w_.mu);
        ops_.clear();
    }
    bool render_tiles(const gvrt_tile* tiles, size_t n, uint32_t width, uint32_t height, void* packed,
                      std::string* err) override {
        if (frame == inj_.fail_render_frame) {
            *err = "injected render failure";
            return false;
        }
        (void)height;
        uint32_t* out = static_cast<uint32_t*>(packed);
        for (size_t i = 0; i < n; ++i)
            for (uint32_t l = 0; l < 64; ++l)
                out[64 * i + l] = pixel_code(tiles[i].tx * 8u + (l & 7u), tiles[i].ty * 8u + (l >> 3), 0);
        (void)width;
        return true;
    }
    bool render_views(const float* view_inv, uint32_t nviews, const float* proj_inv, uint32_t width, uint32_t height,
                      void* out, std::string* err) override {
        (void)proj_inv;
        if (frame == inj_.fail_render_frame) {
            *err = "injected render failure";
            return false;
        }
        uint32_t* o = static_cast<uint32_t*>(out);
        for (uint32_t v = 0; v < nviews; ++v) {
            const uint32_t tag = (uint32_t)view_inv[16 * v + 12];  // the view's index rides in its origin
            for (uint32_t y = 0; y < height; ++y)
                for (uint32_t x = 0; x < width; ++x) o[((size_t)v * height + y) * width + x] = pixel_code(x, y, tag + 1);
        }
        return true;
    }
    bool tile_costs(uint32_t width, uint32_t height, void* scratch, uint8_t* classes, size_t n,
                    std::string* err) override {
        (void)scratch;
        (void)err;
        const uint32_t tx_n = (width + 7) / 8;
        (void)height;
        for (size_t i = 0; i < n; ++i) classes[i] = (uint8_t)((i % tx_n) * 7 + (i / tx_n) * 3) % 24;
        return true;
    }
    bool view_cost(const float* view_inv, const float* proj_inv, uint32_t width, uint32_t height, void* scratch,
                   double* ms, std::string* err) override {
        (void)proj_inv, (void)width, (void)height, (void)scratch, (void)err;
        *ms = 1.0 + 0.25 * ((uint32_t)view_inv[12] % 5);
        return true;
    }
    bool unpack(const void* part, const gvrt_tile* tiles, size_t n, uint32_t width, uint32_t height, void* frame,
                std::string* err) override {
        if (!alive(err)) return false;
        std::lock_guard<std::mutex> g(w_.mu);
        Op o{Op::LOCAL, {}, frame, 0, 0, {}};
        o.fn = [part, tiles, n, width, height](Op& op) {
            const uint32_t* p = static_cast<const uint32_t*>(part);
            uint32_t* f = static_cast<uint32_t*>(op.dst);
            for (size_t i = 0; i < n; ++i)
                for (uint32_t l = 0; l < 64; ++l) {
                    const uint32_t x = tiles[i].tx * 8u + (l & 7u), y = tiles[i].ty * 8u + (l >> 3);
                    if (x < width && y < height) f[(size_t)y * width + x] = p[64 * i + l];
                }
        };
        ops_.push_back(o);
        return true;
    }
    bool sync_renders(std::string* err) override {
        (void)err;
        return true;
    }
    double last_kernel_ms() override { return 1.0; }

  private:
    struct Op {
        enum Kind { SEND, RECV, COLL, LOCAL } kind;
        std::tuple<int, int, uint64_t> key;
        void* dst;
        size_t bytes;
        uint64_t seq;
        std::function<void(Op&)> fn;
    };
    bool alive(std::string* err) {
        if (comm_) return true;
        *err = "communicator aborted";
        return false;
    }
    bool coll(int kind, void* d, size_t bytes, int root, std::string* err) {
        if (!alive(err)) return false;
        std::lock_guard<std::mutex> g(w_.mu);
        const uint64_t seq = coll_seq_++;
        auto& c = w_.coll[seq];
        c.kind = kind;
        c.bytes = bytes;
        c.root = root;
        c.in[rank_].assign((const uint8_t*)d, (const uint8_t*)d + bytes);
        ops_.push_back(Op{Op::COLL, {}, d, bytes, seq, {}});
        return true;
    }

    World& w_;
    int rank_;
    Inject inj_;
    bool comm_ = false;
    int n_alloc_ = 0;
    uint64_t coll_seq_ = 0;
    std::vector<uint64_t> send_seq_, recv_seq_;
    std::vector<Op> ops_;
    std::set<void*> live_;
};

struct Result {
    int status = 0;
    int frames_ok = 0;
    double seconds = 0.0;
    std::string error;
    bool frame_ok = true;
};

std::string esc(const std::string& s) {
    std::string o;
    for (char c : s) o += (c == '"' || c == '\\') ? ' ' : c;
    return o;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: split_fake {healthy|healthy_views|setup_fail|stop|group_fail|render_fail} world\n");
        return 2;
    }
    const std::string scen = argv[1];
    const int world = std::atoi(argv[2]);
    const uint32_t W = 200, H = 120;  // 25 x 15 tiles
    const int frames = 4;
    const double timeout_s = 1.0;
    World w(world);
    std::vector<Result> res(world);
    const int victim = world - 1;
    const bool views = scen == "healthy_views";
    const uint32_t nviews = 11;
    std::vector<float> rig(16 * nviews, 0.0f);
    for (uint32_t v = 0; v < nviews; ++v) rig[16 * v + 12] = (float)v;
    float proj[16] = {};
    auto body = [&](int r) {
        Inject inj;
        if (r == victim) {
            if (scen == "setup_fail") inj.fail_alloc = 3;  // the part buffer (after status words and the calibration)
            if (scen == "stop") inj.stop_after = 1;
            if (scen == "group_fail") inj.fail_send_frame = 1;
            if (scen == "render_fail") inj.fail_render_frame = 1;
        }
        auto* be = new FakeBackend(w, r, inj);
        const auto t0 = std::chrono::steady_clock::now();
        Result& out = res[r];
        {
            SplitFrame sf(std::unique_ptr<SplitBackend>(be), r, world, W, H,
                          views ? SplitFrame::VIEWS : SplitFrame::COST_BANDS, views ? rig : std::vector<float>(),
                          views ? proj : nullptr);
            sf.set_timeout(timeout_s);
            std::vector<uint32_t> frame((size_t)(views ? nviews : 1) * W * H, 0);
            gvrt_status s = sf.status();
            for (int f = 0; s == GVRT_OK && f < frames; ++f) {
                if (f == inj.stop_after) break;  // this rank stops taking part
                be->frame = f;
                std::fill(frame.begin(), frame.end(), 0u);
                s = sf.draw(frame.data());
                if (s == GVRT_OK) s = sf.sync();
                if (s == GVRT_OK) {
                    ++out.frames_ok;
                    if (r == 0)
                        for (uint32_t v = 0; v < (views ? nviews : 1u); ++v)
                            for (uint32_t y = 0; y < H; ++y)
                                for (uint32_t x = 0; x < W; ++x)
                                    out.frame_ok &= frame[((size_t)v * H + y) * W + x] == pixel_code(x, y, views ? v + 1 : 0);
                }
            }
            out.status = (int)s;
            out.error = sf.error();
        }
        out.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r) th.emplace_back(body, r);
    for (auto& t : th) t.join();
    std::printf("{\"scenario\": \"%s\", \"world\": %d, \"timeout_s\": %.1f, \"victim\": %d, \"ranks\": [", scen.c_str(),
                world, timeout_s, victim);
    for (int r = 0; r < world; ++r)
        std::printf("%s{\"rank\": %d, \"status\": %d, \"frames_ok\": %d, \"seconds\": %.3f, \"frame_ok\": %s, "
                    "\"error\": \"%s\"}",
                    r ? ", " : "", r, res[r].status, res[r].frames_ok, res[r].seconds,
                    res[r].frame_ok ? "true" : "false", esc(res[r].error).c_str());
    std::printf("]}\n");
    return 0;
}
