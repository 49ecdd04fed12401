// gvrt_split.h — the multi-GPU frame split of the C++ host (north_star: "the image is optionally
// tile-partitioned across 8 GPUs with RCCL gather over xGMI"), written against a small backend interface.
//
// One process per GPU.  Every rank holds the whole scene (GvrtApp::prepare; the build is deterministic, so the
// ranks' BVHs are identical) and renders its own tiles of each frame: 64x64-pixel blocks dealt round-robin over
// the ranks (rank_tiles, the same lists as the Python layer's dist.rank_tiles), or cost-weighted bands, tile-packed.
// One exchange per frame: grouped sends / receives of the packed parts to rank 0 (rank 0 sends its own part to
// itself, so a one-rank communicator runs the same path), then rank 0 scatters each part into the frame.  The
// render, the exchange and the scatter are queued on one stream, so a frame costs no host round trip.  The
// reference has no multi-GPU path: this replaces the single vkCmdTraceRaysKHR of buildCommandBuffer
// (VulkanFullRT.cpp:1217-1230) by N of them.  Config 5 (the light field, VulkanFullRT.cpp:1900-1976) splits whole
// views instead (layout VIEWS, balanced_views).
//
// SplitFrame makes every device, communicator and renderer call through SplitBackend: RCCL + HIP +
// libgvrt implement it in production (gvrt_rccl.h RcclBackend), and tests/cpp/split_fake.cpp implements it with one
// thread per rank in one process, so the failure paths below run with real peers on a CPU.
//
// Errors are statuses: a communicator failure is GVRT_ERR_RCCL (include/gvrt.h), a renderer or device failure
// GVRT_ERR_HIP; error() has the text.  Failures are made common knowledge where that is possible: set-up failures are
// agreed on by an all-reduce of every rank's status before anything rank-specific, rank 0's calibration result
// travels with a status word in the one broadcast every rank always enters, and a rank that fails inside draw() still
// enters that frame's exchange (sending what its part buffer holds), drains it, and then aborts its communicator.  An
// aborted communicator does not notify peers over P2P / SHM links (ncclCommAbort), so every wait on the exchange is
// bounded instead: wait() polls the stream and the communicator's asynchronous error against a deadline
// (set_timeout, default 120 s) and aborts the communicator when it passes.  The bound covers the waits SplitFrame
// makes; draw() waits (bounded) for the previous frame before it queues the next render unless set_pipelined(true),
// so the renderer's own host waits (camera-ring events, tile-list uploads) never sit behind an exchange whose peer
// is gone.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/gvrt.h"

namespace gvrt_host {

// this rank's 8x8 tiles: (block*8)^2-pixel blocks round-robin over `world` ranks, per camera (dist.rank_tiles)
std::vector<gvrt_tile> rank_tiles(uint32_t width, uint32_t height, uint32_t ncams, int rank, int world,
                                  uint32_t block = 8);

// Every rank's tile list for the cost-weighted band split (dist.band_tiles): the tiles in rank_tiles' block
// order (world 1) cut into `world` runs of equal summed cost, a tile of class c weighing 2^(c/4) (classes:
// gvrt_read_tile_costs of a full frame, [ty][tx]); classes == nullptr: runs of equal tile count.
std::vector<std::vector<gvrt_tile>> band_tiles(uint32_t width, uint32_t height, int world, const uint8_t* classes,
                                               uint32_t block = 8);

// Cost-weighted view assignment (dist.balanced_views): every rank gets floor or ceil(views / world) views, placed
// costliest first on the least-loaded rank with room (ties: lower rank, lower view index); each rank's views in
// increasing index
std::vector<std::vector<uint32_t>> balanced_views(const std::vector<double>& costs, int world);

// What SplitFrame needs from the device, the communicator and the renderer of one rank.  Communicator and render
// calls are queued on the rank's stream; `false` means the call itself failed (text in *err).
class SplitBackend {
  public:
    virtual ~SplitBackend() = default;
    // set-up: the communicator and the rank's stream, the renderer bound to that stream.  *comm_ok: a communicator
    // exists (the status can then be agreed on); the status: whether this rank can take part
    virtual gvrt_status init(bool* comm_ok, std::string* err) = 0;
    // memory on the rank's device; copies are synchronous
    virtual bool alloc(void** p, size_t bytes) = 0;
    virtual void release(void* p) = 0;
    virtual bool upload(void* dst, const void* src, size_t n) = 0;
    virtual bool download(void* dst, const void* src, size_t n) = 0;
    virtual bool fill(void* dst, int value, size_t n) = 0;
    // communicator
    virtual bool allreduce_max_i32(int32_t* d, std::string* err) = 0;
    virtual bool broadcast(void* d, size_t bytes, int root, std::string* err) = 0;
    virtual bool group_start(std::string* err) = 0;
    virtual bool group_end(std::string* err) = 0;
    virtual bool send(const void* p, size_t bytes, int peer, std::string* err) = 0;
    virtual bool recv(void* p, size_t bytes, int peer, std::string* err) = 0;
    virtual bool has_comm() const = 0;
    virtual void abort() = 0;                     // the communicator: its queued operations end, peers are not told
    virtual bool async_error(std::string* err) = 0;  // the communicator failed asynchronously
    // the stream: 1 every queued operation finished, 0 pending, -1 failed (*err)
    virtual int query(std::string* err) = 0;
    virtual void drain() = 0;                     // the stream, unbounded (teardown, after the bounded wait)
    // renderer (the app's camera and parameters)
    virtual bool render_tiles(const gvrt_tile* tiles, size_t n, uint32_t width, uint32_t height, void* packed,
                              std::string* err) = 0;
    virtual bool render_views(const float* view_inv, uint32_t nviews, const float* proj_inv, uint32_t width,
                              uint32_t height, void* out, std::string* err) = 0;
    // calibration (synchronous): the app's frame rendered twice, then its per-tile cost classes [ty][tx]
    virtual bool tile_costs(uint32_t width, uint32_t height, void* scratch, uint8_t* classes, size_t n,
                            std::string* err) = 0;
    // calibration (synchronous): one view rendered twice, the kernel ms of the second (cost-ordered) launch
    virtual bool view_cost(const float* view_inv, const float* proj_inv, uint32_t width, uint32_t height,
                           void* scratch, double* ms, std::string* err) = 0;
    virtual bool unpack(const void* part, const gvrt_tile* tiles, size_t n, uint32_t width, uint32_t height,
                        void* frame, std::string* err) = 0;
    virtual bool sync_renders(std::string* err) = 0;
    virtual double last_kernel_ms() = 0;
};

class SplitFrame {
  public:
    enum Layout { BLOCKS = 0, COST_BANDS = 1, VIEWS = 2 };
    // COST_BANDS: rank 0 renders the app's current frame twice and reads its per-tile cost classes, one broadcast
    // hands them to every rank, and all cut the same bands (band_tiles); BLOCKS: 64x64-pixel blocks round-robin
    // (rank_tiles); VIEWS: the views of `rig` (16 floats each, column-major view inverses; shared projection
    // inverse) split over the ranks: rank 0 times each view alone, one broadcast hands the costs to every rank, and
    // all compute the same balanced_views assignment
    SplitFrame(std::unique_ptr<SplitBackend> backend, int rank, int world, uint32_t width, uint32_t height,
               Layout layout = COST_BANDS, const std::vector<float>& rig = {}, const float* rig_proj_inv = nullptr);
    ~SplitFrame();
    SplitFrame(const SplitFrame&) = delete;
    SplitFrame& operator=(const SplitFrame&) = delete;

    gvrt_status status() const { return st_; }  // of the constructor (communicator, buffers)
    void set_timeout(double seconds) { timeout_s_ = seconds; }  // the bound of every wait on the exchange
    // true: draw() queues the next frame without waiting for the previous one (host launch overlapped with the
    // device; the renderer's own host waits are then not bounded)
    void set_pipelined(bool on) { pipelined_ = on; }
    const std::string& error() const { return err_; }

    // one frame with the app's camera: this rank's tiles rendered tile-packed, gathered to rank 0 and scattered into
    // `frame` (device rgba8 [H][W][4], rank 0 only; ignored elsewhere).  Queued on the stream.
    // VIEWS: this rank's views of the rig, each sent whole into frame's view slot (device rgba8 [views][H][W][4]).
    gvrt_status draw(void* frame);
    gvrt_status sync();  // waits (bounded) for every queued frame on this rank

    int rank() const { return rank_; }
    int world() const { return world_; }
    const std::vector<gvrt_tile>& tiles() const { return tiles_; }
    const std::vector<std::vector<uint32_t>>& views() const { return views_; }  // VIEWS: every rank's views
    const std::vector<double>& view_costs() const { return view_costs_; }    // VIEWS: calibration kernel ms
    double lastKernelMs() const;  // mean kernel time of the frames completed by the last sync

  private:
    gvrt_status fail(gvrt_status s, const std::string& m);
    gvrt_status comm_fail(const std::string& what, const std::string& err);  // GVRT_ERR_RCCL
    gvrt_status cost_classes(std::vector<uint8_t>* classes);
    gvrt_status view_costs_bcast(std::vector<double>* costs);
    gvrt_status agree(gvrt_status local);  // every rank's set-up status, all-reduced: the worst one everywhere
    gvrt_status group_failed();            // a call inside a group failed: end the group, abort
    gvrt_status wait(const char* what);    // the stream, bounded by timeout_s_ and watching the async error

    std::unique_ptr<SplitBackend> be_;
    int rank_, world_;
    uint32_t width_, height_;
    gvrt_status st_ = GVRT_OK;
    std::string err_;
    double timeout_s_ = 120.0;
    bool pipelined_ = false;
    std::vector<gvrt_tile> tiles_;                  // this rank's tile list
    std::vector<std::vector<gvrt_tile>> all_tiles_;  // every rank's (rank 0 scatters with them)
    void* d_part_ = nullptr;                         // this rank's packed part: tiles * 64 px * 4 B
    std::vector<void*> d_recv_;                      // rank 0: one receive buffer per rank
    Layout layout_ = COST_BANDS;
    std::vector<float> rig_;                          // VIEWS: the rig's view inverses, 16 floats each
    float rig_proj_[16] = {};
    std::vector<std::vector<uint32_t>> views_;        // VIEWS: every rank's views (balanced_views)
    std::vector<double> view_costs_;
    std::vector<float> my_vi_;                        // VIEWS: this rank's view inverses, 16 floats each
};

}  // namespace gvrt_host
