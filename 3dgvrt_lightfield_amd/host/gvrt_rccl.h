// gvrt_rccl.h — the multi-GPU frame split of the C++ host over RCCL (north_star: "the image is
// optionally tile-partitioned across 8 GPUs with RCCL gather over xGMI").
//
// One process per GPU.  Every rank holds the whole scene (GvrtApp::prepare; the build is deterministic, so the
// ranks' BVHs are identical) and renders its own tiles of each frame: 64x64-pixel blocks dealt round-robin over
// the ranks (rank_tiles, the same lists as the Python layer's dist.rank_tiles), tile-packed.  One exchange per
// frame: grouped ncclSend / ncclRecv of the packed parts to rank 0 (rank 0 sends its own part to itself, so a
// one-rank communicator runs the same path), then rank 0 scatters each part into the frame with
// gvrt_unpack_tiles_rgba8.  The render, the exchange and the scatter are queued on one HIP stream (the handle
// renders on it, gvrt_set_stream), so a frame costs no host round trip.  The reference has no multi-GPU path:
// this replaces the single vkCmdTraceRaysKHR of buildCommandBuffer (VulkanFullRT.cpp:1217-1230) by N of them.
//
// Config 5 (the light field on N GPUs, VulkanFullRT.cpp:1900-1976 computeGaussianLightField) splits whole views
// instead: layout VIEWS assigns the views of a camera rig to the ranks by cost (balanced_views, bit for bit the
// Python layer's dist.balanced_views), each rank renders its views in one batched launch, and every view goes to
// rank 0 whole, straight into its slot of the [view][H][W][4] frame.
//
// Errors are statuses: an RCCL failure is GVRT_ERR_RCCL (include/gvrt.h), a HIP failure GVRT_ERR_HIP; error()
// has the text.  Failures are made common knowledge where that is possible: set-up failures are agreed on by an
// all-reduce of every rank's status before anything rank-specific, rank 0's calibration result travels with a status
// word in the one broadcast every rank always enters, and a rank that fails inside draw() still enters that frame's
// exchange (sending what its part buffer holds), drains it, and then aborts its communicator.  ncclCommAbort does not
// notify peers over P2P / SHM links, so every wait on the exchange is bounded instead of trusting that: wait() polls
// the stream and ncclCommGetAsyncError against a deadline (set_timeout, default 120 s) and aborts the communicator
// when it passes.  The bound covers the waits SplitFrame itself makes; draw() calls wait() for the previous frame
// before it queues the next render, so the render call's own host waits (camera-ring events, tile-list uploads)
// never sit behind an exchange whose peer is gone.
#pragma once
#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "gvrt_host.h"

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

// Rendezvous of the communicator: rank 0 creates the RCCL unique id and writes it to `path` (written to a
// temporary name and renamed, so a reader never sees half a file); every other rank waits for the file (up to
// timeout_s seconds).  Returns GVRT_OK or GVRT_ERR_RCCL / GVRT_ERR_IO with the text in *err.
gvrt_status rccl_rendezvous(const std::string& path, int rank, ncclUniqueId* id, std::string* err,
                            double timeout_s = 120.0);

class SplitFrame {
  public:
    enum Layout { BLOCKS = 0, COST_BANDS = 1, VIEWS = 2 };
    // ncclCommInitRank(world, id, rank) on the app's device; the app's handle then renders on this object's stream.
    // COST_BANDS: rank 0 renders the app's current frame twice and reads its per-tile cost classes
    // (gvrt_read_tile_costs), one ncclBroadcast hands them to every rank, and all cut the same bands (band_tiles);
    // BLOCKS: 64x64-pixel blocks round-robin (rank_tiles);
    // VIEWS: the views of `rig` (view inverses, shared projection inverse) split over the ranks: rank 0 renders
    // each view alone twice and times the second (cost-ordered) launch, one ncclBroadcast hands the costs to every
    // rank, and all compute the same balanced_views assignment
    SplitFrame(GvrtApp& app, int rank, int world, const ncclUniqueId& id, uint32_t width, uint32_t height,
               Layout layout = COST_BANDS, const std::vector<gm::mat4>* rig = nullptr,
               const gm::mat4* rig_proj_inv = nullptr);
    ~SplitFrame();
    SplitFrame(const SplitFrame&) = delete;
    SplitFrame& operator=(const SplitFrame&) = delete;

    gvrt_status status() const { return st_; }  // of the constructor (communicator, buffers)
    void set_timeout(double seconds) { timeout_s_ = seconds; }  // the bound of every wait on the exchange
    const std::string& error() const { return err_; }

    // one frame with the app's uniformDataDynamic: this rank's tiles rendered tile-packed, gathered to rank 0 and
    // scattered into `frame` (device rgba8 [H][W][4], rank 0 only; ignored elsewhere).  Queued on the stream.
    // VIEWS: this rank's views of the rig, each sent whole into frame's view slot (device rgba8 [views][H][W][4]).
    gvrt_status draw(void* frame);
    gvrt_status sync();  // waits for every queued frame on this rank

    int rank() const { return rank_; }
    int world() const { return world_; }
    const std::vector<gvrt_tile>& tiles() const { return tiles_; }
    const std::vector<std::vector<uint32_t>>& views() const { return views_; }  // VIEWS: every rank's views
    const std::vector<double>& view_costs() const { return view_costs_; }    // VIEWS: calibration kernel ms
    double lastKernelMs() const;  // mean kernel time of the frames completed by the last sync (gvrt_stats)

  private:
    gvrt_status fail(gvrt_status s, const std::string& m);
    gvrt_status rccl(ncclResult_t r, const char* what);
    // rank 0 measures, every rank receives (one broadcast of a status word and the payload, always entered)
    gvrt_status cost_classes(std::vector<uint8_t>* classes);
    gvrt_status view_costs_bcast(std::vector<double>* costs);
    gvrt_status agree(gvrt_status local);  // every rank's set-up status, all-reduced: the worst one everywhere
    void abort_comm();                     // ncclCommAbort: this rank's queued RCCL kernels exit
    gvrt_status group_failed();            // an RCCL call inside a group failed: end the group, abort
    gvrt_status wait(const char* what);    // the stream, bounded by timeout_s_ and watching RCCL's async error

    GvrtApp& app_;
    int rank_, world_;
    uint32_t width_, height_;
    gvrt_status st_ = GVRT_OK;
    std::string err_;
    ncclComm_t comm_ = nullptr;
    double timeout_s_ = 120.0;
    hipStream_t stream_ = nullptr;
    std::vector<gvrt_tile> tiles_;                  // this rank's tile list
    std::vector<std::vector<gvrt_tile>> all_tiles_;  // every rank's (rank 0 scatters with them)
    void* d_part_ = nullptr;                         // this rank's packed part: tiles * 64 px * 4 B
    std::vector<void*> d_recv_;                      // rank 0: one receive buffer per rank
    Layout layout_ = COST_BANDS;
    std::vector<gm::mat4> rig_;                       // VIEWS: the rig's view inverses
    gm::mat4 rig_proj_{};
    std::vector<std::vector<uint32_t>> views_;        // VIEWS: every rank's views (balanced_views)
    std::vector<double> view_costs_;
    std::vector<float> my_vi_;                        // VIEWS: this rank's view inverses, 16 floats each
};

}  // namespace gvrt_host
