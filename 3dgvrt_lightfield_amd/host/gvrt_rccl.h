// gvrt_rccl.h — the production SplitBackend (gvrt_split.h) of the multi-GPU frame split: RCCL over xGMI for the
// exchange, HIP for the rank's stream and memory, libgvrt (through GvrtApp) for the renders.  One process per GPU;
// the frame split itself (tile / band / view layouts, the bounded waits and the failure agreement) is SplitFrame.
#pragma once
#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "gvrt_host.h"
#include "gvrt_split.h"

namespace gvrt_host {

// Rendezvous of the communicator: rank 0 creates the RCCL unique id and writes it to `path` (written to a
// temporary name and renamed, so a reader never sees half a file); every other rank waits for the file (up to
// timeout_s seconds).  Returns GVRT_OK or GVRT_ERR_RCCL / GVRT_ERR_IO with the text in *err.
gvrt_status rccl_rendezvous(const std::string& path, int rank, ncclUniqueId* id, std::string* err,
                            double timeout_s = 120.0);

// ncclCommInitRank(world, id, rank) on the app's device, a non-blocking HIP stream the app's handle then renders on
// (gvrt_set_stream: render -> send / recv -> scatter in stream order), device memory by hipMalloc.
class RcclBackend : public SplitBackend {
  public:
    RcclBackend(GvrtApp& app, int rank, int world, const ncclUniqueId& id);
    ~RcclBackend() override;
    gvrt_status init(bool* comm_ok, std::string* err) override;
    bool alloc(void** p, size_t bytes) override;
    void release(void* p) override;
    bool upload(void* dst, const void* src, size_t n) override;
    bool download(void* dst, const void* src, size_t n) override;
    bool fill(void* dst, int value, size_t n) override;
    bool allreduce_max_i32(int32_t* d, std::string* err) override;
    bool broadcast(void* d, size_t bytes, int root, std::string* err) override;
    bool group_start(std::string* err) override;
    bool group_end(std::string* err) override;
    bool send(const void* p, size_t bytes, int peer, std::string* err) override;
    bool recv(void* p, size_t bytes, int peer, std::string* err) override;
    bool has_comm() const override { return comm_ != nullptr; }
    void abort() override;
    bool async_error(std::string* err) override;
    int query(std::string* err) override;
    void drain() override;
    bool render_tiles(const gvrt_tile* tiles, size_t n, uint32_t width, uint32_t height, void* packed,
                      std::string* err) override;
    bool render_views(const float* view_inv, uint32_t nviews, const float* proj_inv, uint32_t width, uint32_t height,
                      void* out, std::string* err) override;
    bool tile_costs(uint32_t width, uint32_t height, void* scratch, uint8_t* classes, size_t n,
                    std::string* err) override;
    bool view_cost(const float* view_inv, const float* proj_inv, uint32_t width, uint32_t height, void* scratch,
                   double* ms, std::string* err) override;
    bool unpack(const void* part, const gvrt_tile* tiles, size_t n, uint32_t width, uint32_t height, void* frame,
                std::string* err) override;
    bool sync_renders(std::string* err) override;
    double last_kernel_ms() override;

  private:
    bool nccl(ncclResult_t r, const char* what, std::string* err);
    GvrtApp& app_;
    int rank_, world_;
    ncclUniqueId id_;
    ncclComm_t comm_ = nullptr;
    void* stream_ = nullptr;  // hipStream_t
    bool bound_ = false;      // the app's handle renders on stream_
};

// SplitFrame over RCCL: the constructor gvrt_app split uses (rig: view inverses of the VIEWS layout)
class RcclSplitFrame : public SplitFrame {
  public:
    RcclSplitFrame(GvrtApp& app, int rank, int world, const ncclUniqueId& id, uint32_t width, uint32_t height,
                   Layout layout = COST_BANDS, const std::vector<gm::mat4>* rig = nullptr,
                   const gm::mat4* rig_proj_inv = nullptr);

  private:
    static std::vector<float> flat(const std::vector<gm::mat4>* rig);
};

}  // namespace gvrt_host
