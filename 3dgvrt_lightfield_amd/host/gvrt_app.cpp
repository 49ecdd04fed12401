// gvrt_app — the headless VulkanFullRT analogue in C++ (SURVEY §8b "gvrt_app"): prepare() -> load PLY,
// Gaussian Enclosing pass, acceleration structure; then one of the reference app's flows around the
// Particle Rendering pass.  The window / swapchain / UI of VulkanFullRT are out of scope; frames go to
// PNG files instead of the swapchain image.
//
//   gvrt_app render     --ply P [--camera orbit|config1] [--width W --height H] [--variant rq|rt] --out D
//   gvrt_app eval       --ply P --transforms transforms_val.json [--width 800 --height 800] --out D
//   gvrt_app lightfield --ply P [--width 180 --height 180] --out D          (computeGaussianLightField)
//   gvrt_app hitcounts  --ply P [...] --out D                                (printRayHitCounts)
//   gvrt_app bench      --ply P [--duration 10 --warmup 1 --frametimes] --out D   (vks::Benchmark, fps.txt)
//   gvrt_app split      --ply P --rank R --world N --id-file F [--frames K] [--layout cost-bands|blocks] --out D
//                       (one process per GPU: this rank's tiles of each frame, RCCL gather to rank 0, gvrt_rccl.h;
//                        rank 0 writes split_frame.png, checks it against a one-GPU render of the same frame and
//                        prints one JSON line)
//   gvrt_app cameras    [--width W --height H] [--transforms T]   (prints the camera matrices; no GPU)
//   gvrt_app png        OUT.png                                   (writes a test pattern; no GPU)
//   gvrt_app split      ... --layout views [--views V] (config 5: the views of a V-camera light-field rig split
//                       over the ranks by cost, each view gathered whole to rank 0; checked against one batched
//                       render of the whole rig on rank 0's GPU)
//   gvrt_app views      --costs c0,c1,... --world N (the cost-balanced view assignment, one rank per line; no GPU)
//   gvrt_app tiles      --rank R --world N [--width W --height H] [--layout blocks|bands --costs F]
//                       (this rank's split tile list; F: raw uint8 cost classes [ty][tx]; no GPU)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <sys/stat.h>

#include "gvrt_host.h"
#include "gvrt_rccl.h"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <vector>

using gvrt_host::GvrtApp;
using gvrt_host::preset_camera;
using gvrt_host::write_png;

namespace {

struct Args {
    std::string cmd;
    std::map<std::string, std::string> kv;
    std::string get(const std::string& k, const std::string& d = "") const {
        auto it = kv.find(k);
        return it == kv.end() ? d : it->second;
    }
    bool has(const std::string& k) const { return kv.count(k) != 0; }
};

Args parse(int argc, char** argv) {
    Args a;
    if (argc > 1) a.cmd = argv[1];
    for (int i = 2; i < argc; ++i) {
        std::string k = argv[i];
        if (k.rfind("--", 0) == 0) {
            k = k.substr(2);
            if (i + 1 < argc && std::strncmp(argv[i + 1], "--", 2) != 0) a.kv[k] = argv[++i];
            else a.kv[k] = "1";
        } else {
            a.kv["_pos"] = k;
        }
    }
    return a;
}

// matrices as 16 uint32 hex words in glm memory order (bit-exact comparison with the reference's)
void print_mat(const std::string& name, const gm::mat4& m) {
    std::printf("%s", name.c_str());
    for (int i = 0; i < 16; ++i) {
        uint32_t u;
        std::memcpy(&u, m.data() + i, 4);
        std::printf(" %08x", u);
    }
    std::printf("\n");
}

gm::vec3 parse_vec3(const std::string& s) {
    gm::vec3 v;
    if (std::sscanf(s.c_str(), "%f,%f,%f", &v.x, &v.y, &v.z) != 3) throw std::runtime_error("expected x,y,z: " + s);
    return v;
}

int usage() {
    std::fprintf(stderr,
                 "usage: gvrt_app {render|eval|lightfield|hitcounts|bench|split|views|tiles|cameras|png} [--ply P] [--out D]\n"
                 "       [--width W] [--height H] [--camera orbit|config1] [--variant rq|rt] [--transforms T]\n"
                 "       [--duration S] [--warmup S] [--frametimes] [--split-cells N] [--split-min-span N] [--build fast|quality]\n"
                 "       [--device I] [--rank R --world N --id-file F --frames K --layout cost-bands|blocks|views --views V]\n"
                 "       [--costs c0,c1,... (views)]\n");
    return 2;
}

}  // namespace

int main(int argc, char** argv) {
    const Args a = parse(argc, argv);
    if (a.cmd.empty() || a.cmd == "--help" || a.cmd == "-h" || a.has("help")) return usage();
    const uint32_t W = (uint32_t)std::atoi(a.get("width", a.cmd == "eval" ? "800" : a.cmd == "lightfield" ? "180" : "256").c_str());
    const uint32_t H = (uint32_t)std::atoi(a.get("height", a.cmd == "eval" ? "800" : a.cmd == "lightfield" ? "180" : "256").c_str());
    try {
        if (a.cmd == "png") {  // host-only: PNG writer check
            const std::string out = a.get("_pos", "test.png");
            std::vector<uint8_t> img((size_t)4 * W * H);
            for (uint32_t y = 0; y < H; ++y)
                for (uint32_t x = 0; x < W; ++x) {
                    uint8_t* p = &img[((size_t)y * W + x) * 4];
                    p[0] = (uint8_t)(x * 255 / (W > 1 ? W - 1 : 1));
                    p[1] = (uint8_t)(y * 255 / (H > 1 ? H - 1 : 1));
                    p[2] = (uint8_t)((x ^ y) & 0xFF);
                    p[3] = (uint8_t)(255 - ((x + y) & 0x7F));
                }
            return write_png(out, img.data(), W, H) ? 0 : 1;
        }
        if (a.cmd == "tiles") {  // host-only: the tile split of gvrt_rccl.h, "tx ty cam" per line
            const int rank = std::atoi(a.get("rank", "0").c_str()), world = std::atoi(a.get("world", "1").c_str());
            std::vector<gvrt_tile> tl;
            if (a.get("layout", "blocks") == "bands") {
                std::vector<uint8_t> cls;
                if (a.has("costs")) {
                    FILE* f = std::fopen(a.get("costs").c_str(), "rb");
                    if (!f) throw std::runtime_error("cannot open " + a.get("costs"));
                    cls.resize((size_t)((W + 7) / 8) * ((H + 7) / 8));
                    const size_t got = std::fread(cls.data(), 1, cls.size(), f);
                    std::fclose(f);
                    if (got != cls.size()) throw std::runtime_error("cost file: one class byte per tile");
                }
                tl = gvrt_host::band_tiles(W, H, world, cls.empty() ? nullptr : cls.data())[rank];
            } else {
                tl = gvrt_host::rank_tiles(W, H, 1, rank, world);
            }
            for (const gvrt_tile& t : tl) std::printf("%u %u %u\n", t.tx, t.ty, t.cam);
            return 0;
        }
        if (a.cmd == "views") {  // host-only: the cost-balanced view split (balanced_views), one rank per line
            std::vector<double> costs;
            std::string c = a.get("costs");
            for (size_t p = 0; p < c.size();) {
                size_t q = c.find(',', p);
                if (q == std::string::npos) q = c.size();
                costs.push_back(std::strtod(c.substr(p, q - p).c_str(), nullptr));
                p = q + 1;
            }
            const int world = std::atoi(a.get("world", "1").c_str());
            if (world < 1) throw std::runtime_error("--world must be >= 1");
            for (const auto& g : gvrt_host::balanced_views(costs, world)) {
                for (size_t i = 0; i < g.size(); ++i) std::printf(i ? " %u" : "%u", g[i]);
                std::printf("\n");
            }
            return 0;
        }
        if (a.cmd == "cameras") {  // host-only: the camera matrices the C-ABI receives (uint32 bit patterns)
            for (const char* n : {"config1", "orbit"}) {
                const Camera c = preset_camera(n, W, H);
                print_mat(std::string(n) + "_view_inv", gm::inverse(c.matrices.view));
                print_mat(std::string(n) + "_proj_inv", gm::inverse(c.matrices.perspective));
            }
            Camera e;  // camera.hpp Euler camera, as VulkanFullRT drives it
            e.setPerspective(FOV_Y, (float)W / H, NEAR_PLANE, FAR_PLANE);
            e.setPosition(parse_vec3(a.get("position", "0.5,-1,2")));
            e.setRotation(parse_vec3(a.get("rotation", "10,20,30")));
            print_mat("euler_view", e.matrices.view);
            print_mat("euler_view_inv", gm::inverse(e.matrices.view));
            print_mat("euler_proj_inv", gm::inverse(e.matrices.perspective));
            if (a.has("transforms")) {  // EVAL_QUALITY sequence: loadDatasetCamera + setDatasetCamera
                Camera c;
                c.setNearFar(NEAR_PLANE, FAR_PLANE);
                c.loadDatasetCamera(nerf, a.get("transforms"), W, H);
                for (uint32_t i = 0; i < c.getCamNames().size(); ++i) {
                    c.setDatasetCamera(c.dataType, i, (float)W / H);
                    print_mat("nerf_w2c_" + std::to_string(i), c.matrices.view);
                    print_mat("nerf_view_inv_" + std::to_string(i), gm::inverse(c.matrices.view));
                    print_mat("nerf_proj_inv_" + std::to_string(i), gm::inverse(c.matrices.perspective));
                }
            }
            if (a.has("ply")) {  // light-field ring rig of the scene (calculateGaussianLightFieldSamples)
                vk3DGRT::SplatSet s;
                if (!vk3DGRT::PLYLoader().loadPLYModel(a.get("ply").c_str(), s)) throw std::runtime_error("cannot load ply");
                std::vector<gm::mat4> vi;
                gm::mat4 pi;
                gvrt_host::lightfield_ring_rig(s, 4, W, H, vi, pi);
                for (size_t i = 0; i < vi.size(); ++i) print_mat("ring_view_inv_" + std::to_string(i), vi[i]);
                print_mat("ring_proj_inv", pi);
            }
            return 0;
        }
        const std::string ply = a.get("ply");
        if (ply.empty()) return usage();
        const std::string out = a.get("out", "gvrt_out");
        GvrtApp app(std::atoi(a.get("device", "0").c_str()));
        if (a.get("variant", "rq") == "rt") {  // RT pipeline raygen: pixel centre, alpha starts at 1 (Q10, Q11)
            app.params.pixel_offset = 0.5f;
            app.params.alpha_init = 1.0f;
        }
        gvrt_accel_params ap;
        gvrt_default_accel_params(&ap);
        const bool quality = a.get("build", "fast") == "quality";
        // quality (static-scene) build: device binned SAH + SAH-optimal collapse, and the SplitBLAS grid (10 cells,
        // base/Define.h:45-47) applied to the proxies that span 3+ cells (renderer.QUALITY_BUILD in Python)
        ap.split_cells = (uint32_t)std::atoi(a.get("split-cells", quality ? "10" : "0").c_str());
        ap.split_min_span = (uint32_t)std::atoi(a.get("split-min-span", quality ? "3" : "0").c_str());
        if (quality) {
            ap.builder = 2;
            ap.collapse = 1;
        }
        const uint64_t m = app.prepare(ply, nullptr, &ap);
        const gvrt_stats st = app.stats();
        std::printf("prepared: %zu Gaussians, %llu after the enclosing pass; enclose %.3f ms, accel %.3f ms\n",
                    app.gModel.splatSet.size(), (unsigned long long)m, st.enclose_ms, st.accel_ms);
        ::mkdir(out.c_str(), 0755);
        const Camera cam = preset_camera(a.get("camera", "orbit"), W, H);
        if (a.cmd == "render") {
            std::vector<uint8_t> img((size_t)4 * W * H);
            app.draw(cam, W, H, img.data());
            if (!write_png(out + "/frame.png", img.data(), W, H)) throw std::runtime_error("cannot write frame.png");
            std::printf("render %.3f ms -> %s/frame.png\n", app.stats().render_ms, out.c_str());
        } else if (a.cmd == "eval") {
            const size_t n = app.evalCapture(a.get("transforms"), out, W, H);
            std::printf("wrote %zu views to %s\n", n, out.c_str());
        } else if (a.cmd == "lightfield") {
            app.gaussianLightField.sampleImageWidth = W;
            app.gaussianLightField.sampleImageHeight = H;
            const size_t n = app.computeGaussianLightField(out);
            std::printf("wrote %zu views + rayDirs.bin to %s\n", n, out.c_str());
        } else if (a.cmd == "hitcounts") {
            app.printRayHitCounts(cam, W, H, out + "/rayHitCountsOutput.txt");
            std::printf("wrote %s/rayHitCountsOutput.txt\n", out.c_str());
        } else if (a.cmd == "split") {
            const int rank = std::atoi(a.get("rank", "0").c_str()), world = std::atoi(a.get("world", "1").c_str());
            const int frames = std::atoi(a.get("frames", "10").c_str());
            const std::string lay = a.get("layout", "cost-bands");
            const bool by_views = lay == "views";
            ncclUniqueId id;
            std::string err;
            if (gvrt_host::rccl_rendezvous(a.get("id-file", out + "/rccl.id"), rank, &id, &err) != GVRT_OK)
                throw std::runtime_error(err);
            app.updateUniformBuffer(cam);
            // --layout views: config 5, the views of a light-field rig (calculateGaussianLightFieldSamples with
            // --views cameras, the light-field raygen's pixel centres and alpha start) split over the ranks
            std::vector<gm::mat4> rig;
            gm::mat4 rig_pi{};
            uint32_t nv = 1;
            if (by_views) {
                nv = (uint32_t)std::atoi(a.get("views", "16").c_str());
                gvrt_host::lightfield_ring_rig(app.gModel.splatSet, nv, W, H, rig, rig_pi);
                app.params.pixel_offset = 0.5f;
                app.params.alpha_init = 1.0f;
            }
            if (a.has("tile-order-off")) {  // fault injection: no cost-ordered launch, so no tile costs to read
                if (gvrt_set_option(app.handle(), GVRT_OPT_TILE_ORDER, 0) != GVRT_OK) throw std::runtime_error("option");
            }
            const size_t frame_bytes = (size_t)4 * W * H * nv;
            void* frame = nullptr;
            if (rank == 0 && hipMalloc(&frame, frame_bytes) != hipSuccess) throw std::runtime_error("frame alloc");
            std::vector<uint8_t> got(frame_bytes), one(frame_bytes);
            double ms = 0.0;
            std::string assignment;
            {
                const auto layout = by_views ? gvrt_host::SplitFrame::VIEWS
                                    : lay == "blocks" ? gvrt_host::SplitFrame::BLOCKS
                                                      : gvrt_host::SplitFrame::COST_BANDS;
                gvrt_host::RcclSplitFrame sf(app, rank, world, id, W, H, layout, by_views ? &rig : nullptr,
                                         by_views ? &rig_pi : nullptr);
                if (sf.status() != GVRT_OK) throw std::runtime_error("SplitFrame: " + sf.error());
                if (sf.draw(frame) != GVRT_OK || sf.sync() != GVRT_OK) throw std::runtime_error(sf.error());  // warm-up
                const auto t0 = std::chrono::steady_clock::now();
                for (int k = 0; k < frames; ++k)
                    if (sf.draw(frame) != GVRT_OK) throw std::runtime_error(sf.error());
                if (sf.sync() != GVRT_OK) throw std::runtime_error(sf.error());
                ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / frames;
                if (rank == 0 && hipMemcpy(got.data(), frame, got.size(), hipMemcpyDeviceToHost) != hipSuccess)
                    throw std::runtime_error("frame readback");
                for (size_t r = 0; r < sf.views().size(); ++r) {
                    assignment += r ? ", [" : "[";
                    for (size_t i = 0; i < sf.views()[r].size(); ++i)
                        assignment += (i ? ", " : "") + std::to_string(sf.views()[r][i]);
                    assignment += "]";
                }
            }
            if (rank == 0) {
                (void)hipFree(frame);
                if (by_views) {  // the whole rig in one batched launch on this GPU alone
                    std::vector<float> vis;
                    for (const gm::mat4& m : rig) vis.insert(vis.end(), m.data(), m.data() + 16);
                    gvrt_image img{one.data(), nullptr, nullptr, nullptr, 0, 0};
                    if (gvrt_render(app.handle(), &app.params, vis.data(), rig_pi.data(), W, H, nv, nullptr, 0, &img) !=
                        GVRT_OK)
                        throw std::runtime_error(std::string("gvrt_render: ") + gvrt_last_error(app.handle()));
                } else {
                    app.draw(cam, W, H, one.data());  // the same frame on this GPU alone
                }
                const bool same = got == one;
                if (!write_png(out + "/split_frame.png", got.data(), W, H)) throw std::runtime_error("cannot write png");
                std::printf("{\"world\": %d, \"frames\": %d, \"views\": %u, \"ms_per_frame\": %.4f, "
                            "\"identical_to_one_gpu\": %s, \"assignment\": [%s]}\n",
                            world, frames, nv, ms, same ? "true" : "false", assignment.c_str());
                if (!same) return 3;
            }
        } else if (a.cmd == "bench") {  // vks::Benchmark (seconds are whole, as benchmark.hpp's uint32_t)
            vks::Benchmark& b = app.benchmark;
            b.duration = (uint32_t)std::atoi(a.get("duration", "10").c_str());
            b.warmup = (uint32_t)std::atoi(a.get("warmup", "1").c_str());
            b.outputFrameTimes = a.has("frametimes");
            b.filename = out + "/fps.txt";
            app.runBenchmark(cam, W, H);
            b.saveResults();
        } else {
            return usage();
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "gvrt_app: %s\n", e.what());
        return 1;
    }
    return 0;
}
