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
//   gvrt_app cameras    [--width W --height H] [--transforms T]   (prints the camera matrices; no GPU)
//   gvrt_app png        OUT.png                                   (writes a test pattern; no GPU)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <sys/stat.h>

#include "gvrt_host.h"

using namespace gvrt_host;

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

// the presets of the Python app / bench: config-1 pinhole and the config-2 orbit camera
Camera preset_camera(const std::string& name, uint32_t w, uint32_t h) {
    Camera c;
    if (name == "config1") {
        c.setLookAt({0.0, 0.0, 3.0}, {0.0, 0.0, 0.0}, {0.0, 1.0, 0.0});
        c.setPerspective(FOV_Y, (double)w / h, NEAR_PLANE, FAR_PLANE);
    } else {
        const double el = 20.0 * M_PI / 180.0, az = 30.0 * M_PI / 180.0, r = 4.0;
        c.setLookAt({r * std::cos(el) * std::sin(az), r * std::sin(el), r * std::cos(el) * std::cos(az)},
                    {0.0, 0.0, 0.0}, {0.0, 1.0, 0.0});
        c.setPerspective(50.0, (double)w / h, NEAR_PLANE, FAR_PLANE);
    }
    return c;
}

void print_mat(const char* name, const std::array<float, 16>& m) {
    std::printf("%s", name);
    for (float v : m) std::printf(" %.9g", v);
    std::printf("\n");
}

int usage() {
    std::fprintf(stderr,
                 "usage: gvrt_app {render|eval|lightfield|hitcounts|bench|cameras|png} [--ply P] [--out D]\n"
                 "       [--width W] [--height H] [--camera orbit|config1] [--variant rq|rt] [--transforms T]\n"
                 "       [--duration S] [--warmup S] [--frametimes] [--split-cells N] [--build fast|quality]\n"
                 "       [--device I]\n");
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
        if (a.cmd == "cameras") {  // host-only: camera matrices as the C-ABI receives them
            for (const char* n : {"config1", "orbit"}) {
                const Camera c = preset_camera(n, W, H);
                print_mat((std::string(n) + "_view_inv").c_str(), c.matrices.view.inverse().colmajor());
                print_mat((std::string(n) + "_proj_inv").c_str(), c.matrices.perspective.inverse().colmajor());
            }
            Camera e;
            e.setPosition({0.5, -1.0, 2.0});
            e.setRotation({10.0, 20.0, 30.0});
            print_mat("euler_view", e.matrices.view.colmajor());
            if (a.has("transforms")) {
                CameraLoader l;
                std::string err;
                if (!l.loadNerfCameraData(a.get("transforms"), &err)) throw std::runtime_error(err);
                for (size_t i = 0; i < l.views.size(); ++i)
                    print_mat(("nerf_w2c_" + std::to_string(i)).c_str(), l.views[i].colmajor());
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
        ap.split_cells = (uint32_t)std::atoi(a.get("split-cells", "0").c_str());
        if (a.get("build", "fast") == "quality") {  // static-scene build: host binned SAH + SAH-optimal collapse
            ap.builder = 2;
            ap.collapse = 1;
        }
        const uint64_t m = app.prepare(ply, nullptr, &ap);
        const gvrt_stats st = app.stats();
        std::printf("prepared: %zu Gaussians, %llu after the enclosing pass; enclose %.3f ms, accel %.3f ms\n",
                    app.splats.size(), (unsigned long long)m, st.enclose_ms, st.accel_ms);
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
            const size_t n = app.computeGaussianLightField(out, W, H);
            std::printf("wrote %zu views + rayDirs.bin to %s\n", n, out.c_str());
        } else if (a.cmd == "hitcounts") {
            app.printRayHitCounts(cam, W, H, out + "/rayHitCountsOutput.txt");
            std::printf("wrote %s/rayHitCountsOutput.txt\n", out.c_str());
        } else if (a.cmd == "bench") {
            Benchmark b;
            b.duration = std::atof(a.get("duration", "10").c_str());
            b.warmup = std::atof(a.get("warmup", "1").c_str());
            b.outputFrameTimes = a.has("frametimes");
            b.filename = out + "/fps.txt";
            const double fps = app.benchmark(cam, W, H, b);
            b.saveResults();
            std::printf("frames : %zu\nfps    : %.2f\n", b.frameTimes.size(), fps);
        } else {
            return usage();
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "gvrt_app: %s\n", e.what());
        return 1;
    }
    return 0;
}
