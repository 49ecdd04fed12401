// gvrt_host.h — C++ host layer around libgvrt.so: the reference application's own interfaces, kept
// intact on the host side (BASELINE.json north_star: "Host side stays C++ with the repo's
// Vulkan3DGRTModel ... loader and camera/benchmark interfaces intact, calling HIP through a thin C-ABI").
//
//   vk3DGRT::SplatSet / PLYLoader    base/Vulkan3DGRTModel.h:16-36, base/Vulkan3DGRTModel.cpp:7-125
//   Camera (N_IS_UP Euler camera)    base/camera.hpp:31-58, :157-182; glm lookAtRH, and
//                                    perspective_Vulkan_no_depth_reverse (matrix_transform.inl:276-290)
//   CameraLoader (NeRF transforms)   base/LoadCamera.hpp:57-85, :124-147
//   vks::Benchmark                   base/benchmark.hpp:22-104
//   GvrtApp (headless VulkanFullRT)  projects/VulkanFullRT/VulkanFullRT.cpp: prepare() :1990-2113,
//                                    draw() :2115, computeGaussianLightField() :1900-1976,
//                                    calculateGaussianLightFieldSamples() :1518-1628,
//                                    printRayHitCounts() :2182-2195, EVAL_QUALITY capture :2127-2161
//
// Nothing here computes a pixel: every pass is a gvrt_* call.  Matrices are row-major double here
// (m[row][col]) and handed to the C-ABI as column-major float, as updateUniformBuffer uploads glm's
// column-major mat4s (VulkanFullRT.cpp:1331-1349).
#pragma once
#include <array>
#include <chrono>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/gvrt.h"

namespace gvrt_host {

// base/Define.h:33-35
constexpr double FOV_Y = 39.6, NEAR_PLANE = 0.005, FAR_PLANE = 20.0;

using vec3 = std::array<double, 3>;
struct mat4 {
    double m[4][4];  // [row][col]
    static mat4 identity();
    mat4 operator*(const mat4& b) const;
    mat4 inverse() const;                   // Gauss-Jordan, partial pivoting
    std::array<float, 16> colmajor() const;  // glm memory order
};

mat4 look_at(const vec3& eye, const vec3& center, const vec3& up);
mat4 perspective_vulkan_no_depth_reverse(double fovy_rad, double aspect, double znear, double zfar);

// vk3DGRT::SplatSet: SoA host vectors, f_rest coefficient-major interleaved RGB
struct SplatSet {
    std::vector<float> positions, f_dc, f_rest, opacity, scale, rotation;
    size_t size() const { return positions.size() / 3; }
    gvrt_splats view() const;
};

// vk3DGRT::PLYLoader::loadPLYModel (the reorder of f_rest happens inside gvrt_ply_load)
struct PLYLoader {
    bool loadPLYModel(const std::string& filename, SplatSet& out, std::string* err = nullptr);
};

// base/camera.hpp Camera with the N_IS_UP axes of base/Define.h:63
struct Camera {
    vec3 rotation{0, 0, 0}, position{0, 0, 0};
    double fov = FOV_Y, znear = NEAR_PLANE, zfar = FAR_PLANE;
    struct {
        mat4 view = mat4::identity(), perspective = mat4::identity();
    } matrices;
    void updateViewMatrix();
    void setPosition(const vec3& p);
    void setRotation(const vec3& r);
    void setPerspective(double fov_deg, double aspect, double znear, double zfar);
    // look-at placement used by the light-field rig and the orbit / config-1 presets
    void setLookAt(const vec3& eye, const vec3& target, const vec3& up);
};

// CameraLoader::loadNerfCameraData + c2wTow2cRT: w2c view matrices of a transforms_*.json
struct CameraLoader {
    double camera_angle_x = 0.0;
    std::vector<mat4> views;
    bool loadNerfCameraData(const std::string& path, std::string* err = nullptr);
};

// vks::Benchmark
struct Benchmark {
    double warmup = 1.0, duration = 10.0;  // seconds
    std::string filename = "fps.txt";
    bool outputFrameTimes = false;
    std::string device = "unknown", driver = "unknown";
    std::vector<double> frameTimes;  // ms
    double runtime = 0.0;            // ms
    template <class F>
    double run(F&& frame);  // frame() renders and waits; returns fps
    bool saveResults() const;
};

// R8G8B8A8 PNG (stbi_write_png layout; stored deflate blocks, so no zlib dependency)
bool write_png(const std::string& path, const uint8_t* rgba, uint32_t width, uint32_t height);

// VulkanFullRT around one gvrt handle
class GvrtApp {
  public:
    explicit GvrtApp(int device = 0);
    ~GvrtApp();
    GvrtApp(const GvrtApp&) = delete;
    GvrtApp& operator=(const GvrtApp&) = delete;

    gvrt_render_params params;  // UniformDataStatic (VulkanUtils.h:50-61) + variant switches
    SplatSet splats;

    uint64_t prepare(const std::string& ply, const gvrt_enclosing_params* ep = nullptr,
                     const gvrt_accel_params* ap = nullptr);
    // draw(): one Particle Rendering pass; host outputs (rgba8 and/or hit counts may be null)
    void draw(const Camera& cam, uint32_t width, uint32_t height, uint8_t* rgba8, uint32_t* hit_counts = nullptr);
    // EVAL_QUALITY: r_<i>.png per NeRF camera; returns the number of views
    size_t evalCapture(const std::string& transforms, const std::string& out_dir, uint32_t width, uint32_t height);
    // calculateGaussianLightFieldSamples + computeGaussianLightField: 4-camera ring, one batched launch
    size_t computeGaussianLightField(const std::string& out_dir, uint32_t width, uint32_t height);
    // printRayHitCounts: "%u " per pixel, one row per line
    void printRayHitCounts(const Camera& cam, uint32_t width, uint32_t height, const std::string& path);
    // vks::Benchmark over device-resident frames
    double benchmark(const Camera& cam, uint32_t width, uint32_t height, Benchmark& b);

    gvrt_stats stats() const;
    gvrt_handle handle() const { return h_; }

  private:
    gvrt_handle h_ = nullptr;
    int device_ = 0;
};

// ray-traced light-field rig: viewInverse per camera and the shared projInverse (VulkanFullRT.cpp:1518-1628)
void lightfield_ring_rig(const SplatSet& s, uint32_t ncams, uint32_t width, uint32_t height,
                         std::vector<float>& view_inv, std::array<float, 16>& proj_inv);

template <class F>
double Benchmark::run(F&& frame) {
    using clk = std::chrono::high_resolution_clock;
    double tMeas = 0.0;
    while (tMeas < warmup * 1000.0) {  // benchmark.hpp:50-56
        const auto t0 = clk::now();
        frame();
        tMeas += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    }
    while (runtime < duration * 1000.0) {  // :60-66
        const auto t0 = clk::now();
        frame();
        const double dt = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        runtime += dt;
        frameTimes.push_back(dt);
    }
    return frameTimes.size() / (runtime / 1000.0);
}

}  // namespace gvrt_host
