// gvrt_host.h — C++ host layer around libgvrt.so that keeps the reference application's own host
// interfaces intact (BASELINE.json north_star: "Host side stays C++ with the repo's Vulkan3DGRTModel ...
// loader and camera/benchmark interfaces intact, calling HIP through a thin C-ABI").  Same class
// names, member names and argument types as the reference; the Vulkan objects they carried become
// their HIP counterparts behind the C-ABI of include/gvrt.h:
//
//   vk3DGRT::SplatSet / PLYLoader / Model   base/Vulkan3DGRTModel.h:15-52, .cpp:7-222
//       vks::VulkanDevice* -> gvrt_host::Device* (one HIP device), VkQueue -> gvrt_host::Queue (a gvrt
//       handle: one HIP stream), vks::Buffer -> gvrt_host::Buffer (device pointer + bytes)
//   Camera (N_IS_UP Euler camera)           base/camera.hpp (whole public interface used off-window)
//   CameraLoader / CameraFrame / NerfCameraData   base/LoadCamera.hpp:22-147
//   vks::Benchmark                          base/benchmark.hpp:21-105
//       VkPhysicalDeviceProperties -> gvrt_device_properties (deviceName, driverVersion)
//   GvrtApp (headless VulkanFullRT)         projects/VulkanFullRT/VulkanFullRT.cpp: prepare() :1990-2113,
//       updateUniformBuffer() :1331-1349, draw() :2115, computeGaussianLightField() :1900-1976,
//       calculateGaussianLightFieldSamples() :1518-1604, printRayHitCounts() :2182-2195,
//       EVAL_QUALITY capture :2127-2161
//
// Camera math is float32 in glm's operation order (gvrt_math.h), so the matrices uploaded per frame
// are bit-identical to the reference's (tests/test_host_cpp.py checks them against the reference's
// camera.hpp / LoadCamera.hpp / glm compiled from its sources).  Nothing here computes a pixel: every
// pass is a gvrt_* call.  Failures throw std::runtime_error where the reference asserts or exits.
#pragma once
#include <array>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../../include/gvrt.h"
#include "gvrt_math.h"

// base/Define.h:33-35
constexpr float FOV_Y = 39.6f;
constexpr float NEAR_PLANE = 0.005f;
constexpr float FAR_PLANE = 20.00f;

// base/LoadCamera.hpp:24
enum DatasetType { none, nerf, collmap };

namespace gvrt_host {

// vks::VulkanDevice analogue: one HIP device, its identity for the benchmark report
struct Device {
    int ordinal = 0;
    gvrt_device_properties properties{};
    explicit Device(int ordinal = 0);
};

// VkQueue analogue: a gvrt handle is bound to one device and owns one HIP stream (include/gvrt.h)
using Queue = gvrt_handle;

// vks::Buffer analogue: a device allocation owned by the handle (not freed by the holder)
struct Buffer {
    const void* buffer = nullptr;
    uint64_t size = 0;  // bytes
};

}  // namespace gvrt_host

namespace vk3DGRT {

// base/Vulkan3DGRTModel.h:16-28
struct SplatSet {
    std::vector<float> positions;  // x,y,z
    std::vector<float> f_dc;       // 3 per point
    std::vector<float> f_rest;     // 45 per point, coefficient-major interleaved RGB (loader reorders)
    std::vector<float> opacity;    // 1 per point
    std::vector<float> scale;      // 3 per point
    std::vector<float> rotation;   // 4 per point, w,x,y,z
    inline size_t size() const { return positions.size() / 3; }
};

// base/Vulkan3DGRTModel.h:30-36 (the f_rest reorder, .cpp:70-77, happens inside gvrt_ply_load)
class PLYLoader {
  public:
    PLYLoader() {}
    ~PLYLoader() {}
    bool loadPLYModel(const char* filename, SplatSet& output);
};

// base/Vulkan3DGRTModel.h:38-52
class Model {
  public:
    Model() {}
    ~Model() {}

    SplatSet splatSet;

    struct Attributes {
        int count = 0;
        gvrt_host::Buffer storageBuffer;
    } positions, rotations, scales, densities, vertices, indices, featuresAlbedo, featuresSpecular;

    // .cpp:126-161: .ply only; an unsupported or missing extension throws (the reference exitFatal()s)
    void load3DGRTModel(std::string filename, gvrt_host::Device* device);
    // .cpp:163-222: the six SoA arrays to device memory of `queue`'s device (gvrt_load_splats); vertices /
    // indices keep the reference's counts (36N floats / 60N indices) and get their device buffers when the
    // enclosing pass emits the proxy soup (attachEnclosingBuffers)
    void allocateAttributeBuffers(gvrt_host::Device* device, gvrt_host::Queue queue);
    void attachEnclosingBuffers(gvrt_host::Queue queue);
};

}  // namespace vk3DGRT

// base/LoadCamera.hpp:26-38
struct CameraFrame {
    std::string filePath;
    gm::mat4 transformMatrix;
    gm::quat rotation;
    gm::vec3 position;
};

struct NerfCameraData {
    float cameraAngleX = 0.0f;
    gm::mat4 projectionMatrix;
    std::vector<CameraFrame> frames;
    std::vector<gm::vec3> centers;
};

// base/LoadCamera.hpp:40-147
class CameraLoader {
  private:
    void calcIntrinsics(float cameraAngleX, uint32_t width, uint32_t height, float nearPlane, float farPlane);
    void c2wTow2cRT(CameraFrame& frame);

  public:
    NerfCameraData nerfCameras;
    float fovy = 0.0f;
    std::vector<std::string> camNames;

    // throws std::runtime_error("Failed to open file : ...") as loadJsonFromFile does
    void loadNerfCameraData(const std::string& jsonPath, uint32_t width, uint32_t height, float znear, float zfar);
    void PrintCameraData(const NerfCameraData& data);
};

// base/camera.hpp (N_IS_UP, USE_CORRECT_VULKAN_PERSPECTIVE_IHM)
class Camera {
  private:
    float fov = FOV_Y;
    float znear = NEAR_PLANE, zfar = FAR_PLANE;
    CameraLoader cameraLoader;
    void updateViewMatrix();

  public:
    enum CameraType { lookat, firstperson, SG_camera, cameraSize };
    CameraType type = CameraType::lookat;
    gm::vec3 rotation = gm::vec3();
    gm::vec3 position = gm::vec3();
    gm::vec4 viewPos = gm::vec4();
    DatasetType dataType = none;

    float rotationSpeed = 1.0f;
    float movementSpeed = 15.0f;

    bool updated = true;
    bool flipY = false;

    struct {
        gm::mat4 perspective;
        gm::mat4 view;
    } matrices;

    struct {
        bool left = false;
        bool right = false;
        bool up = false;
        bool down = false;
        bool forward = false;
        bool backward = false;
    } keys;

    const std::vector<std::string> getCamNames() { return cameraLoader.camNames; }
    void setNearFar(float _znear, float _zfar);
    void setNerfCamera(uint32_t idx);
    void setDatasetCamera(DatasetType type, uint32_t idx, float aspect);
    void loadDatasetCamera(DatasetType type, std::string path, uint32_t width, uint32_t height);
    void rotateAxis(float rad_angle, gm::vec3* u, gm::vec3* v, gm::vec3* n);
    bool moving() { return keys.left || keys.right || keys.up || keys.down || keys.forward || keys.backward; }
    float getNearClip() { return znear; }
    float getFarClip() { return zfar; }
    float getFov() { return fov; }
    void setPerspective(float fov, float aspect, float znear, float zfar);
    void updateAspectRatio(float aspect);
    void setPosition(gm::vec3 position);
    void setRotation(gm::vec3 rotation);
    void rotate(gm::vec3 delta);
    void setTranslation(gm::vec3 translation);
    void translate(gm::vec3 delta);
    void setRotationSpeed(float rotationSpeed) { this->rotationSpeed = rotationSpeed; }
    void setMovementSpeed(float movementSpeed) { this->movementSpeed = movementSpeed; }
    void update(float deltaTime);  // keyboard movement (firstperson / SG_camera), then updateViewMatrix

    // headless addition (not in camera.hpp): glm::lookAt placement for the bench / test presets
    void setLookAt(const gm::vec3& eye, const gm::vec3& target, const gm::vec3& up);
};

namespace vks {

// base/benchmark.hpp:21-105
class Benchmark {
  private:
    gvrt_device_properties deviceProps{};

  public:
    bool active = false;
    bool outputFrameTimes = false;
    int outputFrames = -1;  // -1 means no frames limit
    uint32_t warmup = 1;    // seconds
    uint32_t duration = 10; // seconds
    std::vector<double> frameTimes;
    std::string filename = "fps.txt";

    double runtime = 0.0;
    uint32_t frameCount = 0;

    void run(std::function<void()> renderFunc, gvrt_device_properties deviceProps);
    void saveResults();
};

}  // namespace vks

namespace gvrt_host {

// R8G8B8A8 PNG (stbi_write_png layout; stored deflate blocks, so no zlib dependency)
bool write_png(const std::string& path, const uint8_t* rgba, uint32_t width, uint32_t height);

// the presets of the Python app / bench: config-1 pinhole and the config-2 orbit camera
Camera preset_camera(const std::string& name, uint32_t width, uint32_t height);
gm::vec3 orbit_eye(float radius, float elevation_deg, float azimuth_deg);

// VulkanFullRT around one gvrt handle (headless: frames go to host / device buffers, PNG files)
class GvrtApp {
  public:
    explicit GvrtApp(int device = 0);
    ~GvrtApp();
    GvrtApp(const GvrtApp&) = delete;
    GvrtApp& operator=(const GvrtApp&) = delete;

    Device device;
    vk3DGRT::Model gModel;
    Camera camera;
    vks::Benchmark benchmark;
    gvrt_render_params params;  // UniformDataStatic (VulkanUtils.h:50-61) + variant switches

    struct {
        gm::mat4 viewInverse;
        gm::mat4 projInverse;
    } uniformDataDynamic;  // VulkanUtils.h:35-39

    struct {
        uint32_t samplingCameraNum = 4;  // VulkanFullRT.cpp:169-171
        uint32_t sampleImageWidth = 180;
        uint32_t sampleImageHeight = 180;
        std::vector<gm::mat4> viewInverse;
        gm::mat4 projInverse;
    } gaussianLightField;

    // prepare(): load3DGRTModel, allocateAttributeBuffers, Gaussian Enclosing pass, acceleration structure
    uint64_t prepare(const std::string& ply, const gvrt_enclosing_params* ep = nullptr,
                     const gvrt_accel_params* ap = nullptr);
    // updateUniformBuffer(): viewInverse / projInverse of `cam` (VulkanFullRT.cpp:1342-1343)
    void updateUniformBuffer(const Camera& cam);
    // draw(): one Particle Rendering pass with uniformDataDynamic; host outputs (may be null)
    void draw(uint32_t width, uint32_t height, uint8_t* rgba8, uint32_t* hit_counts = nullptr);
    void draw(const Camera& cam, uint32_t width, uint32_t height, uint8_t* rgba8, uint32_t* hit_counts = nullptr);
    // EVAL_QUALITY: camera.loadDatasetCamera + setDatasetCamera per view, r_<i>.png; returns the views
    size_t evalCapture(const std::string& transforms, const std::string& out_dir, uint32_t width, uint32_t height);
    void calculateGaussianLightFieldSamples();
    // computeGaussianLightField: 4-camera ring, one batched launch, PNG per view + rayDirs.bin
    size_t computeGaussianLightField(const std::string& out_dir);
    // printRayHitCounts: "%u " per pixel, one row per line
    void printRayHitCounts(const Camera& cam, uint32_t width, uint32_t height, const std::string& path);
    // vks::Benchmark over device-resident frames; returns fps
    double runBenchmark(const Camera& cam, uint32_t width, uint32_t height);

    gvrt_stats stats() const;
    gvrt_handle handle() const { return h_; }

  private:
    gvrt_handle h_ = nullptr;
};

// calculateGaussianLightFieldSamples as a free function: viewInverse per camera (column-major floats)
// and the shared projInverse (VulkanFullRT.cpp:1518-1604)
void lightfield_ring_rig(const vk3DGRT::SplatSet& s, uint32_t ncams, uint32_t width, uint32_t height,
                         std::vector<gm::mat4>& view_inv, gm::mat4& proj_inv);

}  // namespace gvrt_host
