// Compile-and-run check that the host layer keeps the reference's host interfaces (BASELINE.json
// north_star "loader and camera/benchmark interfaces intact"): every entry point is called with the
// reference's own argument types, and its member-function type is asserted to be the reference's
// signature with the Vulkan object types replaced by their HIP counterparts:
//   base/Vulkan3DGRTModel.h:15-52, base/LoadCamera.hpp:40-147, base/camera.hpp, base/benchmark.hpp:21-105.
// Built and run by tests/test_host_cpp.py (no GPU needed: the device calls are type-checked only).
#include <cstdio>
#include <functional>
#include <string>
#include <type_traits>

#include "gvrt_host.h"

using gvrt_host::Device;
using gvrt_host::Queue;
using vk3DGRT::Model;
using vk3DGRT::PLYLoader;
using vk3DGRT::SplatSet;

static_assert(std::is_same<decltype(&PLYLoader::loadPLYModel), bool (PLYLoader::*)(const char*, SplatSet&)>::value,
              "PLYLoader::loadPLYModel(const char*, SplatSet&)");
static_assert(std::is_same<decltype(&Model::load3DGRTModel), void (Model::*)(std::string, Device*)>::value,
              "Model::load3DGRTModel(std::string, vks::VulkanDevice* -> Device*)");
static_assert(std::is_same<decltype(&Model::allocateAttributeBuffers), void (Model::*)(Device*, Queue)>::value,
              "Model::allocateAttributeBuffers(VulkanDevice* -> Device*, VkQueue -> Queue)");
static_assert(std::is_same<decltype(Model::Attributes::count), int>::value, "Attributes::count");
static_assert(std::is_same<decltype(&SplatSet::size), size_t (SplatSet::*)() const>::value, "SplatSet::size");
static_assert(std::is_same<decltype(&CameraLoader::loadNerfCameraData),
                           void (CameraLoader::*)(const std::string&, uint32_t, uint32_t, float, float)>::value,
              "CameraLoader::loadNerfCameraData(const string&, uint32_t, uint32_t, float, float)");
static_assert(std::is_same<decltype(CameraLoader::fovy), float>::value, "CameraLoader::fovy");
static_assert(std::is_same<decltype(&vks::Benchmark::run),
                           void (vks::Benchmark::*)(std::function<void()>, gvrt_device_properties)>::value,
              "vks::Benchmark::run(std::function<void()>, VkPhysicalDeviceProperties -> gvrt_device_properties)");
static_assert(std::is_same<decltype(&vks::Benchmark::saveResults), void (vks::Benchmark::*)()>::value, "saveResults");
static_assert(std::is_same<decltype(vks::Benchmark::warmup), uint32_t>::value &&
                  std::is_same<decltype(vks::Benchmark::duration), uint32_t>::value,
              "Benchmark warmup / duration in whole seconds");
static_assert(std::is_same<decltype(&Camera::setPerspective), void (Camera::*)(float, float, float, float)>::value,
              "Camera::setPerspective");
static_assert(std::is_same<decltype(&Camera::setPosition), void (Camera::*)(gm::vec3)>::value, "Camera::setPosition");
static_assert(std::is_same<decltype(&Camera::setRotation), void (Camera::*)(gm::vec3)>::value, "Camera::setRotation");
static_assert(std::is_same<decltype(&Camera::setDatasetCamera), void (Camera::*)(DatasetType, uint32_t, float)>::value,
              "Camera::setDatasetCamera");
static_assert(std::is_same<decltype(&Camera::loadDatasetCamera),
                           void (Camera::*)(DatasetType, std::string, uint32_t, uint32_t)>::value,
              "Camera::loadDatasetCamera");
static_assert(std::is_same<decltype(&Camera::rotateAxis),
                           void (Camera::*)(float, gm::vec3*, gm::vec3*, gm::vec3*)>::value,
              "Camera::rotateAxis");

// the device-side calls, type-checked with the reference's argument expressions (not run without a GPU)
[[maybe_unused]] static void device_flow(Device* vulkanDevice, Queue queue, const char* ply) {
    Model gModel;
    gModel.load3DGRTModel(std::string(ply), vulkanDevice);
    gModel.allocateAttributeBuffers(vulkanDevice, queue);
    const void* p = gModel.positions.storageBuffer.buffer;
    (void)p;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    // PLYLoader with the reference's argument types
    SplatSet splatSet;
    PLYLoader plyLoader;
    if (!plyLoader.loadPLYModel(argv[1], splatSet)) return 3;
    // CameraLoader / Camera (VulkanFullRT's EVAL_QUALITY sequence)
    CameraLoader loader;
    const std::string path = argv[2];
    uint32_t width = 800, height = 800;
    loader.loadNerfCameraData(path, width, height, NEAR_PLANE, FAR_PLANE);
    Camera camera;
    camera.setNearFar(NEAR_PLANE, FAR_PLANE);
    camera.loadDatasetCamera(nerf, path, width, height);
    camera.setDatasetCamera(camera.dataType, 0, (float)width / height);
    // vks::Benchmark with a std::function<void()> frame
    vks::Benchmark benchmark;
    benchmark.warmup = 0;
    benchmark.duration = 1;
    benchmark.outputFrames = 5;
    gvrt_device_properties props{};
    std::snprintf(props.device_name, sizeof(props.device_name), "host-check");
    int frames = 0;
    benchmark.run([&] { ++frames; }, props);
    std::printf("splats %zu frames %zu cams %zu fovy %.6f bench %u %d\n", splatSet.size(), loader.nerfCameras.frames.size(),
                camera.getCamNames().size(), loader.fovy, benchmark.frameCount, frames);
    return benchmark.frameCount == 5 && frames == 5 ? 0 : 4;
}
