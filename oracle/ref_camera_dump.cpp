// ref_camera_dump.cpp — test-infrastructure driver around the REFERENCE's own camera math, compiled
// from /root/reference by oracle/ref.mk into oracle/_ref/ (never committed, never shipped):
//   Camera (base/camera.hpp:31-58 updateViewMatrix, :124-141 rotateAxis, :157-182 setPerspective),
//   CameraLoader::loadNerfCameraData + c2wTow2cRT (base/LoadCamera.hpp:45-85, :124-147, nlohmann json),
//   glm::lookAt / glm::inverse / glm::perspective_Vulkan_no_depth_reverse
//   (external/glm/glm/gtc/matrix_transform.inl:276-290) — the vendored glm, with the reference's own
//   defines (base/VulkanRTBase.h:51-53).
// The light-field ring rig is VulkanFullRT::calculateGaussianLightFieldSamples
// (projects/VulkanFullRT/VulkanFullRT.cpp:1518-1604), whose translation unit does not compile on Linux
// (SURVEY §8c); its few lines of glm calls are restated here over the reference's Camera/glm headers.
//
// Protocol: one command per stdin line, floats given as C99 hex ("%a") so no decimal rounding enters;
// every matrix is printed as 16 uint32 hex words in glm memory order (column-major m[c][r]).
//   lookat ex ey ez cx cy cz ux uy uz          -> view, inverse(view)
//   persp fovy_deg aspect znear zfar            -> P = perspective_Vulkan_no_depth_reverse(radians(fovy)), inverse(P)
//   euler px py pz rx ry rz fov aspect zn zf    -> Camera: setPerspective, setPosition, setRotation;
//                                                  view, inverse(view), perspective, inverse(perspective)
//   nerf path width height znear zfar          -> per frame (setDatasetCamera(nerf, i, (float)width/height)):
//                                                  view, inverse(view), perspective, inverse(perspective)
//   lfring path.f32 n width height ncams       -> per camera inverse(lookAt), then inverse(persMat)
#include <cfloat>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "camera.hpp"

static float hf(const std::string& s) { return std::strtof(s.c_str(), nullptr); }

static void put(const glm::mat4& m) {
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) {
            uint32_t u;
            float f = m[c][r];
            std::memcpy(&u, &f, 4);
            std::printf("%08x%c", u, (c == 3 && r == 3) ? '\n' : ' ');
        }
}

int main() {
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream is(line);
        std::string cmd;
        is >> cmd;
        std::vector<std::string> a;
        for (std::string t; is >> t;) a.push_back(t);
        if (cmd == "lookat" && a.size() == 9) {
            glm::vec3 e(hf(a[0]), hf(a[1]), hf(a[2])), c(hf(a[3]), hf(a[4]), hf(a[5])), u(hf(a[6]), hf(a[7]), hf(a[8]));
            glm::mat4 v = glm::lookAt(e, c, u);
            put(v);
            put(glm::inverse(v));
        } else if (cmd == "persp" && a.size() == 4) {
            glm::mat4 p = glm::perspective_Vulkan_no_depth_reverse(glm::radians(hf(a[0])), hf(a[1]), hf(a[2]), hf(a[3]));
            put(p);
            put(glm::inverse(p));
        } else if (cmd == "euler" && a.size() == 10) {
            Camera cam;
            cam.setPerspective(hf(a[6]), hf(a[7]), hf(a[8]), hf(a[9]));
            cam.setPosition(glm::vec3(hf(a[0]), hf(a[1]), hf(a[2])));
            cam.setRotation(glm::vec3(hf(a[3]), hf(a[4]), hf(a[5])));
            put(cam.matrices.view);
            put(glm::inverse(cam.matrices.view));
            put(cam.matrices.perspective);
            put(glm::inverse(cam.matrices.perspective));
        } else if (cmd == "nerf" && a.size() == 5) {
            const uint32_t width = (uint32_t)std::atoi(a[1].c_str()), height = (uint32_t)std::atoi(a[2].c_str());
            Camera cam;
            cam.setNearFar(hf(a[3]), hf(a[4]));
            cam.loadDatasetCamera(nerf, a[0], width, height);
            const size_t nf = cam.getCamNames().size();
            std::printf("%zu\n", nf);
            for (uint32_t i = 0; i < nf; ++i) {
                cam.setDatasetCamera(nerf, i, (float)width / height);  // VulkanFullRT.cpp:2154
                put(cam.matrices.view);
                put(glm::inverse(cam.matrices.view));
                put(cam.matrices.perspective);
                put(glm::inverse(cam.matrices.perspective));
            }
        } else if (cmd == "lfring" && a.size() == 5) {
            const size_t n = (size_t)std::atoll(a[1].c_str());
            const unsigned width = (unsigned)std::atoi(a[2].c_str()), height = (unsigned)std::atoi(a[3].c_str());
            const unsigned cameraNum = (unsigned)std::atoi(a[4].c_str());
            std::vector<float> pos(3 * n);
            FILE* f = std::fopen(a[0].c_str(), "rb");
            if (!f || std::fread(pos.data(), 4, 3 * n, f) != 3 * n) return 3;
            std::fclose(f);
            // VulkanFullRT.cpp:1527-1563
            float minX, minY, minZ, maxX, maxY, maxZ;
            minX = minY = minZ = FLT_MAX;
            maxX = maxY = maxZ = FLT_MIN;
            for (size_t i = 0; i < n; i++) {
                float x = pos[i * 3], y = pos[i * 3 + 1], z = pos[i * 3 + 2];
                if (x < minX) minX = x;
                if (y < minY) minY = y;
                if (z < minZ) minZ = z;
                if (x > maxX) maxX = x;
                if (y > maxY) maxY = y;
                if (z > maxZ) maxZ = z;
            }
            glm::vec3 center = glm::vec3((minX + maxX) / 2, (minY + maxY) / 2, (minZ + maxZ) / 2);
            float candX = maxX - minX, candY = maxY - minY, candZ = maxZ - minZ;
            float maxR = std::max(std::max(candX, candY), candZ) / 2;
            glm::vec3 up = glm::vec3(0, 0, 1);
            std::vector<glm::vec3> cameraPos = {glm::vec3(center.x + maxR, center.y, center.z),
                                                glm::vec3(center.x, center.y + maxR, center.z),
                                                glm::vec3(center.x - maxR, center.y, center.z),
                                                glm::vec3(center.x, center.y - maxR, center.z)};
            for (unsigned i = 0; i < cameraNum; i++) put(glm::inverse(glm::lookAt(cameraPos[i % 4], center, up)));
            // :1596, :1604 — aspect is (float)(width / height), integer division (Q15)
            glm::mat4 persMat = glm::perspective_Vulkan_no_depth_reverse(glm::radians(135.0f), (float)(width / height),
                                                                         NEAR_PLANE, FAR_PLANE);
            put(glm::inverse(persMat));
        } else {
            std::fprintf(stderr, "bad command: %s\n", line.c_str());
            return 2;
        }
        std::fflush(stdout);
    }
    return 0;
}
