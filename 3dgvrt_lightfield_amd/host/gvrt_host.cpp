// gvrt_host.cpp — implementation of the C++ host layer (gvrt_host.h).  Reference file:line per class
// in the header; the Python mirror (camera.py, app.py) follows the same float32 formulas.
#include "gvrt_host.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cctype>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <map>
#include <numeric>
#include <sstream>
#include <stdexcept>
#include <sys/stat.h>

namespace {

void check(gvrt_status s, gvrt_handle h, const char* what) {
    if (s != GVRT_OK) throw std::runtime_error(std::string(what) + ": " + gvrt_last_error(h));
}

void make_dir(const std::string& d) { ::mkdir(d.c_str(), 0755); }

}  // namespace

namespace {
struct JVal {
    enum Kind { NUL, NUM, STR, ARR, OBJ, BOOL } kind = NUL;
    double num = 0.0;
    std::string str;
    std::vector<JVal> arr;
    std::map<std::string, JVal> obj;
};

struct JParser {
    const std::string& s;
    size_t i = 0;
    explicit JParser(const std::string& t) : s(t) {}
    void ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
    }
    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("JSON: ") + what + " at offset " + std::to_string(i));
    }
    std::string string() {
        if (s[i] != '"') fail("expected string");
        ++i;
        std::string out;
        while (i < s.size() && s[i] != '"') {
            if (s[i] == '\\' && i + 1 < s.size()) {
                const char e = s[++i];
                out += e == 'n' ? '\n' : e == 't' ? '\t' : e;  // \uXXXX kept verbatim (paths only)
            } else {
                out += s[i];
            }
            ++i;
        }
        if (i >= s.size()) fail("unterminated string");
        ++i;
        return out;
    }
    JVal value() {
        ws();
        if (i >= s.size()) fail("unexpected end");
        JVal v;
        const char c = s[i];
        if (c == '{') {
            v.kind = JVal::OBJ;
            ++i;
            ws();
            if (s[i] == '}') {
                ++i;
                return v;
            }
            while (true) {
                ws();
                const std::string k = string();
                ws();
                if (s[i] != ':') fail("expected ':'");
                ++i;
                v.obj[k] = value();
                ws();
                if (s[i] == ',') {
                    ++i;
                    continue;
                }
                if (s[i] == '}') {
                    ++i;
                    return v;
                }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.kind = JVal::ARR;
            ++i;
            ws();
            if (s[i] == ']') {
                ++i;
                return v;
            }
            while (true) {
                v.arr.push_back(value());
                ws();
                if (s[i] == ',') {
                    ++i;
                    continue;
                }
                if (s[i] == ']') {
                    ++i;
                    return v;
                }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.kind = JVal::STR;
            v.str = string();
            return v;
        }
        if (s.compare(i, 4, "true") == 0 || s.compare(i, 5, "false") == 0) {
            v.kind = JVal::BOOL;
            v.num = s[i] == 't';
            i += s[i] == 't' ? 4 : 5;
            return v;
        }
        if (s.compare(i, 4, "null") == 0) {
            i += 4;
            return v;
        }
        char* end = nullptr;
        v.num = std::strtod(s.c_str() + i, &end);
        if (end == s.c_str() + i) fail("bad value");
        v.kind = JVal::NUM;
        i = (size_t)(end - s.c_str());
        return v;
    }
};
}  // namespace

// ================================================================================== gvrt_host::Device
namespace gvrt_host {
Device::Device(int ord) : ordinal(ord) {
    if (gvrt_get_device_properties(ord, &properties) != GVRT_OK)
        throw std::runtime_error(std::string("gvrt_get_device_properties: ") + gvrt_last_error(nullptr));
}
}  // namespace gvrt_host

// ================================================================================== vk3DGRT
namespace vk3DGRT {

bool PLYLoader::loadPLYModel(const char* filename, SplatSet& output) {
    gvrt_splat_buffers b{};
    if (gvrt_ply_load(filename, &b) != GVRT_OK) {
        std::fprintf(stderr, "PLYLoader: %s\n", gvrt_last_error(nullptr));
        return false;
    }
    const size_t n = b.n;
    auto take = [n](const float* p, size_t k) { return std::vector<float>(p, p + n * k); };
    output.positions = take(b.positions, 3);
    output.f_dc = take(b.f_dc, 3);
    output.f_rest = take(b.f_rest, 45);
    output.opacity = take(b.opacity, 1);
    output.scale = take(b.scale, 3);
    output.rotation = take(b.rotation, 4);
    gvrt_ply_free(&b);
    return true;
}

void Model::load3DGRTModel(std::string filename, gvrt_host::Device* /*device*/) {
    const size_t dot = filename.find_last_of('.');
    if (dot == std::string::npos) throw std::runtime_error("Extension not found");
    const std::string ext = filename.substr(dot + 1);
    if (ext != "ply") throw std::runtime_error("Unsupported Extensnion: \"" + ext);
    PLYLoader plyLoader;
    if (!plyLoader.loadPLYModel(filename.c_str(), splatSet)) throw std::runtime_error("cannot load " + filename);
}

void Model::allocateAttributeBuffers(gvrt_host::Device* /*device*/, gvrt_host::Queue queue) {
    const int n = (int)splatSet.size();
    vertices.count = 3 * 12 * n;
    indices.count = 3 * 20 * n;
    positions.count = 3 * n;
    rotations.count = 4 * n;
    scales.count = 3 * n;
    densities.count = n;
    featuresAlbedo.count = 3 * n;
    featuresSpecular.count = 45 * n;  // SPECULAR_DIMENSION (Define.h:132-133)
    gvrt_splats s{};
    s.n = splatSet.size();
    s.positions = splatSet.positions.data();
    s.f_dc = splatSet.f_dc.data();
    s.f_rest = splatSet.f_rest.data();
    s.opacity = splatSet.opacity.data();
    s.scale = splatSet.scale.data();
    s.rotation = splatSet.rotation.data();
    check(gvrt_load_splats(queue, &s), queue, "gvrt_load_splats");
    gvrt_device_buffers b{};
    check(gvrt_get_device_buffers(queue, &b), queue, "gvrt_get_device_buffers");
    auto bind = [](Attributes& a, const void* p) { a.storageBuffer = {p, sizeof(float) * (uint64_t)a.count}; };
    bind(positions, b.positions);
    bind(rotations, b.rotations);
    bind(scales, b.scales);
    bind(densities, b.densities);
    bind(featuresAlbedo, b.features_albedo);
    bind(featuresSpecular, b.features_specular);
    vertices.storageBuffer = {};
    indices.storageBuffer = {};
}

void Model::attachEnclosingBuffers(gvrt_host::Queue queue) {
    gvrt_device_buffers b{};
    check(gvrt_get_device_buffers(queue, &b), queue, "gvrt_get_device_buffers");
    // the proxy soup of the survivors (saveIdx order); the reference sizes it for all N (Q4)
    vertices.storageBuffer = {b.vertices, b.vertices ? 144 * b.m : 0};
    indices.storageBuffer = {b.indices, b.indices ? 240 * b.m : 0};
}

}  // namespace vk3DGRT

// ================================================================================== CameraLoader
void CameraLoader::calcIntrinsics(float cameraAngleX, uint32_t width, uint32_t height, float, float) {
    float fx, fy;
    fx = fy = 0.5f * width / std::tan(0.5f * cameraAngleX);
    (void)fx;
    fovy = 2 * std::atan(height / (2 * fy));
    fovy *= 57.2957795131;  // RAD2DEGREE (LoadCamera.hpp:20), a double
}

void CameraLoader::c2wTow2cRT(CameraFrame& frame) {
    const gm::mat3 R = gm::mat3_of(frame.transformMatrix);
    const gm::vec3 T(frame.transformMatrix[3].x, frame.transformMatrix[3].y, frame.transformMatrix[3].z);
    const gm::mat3 R_inv = gm::transpose(R);
    const gm::vec3 T_inv = -R_inv * T;
    frame.transformMatrix = gm::mat4(R_inv);
    frame.transformMatrix[3] = gm::vec4(T_inv, 1.0f);
    nerfCameras.centers.push_back(T_inv);
    frame.position = -gm::vec3(frame.transformMatrix[3].x, frame.transformMatrix[3].y, frame.transformMatrix[3].z);
    gm::vec3 scale;
    scale.x = gm::length(gm::vec3(frame.transformMatrix[0].x, frame.transformMatrix[0].y, frame.transformMatrix[0].z));
    scale.y = gm::length(gm::vec3(frame.transformMatrix[1].x, frame.transformMatrix[1].y, frame.transformMatrix[1].z));
    scale.z = gm::length(gm::vec3(frame.transformMatrix[2].x, frame.transformMatrix[2].y, frame.transformMatrix[2].z));
    gm::mat3 rot;
    for (int i = 0; i < 3; ++i)
        rot[i] = gm::vec3(frame.transformMatrix[i].x, frame.transformMatrix[i].y, frame.transformMatrix[i].z) / scale[i];
    frame.rotation = gm::quat_cast(rot);
}

void CameraLoader::loadNerfCameraData(const std::string& jsonPath, uint32_t width, uint32_t height, float znear,
                                      float zfar) {
    std::ifstream fin(jsonPath);
    if (!fin.is_open()) throw std::runtime_error("Failed to open file : " + jsonPath);
    std::stringstream ss;
    ss << fin.rdbuf();
    const std::string txt = ss.str();
    JParser p(txt);
    const JVal j = p.value();
    if (j.kind != JVal::OBJ) throw std::runtime_error("transforms: not an object");
    auto ang = j.obj.find("camera_angle_x");
    if (ang == j.obj.end()) throw std::runtime_error("transforms: no camera_angle_x");
    nerfCameras.cameraAngleX = (float)ang->second.num;  // get<float>()
    calcIntrinsics(nerfCameras.cameraAngleX, width, height, znear, zfar);
    auto fr = j.obj.find("frames");
    if (fr == j.obj.end() || fr->second.kind != JVal::ARR) throw std::runtime_error("transforms: no frames");
    int i = 0;
    for (const JVal& frame : fr->second.arr) {
        CameraFrame f;
        auto fp = frame.obj.find("file_path");
        if (fp != frame.obj.end()) f.filePath = fp->second.str;
        auto tm = frame.obj.find("transform_matrix");
        if (tm == frame.obj.end() || tm->second.arr.size() != 4) throw std::runtime_error("frame without transform_matrix");
        for (int row = 0; row < 4; ++row)
            for (int col = 0; col < 4; ++col) f.transformMatrix[col][row] = (float)tm->second.arr[row].arr.at(col).num;
        c2wTow2cRT(f);
        nerfCameras.frames.push_back(f);
        camNames.push_back(std::to_string(i));
        i++;
    }
}

void CameraLoader::PrintCameraData(const NerfCameraData& data) {
    std::cout << "camera_angle_x: " << data.cameraAngleX << "\n";
    for (const auto& frame : data.frames) {
        std::cout << "File: " << frame.filePath << "\nMatrix:\n";
        std::cout << "transform matrix : \n";
        for (int i = 0; i < 4; ++i)
            std::cout << frame.transformMatrix[0][i] << " " << frame.transformMatrix[1][i] << " "
                      << frame.transformMatrix[2][i] << " " << frame.transformMatrix[3][i] << "\n";
        std::cout << "-----\n";
    }
}

// ================================================================================== Camera
void Camera::updateViewMatrix() {  // camera.hpp:31-58 (N_IS_UP)
    const gm::mat4 currentMatrix = matrices.view;
    gm::vec3 uVec(1.0f, 0.0f, 0.0f), vVec(0.0f, 0.0f, 1.0f), nVec(0.0f, -1.0f, 0.0f);
    if (gm::radians(rotation.y) != 0) rotateAxis(gm::radians(rotation.y), &vVec, &nVec, &uVec);
    if (gm::radians(rotation.x) != 0) rotateAxis(gm::radians(rotation.x), &uVec, &vVec, &nVec);
    if (gm::radians(rotation.z) != 0) rotateAxis(gm::radians(rotation.z), &nVec, &uVec, &vVec);
    const gm::mat4 rot(gm::vec4(uVec, 0.0f), gm::vec4(vVec, 0.0f), gm::vec4(nVec, 0.0f), gm::vec4(0.0f, 0.0f, 0.0f, 1.0f));
    matrices.view = gm::translate(gm::transpose(rot), -position);
    if (matrices.view != currentMatrix) updated = true;
}

void Camera::rotateAxis(float rad_angle, gm::vec3* u, gm::vec3* v, gm::vec3* n) {  // camera.hpp:124-141
    const float sina = std::sin(rad_angle), cosa = std::cos(rad_angle);
    *v = gm::normalize(*v * cosa + gm::cross(*u, *v) * sina);
    *n = gm::normalize(gm::cross(*u, *v));
}

void Camera::setNearFar(float _znear, float _zfar) {
    znear = _znear;
    zfar = _zfar;
}

void Camera::setNerfCamera(uint32_t idx) {
    if (idx >= cameraLoader.nerfCameras.frames.size()) throw std::runtime_error("NeRF camera index out of range");
    matrices.view = cameraLoader.nerfCameras.frames[idx].transformMatrix;
}

void Camera::setDatasetCamera(DatasetType t, uint32_t idx, float aspect) {  // camera.hpp:106-113
    if (t == nerf) {
        setPerspective(cameraLoader.fovy, aspect, znear, zfar);
        setPerspective(FOV_Y, aspect, znear, zfar);
        setNerfCamera(idx);
    }
}

void Camera::loadDatasetCamera(DatasetType t, std::string path, uint32_t width, uint32_t height) {
    if (t == nerf) cameraLoader.loadNerfCameraData(path, width, height, znear, zfar);
    dataType = t;
}

void Camera::setPerspective(float fov_, float aspect, float znear_, float zfar_) {  // camera.hpp:157-182
    const gm::mat4 currentMatrix = matrices.perspective;
    fov = fov_;
    znear = znear_;
    zfar = zfar_;
    matrices.perspective = gm::perspective_Vulkan_no_depth_reverse(gm::radians(fov_), aspect, znear_, zfar_);
    if (matrices.view != currentMatrix) updated = true;  // (sic: the reference compares the view)
}

void Camera::updateAspectRatio(float aspect) {
    const gm::mat4 currentMatrix = matrices.perspective;
    matrices.perspective = gm::perspective_Vulkan_no_depth_reverse(gm::radians(fov), aspect, znear, zfar);
    if (matrices.view != currentMatrix) updated = true;
}

void Camera::setPosition(gm::vec3 p) {
    position = p;
    updateViewMatrix();
}

void Camera::setRotation(gm::vec3 r) {
    rotation = r;
    updateViewMatrix();
}

void Camera::rotate(gm::vec3 delta) {
    rotation += delta;
    updateViewMatrix();
}

void Camera::setTranslation(gm::vec3 t) {
    position = t;
    updateViewMatrix();
}

void Camera::translate(gm::vec3 delta) {
    position += delta;
    updateViewMatrix();
}

void Camera::update(float deltaTime) {  // camera.hpp:229-281
    updated = false;
    if ((type == CameraType::firstperson || type == CameraType::SG_camera) && moving()) {
        const float moveSpeed = deltaTime * movementSpeed;
        gm::vec3 uVec(1.0f, 0.0f, 0.0f), vVec(0.0f, 0.0f, 1.0f), nVec(0.0f, -1.0f, 0.0f);
        if (gm::radians(rotation.y) != 0) rotateAxis(gm::radians(rotation.y), &vVec, &nVec, &uVec);
        if (gm::radians(rotation.x) != 0) rotateAxis(gm::radians(rotation.x), &uVec, &vVec, &nVec);
        if (gm::radians(rotation.z) != 0) rotateAxis(gm::radians(rotation.z), &nVec, &uVec, &vVec);
        if (keys.forward) position -= nVec * moveSpeed;
        if (keys.backward) position += nVec * moveSpeed;
        if (keys.left) position -= uVec * moveSpeed;
        if (keys.right) position += uVec * moveSpeed;
        if (keys.up) position += vVec * moveSpeed;
        if (keys.down) position -= vVec * moveSpeed;
    }
    updateViewMatrix();  // !LOAD_NERF_CAMERA (Define.h:24)
}

void Camera::setLookAt(const gm::vec3& eye, const gm::vec3& target, const gm::vec3& up) {
    position = eye;
    matrices.view = gm::lookAt(eye, target, up);
}

// ================================================================================== vks::Benchmark
// Benchmark::run / saveResults follow base/benchmark.hpp:37-104 of the reference closely (the fps.txt and console
// output are checked byte for byte against it, tests/test_host_cpp.py).  That file carries this notice:
//   Benchmark class
//   Copyright (C) 2016-2017 by Sascha Willems - www.saschawillems.de
//   This code is licensed under the MIT license (MIT) (http://opensource.org/licenses/MIT)
// MIT license text: Permission is hereby granted, free of charge, to any person obtaining a copy of this software
// and associated documentation files (the "Software"), to deal in the Software without restriction, including
// without limitation the rights to use, copy, modify, merge, publish, distribute, sublicense, and/or sell copies of
// the Software, and to permit persons to whom the Software is furnished to do so, subject to the following
// conditions: The above copyright notice and this permission notice shall be included in all copies or substantial
// portions of the Software.  THE SOFTWARE IS PROVIDED "AS IS", WITHOUT WARRANTY OF ANY KIND, EXPRESS OR IMPLIED,
// INCLUDING BUT NOT LIMITED TO THE WARRANTIES OF MERCHANTABILITY, FITNESS FOR A PARTICULAR PURPOSE AND
// NONINFRINGEMENT. IN NO EVENT SHALL THE AUTHORS OR COPYRIGHT HOLDERS BE LIABLE FOR ANY CLAIM, DAMAGES OR OTHER
// LIABILITY, WHETHER IN AN ACTION OF CONTRACT, TORT OR OTHERWISE, ARISING FROM, OUT OF OR IN CONNECTION WITH THE
// SOFTWARE OR THE USE OR OTHER DEALINGS IN THE SOFTWARE.
namespace vks {

void Benchmark::run(std::function<void()> renderFunc, gvrt_device_properties props) {  // benchmark.hpp:37-75
    active = true;
    deviceProps = props;
    std::cout << std::fixed << std::setprecision(3);
    {
        double tMeasured = 0.0;
        while (tMeasured < (warmup * 1000)) {
            auto tStart = std::chrono::high_resolution_clock::now();
            renderFunc();
            tMeasured += std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - tStart).count();
        }
    }
    while (runtime < (duration * 1000.0)) {
        auto tStart = std::chrono::high_resolution_clock::now();
        renderFunc();
        auto tDiff = std::chrono::duration<double, std::milli>(std::chrono::high_resolution_clock::now() - tStart).count();
        runtime += tDiff;
        frameTimes.push_back(tDiff);
        frameCount++;
        if (outputFrames != -1 && outputFrames == (int)frameCount) break;
    }
    std::cout << "Benchmark finished" << "\n";
    std::cout << "device : " << deviceProps.device_name << " (driver version: " << deviceProps.driver_version << ")" << "\n";
    std::cout << "runtime: " << (runtime / 1000.0) << "\n";
    std::cout << "frames : " << frameCount << "\n";
    std::cout << "fps    : " << frameCount / (runtime / 1000.0) << "\n";
}

void Benchmark::saveResults() {  // benchmark.hpp:77-104
    std::ofstream result(filename, std::ios::out);
    if (!result.is_open()) return;
    result << std::fixed << std::setprecision(4);
    result << "device,driverversion,duration (ms),frames,fps" << "\n";
    result << deviceProps.device_name << "," << deviceProps.driver_version << "," << runtime << "," << frameCount << ","
           << frameCount / (runtime / 1000.0) << "\n";
    if (outputFrameTimes && !frameTimes.empty()) {
        result << "\n" << "frame,ms" << "\n";
        for (size_t i = 0; i < frameTimes.size(); i++) result << i << "," << frameTimes[i] << "\n";
        const double tMin = *std::min_element(frameTimes.begin(), frameTimes.end());
        const double tMax = *std::max_element(frameTimes.begin(), frameTimes.end());
        const double tAvg = std::accumulate(frameTimes.begin(), frameTimes.end(), 0.0) / (double)frameTimes.size();
        std::cout << "best   : " << (1000.0 / tMin) << " fps (" << tMin << " ms)" << "\n";
        std::cout << "worst  : " << (1000.0 / tMax) << " fps (" << tMax << " ms)" << "\n";
        std::cout << "avg    : " << (1000.0 / tAvg) << " fps (" << tAvg << " ms)" << "\n";
        std::cout << "\n";
    }
    result.flush();
}

}  // namespace vks

namespace gvrt_host {

// ------------------------------------------------------------------------------------------- PNG
static uint32_t crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            table[i] = c;
        }
        init = true;
    }
    for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return crc;
}

bool write_png(const std::string& path, const uint8_t* rgba, uint32_t w, uint32_t h) {
    // zlib stream of stored deflate blocks over the filtered scanlines (filter byte 0 per row)
    std::vector<uint8_t> raw;
    raw.reserve((size_t)(4 * w + 1) * h);
    for (uint32_t y = 0; y < h; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgba + (size_t)4 * w * y, rgba + (size_t)4 * w * (y + 1));
    }
    std::vector<uint8_t> z{0x78, 0x01};
    uint32_t a = 1, b = 0;
    for (uint8_t v : raw) {
        a = (a + v) % 65521;
        b = (b + a) % 65521;
    }
    for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
        const size_t len = std::min<size_t>(65535, raw.size() - off);
        z.push_back(off + len >= raw.size() ? 1 : 0);
        z.push_back(len & 0xFF);
        z.push_back(len >> 8);
        z.push_back(~len & 0xFF);
        z.push_back((~len >> 8) & 0xFF);
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + len);
        if (raw.empty()) break;
    }
    const uint32_t adler = (b << 16) | a;
    for (int k = 3; k >= 0; --k) z.push_back((adler >> (8 * k)) & 0xFF);

    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    auto be32 = [](uint32_t v, uint8_t* o) {
        o[0] = v >> 24;
        o[1] = v >> 16;
        o[2] = v >> 8;
        o[3] = v;
    };
    auto chunk = [&](const char* type, const std::vector<uint8_t>& data) {
        uint8_t hdr[8];
        be32((uint32_t)data.size(), hdr);
        std::memcpy(hdr + 4, type, 4);
        std::fwrite(hdr, 1, 8, f);
        if (!data.empty()) std::fwrite(data.data(), 1, data.size(), f);
        uint32_t crc = crc32_update(0xFFFFFFFFu, hdr + 4, 4);
        crc = crc32_update(crc, data.data(), data.size()) ^ 0xFFFFFFFFu;
        uint8_t c[4];
        be32(crc, c);
        std::fwrite(c, 1, 4, f);
    };
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    std::fwrite(sig, 1, 8, f);
    std::vector<uint8_t> ihdr(13);
    be32(w, ihdr.data());
    be32(h, ihdr.data() + 4);
    ihdr[8] = 8;  // bit depth
    ihdr[9] = 6;  // RGBA
    chunk("IHDR", ihdr);
    chunk("IDAT", z);
    chunk("IEND", {});
    const bool ok = std::ferror(f) == 0;
    std::fclose(f);
    return ok;
}


// ================================================================================== presets, rig
gm::vec3 orbit_eye(float radius, float elevation_deg, float azimuth_deg) {
    const float el = gm::radians(elevation_deg), az = gm::radians(azimuth_deg);
    const float ce = std::cos(el);
    return gm::vec3(radius * ce * std::sin(az), radius * std::sin(el), radius * ce * std::cos(az));
}

Camera preset_camera(const std::string& name, uint32_t w, uint32_t h) {
    Camera c;
    const float aspect = (float)w / (float)h;
    if (name == "config1") {
        c.setLookAt(gm::vec3(0.0f, 0.0f, 3.0f), gm::vec3(), gm::vec3(0.0f, 1.0f, 0.0f));
        c.setPerspective(FOV_Y, aspect, NEAR_PLANE, FAR_PLANE);
    } else {
        c.setLookAt(orbit_eye(4.0f, 20.0f, 30.0f), gm::vec3(), gm::vec3(0.0f, 1.0f, 0.0f));
        c.setPerspective(50.0f, aspect, NEAR_PLANE, FAR_PLANE);
    }
    return c;
}

void lightfield_ring_rig(const vk3DGRT::SplatSet& s, uint32_t ncams, uint32_t width, uint32_t height,
                         std::vector<gm::mat4>& view_inv, gm::mat4& proj_inv) {
    float minX, minY, minZ, maxX, maxY, maxZ;  // VulkanFullRT.cpp:1527-1544 (max starts at FLT_MIN, Q15)
    minX = minY = minZ = FLT_MAX;
    maxX = maxY = maxZ = FLT_MIN;
    for (size_t i = 0; i < s.size(); i++) {
        const float x = s.positions[i * 3], y = s.positions[i * 3 + 1], z = s.positions[i * 3 + 2];
        if (x < minX) minX = x;
        if (y < minY) minY = y;
        if (z < minZ) minZ = z;
        if (x > maxX) maxX = x;
        if (y > maxY) maxY = y;
        if (z > maxZ) maxZ = z;
    }
    const gm::vec3 center((minX + maxX) / 2, (minY + maxY) / 2, (minZ + maxZ) / 2);
    const float maxR = std::max(std::max(maxX - minX, maxY - minY), maxZ - minZ) / 2;
    const gm::vec3 up(0, 0, 1);
    const gm::vec3 cameraPos[4] = {gm::vec3(center.x + maxR, center.y, center.z),
                                   gm::vec3(center.x, center.y + maxR, center.z),
                                   gm::vec3(center.x - maxR, center.y, center.z),
                                   gm::vec3(center.x, center.y - maxR, center.z)};
    view_inv.clear();
    for (uint32_t i = 0; i < ncams; i++) view_inv.push_back(gm::inverse(gm::lookAt(cameraPos[i % 4], center, up)));
    // 135 degree fov, aspect (float)(width / height) with integer division (Q15), :1596 / :1604
    proj_inv = gm::inverse(gm::perspective_Vulkan_no_depth_reverse(gm::radians(135.0f), (float)(width / height),
                                                                   NEAR_PLANE, FAR_PLANE));
}

// ================================================================================== GvrtApp
GvrtApp::GvrtApp(int dev) : device(dev) {
    check(gvrt_create(dev, &h_), nullptr, "gvrt_create");
    gvrt_default_render_params(&params);
}

GvrtApp::~GvrtApp() {
    if (h_) gvrt_destroy(h_);
}

uint64_t GvrtApp::prepare(const std::string& ply, const gvrt_enclosing_params* ep, const gvrt_accel_params* ap) {
    gModel.load3DGRTModel(ply, &device);
    gModel.allocateAttributeBuffers(&device, h_);
    gvrt_enclosing_params e;
    gvrt_default_enclosing_params(&e);
    uint64_t m = 0;
    check(gvrt_build_enclosing(h_, ep ? ep : &e, &m), h_, "gvrt_build_enclosing");
    gModel.attachEnclosingBuffers(h_);
    if (ap) check(gvrt_build_accel_ex(h_, ap), h_, "gvrt_build_accel_ex");
    else check(gvrt_build_accel(h_), h_, "gvrt_build_accel");
    return m;
}

void GvrtApp::updateUniformBuffer(const Camera& cam) {
    uniformDataDynamic.viewInverse = gm::inverse(cam.matrices.view);
    uniformDataDynamic.projInverse = gm::inverse(cam.matrices.perspective);
}

void GvrtApp::draw(uint32_t width, uint32_t height, uint8_t* rgba8, uint32_t* hit_counts) {
    gvrt_image img{rgba8, nullptr, nullptr, hit_counts, 0, 0};
    check(gvrt_render(h_, &params, uniformDataDynamic.viewInverse.data(), uniformDataDynamic.projInverse.data(), width,
                      height, 1, nullptr, 0, &img),
          h_, "gvrt_render");
}

void GvrtApp::draw(const Camera& cam, uint32_t width, uint32_t height, uint8_t* rgba8, uint32_t* hit_counts) {
    updateUniformBuffer(cam);
    draw(width, height, rgba8, hit_counts);
}

size_t GvrtApp::evalCapture(const std::string& transforms, const std::string& out_dir, uint32_t width,
                            uint32_t height) {
    camera.setNearFar(NEAR_PLANE, FAR_PLANE);
    camera.loadDatasetCamera(nerf, transforms, width, height);
    make_dir(out_dir);
    std::vector<uint8_t> frame((size_t)4 * width * height);
    const size_t nviews = camera.getCamNames().size();
    for (uint32_t i = 0; i < nviews; ++i) {
        camera.setDatasetCamera(camera.dataType, i, (float)width / height);  // VulkanFullRT.cpp:2154
        draw(camera, width, height, frame.data());
        if (!write_png(out_dir + "/r_" + std::to_string(i) + ".png", frame.data(), width, height))
            throw std::runtime_error("cannot write " + out_dir);
    }
    return nviews;
}

void GvrtApp::calculateGaussianLightFieldSamples() {
    lightfield_ring_rig(gModel.splatSet, gaussianLightField.samplingCameraNum, gaussianLightField.sampleImageWidth,
                        gaussianLightField.sampleImageHeight, gaussianLightField.viewInverse,
                        gaussianLightField.projInverse);
}

size_t GvrtApp::computeGaussianLightField(const std::string& out_dir) {
    calculateGaussianLightFieldSamples();
    const uint32_t ncams = gaussianLightField.samplingCameraNum;
    const uint32_t width = gaussianLightField.sampleImageWidth, height = gaussianLightField.sampleImageHeight;
    std::vector<float> vi;
    for (const gm::mat4& m : gaussianLightField.viewInverse) vi.insert(vi.end(), m.data(), m.data() + 16);
    gvrt_render_params p = params;  // the light-field raygen: pixel centre, alpha starts at 1
    p.pixel_offset = 0.5f;
    p.alpha_init = 1.0f;
    p.ray_dirs_layout = 1;  // rayDirs[cam][x][y] (raygenGaussianLightField.rgen:129)
    std::vector<uint8_t> rgba((size_t)4 * width * height * ncams);
    std::vector<float> dirs((size_t)4 * width * height * ncams);
    gvrt_image img{rgba.data(), nullptr, dirs.data(), nullptr, 0, 0};
    check(gvrt_render(h_, &p, vi.data(), gaussianLightField.projInverse.data(), width, height, ncams, nullptr, 0, &img),
          h_, "gvrt_render");
    make_dir(out_dir);
    for (uint32_t c = 0; c < ncams; ++c)
        if (!write_png(out_dir + "/view_" + std::to_string(c) + ".png", rgba.data() + (size_t)4 * width * height * c,
                       width, height))
            throw std::runtime_error("cannot write " + out_dir);
    FILE* f = std::fopen((out_dir + "/rayDirs.bin").c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write rayDirs.bin");
    std::fwrite(dirs.data(), sizeof(float), dirs.size(), f);
    std::fclose(f);
    return ncams;
}

void GvrtApp::printRayHitCounts(const Camera& cam, uint32_t width, uint32_t height, const std::string& path) {
    std::vector<uint32_t> hc((size_t)width * height);
    draw(cam, width, height, nullptr, hc.data());
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) throw std::runtime_error("cannot write " + path);
    for (uint32_t y = 0; y < height; ++y) {
        for (uint32_t x = 0; x < width; ++x) std::fprintf(f, "%u ", hc[(size_t)y * width + x]);
        std::fprintf(f, "\n");
    }
    std::fclose(f);
}

double GvrtApp::runBenchmark(const Camera& cam, uint32_t width, uint32_t height) {
    // frames go to device memory (the reference renders into its swapchain image; no readback)
    void* frame = nullptr;
    if (hipSetDevice(device.ordinal) != hipSuccess || hipMalloc(&frame, (size_t)4 * width * height) != hipSuccess)
        throw std::runtime_error("device frame allocation failed");
    updateUniformBuffer(cam);
    gvrt_image img{frame, nullptr, nullptr, nullptr, 1, 0};
    try {
        benchmark.run(
            [&] {  // one frame = render + wait, as the reference's frame with its fence
                check(gvrt_render(h_, &params, uniformDataDynamic.viewInverse.data(),
                                  uniformDataDynamic.projInverse.data(), width, height, 1, nullptr, 0, &img),
                      h_, "gvrt_render");
            },
            device.properties);
    } catch (...) {
        (void)hipFree(frame);
        throw;
    }
    (void)hipFree(frame);
    return benchmark.frameCount / (benchmark.runtime / 1000.0);
}

gvrt_stats GvrtApp::stats() const {
    gvrt_stats s{};
    gvrt_get_stats(h_, &s);
    return s;
}

}  // namespace gvrt_host
