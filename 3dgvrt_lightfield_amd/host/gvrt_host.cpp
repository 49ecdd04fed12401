// gvrt_host.cpp — implementation of the C++ host layer (gvrt_host.h).  Reference file:line per class
// in the header; the Python mirror (camera.py, app.py) follows the same formulas.
#include "gvrt_host.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cctype>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <sys/stat.h>

namespace gvrt_host {

static void check(gvrt_status s, gvrt_handle h, const char* what) {
    if (s != GVRT_OK) throw std::runtime_error(std::string(what) + ": " + gvrt_last_error(h));
}

static void make_dir(const std::string& d) { ::mkdir(d.c_str(), 0755); }

// ------------------------------------------------------------------------------------------- math
mat4 mat4::identity() {
    mat4 r{};
    for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0;
    return r;
}

mat4 mat4::operator*(const mat4& b) const {
    mat4 r{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 4; ++k) r.m[i][j] += m[i][k] * b.m[k][j];
    return r;
}

mat4 mat4::inverse() const {
    double a[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) a[i][j] = j < 4 ? m[i][j] : (j - 4 == i ? 1.0 : 0.0);
    for (int c = 0; c < 4; ++c) {
        int p = c;
        for (int r = c + 1; r < 4; ++r)
            if (std::fabs(a[r][c]) > std::fabs(a[p][c])) p = r;
        if (a[p][c] == 0.0) throw std::runtime_error("singular matrix");
        if (p != c)
            for (int j = 0; j < 8; ++j) std::swap(a[p][j], a[c][j]);
        const double d = a[c][c];
        for (int j = 0; j < 8; ++j) a[c][j] /= d;
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            const double f = a[r][c];
            if (f != 0.0)
                for (int j = 0; j < 8; ++j) a[r][j] -= f * a[c][j];
        }
    }
    mat4 r{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.m[i][j] = a[i][4 + j];
    return r;
}

std::array<float, 16> mat4::colmajor() const {
    std::array<float, 16> o{};
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) o[4 * c + r] = (float)m[r][c];
    return o;
}

static vec3 sub(const vec3& a, const vec3& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
static vec3 add(const vec3& a, const vec3& b) { return {a[0] + b[0], a[1] + b[1], a[2] + b[2]}; }
static vec3 scale(const vec3& a, double s) { return {a[0] * s, a[1] * s, a[2] * s}; }
static double dot(const vec3& a, const vec3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static vec3 cross(const vec3& a, const vec3& b) {
    return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}
static vec3 normalize(const vec3& a) { return scale(a, 1.0 / std::sqrt(dot(a, a))); }

// glm::lookAtRH
mat4 look_at(const vec3& eye, const vec3& center, const vec3& up) {
    const vec3 f = normalize(sub(center, eye));
    const vec3 s = normalize(cross(f, up));
    const vec3 u = cross(s, f);
    mat4 m = mat4::identity();
    for (int i = 0; i < 3; ++i) {
        m.m[0][i] = s[i];
        m.m[1][i] = u[i];
        m.m[2][i] = -f[i];
    }
    m.m[0][3] = -dot(s, eye);
    m.m[1][3] = -dot(u, eye);
    m.m[2][3] = dot(f, eye);
    return m;
}

// matrix_transform.inl:276-290 (Result[1][1] = -1/tan: image row 0 is the top)
mat4 perspective_vulkan_no_depth_reverse(double fovy_rad, double aspect, double znear, double zfar) {
    const double t = std::tan(fovy_rad / 2.0);
    mat4 m{};
    m.m[0][0] = 1.0 / (aspect * t);
    m.m[1][1] = -1.0 / t;
    m.m[3][2] = -1.0;
    m.m[2][2] = -zfar / (zfar - znear);
    m.m[2][3] = -(zfar * znear) / (zfar - znear);
    return m;
}

// ------------------------------------------------------------------------------------------- model
gvrt_splats SplatSet::view() const {
    gvrt_splats s{};
    s.n = size();
    s.positions = positions.data();
    s.f_dc = f_dc.data();
    s.f_rest = f_rest.data();
    s.opacity = opacity.data();
    s.scale = scale.data();
    s.rotation = rotation.data();
    return s;
}

bool PLYLoader::loadPLYModel(const std::string& filename, SplatSet& out, std::string* err) {
    gvrt_splat_buffers b{};
    if (gvrt_ply_load(filename.c_str(), &b) != GVRT_OK) {
        if (err) *err = gvrt_last_error(nullptr);
        return false;
    }
    const size_t n = b.n;
    auto take = [n](const float* p, size_t k) { return std::vector<float>(p, p + n * k); };
    out.positions = take(b.positions, 3);
    out.f_dc = take(b.f_dc, 3);
    out.f_rest = take(b.f_rest, 45);
    out.opacity = take(b.opacity, 1);
    out.scale = take(b.scale, 3);
    out.rotation = take(b.rotation, 4);
    gvrt_ply_free(&b);
    return true;
}

// ------------------------------------------------------------------------------------------- camera
// camera.hpp rotateAxis: rotate (u, v) about u and rebuild n
static void rotate_axis(double rad, vec3& u, vec3& v, vec3& n) {
    const double s = std::sin(rad), c = std::cos(rad);
    v = normalize(add(scale(v, c), scale(cross(u, v), s)));
    n = normalize(cross(u, v));
}

void Camera::updateViewMatrix() {  // camera.hpp:31-58, N_IS_UP
    vec3 u{1, 0, 0}, v{0, 0, 1}, n{0, -1, 0};
    const double d2r = M_PI / 180.0;
    if (rotation[1] * d2r != 0) rotate_axis(rotation[1] * d2r, v, n, u);
    if (rotation[0] * d2r != 0) rotate_axis(rotation[0] * d2r, u, v, n);
    if (rotation[2] * d2r != 0) rotate_axis(rotation[2] * d2r, n, u, v);
    mat4 rt = mat4::identity();  // transpose of glm::mat4(vec4(u), vec4(v), vec4(n), ...)
    for (int i = 0; i < 3; ++i) {
        rt.m[0][i] = u[i];
        rt.m[1][i] = v[i];
        rt.m[2][i] = n[i];
    }
    mat4 tr = mat4::identity();
    for (int i = 0; i < 3; ++i) tr.m[i][3] = -position[i];
    matrices.view = rt * tr;  // glm::translate(transpose(rot), -position)
}

void Camera::setPosition(const vec3& p) {
    position = p;
    updateViewMatrix();
}

void Camera::setRotation(const vec3& r) {
    rotation = r;
    updateViewMatrix();
}

void Camera::setPerspective(double fov_deg, double aspect, double zn, double zf) {  // camera.hpp:157-182
    fov = fov_deg;
    znear = zn;
    zfar = zf;
    matrices.perspective = perspective_vulkan_no_depth_reverse(fov_deg * M_PI / 180.0, aspect, zn, zf);
}

void Camera::setLookAt(const vec3& eye, const vec3& target, const vec3& up) {
    position = eye;
    matrices.view = look_at(eye, target, up);
}

// ------------------------------------------------------------------------------------------- JSON
// A minimal JSON reader for transforms_*.json (objects, arrays, numbers, strings, literals).
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

// LoadCamera.hpp:57-85 (loadNerfCameraData) and :124-147 (c2wTow2cRT): w2c = [R^T | -R^T t]
bool CameraLoader::loadNerfCameraData(const std::string& path, std::string* err) {
    try {
        std::ifstream f(path);
        if (!f) throw std::runtime_error("cannot open " + path);
        std::stringstream ss;
        ss << f.rdbuf();
        const std::string txt = ss.str();
        JParser p(txt);
        const JVal root = p.value();
        if (root.kind != JVal::OBJ) throw std::runtime_error("transforms: not an object");
        auto it = root.obj.find("camera_angle_x");
        camera_angle_x = it != root.obj.end() ? it->second.num : 0.0;
        auto fr = root.obj.find("frames");
        if (fr == root.obj.end() || fr->second.kind != JVal::ARR) throw std::runtime_error("transforms: no frames");
        views.clear();
        for (const JVal& frame : fr->second.arr) {
            auto tm = frame.obj.find("transform_matrix");
            if (tm == frame.obj.end() || tm->second.arr.size() < 3) throw std::runtime_error("frame without transform_matrix");
            mat4 c2w = mat4::identity();
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 4; ++c) c2w.m[r][c] = tm->second.arr[r].arr.at(c).num;
            mat4 w2c = mat4::identity();
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c) w2c.m[r][c] = c2w.m[c][r];
                w2c.m[r][3] = -(c2w.m[0][r] * c2w.m[0][3] + c2w.m[1][r] * c2w.m[1][3] + c2w.m[2][r] * c2w.m[2][3]);
            }
            views.push_back(w2c);
        }
        return true;
    } catch (const std::exception& e) {
        if (err) *err = e.what();
        return false;
    }
}

// ------------------------------------------------------------------------------------------- benchmark
bool Benchmark::saveResults() const {  // benchmark.hpp:77-104
    FILE* f = std::fopen(filename.c_str(), "w");
    if (!f) return false;
    const size_t n = frameTimes.size();
    std::fprintf(f, "device,driverversion,duration (ms),frames,fps\n");
    std::fprintf(f, "%s,%s,%.4f,%zu,%.4f\n", device.c_str(), driver.c_str(), runtime, n, n / (runtime / 1000.0));
    if (outputFrameTimes) {
        std::fprintf(f, "\nframe,ms\n");
        for (size_t i = 0; i < n; ++i) std::fprintf(f, "%zu,%.4f\n", i, frameTimes[i]);
    }
    std::fclose(f);
    return true;
}

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

// ------------------------------------------------------------------------------------------- app
GvrtApp::GvrtApp(int device) : device_(device) {
    check(gvrt_create(device, &h_), nullptr, "gvrt_create");
    gvrt_default_render_params(&params);
}

GvrtApp::~GvrtApp() {
    if (h_) gvrt_destroy(h_);
}

uint64_t GvrtApp::prepare(const std::string& ply, const gvrt_enclosing_params* ep, const gvrt_accel_params* ap) {
    std::string err;
    if (!PLYLoader().loadPLYModel(ply, splats, &err)) throw std::runtime_error("cannot load " + ply + ": " + err);
    const gvrt_splats s = splats.view();
    check(gvrt_load_splats(h_, &s), h_, "gvrt_load_splats");
    gvrt_enclosing_params e;
    gvrt_default_enclosing_params(&e);
    uint64_t m = 0;
    check(gvrt_build_enclosing(h_, ep ? ep : &e, &m), h_, "gvrt_build_enclosing");
    if (ap) check(gvrt_build_accel_ex(h_, ap), h_, "gvrt_build_accel_ex");
    else check(gvrt_build_accel(h_), h_, "gvrt_build_accel");
    return m;
}

void GvrtApp::draw(const Camera& cam, uint32_t width, uint32_t height, uint8_t* rgba8, uint32_t* hit_counts) {
    const auto vi = cam.matrices.view.inverse().colmajor();
    const auto pi = cam.matrices.perspective.inverse().colmajor();
    gvrt_image img{rgba8, nullptr, nullptr, hit_counts, 0, 0};
    check(gvrt_render(h_, &params, vi.data(), pi.data(), width, height, 1, nullptr, 0, &img), h_, "gvrt_render");
}

size_t GvrtApp::evalCapture(const std::string& transforms, const std::string& out_dir, uint32_t width,
                            uint32_t height) {
    CameraLoader loader;
    std::string err;
    if (!loader.loadNerfCameraData(transforms, &err)) throw std::runtime_error(err);
    make_dir(out_dir);
    Camera cam;
    cam.setPerspective(FOV_Y, (double)width / height, NEAR_PLANE, FAR_PLANE);  // setDatasetCamera's FOV_Y
    std::vector<uint8_t> frame((size_t)4 * width * height);
    for (size_t i = 0; i < loader.views.size(); ++i) {
        cam.matrices.view = loader.views[i];  // camera.setNerfCamera: w2c is the view matrix
        draw(cam, width, height, frame.data());
        if (!write_png(out_dir + "/r_" + std::to_string(i) + ".png", frame.data(), width, height))
            throw std::runtime_error("cannot write " + out_dir);
    }
    return loader.views.size();
}

void lightfield_ring_rig(const SplatSet& s, uint32_t ncams, uint32_t width, uint32_t height,
                         std::vector<float>& view_inv, std::array<float, 16>& proj_inv) {
    // bbox of the raw positions with max initialised to FLT_MIN (Q15)
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {FLT_MIN, FLT_MIN, FLT_MIN};
    for (size_t i = 0; i < s.size(); ++i)
        for (int k = 0; k < 3; ++k) {
            mn[k] = std::min(mn[k], s.positions[3 * i + k]);
            mx[k] = std::max(mx[k], s.positions[3 * i + k]);
        }
    vec3 center;
    float maxr = 0.0f;
    for (int k = 0; k < 3; ++k) {
        center[k] = (double)((mn[k] + mx[k]) / 2.0f);
        maxr = std::max(maxr, mx[k] - mn[k]);
    }
    const double r = (double)maxr / 2.0;
    const vec3 cams[4] = {add(center, {r, 0, 0}), add(center, {0, r, 0}), sub(center, {r, 0, 0}), sub(center, {0, r, 0})};
    view_inv.clear();
    for (uint32_t i = 0; i < ncams; ++i) {
        const auto v = look_at(cams[i % 4], center, {0.0, 0.0, 1.0}).inverse().colmajor();
        view_inv.insert(view_inv.end(), v.begin(), v.end());
    }
    // 135 degree fov, aspect (float)(width / height) with integer division (Q15)
    proj_inv = perspective_vulkan_no_depth_reverse(135.0 * M_PI / 180.0, (double)(float)(width / height), NEAR_PLANE,
                                                   FAR_PLANE)
                   .inverse()
                   .colmajor();
}

size_t GvrtApp::computeGaussianLightField(const std::string& out_dir, uint32_t width, uint32_t height) {
    const uint32_t ncams = 4;  // VulkanFullRT.cpp:169-171
    std::vector<float> vi;
    std::array<float, 16> pi;
    lightfield_ring_rig(splats, ncams, width, height, vi, pi);
    gvrt_render_params p = params;  // the light-field raygen: pixel centre, alpha starts at 1
    p.pixel_offset = 0.5f;
    p.alpha_init = 1.0f;
    p.ray_dirs_layout = 1;  // rayDirs[cam][x][y] (raygenGaussianLightField.rgen:129)
    std::vector<uint8_t> rgba((size_t)4 * width * height * ncams);
    std::vector<float> dirs((size_t)4 * width * height * ncams);
    gvrt_image img{rgba.data(), nullptr, dirs.data(), nullptr, 0, 0};
    check(gvrt_render(h_, &p, vi.data(), pi.data(), width, height, ncams, nullptr, 0, &img), h_, "gvrt_render");
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

double GvrtApp::benchmark(const Camera& cam, uint32_t width, uint32_t height, Benchmark& b) {
    void* frame = nullptr;
    if (hipSetDevice(device_) != hipSuccess || hipMalloc(&frame, (size_t)4 * width * height) != hipSuccess)
        throw std::runtime_error("device frame allocation failed");
    hipDeviceProp_t prop{};
    if (hipGetDeviceProperties(&prop, device_) == hipSuccess) {
        b.device = prop.name;
        std::replace(b.device.begin(), b.device.end(), ',', ' ');
    }
    int drv = 0;
    if (hipDriverGetVersion(&drv) == hipSuccess) b.driver = std::to_string(drv);
    const auto vi = cam.matrices.view.inverse().colmajor();
    const auto pi = cam.matrices.perspective.inverse().colmajor();
    gvrt_image img{frame, nullptr, nullptr, nullptr, 1, 0};
    double fps = 0.0;
    try {
        fps = b.run([&] {  // one frame = render + wait, as the reference's frame with its fence
            check(gvrt_render(h_, &params, vi.data(), pi.data(), width, height, 1, nullptr, 0, &img), h_,
                  "gvrt_render");
        });
    } catch (...) {
        (void)hipFree(frame);
        throw;
    }
    (void)hipFree(frame);
    return fps;
}

gvrt_stats GvrtApp::stats() const {
    gvrt_stats s{};
    gvrt_get_stats(h_, &s);
    return s;
}

}  // namespace gvrt_host
