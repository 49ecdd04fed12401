// gvrt_ply.cpp — 3DGS PLY reader/writer behind gvrt_ply_load / gvrt_ply_save.
//
// Behaviour of vk3DGRT::PLYLoader::loadPLYModel (base/Vulkan3DGRTModel.cpp:7-125), which reads
// with miniply (external/miniply):
//   * the first element named "vertex" with rows is the splat set; other elements are skipped;
//   * property groups are found all-or-nothing: {f_rest_0..44}, {x,y,z}, {opacity},
//     {scale_0..2}, {rot_0..3}, {f_dc_0..2}; a missing group leaves its array zero-filled
//     (the reference resizes every vector before extraction, :51-56);
//   * f_rest is reordered from PLY channel-major (R0..14, G0..14, B0..14) to coefficient-major
//     interleaved RGB: out[45 g + 3 i + c] = f_rest_{i + 15 c} (:70-77);
//   * every numeric property type is converted to float (miniply PLYPropertyType::Float).
// Formats: ascii, binary_little_endian, binary_big_endian.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/gvrt.h"

namespace {

enum class PType { I8, U8, I16, U16, I32, U32, F32, F64, NONE };

PType parse_type(const std::string& t) {
    if (t == "char" || t == "int8") return PType::I8;
    if (t == "uchar" || t == "uint8") return PType::U8;
    if (t == "short" || t == "int16") return PType::I16;
    if (t == "ushort" || t == "uint16") return PType::U16;
    if (t == "int" || t == "int32") return PType::I32;
    if (t == "uint" || t == "uint32") return PType::U32;
    if (t == "float" || t == "float32") return PType::F32;
    if (t == "double" || t == "float64") return PType::F64;
    return PType::NONE;
}

int type_size(PType t) {
    switch (t) {
        case PType::I8: case PType::U8: return 1;
        case PType::I16: case PType::U16: return 2;
        case PType::I32: case PType::U32: case PType::F32: return 4;
        case PType::F64: return 8;
        default: return 0;
    }
}

struct Prop {
    std::string name;
    PType type = PType::NONE;
    bool is_list = false;
    PType count_type = PType::NONE;
};

struct Elem {
    std::string name;
    uint64_t count = 0;
    std::vector<Prop> props;
};

template <typename T>
T load_raw(const unsigned char* p, bool swap) {
    unsigned char b[sizeof(T)];
    std::memcpy(b, p, sizeof(T));
    if (swap)
        for (size_t i = 0; i < sizeof(T) / 2; ++i) std::swap(b[i], b[sizeof(T) - 1 - i]);
    T v;
    std::memcpy(&v, b, sizeof(T));
    return v;
}

double load_num(const unsigned char* p, PType t, bool swap) {
    switch (t) {
        case PType::I8: return (double)load_raw<int8_t>(p, false);
        case PType::U8: return (double)load_raw<uint8_t>(p, false);
        case PType::I16: return (double)load_raw<int16_t>(p, swap);
        case PType::U16: return (double)load_raw<uint16_t>(p, swap);
        case PType::I32: return (double)load_raw<int32_t>(p, swap);
        case PType::U32: return (double)load_raw<uint32_t>(p, swap);
        case PType::F32: return (double)load_raw<float>(p, swap);
        case PType::F64: return load_raw<double>(p, swap);
        default: return 0.0;
    }
}

float to_float(const unsigned char* p, PType t, bool swap) {
    if (t == PType::F32) return load_raw<float>(p, swap);
    return (float)load_num(p, t, swap);
}

bool host_is_little() {
    const uint16_t x = 1;
    unsigned char c;
    std::memcpy(&c, &x, 1);
    return c == 1;
}

}  // namespace

extern "C" {

void gvrt_ply_free(gvrt_splat_buffers* b) {
    if (!b) return;
    std::free(b->positions);
    std::free(b->f_dc);
    std::free(b->f_rest);
    std::free(b->opacity);
    std::free(b->scale);
    std::free(b->rotation);
    std::memset(b, 0, sizeof(*b));
}

gvrt_status gvrt_ply_load(const char* path, gvrt_splat_buffers* out) {
    if (!path || !out) return GVRT_ERR_INVALID_ARG;
    std::memset(out, 0, sizeof(*out));
    std::ifstream f(path, std::ios::binary);
    if (!f) return GVRT_ERR_IO;
    std::string line;
    if (!std::getline(f, line)) return GVRT_ERR_IO;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line != "ply") return GVRT_ERR_IO;
    int fmt = -1;  // 0 ascii, 1 ble, 2 bbe
    std::vector<Elem> elems;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ss(line);
        std::string kw;
        ss >> kw;
        if (kw == "format") {
            std::string t;
            ss >> t;
            fmt = t == "ascii" ? 0 : t == "binary_little_endian" ? 1 : t == "binary_big_endian" ? 2 : -1;
            if (fmt < 0) return GVRT_ERR_IO;
        } else if (kw == "element") {
            Elem e;
            ss >> e.name >> e.count;
            elems.push_back(e);
        } else if (kw == "property") {
            if (elems.empty()) return GVRT_ERR_IO;
            Prop p;
            std::string t;
            ss >> t;
            if (t == "list") {
                std::string ct, it;
                ss >> ct >> it >> p.name;
                p.is_list = true;
                p.count_type = parse_type(ct);
                p.type = parse_type(it);
            } else {
                p.type = parse_type(t);
                ss >> p.name;
            }
            if (p.type == PType::NONE) return GVRT_ERR_IO;
            elems.back().props.push_back(p);
        } else if (kw == "end_header") {
            break;
        }
    }
    if (fmt < 0) return GVRT_ERR_IO;
    const bool swap = (fmt == 1 && !host_is_little()) || (fmt == 2 && host_is_little());

    for (size_t ei = 0; ei < elems.size(); ++ei) {
        const Elem& e = elems[ei];
        const bool is_vertex = e.name == "vertex" && e.count > 0;
        // fixed-size binary rows?
        bool fixed = true;
        uint64_t row = 0;
        for (const Prop& p : e.props) {
            if (p.is_list) fixed = false;
            else row += type_size(p.type);
        }
        if (!is_vertex) {
            // skip this element
            if (fmt == 0) {
                for (uint64_t r = 0; r < e.count; ++r)
                    if (!std::getline(f, line)) return GVRT_ERR_IO;
            } else if (fixed) {
                f.seekg((std::streamoff)(row * e.count), std::ios::cur);
            } else {
                for (uint64_t r = 0; r < e.count; ++r)
                    for (const Prop& p : e.props) {
                        if (p.is_list) {
                            unsigned char cb[8];
                            f.read((char*)cb, type_size(p.count_type));
                            const uint64_t cnt = (uint64_t)load_num(cb, p.count_type, swap);
                            f.seekg((std::streamoff)(cnt * type_size(p.type)), std::ios::cur);
                        } else {
                            f.seekg(type_size(p.type), std::ios::cur);
                        }
                    }
            }
            if (!f) return GVRT_ERR_IO;
            continue;
        }
        // ---- the splat element
        const uint64_t n = e.count;
        auto find = [&](const std::string& nm) -> int {
            for (size_t i = 0; i < e.props.size(); ++i)
                if (e.props[i].name == nm && !e.props[i].is_list) return (int)i;
            return -1;
        };
        auto group = [&](const std::vector<std::string>& names, std::vector<int>& idx) -> bool {
            idx.clear();
            for (const auto& nm : names) {
                const int i = find(nm);
                if (i < 0) return false;
                idx.push_back(i);
            }
            return true;
        };
        std::vector<std::string> frest_names, xyz = {"x", "y", "z"}, opn = {"opacity"},
                                               scn = {"scale_0", "scale_1", "scale_2"},
                                               rtn = {"rot_0", "rot_1", "rot_2", "rot_3"},
                                               dcn = {"f_dc_0", "f_dc_1", "f_dc_2"};
        for (int i = 0; i < 45; ++i) frest_names.push_back("f_rest_" + std::to_string(i));
        std::vector<int> g_frest, g_xyz, g_op, g_sc, g_rt, g_dc;
        const bool h_frest = group(frest_names, g_frest), h_xyz = group(xyz, g_xyz), h_op = group(opn, g_op),
                   h_sc = group(scn, g_sc), h_rt = group(rtn, g_rt), h_dc = group(dcn, g_dc);
        out->n = n;
        out->positions = (float*)std::calloc(3 * n, 4);
        out->f_dc = (float*)std::calloc(3 * n, 4);
        out->f_rest = (float*)std::calloc(45 * n, 4);
        out->opacity = (float*)std::calloc(n, 4);
        out->scale = (float*)std::calloc(3 * n, 4);
        out->rotation = (float*)std::calloc(4 * n, 4);
        if (!out->positions || !out->f_dc || !out->f_rest || !out->opacity || !out->scale || !out->rotation) {
            gvrt_ply_free(out);
            return GVRT_ERR_OOM;
        }
        std::vector<float> vals(e.props.size());
        std::vector<unsigned char> buf(fixed ? row : 0);
        for (uint64_t r = 0; r < n; ++r) {
            if (fmt == 0) {
                if (!std::getline(f, line)) {
                    gvrt_ply_free(out);
                    return GVRT_ERR_IO;
                }
                std::istringstream ls(line);
                for (size_t i = 0; i < e.props.size(); ++i) {
                    const Prop& p = e.props[i];
                    if (p.is_list) {
                        double cnt;
                        ls >> cnt;
                        double dummy;
                        for (uint64_t k = 0; k < (uint64_t)cnt; ++k) ls >> dummy;
                        vals[i] = 0.f;
                    } else {
                        double v;
                        ls >> v;
                        vals[i] = (float)v;
                    }
                }
                if (!ls && !ls.eof()) {
                    gvrt_ply_free(out);
                    return GVRT_ERR_IO;
                }
            } else if (fixed) {
                f.read((char*)buf.data(), (std::streamsize)row);
                if (!f) {
                    gvrt_ply_free(out);
                    return GVRT_ERR_IO;
                }
                uint64_t off = 0;
                for (size_t i = 0; i < e.props.size(); ++i) {
                    vals[i] = to_float(buf.data() + off, e.props[i].type, swap);
                    off += type_size(e.props[i].type);
                }
            } else {
                for (size_t i = 0; i < e.props.size(); ++i) {
                    const Prop& p = e.props[i];
                    unsigned char cb[8];
                    if (p.is_list) {
                        f.read((char*)cb, type_size(p.count_type));
                        const uint64_t cnt = (uint64_t)load_num(cb, p.count_type, swap);
                        f.seekg((std::streamoff)(cnt * type_size(p.type)), std::ios::cur);
                        vals[i] = 0.f;
                    } else {
                        f.read((char*)cb, type_size(p.type));
                        vals[i] = to_float(cb, p.type, swap);
                    }
                }
                if (!f) {
                    gvrt_ply_free(out);
                    return GVRT_ERR_IO;
                }
            }
            if (h_frest)
                for (int i = 0; i < 15; ++i)
                    for (int c = 0; c < 3; ++c) out->f_rest[45 * r + 3 * i + c] = vals[g_frest[i + 15 * c]];
            if (h_xyz)
                for (int k = 0; k < 3; ++k) out->positions[3 * r + k] = vals[g_xyz[k]];
            if (h_op) out->opacity[r] = vals[g_op[0]];
            if (h_sc)
                for (int k = 0; k < 3; ++k) out->scale[3 * r + k] = vals[g_sc[k]];
            if (h_rt)
                for (int k = 0; k < 4; ++k) out->rotation[4 * r + k] = vals[g_rt[k]];
            if (h_dc)
                for (int k = 0; k < 3; ++k) out->f_dc[3 * r + k] = vals[g_dc[k]];
        }
        return GVRT_OK;
    }
    return GVRT_ERR_IO;  // "invalid 3DGS PLY file" (:121)
}

gvrt_status gvrt_ply_save(const char* path, const gvrt_splats* s) {
    if (!path || !s) return GVRT_ERR_INVALID_ARG;
    if (s->n && (!s->positions || !s->f_dc || !s->f_rest || !s->opacity || !s->scale || !s->rotation))
        return GVRT_ERR_INVALID_ARG;
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return GVRT_ERR_IO;
    std::string h = "ply\nformat binary_little_endian 1.0\nelement vertex " + std::to_string(s->n) + "\n";
    const char* names[] = {"x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"};
    for (const char* nm : names) h += std::string("property float ") + nm + "\n";
    for (int i = 0; i < 45; ++i) h += "property float f_rest_" + std::to_string(i) + "\n";
    h += "property float opacity\nproperty float scale_0\nproperty float scale_1\nproperty float scale_2\n";
    h += "property float rot_0\nproperty float rot_1\nproperty float rot_2\nproperty float rot_3\nend_header\n";
    std::fwrite(h.data(), 1, h.size(), fp);
    std::vector<float> row(62);
    for (uint64_t r = 0; r < s->n; ++r) {
        int k = 0;
        for (int j = 0; j < 3; ++j) row[k++] = s->positions[3 * r + j];
        for (int j = 0; j < 3; ++j) row[k++] = 0.f;
        for (int j = 0; j < 3; ++j) row[k++] = s->f_dc[3 * r + j];
        for (int c = 0; c < 3; ++c)
            for (int i = 0; i < 15; ++i) row[k++] = s->f_rest[45 * r + 3 * i + c];
        row[k++] = s->opacity[r];
        for (int j = 0; j < 3; ++j) row[k++] = s->scale[3 * r + j];
        for (int j = 0; j < 4; ++j) row[k++] = s->rotation[4 * r + j];
        if (!host_is_little())
            for (float& v : row) {
                unsigned char b[4];
                std::memcpy(b, &v, 4);
                std::swap(b[0], b[3]);
                std::swap(b[1], b[2]);
                std::memcpy(&v, b, 4);
            }
        if (std::fwrite(row.data(), 4, 62, fp) != 62) {
            std::fclose(fp);
            return GVRT_ERR_IO;
        }
    }
    return std::fclose(fp) == 0 ? GVRT_OK : GVRT_ERR_IO;
}

}  // extern "C"
