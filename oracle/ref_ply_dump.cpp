// ref_ply_dump.cpp — test-infrastructure driver around the REFERENCE's own PLY loader
// (vk3DGRT::PLYLoader::loadPLYModel, /root/reference/base/Vulkan3DGRTModel.cpp:7-125, reading with
// the vendored miniply).  Built by oracle/ref.mk into oracle/_ref/ (never committed, never shipped).
// Usage: ref_ply_dump in.ply out.bin  -> writes u64 n, then positions, f_dc, f_rest, opacity, scale,
// rotation as raw float32 arrays (SplatSet order).
#include <cstdio>
#include <cstdint>
#include "Vulkan3DGRTModel.h"

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    vk3DGRT::SplatSet s;
    vk3DGRT::PLYLoader loader;
    if (!loader.loadPLYModel(argv[1], s)) return 1;
    FILE* f = std::fopen(argv[2], "wb");
    if (!f) return 3;
    const uint64_t n = s.size();
    std::fwrite(&n, 8, 1, f);
    const std::vector<float>* arrs[] = {&s.positions, &s.f_dc, &s.f_rest, &s.opacity, &s.scale, &s.rotation};
    for (auto* a : arrs) std::fwrite(a->data(), 4, a->size(), f);
    std::fclose(f);
    return 0;
}
