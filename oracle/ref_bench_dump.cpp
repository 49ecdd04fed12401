// Test infrastructure (oracle/_ref, built by ref.mk from /root/reference; never shipped or measured).
// Drives the reference's own vks::Benchmark (base/benchmark.hpp:20-106) over given frame times and lets it
// write its fps.txt (saveResults, :77-104), so tests/test_host_cpp.py can compare the C++ host layer's
// vks::Benchmark::saveResults byte for byte.  The Vulkan device properties come from the reference's
// vendored headers (external/vulkan/vulkan_core.h, types only: nothing is linked).
//
//   ref_bench_dump <out file> <device name> <driver version> <output frame times 0|1> <ms> [<ms> ...]
//
// run() is called with warmup = duration = 0 (its loops do not execute), then the frame times are entered
// as run()'s benchmark loop enters them (runtime += t, frameTimes.push_back(t), ++frameCount).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <numeric>

#include <vulkan/vulkan_core.h>

#include "benchmark.hpp"

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: ref_bench_dump out device driver frametimes(0|1) [ms ...]\n");
        return 2;
    }
    VkPhysicalDeviceProperties props{};
    std::strncpy(props.deviceName, argv[2], sizeof(props.deviceName) - 1);
    props.driverVersion = (uint32_t)std::strtoul(argv[3], nullptr, 10);
    vks::Benchmark b;
    b.filename = argv[1];
    b.outputFrameTimes = std::atoi(argv[4]) != 0;
    b.warmup = 0;
    b.duration = 0;
    b.run([] {}, props);
    for (int i = 5; i < argc; ++i) {
        const double t = std::strtod(argv[i], nullptr);
        b.runtime += t;
        b.frameTimes.push_back(t);
        b.frameCount++;
    }
    b.saveResults();
    return 0;
}
