// The C++ host layer's vks::Benchmark (3dgvrt_lightfield_amd/host/gvrt_host.h) driven exactly as
// oracle/ref_bench_dump.cpp drives the reference's (base/benchmark.hpp): same arguments, same fps.txt.
//
//   bench_results <out file> <device name> <driver version> <output frame times 0|1> <ms> [<ms> ...]
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gvrt_host.h"

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: bench_results out device driver frametimes(0|1) [ms ...]\n");
        return 2;
    }
    gvrt_device_properties props{};
    std::snprintf(props.device_name, sizeof(props.device_name), "%s", argv[2]);
    props.driver_version = (uint32_t)std::strtoul(argv[3], nullptr, 10);
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
