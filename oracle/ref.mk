# Builds the reference's PLY loader from its own sources (no reference build system): the two
# translation units on the loader path, compiled where they lie under /root/reference, plus our
# driver.  --gc-sections drops the Vulkan buffer-upload members of the same file, which the dump
# never calls.  Outputs only into oracle/_ref/.
REF ?= /root/reference
CXX ?= g++
INC = -I$(REF)/base -I$(REF)/external -I$(REF)/external/glm -I$(REF)/external/miniply -I$(REF)/external/vulkan
FLAGS = -O2 -std=c++20 -ffunction-sections -fdata-sections -w

all: _ref/ref_ply_dump _ref/ref_camera_dump _ref/ref_bench_dump

_ref/%.o: | _ref
_ref:
	mkdir -p _ref

_ref/miniply.o: $(REF)/external/miniply/miniply.cpp | _ref
	$(CXX) $(FLAGS) $(INC) -c $< -o $@

_ref/Vulkan3DGRTModel.o: $(REF)/base/Vulkan3DGRTModel.cpp | _ref
	$(CXX) $(FLAGS) $(INC) -c $< -o $@

_ref/ref_ply_dump.o: ref_ply_dump.cpp | _ref
	$(CXX) $(FLAGS) $(INC) -c $< -o $@

_ref/ref_ply_dump: _ref/ref_ply_dump.o _ref/Vulkan3DGRTModel.o _ref/miniply.o
	$(CXX) -Wl,--gc-sections -o $@ $^

.PHONY: all

# The reference's camera math (base/camera.hpp, base/LoadCamera.hpp, vendored glm + nlohmann json),
# with the reference's own glm defines (base/VulkanRTBase.h:51-53).  Plain -O2 for x86-64: SSE float
# arithmetic, no FMA contraction, libm sinf/cosf/tanf -- the same arithmetic the host mirrors use.
CAM_DEFS = -DGLM_FORCE_RADIANS -DGLM_FORCE_DEPTH_ZERO_TO_ONE -DGLM_ENABLE_EXPERIMENTAL
_ref/ref_camera_dump: ref_camera_dump.cpp $(REF)/base/camera.hpp $(REF)/base/LoadCamera.hpp | _ref
	$(CXX) -O2 -std=c++17 -ffp-contract=off -w $(CAM_DEFS) -I$(REF)/base -I$(REF)/external/glm -I$(REF)/external/tinygltf $< -o $@

# The reference's vks::Benchmark (base/benchmark.hpp) with its vendored Vulkan headers (types only, nothing
# linked): writes the reference's fps.txt for given frame times.
_ref/ref_bench_dump: ref_bench_dump.cpp $(REF)/base/benchmark.hpp | _ref
	$(CXX) -O2 -std=c++17 -w -I$(REF)/base -I$(REF)/external/vulkan -I$(REF)/external $< -o $@
