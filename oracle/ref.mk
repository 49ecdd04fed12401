# Builds the reference's PLY loader from its own sources (no reference build system): the two
# translation units on the loader path, compiled where they lie under /root/reference, plus our
# driver.  --gc-sections drops the Vulkan buffer-upload members of the same file, which the dump
# never calls.  Outputs only into oracle/_ref/.
REF ?= /root/reference
CXX ?= g++
INC = -I$(REF)/base -I$(REF)/external -I$(REF)/external/glm -I$(REF)/external/miniply -I$(REF)/external/vulkan
FLAGS = -O2 -std=c++20 -ffunction-sections -fdata-sections -w

all: _ref/ref_ply_dump

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
