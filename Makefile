# Builds everything in-tree (the .so files travel to the GPU box with the
# repo snapshot):
#   aby3_amd/lib/libaby3gpu.so   HIP kernels + the C-ABI of include/aby3gpu.h (gfx950)
#   aby3_amd/lib/libaby3.so      C++ host runtime (Sh3Runtime, Sh3Evaluator, ...)
#   oracle/build/liborc.so       CPU oracle (test infrastructure only)
#   tests/cpp/build/*            protocol-level test and bench drivers
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
CXX      ?= g++
CXXFLAGS ?= -std=c++17 -O2 -fPIC -Wall -Wno-unused-function -pthread
JOBS     ?= 8

GPU_SRC  := $(wildcard aby3_amd/csrc/*.hip)
GPU_HDR  := $(wildcard aby3_amd/csrc/*.h) include/aby3gpu.h
GPU_OBJ  := $(GPU_SRC:aby3_amd/csrc/%.hip=build/gpu/%.o)
GPU_LIB  := aby3_amd/lib/libaby3gpu.so

HOST_SRC := $(wildcard aby3_amd/host/*.cpp)
HOST_HDR := $(wildcard aby3_amd/host/*.h) include/aby3gpu.h include/aby3.h
HOST_OBJ := $(HOST_SRC:aby3_amd/host/%.cpp=build/host/%.o)
HOST_LIB := aby3_amd/lib/libaby3.so

TEST_SRC := $(wildcard tests/cpp/*.cpp)
TEST_BIN := $(TEST_SRC:tests/cpp/%.cpp=tests/cpp/build/%)

all: gpu host oracle tests

gpu: $(GPU_LIB)
host: $(HOST_LIB)
tests: $(TEST_BIN)
oracle:
	$(MAKE) -C oracle

build/gpu/%.o: aby3_amd/csrc/%.hip $(GPU_HDR)
	@mkdir -p build/gpu
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(GPU_LIB): $(GPU_OBJ)
	@mkdir -p aby3_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

build/host/%.o: aby3_amd/host/%.cpp $(HOST_HDR)
	@mkdir -p build/host
	$(CXX) $(CXXFLAGS) -Iinclude -Iaby3_amd/host -c $< -o $@

$(HOST_LIB): $(HOST_OBJ) $(GPU_LIB)
	$(CXX) -shared -o $@ $(HOST_OBJ) -Laby3_amd/lib -laby3gpu -Wl,-rpath,'$$ORIGIN' -pthread

tests/cpp/build/%: tests/cpp/%.cpp $(HOST_LIB) oracle
	@mkdir -p tests/cpp/build
	$(CXX) $(CXXFLAGS) -Iinclude -Iaby3_amd/host -Ioracle/src $< -o $@ \
	    -Laby3_amd/lib -laby3 -laby3gpu oracle/build/liborc.a \
	    -Wl,-rpath,'$$ORIGIN/../../../aby3_amd/lib' -pthread

clean:
	rm -rf build aby3_amd/lib tests/cpp/build
	$(MAKE) -C oracle clean

.PHONY: all gpu host tests oracle clean
