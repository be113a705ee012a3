# Native build for triton-mi355x.  `make -j16` builds every shared object
# in-tree (the .so files travel to the GPU box with the repo snapshot).
#   libcshm.so        POSIX shm C ABI (tritonclient.utils.shared_memory)
#   libtcamd_hip.so   HIP runtime glue + CDNA4 kernels (gfx950) + native batch executor
#   libtcamd_host.so  host codecs (BYTES pack/scan)
HIPCC      ?= /opt/rocm/bin/hipcc
CXX        ?= g++
ARCH       ?= gfx950
CXXFLAGS   ?= -O3 -std=c++17 -fPIC -Wall -Wextra
HIPFLAGS   ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall
ROCM       ?= /opt/rocm

CSHM   = tritonclient/utils/shared_memory/libcshm.so
HIPLIB = triton_client_amd/ops/lib/libtcamd_hip.so
HOSTLIB= triton_client_amd/ops/lib/libtcamd_host.so

HIP_SRCS = $(wildcard csrc/kernels/*.hip) $(wildcard csrc/hipshm/*.hip) $(wildcard csrc/runtime/*.hip)
HIP_OBJS = $(patsubst csrc/%.hip,build/%.o,$(HIP_SRCS))

all: $(CSHM) $(HIPLIB) $(HOSTLIB)

$(CSHM): csrc/cshm/cshm.cc
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -shared -o $@ $< -lrt

build/%.o: csrc/%.hip $(wildcard csrc/kernels/*.h) $(wildcard csrc/hipshm/*.h) csrc/cpp/server/tcserve.h
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -Icsrc -c -o $@ $<

$(HIPLIB): $(HIP_OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -L$(ROCM)/lib -lamdhip64

$(HOSTLIB): csrc/host/host_codec.cc
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -shared -o $@ $<

clean:
	rm -rf build $(CSHM) $(HIPLIB) $(HOSTLIB)

.PHONY: all clean
