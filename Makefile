# Build of the product library (libzrt.so: HIP kernels for gfx950 + host C++)
# and the drop-in CLI.  Everything lands in-tree so it travels to the GPU box.
ROCM      ?= /opt/rocm
HIPCC     := $(ROCM)/bin/hipcc
CXX       ?= g++
ARCH      ?= gfx950
PKG       := zig_raytracing_contest_amd
SRC       := $(PKG)/csrc
OBJ       := build/obj
# -ffp-contract=off everywhere: the reference (Zig) never contracts a*b+c.
# -fno-slp-vectorize: the SLP pass pairs f32 products into v_pk_mul_f32 and
# pays for each pair with v_mov copies into adjacent registers (21 in a park
# test sub-round); without it the park kernel is 2.5% and the primary 3%
# faster, 7 VGPRs lighter (r05an).
HIPFLAGS  := -O3 -fPIC -std=c++17 --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
             -Wall -Wno-unused-function -Iinclude
CXXFLAGS  := -O2 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -Wall -Iinclude -pthread
HDRS      := include/zrt.h $(SRC)/zrt_math.h $(SRC)/zrt_internal.h $(SRC)/dda.h $(SRC)/geometry.h $(SRC)/device_geometry.h
HOST_SRCS := $(filter-out $(SRC)/cli.cpp,$(wildcard $(SRC)/*.cpp))
HOST_OBJS := $(patsubst $(SRC)/%.cpp,$(OBJ)/%.o,$(HOST_SRCS))
LIB       := $(PKG)/libzrt.so
CLI       := $(PKG)/bin/zrt

PROBE     := tools/bin/dpp_probe
INITPROBE := tools/bin/hip_init_probe
SWEEP_LIB := tools/bin/sweep/libzrt.so

all: $(LIB) $(if $(wildcard $(SRC)/cli.cpp),$(CLI)) $(PROBE) $(INITPROBE) $(SWEEP_LIB) oracle

$(OBJ)/%.o: $(SRC)/%.cpp $(HDRS) $(wildcard $(SRC)/*.h)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OBJ)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

HIP_OBJS  := $(patsubst $(SRC)/%.hip,$(OBJ)/%.o,$(wildcard $(SRC)/*.hip))

$(LIB): $(HIP_OBJS) $(HOST_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lz -pthread

$(CLI): $(SRC)/cli.cpp $(LIB) include/zrt.h
	@mkdir -p $(PKG)/bin
	$(CXX) $(CXXFLAGS) -o $@ $(SRC)/cli.cpp -L$(PKG) -lzrt -Wl,-rpath,'$$ORIGIN/..' -Wl,-rpath,$(ROCM)/lib

# DPP-under-partial-EXEC check (DESIGN.md §5, round 1's park-mode fault)
$(PROBE): tools/dpp_probe.hip
	@mkdir -p tools/bin
	$(HIPCC) -O3 --offload-arch=$(ARCH) -o $@ $<

# HIP start-up split (tools/startup_probe.py)
$(INITPROBE): tools/hip_init_probe.cpp
	@mkdir -p tools/bin
	$(HIPCC) -O2 -o $@ $< -ldl

# Tuning build: the park-kernel schedule read from ZRT_PARK_T / ZRT_PARK_R,
# ZRT_SETS, and the s_memtime round profiles (ZRT_PARK_PROFILE); used through
# ZRT_LIB=<path> by tools/ and by the schedule-extreme and pass-set parity
# tests (tests/test_gpu_parity.py), never by bench.py or the product path.
sweep: $(SWEEP_LIB)
$(SWEEP_LIB): $(SRC)/render.hip $(HDRS) $(filter-out $(OBJ)/render.o,$(HIP_OBJS)) $(HOST_OBJS)
	@mkdir -p tools/bin/sweep
	$(HIPCC) $(HIPFLAGS) -DZRT_SWEEP -c $(SRC)/render.hip -o tools/bin/sweep/render.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ tools/bin/sweep/render.o $(filter-out $(OBJ)/render.o,$(HIP_OBJS)) $(HOST_OBJS) -lz -pthread

# A/B build of render.hip with extra defines (tools/gpu_ab.sh):
#   make variant V=name D="-DZRT_FOO"  ->  tools/bin/name/libzrt.so
variant: $(filter-out $(OBJ)/render.o,$(HIP_OBJS)) $(HOST_OBJS)
	@mkdir -p tools/bin/$(V)
	$(HIPCC) $(HIPFLAGS) $(D) -c $(SRC)/render.hip -o tools/bin/$(V)/render.o
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o tools/bin/$(V)/libzrt.so tools/bin/$(V)/render.o $^ -lz -pthread

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB) $(PKG)/bin tools/bin
	$(MAKE) -s -C oracle clean

.PHONY: all clean oracle sweep variant
