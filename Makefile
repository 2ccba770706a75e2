# Build the MI355X engine (gfx950) and the CPU oracle.
#   make            -> ctstraffic_amd/libcts_engine.so + oracle/libcts_oracle.so + the C++ device sample
#                      (ctstraffic_amd/build/device_verify) + the ceiling/ablation tools
#   make asm        -> ctstraffic_amd/build/cts_kernels-gfx950.s (disassembly for inspection)
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
HIPFLAGS  ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=$(ARCH) -Iinclude -Ictstraffic_amd/csrc
CSRC      := ctstraffic_amd/csrc
ENGINE_SO := ctstraffic_amd/libcts_engine.so
HDRS      := $(wildcard include/*.h) $(wildcard $(CSRC)/*.hpp)
SRCS      := $(wildcard $(CSRC)/*.hip) $(wildcard $(CSRC)/*.cpp)
OBJS      := $(patsubst $(CSRC)/%,ctstraffic_amd/build/%.o,$(SRCS))

DEVICE_VERIFY := ctstraffic_amd/build/device_verify
TOOLS := tools/hbm_read_ceiling tools/verify_ablation

SYNC_PROBE := tools/sync_probe

all: $(ENGINE_SO) oracle $(DEVICE_VERIFY) $(TOOLS) $(SYNC_PROBE)

# SYNC-mode (per-completion) verify latency probe against the C ABI
$(SYNC_PROBE): tools/sync_probe.cpp $(ENGINE_SO) include/cts_engine.h
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/../ctstraffic_amd' -lpthread

# measurement references used by tools/gpu_round.sh (plain streaming read/write ceilings, verify ablation)
tools/%: tools/%.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 $< -o $@

# C++ device-resident sample against the C ABI (run on the GPU box by tests/test_cpp_abi.py)
$(DEVICE_VERIFY): tests/cpp/device_verify.cpp $(ENGINE_SO) include/cts_engine.h
	@mkdir -p ctstraffic_amd/build
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/..'

ctstraffic_amd/build/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p ctstraffic_amd/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ENGINE_SO): $(OBJS) $(CSRC)/exports.map
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS) -Wl,-soname,libcts_engine.so -Wl,--version-script=$(CSRC)/exports.map

oracle:
	$(MAKE) -s -C oracle

asm: $(CSRC)/cts_kernels.hip $(HDRS)
	@mkdir -p ctstraffic_amd/build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S $< -o ctstraffic_amd/build/cts_kernels-$(ARCH).s

clean:
	rm -rf ctstraffic_amd/build $(ENGINE_SO) $(TOOLS) $(SYNC_PROBE)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle asm clean
