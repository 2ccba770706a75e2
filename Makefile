# Build the MI355X engine (gfx950) and the CPU oracle.
#   make            -> ctstraffic_amd/libcts_engine.so (the product: one kernel per path) + oracle/libcts_oracle.so +
#                      the C++ device sample (ctstraffic_amd/build/device_verify) + what bench.py and the tests run
#                      (tools/libcts_bench_multi.so, tools/pattern_cpu_probe)
#   make probes     -> the measurement probes of tools/ (ceilings, timelines, ablations; built before an A/B call)
#   make asm        -> ctstraffic_amd/build/cts_kernels-gfx950.s (disassembly for inspection)
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
HIPFLAGS  ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=$(ARCH) -Iinclude -Ictstraffic_amd/csrc
CSRC      := ctstraffic_amd/csrc
ENGINE_SO := ctstraffic_amd/libcts_engine.so
HDRS      := $(wildcard include/*.h) $(wildcard $(CSRC)/*.hpp)
SRCS      := $(wildcard $(CSRC)/*.hip) $(wildcard $(CSRC)/*.cpp)
OBJS      := $(patsubst $(CSRC)/%,ctstraffic_amd/build/%.o,$(SRCS))
# -Bsymbolic: calls between the library's own cts_* entry points bind inside it (an A/B build of the same ABI can
# be loaded beside it)
SOFLAGS   := -shared -Wl,-Bsymbolic -Wl,--version-script=$(CSRC)/exports.map

DEVICE_VERIFY := ctstraffic_amd/build/device_verify
PROBES := tools/hbm_read_ceiling tools/verify_ablation tools/mailbox_probe tools/rw_mix_probe tools/write_shape_probe \
          tools/fill_bisect tools/fill_abi_probe tools/mailbox_bisect tools/ring_fill_probe tools/verify_timeline \
          tools/verify_timeline_kp tools/sync_probe tools/deferred_ab tools/slab_verify_probe tools/write_ceiling_rot tools/ring_order_probe \
          tools/first_read_probe
BENCH_MULTI := tools/libcts_bench_multi.so

all: $(ENGINE_SO) oracle $(DEVICE_VERIFY) $(BENCH_MULTI) tools/pattern_cpu_probe

probes: $(PROBES)

# bench.py's single-process leg (--engines N): the timed launches from one native thread per GPU
$(BENCH_MULTI): tools/bench_multi.cpp $(ENGINE_SO) include/cts_engine.h
	$(HIPCC) -O2 -std=c++17 -fPIC -shared -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/../ctstraffic_amd' -lpthread

# the first counter read after cts_counters_allreduce_prepare, by thread and idle time (diagnostic)
tools/first_read_probe: tools/first_read_probe.cpp $(ENGINE_SO) include/cts_engine.h
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/../ctstraffic_amd' -lpthread

# SYNC-mode (per-completion) verify latency probe against the C ABI
tools/sync_probe: tools/sync_probe.cpp $(ENGINE_SO) include/cts_engine.h
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/../ctstraffic_amd' -lpthread

# config-1 DEFERRED vs verify-off A/B: background PCIe reads, recv-ring footprint (diagnostic)
tools/deferred_ab: tools/deferred_ab.cpp $(ENGINE_SO) include/cts_engine.h include/cts_loopback.h
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/../ctstraffic_amd' -lpthread

# receive-thread CPU inside the ctsIoPattern calls (no sockets)
tools/pattern_cpu_probe: tools/pattern_cpu_probe.cpp $(ENGINE_SO) include/cts_pattern.h
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/../ctstraffic_amd' -lpthread

# measurement references used by tools/gpu_round.sh (plain streaming read/write ceilings, verify ablation)
tools/%: tools/%.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 $< -o $@

# the product fill kernel included verbatim (diagnostic)
tools/fill_bisect: tools/fill_bisect.hip $(CSRC)/cts_kernels.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) $< -o $@

# the product verify kernel beside a plain read of the same shape: times and per-workgroup timelines (diagnostic);
# the _kp build preloads the kernel arguments into SGPRs
tools/verify_timeline: tools/verify_timeline.hip $(CSRC)/cts_kernels.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) $< -o $@
tools/verify_timeline_kp: tools/verify_timeline.hip $(CSRC)/cts_kernels.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) -DCTS_TOOL_KERNARG_PRELOAD=1 \
	  -mllvm -amdgpu-kernarg-preload-count=16 $< -o $@

# the same with round 5's kernels (git show 236f346), for a same-box A/B of the verify (diagnostic, profiles/r06/h/)
ctstraffic_amd/build/cts_kernels_r05.hip:
	@mkdir -p ctstraffic_amd/build
	git show 236f346:ctstraffic_amd/csrc/cts_kernels.hip > $@
tools/verify_timeline_r05: tools/verify_timeline.hip ctstraffic_amd/build/cts_kernels_r05.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) -DCTS_TL_COUNTERS=5 \
	  '-DCTS_KERNELS_FILE="../ctstraffic_amd/build/cts_kernels_r05.hip"' $< -o $@

# a slim one-buffer-per-workgroup verify beside the product and the plain slab read (diagnostic, profiles/r05/d/)
tools/slab_verify_probe: tools/slab_verify_probe.hip $(CSRC)/cts_kernels.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) -mllvm -amdgpu-kernarg-preload-count=16 $< -o $@

# the HBM write ceiling on a rotated 4 GiB footprint beside the product fill kernel (diagnostic, profiles/r06/)
tools/write_ceiling_rot: tools/write_ceiling_rot.hip $(CSRC)/cts_kernels.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) $< -o $@

# the MediaStream ring fill in piece order beside the product's (diagnostic, profiles/r06/g/)
tools/ring_order_probe: tools/ring_order_probe.hip $(CSRC)/cts_kernels.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) $< -o $@

# the product MediaStream fill beside flat ring walks (diagnostic)
tools/ring_fill_probe: tools/ring_fill_probe.hip $(CSRC)/cts_kernels.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) $< -o $@

# the product mailbox kernel driven by a bare host loop (diagnostic)
tools/mailbox_bisect: tools/mailbox_bisect.hip $(CSRC)/cts_kernels.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) $< -o $@

# cts_fill through the C ABI without PyTorch (diagnostic)
tools/fill_abi_probe: tools/fill_abi_probe.cpp $(ENGINE_SO) include/cts_engine.h
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/../ctstraffic_amd'

# C++ device-resident sample against the C ABI (run on the GPU box by tests/test_cpp_abi.py)
$(DEVICE_VERIFY): tests/cpp/device_verify.cpp $(ENGINE_SO) include/cts_engine.h
	@mkdir -p ctstraffic_amd/build
	$(HIPCC) -O2 -std=c++17 -Iinclude $< -o $@ -Lctstraffic_amd -lcts_engine -Wl,-rpath,'$$ORIGIN/..'

# the kernels' arguments arrive preloaded in SGPRs instead of through a dependent scalar load from the kernarg
# segment: 0.23-0.29 us off every launch's start (config-2 verify 41.11 -> 40.82 us, a plain read 40.55 -> 40.32 us,
# tools/verify_timeline vs verify_timeline_kp alternated on one box, profiles/r04/b/); firmware without the feature
# runs the compiler's fallback prologue, which loads them as before
KERNARG_PRELOAD := -mllvm -amdgpu-kernarg-preload-count=16
ctstraffic_amd/build/cts_kernels.hip.o: HIPFLAGS += $(KERNARG_PRELOAD)

ctstraffic_amd/build/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p ctstraffic_amd/build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ENGINE_SO): $(OBJS) $(CSRC)/exports.map
	$(HIPCC) $(HIPFLAGS) $(SOFLAGS) -o $@ $(OBJS) -Wl,-soname,libcts_engine.so

oracle:
	$(MAKE) -s -C oracle

asm: $(CSRC)/cts_kernels.hip $(HDRS)
	@mkdir -p ctstraffic_amd/build
	$(HIPCC) $(HIPFLAGS) $(KERNARG_PRELOAD) --cuda-device-only -S $< -o ctstraffic_amd/build/cts_kernels-$(ARCH).s

clean:
	rm -rf ctstraffic_amd/build $(ENGINE_SO) $(PROBES) $(BENCH_MULTI) tools/pattern_cpu_probe
	$(MAKE) -s -C oracle clean

.PHONY: all probes oracle asm clean
