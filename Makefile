# Build of libpptkrx.so (product) and the oracle (test infrastructure).
#   make            -> pptk_amd/libpptkrx.so + oracle/liboracle.so (+ oracle/_ref),
#                      tests/hooks/libpptkrx_hooks.so, harness/*.so
#   make tools      -> the probe libraries under tools/ (not built by default)
# gfx950 only; hipcc cross-compiles without a GPU.
HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
ARCH ?= gfx950
OBJDIR := build/obj
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -Iinclude -I/opt/rocm/include
CFLAGS := -O2 -std=gnu11 -fPIC -Wall -Wextra -Iinclude

LIB := pptk_amd/libpptkrx.so
HIP_SRCS := pptk_amd/csrc/rx_kernel.hip pptk_amd/csrc/rx_bin.hip pptk_amd/csrc/rx_permit.hip \
            pptk_amd/csrc/rx_capi.hip pptk_amd/csrc/rx_comm.hip pptk_amd/csrc/rx_ring.hip
C_SRCS := pptk_amd/csrc/host/ipcksum.c pptk_amd/csrc/host/hashseed.c pptk_amd/csrc/host/tcpopt.c \
          pptk_amd/csrc/host/iphash.c pptk_amd/csrc/host/timerlink.c
HDRS := $(wildcard include/*.h) pptk_amd/csrc/rx_internal.h
HIP_OBJS := $(patsubst pptk_amd/csrc/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))
C_OBJS := $(patsubst pptk_amd/csrc/host/%.c,$(OBJDIR)/host/%.o,$(C_SRCS))

all: $(LIB) oracle

$(OBJDIR)/%.o: pptk_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/host/%.o: pptk_amd/csrc/host/%.c $(HDRS)
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS) $(C_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl

oracle:
	$(MAKE) -C oracle

# The test library: the product with its fault-injection knobs compiled in
# (-DPPTK_RX_TEST_HOOKS: a rate-limiter workgroup held past its barrier
# deadline, a stalled communicator warm-up).  Only the failure-path tests load
# it; the product library never reads those knobs.
HOOKS_LIB := tests/hooks/libpptkrx_hooks.so
HOOKS_SRCS := pptk_amd/csrc/rx_permit.hip pptk_amd/csrc/rx_comm.hip
HOOKS_OBJS := $(patsubst pptk_amd/csrc/%.hip,$(OBJDIR)/hooks/%.o,$(HOOKS_SRCS))

$(OBJDIR)/hooks/%.o: pptk_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DPPTK_RX_TEST_HOOKS -c $< -o $@

$(HOOKS_LIB): $(filter-out $(OBJDIR)/rx_permit.o $(OBJDIR)/rx_comm.o,$(HIP_OBJS)) $(HOOKS_OBJS) $(C_OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -ldl

hooks: $(HOOKS_LIB)
all: $(HOOKS_LIB)

# A/B builds of the product library with extra defines, e.g.
#   make abvariant NAME=full DEFS=-DPPTK_RX_FULL_UNROLL
abvariant:
	$(MAKE) OBJDIR=build/ab_$(NAME)/obj LIB=build/ab_$(NAME)/libpptkrx.so \
	  HIPFLAGS="$(HIPFLAGS) $(DEFS)" build/ab_$(NAME)/libpptkrx.so

asm: $(HIP_SRCS)
	@mkdir -p build/asm
	cd build/asm && $(HIPCC) $(HIPFLAGS) -I../../include -c ../../pptk_amd/csrc/rx_kernel.hip -save-temps -o rx_kernel.o -Rpass-analysis=kernel-resource-usage 2> resource.txt; true

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean asm

# Measurement harness (bench.py and the GPU tests): synthetic frames generated
# in HBM and the trivial kernels that give the box's speed of light.
HARNESS_LIBS := harness/libpptksynth.so harness/libmembench.so harness/librwmix.so

harness/lib%.so: harness/%.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -fPIC -shared -std=c++17 -o $@ $<

harness/libpptksynth.so: harness/synth.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -fPIC -shared -std=c++17 -o $@ $<

all: $(HARNESS_LIBS)

# Probes (measured-and-kept evidence for DESIGN.md, not part of the product
# or of the default build): make tools
PROBE_LIBS := tools/libglds_probe.so tools/libteam_probe.so tools/libepoch_probe.so \
              tools/libstandin.so

tools/lib%.so: tools/%.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -fPIC -shared -std=c++17 -o $@ $<

tools: $(PROBE_LIBS)

.PHONY: tools
