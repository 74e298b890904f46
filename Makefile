# Builds librvx.so (HIP/gfx950, the product) and the CPU oracle (test infrastructure).
# `python -c "import __graft_entry__ as g; g.build()"` drives this file.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CSRC     := ruvector_amd/csrc
BUILD    := build
# -ffp-contract=off: no implicit FMA, so kernels that restate the reference's
# scalar arithmetic (distances, aggregation) reproduce it bit for bit; FMA is
# only used where a kernel asks for it (MFMA, fmaf).
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -Iinclude -I$(CSRC) \
            -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-result -Wno-unused-value
LDFLAGS  := -shared --offload-arch=$(ARCH) -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib

SRCS := $(wildcard $(CSRC)/*.cpp) $(wildcard $(CSRC)/*.hip)
OBJS := $(patsubst $(CSRC)/%,$(BUILD)/%.o,$(SRCS))
HDRS := $(wildcard $(CSRC)/*.hpp) include/rvx/rvx.h
# Binary provenance: sha256 over every source the library is built from (sorted
# paths, contents concatenated), compiled into rvx_version(); ruvector_amd
# recomputes it from the shipped sources and refuses a stale librvx.so.
PROV := $(sort $(SRCS) $(HDRS))
SRC_HASH = $(shell cat $(PROV) | sha256sum | cut -c1-16)

LIB := ruvector_amd/librvx.so

all: $(LIB) oracle

$(BUILD)/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

# runtime.cpp carries the source hash, so it rebuilds whenever any source changes
$(BUILD)/runtime.cpp.o: $(CSRC)/runtime.cpp $(SRCS) $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DRVX_SRC_HASH=\"$(SRC_HASH)\" -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) $(LDFLAGS) -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
