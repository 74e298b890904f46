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

# Host-side sanitizer build (tests/test_asan.py): the translation units that parse
# caller-supplied files and text — hnsw_rs dumps (api_hnswio.cpp), feature files
# (api_io.cpp), RuvectorLayer JSON (api_gnn.cpp + json.hpp) — and the error plumbing
# (runtime.cpp) compiled with ASan + UBSan on the host side only (-Xarch_host: device
# code is never instrumented), linked with the normal objects of every other file.
# Loaded through RVX_LIB with the clang ASan runtime preloaded; never shipped.
ASAN_DIR   := $(BUILD)/asan
ASAN_SRCS  := api_hnswio.cpp api_io.cpp api_gnn.cpp runtime.cpp
ASANFLAGS  := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
              -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer
ASAN_OBJS  := $(patsubst %,$(ASAN_DIR)/%.o,$(ASAN_SRCS))
PLAIN_OBJS := $(filter-out $(patsubst %,$(BUILD)/%.o,$(ASAN_SRCS)),$(OBJS))
ASAN_LIB   := $(ASAN_DIR)/librvx_asan.so

$(ASAN_DIR)/%.o: $(CSRC)/% $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(HIPFLAGS) $(ASANFLAGS) -DRVX_SRC_HASH=\"$(SRC_HASH)\" -x hip -c $< -o $@

$(ASAN_LIB): $(ASAN_OBJS) $(PLAIN_OBJS)
	$(HIPCC) $(LDFLAGS) -fsanitize=address,undefined -shared-libsan -o $@ $(ASAN_OBJS) $(PLAIN_OBJS)

asan: $(ASAN_LIB)
	$(MAKE) -C oracle asan

clean:
	rm -rf $(BUILD) $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean asan
