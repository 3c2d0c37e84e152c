# Top-level build: libdgn.so (HIP kernels + C ABI, gfx950), the C++ facade, and the oracle.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := defect-gnn-cpp_amd
CSRC     := $(PKG)/csrc
BUILD    := $(PKG)/build
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -I$(CSRC) -Iinclude
LIB      := $(PKG)/lib/libdgn.so

KOBJS := $(BUILD)/graph_kernels.o $(BUILD)/betti_kernels.o $(BUILD)/dgn_api.o

all: $(LIB) oracle

$(BUILD)/%.o: $(CSRC)/%.hip $(CSRC)/dgn_device.hpp $(CSRC)/dgn_internal.hpp
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/dgn_api.o: $(CSRC)/dgn_api.cpp include/dgn.h $(CSRC)/dgn_internal.hpp
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(KOBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(KOBJS)

oracle:
	$(MAKE) -C oracle

# diagnostics variant: per-phase cycle stamps in the Betti kernel (never used by bench/tests)
DBUILD := $(PKG)/build_diag
DIAG   := $(PKG)/lib/libdgn_diag.so
diag: $(DIAG)
$(DBUILD)/%.o: $(CSRC)/%.hip $(CSRC)/dgn_device.hpp $(CSRC)/dgn_internal.hpp
	@mkdir -p $(DBUILD)
	$(HIPCC) $(HIPFLAGS) -DDGN_PHASE_TIMING -c $< -o $@
$(DBUILD)/dgn_api.o: $(CSRC)/dgn_api.cpp include/dgn.h $(CSRC)/dgn_internal.hpp
	@mkdir -p $(DBUILD)
	$(HIPCC) $(HIPFLAGS) -DDGN_PHASE_TIMING -x hip -c $< -o $@
$(DIAG): $(DBUILD)/graph_kernels.o $(DBUILD)/betti_kernels.o $(DBUILD)/dgn_api.o
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

clean:
	rm -rf $(BUILD) $(LIB) $(DBUILD) $(DIAG)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean diag
