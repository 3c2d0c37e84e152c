# Top-level build: libdgn.so (HIP kernels + C ABI, gfx950), the C++ facade, and the oracle.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := defect-gnn-cpp_amd
CSRC     := $(PKG)/csrc
BUILD    := $(PKG)/build
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -I$(CSRC) -Iinclude \
            -mllvm -amdgpu-atomic-optimizer-strategy=DPP
LIB      := $(PKG)/lib/libdgn.so

KOBJS := $(BUILD)/graph_kernels.o $(BUILD)/betti_kernels.o $(BUILD)/betti_wide.o $(BUILD)/betti_rank.o \
         $(BUILD)/betti_split.o $(BUILD)/node_kernels.o $(BUILD)/dgn_api.o

all: $(LIB) facade oracle

# C++ facade mirroring the reference include/graph + include/topology API over the C ABI
FDIR     := $(PKG)/cpp
FBUILD   := $(PKG)/build/facade
FACADE   := $(PKG)/lib/libdgn_facade.so
FBIN     := $(PKG)/bin
CXX      ?= g++
FFLAGS   := -O2 -std=c++17 -fPIC -Wall -Wextra -Iinclude -I$(FDIR)/include
FSRCS    := $(wildcard $(FDIR)/src/*.cpp)
FOBJS    := $(patsubst $(FDIR)/src/%.cpp,$(FBUILD)/%.o,$(FSRCS))
FHDRS    := $(shell find $(FDIR)/include -name '*.hpp') include/dgn.h
facade: $(FACADE) $(FBIN)/preprocess_betti $(FBIN)/facade_check
$(FBUILD)/%.o: $(FDIR)/src/%.cpp $(FHDRS)
	@mkdir -p $(FBUILD)
	$(CXX) $(FFLAGS) -c $< -o $@
$(FACADE): $(FOBJS) $(LIB)
	$(CXX) -shared -o $@ $(FOBJS) -L$(PKG)/lib -ldgn -Wl,-rpath,'$$ORIGIN'
$(FBIN)/%: $(FDIR)/tools/%.cpp $(FACADE) $(FHDRS)
	@mkdir -p $(FBIN)
	$(CXX) $(FFLAGS) -o $@ $< -L$(PKG)/lib -ldgn_facade -ldgn -Wl,-rpath,'$$ORIGIN/../lib'

$(BUILD)/%.o: $(CSRC)/%.hip $(CSRC)/dgn_device.hpp $(CSRC)/dgn_internal.hpp
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the narrow Betti kernel (issue-bound, 64 VGPRs at 8 waves per SIMD) with the register-minimising
# iterative scheduler: betti_vr -0.6 ms per shard (same-box A/B, five rounds);
# the other kernels lose with it (distance kernel +0.1 ms, 10 A wide kernel +5 %)
$(BUILD)/betti_kernels.o: HIPFLAGS += -mllvm -amdgpu-sched-strategy=iterative-minreg

$(BUILD)/dgn_api.o: $(CSRC)/dgn_api.cpp include/dgn.h $(CSRC)/dgn_internal.hpp $(CSRC)/dgn_device.hpp
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(KOBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(KOBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(SAN) $(LIB) $(FACADE) $(FBIN)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean facade

# Host-code sanitizer run (ASan + UBSan) over the CPU oracle and the facade's host-only code
# (parser, Structure, PCA): builds build_san/san_check and runs it on the POSCAR fixtures.
SAN      := $(PKG)/build_san
SANFLAGS := -O1 -g -std=c++17 -fno-omit-frame-pointer -ffp-contract=off -fsanitize=address,undefined \
            -fno-sanitize-recover=undefined -Iinclude -I$(FDIR)/include -Ioracle
sanitize: $(SAN)/san_check
	mkdir -p $(SAN)/tmp
	ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1 $(SAN)/san_check tests/golden/poscar $(SAN)/tmp
$(SAN)/san_check: $(FDIR)/tools/san_check.cpp oracle/oracle.cpp oracle/oracle.h $(FDIR)/src/vasp_parser.cpp \
                  $(FDIR)/src/structure.cpp $(FDIR)/src/pca.cpp $(FHDRS)
	@mkdir -p $(SAN)
	$(CXX) $(SANFLAGS) -o $@ $(FDIR)/tools/san_check.cpp oracle/oracle.cpp $(FDIR)/src/vasp_parser.cpp \
	    $(FDIR)/src/structure.cpp $(FDIR)/src/pca.cpp
.PHONY: sanitize
