# Builds the hipgle C-ABI library for gfx950 (MI355X) in-tree.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value
SRC := sclmd_amd/csrc/gle_api.hip sclmd_amd/csrc/gle_kernels.hip sclmd_amd/csrc/gle_chain.hip sclmd_amd/csrc/gle_gmem.hip
HDR := sclmd_amd/csrc/gle_internal.h include/hipgle.h
LDLIBS := -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
LIB := sclmd_amd/_lib/libhipgle.so
# experiment build: GLE_* environment switches (plan variants, timing-only variants that skip
# work); load it with SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so.  Never used by tests/bench.
LIB_EXP := sclmd_amd/_lib/libhipgle_exp.so

all: $(LIB)

$(LIB): $(SRC) $(HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -shared -o $@ $(SRC) $(LDLIBS)

experiments: $(LIB_EXP)

$(LIB_EXP): $(SRC) $(HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -DGLE_EXPERIMENTS -shared -o $@ $(SRC) $(LDLIBS)

clean:
	rm -f $(LIB) $(LIB_EXP)

.PHONY: all clean experiments
