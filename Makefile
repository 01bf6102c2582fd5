# Builds the hipgle C-ABI library for gfx950 (MI355X) in-tree (one object per source, `make -j`).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value
SRC := sclmd_amd/csrc/gle_api.hip sclmd_amd/csrc/gle_kernels.hip sclmd_amd/csrc/gle_chain.hip sclmd_amd/csrc/gle_gmem.hip
HDR := sclmd_amd/csrc/gle_internal.h sclmd_amd/csrc/gle_cgemm.h include/hipgle.h
LDLIBS := -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
OBJDIR := build/rel
OBJ := $(patsubst sclmd_amd/csrc/%.hip,$(OBJDIR)/%.o,$(SRC))
LIB := sclmd_amd/_lib/libhipgle.so
# experiment build: GLE_* environment switches (plan variants, timing-only variants that skip
# work); load it with SCLMD_AMD_LIB=sclmd_amd/_lib/libhipgle_exp.so.  Never used by tests/bench.
# EXPFLAGS adds compile-time variants (e.g. EXPFLAGS="-DCH_U1=4" EXPNAME=u4).
EXPNAME ?= exp
EXPFLAGS ?=
EXPDIR := build/$(EXPNAME)
EXPOBJ := $(patsubst sclmd_amd/csrc/%.hip,$(EXPDIR)/%.o,$(SRC))
LIB_EXP := sclmd_amd/_lib/libhipgle_$(EXPNAME).so

all: $(LIB)

$(OBJDIR)/%.o: sclmd_amd/csrc/%.hip $(HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -c -o $@ $<

$(LIB): $(OBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ) $(LDLIBS)

experiments: $(LIB_EXP)

$(EXPDIR)/%.o: sclmd_amd/csrc/%.hip $(HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -DGLE_EXPERIMENTS $(EXPFLAGS) -c -o $@ $<

$(LIB_EXP): $(EXPOBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(EXPOBJ) $(LDLIBS)

clean:
	rm -rf build $(LIB) sclmd_amd/_lib/libhipgle_*.so

.PHONY: all clean experiments
