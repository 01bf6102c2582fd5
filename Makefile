# Builds the hipgle C-ABI library for gfx950 (MI355X) in-tree.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value
SRC := sclmd_amd/csrc/gle_api.hip sclmd_amd/csrc/gle_kernels.hip sclmd_amd/csrc/gle_chain.hip sclmd_amd/csrc/gle_gmem.hip
HDR := sclmd_amd/csrc/gle_internal.h include/hipgle.h
LIB := sclmd_amd/_lib/libhipgle.so

all: $(LIB)

$(LIB): $(SRC) $(HDR)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -shared -o $@ $(SRC)

clean:
	rm -f $(LIB)

.PHONY: all clean
