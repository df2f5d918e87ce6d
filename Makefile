# Builds rrin_amd/librrin_hip.so for gfx950 (MI355X).  `make -j16`
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
# No packed FP32 VALU ops (v_pk_fma/mul/add_f32) in any kernel: measured on MI355X,
# the low element of a v_pk_fma_f32 in lanes 48-63 of a wave came out perturbed
# when a co-resident workgroup of another kernel on the CU ran LDS-DMA + MFMA
# (DESIGN.md §9).  The flag also reaches the host compile, which ignores it
# (one "not a recognized feature" line per file).
NOPK := -Xclang -target-feature -Xclang -packed-fp32-ops
CXXFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Iinclude $(NOPK)
SRC_DIR := rrin_amd/csrc
OBJ_DIR := build/obj
SRCS := $(wildcard $(SRC_DIR)/*.hip)
OBJS := $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(SRCS))
LIB := rrin_amd/librrin_hip.so
# kernel lab (tools/conv_lab.py ablate): the split16 conv with schedule knobs / ablations
LAB := rrin_amd/librrin_lab.so
# exact-fp32 conv with ablation knobs (tools/conv_lab.py ablate32)
LAB32 := rrin_amd/librrin_lab32.so

all: $(LIB)

lab: $(LAB) $(LAB32)

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(SRC_DIR)/common.hpp include/rrin_hip.h
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS)

$(LAB): $(SRC_DIR)/conv_f16.hip $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(CXXFLAGS) -DRRIN_LAB -shared -o $@ $<

$(LAB32): $(SRC_DIR)/conv_mfma.hip $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(CXXFLAGS) -DRRIN_LAB -shared -o $@ $<

# kernel register / LDS / occupancy report
resource: $(SRCS)
	$(HIPCC) $(CXXFLAGS) -Rpass-analysis=kernel-resource-usage -c $(SRC_DIR)/conv_mfma.hip -o /dev/null

clean:
	rm -rf build $(LIB) $(LAB) $(LAB32)

.PHONY: all lab clean resource
