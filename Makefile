# Builds rrin_amd/librrin_hip.so for gfx950 (MI355X).  `make -j16`
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
CXXFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Iinclude
SRC_DIR := rrin_amd/csrc
OBJ_DIR := build/obj
SRCS := $(wildcard $(SRC_DIR)/*.hip)
OBJS := $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(SRCS))
LIB := rrin_amd/librrin_hip.so
# kernel lab (tools/conv_lab.py ablate): the split16 conv with schedule knobs / ablations
LAB := rrin_amd/librrin_lab.so

all: $(LIB)

lab: $(LAB)

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(SRC_DIR)/common.hpp include/rrin_hip.h
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS)

$(LAB): $(SRC_DIR)/conv_f16.hip $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(CXXFLAGS) -DRRIN_LAB -shared -o $@ $<

# kernel register / LDS / occupancy report
resource: $(SRCS)
	$(HIPCC) $(CXXFLAGS) -Rpass-analysis=kernel-resource-usage -c $(SRC_DIR)/conv_mfma.hip -o /dev/null

clean:
	rm -rf build $(LIB) $(LAB)

.PHONY: all lab clean resource
