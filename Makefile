# Builds rrin_amd/librrin_hip.so for gfx950 (MI355X).  `make -j16`
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
# No packed FP32 VALU ops (v_pk_fma/mul/add_f32) in any kernel: measured on MI355X,
# a v_pk_fma_f32 whose low result reads src1's high half through op_sel:[0,1,0]
# gives a perturbed low element (lanes 48-63) while a co-resident workgroup of
# another kernel runs LDS-DMA + MFMA; the splat / op_sel_hi forms stay exact and
# packed code measured no faster.  The flag also reaches the host
# compile, which ignores it (one "not a recognized feature" line per file).
NOPK := -Xclang -target-feature -Xclang -packed-fp32-ops
CXXFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Iinclude $(NOPK)
# Machine scheduler (A/B: `make SCHED=max-ilp`).  The conv tiles' counted waits
# (RRIN_VMWAIT, common.hpp) hold for any VMEM issue order the vm_fence()s allow; every build
# checks that on its own gfx950 ISA (check-isa below) -- round 5's max-ilp build moved U loads
# across a DMA issue group and ran wrong (profiles/r06/isa/).
SCHED ?=
ifneq ($(SCHED),)
CXXFLAGS += -mllvm -amdgpu-sched-strategy=$(SCHED)
endif
# Per-source scheduler: the kind-6 tile (conv_winoc.hip) under max-ilp, 144.4-144.6 vs 143.6-144.0
# pairs/s on one box interleaved, GPU suite and repeat-bitwise green (profiles/r06/sched/).
SCHED_conv_winoc := max-ilp
sched_of = $(if $(SCHED_$(1)),-mllvm -amdgpu-sched-strategy=$(SCHED_$(1)))
SRC_DIR := rrin_amd/csrc
OBJ_DIR := build/obj
SRCS := $(wildcard $(SRC_DIR)/*.hip)
HDRS := $(wildcard $(SRC_DIR)/*.hpp) include/rrin_hip.h
OBJS := $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(SRCS))
LIB := rrin_amd/librrin_hip.so
# kernel lab (tools/conv_lab.py ablate): the split16 conv with schedule knobs / ablations
LAB := rrin_amd/librrin_lab.so
# exact-fp32 conv with ablation knobs (tools/conv_lab.py ablate32)
LAB32 := rrin_amd/librrin_lab32.so

all: $(LIB)

# check-isa: the device ISA of every product source (same flags), and tools/isa_vmcheck.py over
# it -- each declared counted wait must see exactly its declared loads on every path.  A
# prerequisite of the library, so a build whose compiler or flags reorder the staging loads fails
# here instead of computing wrong tiles on the GPU.
ISA_DIR := build/isa
ISA_OK := $(patsubst $(SRC_DIR)/%.hip,$(ISA_DIR)/%.ok,$(SRCS))
check-isa: $(ISA_OK)

$(ISA_DIR)/%.ok: $(SRC_DIR)/%.hip $(HDRS) tools/isa_vmcheck.py
	@mkdir -p $(ISA_DIR)
	$(HIPCC) $(CXXFLAGS) $(call sched_of,$*) --cuda-device-only -S -o $(ISA_DIR)/$*.s $< 2>/dev/null
	python3 tools/isa_vmcheck.py $(ISA_DIR)/$*.s
	@touch $@

lab: $(LAB) $(LAB32)

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) $(call sched_of,$*) -c $< -o $@

$(LIB): $(OBJS) $(ISA_OK)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS)

LAB_SRCS := $(SRC_DIR)/conv_f16.hip $(SRC_DIR)/conv_block0.hip $(SRC_DIR)/conv_wino.hip $(SRC_DIR)/conv_winoc.hip $(SRC_DIR)/conv_winoc42.hip $(SRC_DIR)/conv_winoh.hip
$(LAB): $(LAB_SRCS) $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(CXXFLAGS) -DRRIN_LAB -shared -o $@ $(LAB_SRCS)

$(LAB32): $(SRC_DIR)/conv_mfma.hip $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(CXXFLAGS) -DRRIN_LAB -shared -o $@ $<

# Packed-FP32 experiment: library variants with packed FP32 ops
# in every kernel (pk_all), only the ring fix-up (pk_edge) or only the convs
# (pk_conv), or the fix-up's FMAs in hand-placed packed form (pk_asm1/2).  Not used by the product; tools/gpu_pk.sh swaps them in on a box.
PKV := rrin_amd/librrin_hip_pk_all.so rrin_amd/librrin_hip_pk_edge.so rrin_amd/librrin_hip_pk_conv.so \
       rrin_amd/librrin_hip_pk_asm1.so rrin_amd/librrin_hip_pk_asm2.so
pk-variants: $(PKV)

rrin_amd/librrin_hip_pk_all.so: $(SRCS) $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(filter-out $(NOPK),$(CXXFLAGS)) -shared -o $@ $(SRCS)

rrin_amd/librrin_hip_pk_edge.so: $(SRCS) $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(CXXFLAGS) -DRRIN_PK_EDGE -shared -o $@ $(SRCS)

rrin_amd/librrin_hip_pk_conv.so: $(SRCS) $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(CXXFLAGS) -DRRIN_PK_CONV -shared -o $@ $(SRCS)

# ring fix-up FMAs as hand-placed v_pk_fma_f32: 1 splat src1, 2 op_sel form
rrin_amd/librrin_hip_pk_asm%.so: $(SRCS) $(SRC_DIR)/common.hpp include/rrin_hip.h
	$(HIPCC) $(CXXFLAGS) -DRRIN_PK_EDGE_ASM=$* -shared -o $@ $(SRCS)

# kernel register / LDS / occupancy report
resource: $(SRCS)
	$(HIPCC) $(CXXFLAGS) -Rpass-analysis=kernel-resource-usage -c $(SRC_DIR)/conv_mfma.hip -o /dev/null

clean:
	rm -rf build $(LIB) $(LAB) $(LAB32) $(PKV)

.PHONY: all lab clean resource pk-variants check-isa
