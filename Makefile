# Builds the gfx950 engine library (HIP kernels + C ABI + host packing) in-tree.
PKG := stif-continuous-video-representation_amd
HIP_SRC := $(wildcard $(PKG)/csrc/*.hip)
HDR := $(wildcard $(PKG)/csrc/*.h) include/stif.h
LIB := $(PKG)/libstif_hip.so
OBJDIR := build
OBJ := $(patsubst $(PKG)/csrc/%.hip,$(OBJDIR)/%.o,$(HIP_SRC)) $(OBJDIR)/pack.o
HIPCC ?= /opt/rocm/bin/hipcc
HIPFLAGS := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$(PKG)/csrc -Wall -Wno-unused-function
# No kernel object uses packed fp32 (v_pk_fma/add/mul_f32). Beside MFMAs one v_pk_fma_f32 costs more
# issue cycles than the two v_fma_f32 it replaces (MI355X_MICROARCH.md): in same-box A/B runs the C0 step
# is 0.7-1.5 % faster without them (Winograd transforms, SIREN sines and gathers, stride-2 / 1x1 convs,
# upsample), and round 6 moved the fused DCN_sep kernel over as well: k_dcn_sep<0> 349 vs 362 us per
# launch (profiles/r06_nopk_ab.log), and the tap-pipelined diagnostic variant whose output depended on
# the co-resident workgroup is bit-stable without them.
# Device-only feature: the host pass prints "not a recognized feature for this target (ignoring feature)".
NOPK := -Xclang -target-feature -Xclang -packed-fp32-ops
NOPK_SRC := wino decoder conv resample dcnsep dcn

all: $(LIB)

$(OBJDIR)/%.o: $(PKG)/csrc/%.hip $(HDR) Makefile | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(if $(filter $*,$(NOPK_SRC)),$(NOPK)) -c -o $@ $<

$(OBJDIR)/pack.o: $(PKG)/csrc/pack.cpp $(HDR) Makefile | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJDIR):
	mkdir -p $@

$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)

clean:
	rm -rf $(LIB) $(OBJDIR)

.PHONY: all clean
