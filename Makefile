# Builds the gfx950 engine library (HIP kernels + C ABI + host packing) in-tree.
PKG := stif-continuous-video-representation_amd
SRC := $(wildcard $(PKG)/csrc/*.hip) $(PKG)/csrc/pack.cpp
HDR := $(wildcard $(PKG)/csrc/*.h) include/stif.h
LIB := $(PKG)/libstif_hip.so
HIPCC ?= /opt/rocm/bin/hipcc
HIPFLAGS := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$(PKG)/csrc -Wall -Wno-unused-function

all: $(LIB)

$(LIB): $(SRC) $(HDR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRC)

clean:
	rm -f $(LIB)

.PHONY: all clean
