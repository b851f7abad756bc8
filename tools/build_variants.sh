#!/bin/bash
# Kernel-experiment builds of the engine library with -D switches (tools/exp_*.so; not shipped).
set -e
cd "$(dirname "$0")/.."
PKG=stif-continuous-video-representation_amd
SRC="$(ls $PKG/csrc/*.hip) $PKG/csrc/pack.cpp"
for v in "$@"; do
  flags=""
  for f in ${v//+/ }; do flags="$flags -D$f"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$PKG/csrc $flags -shared -o tools/exp_$v.so $SRC &
done
wait
