#!/bin/bash
# Kernel-experiment builds of the engine library with -D switches (tools/exp_*.so; not shipped).
set -e
cd "$(dirname "$0")/.."
PKG=stif-continuous-video-representation_amd
SRC="$(ls $PKG/csrc/*.hip) $PKG/csrc/pack.cpp"
for v in "$@"; do
  flags=""
  for f in ${v//+/ }; do flags="$flags -D$f"; done
  name=$(echo "$v" | tr -c 'A-Za-z0-9_+\n' '_')   # no '=' in file names sent to the GPU box
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$PKG/csrc $flags -shared -o tools/exp_$name.so $SRC &
done
wait
