#!/bin/bash
# Build the engine library of a git revision (default HEAD) as tools/exp_base.so, for same-box A/B
# runs against the working tree's in-tree build (tools/r2_ab*.sh).
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
T=$(mktemp -d)
git archive "$REV" stif-continuous-video-representation_amd/csrc include | tar -x -C "$T"
PKG=$T/stif-continuous-video-representation_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$T/include -I$PKG/csrc -shared \
  -o tools/exp_base.so $PKG/csrc/*.hip $PKG/csrc/pack.cpp
rm -rf "$T"
