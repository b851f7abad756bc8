#!/bin/bash
# Build the engine library of a git revision (default HEAD) with that revision's Makefile as
# tools/exp_base.so, for same-box A/B runs against the working tree's in-tree build (tools/r2_ab*.sh).
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
T=$(mktemp -d)
git archive "$REV" Makefile stif-continuous-video-representation_amd/csrc include | tar -x -C "$T"
make -C "$T" -j8 > "$T/build.log" 2>&1 || { tail -20 "$T/build.log"; exit 1; }
cp "$T/stif-continuous-video-representation_amd/libstif_hip.so" tools/exp_base.so
rm -rf "$T"
