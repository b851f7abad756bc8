#!/bin/bash
# Export a git revision (default HEAD) -- sources, scripts, bench -- to tools/base_tree/ and build its
# library with that revision's Makefile; also copy the library to tools/exp_base.so.  Same-box A/B
# runs (tools/r2_ab*.sh) time the working tree against it.
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
rm -rf tools/base_tree && mkdir -p tools/base_tree
git archive "$REV" -- . ':!tests/golden' ':!profiles' ':!tools' | tar -x -C tools/base_tree
make -C tools/base_tree -j8 > tools/base_tree/build.log 2>&1 || { tail -20 tools/base_tree/build.log; exit 1; }
cp tools/base_tree/stif-continuous-video-representation_amd/libstif_hip.so tools/exp_base.so
