#!/bin/bash
# tools/r6/build_flag_variant.sh NAME "OBJECTS" "FLAGS": the product library with OBJECTS (csrc basenames) recompiled
# with extra FLAGS (same per-object NOPK rule as the Makefile) -> tools/exp_NAME.so
set -e
NAME=$1; OBJS=$2; FLAGS=$3
PKG=stif-continuous-video-representation_amd
NOPK="-Xclang -target-feature -Xclang -packed-fp32-ops"
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$PKG/csrc -Wall -Wno-unused-function"
link=""
for o in build/abi_util.o build/conv.o build/dcn.o build/dcnsep.o build/decoder.o build/resample.o build/wino.o build/pack.o; do
  b=$(basename $o .o)
  if [[ " $OBJS " == *" $b "* ]]; then
    /opt/rocm/bin/hipcc $HF $NOPK $FLAGS -c -o build/exp_${NAME}_$b.o $PKG/csrc/$b.hip 2>/dev/null
    link="$link build/exp_${NAME}_$b.o"
  else
    link="$link $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o tools/exp_$NAME.so $link
echo tools/exp_$NAME.so
