#!/bin/bash
# Kernel-experiment libraries that differ from the in-tree build in ONE object: SRC (a csrc/*.hip
# basename) compiled with -D switches (VAR = 'A+B=2' -> -DA -DB=2) and linked with the other in-tree
# objects (make first), so every other kernel keeps the Makefile's exact flags.  -> tools/exp_<VAR>.so
set -e
cd "$(dirname "$0")/.."
SRC=$1; shift
PKG=stif-continuous-video-representation_amd
make -s -j8 > /dev/null
NOPK=""
case " wino decoder conv resample dcnsep dcn " in *" $SRC "*) NOPK="-Xclang -target-feature -Xclang -packed-fp32-ops";; esac
for v in "$@"; do
  flags=""
  for f in ${v//+/ }; do flags="$flags -D$f"; done
  name=$(echo "$v" | tr -c 'A-Za-z0-9_+\n' '_')
  (
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -I$PKG/csrc -Wall -Wno-unused-function \
      $NOPK $flags -c -o build/exp_$name.o $PKG/csrc/$SRC.hip 2> build/exp_$name.log
    objs=$(ls build/*.o | grep -v '/exp_' | grep -v "/$SRC.o")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o tools/exp_$name.so $objs build/exp_$name.o
  ) &
done
wait
ls -la tools/exp_*.so
