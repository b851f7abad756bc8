#!/bin/bash
# item 4, second step: the tap-pipelined variant with an s_nop 4 after every split_f16x3 asm block
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for lib in "tools/exp_DCNSEP_TAPPIPE_1+STIF_SPLIT_NOP_1.so" tools/exp_DCNSEP_TAPPIPE_1.so; do
  export STIF_HIP_LIB="$R/$lib"
  QUICK=1 timeout -k 10 300 python -u tools/r6/tappipe_diag.py || exit 1
done
