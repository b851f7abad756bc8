#!/bin/bash
# item 4, fifth step: the tap-pipelined variant (and the in-tree kernel) at one workgroup per CU (48 KB LDS pad)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for lib in "tools/exp_DCNSEP_TAPPIPE_1+DCNSEP_SOLO_1.so" "tools/exp_DCNSEP_SOLO_1.so"; do
  export STIF_HIP_LIB="$R/$lib"
  QUICK=1 timeout -k 10 300 python -u tools/r6/tappipe_diag.py || exit 1
done
