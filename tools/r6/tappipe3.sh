#!/bin/bash
# item 4, third step: which part of the tap-pipelined variant makes repeated launches differ
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for lib in "tools/exp_DCNSEP_TAPPIPE_1+DCNSEP_TP_NOFB_1.so" "tools/exp_DCNSEP_TAPPIPE_1+DCNSEP_TP_WAIT_1.so"; do
  export STIF_HIP_LIB="$R/$lib"
  QUICK=1 timeout -k 10 300 python -u tools/r6/tappipe_diag.py || exit 1
done
