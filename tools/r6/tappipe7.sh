#!/bin/bash
# item 4, seventh step: the tap-pipelined variant with phase 1 fully drained and synchronised at every step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export STIF_HIP_LIB="$R/tools/exp_DCNSEP_TAPPIPE_1+DCNSEP_P1_SAFE_1.so"
QUICK=1 timeout -k 10 300 python -u tools/r6/tappipe_diag.py
