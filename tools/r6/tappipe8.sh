#!/bin/bash
# item 4, eighth step: the tap-pipelined variant compiled without packed-fp32 VALU ops (-packed-fp32-ops)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export STIF_HIP_LIB="$R/tools/exp_TAPPIPE_NOPK.so"
QUICK=1 timeout -k 10 300 python -u tools/r6/tappipe_diag.py
