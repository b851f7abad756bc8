#!/bin/bash
# item 4, tenth step: where the tap-pipelined (packed fp32) variant's re-runs differ (DIFF=1: element count, size,
# channel half, tile row, lane column, border distance, item), and the variant with s_nop 15 before every instruction.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in PK SNOP15; do
  echo "### TP_$v"
  DIFF=1 STIF_HIP_LIB="$R/tools/exp_TP_$v.so" QUICK=1 timeout -k 10 400 python -u tools/r6/tappipe_diag.py || exit 1
done
