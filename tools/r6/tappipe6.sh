#!/bin/bash
# item 4, sixth step: the tap-pipelined variant with every LDS corner / B-fragment read checked against HBM
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export STIF_HIP_LIB="$R/tools/exp_DCNSEP_TAPPIPE_1+DCNSEP_TP_CHECK_1.so"
QUICK=1 timeout -k 10 300 python -u tools/r6/tappipe_diag.py > gpurun_out/r6/tappipe6_full.log 2>&1 || { tail -20 gpurun_out/r6/tappipe6_full.log; exit 1; }
grep -c TPCHECK gpurun_out/r6/tappipe6_full.log || true
grep -v TPCHECK gpurun_out/r6/tappipe6_full.log | grep -v Warn
grep TPCHECK gpurun_out/r6/tappipe6_full.log | head -40
