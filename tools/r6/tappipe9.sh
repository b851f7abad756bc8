#!/bin/bash
# item 4, ninth step: the tap-pipelined variant WITH packed fp32 (control), and with compiler-wide padding:
# an s_nop 4 before every instruction (-amdgpu-snop-padding=4: covers every VALU/MFMA register hazard of up to
# 5 wait states), every s_waitcnt forced to vmcnt(0) expcnt(0) lgkmcnt(0) (-amdgpu-waitcnt-forcezero), and the
# latency between neighbouring MFMAs filled with s_nop (-amdgpu-mfma-padding-ratio=100).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in PK SNOP4 WAIT0 MFMAPAD; do
  echo "### TP_$v"
  STIF_HIP_LIB="$R/tools/exp_TP_$v.so" QUICK=1 timeout -k 10 300 python -u tools/r6/tappipe_diag.py || exit 1
done
