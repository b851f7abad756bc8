#!/bin/bash
# item 4, fourth step: nops before the split's writes (WAR against in-flight MFMA source reads), and the split as
# plain expressions (the compiler's hazard recognizer sees the VALU writes)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for lib in "tools/exp_DCNSEP_TAPPIPE_1+STIF_SPLIT_NOP_PRE_1.so" "tools/exp_DCNSEP_TAPPIPE_1+STIF_SPLIT_C_1.so"; do
  export STIF_HIP_LIB="$R/$lib"
  QUICK=1 timeout -k 10 300 python -u tools/r6/tappipe_diag.py || exit 1
done
