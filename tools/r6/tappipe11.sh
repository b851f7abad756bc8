#!/bin/bash
# item 4, eleventh step: dump bisect (tools/r6/tappipe_dump.py) on the tap-pipelined variant with and without packed fp32
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in ${VARS:-PK NOPK}; do
  echo "### TPD_$v"
  STIF_HIP_LIB="$R/tools/exp_TPD_$v.so" timeout -k 10 300 python -u tools/r6/tappipe_dump.py || exit 1
done
