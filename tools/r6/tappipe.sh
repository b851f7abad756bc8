#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6
for lib in "" tools/exp_DCNSEP_TAPPIPE_1.so; do
  if [ -n "$lib" ]; then export STIF_HIP_LIB=$R/$lib; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u tools/r6/tappipe_diag.py || exit 1
done
