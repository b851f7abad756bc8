#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in tools/exp_*TRACE*.so; do
  STIF_HIP_LIB=$R/$v timeout -k 10 120 python -u tools/r5/sp_trace.py 2>&1 | grep -v amdgpu.ids || exit 1
done
