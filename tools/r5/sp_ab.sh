#!/bin/bash
# k_wino_sp variants: the microbenchmark under the in-tree library and every tools/exp_*.so
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in in-tree tools/exp_*.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  echo "== $v"
  REPS=${REPS:-2} timeout -k 10 200 python -u tools/r5/bench_wsp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
