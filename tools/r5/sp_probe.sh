#!/bin/bash
# k_wino_sp: bit-identity tests, then the microbenchmark under the in-tree library and every tools/exp_*.so.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q -k "sp" --timeout 120 --timeout-method thread \
  > $O/sp_tests.log 2>&1 || { tail -40 $O/sp_tests.log; exit 1; }
tail -1 $O/sp_tests.log
for v in in-tree tools/exp_*.so; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
  echo "== $v"
  REPS=${REPS:-2} timeout -k 10 200 python -u tools/r5/bench_wsp.py 2>&1 | grep -v amdgpu.ids || exit 1
done
