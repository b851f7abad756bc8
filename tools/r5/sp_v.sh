#!/bin/bash
# k_wino_sp check: bit-identity tests, the microbenchmark, and the per-step trace (tools/exp_*TRACE*.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q -k "sp" --timeout 120 --timeout-method thread \
  > $O/sp_tests.log 2>&1 || { tail -40 $O/sp_tests.log; exit 1; }
tail -1 $O/sp_tests.log
REPS=${REPS:-3} timeout -k 10 200 python -u tools/r5/bench_wsp.py 2>&1 | grep -v amdgpu.ids || exit 1
for v in tools/exp_*TRACE*.so; do
  STIF_HIP_LIB=$R/$v timeout -k 10 120 python -u tools/r5/sp_trace.py > $O/sp_trace.txt 2>&1 || { tail $O/sp_trace.txt; exit 1; }
  tail -6 $O/sp_trace.txt
done
