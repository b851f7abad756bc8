#!/bin/bash
# k_wino_sp first GPU check: bit-identity tests vs k_wino, then the microbenchmark.  Every GPU step under
# its own timeout; the first failure ends the call.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q -k "sp" --timeout 120 --timeout-method thread \
  > $O/sp_tests.log 2>&1 || { tail -40 $O/sp_tests.log; exit 1; }
tail -3 $O/sp_tests.log
timeout -k 10 200 python -u tools/r5/bench_wsp.py 2>&1 | grep -v amdgpu.ids
