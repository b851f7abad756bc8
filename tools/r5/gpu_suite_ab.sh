#!/bin/bash
# Round-5 GPU check: the whole GPU suite (in-tree), then the decoder microbenchmark at C0 and C2 for the in-tree
# library and tools/exp_base.so (round-4 end), alternating.  Every GPU step under its own timeout.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
for rep in 1 2; do
  for v in in-tree tools/exp_base.so; do
    if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
    for cfg in c0 c2; do
      echo "$v $cfg: $(CFG=$cfg REPS=5 timeout -k 10 200 python -u tools/bench_dec.py 2>&1 | grep -v amdgpu.ids | grep "dec" | tr '\n' ' ')" || exit 1
    done
  done
done
