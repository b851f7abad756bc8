#!/bin/bash
# DCNSEP_P2PROG (phase-2 stage waited for in 3 / 9 tap groups): parity + determinism GPU tests on each variant, then a
# same-box C0 A/B (3 alternating reps x 20 steps) and the trace-free k_dcn_sep timing
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in 3 9; do
  STIF_HIP_LIB=$R/tools/exp_DCNSEP_P2PROG_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_model.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/p2prog_tests_$v.log 2>&1 || { echo "P2PROG=$v tests FAILED"; tail -30 gpurun_out/r6/p2prog_tests_$v.log; exit 1; }
  echo "P2PROG=$v: $(tail -1 gpurun_out/r6/p2prog_tests_$v.log)"
done
REPS=3 STEPS=20 bash tools/ab_libs.sh
