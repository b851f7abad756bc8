#!/bin/bash
# Item 4 resolved: the tap-pipelined fused DCN_sep without packed-fp32 VALU ops (exp_TAPPIPE_NOPK) is deterministic.
# Its GPU tests (fused DCN_sep ops, C0 window incl. both determinism tests and the large-config pins), then a same-box
# C0 A/B: in-tree (packed fp32) / exp_NOPK (in-tree kernel without packed fp32) / exp_TAPPIPE_NOPK.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
STIF_HIP_LIB=$R/tools/exp_TAPPIPE_NOPK.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_model.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/nopk_tests.log 2>&1 || { tail -30 gpurun_out/r6/nopk_tests.log; exit 1; }
tail -1 gpurun_out/r6/nopk_tests.log
REPS=3 bash tools/ab_libs.sh
