#!/bin/bash
# Fused DCN_sep without the two all-pad weight DMA pieces per phase-1 step (DCNSEP_WTRIM=1): the fused-DCN_sep GPU tests
# under the variant, then a same-box C0 A/B (tools/ab_libs.sh, 3 reps).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
STIF_HIP_LIB=$R/tools/exp_DCNSEP_WTRIM_1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -m gpu \
  -k "dcn_sep or c0 or large_config" -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/wtrim_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6/wtrim_tests.log; exit 1; }
tail -1 gpurun_out/r6/wtrim_tests.log
REPS=3 bash tools/ab_libs.sh
