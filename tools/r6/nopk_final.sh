#!/bin/bash
# Product build now has no packed fp32 in any kernel object. Full GPU suite on it, then the fp32-MFMA line
# A/B: in-tree (k_dcn without packed fp32) vs exp_DCN_PK (k_dcn with them), 3 alternating reps of 10 steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_tests_nopk.log 2>&1 || { tail -30 gpurun_out/r6/gpu_tests_nopk.log; exit 1; }
tail -1 gpurun_out/r6/gpu_tests_nopk.log
echo "# fp32-MFMA line (--mfma f32)"
REPS=3 STEPS=10 BENCH_ARGS="--mfma f32" bash tools/ab_libs.sh
