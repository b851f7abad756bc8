#!/bin/bash
# DEC1_RES: bit-identity of the decoded window vs the streamed stage 1, the GPU suite's decoder / model / config tests on
# the variant, then a same-box C0 A/B (3 reps x 20 steps) and one C2 pair of runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u tools/r6/dec_res_bitcheck.py save gpurun_out/r6/dec_ref.npz || exit 1
STIF_HIP_LIB=$R/tools/exp_DEC1_RES_1.so timeout -k 10 300 python -u tools/r6/dec_res_bitcheck.py check gpurun_out/r6/dec_ref.npz || exit 1
STIF_HIP_LIB=$R/tools/exp_DEC1_RES_1.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r6/dec_res_tests.log 2>&1 || { echo "tests FAILED"; tail -30 gpurun_out/r6/dec_res_tests.log; exit 1; }
echo "GPU suite on DEC1_RES: $(tail -1 gpurun_out/r6/dec_res_tests.log)"
REPS=3 STEPS=20 bash tools/ab_libs.sh
for lib in "" tools/exp_DEC1_RES_1.so; do
  if [ -n "$lib" ]; then export STIF_HIP_LIB=$R/$lib; else unset STIF_HIP_LIB; fi
  timeout -k 10 600 python -u bench.py --no-extras --no-cpu-baseline --config c2 --steps 2 --warmup 1 --kernel-report > gpurun_out/r6/c2.json 2> gpurun_out/r6/c2.err || { tail -20 gpurun_out/r6/c2.err; exit 1; }
  echo "== c2 ${lib:-in-tree}: $(python -c "import json;d=json.loads(open('gpurun_out/r6/c2.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
  grep -E "\('dec[12]',\)" gpurun_out/r6/c2.err | head -3
done
