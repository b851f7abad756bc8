#!/bin/bash
# Round-6 decoder probe at C0: k_dec1 / k_dec2q with and without the MLP weight streaming (DEC_EXP=1: no LDS-DMA of
# the weight segments -- wrong results, timing only).  bench --kernel-report, HIP events, 2 reps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
run() {
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 5 --kernel-report --range-check off $2 > $O/dp.json 2> $O/dp.err \
    || { tail -30 $O/dp.err; exit 1; }
  echo "== $1: $(python -c "import json;d=json.loads(open('$O/dp.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
  grep -E "\('dec" $O/dp.err | head -6
}
for rep in 1 2; do
unset STIF_HIP_LIB; run in-tree ""
export STIF_HIP_LIB=$R/tools/exp_DEC_EXP_1.so; run "DEC_EXP=1 (no weight streaming)" ""
done
