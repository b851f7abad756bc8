#!/bin/bash
# Decoder weight stream: what costs, the DMA instructions or their memory traffic?  C0, --range-check off, 2 reps.
# DEC_EXP=1: no weight DMA at all; DEC_EXP=3: every DMA piece issued out of range (same instructions, no traffic).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
run() {
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 5 --range-check off --kernel-report > $O/dp.json 2> $O/dp.err \
    || { tail -30 $O/dp.err; exit 1; }
  echo "== $1: $(python -c "import json;d=json.loads(open('$O/dp.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
  grep -E "\('dec[12]',\)" $O/dp.err | head -4
}
for rep in 1 2; do
  unset STIF_HIP_LIB; run in-tree
  export STIF_HIP_LIB=$R/tools/exp_DEC_EXP_1.so; run "DEC_EXP=1 (no weight DMA)"
  export STIF_HIP_LIB=$R/tools/exp_DEC_EXP_3.so; run "DEC_EXP=3 (DMA pieces out of range: instructions, no traffic)"
done
