#!/bin/bash
# Round-6 decoder probe, second step (C0, --range-check off, kernel report, 2 reps): DEC_EXP=1 (no weight streaming) vs
# DEC_EXP=2 (the stream issued, but the segment barriers do not wait for it) vs in-tree -- DMA issue vs DMA latency.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
run() {
  if [ -n "$2" ]; then export STIF_HIP_LIB=$R/$2; else unset STIF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 5 --kernel-report --range-check off > $O/dp.json 2> $O/dp.err \
    || { tail -30 $O/dp.err; exit 1; }
  echo "== $1: $(python -c "import json;d=json.loads(open('$O/dp.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
  grep -E "\('dec" $O/dp.err | head -4
}
for rep in 1 2; do
  run in-tree ""
  run "DEC_EXP=1 (no stream)" tools/exp_DEC_EXP_1.so
  run "DEC_EXP=2 (no wait)" tools/exp_DEC_EXP_2.so
done
