#!/bin/bash
# Round-6 fused-DCN_sep phase probes at C0: per-kind kernel times (bench --kernel-report, HIP events) for the
# in-tree kernel, the two-kernel path (k_wino_om + k_dcn, --fused-dcn 0), and the timing probes
# DCNSEP_EXP = 1 (no phase 1), 3 (no phase 2), 7 (phase-1 weight DMA only for the first two steps).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
run() {  # label, extra args
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 10 --kernel-report $2 > $O/p.json 2> $O/p.err \
    || { tail -30 $O/p.err; exit 1; }
  echo "== $1: $(python -c "import json;d=json.loads(open('$O/p.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
  grep -E "dcn|wino', 3, 1, 4|'om'" $O/p.err | head -12
}
for rep in 1 2; do
unset STIF_HIP_LIB
run in-tree ""
run two-kernel "--fused-dcn 0"
for v in 1 3 7; do
  export STIF_HIP_LIB=$R/tools/exp_DCNSEP_EXP_$v.so
  run "EXP=$v" ""
done
done
