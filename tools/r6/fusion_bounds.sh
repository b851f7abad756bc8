#!/bin/bash
# Round-6 bounds for review items 1 and 2 (C0, bench --kernel-report, HIP events, trunk on one stream):
#  * trunk ResidualBlock: conv1 (RELU) without its output stores (WINO_EXP=5) and every Winograd conv without input
#    staging after its first phase (WINO_EXP=1) -- what a fused block could at most save on the intermediate's traffic;
#  * the Winograd offset/mask conv k_wino_om without its 216-channel HBM stores (WINO_EXP=6, two-kernel path) -- the
#    floor of a Winograd phase 1 before any hand-off to the sampling lanes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
run() {  # label, extra args
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 5 --trunk-lanes 1 --kernel-report $2 > $O/fb.json 2> $O/fb.err \
    || { tail -30 $O/fb.err; exit 1; }
  echo "== $1: $(python -c "import json;d=json.loads(open('$O/fb.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
  grep -E "\('wino', 3, 1, [23], 0, 64\)|\('wino', 3, 1, 4, 0, 216\)|\('dcnsep', 0\)|\('dcn', 0\)" $O/fb.err | head -8
}
for rep in 1 2; do
unset STIF_HIP_LIB
run in-tree ""
export STIF_HIP_LIB=$R/tools/exp_WINO_EXP_5.so; run "WINO_EXP=5 (RELU convs store nothing)" ""
export STIF_HIP_LIB=$R/tools/exp_WINO_EXP_1.so; run "WINO_EXP=1 (no staging after phase 0)" ""
unset STIF_HIP_LIB; run "two-kernel" "--fused-dcn 0"
export STIF_HIP_LIB=$R/tools/exp_WINO_EXP_6.so; run "two-kernel, WINO_EXP=6 (k_wino_om stores nothing)" "--fused-dcn 0"
done
