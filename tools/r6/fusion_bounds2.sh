#!/bin/bash
# Review item 2, measured floor of a fused ResidualBlock_noBN (C0, bench --kernel-report, HIP events, trunk on one stream):
#  in-tree; WINO_EXP=5 (conv1 stores nothing: the intermediate's write removed); WINO_EXP=7 (conv1 does 1.5x its
#  transform / split / MFMA work -- the work of a conv1 over the 1-px halo a fused block's conv2 needs -- and stores
#  nothing).  Then one SQ PMC pass per library over one C0 step (8 SQ counters + GRBM), summarised per kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6
mkdir -p $O
cd $R
run() {  # label
  timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 5 --trunk-lanes 1 --kernel-report > $O/fb.json 2> $O/fb.err \
    || { tail -30 $O/fb.err; exit 1; }
  echo "== $1: $(python -c "import json;d=json.loads(open('$O/fb.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
  grep -E "\('wino', 3, 1, [23], 0, 64\)" $O/fb.err | head -4
}
for rep in 1 2; do
  unset STIF_HIP_LIB; run in-tree
  export STIF_HIP_LIB=$R/tools/exp_WINO_EXP_5.so; run "WINO_EXP=5 (conv1 stores nothing)"
  export STIF_HIP_LIB=$R/tools/exp_WINO_EXP_7.so; run "WINO_EXP=7 (conv1 1.5x work, stores nothing)"
done
unset STIF_HIP_LIB
cd /tmp && export TMPDIR=/tmp
for v in base 7; do
  if [ $v = base ]; then unset STIF_HIP_LIB; else export STIF_HIP_LIB=$R/tools/exp_WINO_EXP_7.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/fb_pmc_$v -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 1 --warmup 1 --trunk-lanes 1 > $O/fb_pmc_$v.log 2>&1 || { tail -20 $O/fb_pmc_$v.log; exit 1; }
  echo "== PMC ($v)"
  python3 $R/tools/sq_summary.py "k_wino<0, 2, 1>" $O/fb_pmc_$v
  python3 $R/tools/sq_summary.py "k_wino<0, 3, 1>" $O/fb_pmc_$v
done
