#!/bin/bash
# Fused DCN_sep LDS bank conflicts in the real C0 workload: the C0 bench kernel report and one SQ pass
# (LDS counters) for the in-tree library and the offset-free sampling probe (tools/exp_DCNSEP_EXP_6.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in in-tree tools/exp_DCNSEP_EXP_6.so; do
    if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > $O/ab.json 2> $O/ab.err \
      || { tail -30 $O/ab.err; exit 1; }
    echo "$v: $(python -c "import json;d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]);print(d['value'],'Mpix/s',d['ms_per_step'],'ms')")"
    grep "'dcnsep'" $O/ab.err
  done
done
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in in-tree exp_DCNSEP_EXP_6; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/tools/$v.so; else unset STIF_HIP_LIB; fi
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/sq_dcnsep_$v -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 1 --warmup 1 > $O/sq_dcnsep_$v.log 2>&1 || { tail -20 $O/sq_dcnsep_$v.log; exit 1; }
  echo "$v SQ pass done"
done
