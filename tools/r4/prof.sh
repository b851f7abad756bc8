#!/bin/bash
# Round-4 profile of the default (C0) bench: rocprofv3 kernel trace + stats (3 steps) and, with PMC=1, the
# FETCH_SIZE / WRITE_SIZE / SQ passes (separate runs, MI355X_MICROARCH.md PMC rules).  TAG names the outputs.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r04}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $B --steps 3 --warmup 1 \
  > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
f=$(ls $O/kt/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $O/kt -name '*kernel_trace.csv' | head -1)
python3 $R/tools/r4/ktrace.py "$f" > $O/ktrace.txt && cat $O/ktrace.txt
s=$(find $O/kt -name '*kernel_stats.csv' | head -1); python3 $R/tools/kstats.py "$s" 24
if [ "${PMC:-0}" = 1 ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B --steps 1 --warmup 1 > $O/fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B --steps 1 --warmup 1 > $O/write.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/mfma -o run -- python3 $B --steps 1 --warmup 1 > $O/mfma.log 2>&1 || exit 1
fi
echo done
