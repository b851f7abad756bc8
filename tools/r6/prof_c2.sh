#!/bin/bash
# C2 (the decoder-heavy config: 540x960 -> 4x) kernel stats and one SQ MFMA pass, 1 timed step each
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6/c2_stats -o run -- python3 $R/bench.py --config c2 --no-cpu-baseline --no-extras --steps 1 --warmup 1 > $R/gpurun_out/r6/c2_stats.log 2>&1 || { tail -20 $R/gpurun_out/r6/c2_stats.log; exit 1; }
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r6/c2_mfma -o run -- python3 $R/bench.py --config c2 --no-cpu-baseline --no-extras --steps 1 --warmup 1 > $R/gpurun_out/r6/c2_mfma.log 2>&1 || { tail -20 $R/gpurun_out/r6/c2_mfma.log; exit 1; }
echo done
