#!/bin/bash
# TA / TCP counters over one C0 step (is k_dec2q's gather bound by address / line-request throughput?)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r6/ta_pass -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras --steps 1 --warmup 1 > $R/gpurun_out/r6/ta_pass.log 2>&1 || { tail -20 $R/gpurun_out/r6/ta_pass.log; exit 1; }
python3 $R/tools/sq_summary.py "k_dec" $R/gpurun_out/r6/ta_pass
python3 $R/tools/sq_summary.py "k_wino<0, 2, 1>" $R/gpurun_out/r6/ta_pass
python3 $R/tools/sq_summary.py "k_dcn_sep<0>" $R/gpurun_out/r6/ta_pass
