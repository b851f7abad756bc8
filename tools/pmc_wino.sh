# SQ counters of the Winograd conv on the trunk shape (tools/bench_conv.py, ONLY=wino)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
ONLY=wino timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_wino1 -o p -- python3 $R/tools/bench_conv.py > $R/gpurun_out/pmc_wino1.log 2>&1
