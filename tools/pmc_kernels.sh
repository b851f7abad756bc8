# One SQ counter pass over the DCN and Winograd microbenchmarks (tools/bench_dcn16.py,
# tools/bench_conv.py): wait / issue / LDS-conflict breakdown per kernel (MI355X_MICROARCH.md SQ notes).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_dcn -o run -- python3 $R/tools/bench_dcn16.py > $R/gpurun_out/pmc_dcn.log 2>&1
ONLY=wino16 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_wino -o run -- python3 $R/tools/bench_conv.py > $R/gpurun_out/pmc_wino.log 2>&1
echo done
