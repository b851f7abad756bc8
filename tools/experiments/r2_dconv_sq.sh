# SQ counters of the direct f16x3 conv and the f16x3 Winograd conv on the C1 trunk shape
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
for o in dconv16 wino16; do
ONLY=$o timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/sq_$o -o run -- python3 $R/tools/bench_conv.py > $R/gpurun_out/sq_$o.log 2>&1
done
C2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
ONLY=dconv16 timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $R/gpurun_out/sq2_dconv16 -o run -- python3 $R/tools/bench_conv.py > $R/gpurun_out/sq2_dconv16.log 2>&1
echo done
