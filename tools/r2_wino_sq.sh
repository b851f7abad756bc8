# SQ counter passes over the f16x3 Winograd conv microbenchmark at the C0 trunk shape
# (tools/bench_conv.py, ONLY=wino16, 18 x 128 x 128 x 64): issue / wait / LDS / VMEM / MFMA breakdown
# of k_wino (one pass per counter set, MI355X_MICROARCH.md SQ notes).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export ONLY=wino16 N=18 HW=128
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F16"
C3="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
C4="SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_IFETCH SQ_WAVES SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_MFMA"
i=0
for C in "$C1" "$C2" "$C3" "$C4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/wino_sq$i -o run -- python3 $R/tools/bench_conv.py > $R/gpurun_out/wino_sq$i.log 2>&1
done
python3 $R/tools/sq_summary.py "k_wino<0, 3, 1>" $R/gpurun_out/wino_sq1 $R/gpurun_out/wino_sq2 $R/gpurun_out/wino_sq3 $R/gpurun_out/wino_sq4
