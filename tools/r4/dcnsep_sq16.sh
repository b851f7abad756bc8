# SQ counter passes over the fused-DCN_sep microbenchmark (tools/bench_dcnsep.py, 48 x 128^2) for the 32-pixel
# kernel (in-tree) and the 16-pixel one (tools/exp_DCNSEP_P16_1.so), one rocprofv3 pass per counter set
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F16"
C3="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in in-tree exp_DCNSEP_P16_1; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/tools/$v.so; else unset STIF_HIP_LIB; fi
  i=0
  for C in "$C1" "$C2" "$C3"; do
    i=$((i+1))
    REPS=5 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/r4/sq_${v}_$i -o run -- python3 $R/tools/bench_dcnsep.py > $R/gpurun_out/r4/sq_${v}_$i.log 2>&1
  done
  echo "$v done"
  python3 $R/tools/sq_summary.py k_dcn_sep $R/gpurun_out/r4/sq_${v}_1 $R/gpurun_out/r4/sq_${v}_2 $R/gpurun_out/r4/sq_${v}_3
done
