# SQ counter passes over the fused-DCN_sep microbenchmark (tools/bench_dcnsep.py, C0 L1 shape 48 x 128^2,
# offsets N(0, 2^2) px): the full kernel and the phase probes (tools/exp_DCNSEP_EXP_{1,3}.so: no phase 1 /
# no phase 2), one rocprofv3 pass per counter set (MI355X_MICROARCH.md PMC limits)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F16"
C3="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in in-tree exp_DCNSEP_EXP_1 exp_DCNSEP_EXP_3; do
  if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/tools/$v.so; else unset STIF_HIP_LIB; fi
  i=0
  for C in "$C1" "$C2" "$C3"; do
    i=$((i+1))
    REPS=5 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/r3/sq_${v}_$i -o run -- python3 $R/tools/bench_dcnsep.py > $R/gpurun_out/r3/sq_${v}_$i.log 2>&1
  done
  echo "$v done"
done
