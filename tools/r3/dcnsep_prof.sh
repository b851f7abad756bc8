# k_dcn_sep at the C0 L1 shape (48 x 128^2): microbenchmark of the in-tree kernel, the two-kernel path and
# the timing probes (tools/exp_DCNSEP_EXP_*.so), then SQ counter passes of the in-tree kernel.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for rep in 1 2; do
  FUSED=0 timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids
  timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids
  for lib in tools/exp_*.so; do
    echo "$lib: $(STIF_HIP_LIB=$R/$lib timeout -k 10 120 python3 tools/bench_dcnsep.py 2>&1 | grep -v amdgpu.ids)"
  done
done
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_F16"
C3="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for C in "$C1" "$C2" "$C3"; do
  i=$((i+1))
  REPS=3 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/r3/dcnsep_sq$i -o run -- python3 $R/tools/bench_dcnsep.py > $R/gpurun_out/r3/dcnsep_sq$i.log 2>&1
done
python3 $R/tools/sq_summary.py k_dcn_sep $R/gpurun_out/r3/dcnsep_sq1 $R/gpurun_out/r3/dcnsep_sq2 $R/gpurun_out/r3/dcnsep_sq3
